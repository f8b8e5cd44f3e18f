# C4 (3840x2160, the room) on one GPU at full size against the oracle: Reset +
# Run(2) + 238 rounds through the bench's batched schedule (three tile groups),
# every slot and pixel compared at the end.
set -u
O=gpurun_out/r06_long_c4
mkdir -p "$O"
timeout -k 10 1000 python3 -u tools/long_parity.py 4 240 --batched > "$O/c4.json" 2> "$O/c4.err" || { echo FAILED; tail -20 "$O/c4.err"; cat "$O/c4.json"; exit 1; }
cat "$O/c4.json"
