# A whole 1024-spp C3 frame's rounds (Reset + Run(2) + 2760 rounds) with the
# GPU side through ptRunBasicRendererRounds in chunks of 50, so the rounds run
# in three tile groups on concurrent streams; every slot and pixel compared
# with the oracle at the end.
set -u
O=gpurun_out/r05_long_split
mkdir -p "$O"
timeout -k 10 1150 python3 -u tools/long_parity.py 3 2762 --batched > "$O/c3_2762.json" 2> "$O/c3_2762.err" \
  || { echo FAILED; tail -20 "$O/c3_2762.err"; exit 1; }
cat "$O/c3_2762.json"
