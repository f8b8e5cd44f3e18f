# A whole 1024-spp C3 frame (ptRenderFrame, the bench's schedule) against the
# oracle: the end round, the samples, every pixel and slot.
set -u
O=gpurun_out/r06_long_frame
mkdir -p "$O"
timeout -k 10 1150 python3 -u tools/long_frame.py 3 > "$O/c3.json" 2> "$O/c3.err" || { echo FAILED; tail -20 "$O/c3.err"; cat "$O/c3.json"; exit 1; }
cat "$O/c3.json"
