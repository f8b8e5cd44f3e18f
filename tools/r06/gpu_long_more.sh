# C5's second camera (360) over 300 rounds and C1 over 1000 rounds (fused
# round batches), the bench's batched schedule against the oracle.
set -u
O=gpurun_out/r06_long_more
mkdir -p "$O"
timeout -k 10 500 python3 -u tools/long_parity.py 5 300 1 --batched > "$O/c5_cam1.json" 2> "$O/c5_cam1.err" || { echo C5 FAILED; tail -5 "$O/c5_cam1.err"; exit 1; }
cat "$O/c5_cam1.json"
timeout -k 10 500 python3 -u tools/long_parity.py 1 1000 --batched > "$O/c1.json" 2> "$O/c1.err" || { echo C1 FAILED; tail -5 "$O/c1.err"; exit 1; }
cat "$O/c1.json"
