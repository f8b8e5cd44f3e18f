# Long-run parity on the other twelve fuzz scenes (seeds 12-23, 320x240,
# 400 rounds each; gpu_long2.sh ran seeds 0-11).  One JSON line per run
# under gpurun_out/r03_long4/; stops at the first run that fails.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03_long4
mkdir -p "$O"
for s in 12 13 14 15 16 17 18 19 20 21 22 23; do
  timeout -k 10 150 python3 -u tools/long_parity.py fuzz:$s 400 > "$O/fuzz${s}_400.json" 2> "$O/fuzz${s}_400.err" \
    || { echo "FAILED fuzz$s"; tail -20 "$O/fuzz${s}_400.err"; exit 1; }
  cat "$O/fuzz${s}_400.json"
done
