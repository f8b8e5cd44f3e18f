# Long-run parity: C5 at full size through its second camera (the 360-degree
# one) over 1000 rounds, and C2 at 1024x1024 over 800 rounds (more than its
# 256-spp frame).  Output under gpurun_out/r03_long5/.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03_long5
mkdir -p "$O"
run() {  # name config rounds camera seconds
  timeout -k 10 "$5" python3 -u tools/long_parity.py "$2" "$3" "$4" > "$O/$1.json" 2> "$O/$1.err" \
    || { echo "FAILED $1"; tail -20 "$O/$1.err"; exit 1; }
  cat "$O/$1.json"
}
run c5_cam1_1000 5 1000 1 400
run c2_800 2 800 0 300
