# Long-run parity beyond profiles/r03_long: C1 at full size for 1000 rounds,
# twelve random fuzz scenes (every material, nested media, HDR skies, every
# camera) at 320x240 for 400 rounds each, and C4's whole 3840x2160 frame for
# 120 rounds.  One JSON line per run under gpurun_out/r03_long2/; stops at the
# first run that fails or times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03_long2
mkdir -p "$O"
run() {  # name config rounds seconds
  timeout -k 10 "$4" python3 -u tools/long_parity.py "$2" "$3" > "$O/$1.json" 2> "$O/$1.err" \
    || { echo "FAILED $1"; tail -20 "$O/$1.err"; exit 1; }
  cat "$O/$1.json"
}
run c1_1000 1 1000 300
for s in 0 1 2 3 4 5 6 7 8 9 10 11; do run fuzz${s}_400 fuzz:$s 400 150; done
run c4_120 4 120 400
