# Round 5 (grey path records + LDS node cache build): the same whole-frame run.
# A whole 1024-spp frame's worth of rounds of C3 at its full 1920x1080
# (Reset + Run(2) + 2760 x Run(1), the rounds bench.py's frame takes) on the
# GPU and in the CPU oracle, every slot and pixel compared at the end
# (about 800 s of oracle time on the box's 16 threads).  Output under
# gpurun_out/r05_long3/.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_long3
mkdir -p "$O"
timeout -k 10 1150 python3 -u tools/long_parity.py 3 2762 > "$O/c3_2762.json" 2> "$O/c3_2762.err" \
  || { echo FAILED; tail -20 "$O/c3_2762.err"; exit 1; }
cat "$O/c3_2762.json"
