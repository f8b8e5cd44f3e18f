# Round 6: a BLAS step's face and node loads issued before either half
# computes (-DPT_HOIST=2/3, with occupancy floors) -- parity on two variants,
# then same-box A/B against the in-tree build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_hoist}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
for v in h3m7 h2m8; do
PT_HIP_LIB=$R/build/variants/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_path.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/tests_$v.log" 2>&1
rc=$?; echo "tests $v rc=$rc"; tail -2 "$O/tests_$v.log"; [ $rc -eq 0 ] || exit $rc
done
bash tools/r06/gpu_ab_lib.sh ${1:-r06_hoist} "3 5" base h2 h3m7 h2m8 h3m8
