# Round 6: compiler scheduling strategy A/B (-mllvm -amdgpu-sched-strategy=
# max-memory-clause, build/variants/memclause.so) -- parity tests on the
# variant, then same-box bench A/B against the in-tree build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_sched}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
PT_HIP_LIB=$R/build/variants/memclause.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gates.py tests/test_gpu_bench_path.py -v -m gpu -x --timeout 400 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
bash tools/r06/gpu_ab_lib.sh ${1:-r06_sched} "3 5 2" base memclause
