# Round-5 new GPU tests (resume, host-gate negatives, record-form switches),
# then the C3 steady-state PMC passes of the grey-record build.
set -e
O=gpurun_out/r05_grey2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_resume.py tests/test_gpu_gates.py -v -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests.log | tail -30
bash tools/r04/gpu_pmc.sh r05_grey2/pmc_c3 python3 $PWD/tools/run_rounds.py --config 3
