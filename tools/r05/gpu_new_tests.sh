# Round-5 new GPU tests only (resume, host-gate negatives, record-form switches).
set -e
O=gpurun_out/r05_newtests; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_resume.py tests/test_gpu_gates.py -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|ERROR|Error|assert" $O/tests.log | tail -60; exit 1; }
grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests.log | tail -30
