# One GPU test by -k expression: bash tools/r05/gpu_one_test.sh EXPR
set -e
O=gpurun_out/r05_one; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v -k "$1" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert|status" $O/tests.log | tail -40; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/tests.log | tail -20
