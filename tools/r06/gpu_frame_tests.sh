cd $GRAFT_REPO_ROOT && timeout -k 10 600 python -u -m pytest tests/test_gpu_frame.py -v -m gpu -x --timeout 300 --timeout-method thread 2>&1 | tail -25
