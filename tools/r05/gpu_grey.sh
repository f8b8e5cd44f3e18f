# Grey path records (one Probability float, no stack read where the shade
# mask proves them redundant): the GPU tests, a C3 A/B against the round-4
# build (build/variants/head.so), and the C3 PMC passes.
set -e
O=gpurun_out/r05_grey; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r04/gpu_ab.sh r05_grey_c3 3 3 head base
bash tools/r04/gpu_pmc.sh r05_grey/pmc_c3 python3 tools/run_rounds.py --config 3
