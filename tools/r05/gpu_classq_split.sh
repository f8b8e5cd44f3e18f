# Class-pure shade (per-class lists, -DPT_EXP_CLASSQ=1) inside tile groups:
# the lists' latency and the gathers may hide behind the other groups'
# launches.  C2 / C5 split tests on the variant (bit-exact against unsplit
# and the oracle), then C2 / C5 A/B against the in-tree build.
set -e
O=gpurun_out/r05_classq_split; mkdir -p $O
PT_HIP_LIB=$PWD/build/variants/classq1s.so timeout -k 10 500 python -u -m pytest tests/test_gpu_split.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "2-96 or 5-128 or 2-1024 or 5-2048" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
STEPS=3 bash tools/r04/gpu_ab.sh r05_classq_split_c2 2 2 base classq1s
STEPS=2 bash tools/r04/gpu_ab.sh r05_classq_split_c5 5 2 base classq1s
