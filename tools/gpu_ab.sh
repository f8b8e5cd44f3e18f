# A/B of library variants (build/variants/*.so, tools/build_variant.py):
# GPU parity tests + bench lines per config (CONFIGS, default "3");
# "base" is the in-tree library.
mkdir -p gpurun_out
# A variant named env:NAME=VALUE sets that environment variable on the in-tree library.
for v in base ${VARIANTS}; do
  unset PT_HIP_LIB PT_NODE_ALIGN PT_ROUND_FUSED PT_STACK16 PT_BLAS_WORDS
  case "$v" in
    base) ;;
    env:*) export "${v#env:}";;
    *) export PT_HIP_LIB=$GRAFT_REPO_ROOT/build/variants/$v.so;;
  esac
  case " ${TIMING_ONLY} " in
    *" $v "*) echo "tests $v skipped (timing-only variant)";;
    *) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > "gpurun_out/ab_tests_$v.log" 2>&1; rc=$?; echo "tests $v rc=$rc: $(tail -1 "gpurun_out/ab_tests_$v.log")"
       [ $rc -eq 0 ] || exit $rc;;
  esac
  for c in ${CONFIGS:-3}; do
    for rep in 1 2; do
      timeout -k 10 300 python bench.py --config $c --steps 64 --warmup 4 --no-cpu-baseline > "gpurun_out/ab_bench_$v.log" 2>&1; rc=$?
      [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; exit $rc; }
      python -c "import json;d=json.loads(open('gpurun_out/ab_bench_$v.log').read().strip().splitlines()[-1]);print('$v C$c',d['value'],d['roofline']['launch_avg_ms'])"
    done
  done
done
