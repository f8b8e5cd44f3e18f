# Global per-class shade lists, two ways of building them:
# build/variants/classq1.so (-DPT_EXP_CLASSQ=1: a list kernel between extend and
# shade, one list per class, 16 tiles per block) and classq8.so (=2: extend's
# last wave of each tile appends the tile, 8 sub-lists per class).  Bit-exact
# checks on C2 / C5 (the experiment instantiates the non-grey shade kernels
# only), C2 / C5 A/B against the in-tree build, then kernel-trace stats.
set -e
R=$PWD
O=gpurun_out/r05_classq; mkdir -p $O
for v in classq1 classq8; do
PT_HIP_LIB=$R/build/variants/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread \
  -k "(slot_state and (2-96 or 5-128)) or (full_size and (2-1024 or 5-2048)) or diffuse_metal or (image_rel and (2-96 or 5-128))" \
  > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
tail -1 $O/tests_$v.log
done
STEPS=3 bash tools/r04/gpu_ab.sh r05_classq_c2 2 2 base classq1 classq8
STEPS=2 bash tools/r04/gpu_ab.sh r05_classq_c5 5 2 base classq1 classq8
cd /tmp && export TMPDIR=/tmp
for c in 2 5; do
  for v in base classq1 classq8; do
    if [ "$v" = base ]; then L=$R/path-tracer_amd/libpathtracer.so; else L=$R/build/variants/$v.so; fi
    PT_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_${v}_c$c -o run -- \
      python3 $R/bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-steady > $R/$O/trace_${v}_c$c.log 2>&1
    find $R/$O -name "*kernel_trace.csv" -delete
  done
done
cd $R
export PT_HIP_LIB=$R/build/variants/classq1.so
for c in 2 5; do
  bash tools/r04/gpu_pmc.sh r05_classq/pmc_classq1_c$c python3 $R/tools/run_rounds.py --config $c --settle 34 --rounds 32
  find $O/pmc_classq1_c$c -name "*.csv" -delete
done
find $O -name "*.db" -delete
