# Pooled multi-tile shade (PT_SHADE_TILES): parity, then A/B on C5 / C2 / C3.
O=gpurun_out/r04_tiles3; mkdir -p $O
for v in tiles2 tiles4; do
  PT_HIP_LIB=$PWD/build/variants/$v.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/${v}_tests.log 2>&1; rc=$?
  echo "$v tests rc=$rc: $(tail -1 $O/${v}_tests.log)"; [ $rc -eq 0 ] || exit $rc
done
STEPS=2 ARGS="--spp 1024" bash tools/r04/gpu_ab.sh r04_tiles3/c5 5 2 base tiles2 tiles4 || exit 1
bash tools/r04/gpu_ab.sh r04_tiles3/c2 2 2 base tiles2 tiles4 || exit 1
bash tools/r04/gpu_ab.sh r04_tiles3/c3 3 1 base tiles2 tiles4
