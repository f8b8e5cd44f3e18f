# Parity of the shade completion-queue variants, then A/B on C3 / C2 / C5.
O=gpurun_out/r04_ab3; mkdir -p $O
for v in compact compact2; do
  PT_HIP_LIB=$PWD/build/variants/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/${v}_tests.log 2>&1; rc=$?
  echo "$v tests rc=$rc: $(tail -1 $O/${v}_tests.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/r04/gpu_ab.sh r04_ab3 3 2 base uvall compact compact2 || exit 1
bash tools/r04/gpu_ab.sh r04_ab3c2 2 2 base uvall compact compact2 || exit 1
STEPS=2 ARGS="--spp 1024" bash tools/r04/gpu_ab.sh r04_ab3c5 5 2 base uvall compact compact2
