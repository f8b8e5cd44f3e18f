# Tile-order sort period A/B on C3 / C5 / C2 (bench, interleaved, twice),
# after the parity tests of the current build.
set -u
O=gpurun_out/period_ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for cfg in 3 5 2; do for p in 16 4 1; do
  PT_TILE_ORDER_PERIOD=$p timeout -k 10 120 python bench.py --config $cfg --steps 64 --warmup 8 --no-cpu-baseline > $O/b_${cfg}_${p}_$rep.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
  python -c "import json;d=json.loads(open('$O/b_${cfg}_${p}_$rep.log').read().strip().splitlines()[-1]);print('C$cfg period=$p rep=$rep',d['value'],d['roofline']['launch_avg_ms'])"
done; done; done
