# The bench's own CPU baseline and tools/cpu_scaling.py at 16 threads, back to
# back on one box (they should agree within 15 %).
set -e
O=gpurun_out/r05_cpu; mkdir -p $O
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-steady > $O/bench.log 2>&1
grep '^{' $O/bench.log > $O/bench.json
timeout -k 10 300 python tools/cpu_scaling.py $O/cpu_scaling16.json --threads 16,8,16 > $O/cpu_scaling16.log 2>&1
python3 -c "import json; b=json.load(open('$O/bench.json'))['cpu_baseline']; s=json.load(open('$O/cpu_scaling16.json')); print('bench', b['value'], b['sample']); print('scaling', [(r['threads'], r['mrays_per_s']) for r in s['rows']])"
