# CPU baseline with pinned threads (bench.pick_cores): the driver's bench
# command with its CPU baseline, then the pinned thread-scaling table
# (1..16 threads, 32 settled rounds each) on the same box.
set -e
O=gpurun_out/r05_cpu3; mkdir -p $O
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log > $O/bench_c3.json
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); print(d['value'], json.dumps(d['cpu_baseline']))"
timeout -k 10 600 python3 -u tools/cpu_scaling.py $O/cpu_scaling.json --threads 16,8,4,2,1 --settle 34 --rounds 32 > $O/cpu_scaling.log 2>&1 || { tail -5 $O/cpu_scaling.log; exit 1; }
grep '"threads"' $O/cpu_scaling.log | cut -c1-200
