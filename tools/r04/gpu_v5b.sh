O=gpurun_out/r04_v5; mkdir -p $O
timeout -k 10 300 python -u tools/shade_stats.py $O/shade_stats.json 2 3 5 > $O/stats.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config 2 --steps 10 --warmup 2 --no-cpu-baseline > $O/c2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config 5 --spp 1024 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/c3.log 2>&1 || exit 1
for c in c2 c5 c3; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['roofline']['launch_avg_ms'])" $O/$c.log; done
timeout -k 10 400 python -u tools/rehearse_scaling.py $O/rehearse.json --steps 48 --configs 3,4 --ns 1,2,4,8 > $O/rehearse.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/rehearse_scaling.py $O/rehearse_k1.json --steps 48 --configs 3,4 --ns 8 --streams 1 > $O/rehearse_k1.log 2>&1 || exit 1
python3 -c "import json,sys; [print(r['config'], r['n_gpus'], r['streams'], r['rank0_mrays_per_s'], r.get('predicted_efficiency'), r['kernel_ms_per_round']) for f in sys.argv[1:] for r in json.load(open(f))['rows']]" $O/rehearse.json $O/rehearse_k1.json
