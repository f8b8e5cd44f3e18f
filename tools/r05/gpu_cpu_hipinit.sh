# Is the bench's faster CPU baseline the HIP runtime's doing?  cpu_scaling at
# 16 threads without and with a HIP device created first, alternating.
set -e
O=gpurun_out/r05_cpu2; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python tools/cpu_scaling.py $O/plain_$i.json --threads 16 > $O/plain_$i.log 2>&1
  timeout -k 10 200 python tools/cpu_scaling.py $O/hip_$i.json --threads 16 --init-gpu > $O/hip_$i.log 2>&1
  python3 -c "import json; [print(n, json.load(open('$O/'+n+'_$i.json'))['rows'][0]['mrays_per_s']) for n in ('plain','hip')]"
done
