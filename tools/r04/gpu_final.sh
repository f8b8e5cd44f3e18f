# Round 4's final measurement call: GPU tests, smoke, the driver's bench command
# with the CPU baseline and under rocprofv3 --kernel-trace --stats, bench lines
# of C1 / C2 / C5 (8192 spp) / C4, steady-state PMC passes of C2 / C3 / C5 and
# the CPU baseline's thread scaling.
set -e
bash tools/gpu.sh r04_fin tests smoke benchcpu trace cfg=1 bench cfg=2 args=--steps,5,--warmup,1 bench \
  cfg=5 args=--steps,3,--warmup,1 bench cfg=4 args=--steps,2,--warmup,1 bench
P="python3 $PWD/tools/run_rounds.py"
for c in 2 3 5; do bash tools/r04/gpu_pmc.sh r04_fin/pmc_c$c $P --config $c --settle 34 --rounds 32; done
timeout -k 10 300 python3 tools/cpu_scaling.py gpurun_out/r04_fin/cpu_scaling.json > gpurun_out/r04_fin/cpu_scaling.log 2>&1
tail -2 gpurun_out/r04_fin/cpu_scaling.log | cut -c1-600
