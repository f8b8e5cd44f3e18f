# The round-3 tree (build/r03, commit 6c95f4a, its own bench.py and library)
# against the current one on the same box, interleaved.
O=$PWD/gpurun_out/r04_vs_r03; mkdir -p $O
run() {  # dir tag cfg args
  (cd $1 && timeout -k 10 300 python bench.py --config $3 $4 --warmup 2 --no-cpu-baseline --no-steady > $O/$2_c$3_$5.log 2>&1) || { tail -3 $O/$2_c$3_$5.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['launch_avg_ms'])" $O/$2_c$3_$5.log "$2 C$3"
}
for i in 1 2 3; do run build/r03 r03 3 "--steps 5" $i; run . r04 3 "--steps 5" $i; done
run build/r03 r03 2 "--steps 10" 1; run . r04 2 "--steps 10" 1
run build/r03 r03 5 "--steps 2 --spp 1024" 1; run . r04 5 "--steps 2 --spp 1024" 1
