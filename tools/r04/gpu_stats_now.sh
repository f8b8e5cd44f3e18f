# Shade branch occupancy of the current tree (shadestats build) on C2 / C3 / C5.
set -e
O=gpurun_out/r04_stats_now; mkdir -p $O
timeout -k 10 300 python tools/shade_stats.py $O/stats.json 2 3 5 > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
cat $O/stats.log
