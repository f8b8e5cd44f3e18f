# PMC passes (tools/r04/gpu_pmc.sh) over settled rounds of the tile-group
# build (automatic split: three groups on full frames, so a launch covers one
# group's tiles): C3, C2, C5, C4 whole frame, C4 rank 0 of 8 with two path
# streams.  The split tests first.
set -e
O=gpurun_out/r05_pmc2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/split_tests.log 2>&1 || { tail -30 $O/split_tests.log; exit 1; }
tail -1 $O/split_tests.log
P="python3 $PWD/tools/run_rounds.py"
bash tools/r04/gpu_pmc.sh r05_pmc2/c3 $P --config 3 --settle 34 --rounds 32
bash tools/r04/gpu_pmc.sh r05_pmc2/c2 $P --config 2 --settle 34 --rounds 32
bash tools/r04/gpu_pmc.sh r05_pmc2/c5 $P --config 5 --settle 34 --rounds 32
bash tools/r04/gpu_pmc.sh r05_pmc2/c4 $P --config 4 --settle 16 --rounds 16
bash tools/r04/gpu_pmc.sh r05_pmc2/c4_bands8x2 $P --config 4 --rank 0 --nranks 8 --streams 2 --settle 34 --rounds 32
find $O -name "*.csv" -delete
find $O -name "*.db" -delete
