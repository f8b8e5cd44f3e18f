# Frame loop with a read-back-free first batch and guarded last rounds: the
# whole GPU suite (whole-frame bit-exactness and minimality included), then
# bench A/B against the old loop (build/variants/noguard.so) on C1, C3, C2.
set -e
O=gpurun_out/r05_guard; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
STEPS=20 bash tools/r04/gpu_ab.sh r05_guard_c1 1 2 base noguard
bash tools/r04/gpu_ab.sh r05_guard_c3 3 2 base noguard
STEPS=5 bash tools/r04/gpu_ab.sh r05_guard_c2 2 1 base noguard
for f in $O/../r05_guard_c*/ab_*.log; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-2:], d['value'], d['frame']['rounds_per_frame_rank0'][:3], d['frame']['samples_per_frame_rank0'][:2])" $f; done
