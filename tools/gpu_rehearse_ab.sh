# A/B of library variants on rank-0-of-N partitions (tools/rehearse_scaling.py).
# usage: VARIANTS="a b" NS=1,8 CONFIGS=3 bash tools/gpu_rehearse_ab.sh
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/rehearse_ab
mkdir -p "$O"
# A variant named env:NAME=VALUE sets that environment variable on the base library.
for v in base ${VARIANTS:-}; do
  unset PT_HIP_LIB PT_ROUND_FUSED
  case "$v" in
    base) ;;
    env:*) export "${v#env:}";;
    *) export PT_HIP_LIB=$GRAFT_REPO_ROOT/build/variants/$v.so;;
  esac
  for rep in 1 2; do
    timeout -k 10 300 python3 tools/rehearse_scaling.py "$O/$v.$rep.json" --configs ${CONFIGS:-3} --ns ${NS:-1,8} --steps 64 > "$O/$v.$rep.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 "$O/$v.$rep.log"; exit $rc; }
    python3 -c "
import json
for r in json.load(open('$O/$v.$rep.json'))['rows']:
    print('$v', 'C%d N=%d' % (r['config'], r['n_gpus']), r['rank0_ms_per_step'], 'ext', r['extend_ms'], 'sh', r['shade_ms'], 'round', r.get('round_ms'))"
  done
done
