# Reorder experiment under two extend variants (in-kernel octant sort on/off).
set -u
R=$GRAFT_REPO_ROOT
for v in ${VARIANTS:-0 4}; do
  O=$R/gpurun_out/reorder_v$v
  mkdir -p "$O"
  (cd /tmp && export TMPDIR=/tmp && PT_EXTEND_VARIANT=$v timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o run -- python3 $R/tools/exp_reorder.py 8 > "$O/run.log" 2>&1)
  rc=$?; echo "v$v run rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/run.log"; exit $rc; }
  grep -c MISMATCH "$O/run.log" || true
  cd "$R" && python3 tools/exp_reorder_report.py "$O/trace"
done
