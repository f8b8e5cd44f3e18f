set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03_gs
bash tools/gpu.sh r03_gs ab=PT_GLOBAL_SORT=0/1 || exit $?
PT_GLOBAL_SORT=1 timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_gs/gpu_tests_gs.log 2>&1
rc=$?; echo "gs tests rc=$rc"; tail -15 gpurun_out/r03_gs/gpu_tests_gs.log
[ $rc -le 1 ] || exit $rc
bash tools/gpu.sh r03_gs env=PT_GLOBAL_SORT=1 trace
