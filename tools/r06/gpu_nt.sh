# Round 6: streaming-hint (non-temporal) slot-record loads/stores, same-box A/B.
set -u
bash tools/r06/gpu_ab_lib.sh ${1:-r06_nt} "3 5 2" base nt_st nt_ld nt_all
