# Round 6: extend blocks per CU under tile groups -- unused dynamic LDS on the
# node-cache extend launch (2.5 KB: 7 blocks per CU, 6 KB: 6) leaves room for
# the other groups' shade blocks; same-box A/B against the in-tree build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/r06/gpu_ab_lib.sh ${1:-r06_pad} "3 4" base pad7 pad6
