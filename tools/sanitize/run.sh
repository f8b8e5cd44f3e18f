# Host sanitizer run: ASan+UBSan over every file decoder and
# the oracle, TSan over the threaded BVH builder and the oracle's threads.
# CPU only.  usage: bash tools/sanitize/run.sh OUT_DIR   (log: OUT_DIR/summary.txt)
set -u
R=$(cd "$(dirname "$0")/../.." && pwd)
O=${1:-/tmp/san_run}
mkdir -p "$O"
make -s -C "$R/tools/sanitize" all || exit 1
A=$R/tools/sanitize/_build/san_driver_asan
T=$R/tools/sanitize/_build/san_driver_tsan
C=$O/corpus
rm -rf "$C"
python "$R/tools/sanitize/make_corpus.py" "$C" > "$O/corpus.log" 2>&1 || { cat "$O/corpus.log"; exit 1; }
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:halt_on_error=1:max_allocation_size_mb=3000:allocator_may_return_null=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1
export PT_SPECTRUM_TABLE=$O/sRGBSpectrumTable.dat
fails=0
run() {   # run NAME CMD...: one process; non-zero status or a sanitizer report = failure
  local name=$1; shift
  "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  if [ $rc -ne 0 ] || grep -qE "ERROR: (Address|Thread|Leak)Sanitizer|runtime error:|WARNING: ThreadSanitizer" "$O/$name.err"; then
    echo "FAIL $name rc=$rc"; tail -30 "$O/$name.err"; fails=$((fails+1))
  else
    echo "ok   $name ($(wc -l < "$O/$name.out") lines)"
  fi
}
# images in batches of 100 files (a failing batch is re-run file by file)
ls "$C/images" | sort > "$O/images.lst"
split -l 100 "$O/images.lst" "$O/batch."
for b in "$O"/batch.*; do
  n=$(basename "$b")
  run "asan_decode_$n" "$A" decode $(sed "s|^|$C/images/|" "$b")
done
run asan_models "$A" model $(ls -d "$C"/models/m*/ | while read d; do ls "$d"*.obj; done) "$C"/models/*.obj
run asan_scenes "$A" scene $(ls -d "$C"/scenes/s*/ | sed 's|$|scene.json|') "$C/scenes/src/scene.json"
run asan_render "$A" render
PT_BVH_THREADS=8 run tsan_bvh "$T" bvh 300000
run tsan_render "$T" render
PT_BVH_THREADS=8 run asan_bvh "$A" bvh 200000
cat "$O"/asan_decode_*.out > "$O/decode_results.txt"
{
  echo "host sanitizer run: $(date -u +%Y-%m-%dT%H:%MZ), $(g++ --version | head -1)"
  cat "$O/corpus.log"
  echo "decode: $(grep -c ': ok ' "$O/decode_results.txt") decoded, $(grep -c ': error: ' "$O/decode_results.txt") rejected with an error, $(grep -c 'disagrees' "$O/decode_results.txt") float-path disagreements"
  echo "models: $(grep -c ': ok' "$O/asan_models.out") loaded, $(grep -c ': error' "$O/asan_models.out") rejected"
  echo "scenes: $(grep -c ': ok' "$O/asan_scenes.out") loaded, $(grep -c ': error' "$O/asan_scenes.out") rejected"
  echo "huge-header files:"; grep "/huge\|short_raw" "$O/decode_results.txt" | sed "s|$C/images/||"
  echo "sanitizer failures: $fails"
} > "$O/summary.txt"
cat "$O/summary.txt"
exit $fails
