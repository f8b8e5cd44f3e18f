# Long parity runs of the tile-group schedule against the oracle: the 24 fuzz
# scenes (320x240, 400 rounds, three forced groups), C2's whole 256-spp
# frame's rounds (653) and 400 rounds of C5, all in 50-round batches.
set -u
O=gpurun_out/${TAG:-r05_long_split2}
mkdir -p "$O"
for s in $(seq 0 23); do
  timeout -k 10 200 python3 -u tools/long_parity.py fuzz:$s 400 --batched --split 3 > "$O/fuzz_$s.json" 2> "$O/fuzz_$s.err" \
    || { echo "fuzz $s FAILED"; tail -5 "$O/fuzz_$s.err"; exit 1; }
done
echo fuzz done
timeout -k 10 400 python3 -u tools/long_parity.py 2 653 --batched > "$O/c2_653.json" 2> "$O/c2_653.err" || { echo C2 FAILED; tail -5 "$O/c2_653.err"; exit 1; }
timeout -k 10 400 python3 -u tools/long_parity.py 5 400 --batched > "$O/c5_400.json" 2> "$O/c5_400.err" || { echo C5 FAILED; tail -5 "$O/c5_400.err"; exit 1; }
python3 - "$O" <<'PY'
import json, glob, sys
bad = 0
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f))
    m = sum(d["state_mismatch_px"].values()) + d["accum_mismatch_px"]
    bad += m
    print(f.split("/")[-1], d["config"], d["rounds"], d.get("split"), "mismatch", m)
print("total mismatching pixel fields:", bad)
PY
