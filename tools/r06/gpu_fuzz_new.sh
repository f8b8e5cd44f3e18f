# 32 fuzz scenes never run before (seeds 24-55; tests use 0-23): 320x240,
# 300 rounds each in three forced tile groups (50-round batches), every slot
# field and pixel against the oracle.
set -u
O=gpurun_out/${TAG:-r06_fuzz_new}
mkdir -p "$O"
for s in $(seq 24 55); do
  timeout -k 10 200 python3 -u tools/long_parity.py fuzz:$s 300 --batched --split 3 > "$O/fuzz_$s.json" 2> "$O/fuzz_$s.err" \
    || { echo "fuzz $s FAILED"; tail -5 "$O/fuzz_$s.err"; exit 1; }
done
python3 - "$O" <<'PY'
import json, glob, sys
bad = 0
rows = []
for f in sorted(glob.glob(sys.argv[1] + "/fuzz_*.json")):
    d = json.load(open(f))
    m = sum(d["state_mismatch_px"].values()) + d["accum_mismatch_px"]
    bad += m
    rows.append({"file": f.split("/")[-1], "rounds": d["rounds"], "split": d.get("split"),
                 "class_lists": d.get("class_lists"), "mismatch": m})
    print(f.split("/")[-1], d["rounds"], d.get("split"), d.get("class_lists"), "mismatch", m)
print("total mismatching pixel fields:", bad)
json.dump({"scenes": rows, "total_mismatch": bad}, open(sys.argv[1] + "/summary.json", "w"), indent=1)
PY
