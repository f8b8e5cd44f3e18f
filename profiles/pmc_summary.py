import csv, collections, sys, json
def load(path):
    rows=list(csv.DictReader(open(path)))
    per=collections.defaultdict(float); kn={}
    for r in rows:
        key=(r["Dispatch_Id"], r["Counter_Name"]); per[key]+=float(r["Counter_Value"]); kn[r["Dispatch_Id"]]=r["Kernel_Name"]
    agg=collections.defaultdict(lambda: collections.defaultdict(list))
    for (d,c),v in per.items(): agg[kn[d]][c].append(v)
    return {k:{c:sum(v)/len(v) for c,v in d.items()} for k,d in agg.items()}
out={}
for p in sys.argv[1:]:
    for k,d in load(p).items():
        out.setdefault(k,{}).update(d)
for k,d in out.items():
    if "extend" in k or "shade" in k:
        print(k, json.dumps({c: round(v,1) for c,v in d.items()}))
