"""rocprofv3 counter_collection CSVs -> per-kernel means of every counter
(values summed over the counter's dimensions per dispatch, then averaged
over dispatches). Usage: python scripts/sq_json.py out.json method a.csv [b.csv ...]"""
import csv
import json
import sys
from collections import defaultdict

out, method, files = sys.argv[1], sys.argv[2], sys.argv[3:]
per = defaultdict(lambda: defaultdict(float))      # (kernel, dispatch) -> counter -> value
for f in files:
    with open(f) as fh:
        for r in csv.DictReader(fh):
            per[(r["Kernel_Name"], f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
agg = defaultdict(lambda: defaultdict(list))
for (k, _, _), cs in per.items():
    for c, v in cs.items():
        agg[k][c].append(v)
res = {"method": method, "kernels": {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}}
json.dump(res, open(out, "w"), indent=1)
for k, cs in res["kernels"].items():
    w = cs.get("SQ_WAVES", 0) or 1
    print(k[:70], {c: round(v / w, 1) for c, v in cs.items() if c.startswith("SQ_INSTS")}, "waves", w)
