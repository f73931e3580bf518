#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 PMC passes (scripts/pmc.sh):
FETCH_SIZE (KiB, doubled: gfx950 reports half of wide streaming reads, per
MI355X_MICROARCH.md) + WRITE_SIZE (KiB). Writes profiles/traffic_<tag>.json
in the form bench.py reads (keyed by the runtime's kernel names)."""
import collections
import csv
import json
import re
import sys

fetch_csv, write_csv, out, records, workload = sys.argv[1:6]


# kernel symbol -> the runtime's kernel id name (runtime.K_NAMES): both
# enc_emit kernels (wave-per-tile enc_emit_kernel_t, wave-specialised
# enc_emit_ws_kernel) are the ONC_K_ENC_EMIT launch
ALIASES = {"enc_emit_ws_kernel": "enc_emit_kernel"}


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("onc::", "")
    n = re.sub(r"_t$", "", re.sub(r"<.*>$", "", n))
    return ALIASES.get(n, n)


res = collections.defaultdict(dict)
syms = collections.defaultdict(set)
for path, counter in ((fetch_csv, "FETCH_SIZE"), (write_csv, "WRITE_SIZE")):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if "onc::" not in r["Kernel_Name"]:
            continue
        vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        syms[short(r["Kernel_Name"])].add(r["Kernel_Name"].split("(")[0].replace("void ", ""))
    for k, v in vals.items():
        res[k][counter + "_KiB_avg"] = sum(v) / len(v)
        res[k]["dispatches"] = len(v)
kernels = {}
for k, v in res.items():
    f = v.get("FETCH_SIZE_KiB_avg", 0.0) * 1024 * 2
    w = v.get("WRITE_SIZE_KiB_avg", 0.0) * 1024
    kernels[k] = {"fetch_bytes_corrected": f, "write_bytes": w, "hbm_bytes_per_launch": f + w, **v,
                  "symbols": sorted(syms[k])}
doc = {"records": int(records), "workload_id": workload,
       "method": "rocprofv3 --kernel-trace --pmc <one counter> per pass (scripts/pmc.sh); FETCH_SIZE and "
                 "WRITE_SIZE in KiB; FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports 1/2 of wide "
                 "streaming reads); calibration: every fabric read request is 128 B and FETCH_SIZE counts "
                 "64 B per request for scattered window reads too (profiles/calib_r02_fetch_size.json), so "
                 "FETCH_SIZE x 2 is exact here",
       "kernels": kernels}
json.dump(doc, open(out, "w"), indent=1)
print(json.dumps({k: round(v["hbm_bytes_per_launch"] / 1e6, 1) for k, v in kernels.items()}))
