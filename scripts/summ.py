"""Print value + per-kernel averages of bench JSON lines (dev helper)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    k = d["kernels_breakdown_pass"]
    print(f, round(d["value"], 1), round(d["ms_per_step"] * 1e3, 1), "us/step",
          {n: round(v["avg_us"] * v.get("launches_per_step", 1), 1) for n, v in k.items()}, "us/step per kernel;",
          "frac", round(d["roofline"]["frac"], 3), d["roofline"]["kernel"], round(d["roofline"]["avg_launch_us"], 1), "us")
    p = d.get("pcie_inclusive") or {}
    if p:
        def v(x):
            return None if not x or x.get("value") is None else (round(x["value"], 1), x.get("validated"))
        print("  pcie:", {"serialised": v(p) if "serialised" not in p else v(p["serialised"]),
                          "pipelined": v(p.get("pipelined")), "zero_copy": v(p.get("zero_copy")),
                          "zc_variants": {k: v(x) for k, x in (p.get("zero_copy") or {}).get("variants", {}).items()},
                          "err": (p.get("zero_copy") or {}).get("error") or p.get("error")})
    cb = d.get("cpu_baseline")
    if cb:
        print("  cpu:", round(cb["value"], 1), "on", cb["cores"], "threads; 1 thread", round(cb["single_thread"]["value"], 1))
