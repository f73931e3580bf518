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
