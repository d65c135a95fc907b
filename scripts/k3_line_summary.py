"""One line from a K3 bench json: label, ms per pair, isolated query stage,
isolated build and per-kernel isolated times (A/B sessions)."""
import json
import sys

d = json.load(open(sys.argv[2]))
r = d["roofline"]
print(sys.argv[1], d["ms_per_step"], r.get("avg_us_isolated"), r["build"].get("avg_us_isolated"),
      d.get("kernel_us_isolated"))
