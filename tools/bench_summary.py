#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (development helper)."""
import json
import sys

d = json.load(open(sys.argv[1]))
print("value %.4g %s  ms/step %.4f  e2e %.4f" % (d["value"], d["unit"], d["ms_per_step"], d.get("e2e_ms_median", 0)))
print("stage_ms", d.get("stage_ms"))
print("device_ms", d.get("device_ms"), "parity", d.get("parity"))
print("in_batch", d.get("stage_ms_in_batch"))
r = d.get("roofline") or {}
print("roofline", r.get("kernel"), "frac %.4f achieved %.1f GB/s" % (r.get("frac", 0), r.get("achieved", 0)))
for k, v in sorted((d.get("kernel_table") or {}).items(), key=lambda kv: -kv[1]["ms_per_step"]):
    print("  %-16s %8.4f ms/step  %8.2f us/launch  %6.1f launches" % (k, v["ms_per_step"], v["avg_launch_us"],
                                                                      v["launches_per_step"]))
