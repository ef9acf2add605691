"""Per-kernel means of arbitrary rocprofv3 PMC counters (one or more pass dirs).
Usage: python tools/pmc_sq.py DIR [DIR ...]  -> table of kernel x counter (per-dispatch
mean, dispatches whose SQ_WAVES is 0 or whose counters are all 0 left out)."""
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:30]


acc = {}
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = (short(row["Kernel_Name"]), row["Dispatch_Id"])
                acc.setdefault(k, {})[row["Counter_Name"]] = float(row["Counter_Value"])
by = {}
for (k, _), cs in acc.items():
    if not any(cs.values()):
        continue
    by.setdefault(k, []).append(cs)
names = sorted({c for v in by.values() for cs in v for c in cs})
print("kernel".ljust(22), "n".rjust(4), *[c[:16].rjust(16) for c in names])
for k in sorted(by, key=lambda k: -sum(cs.get("SQ_WAVE_CYCLES", 0) for cs in by[k])):
    v = by[k]
    print(k[:22].ljust(22), str(len(v)).rjust(4),
          *[("%.4g" % (sum(cs.get(c, 0) for cs in v) / len(v))).rjust(16) for c in names])
