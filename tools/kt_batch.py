"""Dev: per-kernel durations of a rocprofv3 kernel trace split by batch width
(Grid_Size_Y = clouds per launch).  Usage: python tools/kt_batch.py TRACE_DIR OUT.txt"""
import collections
import csv
import glob
import re
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
acc = collections.defaultdict(list)
for r in rows:
    gy = int(r.get("Grid_Size_Y", "1"))
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    if not m:
        continue
    acc[(m.group(1), gy)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
with open(sys.argv[2], "w") as out:
    for (k, gy), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        out.write(f"{k:24s} y={gy} n={len(v):5d} avg {sum(v) / len(v):8.2f} us total {sum(v) / 1e3:8.2f} ms\n")
