"""Dev: per-round durations of K1's sort rounds from a rocprofv3 kernel trace.

Launches of k_is_count_plan_s / k_is_scatter_s (and the large forms) at one launch width
(Grid_Size_Y) are numbered by their position after the preceding k_is_prep of the same
width on the same queue; prints the mean duration per round index, plus the finish kernels.

Usage: python tools/round_times.py TRACE_DIR [WIDTH]"""
import collections
import csv
import glob
import re
import sys

width = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
per = collections.defaultdict(list)
fin = collections.defaultdict(list)
rnd = {}
for r in rows:
    if int(r.get("Grid_Size_Y", "1")) != width:
        continue
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    if not m:
        continue
    k = m.group(1)
    q = r.get("Queue_Id", "0")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if k == "k_is_prep":
        rnd[q] = 0
    elif k.startswith("k_is_count_plan"):
        per[(rnd.get(q, 0), "count")].append(d)
    elif k.startswith("k_is_scatter"):
        per[(rnd.get(q, 0), "scatter")].append(d)
        rnd[q] = rnd.get(q, 0) + 1
    elif k in ("k_is_block", "k_is_wave"):
        fin[k].append(d)
tot = 0.0
print(f"width {width}: round  count_us  scatter_us  (launches)")
for i in range(max([k[0] for k in per] + [-1]) + 1):
    c, s = per.get((i, "count"), []), per.get((i, "scatter"), [])
    mc = sum(c) / len(c) if c else 0.0
    ms = sum(s) / len(s) if s else 0.0
    tot += mc + ms
    print(f"  {i:2d}  {mc:8.2f}  {ms:8.2f}  ({len(c)}, {len(s)})")
print(f"  rounds total {tot:.1f} us per stage")
for k, v in fin.items():
    print(f"  {k:12s} {sum(v) / len(v):8.2f} us  ({len(v)})")
