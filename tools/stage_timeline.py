"""Dev: the kernels of one steady-state cloud stage of a pipelined batch, from a
rocprofv3 kernel trace (csv): start offset, duration, workgroups, clouds per launch,
with the gaps between consecutive kernels on the stage's stream and the kernels of
other streams that overlap it.
Usage: python tools/stage_timeline.py TRACE_DIR [which=3]"""
import csv
import glob
import re
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
which = int(sys.argv[2]) if len(sys.argv) > 2 else 3


def short(n):
    m = re.search(r"(k_\w+|__amd\w+)", n)
    return m.group(1) if m else n[:30]


ks = []
for r in rows:
    wg = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", "1")) or 1)
    gx = int(r.get("Grid_Size_X", r.get("Grid_Size", "1")) or 1)
    ks.append(dict(name=short(r["Kernel_Name"]), s=int(r["Start_Timestamp"]), e=int(r["End_Timestamp"]),
                   q=r.get("Queue_Id", r.get("Stream_Id", "?")), gy=int(r.get("Grid_Size_Y", "1")), wgs=gx // max(1, wg)))
ks.sort(key=lambda k: k["s"])
starts = [i for i, k in enumerate(ks) if k["name"] == "k_vg_bbox" and k["gy"] == 8]
# stage starts: a k_vg_bbox of 8 clouds whose predecessor is not a k_vg_bbox-of-the-same stage (pass 1)
stage = [i for j, i in enumerate(starts) if j % 2 == 0]
i0 = stage[min(which, len(stage) - 1)]
i1 = next(i for i in range(i0 + 1, len(ks)) if ks[i]["name"] == "k_compact_planar" and ks[i]["gy"] == 8)
t0 = ks[i0]["s"]
q0 = ks[i0]["q"]
print(f"stage from {ks[i0]['name']} to {ks[i1]['name']}: {(ks[i1]['e'] - t0) / 1e3:.1f} us")
prev_e = t0
for k in ks:
    if k["e"] < t0 or k["s"] > ks[i1]["e"]:
        continue
    same = k["q"] == q0
    gap = (k["s"] - prev_e) / 1e3 if same else 0.0
    if same:
        prev_e = k["e"]
    print(f"{(k['s'] - t0) / 1e3:9.1f} {(k['e'] - k['s']) / 1e3:8.1f} {'' if same else '  *'}{k['name']:24s} "
          f"wg {k['wgs']:6d} y {k['gy']}  {'gap %.1f' % gap if same and gap > 1.0 else ''}")
