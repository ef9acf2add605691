"""Print the kernel timeline of one registration in a rocprofv3 rocpd database.

Usage: python tools/trace_reg.py <run_results.db> [registration_index] [--brief]
A registration starts at its first first-pass VoxelGrid bbox kernel (k_vg_bbox,
4 launches per registration: 2 passes x 2 clouds).  Index -1 = the last one.
--brief prints per-kernel totals and the per-stream busy time instead of every launch.
"""
import re
import sqlite3
import sys

db = sys.argv[1]
idx = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else -1
brief = "--brief" in sys.argv
c = sqlite3.connect(db)
rows = list(c.execute("select name, stream_id, start, end from kernels order by start"))
starts = [i for i, r in enumerate(rows) if "k_vg_bbox" in r[0]][::4]
i0 = starts[idx]
i1 = starts[idx + 1] if idx != -1 and idx + 1 < len(starts) else len(rows)
reg = rows[i0:i1]
t0 = reg[0][2]


def short(n):
    m = re.search(r"(k_\w+|__amd\w+)(<[^>]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:40]


busy, tot = {}, {}
for name, sid, s, e in reg:
    if not brief:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  s{sid:<3} {short(name)}")
    busy[sid] = busy.get(sid, 0) + (e - s)
    k = short(name)
    n, d = tot.get(k, (0, 0))
    tot[k] = (n + 1, d + e - s)
if brief:
    for k, (n, d) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:40s} {n:4d} {d / 1e3:9.1f} us")
print("registrations", len(starts), "span us", (max(r[3] for r in reg) - t0) / 1e3,
      "busy per stream us", {k: round(v / 1e3, 1) for k, v in busy.items()})
