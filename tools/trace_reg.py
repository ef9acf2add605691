"""Print the kernel timeline of the last registration in a rocprofv3 rocpd database.

Usage: python tools/trace_reg.py <run_results.db> [first_kernel_substring]
A registration starts at the first-pass VoxelGrid bbox kernel (k_vg_bbox).
"""
import re
import sqlite3
import sys

db = sys.argv[1]
mark = sys.argv[2] if len(sys.argv) > 2 else "k_vg_bbox"
c = sqlite3.connect(db)
rows = list(c.execute("select name, stream_id, start, end from kernels order by start"))
starts = [i for i, r in enumerate(rows) if mark in r[0]]
# 4 bbox launches per registration (2 passes x 2 clouds): take the last registration
i0 = starts[-4]
reg = rows[i0:]
t0 = reg[0][2]
def short(n):
    m = re.search(r"(k_\w+|__amd\w+)(<[^>]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:40]
busy = {}
for name, sid, s, e in reg:
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  s{sid:<3} {short(name)}")
    busy[sid] = busy.get(sid, 0) + (e - s)
print("span us", (reg[-1][3] - t0) / 1e3, "busy per stream us", {k: round(v / 1e3, 1) for k, v in busy.items()})
