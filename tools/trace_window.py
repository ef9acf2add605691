"""Print every kernel (stream, start, end, name) of a rocprofv3 rocpd db between
two occurrences of a marker kernel (development).

Usage: python tools/trace_window.py run_results.db [marker=k_vg_bbox] [first_occurrence] [count]
"""
import re
import sqlite3
import sys

db = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_vg_bbox"
first = int(sys.argv[3]) if len(sys.argv) > 3 else 40
count = int(sys.argv[4]) if len(sys.argv) > 4 else 8
c = sqlite3.connect(db)
rows = list(c.execute("select name, stream_id, start, end from kernels order by start"))
idx = [i for i, r in enumerate(rows) if marker in r[0]]
i0, i1 = idx[first], idx[min(first + count, len(idx) - 1)]
t0 = rows[i0][2]
for name, sid, s, e in rows[i0:i1]:
    m = re.search(r"(k_\w+|__amd\w+)", name)
    print(f"s{sid} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {m.group(1) if m else name[:30]}")
