#!/usr/bin/env python3
"""Short per-kernel summary (calls, total, mean, max in us) of a rocprofv3 rocpd db."""
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
agg = {}
for name, d in con.execute("select name, duration from kernels"):
    short = name.replace("fccf::(anonymous namespace)::", "").replace("(anonymous namespace)::", "").split("(")[0]
    agg.setdefault(short, []).append(d)
tot = sum(sum(v) for v in agg.values())
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[: int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    print(f"{k[:48]:48s} n {len(v):5d} tot {sum(v) / 1e3:10.1f} us  avg {sum(v) / len(v) / 1e3:8.2f}  max {max(v) / 1e3:8.2f}  {100 * sum(v) / tot:5.1f}%")
