"""Dev: path counters and round records of K1's sort on the c3 source cloud's leaf keys
(one cloud, fccf_debug_sort_keys).  Usage: python tools/sort_stats.py [cfg]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fccf-pcr_amd"), os.path.join(ROOT, "tools")]
import fccf_amd as F  # noqa: E402
from is_bench import leaf_keys  # noqa: E402

c = F.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
for which, (src, tar, _) in (("src", F.synth_pair(c["n"], c["room"])),):
    k = leaf_keys(src, c["leaf"])
    with F.Ctx(0) as ctx:
        ctx.sort_keys(k)
        st = ctx.sort_stats()
        st.pop("raw")
        print(which, len(k), st)
        r = ctx.sort_rounds()
        print("rounds {segments, tiles, owned, elements}:")
        for i, row in enumerate(r):
            if row.any():
                print(" ", i, list(map(int, row)))
