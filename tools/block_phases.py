"""Dev: phase cycles of the block kernel's items (IS_PHASES variant build, lds_block's
IS_PH(10..13): load, partitions, task list, leaves + write-back) over the c3 keys'
sorts.  Usage: FCCF_LIB=fccf-pcr_amd/lib_<ph>/libfccf.so python tools/block_phases.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fccf-pcr_amd"), os.path.join(ROOT, "tools")]
import fccf_amd as F  # noqa: E402
from is_bench import leaf_keys  # noqa: E402

names = {10: "load", 11: "load + partitions", 12: "task list", 13: "leaves + write-back"}
src, _, _ = F.synth_pair(1_000_000, (20.0, 15.0, 4.0))
k = leaf_keys(src, 0.05)
fns = [F._lib.fccf_debug_is_phases, F._lib.fccf_debug_is_phases_b2]  # (the block kernel's two forms)
for f in fns:
    f.argtypes = [ctypes.c_void_p]
out = np.zeros(32, np.uint64)


def fn(o):
    o[:] = 0
    t = np.zeros(32, np.uint64)
    for f in fns:
        f(t.ctypes.data)
        o += t
with F.Ctx(0) as ctx:
    ctx.sort_keys(k)
    fn(out)
    reps = 5
    for _ in range(reps):
        ctx.sort_keys(k)
    fn(out)
cyc, cnt = out[:16].astype(float) / reps, out[16:].astype(float) / reps
for i in range(10, 14):
    if cnt[i]:
        print(f"{names[i]:20s} items {cnt[i]:6.0f}  cycles/item {cyc[i] / cnt[i]:9.0f}  sum {cyc[i]:.3g}")
