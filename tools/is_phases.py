"""Phase profile of the IS_PH-instrumented kernel (k_is_scatter_s; development): cycles per phase from a variant build
(make VAR=ph EXTRA=-DIS_PHASES; FCCF_LIB=fccf-pcr_amd/lib_ph/libfccf.so).
Usage: FCCF_LIB=... python tools/is_phases.py [config]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fccf-pcr_amd"))
import fccf_amd as F  # noqa: E402

cfg = F.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
names = ["sc:desc+tile+prefix", "sc:ballots+bar", "sc:chunkscan+bar", "sc:dest+stores", "sc:cut+bar", "ct:plan", "ct:tile+median+desc", "ct:ballots+bar", "ct:chunkscan+bar", "ct:lists"]
with F.Ctx(0) as c:
    fn = F._lib.fccf_debug_is_phases
    fn.argtypes = [ctypes.c_void_p]
    ds, dt = c.upload(src), c.upload(tar)
    c.register_device(ds, src.shape[0], dt, tar.shape[0], cfg["leaf"])
    out = np.zeros(32, np.uint64)
    fn(out.ctypes.data)
    for _ in range(5):
        c.register_device(ds, src.shape[0], dt, tar.shape[0], cfg["leaf"])
    fn(out.ctypes.data)
    cyc, cnt = out[:16].astype(float) / 5, out[16:].astype(float) / 5
    tot = cyc.sum()
    for i in range(10):
        if cnt[i]:
            print(f"{names[i]:14s} count {cnt[i]:9.0f}  cycles/event {cyc[i] / cnt[i]:9.0f}  share {cyc[i] / tot:6.1%}")
    print(f"total cycles per registration (summed over workgroups) {tot:.3e}")
