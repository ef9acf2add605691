"""Dev probe: host vs GPU forms of the serial stages at a config -- K4 growth
(fccf_ctx_set_grow_device), quick_verify + LM (fccf_ctx_set_lm_device) and the
clustering (fccf_ctx_set_cluster_device): median grow / match+cluster / verify stage
ms, single-registration ms and pipelined ms per registration.
Usage: python tools/grow_ab.py [config] [reps]"""
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fccf-pcr_amd"))
import fccf_amd as F  # noqa: E402

cfg = F.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
ctx = F.Ctx(0)
ds, dt = ctx.upload(src), ctx.upload(tar)
ref = None
MODES = [("host", False, False, False), ("grow_dev", True, False, False), ("lm_dev", False, True, False),
         ("clus_dev", False, False, True)] * 2
for name, gdev, ldev, cdev in MODES:
    ctx.set_grow_device(gdev)
    ctx.set_lm_device(ldev)
    ctx.set_cluster_device(cdev)
    for _ in range(3):
        ctx.register_device(ds, len(src), dt, len(tar), cfg["leaf"])
    g, e, v, mc = [], [], [], []
    for _ in range(reps):
        a = time.perf_counter()
        T, st = ctx.register_device(ds, len(src), dt, len(tar), cfg["leaf"])
        e.append((time.perf_counter() - a) * 1e3)
        g.append(st.ms[2])
        v.append(st.ms[6])
        mc.append(st.ms[4] + st.ms[5])
    ref = T if ref is None else ref
    assert np.array_equal(T.view(np.uint32), ref.view(np.uint32))
    a = time.perf_counter()
    ctx.register_batch([((ds, len(src)), (dt, len(tar)))] * reps, cfg["leaf"], on_device=True)
    pb = (time.perf_counter() - a) / reps * 1e3
    print(f"{name:9s}: vox {st.vox1}/{st.vox2} lm {st.lm_solves} grow {statistics.median(g):.4f} ms  "
          f"match+cluster {statistics.median(mc):.4f} ms  verify {statistics.median(v):.4f} ms  "
          f"e2e {statistics.median(e):.3f} ms  pipelined {pb:.3f} ms/reg", flush=True)
