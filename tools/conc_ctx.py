"""Throughput of C independent fccf_ctx pipelines on one GPU (one host thread each).
Usage: python tools/conc_ctx.py [steps] [max_ctx]"""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fccf-pcr_amd"))
import fccf_amd as F  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
cmax = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cfg = F.CONFIGS["c3"]
src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
ctxs = [F.Ctx(0) for _ in range(cmax)]
pairs = []
for c in ctxs:
    pairs.append(((c.upload(src), src.shape[0]), (c.upload(tar), tar.shape[0])))
ref = None
for c, p in zip(ctxs, pairs):  # warm: graphs captured
    T, _ = c.register_batch([p] * 4, cfg["leaf"], on_device=True)
    ref = T[-1] if ref is None else ref
    assert np.array_equal(T[-1].view(np.uint32), ref.view(np.uint32))
for C in range(1, cmax + 1):
    for rep in range(2):
        out = [None] * C
        bar = threading.Barrier(C + 1)

        def work(i):
            bar.wait()
            out[i] = ctxs[i].register_batch([pairs[i]] * steps, cfg["leaf"], on_device=True)

        th = [threading.Thread(target=work, args=(i,)) for i in range(C)]
        for t in th:
            t.start()
        bar.wait()
        t0 = time.perf_counter()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        for o in out:
            assert np.array_equal(o[0][-1].view(np.uint32), ref.view(np.uint32))
        print(f"ctx={C} rep={rep}: {dt / (C * steps) * 1e3:.3f} ms/registration  ({C * steps} regs in {dt * 1e3:.1f} ms)",
              flush=True)
