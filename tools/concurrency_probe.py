"""Throughput of T independent fccf contexts on one GPU, each on its own host
thread running a pipelined batch of B registrations of the c3 pair (development).

Usage (GPU box): python tools/concurrency_probe.py [B] [T ...]
"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fccf-pcr_amd"))
import numpy as np  # noqa: E402
import fccf_amd as F  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 20
Ts = [int(x) for x in sys.argv[2:]] or [1, 2, 3, 4]
c = F.CONFIGS["c3"]
src, tar, _ = F.synth_pair(c["n"], c["room"])
ctxs = [F.Ctx(0) for _ in range(max(Ts))]
dev = [(x.upload(src), x.upload(tar)) for x in ctxs]
ref = None
for x, (ds, dt) in zip(ctxs, dev):  # warm-up (graph capture) + per-context result
    Tb, _ = x.register_batch([((ds, src.shape[0]), (dt, tar.shape[0]))] * 3, c["leaf"], on_device=True)
    ref = Tb[-1] if ref is None else ref
    assert np.array_equal(Tb[-1].view(np.uint32), ref.view(np.uint32))
for T in Ts:
    out = [None] * T
    bar = threading.Barrier(T + 1)

    def work(i):
        x, (ds, dt) = ctxs[i], dev[i]
        bar.wait()
        out[i] = x.register_batch([((ds, src.shape[0]), (dt, tar.shape[0]))] * B, c["leaf"], on_device=True)
        bar.wait()

    th = [threading.Thread(target=work, args=(i,)) for i in range(T)]
    for t in th:
        t.start()
    bar.wait()
    t0 = time.perf_counter()
    bar.wait()
    el = time.perf_counter() - t0
    for t in th:
        t.join()
    ok = all(np.array_equal(Tb[-1].view(np.uint32), ref.view(np.uint32)) for Tb, _ in out)
    print(f"T={T} B={B}: {T * B} registrations in {el * 1e3:.1f} ms -> {el * 1e3 / (T * B):.3f} ms/registration"
          f" (per-thread {el * 1e3 / B:.3f} ms) identical={ok}", flush=True)
