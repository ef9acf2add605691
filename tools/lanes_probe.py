"""Lanes vs separate contexts, one variant per process (stream creation order matters).
Usage: python tools/lanes_probe.py {conc,conc_shared,lanes,lanes_copies} [steps]"""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fccf-pcr_amd"))
import fccf_amd as F  # noqa: E402

mode = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
cfg = F.CONFIGS["c3"]
src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
leaf = cfg["leaf"]


def timed(f):
    f()  # warm
    best = []
    for _ in range(3):
        t0 = time.perf_counter()
        f()
        best.append(time.perf_counter() - t0)
    return min(best), best


if mode.startswith("conc"):
    ctxs = [F.Ctx(0) for _ in range(3 if mode == "conc3" else 2)][-2:]
    for c in ctxs:
        c.set_lanes(1)
    ins = []
    for c in ctxs:
        if mode == "conc_shared" and ins:
            ins.append(ins[0])
        else:
            ins.append(((c.upload(src), src.shape[0]), (c.upload(tar), tar.shape[0])))

    def run():
        th = [threading.Thread(target=lambda i=i: ctxs[i].register_batch([ins[i]] * steps, leaf, on_device=True))
              for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    dt, all_ = timed(run)
    n = 2 * steps
else:
    c = F.Ctx(0)
    c.set_lanes(2, 4)
    a = ((c.upload(src), src.shape[0]), (c.upload(tar), tar.shape[0]))
    b = ((c.upload(src), src.shape[0]), (c.upload(tar), tar.shape[0])) if mode == "lanes_copies" else a
    pairs = [a if i % 2 == 0 else b for i in range(2 * steps)]

    def run():
        c.register_batch(pairs, leaf, on_device=True)
    dt, all_ = timed(run)
    n = 2 * steps
print(f"{mode}: {dt / n * 1e3:.3f} ms/registration (runs {[round(x / n * 1e3, 3) for x in all_]})", flush=True)
