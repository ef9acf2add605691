"""Dev: median per-stage host/device times (fccf_stats.ms) of single c3 registrations.
Usage: python tools/stage_ms.py [reps]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fccf-pcr_amd"))
import fccf_amd as F  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfg = F.CONFIGS["c3"]
src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
ctx = F.Ctx(0)
ds, dt = ctx.upload(src), ctx.upload(tar)
for _ in range(3):
    ctx.register_device(ds, len(src), dt, len(tar), cfg["leaf"])
ms, e2e = [], []
for _ in range(reps):
    a = time.perf_counter()
    T, st = ctx.register_device(ds, len(src), dt, len(tar), cfg["leaf"])
    e2e.append((time.perf_counter() - a) * 1e3)
    ms.append(st.as_dict()["ms"])
keys = ms[0].keys()
g = sorted(m["grow"] for m in ms)
e = sorted(e2e)
q = lambda v, f: v[min(len(v) - 1, int(f * len(v)))]
print(f"spread: grow p10 {q(g, .1):.4f} p50 {q(g, .5):.4f} p90 {q(g, .9):.4f}; e2e p10 {q(e, .1):.3f} p90 {q(e, .9):.3f}")
print(f"e2e {statistics.median(e2e):.3f} ms | " + " ".join(f"{k} {statistics.median(m[k] for m in ms):.4f}" for k in keys),
      flush=True)
