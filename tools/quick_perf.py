"""Dev: c3 single-registration median, main-VoxelGrid device span and pipelined
ms/registration (device-resident inputs).  Usage: python tools/quick_perf.py [reps]"""
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
pair = ((ds, len(src)), (dt, len(tar)))
for _ in range(3):
    ctx.register_device(ds, len(src), dt, len(tar), cfg["leaf"])
ctx.register_batch([pair] * 8, cfg["leaf"], on_device=True)  # both stage groups
e, vg = [], []
for _ in range(reps):
    a = time.perf_counter()
    T, st = ctx.register_device(ds, len(src), dt, len(tar), cfg["leaf"])
    e.append((time.perf_counter() - a) * 1e3)
    vg.append(st.dev_ms[0])
pb = []
for _ in range(3):
    a = time.perf_counter()
    ctx.register_batch([pair] * reps, cfg["leaf"], on_device=True)
    pb.append((time.perf_counter() - a) / reps * 1e3)
print(f"e2e {statistics.median(e):.3f} ms  vg_main {statistics.median(vg):.3f} ms  pipelined {min(pb):.3f} ms/reg"
      f"  (batches: {' '.join(f'{x:.3f}' for x in pb)})", flush=True)
