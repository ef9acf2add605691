"""Dev: consecutive pipelined c3 batches of 20 in one process, optionally after the
bench's probe passes (argv[1] == 'probe'): ms per registration of each batch."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fccf-pcr_amd"))
sys.path.insert(0, ROOT)
import fccf_amd as F  # noqa: E402

cfg = F.CONFIGS["c3"]
src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
ctx = F.Ctx(0)
ds, dt = ctx.upload(src), ctx.upload(tar)
pair = ((ds, len(src)), (dt, len(tar)))
if len(sys.argv) > 1 and sys.argv[1] == "probe":
    import bench
    for k in bench.PROBE_KERNELS:
        bench.probe_pass(ctx, lambda: ctx.register_batch([pair] * bench.PROBE_BATCH, cfg["leaf"], on_device=True), k, 1)
    ctx.set_probe(None)
for _ in range(3):
    ctx.register_device(ds, len(src), dt, len(tar), cfg["leaf"])
out = []
for _ in range(6):
    a = time.perf_counter()
    ctx.register_batch([pair] * 20, cfg["leaf"], on_device=True)
    out.append((time.perf_counter() - a) / 20 * 1e3)
print(("after probes: " if len(sys.argv) > 1 else "plain: ") + " ".join(f"{x:.3f}" for x in out), flush=True)
