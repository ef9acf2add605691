"""Dev: runtime blit kernels per registration in the steady state.  Run under
`rocprofv3 --kernel-trace --stats`: a pipelined batch of device-resident c3 pairs
(no probes, no parity legs), after one warm-up batch.  Usage: python tools/blit_count.py [pairs]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fccf-pcr_amd"))
import fccf_amd as F  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
c = F.CONFIGS["c3"]
src, tar, _ = F.synth_pair(c["n"], c["room"])
with F.Ctx(0) as ctx:
    ds, dt = ctx.upload(src), ctx.upload(tar)
    pairs = [((ds, len(src)), (dt, len(tar)))] * n
    ctx.register_batch(pairs[:3], c["leaf"], on_device=True)  # warm-up: graphs captured
    print("marker: steady batch of", n, flush=True)
    ctx.register_batch(pairs, c["leaf"], on_device=True)
    ctx.free(ds)
    ctx.free(dt)
