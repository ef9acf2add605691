"""PMC workload of the timed region's own shape: pipelined batches
of one config's pair, five pairs per cloud stage (ten clouds per launch), and nothing
else -- no single registrations, whose two-cloud launches would mix into the per-kernel
means.  Run under rocprofv3 --pmc (tools/gpu_pmc_calib.sh BATCH=1); prints one JSON line
whose kernel_table carries the probe's algorithmic bytes per launch at that width, the
input tools/pmc_traffic.py divides by.

Usage: python tools/pmc_batch.py CONFIG STEPS [KERNEL ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fccf-pcr_amd"))
import fccf_amd as F  # noqa: E402

cfg_name, steps = sys.argv[1], int(sys.argv[2])
kernels = sys.argv[3:] or ["k_is_scatter", "k_is_count_plan", "k_is_wave", "k_is_block", "k_vg_centroid",
                          "k_gather", "k_voxel_fit", "k_rs_scatter", "k_vg_keys"]
cfg = F.CONFIGS[cfg_name]
src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
with F.Ctx(0) as ctx:
    ds, dt = ctx.upload(src), ctx.upload(tar)
    pairs = [((ds, src.shape[0]), (dt, tar.shape[0]))] * steps
    ctx.register_batch(pairs, cfg["leaf"], on_device=True)  # warm: graphs of the batch's shape
    ctx.register_batch(pairs, cfg["leaf"], on_device=True)
    table = {}
    for k in kernels:  # algorithmic bytes per launch at the batch's width (probe.h)
        ctx.set_probe(k)
        ctx.register_batch(pairs[:10], cfg["leaf"], on_device=True)  # two full stage groups
        w = ctx.probe_read_widths()
        if w:
            width = max(w, key=lambda x: w[x][1])
            ms, n, b = w[width]
            table[k] = {"algorithmic_bytes_per_launch": b / n, "launch_width": width, "avg_launch_us": ms * 1e3 / n}
    ctx.set_probe(None)
    ctx.free(ds)
    ctx.free(dt)
print(json.dumps({"config": cfg_name, "shape": "pipelined batch", "steps": steps, "kernel_table": table}), flush=True)
