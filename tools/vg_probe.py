"""Dev probe: the VoxelGrid stage alone (fccf_stage_downsample), repeated, for a
kernel trace without other streams' work.  Usage: python tools/vg_probe.py [n] [reps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fccf-pcr_amd")]
import fccf_amd as F  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
src, tar, _ = F.synth_pair(n, (20.0, 15.0, 4.0))
ctx = F.Ctx(0)
for _ in range(reps):
    ctx.downsample(src, 0.05)
ctx.close()
print("ok")
