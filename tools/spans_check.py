import sys, os
sys.path.insert(0, "fccf-pcr_amd")
import fccf_amd as F
cfg = F.CONFIGS["c3"]
src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
ctx = F.Ctx(0)
for _ in range(3):
    T, st = ctx.register(src, tar, cfg["leaf"])
    print(st.as_dict()["dev_ms"], st.as_dict()["ms"]["downsample"], st.as_dict()["ms"]["voxelfit"], flush=True)
