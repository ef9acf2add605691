"""Cloud-stage segment timings (FCCF_SEG_TIMING=1 prints them to stderr) for c3."""
import os
import sys

os.environ.setdefault("FCCF_SEG_TIMING", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fccf-pcr_amd"))
import fccf_amd as F  # noqa: E402

cfg = F.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
with F.Ctx(0) as c:
    ds, dt = c.upload(src), c.upload(tar)
    for i in range(12):
        T, st = c.register_device(ds, src.shape[0], dt, tar.shape[0], cfg["leaf"])
        print({k: round(v, 4) for k, v in st.as_dict()["ms"].items() if v}, round(st.ms_total, 4), flush=True)
