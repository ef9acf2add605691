"""Dev: whether the configs' K1 sorts reach std::sort's depth limit (sort_stats: heap
sorts and distinct-key depth-limit segments), first-pass leaf keys of both clouds.
Usage: python tools/depth_check.py [configs...]   (GPU; default c2 c3 c4 c5)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fccf-pcr_amd"), os.path.join(ROOT, "tools")]
import fccf_amd as F  # noqa: E402
from is_bench import leaf_keys  # noqa: E402

with F.Ctx(0) as ctx:
    for name in sys.argv[1:] or ["c2", "c3", "c4", "c5"]:
        c = F.CONFIGS[name]
        src, tar, _ = F.synth_pair(c["n"], c["room"])
        for which, pts in (("src", src), ("tar", tar)):
            ctx.sort_keys(leaf_keys(pts, c["leaf"]))
            st = ctx.sort_stats()
            print(f"{name} {which}: n={st['n']} heaps={st['heaps']} depth0_distinct={st['depth0_distinct']} "
                  f"global_parts={st['global_parts']} flags={st['flags']}", flush=True)
