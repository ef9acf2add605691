"""Row D projection: the device time of K1's sort of the c4 / c5
first-pass keys unsharded, and as each rank r of N (FCCF_SHARD_D_SIM=r/N: the
replicated first rounds, then only rank r's range; no exchange), on ONE GPU.  The
sharded sort's time on N GPUs is projected as the slowest rank plus the rank-ordered
all-gather of the sorted (key, value) slices -- the exchange itself is not measured
here (one GPU).  Usage: python tools/shard_projection.py [cfg:N ...]  (GPU)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fccf-pcr_amd"), os.path.join(ROOT, "tools")]
import fccf_amd as F  # noqa: E402
from is_bench import leaf_keys  # noqa: E402


def dev_ms(ctx, k, reps=3):
    ts = []
    for _ in range(reps):
        ctx.sort_keys(k)
        ts.append(int(ctx.sort_stats()["raw"][31]) / 1e6)
    return min(ts)


def main():
    specs = sys.argv[1:] or ["c4:4", "c5:8"]
    with F.Ctx(0) as ctx:
        for spec in specs:
            cfg, n = spec.split(":")
            n = int(n)
            c = F.CONFIGS[cfg]
            src, tar, _ = F.synth_pair(c["n"], c["room"])
            for which, pts in (("src", src), ("tar", tar)):
                k = leaf_keys(pts, c["leaf"])
                os.environ.pop("FCCF_SHARD_D_SIM", None)
                whole = dev_ms(ctx, k)
                per = []
                for r in range(n):
                    os.environ["FCCF_SHARD_D_SIM"] = f"{r}/{n}"
                    per.append(dev_ms(ctx, k))
                    raw = ctx.sort_stats()["raw"]
                    per[-1] = (per[-1], int(raw[29]) - int(raw[28]))
                os.environ.pop("FCCF_SHARD_D_SIM", None)
                worst = max(p[0] for p in per)
                print(f"{cfg} {which}: n={k.size} unsharded {whole:.3f} ms; as rank r of {n}: "
                      + " ".join(f"{t:.3f}({m})" for t, m in per)
                      + f"; slowest rank {worst:.3f} ms ({whole / worst:.2f}x)", flush=True)


if __name__ == "__main__":
    main()
