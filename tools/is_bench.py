"""Dev probe: time K1's std::sort-order sort (fccf_debug_sort_keys) and the VoxelGrid
stage export on the c3 workload; run under rocprofv3 --kernel-trace --stats for the
per-kernel split.  Usage: python tools/is_bench.py [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fccf-pcr_amd"), os.path.join(ROOT, "tests")]
import fccf_amd as F  # noqa: E402


def leaf_keys(pts, leaf):
    inv = np.float32(1.0) / np.float32(leaf)
    minb = np.floor(pts.min(0) * inv).astype(np.int64)
    div = np.floor(pts.max(0) * inv).astype(np.int64) - minb + 1
    ijk = (np.floor(pts * inv) - minb.astype(np.float32)).astype(np.int64)
    return (ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]).astype(np.uint32)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    c = F.CONFIGS[os.environ.get("CFG", "c3")]
    src, tar, _ = F.synth_pair(c["n"], c["room"])
    k = leaf_keys(src, c["leaf"])
    ctx = F.Ctx(0)
    for name, fn in (("sort_keys", lambda: ctx.sort_keys(k)), ("downsample", lambda: ctx.downsample(src, c["leaf"]))):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        print(f"{name}: median {np.median(ts) * 1e3:.3f} ms (host wall incl. copies)", flush=True)
        if name == "sort_keys":
            print(ctx.sort_stats(), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
