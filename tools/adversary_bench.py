"""Sort edge behaviour: K1's sort on McIlroy adversaries against
libstdc++ std::sort (oracle.sort_adversary), which drive it to the depth limit (heap
sort) on segments beyond the LDS.  For each case: the GPU sort's time (host wall,
fccf_debug_sort_keys incl. copies), its path counters, and exactness against the
oracle's std::sort; then the adversary as a point cloud (one voxel per key along x)
through the VoxelGrid stage (fccf_stage_downsample) against the oracle's VoxelGrid.
Usage: python tools/adversary_bench.py [sizes...]   (GPU; default 20000 65536 262144 1048576)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fccf-pcr_amd"), os.path.join(ROOT, "tests")]
import fccf_amd as F  # noqa: E402
import oracle_py as O  # noqa: E402  (test infrastructure: the checker)


def timed(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return out, float(np.median(ts)) * 1e3


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [20_000, 65_536, 262_144, 1_048_576]
    ctx = F.Ctx(0)
    for n in sizes:
        adv = O.sort_adversary(n)
        t0 = time.perf_counter()
        ref = O.sort_pairs(adv)
        cpu_ms = (time.perf_counter() - t0) * 1e3
        cases = [("distinct", adv)]
        if n <= 65_536:  # repeated keys keep the sequential heap sort: bounded sizes only
            cases.append(("ties", (adv // 2).astype(np.uint32)))
        for name, k in cases:
            r = ref if name == "distinct" else O.sort_pairs(k)
            got, ms = timed(lambda: ctx.sort_keys(k), reps=1 if name == "ties" else 3)
            st = ctx.sort_stats()
            print(f"n={n:8d} {name:8s} gpu sort {ms:9.2f} ms  exact={np.array_equal(got, r)}  "
                  f"depth0_distinct={st['depth0_distinct']} heaps={st['heaps']} global_parts={st['global_parts']} "
                  f"flags={st['flags']}  (oracle std::sort {cpu_ms:.1f} ms)", flush=True)
        # the adversary as a cloud: key k -> a point in voxel k along x (leaf 0.05)
        leaf = 0.05
        pts = np.zeros((n, 3), np.float32)
        pts[:, 0] = (adv.astype(np.float64) + 0.5) * leaf
        pts[:, 1] = 0.01
        pts[:, 2] = 0.01
        out, ms = timed(lambda: ctx.downsample(pts, leaf), reps=1)
        want, _ = O.voxel_grid(pts, leaf, O.INTROSORT)
        same = out.shape == want.shape and np.array_equal(out.view(np.uint32), want.view(np.uint32))
        print(f"n={n:8d} cloud    VoxelGrid stage {ms:9.2f} ms  bit-exact={same}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
