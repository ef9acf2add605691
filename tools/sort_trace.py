"""Dev: per block item / wave task timestamps of K1's sort on the c3 VoxelGrid keys
(FCCF_IS_TRACE_OUT, fccf_debug_sort_keys), then a summary: makespan of each phase,
the longest items and how many workgroups are busy over time.
Usage: python tools/sort_trace.py [out_dir]   (GPU)  /  python tools/sort_trace.py --analyze file"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def analyze(path):
    rows = [l.split() for l in open(path).read().splitlines()[1:]]
    for kind in ("B", "W"):
        r = np.array([[int(x) for x in row[1:]] for row in rows if row[0] == kind], dtype=np.int64)
        if not len(r):
            continue
        t0, t1 = r[:, 0].min(), r[:, 1].max()
        d = (r[:, 1] - r[:, 0]) / 100.0  # us (100 MHz)
        print(f"{kind}: {len(r)} items, span {(t1 - t0) / 100.0:.1f} us, item us: median {np.median(d):.2f} "
              f"p90 {np.percentile(d, 90):.2f} max {d.max():.1f}, sum {d.sum():.0f}")
        idx = np.argsort(-d)[:8]
        for i in idx:
            print(f"   size {r[i, 2]:6d} who {r[i, 3]:5d} start +{(r[i, 0] - t0) / 100.0:7.1f} dur {d[i]:7.1f} us")
        # per-worker busy time and last end
        who = r[:, 3]
        ends = {}
        for w, e in zip(who, r[:, 1]):
            ends[w] = max(ends.get(w, 0), e)
        busy = {}
        for w, dd in zip(who, d):
            busy[w] = busy.get(w, 0) + dd
        b = np.array(list(busy.values()))
        print(f"   workers {len(busy)}, busy us per worker: median {np.median(b):.1f} max {b.max():.1f}")
        for q in (10, 25, 50, 75, 90):
            print(f"   size p{q}: {np.percentile(r[:, 2], q):.0f}", end="")
        print()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
        sys.exit(0)
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/strace"
    os.makedirs(out, exist_ok=True)
    os.environ["FCCF_IS_TRACE_OUT"] = os.path.join(out, "trace.txt")
    sys.path[:0] = [os.path.join(ROOT, "fccf-pcr_amd"), os.path.join(ROOT, "tools")]
    import fccf_amd as F
    from is_bench import leaf_keys
    src, tar, _ = F.synth_pair(1_000_000, (20.0, 15.0, 4.0))
    with F.Ctx(0) as ctx:
        for name, pts in (("src", src), ("tar", tar)):
            k = leaf_keys(pts, 0.05)
            for _ in range(2):
                ctx.sort_keys(k)
            os.replace(os.environ["FCCF_IS_TRACE_OUT"], os.path.join(out, f"trace_{name}.txt"))
            print(name, ctx.sort_stats())
            analyze(os.path.join(out, f"trace_{name}.txt"))
