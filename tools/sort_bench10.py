"""Dev: K1's sort at a stage group's width, in isolation: ten copies of the c3 source
cloud's leaf keys sorted in one batched launch sequence (fccf_debug_sort_keys_batch,
the sorted points written as VoxelGrid's first pass does), device ms per call; run
under rocprofv3 --kernel-trace for the per-kernel split.  --check compares copy 0's
order with the oracle's std::sort.  Usage: python tools/sort_bench10.py [reps] [--check]"""
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fccf-pcr_amd"), os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")]
import fccf_amd as F  # noqa: E402
from is_bench import leaf_keys  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10
    copies = int(os.environ.get("COPIES", "10"))
    c = F.CONFIGS[os.environ.get("CFG", "c3")]
    src, _, _ = F.synth_pair(c["n"], c["room"])
    k = leaf_keys(src, c["leaf"])
    with F.Ctx(0) as ctx:
        perm, _ = ctx.sort_keys_batch(k, copies, src)
        if "--check" in sys.argv:
            import oracle_py
            ok = np.array_equal(perm, oracle_py.sort_pairs(k))
            print(f"order equals std::sort: {ok}", flush=True)
            if not ok:
                sys.exit(1)
        ms = [ctx.sort_keys_batch(k, copies, src)[1] for _ in range(reps)]
    print(f"sort x{copies}: median {statistics.median(ms):.3f} ms, min {min(ms):.3f} ms ({reps} reps)", flush=True)


if __name__ == "__main__":
    main()
