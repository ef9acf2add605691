"""Stress the pipelined batch where graph captures overlap cross-thread event waits:
fresh contexts (first captures), and pairs whose sizes change every step (every
graph re-captured).  Every pair's T must equal its single registration."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fccf-pcr_amd"))
import fccf_amd as F  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfg = F.CONFIGS["c2"]
pairs = []
for n in (60_000, 80_000, 100_000):
    s, t, _ = F.synth_pair(n, cfg["room"])
    pairs.append((s, t))
ref = []
with F.Ctx(0) as c:
    for s, t in pairs:
        ref.append(c.register(s, t, cfg["leaf"])[0])
t0 = time.time()
for r in range(rounds):
    with F.Ctx(0) as c:
        seq = [pairs[(r + i) % 3] for i in range(6)]
        T, _ = c.register_batch(seq, cfg["leaf"])
        for i in range(6):
            assert np.array_equal(T[i].view(np.uint32), ref[(r + i) % 3].view(np.uint32)), (r, i)
        d = [(c.upload(s), len(s), c.upload(t), len(t)) for s, t in seq[:2]]
        T, _ = c.register_batch([((a, na), (b, nb)) for a, na, b, nb in d] * 2, cfg["leaf"], on_device=True)
        for i in range(4):
            assert np.array_equal(T[i].view(np.uint32), ref[(r + i % 2) % 3].view(np.uint32)), (r, i)
        for a, _, b, _ in d:
            c.free(a)
            c.free(b)
    print(f"round {r} ok ({time.time() - t0:.1f} s)", flush=True)
