"""Dev: the batch fine-overflow case of tests/test_gpu_register.py with per-pair stats."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fccf-pcr_amd")]
import numpy as np  # noqa: E402
import fccf_amd as F  # noqa: E402

os.environ["FCCF_PAIR_BATCH"] = "4"
os.environ["FCCF_FINE_LDS_CAP"] = "16"
base_src, base_tar, _ = F.synth_pair(80_000)
rng = np.random.default_rng(41)
pairs = []
for k in range(6):
    jit = rng.normal(0, 0.002, base_src.shape).astype(np.float32)
    pairs.append(((base_src + jit).astype(np.float32), base_tar[: 80_000 - 4000 * k]))
for rep in range(3):
    c = F.Ctx(0)
    Tb, sb = c.register_batch(pairs, 0.1)
    print("reruns", [int(x.fine_reruns) for x in sb], "evals", [int(x.fine_evals) for x in sb],
          "K", [int(x.K) for x in sb], flush=True)
    c.close()
