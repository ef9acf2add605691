"""f3: transform_cluster's seed pass, range_cluster's exchange sort
and the cluster averaging on the GPU (csrc/cluster.hip; FCCF.cpp:1040-1231,
:1020-1038), enabled per ctx with fccf_ctx_set_cluster_device.  Bar: the fused
candidates (fine0-2) and the cluster counts bit-identical to the CPU oracle through
the registration (c2-c5), and to the host path through fccf_stage_cluster on
synthetic candidate sets that reach the kernels' edges: tied sizes and tied
distances, empty rows, the LDS row cache vs HBM rows, a cluster past the member
capacity (that type falls back to the host) and sets too large for the rows."""
import numpy as np
import pytest

from test_gpu_register import as_bits, compare_all

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dctx(fccf):
    c = fccf.Ctx(0, debug=True)
    c.set_cluster_device(True)
    yield c
    c.close()


@pytest.fixture(scope="module")
def hctx(fccf):
    c = fccf.Ctx(0)
    yield c
    c.close()


@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "c5"])
def test_register_with_device_clustering_bit_exact(dctx, oracle, fccf, cfg):
    c = fccf.CONFIGS[cfg]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    run = oracle.Run(src, tar, c["leaf"], oracle.INTROSORT)
    T, st = dctx.register(src, tar, c["leaf"])
    for t in range(3):
        np.testing.assert_array_equal(as_bits(dctx.debug(f"fine{t}")), as_bits(run.get(f"fine{t}")), err_msg=f"fine{t}")
    compare_all(dctx, run)  # includes the cluster counts
    np.testing.assert_array_equal(T.view(np.uint32), run.T.view(np.uint32))


def _quat_to_R(q):
    w, x, y, z = q / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def synth_candidates(rng, n, centres, spread_t=0.3, spread_deg=0.8, dup=0.1):
    """n candidate transforms around `centres` random poses (within the 0.8 m / 2 deg
    cluster thresholds of their centre), with a fraction of exact duplicates (tied
    distances, tied sizes)."""
    cq = rng.normal(size=(centres, 4))
    ct = rng.uniform(-5, 5, size=(centres, 3))
    out = np.zeros((n, 4, 4), np.float32)
    for i in range(n):
        if i and rng.random() < dup:
            out[i] = out[rng.integers(0, i)]
            continue
        k = rng.integers(0, centres)
        q = cq[k] / np.linalg.norm(cq[k]) + rng.normal(scale=np.deg2rad(spread_deg) / 4, size=4)
        out[i, :3, :3] = _quat_to_R(q)
        out[i, :3, 3] = ct[k] + rng.normal(scale=spread_t / 2, size=3)
        out[i, 3, 3] = 1.0
    return out


@pytest.mark.parametrize("n,centres,cnum", [
    (12, 3, 5),        # just past cluster_number_threshold
    (200, 8, 40),      # rows in the LDS cache
    (200, 200, 150),   # mostly singletons: the emission loop's size-1 tail
    (700, 40, 120),    # W = 11: 7700 words, still cached
    (1500, 30, 200),   # rows read from HBM
    (3000, 2, 60),     # big clusters (> 1024 members: that type on the host)
    (6000, 50, 200),   # past the row capacity: the host's own radius search
])
def test_stage_cluster_device_equals_host(dctx, hctx, fccf, n, centres, cnum):
    rng = np.random.default_rng(n * 7 + centres)
    cand = synth_candidates(rng, n, centres)
    fh, nh = hctx.cluster(cand, cnum)
    fd, nd = dctx.cluster(cand, cnum)
    assert nd == nh
    assert fd.shape == fh.shape
    np.testing.assert_array_equal(as_bits(fd), as_bits(fh))


def test_stage_cluster_device_edge_cases(dctx, hctx, fccf):
    rng = np.random.default_rng(3)
    base = synth_candidates(rng, 64, 4)
    cases = {
        "all_identical": np.repeat(base[:1], 50, axis=0),
        "non_finite_t": base.copy(),
        "cluster_num_0": base,
        "cluster_num_huge": base,
        "at_threshold": base[:10],
        "empty": base[:0],
    }
    cases["non_finite_t"][[3, 9, 17], 0, 3] = np.nan
    for name, cand in cases.items():
        cnum = {"cluster_num_0": 0, "cluster_num_huge": 5000}.get(name, 20)
        fh, nh = hctx.cluster(cand, cnum)
        fd, nd = dctx.cluster(cand, cnum)
        assert nd == nh, name
        assert fd.shape == fh.shape, name
        np.testing.assert_array_equal(as_bits(fd), as_bits(fh), err_msg=name)


def test_stage_cluster_device_matches_oracle_lists(dctx, oracle, fccf):
    """fccf_stage_cluster on the oracle's own candidate lists (c3): its fine lists."""
    c = fccf.CONFIGS["c3"]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    run = oracle.Run(src, tar, c["leaf"], oracle.INTROSORT)
    counts = run.get("counts", np.int64)
    cands = [run.get(f"cand{t}").reshape(-1, 4, 4) for t in range(3)]
    total = sum(len(x) for x in cands)
    for t in range(3):
        cluster_num = int(np.float32(200.0) * np.float32(len(cands[t])) / np.float32(total)) if total else 0
        fine, ncl = dctx.cluster(cands[t], cluster_num)
        ref = run.get(f"fine{t}").reshape(-1, 8)
        assert fine.shape == ref.shape, t
        np.testing.assert_array_equal(as_bits(fine), as_bits(ref))
        assert ncl == counts[5 + t]
