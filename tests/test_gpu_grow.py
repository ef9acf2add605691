"""K4: face_extrate's region growing on the GPU (FCCF.cpp:536-648, SURVEY.md §8(a) rows
a5/a6; csrc/grow.hip), enabled per ctx with fccf_ctx_set_grow_device.  Bar: every
group (centre, normal, point weight, voxel count, allocation flag) and every downstream
output bit-identical to the CPU oracle and to the host growth, on the registration
path (c2-c5) and through the fccf_stage_grow export, incl. synthetic voxel sets that
stress the scan (many seeds, long merges, the LDS capacity)."""
import numpy as np
import pytest

from test_gpu_register import STAGES, as_bits, compare_all

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gctx(fccf):
    c = fccf.Ctx(0, debug=True)
    c.set_grow_device(True)
    yield c
    c.close()


@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "c5"])
def test_register_with_device_growth_bit_exact(gctx, oracle, fccf, cfg):
    c = fccf.CONFIGS[cfg]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    run = oracle.Run(src, tar, c["leaf"], oracle.INTROSORT)
    T, st = gctx.register(src, tar, c["leaf"])
    for k in (1, 2):  # all groups after stage 2 and their flags, not only the selected planes
        for name, dt in ((f"groups{k}", np.float32), (f"galloc{k}", np.int32)):
            np.testing.assert_array_equal(as_bits(gctx.debug(name, dt)), as_bits(run.get(name, dt)), err_msg=name)
    compare_all(gctx, run)
    np.testing.assert_array_equal(T.view(np.uint32), run.T.view(np.uint32))


def random_voxels(fccf, n, seed, planes=6):
    """Voxel records on a few noisy planes (long merges) plus scattered ones (many seeds)."""
    rng = np.random.default_rng(seed)
    v = np.zeros(n, fccf.VOXEL_DTYPE)
    k = rng.integers(0, planes + 1, n)
    nrm = rng.normal(size=(planes + 1, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    c = rng.uniform(-10, 10, (n, 3)).astype(np.float32)
    on = k < planes
    # project plane members onto their plane through the origin shifted by k
    d = (c[on] * nrm[k[on]]).sum(1, keepdims=True) - k[on, None]
    c[on] -= (d * nrm[k[on]]).astype(np.float32)
    n3 = nrm[k] + rng.normal(scale=0.02, size=(n, 3))
    n3[~on] = rng.normal(size=((~on).sum(), 3))
    v["c"] = c
    v["n"] = (n3 / np.linalg.norm(n3, axis=1, keepdims=True)).astype(np.float32)
    v["count"] = rng.integers(6, 400, n)
    v["curvature"] = 0.01
    return v


@pytest.mark.parametrize("n,seed", [(1, 0), (2, 1), (63, 2), (64, 3), (65, 4), (777, 5), (3072, 6), (3073, 7)])
def test_stage_grow_device_equals_host(fccf, n, seed):
    vox = random_voxels(fccf, n, seed)
    with fccf.Ctx(0) as h, fccf.Ctx(0) as d:
        d.set_grow_device(True)
        for side in (1, 2):
            ph, th, bh = h.grow(vox, side)
            pd, td, bd = d.grow(vox, side)
            np.testing.assert_array_equal(pd.view(np.uint8), ph.view(np.uint8))
            np.testing.assert_array_equal(td.view(np.uint64), th.view(np.uint64))
            np.testing.assert_array_equal(bd.view(np.uint8), bh.view(np.uint8))


def test_stage_grow_device_matches_oracle(gctx, oracle, fccf):
    from test_gpu_stages import voxels_from_dump
    c = fccf.CONFIGS["c3"]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    run = oracle.Run(src, tar, c["leaf"], oracle.INTROSORT)
    for k in (1, 2):
        planes, theta, bases = gctx.grow(voxels_from_dump(fccf, run.get(f"vox{k}")), k)
        np.testing.assert_array_equal(planes.view(np.uint8), fccf.planes_from_dump(run.get(f"planes{k}")).view(np.uint8))
        np.testing.assert_array_equal(theta.view(np.uint64), run.get(f"theta{k}", np.float64).view(np.uint64))
        np.testing.assert_array_equal(bases.view(np.uint8),
                                      fccf.bases_from_dump(run.get(f"bases{k}", np.int32)).view(np.uint8))
