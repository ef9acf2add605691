"""K1 parity: GPU VoxelGrid (FCCF.cpp:1668-1678, :1377-1387) vs the CPU oracle.

Integer/ordering work and the per-leaf float sums follow the same sequence, so the
bar is bit-exact (compared as uint32 bit patterns)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def check(ctx, oracle, xyz, leaf, presorted=False):
    ref, ovf = oracle.voxel_grid(xyz, leaf, oracle.INTROSORT)
    got = ctx.downsample(xyz, leaf, presorted)
    assert got.shape == ref.shape, (got.shape, ref.shape, ovf)
    np.testing.assert_array_equal(bits(got), bits(ref))
    return ref


@pytest.mark.parametrize("n,leaf", [(100_000, 0.1), (1_000_000, 0.05), (20_000, 0.37)])
def test_scene(ctx, oracle, fccf, n, leaf):
    xyz = fccf.synth_scene(n, seed=3)
    m1 = check(ctx, oracle, xyz, leaf)
    check(ctx, oracle, m1, leaf, presorted=True)  # the driver's second pass on main's output


def test_transformed_negative_coords(ctx, oracle, fccf):
    src, tar, _ = fccf.synth_pair(200_000)
    check(ctx, oracle, src, 0.05)
    check(ctx, oracle, tar, 0.05)


def test_edge_cases(ctx, oracle):
    rng = np.random.default_rng(0)
    check(ctx, oracle, np.zeros((0, 3), np.float32), 0.1)
    check(ctx, oracle, np.array([[1.0, 2.0, 3.0]], np.float32), 0.1)
    check(ctx, oracle, np.full((5000, 3), 0.25, np.float32), 0.1)             # one leaf, 5000 points
    lat = (np.stack(np.meshgrid(*[np.arange(12)] * 3), -1).reshape(-1, 3) * 0.1).astype(np.float32)
    check(ctx, oracle, lat, 0.1)                                              # points on leaf boundaries
    check(ctx, oracle, np.repeat(lat, 3, axis=0), 0.1)                         # duplicates
    x = rng.normal(size=(50_000, 3)).astype(np.float32) * 7
    x[::97] = np.nan
    x[5::101, 1] = np.inf
    check(ctx, oracle, x, 0.2)                                                # non-finite points dropped


def test_overflow_passthrough(ctx, oracle):
    rng = np.random.default_rng(1)
    x = rng.uniform(-5000, 5000, size=(30_000, 3)).astype(np.float32)
    ref, ovf = oracle.voxel_grid(x, 0.01)
    assert ovf
    check(ctx, oracle, x, 0.01)


def test_many_leaves_random(ctx, oracle):
    rng = np.random.default_rng(2)
    x = rng.uniform(-30, 30, size=(2_000_000, 3)).astype(np.float32)
    check(ctx, oracle, x, 0.5)


def test_presorted_check_paths(ctx, oracle, fccf):
    """fccf_stage_downsample_presorted (the driver's second pass): sorted input takes
    the identity path (no sort), anything else the single-workgroup tail sort.  Both
    must equal the oracle on inputs near the boundary of the check."""
    m1 = check(ctx, oracle, fccf.synth_scene(120_000, seed=5), 0.1)
    check(ctx, oracle, m1, 0.1, True)                                   # strictly increasing: identity
    sw = m1.copy()
    sw[[1000, 1001]] = sw[[1001, 1000]]
    check(ctx, oracle, sw, 0.1, True)                                   # one descent: tail sort
    check(ctx, oracle, np.concatenate([m1, m1[-1:]]), 0.1, True)        # equal last keys
    check(ctx, oracle, np.concatenate([m1, np.full((1, 3), np.nan, np.float32)]), 0.1, True)  # non-finite last
    check(ctx, oracle, m1[::-1].copy(), 0.1, True)                      # descending
    check(ctx, oracle, fccf.synth_scene(60_000, seed=6), 0.05, True)    # random order: tail sort
    check(ctx, oracle, np.zeros((0, 3), np.float32), 0.1, True)
    check(ctx, oracle, np.full((3, 3), np.nan, np.float32), 0.1, True)  # no finite point
    x = np.random.default_rng(1).uniform(-5000, 5000, size=(3000, 3)).astype(np.float32)
    check(ctx, oracle, x, 0.01, True)                                   # overflow pass-through
