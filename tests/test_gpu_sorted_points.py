"""The sorted-points VoxelGrid path (round 3, 7c1b16e) on the clouds that reach its
rare write sites, with the poison hook on.

K1's finish kernels write every point's xyz in std::sort order beside its key and
value (IsBufs::xyzs, put_xyz in introsort.hip) and the centroid kernel reads each
leaf's members from there (voxelgrid.hip).  The write sites are: the wave tasks
(level form and the <= 64 register form), the block kernel's leaves, and the global
heap sort at the depth limit.  A final position that no site writes would keep the
previous call's point (the arena is reused) and give a silently wrong centroid, so
every case here runs with IS_POISON_XYZS (fccf_debug_inject_sort_fault bit 0x20000):
the buffer is NaN before each sort, and a missed position becomes a NaN centroid.

Cases (FCCF.cpp:1668-1678, PCL VoxelGrid): point clouds whose
first-pass leaf keys ARE a McIlroy adversary against this std::sort (pairwise
distinct: the parallel depth-limit paths, including the distinct-key global path
beyond the LDS; halved, every key repeats: the sequential heap sorts), and a cloud
with non-finite points but no int32 overflow (k_is_prep compacts; put_xyz reads
through the compacted values).  Bar: bit-exact against the oracle's INTROSORT mode,
through fccf_stage_downsample and through fccf_register.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POISON = 0x20000


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def cloud_from_keys(keys, leaf, seed):
    """Points whose VoxelGrid leaf keys at `leaf` are exactly `keys`, in input order:
    a one-row grid along x (key = floor(x / leaf)), with y and z spread inside one
    leaf so that the within-leaf summation order changes the centroid's bits.  leaf
    is a power of two, so every coordinate and x * (1 / leaf) is exact."""
    rng = np.random.default_rng(seed)
    k = np.asarray(keys, np.float64)
    n = k.size
    x = (k + rng.uniform(0.1, 0.9, n)) * leaf
    y = rng.uniform(0.05, 0.95, n) * leaf
    z = rng.uniform(0.05, 0.95, n) * leaf
    pts = np.stack([x, y, z], 1).astype(np.float32)
    inv = np.float32(1.0) / np.float32(leaf)
    assert np.array_equal(np.floor(pts[:, 0] * inv).astype(np.int64), np.asarray(keys, np.int64))
    assert np.all(np.floor(pts[:, 1:] * inv) == 0)
    return pts


@pytest.fixture
def poisoned(ctx):
    ctx.inject_sort_fault(POISON)
    try:
        yield ctx
    finally:
        ctx.inject_sort_fault(0)


def check_downsample(ctx, oracle, pts, leaf):
    ref, ovf = oracle.voxel_grid(pts, leaf, oracle.INTROSORT)
    assert not ovf
    got = ctx.downsample(pts, leaf)
    assert got.shape == ref.shape
    np.testing.assert_array_equal(bits(got), bits(ref))
    assert np.all(np.isfinite(got))
    return ctx.sort_stats()


def test_poison_hook_is_live(poisoned, oracle, fccf):
    """The hook really poisons: with it on, a plain cloud still matches (every position
    is written), and the sort path counters are reported for the downsample."""
    pts = fccf.synth_scene(150_000, seed=2)
    st = check_downsample(poisoned, oracle, pts, 0.05)
    assert st["n"] == pts.shape[0] and st["wave_tasks"] > 0 and st["lds_segments"] > 0


@pytest.mark.parametrize("n", [200, 5000, 20_000, 65_536, 262_144])
def test_adversary_distinct_keys(poisoned, oracle, n):
    """McIlroy adversary (pairwise distinct keys): the depth limit is reached in a wave
    task (200), in a workgroup's LDS (5000) and beyond the LDS (>= 20000: the
    distinct-key global path, flag 4), every position ranked in parallel."""
    keys = oracle.sort_adversary(n)
    leaf = 0.0625
    st = check_downsample(poisoned, oracle, cloud_from_keys(keys, leaf, seed=n), leaf)
    assert st["depth0_distinct"] > 0 or n == 200, st
    if n >= 20_000:
        assert st["flags"] & 4, st  # k_is_block's distinct-key global path ran


@pytest.mark.parametrize("n", [200, 5000, 20_000])
def test_adversary_tied_keys(poisoned, oracle, n):
    """The halved adversary: every key repeats, so each depth-limit segment is heap
    sorted sequentially (wave lane 0, workgroup thread 0, and in global memory for the
    20000-point cloud: flag 2), and the tie order decides the centroid's bits."""
    keys = (oracle.sort_adversary(n) // 2).astype(np.uint32)
    leaf = 0.0625
    st = check_downsample(poisoned, oracle, cloud_from_keys(keys, leaf, seed=n + 1), leaf)
    if n == 20_000:
        assert st["flags"] & 2, st  # the global heap sort (introsort.hip, k_is_block) ran
    if n >= 5000:
        assert st["heaps"] > 0, st


@pytest.mark.parametrize("plan", ["large", "small"])
def test_adversary_both_round_plans(poisoned, oracle, plan, monkeypatch):
    """The same distinct adversary under both round-plan forms (FCCF_IS_PLAN)."""
    monkeypatch.setenv("FCCF_IS_PLAN", plan)
    keys = oracle.sort_adversary(65_536)
    check_downsample(poisoned, oracle, cloud_from_keys(keys, 0.0625, seed=3), 0.0625)


def test_nonfinite_points_without_overflow(poisoned, oracle, fccf):
    """NaN/inf points in a cloud whose leaf index does not overflow: k_is_prep compacts
    the finite points' (key, value) pairs and put_xyz reads the input through the
    compacted values.  Also at c3 size with the large and small round plans."""
    rng = np.random.default_rng(8)
    x = rng.normal(size=(300_000, 3)).astype(np.float32) * 6
    x[::89] = np.nan
    x[7::131, 0] = np.inf
    x[11::173, 2] = -np.inf
    st = check_downsample(poisoned, oracle, x, 0.1)
    assert st["n"] == np.count_nonzero(np.all(np.isfinite(x), 1))
    room = fccf.synth_scene(1_000_000, seed=4)
    room[rng.integers(0, room.shape[0], 3000)] = np.nan
    check_downsample(poisoned, oracle, room, 0.05)


def test_register_with_poison(poisoned, oracle, fccf):
    """Whole registrations with the hook on: the c3 pair (both clouds through the
    pipeline's graphs, both round forms' sorted points), and then a pair whose source
    cloud's first-pass keys are the distinct adversary and whose target is the halved
    one (leaf 1/16 m): every intermediate and T bit-exact against the oracle."""
    from test_gpu_register import compare_all

    c = fccf.CONFIGS["c3"]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    run = oracle.Run(src, tar, c["leaf"], oracle.INTROSORT)
    T, _ = poisoned.register(src, tar, c["leaf"])
    compare_all(poisoned, run)
    np.testing.assert_array_equal(T.view(np.uint32), run.T.view(np.uint32))

    leaf = 0.0625
    a = cloud_from_keys(oracle.sort_adversary(65_536), leaf, seed=21)
    b = cloud_from_keys((oracle.sort_adversary(20_000) // 2).astype(np.uint32), leaf, seed=22)
    run = oracle.Run(a, b, leaf, oracle.INTROSORT)
    T, _ = poisoned.register(a, b, leaf)
    for name in ("ds_src", "ds_tar", "ds1", "ds2"):
        ref, got = run.get(name), poisoned.debug(name)
        assert got.shape == ref.shape, name
        np.testing.assert_array_equal(bits(got), bits(ref), err_msg=name)
    np.testing.assert_array_equal(T.view(np.uint32), run.T.view(np.uint32))
