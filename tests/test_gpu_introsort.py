"""K1's sort in the reference's order: the GPU reproduction of libstdc++ std::sort
(introsort) over PCL VoxelGrid's (idx, cloud_point_index) pairs (FCCF.cpp:1668-1678,
:1377-1387), compared with the oracle's std::sort, and the
VoxelGrid passes built on it compared with the oracle's INTROSORT mode.

Integer permutation work: the bar is bit-exact equality.  The CPU tests pin the
oracle side (std::sort is a valid sort, the adversary reaches the heap-sort depth).
"""
import numpy as np
import pytest

INVALID = np.uint32(0xFFFFFFFF)


def _keys_cases(fccf, oracle):
    rng = np.random.default_rng(7)
    cases = {}
    for n in (0, 1, 2, 3, 16, 17, 18, 33, 64, 65, 100, 1000, 1023, 1024, 1025, 4096, 7680, 7681, 7700, 15000, 40000):
        cases[f"rand8_{n}"] = rng.integers(0, 8, n).astype(np.uint32)
        cases[f"randbig_{n}"] = rng.integers(0, 1 << 30, n).astype(np.uint32)
    cases["sorted_50k"] = np.arange(50_000, dtype=np.uint32) // 3
    cases["reversed_50k"] = (np.arange(50_000, dtype=np.uint32) // 3)[::-1].copy()
    cases["const_30k"] = np.full(30_000, 5, np.uint32)
    cases["dups_300k"] = rng.integers(0, 60_000, 300_000).astype(np.uint32)
    # spatially ordered leaf keys of a synthetic room (the VoxelGrid workload's structure)
    pts = fccf.synth_scene(200_000, seed=3)
    inv = np.float32(1.0) / np.float32(0.05)
    mn = pts.min(0)
    minb = np.floor(mn * inv).astype(np.int64)
    div = np.floor(pts.max(0) * inv).astype(np.int64) - minb + 1
    ijk = (np.floor(pts * inv) - minb.astype(np.float32)).astype(np.int64)
    cases["room_200k"] = (ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]).astype(np.uint32)
    k = cases["room_200k"].copy()
    k[rng.integers(0, k.size, 500)] = INVALID  # non-finite points: PCL skips them
    cases["room_200k_nan"] = k
    cases["all_invalid_100"] = np.full(100, INVALID, np.uint32)
    # depth-limit (heap sort) paths: McIlroy adversaries against this std::sort.  Their
    # keys are pairwise distinct (the parallel depth-limit paths: wave, workgroup, and
    # beyond the LDS); halved, every key repeats (the sequential heap sort, tie order)
    for n in (200, 5000, 20_000, 65_536):
        cases[f"adversary_{n}"] = oracle.sort_adversary(n)
    for n in (200, 5000, 20_000):
        cases[f"adversary_ties_{n}"] = (oracle.sort_adversary(n) // 2).astype(np.uint32)
    return cases


def test_oracle_sort_pairs_is_a_sort(oracle):
    rng = np.random.default_rng(1)
    k = rng.integers(0, 50, 10_000).astype(np.uint32)
    k[::97] = INVALID
    p = oracle.sort_pairs(k)
    assert p.size == np.count_nonzero(k != INVALID)
    assert np.all(np.diff(k[p].astype(np.int64)) >= 0)
    assert np.array_equal(np.sort(p), np.flatnonzero(k != INVALID))
    # unstable: equal keys are not all in input order (otherwise the order would not matter)
    assert not np.array_equal(p, np.flatnonzero(k != INVALID)[np.argsort(k[k != INVALID], kind="stable")])


def test_oracle_adversary_is_deep(oracle):
    k = oracle.sort_adversary(4096)
    assert k.size == 4096 and np.all(np.diff(k[oracle.sort_pairs(k)].astype(np.int64)) >= 0)


@pytest.mark.gpu
def test_sort_keys_equals_std_sort(ctx, fccf, oracle):
    bad = []
    for name, k in _keys_cases(fccf, oracle).items():
        got = ctx.sort_keys(k)
        ref = oracle.sort_pairs(k)
        if not np.array_equal(got, ref):
            bad.append((name, k.size, int(np.count_nonzero(got[:ref.size] != ref)) if got.size == ref.size else -1))
    assert not bad, bad


@pytest.mark.gpu
def test_block_kernel_second_form_equals_std_sort(ctx, fccf, oracle, monkeypatch):
    """The block kernel's second form (introsort_b2.hip: 256-thread workgroups over
    segments of up to 4,096 elements, three per CU; stage groups of three to five pairs use
    it) forced for every sort (FCCF_IS_BLOCK_B2=1) on every case and a c3 downsample (whose
    last round leaves a segment above 4,096 for the global-memory partition), against the
    oracle's std::sort."""
    monkeypatch.setenv("FCCF_IS_BLOCK_B2", "1")
    bad = [name for name, k in _keys_cases(fccf, oracle).items()
           if not np.array_equal(ctx.sort_keys(k), oracle.sort_pairs(k))]
    assert not bad, bad
    c = fccf.CONFIGS["c3"]
    src, _, _ = fccf.synth_pair(c["n"], c["room"])
    out = ctx.downsample(src, c["leaf"])
    ref, _ = oracle.voxel_grid(src, c["leaf"], oracle.INTROSORT)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
def test_sort_keys_exact_gate_equals_std_sort(ctx, fccf, oracle):
    """The presorted pass's single-workgroup form (no rounds) on the same cases."""
    bad = []
    for name, k in _keys_cases(fccf, oracle).items():
        if k.size > 60_000:
            continue
        if not np.array_equal(ctx.sort_keys(k, exact_gate=True), oracle.sort_pairs(k)):
            bad.append(name)
    assert not bad, bad


@pytest.mark.gpu
def test_sort_keys_c3_leaf_keys(ctx, fccf, oracle):
    """The headline workload's first-pass keys (1M points, 0.05 m): deep, unbalanced tree."""
    c = fccf.CONFIGS["c3"]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    for pts in (src, tar):
        inv = np.float32(1.0) / np.float32(c["leaf"])
        minb = np.floor(pts.min(0) * inv).astype(np.int64)
        div = np.floor(pts.max(0) * inv).astype(np.int64) - minb + 1
        ijk = (np.floor(pts * inv) - minb.astype(np.float32)).astype(np.int64)
        k = (ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]).astype(np.uint32)
        assert np.array_equal(ctx.sort_keys(k), oracle.sort_pairs(k))


@pytest.mark.gpu
@pytest.mark.parametrize("n,leaf,seed", [(20_000, 0.1, 1), (150_000, 0.05, 2), (1_000_000, 0.05, 5)])
def test_downsample_equals_reference_order(ctx, fccf, oracle, n, leaf, seed):
    pts = fccf.synth_scene(n, seed=seed)
    out = ctx.downsample(pts, leaf)
    ref, _ = oracle.voxel_grid(pts, leaf, oracle.INTROSORT)
    assert out.shape == ref.shape
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("plan", ["large", "small"])
def test_round_plan_forms_equal_std_sort(ctx, fccf, oracle, plan, monkeypatch):
    """Both forms of the rounds' plan (FCCF_IS_PLAN: once per round by the last
    workgroups, the default from 2M points; or derived by every workgroup, below it) on
    every case and on the c3 keys, against the oracle's std::sort."""
    monkeypatch.setenv("FCCF_IS_PLAN", plan)
    cases = _keys_cases(fccf, oracle)
    c = fccf.CONFIGS["c3"]
    src, _, _ = fccf.synth_pair(c["n"], c["room"])
    inv = np.float32(1.0) / np.float32(c["leaf"])
    minb = np.floor(src.min(0) * inv).astype(np.int64)
    div = np.floor(src.max(0) * inv).astype(np.int64) - minb + 1
    ijk = (np.floor(src * inv) - minb.astype(np.float32)).astype(np.int64)
    cases["c3_src"] = (ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]).astype(np.uint32)
    bad = [name for name, k in cases.items() if not np.array_equal(ctx.sort_keys(k), oracle.sort_pairs(k))]
    assert not bad, bad
    out = ctx.downsample(src, c["leaf"])
    ref, _ = oracle.voxel_grid(src, c["leaf"], oracle.INTROSORT)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_sort_rank_ranges(ctx, fccf, oracle, world, monkeypatch):
    """Row D on the device: the sort run as rank r of N (FCCF_SHARD_D_SIM; the ranks'
    exchange itself is covered by the virtual-rank registrations in test_gpu_group.py)
    sorts exactly its range [lo, hi) of the std::sort order, and the ranges tile the
    whole sort."""
    rng = np.random.default_rng(11)
    c = fccf.CONFIGS["c3"]
    src, _, _ = fccf.synth_pair(c["n"], c["room"])
    inv = np.float32(1.0) / np.float32(c["leaf"])
    minb = np.floor(src.min(0) * inv).astype(np.int64)
    div = np.floor(src.max(0) * inv).astype(np.int64) - minb + 1
    ijk = (np.floor(src * inv) - minb.astype(np.float32)).astype(np.int64)
    cases = {"c3_src": (ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]).astype(np.uint32),
             "dups_300k": rng.integers(0, 60_000, 300_000).astype(np.uint32)}
    for name, k in cases.items():
        ref = oracle.sort_pairs(k)
        prev = 0
        for r in range(world):
            monkeypatch.setenv("FCCF_SHARD_D_SIM", f"{r}/{world}")
            got = ctx.sort_keys(k)
            raw = ctx.sort_stats()["raw"]
            lo, hi = int(raw[28]), int(raw[29])
            assert lo == prev and hi >= lo, (name, r, lo, hi)
            assert np.array_equal(got[lo:hi], ref[lo:hi]), (name, r)
            prev = hi
        assert prev == ref.size, name
        monkeypatch.delenv("FCCF_SHARD_D_SIM")


@pytest.mark.gpu
@pytest.mark.parametrize("copies", [2, 6, 10])
def test_batched_sort_equals_std_sort(ctx, fccf, oracle, copies):
    """The sort as a pipelined stage group runs it: `copies` clouds per launch (grid y;
    the block kernel's second form from six on), with the sorted points written by the
    finish kernels (fccf_debug_sort_keys_batch).  Copy 0's order equals std::sort on
    structured, duplicate-heavy and adversarial keys."""
    cases = _keys_cases(fccf, oracle)
    rng = np.random.default_rng(5)
    for name in ("room_200k", "room_200k_nan", "dups_300k", "adversary_20000", "adversary_ties_5000",
                 "rand8_40000", "randbig_15000"):
        k = cases[name]
        pts = rng.random((k.size, 3), dtype=np.float32)
        perm, ms = ctx.sort_keys_batch(k, copies, pts)
        ref = oracle.sort_pairs(k)
        assert ms > 0.0
        assert np.array_equal(perm[:ref.size], ref), name
