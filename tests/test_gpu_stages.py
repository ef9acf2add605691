"""GPU stage exports against the CPU oracle's intermediates (SURVEY.md §8(b) "stage
exports"): fccf_stage_match (the coplane-pair correspondence search + candidate
transforms, FCCF.cpp:1410-1428, :841-1018), its source-pair sharding (§8(e)), and
fccf_stage_fine_verify (FCCF.cpp:785-839).  Inputs are the oracle's own planes,
pairs, residual clouds and evaluated transforms; the bar is bit-exact."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module", params=["c2", "c3"])
def case(request, oracle, fccf):
    c = fccf.CONFIGS[request.param]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    run = oracle.Run(src, tar, c["leaf"], oracle.INTROSORT)
    tabs = dict(F1=fccf.planes_from_dump(run.get("planes1")), B1=fccf.bases_from_dump(run.get("bases1", np.int32)),
                F2=fccf.planes_from_dump(run.get("planes2")), B2=fccf.bases_from_dump(run.get("bases2", np.int32)))
    return run, tabs


def test_match_stage_bit_exact(ctx, case):
    run, t = case
    cands, k_pass = ctx.match(t["F1"], t["B1"], t["F2"], t["B2"])
    for ty in range(3):
        ref = run.get(f"cand{ty}").reshape(-1, 4, 4)
        assert cands[ty].shape == ref.shape, ty
        np.testing.assert_array_equal(bits(cands[ty]), bits(ref))
    assert sum(len(c) for c in cands) > 0
    assert k_pass == run.get("counts", np.int64)[1] > 0


@pytest.mark.parametrize("world", [2, 3, 8, 200])
def test_match_sharded_concat_equals_full(ctx, case, fccf, world):
    import shard
    _, t = case
    full, kp = ctx.match(t["F1"], t["B1"], t["F2"], t["B2"])
    parts = []
    for r in range(world):
        lo, hi = shard.shard_range(len(t["B1"]), r, world)
        parts.append(shard.pack(*ctx.match(t["F1"], t["B1"], t["F2"], t["B2"], lo, hi)))
    got, kp2 = shard.combine(parts)
    assert kp2 == kp
    for ty in range(3):
        np.testing.assert_array_equal(bits(got[ty]), bits(full[ty]))


def test_match_stage_edges(ctx, fccf, case):
    _, t = case
    c, kp = ctx.match(t["F1"], t["B1"][:0], t["F2"], t["B2"])  # no source pairs
    assert kp == 0 and all(len(x) == 0 for x in c)
    c, kp = ctx.match(t["F1"], t["B1"], t["F2"], t["B2"], 3, 3)  # empty shard
    assert kp == 0 and all(len(x) == 0 for x in c)
    bad = t["B1"].copy()
    bad[0]["i1"] = len(t["F1"])  # a pair naming a plane past the table
    with pytest.raises(fccf.FCCFError) as e:
        ctx.match(t["F1"], bad, t["F2"], t["B2"])
    assert e.value.code == fccf.E_ARG
    with pytest.raises(fccf.FCCFError):
        ctx.match(t["F1"], t["B1"], t["F2"], t["B2"], 2, 1)


def test_fine_verify_stage_bit_exact(ctx, case):
    run, _ = case
    fv = np.concatenate([run.get(f"fv{ty}").reshape(-1, 18) for ty in range(3)])
    assert len(fv) > 0
    s1, s2 = run.get("res1").reshape(-1, 3), run.get("res2").reshape(-1, 3)
    got = ctx.fine_verify(s1, s2, fv[:, :16].reshape(-1, 4, 4), 0.5)
    np.testing.assert_array_equal(bits(got), bits(fv[:, 17]))
    # the same transforms one at a time, and in reverse order: evaluations are independent
    one = np.array([ctx.fine_verify(s1, s2, fv[i, :16], 0.5)[0] for i in range(len(fv))], np.float32)
    np.testing.assert_array_equal(bits(one), bits(fv[:, 17]))
    rev = ctx.fine_verify(s1, s2, fv[::-1, :16].reshape(-1, 4, 4), 0.5)
    np.testing.assert_array_equal(bits(rev[::-1]), bits(fv[:, 17]))


def test_fine_verify_identity_and_args(ctx, fccf):
    rng = np.random.default_rng(3)
    s = (rng.random((5000, 3)) * 10).astype(np.float32)
    sc = ctx.fine_verify(s, s, np.eye(4, dtype=np.float32), 0.5)
    assert sc[0] == np.float32(1.0)  # identical clouds: every leaf has s == t
    with pytest.raises(fccf.FCCFError):
        ctx.fine_verify(s, s, np.tile(np.eye(4, dtype=np.float32), (17, 1, 1)), 0.5)  # > 16 evaluations
    with pytest.raises(fccf.FCCFError):
        ctx.fine_verify(s[:0], s, np.eye(4, dtype=np.float32), 0.5)


def test_match_sharded_two_ranks_gloo(tmp_path, oracle, fccf):
    """Two processes, one fccf_ctx each, source pairs split over the ranks, candidates
    all-gathered over gloo; rank 0's combined lists equal the oracle's."""
    c = fccf.CONFIGS["c2"]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    run = oracle.Run(src, tar, c["leaf"], oracle.INTROSORT)
    np.savez(tmp_path / "in.npz", planes1=run.get("planes1"), bases1=run.get("bases1", np.int32),
             planes2=run.get("planes2"), bases2=run.get("bases2", np.int32))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29547", os.path.join(ROOT, "tests", "shard_worker.py"),
           str(tmp_path / "in.npz"), str(tmp_path / "out.npz")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = np.load(tmp_path / "out.npz")
    for ty in range(3):
        np.testing.assert_array_equal(bits(out[f"cand{ty}"]), bits(run.get(f"cand{ty}").reshape(-1, 4, 4)))
    assert json.loads(str(out["meta"]))["world"] == 2


def voxels_from_dump(fccf, a):
    a = np.asarray(a, np.float32).reshape(-1, 8)
    v = np.zeros(len(a), fccf.VOXEL_DTYPE)
    v["c"], v["n"], v["count"] = a[:, 0:3], a[:, 3:6], a[:, 6].astype(np.int32)
    return v


@pytest.mark.parametrize("k", [1, 2])
def test_voxel_planes_stage_bit_exact(ctx, case, fccf, k):
    run, _ = case
    vox, res, cen = ctx.voxel_planes(run.get(f"ds{k}").reshape(-1, 3))
    ref = run.get(f"vox{k}").reshape(-1, 8)
    assert len(vox) == len(ref) > 0
    np.testing.assert_array_equal(bits(vox["c"]), bits(ref[:, 0:3]))
    np.testing.assert_array_equal(bits(vox["n"]), bits(ref[:, 3:6]))
    np.testing.assert_array_equal(vox["count"], ref[:, 6].astype(np.int32))
    np.testing.assert_array_equal(bits(res), bits(run.get(f"res{k}").reshape(-1, 3)))
    np.testing.assert_array_equal(bits(cen), bits(run.get(f"centroid{k}")))


@pytest.mark.parametrize("k", [1, 2])
def test_grow_stage_bit_exact(ctx, case, fccf, k):
    run, _ = case
    planes, theta, bases = ctx.grow(voxels_from_dump(fccf, run.get(f"vox{k}")), k)
    ref_p = fccf.planes_from_dump(run.get(f"planes{k}"))
    assert len(planes) == len(ref_p) > 0
    np.testing.assert_array_equal(planes.view(np.uint8), ref_p.view(np.uint8))
    np.testing.assert_array_equal(theta.view(np.uint64), run.get(f"theta{k}", np.float64).view(np.uint64))
    np.testing.assert_array_equal(bases.view(np.uint8),
                                  fccf.bases_from_dump(run.get(f"bases{k}", np.int32)).view(np.uint8))


def test_stage_chain_equals_registration(ctx, case, fccf):
    """ds -> voxel_planes -> grow -> match through the stage exports alone reproduces
    the registration's candidate lists."""
    run, _ = case
    tabs = []
    for k in (1, 2):
        vox, _, _ = ctx.voxel_planes(run.get(f"ds{k}").reshape(-1, 3))
        planes, _, bases = ctx.grow(vox, k)
        tabs += [planes, bases]
    cands, _ = ctx.match(*tabs)
    for ty in range(3):
        np.testing.assert_array_equal(bits(cands[ty]), bits(run.get(f"cand{ty}").reshape(-1, 4, 4)))


def test_voxel_planes_and_grow_edges(ctx, fccf):
    vox, res, cen = ctx.voxel_planes(np.zeros((0, 3), np.float32))
    assert len(vox) == 0 and len(res) == 0
    planes, theta, bases = ctx.grow(vox, 1)
    assert len(planes) == 0 and len(bases) == 0
    with pytest.raises(fccf.FCCFError):
        ctx.grow(vox, 3)


def test_cluster_stage_bit_exact(ctx, case, fccf):
    run, _ = case
    counts = run.get("counts", np.int64)  # K, K_pass, |cand t| x3, clusters t x3, ...
    cands = [run.get(f"cand{t}").reshape(-1, 4, 4) for t in range(3)]
    total = sum(len(c) for c in cands)
    for t in range(3):
        cluster_num = int(np.float32(200.0) * np.float32(len(cands[t])) / np.float32(total)) if total else 0
        fine, ncl = ctx.cluster(cands[t], cluster_num)
        ref = run.get(f"fine{t}").reshape(-1, 8)
        assert fine.shape == ref.shape, t
        np.testing.assert_array_equal(bits(fine), bits(ref))
        assert ncl == counts[5 + t]


@pytest.mark.parametrize("world", [2, 3])
def test_downsample_sharded_by_leaf_ranges(ctx, oracle, fccf, world):
    """§8(e) row D: a cloud held as `world` input-order slices (one fccf_ctx per rank,
    threads on one GPU): every rank's output == the whole-cloud GPU pass == the
    oracle (reference std::sort order), bitwise."""
    import test_shard
    c = fccf.CONFIGS["c2"]
    src, _, _ = fccf.synth_pair(c["n"], c["room"])
    src = src.copy()
    src[[5, 777, 40_000]] = np.nan
    whole = ctx.downsample(src, c["leaf"])
    np.testing.assert_array_equal(bits(whole), bits(oracle.voxel_grid(src, c["leaf"], oracle.INTROSORT)[0]))
    ctxs = [fccf.Ctx(0) for _ in range(world)]
    try:
        outs = test_shard.run_sharded(src, c["leaf"], world, ctx_of=lambda r: ctxs[r])
    finally:
        for x in ctxs:
            x.close()
    for got in outs:
        np.testing.assert_array_equal(bits(got), bits(whole))
