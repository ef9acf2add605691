"""CPU checks of the sharded stages' host logic (fccf-pcr_amd/shard.py): block ranges,
the message format, rank-ordered concatenation (K5 search, F fine verification, D
VoxelGrid, and the K1 sort's row-D split via tests/introsort_model.py), and the gloo
gather with world_size 2.  The GPU search itself is stubbed by a deterministic b1-major generator;
the real one is tested in tests/test_gpu_stages.py."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fccf-pcr_amd"))
import shard  # noqa: E402


class StubCtx:
    """ctx.match stand-in: b1 emits (b1 % 3) candidates of type (b1 % 3) ... in b1-major order."""

    def match(self, F1, B1, F2, B2, lo=0, hi=-1, params=None):
        hi = len(B1) if hi < 0 else hi
        out = [[], [], []]
        kp = 0
        for b1 in range(lo, hi):
            for b2 in range(len(B2)):
                k = (b1 * 7 + b2) % 4
                kp += k > 0
                for j in range(k):
                    m = np.eye(4, dtype=np.float32)
                    m[:3, 3] = (b1, b2, j)
                    out[(b1 + b2) % 3].append(m)
        return [np.array(o, np.float32).reshape(-1, 4, 4) for o in out], kp


@pytest.mark.parametrize("n,world", [(0, 1), (0, 4), (5, 8), (120, 7), (136, 8), (14, 3)])
def test_shard_range_partitions(n, world):
    rs = [shard.shard_range(n, r, world) for r in range(world)]
    assert rs[0][0] == 0 and rs[-1][1] == n
    for (a, b), (c, d) in zip(rs, rs[1:]):
        assert b == c and a <= b
    sizes = [b - a for a, b in rs]
    assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)


def test_shard_range_rejects():
    with pytest.raises(ValueError):
        shard.shard_range(4, 2, 2)
    with pytest.raises(ValueError):
        shard.shard_range(4, 0, 0)


def test_pack_roundtrip():
    c = [np.arange(32, dtype=np.float32).reshape(2, 4, 4), np.zeros((0, 4, 4), np.float32),
         np.full((1, 4, 4), np.nan, np.float32)]
    got, kp = shard.unpack(shard.pack(c, 5))
    assert kp == 5
    for a, b in zip(got, c):
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    with pytest.raises(ValueError):
        shard.unpack(shard.pack(c, 5)[:-1])


@pytest.mark.parametrize("world", [1, 2, 3, 8, 40])
def test_stub_sharded_equals_full(world):
    ctx = StubCtx()
    B1, B2 = list(range(37)), list(range(11))
    full, kp = ctx.match(None, B1, None, B2)
    msgs = []
    for r in range(world):
        lo, hi = shard.shard_range(len(B1), r, world)
        msgs.append(shard.pack(*ctx.match(None, B1, None, B2, lo, hi)))
    got, kp2 = shard.combine(msgs)
    assert kp2 == kp
    for a, b in zip(got, full):
        np.testing.assert_array_equal(a, b)


WORKER = r'''
import sys, numpy as np, torch.distributed as dist
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import shard, test_shard
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
ctx = test_shard.StubCtx()
B1, B2 = list(range(29)), list(range(9))
got, kp = shard.match_sharded(ctx, None, B1, None, B2, r, w, shard.torch_gather())
full, kp0 = ctx.match(None, B1, None, B2)
assert kp == kp0, (kp, kp0)
for a, b in zip(got, full):
    assert np.array_equal(a, b)
T = test_shard.evals(7)
sc = shard.fine_verify_sharded(test_shard.StubFineCtx(), None, None, T, 0.5, r, w, shard.torch_gather())
assert np.array_equal(sc.view(np.uint32), test_shard.StubFineCtx().fine_verify(None, None, T, 0.5).view(np.uint32))
import introsort_model as IM
keys = test_shard.sort_case(2500, 5)
(lo, hi), part = IM.sharded_rank(keys, r, w, 64, 4)
whole = np.concatenate(shard.torch_gather()(np.asarray(part, np.float64))).astype(np.int64)
assert whole.tolist() == IM.std_sort(keys), "sharded sort differs"
xyz = test_shard.cloud(3000, 11)
lo, hi = shard.shard_range(len(xyz), r, w)
vctx = test_shard.StubVoxelCtx()
got = shard.downsample_sharded(vctx, xyz[lo:hi], 0.25, r, w, shard.torch_gather())
assert np.array_equal(got.view(np.uint32), vctx.downsample(xyz, 0.25).view(np.uint32))
codes, nbits = test_shard.face_codes(40000, 9)
part = shard.face_rank_points(codes, nbits, r, w)
whole = np.concatenate(shard.torch_gather()(part.astype(np.float64))).astype(np.int64)
assert np.array_equal(whole, np.argsort(codes, kind="stable")), "row P split differs"
dist.barrier(); dist.destroy_process_group()
print("ok", r)
'''


class StubFineCtx:
    """ctx.fine_verify stand-in: a score per transform that depends on that transform only."""

    def fine_verify(self, s1, s2, T, voxel):
        T = np.asarray(T, np.float32).reshape(-1, 4, 4)
        return (T[:, :3, 3].sum(axis=1) * np.float32(voxel) + np.float32(1)).astype(np.float32)


def evals(E, seed=3):
    rng = np.random.default_rng(seed)
    T = np.tile(np.eye(4, dtype=np.float32), (E, 1, 1))
    T[:, :3, 3] = rng.random((E, 3), np.float32)
    return T


@pytest.mark.parametrize("E,world", [(0, 2), (1, 3), (5, 2), (16, 3), (15, 8), (3, 16)])
def test_fine_verify_sharded_equals_whole(E, world):
    """Row F's exchange: blocks of the E evaluations, gathered in rank order (ranks past
    E contribute empty blocks)."""
    T = evals(E)
    want = StubFineCtx().fine_verify(None, None, T, 0.5)
    import threading
    gs, res = thread_gathers(world), [None] * world

    def work(r):
        res[r] = shard.fine_verify_sharded(StubFineCtx(), None, None, T, 0.5, r, world, gs[r])
    th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for got in res:
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def sort_case(n, seed):
    """VoxelGrid-like keys: many duplicates, a few invalid (non-finite) points."""
    rng = np.random.default_rng(seed)
    k = rng.integers(0, max(1, n // 4), n).astype(np.uint32)
    k[rng.integers(0, n, 5)] = 0xFFFFFFFF
    return k


@pytest.mark.parametrize("n,world,seed", [(3000, 2, 1), (5000, 3, 2), (4000, 8, 3), (700, 4, 4)])
def test_sharded_sort_model_equals_std_sort(oracle, n, world, seed):
    """Row D's decomposition of K1's sort (csrc/introsort.hip plan_round / k_is_block):
    levels < r0 replicated, then each rank finishes the segments starting in its
    range; the rank-ordered concatenation equals std::sort (the oracle's) exactly."""
    import introsort_model as IM
    keys = sort_case(n, seed)
    ref = oracle.sort_pairs(keys).tolist()
    assert IM.std_sort(keys) == ref
    r0 = (world - 1).bit_length() + 3
    parts = [IM.sharded_rank(keys, r, world, 64, r0) for r in range(world)]
    assert parts[0][0][0] == 0 and parts[-1][0][1] == len(ref)
    for (a, b), _ in parts:
        assert a <= b
    for ((_, b), _), ((c, _), _) in zip(parts, parts[1:]):
        assert b == c
    assert [i for _, p in parts for i in p] == ref
    assert sum(1 for (a, b), _ in parts if b > a) > 1  # the work is actually split


def cloud(n, seed, nan=True):
    rng = np.random.default_rng(seed)
    xyz = (rng.random((n, 3)) * np.array([6.0, 4.0, 2.0]) - 1.0).astype(np.float32)
    if nan:
        xyz[rng.integers(0, n, 7)] = np.nan
        xyz[rng.integers(0, n, 3), 1] = np.inf
    return xyz


class StubVoxelCtx:
    """Stand-in for the GPU VoxelGrid (tests only) with PCL's leaf keys, overflow guard
    and sequential float32 sums; the within-leaf order here is the input order (the
    exchange logic under test does not depend on it)."""

    def downsample(self, xyz, leaf):
        a = np.asarray(xyz, np.float32).reshape(-1, 3)
        f, fin = shard.leaf_coords(a, leaf)
        if not fin.any():
            return np.zeros((0, 3), np.float32)
        mn, mx = a[fin].min(axis=0), a[fin].max(axis=0)
        if shard.voxel_grid_overflows(mn, mx, leaf):
            return a.copy()
        lo = f[fin].min(axis=0)
        div = f[fin].max(axis=0) - lo + 1
        key = (f[:, 0] - lo[0]) + div[0] * ((f[:, 1] - lo[1]) + div[1] * (f[:, 2] - lo[2]))
        idx = np.flatnonzero(fin)
        idx = idx[np.argsort(key[idx], kind="stable")]
        out, s = [], 0
        while s < len(idx):
            e = s
            acc = np.zeros(3, np.float32)
            while e < len(idx) and key[idx[e]] == key[idx[s]]:
                acc = (acc + a[idx[e]]).astype(np.float32)
                e += 1
            out.append(acc / np.float32(e - s))
            s = e
        return np.array(out, np.float32).reshape(-1, 3)


def thread_gathers(world):
    """In-process stand-in for the collective: one gather per rank thread."""
    import threading
    buf = [None] * world
    bar = threading.Barrier(world)

    def make(r):
        def g(a):
            buf[r] = np.array(a).reshape(-1)
            bar.wait()
            out = list(buf)
            bar.wait()
            return out
        return g
    return [make(r) for r in range(world)]


def run_sharded(xyz, leaf, world, ctx_of=lambda r: StubVoxelCtx()):
    import threading
    gs, res = thread_gathers(world), [None] * world

    def work(r):
        lo, hi = shard.shard_range(len(xyz), r, world)
        res[r] = shard.downsample_sharded(ctx_of(r), xyz[lo:hi], leaf, r, world, gs[r])
    th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return res


@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_downsample_sharded_equals_whole(world):
    xyz = cloud(4000, world)
    want = StubVoxelCtx().downsample(xyz, 0.2)
    for got in run_sharded(xyz, 0.2, world):
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def test_downsample_sharded_overflow_and_empty():
    xyz = cloud(500, 9, nan=False)
    xyz[0] = (-3e4, -3e4, -3e4)  # (extent / leaf)^3 past int32: PCL passes the cloud through
    xyz[1, 1] = np.nan
    for got in run_sharded(xyz, 0.05, 3):
        np.testing.assert_array_equal(got.view(np.uint32), xyz.view(np.uint32))
    allnan = np.full((10, 3), np.nan, np.float32)
    for got in run_sharded(allnan, 0.1, 2):
        assert got.shape == (0, 3)


def test_gloo_two_ranks(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(WORKER)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29539", str(script),
           os.path.join(ROOT, "fccf-pcr_amd"), os.path.join(ROOT, "tests")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.count("ok") == 2


def face_codes(n, seed):
    """Leaf codes of a synthetic cloud: ~n/20 occupied leaves of a depth-7 octree (22-bit
    codes), clustered like a room's surfaces, points of a leaf scattered in input order."""
    rng = np.random.default_rng(seed)
    leaves = np.unique(rng.integers(0, 1 << 21, n // 20) * 2 + (rng.random(n // 20) < 0.1))
    leaves = np.sort(leaves)[: max(1, n // 20)]
    return leaves[np.minimum(rng.zipf(1.3, n), leaves.size) - 1].astype(np.uint64), 22


@pytest.mark.parametrize("world", [1, 2, 3, 8, 64])
def test_face_split_concatenates_to_leaf_order(world):
    """Row P: the ranks' bin ranges tile the code space, no leaf is
    split across ranks, the ranks' sizes are balanced, and their leaf-ordered points
    concatenated in rank order are the unsharded leaf order (code, then input position)."""
    codes, nbits = face_codes(50_000, 4)
    parts = [shard.face_rank_points(codes, nbits, r, world) for r in range(world)]
    whole = np.concatenate(parts)
    assert np.array_equal(whole, np.argsort(codes, kind="stable"))
    leaf_rank = {}
    for r, p in enumerate(parts):
        for c in np.unique(codes[p]):
            assert leaf_rank.setdefault(int(c), r) == r
    sizes = [len(p) for p in parts]
    assert sum(sizes) == len(codes)
