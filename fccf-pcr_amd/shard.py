"""Sharded coplane-pair correspondence search (SURVEY.md §8(e), row "K5").

The reference runs the search as one loop nest, source pairs outer, target pairs
inner (FCCF.cpp:1410-1428), and appends every candidate transform to T_vec[type] in
that order.  Here the source pairs B1 are split into contiguous blocks, one per rank
(`shard_range`).  Every rank runs the GPU search (`Ctx.match`, i.e. fccf_stage_match)
for its block against all target pairs.  The per-type candidate lists are then
all-gathered and concatenated in rank order.  Because the loop order is b1-major, the
result equals the unsharded list bit for bit.

Plane extraction, growth and selection stay replicated on every rank (they are
sequential and tiny), so F1, B1, F2 and B2 are already identical everywhere. The
only exchange is the candidate gather: a variable-length all-gather of <= a few MB.
It runs on the process group's CPU backend (gloo): libfccf owns the GPU through the
system HIP runtime, and torch's own ROCm runtime cannot share the device in the same
process.

`gather` is injectable so the exchange logic can be tested without a GPU.
"""
from __future__ import annotations

import numpy as np


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block [lo, hi) of n items for `rank`: sizes differ by at most one,
    lower ranks take the larger blocks, ranks past n get empty blocks."""
    if world < 1 or not 0 <= rank < world or n < 0:
        raise ValueError(f"bad shard: n={n} rank={rank} world={world}")
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def torch_gather(group=None):
    """All-gather of one float32 or float64 array of any length per rank over
    torch.distributed (CPU tensors: gloo).  Returns the arrays in rank order."""
    import torch
    import torch.distributed as dist

    def gather(a: np.ndarray) -> list[np.ndarray]:
        a = np.ascontiguousarray(a).reshape(-1)
        if a.dtype not in (np.float32, np.float64):
            raise TypeError(f"gather: float32/float64 only, got {a.dtype}")
        dt = torch.float64 if a.dtype == np.float64 else torch.float32
        world = dist.get_world_size(group)
        n = torch.tensor([a.size], dtype=torch.int64)
        ns = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(ns, n, group=group)
        sizes = [int(x.item()) for x in ns]
        cap = max(max(sizes), 1)
        buf = torch.zeros(cap, dtype=dt)
        buf[: a.size] = torch.from_numpy(a)
        outs = [torch.zeros(cap, dtype=dt) for _ in range(world)]
        dist.all_gather(outs, buf, group=group)
        return [o[:s].numpy().copy() for o, s in zip(outs, sizes)]

    return gather


def pack(cands: list[np.ndarray], k_pass: int) -> np.ndarray:
    """One float32 message per rank: [n0, n1, n2, k_pass] as exact integer floats
    (all < 2^24), then the three candidate lists (16 floats per candidate)."""
    head = np.array([len(c) for c in cands] + [k_pass], np.float64)
    if head.max(initial=0) >= 2 ** 24:
        raise ValueError("candidate count past the exact float32 range")
    return np.concatenate([head.astype(np.float32)] + [np.asarray(c, np.float32).reshape(-1) for c in cands])


def unpack(msg: np.ndarray) -> tuple[list[np.ndarray], int]:
    n = [int(x) for x in msg[:3]]
    k_pass = int(msg[3])
    out, o = [], 4
    for t in range(3):
        out.append(msg[o: o + 16 * n[t]].reshape(n[t], 4, 4))
        o += 16 * n[t]
    if o != msg.size:
        raise ValueError("malformed candidate message")
    return out, k_pass


def combine(msgs: list[np.ndarray]) -> tuple[list[np.ndarray], int]:
    """Rank-ordered concatenation of every rank's lists = the reference loop order."""
    parts = [unpack(m) for m in msgs]
    cands = [np.concatenate([p[0][t] for p in parts]).reshape(-1, 4, 4) for t in range(3)]
    return cands, sum(p[1] for p in parts)


def match_sharded(ctx, F1, B1, F2, B2, rank: int, world: int, gather, params=None):
    """This rank's block of the search on its GPU, then the ordered gather.
    Every rank returns the full ([cand_t], k_pass), identical to ctx.match(F1, B1, F2, B2)."""
    lo, hi = shard_range(len(B1), rank, world)
    cands, k_pass = ctx.match(F1, B1, F2, B2, lo, hi, params)
    return combine(gather(pack(cands, k_pass)))


# ---------------------------------------------------------------- fine_verify (row F)
# SURVEY.md §8(e) row F.  The <= 16 evaluations (the top fine_verify_number candidates
# of each type, FCCF.cpp:1526-1536) are independent: each rank scores a contiguous
# block (shard_range) on its GPU, the scores are gathered in rank order, and every rank
# fuses the same E scores.  Inside libfccf the same split runs over the group's own
# fine-verification communicator (group.cpp, group_fine_gather); this is its mirror for
# callers that drive the stages themselves.


def fine_verify_sharded(ctx, s1, s2, T, voxel: float, rank: int, world: int, gather):
    """This rank's block of fine_verify(s1, s2, T[e]) on its GPU, then the ordered gather.
    Every rank returns the E float32 scores, identical to ctx.fine_verify(s1, s2, T, voxel)."""
    T = np.ascontiguousarray(T, np.float32).reshape(-1, 4, 4)
    lo, hi = shard_range(len(T), rank, world)
    mine = ctx.fine_verify(s1, s2, T[lo:hi], voxel) if hi > lo else np.zeros(0, np.float32)
    parts = gather(np.asarray(mine, np.float32))
    out = np.concatenate([np.asarray(p, np.float32).reshape(-1) for p in parts])
    if out.size != len(T):
        raise ValueError(f"fine_verify gather: {out.size} scores for {len(T)} evaluations")
    return out


# ---------------------------------------------------------------- VoxelGrid (row D)
# SURVEY.md §8(e) row D.  Helpers shared with the tests' CPU stand-in: PCL's leaf
# coordinates floor(p * (1/leaf)) in float32 and its int32 overflow guard
# ("Integer indices would overflow": output = input) on the finite bounding box.


def leaf_coords(xyz: np.ndarray, leaf: float):
    """floor(p * (1/leaf)) computed in float32 as PCL does (int64), and the finite mask."""
    a = np.asarray(xyz, np.float32).reshape(-1, 3)
    inv = np.float32(1.0) / np.float32(leaf)
    fin = np.isfinite(a).all(axis=1)
    with np.errstate(invalid="ignore", over="ignore"):
        f = np.floor(a * inv)
    return np.where(fin[:, None], f, 0).astype(np.int64), fin


def voxel_grid_overflows(mn, mx, leaf: float) -> bool:
    """PCL's guard, (int)((max - min) * inv) + 1 per axis in float32, on the finite bbox."""
    inv = np.float32(1.0) / np.float32(leaf)
    d = [int(np.float32(np.float32(mx[a]) - np.float32(mn[a])) * inv) + 1 for a in range(3)]
    return d[0] * d[1] * d[2] > 2 ** 31 - 1


def downsample_sharded(ctx, xyz_slice, leaf: float, rank: int, world: int, gather):
    """Global VoxelGrid of a cloud split over ranks in input order (rank r holds the
    r-th contiguous slice).  Every rank returns the full output, equal to
    ctx.downsample(whole cloud).

    PCL orders the points of a leaf by one std::sort over the cloud's whole index
    vector (FCCF.cpp:1668-1678); that introsort's partition tree spans every leaf, so
    no split by leaf ranges reproduces the within-leaf summation order.  The pass is
    therefore replicated: the slices are gathered in rank order (= input order) and
    each rank runs the whole-cloud pass (one ~0.1 ms GPU pass at c3)."""
    a = np.ascontiguousarray(np.asarray(xyz_slice, np.float32).reshape(-1))
    whole = np.concatenate([np.asarray(s, np.float32).reshape(-1) for s in gather(a)]).reshape(-1, 3)
    if whole.shape[0] == 0:
        return np.zeros((0, 3), np.float32)
    return ctx.downsample(whole, leaf)


# ---------------------------------------------------------------- row P (face stage)
FACE_BINS_LG = 12  # facefit.hip FACE_BINS_LG


def face_bin_bounds(codes, nbits: int, world: int) -> np.ndarray:
    """Row P's split (group.cpp face_voxels_sharded, facefit.hip k_face_range): the
    points' leaf codes binned by their top FACE_BINS_LG bits (a leaf's points share one
    code, so a bin never splits a leaf); bound j = the first bin b whose preceding
    points * world >= j * n; rank r takes bins [bounds[r], bounds[r + 1])."""
    shift = max(0, int(nbits) - FACE_BINS_LG)
    c = np.asarray(codes, np.uint64)
    hist = np.bincount((c >> np.uint64(shift)).astype(np.int64) & ((1 << FACE_BINS_LG) - 1),
                       minlength=1 << FACE_BINS_LG)
    before = np.concatenate([[0], np.cumsum(hist)[:-1]]).astype(np.int64)
    n = int(c.size)
    b = np.full(world + 1, 1 << FACE_BINS_LG, np.int64)
    b[0] = 0
    for j in range(1, world):
        hit = np.flatnonzero(before * world >= j * n)
        b[j] = hit[0] if hit.size else 1 << FACE_BINS_LG
    return b


def face_rank_points(codes, nbits: int, rank: int, world: int) -> np.ndarray:
    """The input positions of rank `rank`'s points in leaf order: its bins' points in
    input order, stably sorted by code (PCL's insertion order within a leaf)."""
    c = np.asarray(codes, np.uint64)
    shift = max(0, int(nbits) - FACE_BINS_LG)
    b = face_bin_bounds(c, nbits, world)
    bins = (c >> np.uint64(shift)).astype(np.int64) & ((1 << FACE_BINS_LG) - 1)
    mine = np.flatnonzero((bins >= b[rank]) & (bins < b[rank + 1]))
    return mine[np.argsort(c[mine], kind="stable")]
