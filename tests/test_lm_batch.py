"""quick_verify's LM (FCCF.cpp:210-249, Ceres 1.14 LM; host_stages.cpp lm_solve) solved
several problems at a time with SIMD across the problems (csrc/lm_batch.cpp) must give
every problem the scalar form's result bit for bit, whatever its lane neighbours do
(different pair counts, early exits, failed evaluations).  Host only: runs without a GPU.
The scalar form itself is pinned against the oracle by the GPU registration tests
(`qv0-2` intermediates, tests/test_gpu_register.py)."""
import ctypes

import numpy as np
import pytest


def _rot(rng, deg):
    a = rng.normal(size=3)
    a /= np.linalg.norm(a)
    th = np.radians(deg)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def _problems(seed, n):
    """n plane-pair problems like quick_verify's: planes (point, unit normal) of a scene,
    the same planes moved by a small transform with noise, weights in (0, 1]; plus the
    edge cases the LM's control flow branches on."""
    rng = np.random.default_rng(seed)
    probs = []
    for i in range(n):
        P = int(rng.integers(4, 12))
        p1 = rng.uniform(-10, 10, (P, 3))
        n1 = rng.normal(size=(P, 3))
        n1 /= np.linalg.norm(n1, axis=1, keepdims=True)
        R = _rot(rng, rng.uniform(0, 3))
        t = rng.uniform(-0.3, 0.3, 3)
        p2 = (p1 - t) @ R + rng.normal(scale=0.02, size=(P, 3))
        n2 = n1 @ R + rng.normal(scale=0.01, size=(P, 3))
        w = rng.uniform(0.05, 1.0, (P, 1))
        kind = i % 11
        if kind == 3:
            w[:] = 0.0  # zero residuals: gradient test ends it at once
        elif kind == 5:
            p2[0, 0] = np.nan  # the first evaluation fails
        elif kind == 7:
            p2 = p1.copy()  # already aligned
            n2 = n1.copy()
        elif kind == 9:
            p1 *= 1e6  # badly scaled
        probs.append(np.hstack([p1, n1, p2, n2, w]).astype(np.float32))
    return probs


def _solve(fccf, probs, lanes):
    pairs = np.ascontiguousarray(np.vstack(probs), dtype=np.float32)
    P = np.array([p.shape[0] for p in probs], np.int32)
    best = np.zeros((len(probs), 7), np.float64)
    fn = fccf._lib.fccf_debug_lm_batch
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
    rc = fn(pairs.ctypes.data, P.ctypes.data, len(probs), lanes, best.ctypes.data)
    return rc, best


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_lm_batch_lanes_equal_scalar(fccf, seed):
    probs = _problems(seed, 61)  # 61: ragged last groups of 4 and 8
    rc, ref = _solve(fccf, probs, 1)
    assert rc == 0
    assert np.isfinite(ref).all()
    tried = 0
    for lanes in (4, 8, 0):
        rc, got = _solve(fccf, probs, lanes)
        if rc == fccf.E_ARG:  # this CPU lacks that vector width
            continue
        assert rc == 0
        tried += 1
        bad = np.flatnonzero((got.view(np.uint64) != ref.view(np.uint64)).any(axis=1))
        assert bad.size == 0, (lanes, bad[:10])
    assert tried >= 1


def test_lm_batch_moves_the_problems(fccf):
    """The LM actually runs: well-posed problems leave the identity."""
    probs = _problems(4, 22)
    rc, best = _solve(fccf, probs, 0)
    assert rc == 0
    moved = np.abs(best - np.array([0, 0, 0, 1, 0, 0, 0])).max(axis=1) > 1e-6
    assert moved.sum() >= 10
