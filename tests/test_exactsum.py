"""Exact parallel left-to-right float32 sums (fccf-pcr_amd/csrc/exactsum.h).

The reference accumulates compute3DCentroid (FCCF.cpp:473) and fine_verify's
similar_num (FCCF.cpp:830-835) sequentially in float; libfccf reproduces those bits
with a parallel binade/envelope decomposition.  CPU: the algorithm itself (host
build of the header) against the naive loop.  GPU: the device kernels through the
C-ABI stage exports against numpy's strictly sequential float32 accumulate.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _seq(x):
    """((0 + x0) + x1) + ... in float32.  The leading +0 matters: 0 + (-0) = +0."""
    x = np.concatenate([np.zeros(1, np.float32), np.asarray(x, np.float32).reshape(-1)])
    return np.cumsum(x, dtype=np.float32)[-1]


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_algorithm_fuzz_host(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = tmp_path / "xs_fuzz"
    subprocess.run([hipcc, "-O2", "-std=c++17", "-ffp-contract=off", os.path.join(HERE, "xs_fuzz.cpp"), "-o",
                    str(exe)], check=True, capture_output=True)
    r = subprocess.run([str(exe), "450", "11"], capture_output=True, text=True, timeout=600)
    assert "mismatches 0" in r.stdout, r.stdout
    assert r.returncode == 0


def _cases():
    rng = np.random.default_rng(5)
    yield "empty", np.zeros(0, np.float32)
    yield "one", np.array([3.25], np.float32)
    yield "neg_zero", np.array([-0.0, -0.0], np.float32)
    for n in (255, 256, 257, 16383, 16384, 16385, 300001):
        yield f"pos{n}", (10 + 5 * rng.standard_normal(n)).astype(np.float32)
    yield "walk", (5 * rng.standard_normal(1 << 20)).astype(np.float32)
    yield "ties", (np.round(rng.standard_normal(200000) * 8) / 2).astype(np.float32)
    yield "mixed", np.where(rng.random(400000) < 0.5, 1e-3, 1e3).astype(np.float32) * \
        rng.standard_normal(400000).astype(np.float32)
    yield "tiny", (rng.random(100000) * 1e-30).astype(np.float32)
    x = (3 + rng.standard_normal(100000)).astype(np.float32)
    x[7::1000] = np.inf
    x[5000] = np.nan
    yield "nonfinite", x
    yield "big", (1e30 * rng.standard_normal(70000)).astype(np.float32)
    yield "terms", (rng.integers(2, 40, 2_000_000) * rng.random(2_000_000)).astype(np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("name,x", list(_cases()), ids=[c[0] for c in _cases()])
def test_seqsum_bitexact(ctx, name, x):
    got = ctx.seqsum(x)
    want = _seq(x)
    assert np.array_equal(np.array([got]).view(np.uint32), np.array([want]).view(np.uint32)) or \
        (np.isnan(got) and np.isnan(want)), (name, got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 1000, 262144, 1_500_001])
def test_centroid_bitexact(ctx, n):
    rng = np.random.default_rng(n)
    xyz = (rng.random((n, 3)) * np.array([20, -15, 4]) + np.array([-3, 2, 0.01])).astype(np.float32)
    got = ctx.centroid(xyz)
    if n == 0:
        want = np.array([0, 0, 0, 1], np.float32)
    else:
        want = np.array([_seq(xyz[:, k]) / np.float32(n) for k in range(3)] + [1], np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (got, want)


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_key_div_fuzz_host(tmp_path):
    """Octree keys without a double division (fccf_math.h key_div, used by k_oct_codes and
    k_fv_entries): the same integer as (uint32_t)(a / res) at and around every multiple
    of res, for the reference's voxel sizes and random ones."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = tmp_path / "keydiv_fuzz"
    subprocess.run([hipcc, "-O2", "-std=c++17", "-ffp-contract=off", "-x", "hip", "--offload-arch=gfx950",
                    os.path.join(HERE, "keydiv_fuzz.cpp"), "-o", str(exe)], check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert "mismatches 0" in r.stdout, r.stdout
    assert r.returncode == 0
