"""CPU checks of the sharded correspondence search's host logic (fccf-pcr_amd/shard.py):
block ranges, the message format, rank-ordered concatenation, and the gloo gather with
world_size 2.  The GPU search itself is stubbed by a deterministic b1-major generator;
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
dist.barrier(); dist.destroy_process_group()
print("ok", r)
'''


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
