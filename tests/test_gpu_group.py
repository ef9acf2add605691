"""Multi-GPU inside libfccf over RCCL (SURVEY.md §8(b) fccf_group_create, §8(e) row
K5, FCCF.cpp:1410-1428): with a group attached, the coplane-pair correspondence search
is sharded by source-pair blocks and the candidate lists are gathered in rank order over
RCCL; the registration must equal the unsharded one bit for bit.  A 1-rank
communicator runs the whole RCCL path (count all-gather, grouped broadcasts) on the
one-GPU box; two ranks on one GPU are attempted and skipped if RCCL refuses them.
The exchange logic itself is covered on CPU with world_size 2 (tests/test_shard.py)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def pair(fccf):
    c = fccf.CONFIGS["c2"]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    return src, tar, c["leaf"]


def test_single_rank_group_register_bit_exact(fccf, pair):
    src, tar, leaf = pair
    with fccf.Ctx(0) as ctx:
        T0, s0 = ctx.register(src, tar, leaf)
        with fccf.Group(ctx, fccf.group_unique_id(), 1, 0) as g:
            assert g.info() == (1, 0)
            T1, s1 = ctx.register(src, tar, leaf)
            Tb, _ = ctx.register_batch([(src, tar)] * 3, leaf)
        T2, _ = ctx.register(src, tar, leaf)  # detached again
    np.testing.assert_array_equal(bits(T1), bits(T0))
    np.testing.assert_array_equal(bits(T2), bits(T0))
    for T in Tb:
        np.testing.assert_array_equal(bits(T), bits(T0))
    assert (s1.K, s1.K_pass, list(s1.cand)) == (s0.K, s0.K_pass, list(s0.cand))


def test_single_rank_group_stage_match(fccf, oracle, pair):
    src, tar, leaf = pair
    run = oracle.Run(src, tar, leaf, oracle.INTROSORT)
    F1, B1 = fccf.planes_from_dump(run.get("planes1")), fccf.bases_from_dump(run.get("bases1", np.int32))
    F2, B2 = fccf.planes_from_dump(run.get("planes2")), fccf.bases_from_dump(run.get("bases2", np.int32))
    with fccf.Ctx(0) as ctx:
        ref, kp = ctx.match(F1, B1, F2, B2)
        with fccf.Group(ctx, fccf.group_unique_id(), 1, 0) as g:
            got, kp2 = g.match(F1, B1, F2, B2)
    assert kp2 == kp
    for t in range(3):
        np.testing.assert_array_equal(bits(got[t]), bits(ref[t]))
        np.testing.assert_array_equal(bits(got[t]), bits(run.get(f"cand{t}").reshape(-1, 4, 4)))


def test_group_rejects_bad_arguments(fccf):
    with fccf.Ctx(0) as ctx:
        with pytest.raises(ValueError):
            fccf.Group(ctx, b"short", 1, 0)
        with pytest.raises(fccf.FCCFError):
            fccf.Group(ctx, fccf.group_unique_id(), 1, 1)  # rank outside the group


def test_two_ranks_on_one_gpu(fccf, pair, tmp_path):
    src, tar, leaf = pair
    with fccf.Ctx(0) as ctx:
        T0, s0 = ctx.register(src, tar, leaf)
    idf = str(tmp_path / "uid")
    outs = [str(tmp_path / f"r{r}.json") for r in range(2)]
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "group_worker.py"), str(r), "2", idf, outs[r]])
             for r in range(2)]
    try:
        for p in procs:
            p.wait(timeout=100)
    except subprocess.TimeoutExpired:
        for p in procs:
            p.kill()
        pytest.skip("RCCL with two ranks on one GPU did not complete (one GPU per rank is the supported layout)")
    res = [json.load(open(o)) for o in outs]
    if any("error" in r for r in res):
        pytest.skip("RCCL refuses two ranks on one GPU: " + "; ".join(r.get("msg", "") for r in res))
    assert all(p.returncode == 0 for p in procs)
    for r in res:
        assert np.array_equal(np.array(r["T"], np.uint32), bits(T0).ravel())
        assert (r["K"], r["K_pass"], r["cand"]) == (s0.K, s0.K_pass, list(s0.cand))


def test_ctx_destroyed_before_its_group(fccf):
    """fccf_ctx_destroy detaches an attached group instead of leaving it pointing at
    freed memory; destroying the group afterwards only releases the communicator."""
    ctx = fccf.Ctx(0)
    g = fccf.Group(ctx, fccf.group_unique_id(), 1, 0)
    ctx.close()
    assert g.info() == (1, 0)
    g.close()
    with fccf.Ctx(0) as ctx2:  # the device is still usable
        g2 = fccf.Group(ctx2, fccf.group_unique_id(), 1, 0)
        g2.close()


def _on_threads(fn, n):
    """fn(r) on n threads at once (virtual ranks block in each other's collectives)."""
    import threading
    res, errs = [None] * n, []

    def run(r):
        try:
            res[r] = fn(r)
        except BaseException as e:  # noqa: BLE001 (re-raised below)
            errs.append(e)

    th = [threading.Thread(target=run, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a virtual rank did not finish"
    if errs:
        raise errs[0]
    return res


@pytest.mark.parametrize("n", [2, 3])
def test_virtual_ranks_shard_search_and_fine_verify(fccf, pair, n):
    """n virtual ranks on the one GPU (fccf_group_create_local): the K5 search and the
    F evaluations are split into rank blocks and gathered through the same host-side
    exchange code as the RCCL path; every rank's registration (single and pipelined
    batch) equals the unsharded one bit for bit."""
    src, tar, leaf = pair
    with fccf.Ctx(0) as ctx:
        T0, s0 = ctx.register(src, tar, leaf)
    assert s0.fine_evals >= n  # every rank scores a non-empty block
    ctxs = [fccf.Ctx(0) for _ in range(n)]
    try:
        groups = fccf.local_groups(ctxs)
        assert [g.info() for g in groups] == [(n, r) for r in range(n)]

        def work(r):
            T, s = ctxs[r].register(src, tar, leaf)
            Tb, _ = ctxs[r].register_batch([(src, tar)] * 3, leaf)
            return T, s, Tb

        out = _on_threads(work, n)
        for g in groups:
            g.close()
    finally:
        for c in ctxs:
            c.close()
    for T, s, Tb in out:
        np.testing.assert_array_equal(bits(T), bits(T0))
        for Tx in Tb:
            np.testing.assert_array_equal(bits(Tx), bits(T0))
        assert (s.K, s.K_pass, list(s.cand), s.fine_evals) == (s0.K, s0.K_pass, list(s0.cand), s0.fine_evals)


@pytest.mark.parametrize("n,cfg", [(2, "c2"), (3, "c2"), (2, "c3")])
def test_virtual_ranks_shard_the_sort(fccf, n, cfg, monkeypatch):
    """Row D: with FCCF_SHARD_D_MIN=0 every virtual rank sorts only its range of K1's
    std::sort order after the first rounds and the sorted slices are gathered in rank
    order (group.cpp shard_gather_sorted) -- every rank's registration equals the
    unsharded one bit for bit (single and pipelined batch)."""
    c = fccf.CONFIGS[cfg]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    leaf = c["leaf"]
    with fccf.Ctx(0) as ctx:
        T0, s0 = ctx.register(src, tar, leaf)
    monkeypatch.setenv("FCCF_SHARD_D_MIN", "0")
    ctxs = [fccf.Ctx(0) for _ in range(n)]
    try:
        groups = fccf.local_groups(ctxs)

        def work(r):
            T, s = ctxs[r].register(src, tar, leaf)
            Tb, _ = ctxs[r].register_batch([(src, tar)] * 2, leaf)
            return T, s, Tb

        out = _on_threads(work, n)
        for g in groups:
            g.close()
    finally:
        for cx in ctxs:
            cx.close()
    for T, s, Tb in out:
        np.testing.assert_array_equal(bits(T), bits(T0))
        for Tx in Tb:
            np.testing.assert_array_equal(bits(Tx), bits(T0))
        assert (s.K, s.K_pass, list(s.cand), s.vox1, s.vox2) == (s0.K, s0.K_pass, list(s0.cand), s0.vox1, s0.vox2)


def test_virtual_ranks_stage_match(fccf, oracle, pair):
    src, tar, leaf = pair
    run = oracle.Run(src, tar, leaf, oracle.INTROSORT)
    F1, B1 = fccf.planes_from_dump(run.get("planes1")), fccf.bases_from_dump(run.get("bases1", np.int32))
    F2, B2 = fccf.planes_from_dump(run.get("planes2")), fccf.bases_from_dump(run.get("bases2", np.int32))
    ctxs = [fccf.Ctx(0) for _ in range(3)]
    try:
        groups = fccf.local_groups(ctxs)
        out = _on_threads(lambda r: groups[r].match(F1, B1, F2, B2), 3)
        for g in groups:
            g.close()
    finally:
        for c in ctxs:
            c.close()
    for got, kp in out:
        for t in range(3):
            np.testing.assert_array_equal(bits(got[t]), bits(run.get(f"cand{t}").reshape(-1, 4, 4)))


def test_fine_verify_sharded_host_mirror(fccf, pair):
    """shard.fine_verify_sharded (row F for callers that drive the stages): blocks of the
    evaluations scored on the GPU by three rank threads, gathered in rank order, equal
    to one unsharded fccf_stage_fine_verify bit for bit."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "fccf-pcr_amd"))
    sys.path.insert(0, HERE)
    import shard
    import test_shard
    src, tar, leaf = pair
    rng = np.random.default_rng(5)
    T = np.tile(np.eye(4, dtype=np.float32), (7, 1, 1))
    T[:, :3, 3] = rng.normal(0, 0.05, (7, 3)).astype(np.float32)
    with fccf.Ctx(0) as ctx:
        s1, s2 = ctx.downsample(src, leaf), ctx.downsample(tar, leaf)
        want = ctx.fine_verify(s1, s2, T, 0.5)
    ctxs = [fccf.Ctx(0) for _ in range(3)]  # one per rank thread, as one per process
    try:
        gs = test_shard.thread_gathers(3)
        got = _on_threads(lambda r: shard.fine_verify_sharded(ctxs[r], s1, s2, T, 0.5, r, 3, gs[r]), 3)
    finally:
        for c in ctxs:
            c.close()
    for g in got:
        np.testing.assert_array_equal(g.view(np.uint32), np.asarray(want, np.float32).view(np.uint32))


@pytest.mark.parametrize("n,cfg", [(4, "c4"), (8, "c5")])
def test_virtual_ranks_baseline_multi_gpu_configs(fccf, oracle, n, cfg):
    """BASELINE configs[3]/[4] as named: c4 (5M/5M points) over 4 ranks and c5
    (10M/10M) over 8, with the default FCCF_SHARD_D_MIN (2M points), so the K1 sort
    (row D), the correspondence search (K5) and the fine evaluations (F) are all split
    across the ranks and gathered in rank order.  Every virtual rank's single and
    pipelined-batch registration equals the unsharded one and the oracle bit for bit
    (FCCF.cpp:1410-1428, :785-839, :1668-1678), and the stats name the sharded stages."""
    c = fccf.CONFIGS[cfg]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    leaf = c["leaf"]
    run = oracle.Run(src, tar, leaf, oracle.INTROSORT)
    T_orc = run.T.copy()
    del run
    with fccf.Ctx(0) as ctx:
        T0, s0 = ctx.register(src, tar, leaf)
    np.testing.assert_array_equal(bits(T0), bits(T_orc))
    assert s0.shard_ranks == 1 and s0.sharded == 0 and list(s0.xch_bytes) == [0, 0, 0]
    ctxs = [fccf.Ctx(0) for _ in range(n)]
    try:
        groups = fccf.local_groups(ctxs)

        def work(r):
            b0 = groups[r].rx_bytes()
            T, s = ctxs[r].register(src, tar, leaf)
            b1 = groups[r].rx_bytes()
            Tb, sb = ctxs[r].register_batch([(src, tar)] * 2, leaf)
            return T, s, Tb, sb, [y - x for x, y in zip(b0, b1)]

        out = _on_threads(work, n)
        for g in groups:
            g.close()
    finally:
        for cx in ctxs:
            cx.close()
    for T, s, Tb, sb, rx in out:
        # fccf_group_bytes: every channel exchanged; row D alone brings each rank the
        # other ranks' sorted (key, value) slices of both clouds, ~(n-1)/n of 8 B per point
        assert rx[0] > 0 and rx[1] > 0, rx
        assert rx[2] >= 0.5 * 8 * 2 * c["n"] * (n - 1) / n, rx
        # fccf_stats.xch_bytes: the same per-call difference, in the registration's stats
        assert list(s.xch_bytes) == rx, (list(s.xch_bytes), rx)
        for st in sb:
            assert st.xch_bytes[2] >= 2 * rx[2] * 0.9, (list(st.xch_bytes), rx)
        np.testing.assert_array_equal(bits(T), bits(T0))
        for Tx in Tb:
            np.testing.assert_array_equal(bits(Tx), bits(T0))
        assert (s.K, s.K_pass, list(s.cand), s.vox1, s.vox2) == (s0.K, s0.K_pass, list(s0.cand), s0.vox1, s0.vox2)
        for st in [s] + list(sb):
            assert st.shard_ranks == n
            assert sorted(st.as_dict()["sharded"]) == ["faces", "fine", "search", "sort"], st.as_dict()["sharded"]


@pytest.mark.parametrize("n,cfg", [(2, "c2"), (3, "c3")])
def test_virtual_ranks_shard_the_face_stage_debug_exact(fccf, oracle, n, cfg, monkeypatch):
    """Row P (the 1 m face stage split by Morton range of leaves, FCCF.cpp:470-534) with
    row D (FCCF_SHARD_D_MIN=0): every virtual rank's intermediates -- downsampled clouds,
    octree bounds, per-leaf counts / flags / curvatures, planar records, residual clouds
    -- and T equal the oracle bit for bit, on debug contexts."""
    from test_gpu_register import STAGES, as_bits
    c = fccf.CONFIGS[cfg]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    leaf = c["leaf"]
    run = oracle.Run(src, tar, leaf, oracle.INTROSORT)
    monkeypatch.setenv("FCCF_SHARD_D_MIN", "0")
    ctxs = [fccf.Ctx(0, debug=True) for _ in range(n)]
    try:
        groups = fccf.local_groups(ctxs)
        out = _on_threads(lambda r: ctxs[r].register(src, tar, leaf), n)
        dumps = [{name: ctxs[r].debug(name, dt) for name, dt in STAGES} for r in range(n)]
        for g in groups:
            g.close()
    finally:
        for cx in ctxs:
            cx.close()
    for r, (T, s) in enumerate(out):
        assert sorted(s.as_dict()["sharded"]) == ["faces", "fine", "search", "sort"]
        for name, dt in STAGES:
            ref, got = run.get(name, dt), dumps[r][name]
            assert got is not None and got.shape == ref.shape, (r, name)
            assert np.array_equal(as_bits(got), as_bits(ref)), (r, name)
        np.testing.assert_array_equal(bits(T), bits(run.T))


FCCF_E_RCCL = -3


def test_single_rank_group_failure_aborts_and_recovers(fccf, pair):
    """VERDICT r4 item 2 on a real RCCL communicator (one rank: the box has one GPU): a
    registration that fails at the candidate gather aborts the group (ncclCommAbort of
    its three communicators) and returns FCCF_E_RCCL; the aborted group fails the next
    call at once; after fccf_group_destroy the ctx registers bit-exactly again, and a new
    group works."""
    import time
    src, tar, leaf = pair
    with fccf.Ctx(0) as ctx:
        T0, _ = ctx.register(src, tar, leaf)
        g = fccf.Group(ctx, fccf.group_unique_id(), 1, 0)
        try:
            g.inject_failure(1)
            with pytest.raises(fccf.FCCFError) as e:
                ctx.register(src, tar, leaf)
            assert e.value.code == FCCF_E_RCCL and "injected" in str(e.value)
            assert g.aborted()
            a = time.perf_counter()
            with pytest.raises(fccf.FCCFError) as e:
                ctx.register_batch([(src, tar)] * 2, leaf)
            assert e.value.code == FCCF_E_RCCL and time.perf_counter() - a < 5.0
        finally:
            g.close()
        T1, _ = ctx.register(src, tar, leaf)
        with fccf.Group(ctx, fccf.group_unique_id(), 1, 0) as g2:
            T2, _ = ctx.register(src, tar, leaf)
            assert not g2.aborted()
    np.testing.assert_array_equal(bits(T1), bits(T0))
    np.testing.assert_array_equal(bits(T2), bits(T0))


@pytest.mark.parametrize("site,silent,batch", [(1, False, False), (2, False, True), (3, False, True), (1, True, False)])
def test_virtual_rank_failure_ends_every_rank(fccf, pair, monkeypatch, site, silent, batch):
    """three virtual ranks, rank 1 made to fail mid-registration at a
    collective site (1 candidate gather, 2 fine-score gather, 3 sharded sort gather).  A
    failing rank aborts the group, so every rank returns an error promptly; a silent
    failure (a dead peer that aborts nothing) is found by the others at the group's
    time limit (FCCF_GROUP_TIMEOUT_S=3 here).  No rank hangs; the groups are aborted,
    refuse the next call at once, and after they are destroyed every ctx registers
    bit-exactly."""
    import time
    src, tar, leaf = pair
    with fccf.Ctx(0) as ctx:
        T0, _ = ctx.register(src, tar, leaf)
    monkeypatch.setenv("FCCF_GROUP_TIMEOUT_S", "3")
    if site == 3:
        monkeypatch.setenv("FCCF_SHARD_D_MIN", "0")
    n = 3
    ctxs = [fccf.Ctx(0) for _ in range(n)]
    try:
        groups = fccf.local_groups(ctxs)
        groups[1].inject_failure(site, silent)

        def work(r):
            a = time.perf_counter()
            try:
                if batch:
                    ctxs[r].register_batch([(src, tar)] * 3, leaf)
                else:
                    ctxs[r].register(src, tar, leaf)
                return ("ok", time.perf_counter() - a, 0, "")
            except fccf.FCCFError as e:
                return ("err", time.perf_counter() - a, e.code, str(e))

        out = _on_threads(work, n)
        for r, (status, dt, code, msg) in enumerate(out):
            assert status == "err", (r, out)
            assert code == FCCF_E_RCCL, (r, out)
            assert dt < (12.0 if silent else 8.0), (r, out)
        assert all(g.aborted() for g in groups)
        a = time.perf_counter()
        for cx in ctxs:
            with pytest.raises(fccf.FCCFError):
                cx.register(src, tar, leaf)
        assert time.perf_counter() - a < 5.0
        for g in groups:
            g.close()
        for cx in ctxs[:1]:
            T, _ = cx.register(src, tar, leaf)
            np.testing.assert_array_equal(bits(T), bits(T0))
    finally:
        for cx in ctxs:
            cx.close()


@pytest.mark.parametrize("n,cfg,npairs,pp", [(2, "c2", 6, "4"), (3, "c3", 5, "4"), (2, "c2", 7, "5")])
def test_virtual_ranks_pair_batched_stages(fccf, oracle, monkeypatch, n, cfg, npairs, pp):
    """a group no longer forces one pair per cloud stage.  With rows D
    and P sharded (FCCF_SHARD_D_MIN=0) and four or five pairs per stage (FCCF_PAIR_BATCH:
    stage groups of that size and the remainder; five, ten clouds per exchange, is the
    default the driver's sharded leg runs), every cloud of a stage is gathered in one
    exchange, and the next stage's gathers wait for all of this stage's phase-B1
    collectives (one issue order per rank).  Every rank's T equals the oracle's bit for
    bit."""
    c = fccf.CONFIGS[cfg]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    leaf = c["leaf"]
    rng = np.random.default_rng(17)
    pairs = [(src, tar)]
    for k in range(npairs - 1):
        jit = rng.normal(0, 0.002, src.shape).astype(np.float32)
        pairs.append(((src + jit).astype(np.float32), tar[: len(tar) - 1000 * (k + 1)]))
    refs = [oracle.Run(s, t, leaf, oracle.INTROSORT).T.copy() for s, t in pairs]
    monkeypatch.setenv("FCCF_SHARD_D_MIN", "0")
    monkeypatch.setenv("FCCF_PAIR_BATCH", pp)
    ctxs = [fccf.Ctx(0) for _ in range(n)]
    try:
        groups = fccf.local_groups(ctxs)
        out = _on_threads(lambda r: ctxs[r].register_batch(pairs, leaf), n)
        for g in groups:
            g.close()
    finally:
        for cx in ctxs:
            cx.close()
    for Tb, sb in out:
        for i, (T, ref) in enumerate(zip(Tb, refs)):
            np.testing.assert_array_equal(bits(T), bits(ref), err_msg=f"pair {i}")
        for st in sb:
            assert st.shard_ranks == n
            assert sorted(st.as_dict()["sharded"]) == ["faces", "fine", "search", "sort"], st.as_dict()["sharded"]
