"""End-to-end parity: libfccf (GPU) vs the CPU oracle on identical inputs.

Every intermediate the reference computes is compared, in pipeline order, so a
failure names the first stage that diverges.  Bar: bit-exact for every stage
(integer/index work exactly, float stages as identical bit patterns), which
implies the north-star tolerance (1e-5 rad / 1e-4 m) on the final transform."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# (name, dtype) in pipeline order; names are shared by orc_get and fccf_debug_get.
STAGES = [("ds_src", np.float32), ("ds_tar", np.float32), ("ds1", np.float32), ("ds2", np.float32),
          ("centroid1", np.float32), ("centroid2", np.float32), ("oct1", np.float64), ("oct2", np.float64),
          ("vstat1", np.int32), ("vstat2", np.int32), ("vcurv1", np.float32), ("vcurv2", np.float32),
          ("vox1", np.float32), ("vox2", np.float32), ("res1", np.float32), ("res2", np.float32),
          ("groups1", np.float32), ("groups2", np.float32), ("galloc1", np.int32), ("galloc2", np.int32),
          ("planes1", np.float32), ("planes2", np.float32), ("theta1", np.float64), ("theta2", np.float64),
          ("bases1", np.int32), ("bases2", np.int32),
          ("cand0", np.float32), ("cand1", np.float32), ("cand2", np.float32),
          ("fine0", np.float32), ("fine1", np.float32), ("fine2", np.float32),
          ("qv0", np.float32), ("qv1", np.float32), ("qv2", np.float32),
          ("fv0", np.float32), ("fv1", np.float32), ("fv2", np.float32),
          ("high", np.float32), ("T", np.float32)]


def as_bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint64) if a.dtype == np.float64 else (a.view(np.uint32) if a.dtype == np.float32 else a)


def compare_all(ctx, run):
    for name, dt in STAGES:
        ref = run.get(name, dt)
        got = ctx.debug(name, dt)
        assert ref is not None, name
        assert got is not None, name
        assert got.shape == ref.shape, f"{name}: shape {got.shape} vs oracle {ref.shape}"
        if not np.array_equal(as_bits(got), as_bits(ref)):
            bad = np.flatnonzero(as_bits(got) != as_bits(ref))
            raise AssertionError(f"first divergent stage {name}: {bad.size} of {ref.size} differ, "
                                 f"first at {bad[0]}: got {got.ravel()[bad[0]]!r} oracle {ref.ravel()[bad[0]]!r}")
    c_ref = run.get("counts", np.int64)
    c_got = ctx.debug("counts", np.int64)
    np.testing.assert_array_equal(c_got[:-1], c_ref[:-1])  # last = overflow flag (oracle: driver passes only)


def _nearest_rotation(M):
    u, _, vt = np.linalg.svd(M[:3, :3].astype(np.float64))
    return u @ vt


def rot_err_rad(A, B):
    """Angle of the relative rotation.  The reference's rotations are not exactly
    orthonormal (averaged normals are never renormalised), so each
    is first projected to its nearest rotation: identical matrices give 0."""
    R = _nearest_rotation(A).T @ _nearest_rotation(B)
    return float(np.arccos(np.clip((np.trace(R) - 1) / 2, -1, 1)))


@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "c5"])
def test_register_bit_exact(ctx, oracle, fccf, cfg):
    c = fccf.CONFIGS[cfg]
    src, tar, T_gt = fccf.synth_pair(c["n"], c["room"])
    run = oracle.Run(src, tar, c["leaf"], oracle.INTROSORT)
    T, st = ctx.register(src, tar, c["leaf"])
    compare_all(ctx, run)
    np.testing.assert_array_equal(T.view(np.uint32), run.T.view(np.uint32))
    # north-star tolerance, stated explicitly (implied by the bitwise check above)
    assert rot_err_rad(T, run.T) <= 1e-5 and np.linalg.norm(T[:3, 3] - run.T[:3, 3]) <= 1e-4
    # and the registration is actually right (published accuracy band, Tables II/III)
    assert np.degrees(rot_err_rad(T, T_gt)) < 1.0
    assert np.linalg.norm(T[:3, 3] - T_gt[:3, 3]) < 0.3
    assert st.K > 0 and st.K_pass > 0


def test_register_device_resident_matches_host_path(ctx, fccf):
    src, tar, _ = fccf.synth_pair(60_000)
    T1, _ = ctx.register(src, tar, 0.1)
    ds, dt = ctx.upload(src), ctx.upload(tar)
    try:
        T2, _ = ctx.register_device(ds, src.shape[0], dt, tar.shape[0], 0.1)
    finally:
        ctx.free(ds)
        ctx.free(dt)
    np.testing.assert_array_equal(T1.view(np.uint32), T2.view(np.uint32))


def test_device_inputs_read_in_place_across_buffers(ctx, oracle, fccf):
    """Device-resident clouds are read in place: the cached cloud-stage graph is
    replayed with pass 1's entry node patched to each call's pointers and counts
    (CachedGraph patch, VGEntry).  Alternating buffers, counts that change under the
    same capacity, and a 4-byte-misaligned input (the kernels' scalar-load path) must
    each equal the oracle bitwise."""
    src, tar, _ = fccf.synth_pair(60_000)
    rng = np.random.default_rng(11)
    src2 = (src + rng.normal(0, 0.002, src.shape)).astype(np.float32)
    runs = [(src, tar), (src2, tar), (src, tar[:59_000]), (tar, src)]
    pad = np.zeros(3 * (src2.shape[0] + 1), np.float32)
    pad[1:1 + src2.size] = src2.reshape(-1)  # src2 at byte offset 4
    bufs = {}
    try:
        for i, (s, t) in enumerate(runs):
            ds, dt = ctx.upload(s), ctx.upload(t)
            bufs[i] = (ds, dt)
            T, _ = ctx.register_device(ds, s.shape[0], dt, t.shape[0], 0.1)
            np.testing.assert_array_equal(T.view(np.uint32), oracle.Run(s, t, 0.1).T.view(np.uint32))
        dp = ctx.upload(pad.reshape(-1, 3))
        bufs["pad"] = (dp,)
        T, _ = ctx.register_device(dp + 4, src2.shape[0], bufs[1][1], tar.shape[0], 0.1)
        np.testing.assert_array_equal(T.view(np.uint32), oracle.Run(src2, tar, 0.1).T.view(np.uint32))
        T, _ = ctx.register_device(bufs[0][0], src.shape[0], bufs[0][1], tar.shape[0], 0.1)  # back to the first
        np.testing.assert_array_equal(T.view(np.uint32), oracle.Run(src, tar, 0.1).T.view(np.uint32))
    finally:
        for b in bufs.values():
            for d in b:
                ctx.free(d)


def test_register_repeatable(ctx, fccf):
    src, tar, _ = fccf.synth_pair(50_000)
    a, _ = ctx.register(src, tar, 0.1)
    b, _ = ctx.register(src, tar, 0.1)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


def test_identical_clouds(ctx, oracle, fccf):
    x = fccf.synth_scene(80_000, seed=9)
    run = oracle.Run(x, x, 0.1)
    T, _ = ctx.register(x, x, 0.1)
    compare_all(ctx, run)
    assert rot_err_rad(T, np.eye(4, dtype=np.float32)) < 1e-3


def test_other_room(ctx, oracle, fccf):
    src, tar, _ = fccf.synth_pair(150_000, (30.0, 24.0, 6.0))
    run = oracle.Run(src, tar, 0.08)
    ctx.register(src, tar, 0.08)
    compare_all(ctx, run)


def test_graph_replay_with_new_data_and_sizes(ctx, oracle, fccf):
    """The device stages run as captured hipGraphs keyed by workspace layout: a
    second call with different points of the same size replays the graph, a call
    with a different size re-captures.  Each must match the oracle bitwise."""
    src, tar, _ = fccf.synth_pair(80_000)
    rng = np.random.default_rng(3)
    src2 = (src + rng.normal(0, 0.002, src.shape)).astype(np.float32)  # same n: replay
    for s, t in ((src, tar), (src2, tar), (src2[:70_001], tar)):  # last: new capacity, re-capture
        run = oracle.Run(s, t, 0.1, oracle.INTROSORT)
        T, _ = ctx.register(s, t, 0.1)
        compare_all(ctx, run)
        np.testing.assert_array_equal(T.view(np.uint32), run.T.view(np.uint32))


def test_graph_replay_layout_check(fccf, oracle):
    """Every replay of the cached cloud-stage graph compares the patched entry kernel's
    layout arguments (everything but the inputs) with the ones it was captured with
    (CachedGraph).  A replay deliberately patched with a wrong
    workspace pointer (fccf_debug_graph_mismatch) fails with FCCF_E_INTERNAL before
    anything is launched, and the same ctx then replays correctly, bit-exact."""
    src, tar, _ = fccf.synth_pair(60_000)
    ref = oracle.Run(src, tar, 0.1, oracle.INTROSORT).T
    FCCF_E_INTERNAL = -6
    c = fccf.Ctx(0)
    try:
        T0, _ = c.register(src, tar, 0.1)  # captures
        T1, st1 = c.register(src, tar, 0.1)  # replays
        assert st1.graph_captures == 0
        c.graph_mismatch()
        with pytest.raises(fccf.FCCFError) as e:
            c.register(src, tar, 0.1)
        assert e.value.code == FCCF_E_INTERNAL and "graph replay" in str(e.value)
        T2, st2 = c.register(src, tar, 0.1)  # the hook is consumed; the graph is intact
        assert st2.graph_captures == 0
        for T in (T0, T1, T2):
            np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32))
    finally:
        c.close()


def test_probe_path_is_exact_and_counts_launches(ctx, oracle, fccf):
    """With a kernel probe on, the device stages launch eagerly (no graphs) and the
    probed launches go through hipExtLaunchKernelGGL; results must not change."""
    src, tar, _ = fccf.synth_pair(80_000)
    run = oracle.Run(src, tar, 0.1, oracle.INTROSORT)
    for k in ("k_rs_scatter", "k_oct_sim", "k_xs_chain"):
        ctx.set_probe(k)
        T, _ = ctx.register(src, tar, 0.1)
        ms, n, b = ctx.probe_read()
        ctx.set_probe(None)
        np.testing.assert_array_equal(T.view(np.uint32), run.T.view(np.uint32))
        assert n > 0 and ms > 0 and b > 0, (k, ms, n, b)
    compare_all(ctx, run)


def test_batch_pipeline_equals_single_registrations(ctx, oracle, fccf):
    """fccf_register_batch overlaps pair i+1's cloud stage with pair i's later
    stages (double-buffered cloud workspaces); every result must equal the
    single-pair registration and the oracle, for host and device inputs."""
    base_src, base_tar, _ = fccf.synth_pair(70_000)
    rng = np.random.default_rng(9)
    pairs = [(base_src, base_tar)]
    for k in range(3):
        jit = rng.normal(0, 0.002, base_src.shape).astype(np.float32)
        pairs.append(((base_src + jit).astype(np.float32), base_tar[: 60_000 + 5000 * k]))
    Tb, stb = ctx.register_batch(pairs, 0.1)
    for (s, t), T in zip(pairs, Tb):
        ref = oracle.Run(s, t, 0.1, oracle.INTROSORT).T
        np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32))
    assert all(st.K > 0 for st in stb)
    dev = [(ctx.upload(s), ctx.upload(t)) for s, t in pairs]
    try:
        Td, _ = ctx.register_batch([((ds, s.shape[0]), (dt, t.shape[0])) for (ds, dt), (s, t) in zip(dev, pairs)], 0.1,
                                   on_device=True)
    finally:
        for ds, dt in dev:
            ctx.free(ds)
            ctx.free(dt)
    np.testing.assert_array_equal(Td.view(np.uint32), Tb.view(np.uint32))


def test_deep_octree_tail_sort(ctx, oracle, fccf):
    """A clump of points ~1.5 km away makes both octrees (1 m face voxels, 0.5 m
    fine verify) deeper than the four fast radix passes cover (3 bits per level),
    so the single-workgroup tail sort (k_rs_tail) finishes them; bitwise parity."""
    src, tar, _ = fccf.synth_pair(60_000)
    rng = np.random.default_rng(4)
    far = (np.array([1500.0, 40.0, 2.0]) + rng.uniform(0, 0.9, size=(12, 3))).astype(np.float32)
    src2 = np.concatenate([src, far])
    tar2 = np.concatenate([far + np.float32(0.01), tar])
    run = oracle.Run(src2, tar2, 0.1, oracle.INTROSORT)
    assert run.get("oct1", np.float64)[3] > 10 and run.get("oct2", np.float64)[3] > 10  # depth
    T, _ = ctx.register(src2, tar2, 0.1)
    compare_all(ctx, run)
    np.testing.assert_array_equal(T.view(np.uint32), run.T.view(np.uint32))


def test_host_radius_search_path_matches(ctx, oracle, fccf, monkeypatch):
    """transform_cluster's neighbour sets come from the device bitmask rows
    (k_cluster_bits) by default; FCCF_CLUSTER_BITS=0 selects the host radius search.
    Both must reproduce the oracle bit for bit."""
    src, tar, _ = fccf.synth_pair(120_000)
    run = oracle.Run(src, tar, 0.1, oracle.INTROSORT)
    monkeypatch.setenv("FCCF_CLUSTER_BITS", "0")
    T0, _ = ctx.register(src, tar, 0.1)
    compare_all(ctx, run)
    monkeypatch.delenv("FCCF_CLUSTER_BITS")
    T1, _ = ctx.register(src, tar, 0.1)
    compare_all(ctx, run)
    np.testing.assert_array_equal(T0.view(np.uint32), T1.view(np.uint32))


def test_nonfinite_points_through_overflow_passthrough(ctx, oracle, fccf):
    """A far outlier makes the first VoxelGrid pass overflow its int32 leaf index,
    so PCL passes the cloud through unfiltered, NaN points included; the driver's
    removeNaNFromPointCloud (FCCF.cpp:1374-1375) then has real work (the rare path
    of k_finite_fix).  Bitwise parity with the oracle at every stage."""
    src, tar, _ = fccf.synth_pair(60_000)
    src = src.copy()
    src[::997] = np.nan
    src[5::1009, 2] = np.inf
    far = np.array([[2500.0, -2500.0, 2500.0]], np.float32)
    src2 = np.concatenate([src, far])
    run = oracle.Run(src2, tar, 0.1, oracle.INTROSORT)
    T, _ = ctx.register(src2, tar, 0.1)
    compare_all(ctx, run)
    np.testing.assert_array_equal(T.view(np.uint32), run.T.view(np.uint32))


def test_stats_time_the_host_input_copy(ctx, fccf):
    """fccf_stats.ms[h2d] is the staged copy of host inputs (0 for device-resident clouds)."""
    src, tar, _ = fccf.synth_pair(200_000)
    _, st = ctx.register(src, tar, 0.1)
    d = st.as_dict()["ms"]
    assert d["h2d"] > 0 and d["voxelfit"] > 0 and d["select"] > 0
    ds, dt = ctx.upload(src), ctx.upload(tar)
    try:
        _, st2 = ctx.register_device(ds, len(src), dt, len(tar), 0.1)
    finally:
        ctx.free(ds)
        ctx.free(dt)
    assert st2.as_dict()["ms"]["h2d"] == 0.0


@pytest.mark.parametrize("bit", [0x100, 0x200, 0x400, 0x1000])
def test_sort_invariant_flag_fails_registration(ctx, oracle, fccf, bit):
    """A K1 sort invariant flag (IS_FAULT_*, raised through the injection hook at its
    kernel) makes every path fail with FCCF_E_INTERNAL instead of returning a
    transform computed from a possibly wrong VoxelGrid order (FCCF.cpp:1668-1678);
    with the hook off again the same ctx registers bit-exactly."""
    src, tar, _ = fccf.synth_pair(100_000)
    FCCF_E_INTERNAL = -6
    ctx.inject_sort_fault(bit)
    try:
        with pytest.raises(fccf.FCCFError) as e:
            ctx.register(src, tar, 0.1)
        assert e.value.code == FCCF_E_INTERNAL and "sort invariant" in str(e.value)
        with pytest.raises(fccf.FCCFError) as e:
            ctx.register_batch([(src, tar)] * 3, 0.1)
        assert e.value.code == FCCF_E_INTERNAL
        with pytest.raises(fccf.FCCFError) as e:
            ctx.downsample(src, 0.1)
        assert e.value.code == FCCF_E_INTERNAL
    finally:
        ctx.inject_sort_fault(0)
    T, _ = ctx.register(src, tar, 0.1)
    np.testing.assert_array_equal(T.view(np.uint32), oracle.Run(src, tar, 0.1, oracle.INTROSORT).T.view(np.uint32))


def test_outdoor_extent_face_sort_stays_on_fast_passes(ctx, oracle, fccf):
    """A scene ~120 m across (the first-point-anchored 1 m octree grows to depth 9:
    28-bit face codes, about 500 x face_voxel_size of root cell).  The cloud stage
    launches three face-code radix passes until a scene needs a fourth digit: the first
    registration sorts it in the single-workgroup tail (bitwise parity), flags the
    cloud (FACE_DEEP) and the ctx launches four device-wide passes from then on, so the
    face stage's device span stays well under a millisecond (the tail path over the
    whole cloud takes several)."""
    src, tar, _ = fccf.synth_pair(400_000, (120.0, 90.0, 8.0))
    run = oracle.Run(src, tar, 0.1, oracle.INTROSORT)
    assert run.get("oct1", np.float64)[3] == 9 and run.get("oct2", np.float64)[3] == 9  # depth
    T, st = ctx.register(src, tar, 0.1)
    compare_all(ctx, run)
    np.testing.assert_array_equal(T.view(np.uint32), run.T.view(np.uint32))
    spans = [ctx.register(src, tar, 0.1)[1].dev_ms[2] for _ in range(3)]
    print(f"face stage span at 400 m extent: {min(spans):.3f} ms")
    assert min(spans) < 1.0


def test_optimistic_driver_pass_redo(ctx, oracle, fccf):
    """The pipeline's driver pass (FCCF.cpp:1377-1387 over main's output) runs without
    the fallback sort and segmentation launches (VG_OPTIMISTIC); a pass whose input is
    not in leaf order outputs nothing and sets VG_REDO, and the host redoes the stage
    with the exact second pass.  Forced through the test hook (VG_FORCE_REDO): T stays
    bit-exact against the oracle, and the stats count the redo, single and batched."""
    src, tar, _ = fccf.synth_pair(100_000)
    ref = oracle.Run(src, tar, 0.1, oracle.INTROSORT).T
    T0, st0 = ctx.register(src, tar, 0.1)
    assert st0.stage_redos == 0
    ctx.inject_sort_fault(0x10000)
    try:
        T1, st1 = ctx.register(src, tar, 0.1)
        Tb, stb = ctx.register_batch([(src, tar)] * 3, 0.1)
    finally:
        ctx.inject_sort_fault(0)
    assert st1.stage_redos == 1 and all(x.stage_redos == 1 for x in stb)
    for T in (T0, T1, *Tb):
        np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32))
    T2, st2 = ctx.register(src, tar, 0.1)  # the cached graphs are intact afterwards
    assert st2.stage_redos == 0
    np.testing.assert_array_equal(T2.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("pp", ["2", "4"])
def test_redo_raised_by_a_later_pair_of_the_group(fccf, oracle, monkeypatch, pp):
    """A stage group's later pair alone finds the driver pass's input out of leaf order
    (test hook 0x40000: clouds >= 2 of the stage only), after the group's first pair has
    already handed the next group's cloud stage to the helper thread.  The redo joins the
    helper first, so its eager launches never land in a capture; every
    T stays bit-exact, and the pairs from the flagged one on count the redo."""
    monkeypatch.setenv("FCCF_PAIR_BATCH", pp)
    base_src, base_tar, _ = fccf.synth_pair(70_000)
    rng = np.random.default_rng(31)
    pairs = []
    for k in range(6):
        jit = rng.normal(0, 0.002, base_src.shape).astype(np.float32)
        pairs.append(((base_src + jit).astype(np.float32)[: 70_000 - 3000 * k], base_tar))
    refs = [oracle.Run(s, t, 0.1, oracle.INTROSORT).T for s, t in pairs]
    c = fccf.Ctx(0)
    try:
        c.inject_sort_fault(0x40000)
        try:
            Tb, sb = c.register_batch(pairs, 0.1)
        finally:
            c.inject_sort_fault(0)
        for T, ref in zip(Tb, refs):
            np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32))
        # pair j >= 1 of each group found the flag (j = 1) or ran after the redo; the
        # group's first pair had finished its phase B1 before it, with a correct result
        got = [int(x.stage_redos) for x in sb]
        assert got == [1 if i % int(pp) else 0 for i in range(len(pairs))], got
        Tb2, sb2 = c.register_batch(pairs, 0.1)  # hook off: cached graphs intact, no redo
        for T, ref in zip(Tb2, refs):
            np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32))
        assert all(x.stage_redos == 0 for x in sb2)
    finally:
        c.close()


@pytest.mark.parametrize("pp", ["1", "4"])
def test_batch_fine_overflow_registers_the_pair_again(fccf, oracle, monkeypatch, pp):
    """in a pipelined batch, fine verification past the LDS form's
    capacity (FV_ERR_LDS, forced with FCCF_FINE_LDS_CAP=16) cannot be rerun from the stage
    arena, which a later stage group may already be recycling; the pair is registered
    again after the batch's last pair instead (sorted form, sticky).  Every T bit-exact
    against the oracle, the overflowing pairs count fine_reruns = 1, and the pairs whose
    fine launch came after the first overflow was seen use the sorted form from the start."""
    monkeypatch.setenv("FCCF_PAIR_BATCH", pp)
    monkeypatch.setenv("FCCF_FINE_LDS_CAP", "16")
    base_src, base_tar, _ = fccf.synth_pair(80_000)
    rng = np.random.default_rng(41)
    pairs = []
    for k in range(6):
        jit = rng.normal(0, 0.002, base_src.shape).astype(np.float32)
        pairs.append(((base_src + jit).astype(np.float32), base_tar[: 80_000 - 4000 * k]))
    refs = [oracle.Run(s, t, 0.1, oracle.INTROSORT).T for s, t in pairs]
    c = fccf.Ctx(0)
    try:
        Tb, sb = c.register_batch(pairs, 0.1)
        for i, (T, ref) in enumerate(zip(Tb, refs)):
            np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32), err_msg=f"pair {i}")
        # which pairs launch in the LDS form before the first overflow is seen depends on
        # timing when two phase-B chains run (pipeline.cpp): at least one pair reruns,
        # and the last pair's phase B1 follows an overflow seen by its own chain
        reruns = [int(x.fine_reruns) for x in sb]
        assert max(reruns) == 1 and set(reruns) <= {0, 1}, reruns
        assert reruns[-1] == 0, reruns
        Tb2, sb2 = c.register_batch(pairs, 0.1)  # sorted form from the start now
        for T, ref in zip(Tb2, refs):
            np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32))
        assert all(x.fine_reruns == 0 for x in sb2)
    finally:
        c.close()


def test_pair_batched_stages_equal_single_registrations(ctx, oracle, fccf, monkeypatch):
    """fccf_register_batch runs the clouds of two pairs in the same launches (stage
    groups of two pairs, the last one single for an odd count; pipeline.cpp
    clouds_enqueue_group).  Pairs of different sizes within a group, single
    registrations between batches (the one-pair and two-pair stages lay the workspace
    out differently, so their cached graphs must never be mixed), and the other stage
    forms (FCCF_PAIR_BATCH=1, 3, 4, 5: up to ten clouds per launch) must all give the
    oracle's T bit for bit."""
    base_src, base_tar, _ = fccf.synth_pair(90_000)

    def make_pairs(seed):  # the same sizes (so the same cached stage graphs), new points
        rng = np.random.default_rng(seed)
        out = []
        for k in range(5):
            jit = rng.normal(0, 0.002, base_src.shape).astype(np.float32)
            out.append(((base_src + jit).astype(np.float32)[: 90_000 - 7000 * k], base_tar[: 60_000 + 6000 * k]))
        return out

    for rep in range(2):
        # a replayed two-pair graph after one-pair captures (rep 1) must patch its own
        # entry arguments: new points of the same sizes show stale ones as a wrong T
        pairs = make_pairs(21 + rep)
        refs = [oracle.Run(s, t, 0.1, oracle.INTROSORT).T for s, t in pairs]
        Tb, sb = ctx.register_batch(pairs, 0.1)
        for T, ref in zip(Tb, refs):
            np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32))
        for x in sb:  # every pair's device spans come from its own stage's stamps
            ms = x.as_dict()["ms"]
            assert 0.0 < ms["downsample"] < 1000.0 and 0.0 < ms["voxelfit"] < 1000.0, ms
        for (s, t), ref in list(zip(pairs, refs))[:2]:  # one-pair stages between the batches
            T, _ = ctx.register(s, t, 0.1)
            np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32))
    Tb, _ = ctx.register_batch(pairs[:2], 0.1)  # one group of two
    for T, ref in zip(Tb, refs[:2]):
        np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32))
    for pp in ("1", "3", "4", "5"):  # one pair per stage, and three to five (up to 10 clouds per launch)
        monkeypatch.setenv("FCCF_PAIR_BATCH", pp)
        Tb1, sb1 = ctx.register_batch(pairs, 0.1)
        for T, ref in zip(Tb1, refs):
            np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32), err_msg=f"{pp} pairs per stage")
        for x in sb1:
            ms = x.as_dict()["ms"]
            assert 0.0 < ms["downsample"] < 1000.0 and 0.0 < ms["voxelfit"] < 1000.0, (pp, ms)


def test_fine_verify_leaf_forms_agree(fccf, oracle, monkeypatch):
    """fine_verify (FCCF.cpp:785-839) in its two leaf forms: per evaluation in LDS
    (default: the tile entries merged, the nonzero terms placed in code order by rank and
    summed by one workgroup) and sorted
    device-wide (FCCF_FINE_SORTED=1, the fallback).  Scores bit-equal between the forms
    through the stage export; a capacity below the scene's leaf count (FCCF_FINE_LDS_CAP)
    makes the pipeline rerun the batch in the sorted form (fine_reruns = 1) with T still
    bit-exact, and the ctx keeps the sorted form afterwards."""
    src, tar, _ = fccf.synth_pair(100_000)
    ref = oracle.Run(src, tar, 0.1, oracle.INTROSORT)
    c = fccf.Ctx(0, debug=True)
    try:
        T, st = c.register(src, tar, 0.1)
        np.testing.assert_array_equal(T.view(np.uint32), ref.T.view(np.uint32))
        assert st.fine_reruns == 0
        s1, s2 = c.debug("res1").reshape(-1, 3), c.debug("res2").reshape(-1, 3)
        Ts = np.stack([np.eye(4, dtype=np.float32)] + [fv.reshape(-1, 18)[:, :16].reshape(-1, 4, 4)[0]
                                                       for fv in (c.debug("fv0"), c.debug("fv2")) if fv.size])
        a = c.fine_verify(s1, s2, Ts)
        monkeypatch.setenv("FCCF_FINE_SORTED", "1")
        b = c.fine_verify(s1, s2, Ts)
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
        monkeypatch.delenv("FCCF_FINE_SORTED")
        monkeypatch.setenv("FCCF_FINE_LDS_CAP", "16")
        d = c.fine_verify(s1, s2, Ts)  # the export falls back by itself
        np.testing.assert_array_equal(a.view(np.uint32), d.view(np.uint32))
        T2, st2 = c.register(src, tar, 0.1)
        np.testing.assert_array_equal(T2.view(np.uint32), ref.T.view(np.uint32))
        assert st2.fine_reruns == 1
        monkeypatch.delenv("FCCF_FINE_LDS_CAP")
        T3, st3 = c.register(src, tar, 0.1)  # sticky: sorted from the start, no rerun
        np.testing.assert_array_equal(T3.view(np.uint32), ref.T.view(np.uint32))
        assert st3.fine_reruns == 0
    finally:
        c.close()


def test_mailbox_flags_and_event_waits_agree(ctx, oracle, fccf, monkeypatch):
    """Phase B wakes on pinned mailbox flags that the stages' last kernels set after a
    system-scope fence (k_mail_done, k_fv_mail_err; ctx.h mail_wait); FCCF_SPIN_US=0 takes
    the event waits instead.  Both must read complete mailboxes: T bit-exact against the
    oracle, single and batched, and the fine device span (from the mailbox stamps) set."""
    src, tar, _ = fccf.synth_pair(80_000)
    ref = oracle.Run(src, tar, 0.1, oracle.INTROSORT).T
    for spin in ("", "0", "1"):  # default bound, event waits only, a 1 us bound (mostly events)
        if spin:
            monkeypatch.setenv("FCCF_SPIN_US", spin)
        else:
            monkeypatch.delenv("FCCF_SPIN_US", raising=False)
        for _ in range(2):
            T, st = ctx.register(src, tar, 0.1)
            np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32), err_msg=f"FCCF_SPIN_US={spin!r}")
            assert 0.0 < st.dev_ms[3] < 1000.0, (spin, list(st.dev_ms))
        Tb, sb = ctx.register_batch([(src, tar)] * 5, 0.1)
        for T, x in zip(Tb, sb):
            np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32), err_msg=f"batch, FCCF_SPIN_US={spin!r}")
            assert 0.0 < x.dev_ms[3] < 1000.0, (spin, list(x.dev_ms))


def test_event_waits_while_other_chains_capture(oracle, fccf, monkeypatch):
    """with FCCF_SPIN_US=0 phase B2 waits on the fine-verification event
    instead of the mailbox flag, and that event is recorded on a stream the other chains
    capture their fine graphs on whenever a pair's sizes change the graph key.  Pairs of
    different sizes in a multi-chain batch (a non-debug ctx: the chains run) make those
    captures overlap the event waits; every T must equal the oracle's."""
    monkeypatch.setenv("FCCF_SPIN_US", "0")
    base_src, base_tar, _ = fccf.synth_pair(40_000)
    rng = np.random.default_rng(57)
    pairs, refs = [], []
    for k in range(12):
        jit = rng.normal(0, 0.003, base_src.shape).astype(np.float32)
        s, t = (base_src + jit).astype(np.float32)[: 40_000 - 700 * k], base_tar[: 33_000 + 600 * k]
        pairs.append((s, t))
        refs.append(oracle.Run(s, t, 0.1, oracle.INTROSORT).T)
    with fccf.Ctx(0) as c:
        for _ in range(2):
            Tb, sb = c.register_batch(pairs, 0.1)
            for i, (T, ref) in enumerate(zip(Tb, refs)):
                np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32), err_msg=f"pair {i}")


@pytest.mark.parametrize("drain4", ["1", "0"])
@pytest.mark.parametrize("pp,ns", [("4", (11, 12)), ("5", (13, 14, 15))])
def test_batch_drain_with_a_chain_per_pair(oracle, fccf, monkeypatch, drain4, pp, ns):
    """A batch whose last stage group holds three to five pairs drains with a phase-B
    chain per pair (pipeline.cpp; FCCF_DRAIN4=0: two chains throughout).  Its third to
    fifth pairs go to the drain's own workers, on the idle cloud-stage streams, and reuse
    the slots of pairs two groups back, whose phase B2 ran on the other workers.  Every
    T equals the oracle's, for groups 4 + 4 + 3 and 4 + 4 + 4 at four pairs per stage,
    and 5 + 5 + 3, 5 + 5 + 4 and 5 + 5 + 5 at five (the default).  Distinct pairs, so a
    result read from another pair's slot, or a pair left out, would show.  A ctx of its
    own: the session's debug ctx runs batches on one chain."""
    monkeypatch.setenv("FCCF_DRAIN4", drain4)
    monkeypatch.setenv("FCCF_PAIR_BATCH", pp)
    base_src, base_tar, _ = fccf.synth_pair(40_000)
    rng = np.random.default_rng(31)
    pairs, refs = [], []
    for k in range(max(ns)):
        jit = rng.normal(0, 0.003, base_src.shape).astype(np.float32)
        s, t = (base_src + jit).astype(np.float32), base_tar[: 34_000 + 500 * k]
        pairs.append((s, t))
        refs.append(oracle.Run(s, t, 0.1, oracle.INTROSORT).T)
    with fccf.Ctx(0) as c:
        for n in ns:
            Tb, sb = c.register_batch(pairs[:n], 0.1)
            for i, (T, ref) in enumerate(zip(Tb, refs)):
                np.testing.assert_array_equal(T.view(np.uint32), ref.view(np.uint32), err_msg=f"n={n} pair {i}")
            assert all(x.K > 0 for x in sb)
