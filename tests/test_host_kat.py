"""Known-answer tests of the host-only stages, derived by reading FCCF.cpp.

The expected outputs here are worked out from the reference source by hand (the
numbers in each docstring), not taken from the oracle, so they pin the two restatements
independently: the oracle (oracle/fccf_oracle.cpp, `oracle_py.stage_*`) and libfccf's
host stages (`fccf_stage_grow`, `fccf_stage_cluster`, `fccf_stage_fuse` through the
C-ABI; host code, so these CPU tests call them without a device ctx).  Every test names
the quirk of SURVEY.md App. B it pins and fails if that quirk is "fixed":

  Q5   a NaN roughness pushes no type, so type_index runs short of the bases (:454-461)
  Q8   range_face's exchange sort reorders ties (:409-427)
  Q9   at most 16 planes: the break on currentSelectNum > 15 (:670); a group absorbed in
       stage 2 keeps its place in range_face but is not selected (:657)
  Q12  transform_cluster: the last candidate never seeds (:1084), allocated neighbours
       are added again (:1093-1114), the angle test uses the rotated x-axis only
       (:1105-1110), <= cluster_number_threshold candidates pass through and none gives
       the identity (:1043-1063)
  Q13  the cluster selection: range_cluster's tie order (:1020-1038), a short cluster
       decrements clusternum and is skipped (:1213-1222), `stop` ends it (:1225),
       cluster_num + 1 clusters at most (:1208)
  Q15  fusion: score sums over every type before normalising (:1539-1540, :1558), an
       empty type yields a zero score (:1551-1595), the 0.8 cut (:1601)

The "device" parametrisation (-m gpu) runs the device forms (K4 growth, f3 clustering)
on the same inputs through a ctx.
"""
import math

import numpy as np
import pytest

import oracle_py as O


_dev = {}


def _impls(fccf):
    impls = {
        "oracle": (O.stage_grow, O.stage_cluster, O.stage_fuse),
        "libfccf": (lambda v, s: fccf.stage_grow(v, s), lambda c, k: fccf.stage_cluster(c, k),
                    lambda l, a=4: fccf.stage_fuse(l, a)),
    }
    if "device" in _dev:
        c = _dev["device"]
        impls["device"] = (c.grow, c.cluster, c.fuse)
    return impls


@pytest.fixture
def device_ctx(fccf, request):
    """The device forms (K4 growth, f3 clustering) on a ctx of their own, for the
    'device' parametrisation (GPU only)."""
    if request.node.callspec.params.get("impl") != "device":
        yield None
        return
    c = fccf.Ctx(0)
    c.set_grow_device(True)
    c.set_cluster_device(True)
    _dev["device"] = c
    yield c
    _dev.pop("device")
    c.close()


IMPLS = ["oracle", "libfccf", pytest.param("device", marks=pytest.mark.gpu)]
f32 = np.float32


def vox(items):
    """Voxel records from (centre, normal, point count)."""
    v = np.zeros(len(items), O.VOXEL_DTYPE)
    for i, (c, n, cnt) in enumerate(items):
        v[i]["c"], v[i]["n"], v[i]["count"], v[i]["curvature"] = c, n, cnt, 0.01
    return v


def summary(members):
    """A group's facenode summary as FCCF.cpp:570-586 recomputes it: float sums over the
    members in voxelgrothnode order, weighted by the point count, then divided."""
    s = f32(0)
    c = [f32(0)] * 3
    n = [f32(0)] * 3
    for (cc, nn, cnt) in members:
        w = f32(cnt)
        s = f32(s + w)
        c = [f32(c[a] + f32(f32(cc[a]) * w)) for a in range(3)]
        n = [f32(n[a] + f32(f32(nn[a]) * w)) for a in range(3)]
    return [f32(x / s) for x in c], [f32(x / s) for x in n], s, len(members)


def check_planes(planes, expected):
    assert len(planes) == len(expected)
    for p, (c, n, fps, nv) in zip(planes, expected):
        assert np.array_equal(p["c"], np.array(c, np.float32))
        assert np.array_equal(p["n"], np.array(n, np.float32))
        assert p["fps"] == fps and p["nvox"] == nv


UP = (0.0, 0.0, 1.0)


@pytest.mark.parametrize("impl", IMPLS)
def test_q8_range_face_reorders_ties(fccf, device_ctx, impl):
    """Four parallel planes z = 0..3 (never coplanar: 1 m apart along the normal) of 1, 2,
    2 and 3 voxels, seeded in that order: groups A1 B2 C2 D3.  range_face (:411-426), for
    i, for j > i, swap when size[i] < size[j]:
      i=0: j=1 2>1 swap -> B A C D;  j=2 2<2 no;  j=3 2<3 swap -> D A C B
      i=1: j=2 1<2 swap -> D C A B;  j=3 2<2 no
      i=2: j=3 1<2 swap -> D C B A
    so C comes before B, although B was grown first (a stable sort gives D B C A)."""
    grow = _impls(fccf)[impl][0]
    A = [((0, 0, 0), UP, 10)]
    B = [((0, 0, 1), UP, 10), ((1, 0, 1), UP, 12)]
    C = [((0, 0, 2), UP, 10), ((1, 0, 2), UP, 14)]
    D = [((0, 0, 3), UP, 10), ((1, 0, 3), UP, 10), ((2, 0, 3), UP, 10)]
    planes, theta, bases = grow(vox(A + B + C + D), 1)
    check_planes(planes, [summary(D), summary(C), summary(B), summary(A)])
    assert np.array_equal(theta, np.zeros(4))
    assert len(bases) == 0  # parallel planes: no angle in (30, 150)


@pytest.mark.parametrize("impl", IMPLS)
def test_q9_at_most_sixteen_planes(fccf, device_ctx, impl):
    """18 parallel planes of 1..18 voxels in a scrambled order: the selection breaks once
    currentSelectNum > select_plane_number = 15 (:668-673), so exactly the 16 largest,
    largest first (distinct sizes: the exchange sort is a plain descending sort)."""
    grow = _impls(fccf)[impl][0]
    sizes = [7, 18, 3, 12, 1, 16, 9, 14, 5, 11, 2, 17, 8, 13, 4, 15, 6, 10]
    groups = []
    for k, s in enumerate(sizes):
        groups.append([((x, 0, k), UP, 10) for x in range(s)])
    planes, theta, _ = grow(vox([v for g in groups for v in g]), 2)
    order = sorted(range(len(sizes)), key=lambda k: -sizes[k])[:16]
    check_planes(planes, [summary(groups[k]) for k in order])
    assert len(theta) == 16


@pytest.mark.parametrize("impl", IMPLS)
def test_q9_absorbed_group_is_ranked_but_not_selected(fccf, device_ctx, impl):
    """M (3 voxels, normal +z) and T (2 voxels whose normals lean 6 degrees towards x) lie
    in one plane z = 50.  Stage 1 keeps them apart (6 > normal_vector_threshold1 = 5,
    :557); stage 2 merges T into M (6 < 8 and both normals are perpendicular to the
    centre offset along y, :609-610): M has 5 voxels, summary over M + T in that order;
    T stays in the vector, allocated, with its 2 voxels.  With 16 more planes of 3..18
    voxels (z = 0..15), T (2) ranks below every other group and M (5) among them; the
    selection skips nothing but T, so the 16 planes are the 16 largest unallocated:
    sizes 18..4 of the stack and M (5 ties the stack's 5: the exchange sort decides)."""
    grow = _impls(fccf)[impl][0]
    s6, c6 = math.sin(math.radians(6.0)), math.cos(math.radians(6.0))
    M = [((0, y, 50), UP, 10) for y in range(3)]
    T = [((0, y, 50), (s6, 0.0, c6), 10) for y in (10, 11)]
    sizes = list(range(3, 19))
    stack = [[((x, 0, k), UP, 10) for x in range(s)] for k, s in enumerate(sizes)]
    items = M + T + [v for g in stack for v in g]
    planes, _, _ = grow(vox(items), 1)
    # groups in creation order: M, T, stack 3..18; exchange-sort them by size
    groups = [("M", 5), ("T", 2)] + [(k, s) for k, s in enumerate(sizes)]
    g = list(groups)
    for i in range(len(g) - 1):
        for j in range(i + 1, len(g)):
            if g[i][1] < g[j][1]:
                g[i], g[j] = g[j], g[i]
    chosen = [x for x in g if x[0] != "T"][:16]
    exp = [summary(M + T) if k == "M" else summary(stack[k]) for k, _ in chosen]
    check_planes(planes, exp)
    assert all(p["nvox"] != 2 for p in planes)


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("side", [1, 2])
def test_q5_nan_roughness_misaligns_type_index(fccf, device_ctx, impl, side):
    """Plane P (normal +z) absorbs a voxel with a zero normal in stage 1: the angle is
    acos(0/0) = NaN, and compare_normal returns true for NaN (:382), compare_plane true
    (both dot products 0).  P's normal becomes (0, 0, 0.5); its roughness theta-bar is
    (0 + NaN) / 2 = NaN (:662-666).  With Q (normal +x, 3 voxels) and R (normal +y, 1
    voxel): range_face orders [Q3, P2, R1].  select_base (:436-467): every pair is 90
    degrees apart, so the bases are (0,1), (0,2), (1,2); only (0,2) has two non-NaN
    roughnesses and pushes a type (0, both smooth).  type_index = [0]: base 0 reads the
    type of base 1, and bases 1 and 2 read past its end -- libfccf's sentinel (-1 for the
    driver source, -2 for the target: they never match each other)."""
    grow = _impls(fccf)[impl][0]
    P = [((0, 0, 0), UP, 10), ((1, 0, 0), (0.0, 0.0, 0.0), 10)]
    Q = [((5, y, 0), (1.0, 0.0, 0.0), 10) for y in range(3)]
    R = [((0, 5, 3), (0.0, 1.0, 0.0), 10)]
    planes, theta, bases = grow(vox(P + Q + R), side)
    assert len(planes) == 3
    assert list(planes["nvox"]) == [3, 2, 1]
    assert np.array_equal(planes[1]["n"], np.array([0, 0, 0.5], np.float32))
    assert theta[0] == 0.0 and math.isnan(theta[1]) and theta[2] == 0.0
    s = -1 if side == 1 else -2
    assert [(b["i1"], b["i2"]) for b in bases] == [(0, 1), (0, 2), (1, 2)]
    assert list(bases["angle"]) == [90.0, 90.0, 90.0]
    assert list(bases["type"]) == [0, s, s]


def T_of(t, axis=None, deg=0.0):
    """Row-major 4x4: a rotation about a coordinate axis, then translation t."""
    T = np.eye(4, dtype=np.float64)
    if axis is not None:
        a = math.radians(deg)
        c, s = math.cos(a), math.sin(a)
        i, j = {"x": (1, 2), "y": (2, 0), "z": (0, 1)}[axis]
        T[i, i], T[i, j], T[j, i], T[j, j] = c, -s, s, c
    T[:3, 3] = t
    return T.astype(np.float32)


@pytest.mark.parametrize("impl", IMPLS)
def test_q12_q13_transform_cluster(fccf, device_ctx, impl):
    """12 candidates (> cluster_number_threshold = 10), identity rotations unless noted,
    translations along x.  Radius search (:1091): d^2 < 0.8^2, neighbours by distance.
      c0 0     c1 0.5   c2 1.0       seeds c0 -> {c0, c1};  c2 -> {c2, c1}: c1 again (Q12)
      c3 10    c4 10.25 c5 10.5      seed c3 -> {c3, c4, c5}
      c6 20    c7 20.25 (90 deg about x: its x-axis is unchanged)   -> {c6, c7} (Q12)
      c8 30    c9 30.25 (90 deg about z: its x-axis turns to y)      -> {c8}, then {c9}
      c10 40                                                        -> {c10}
      c11 100  the last candidate: never seeds (:1084), so 7 clusters, not 8 (Q12)
    range_cluster on sizes [2 2 3 2 1 1 1] (K0 K2 K3 K6 K8 K9 K10): i=0 j=2 swaps K0 and
    K3, nothing else moves: [K3 K2 K0 K6 K8 K9 K10] -- K2 now precedes K0 (Q13).
    Selection with cluster_num 4 (clusternum = 3): K3 emitted (tx 30.75 / 3 = 10.25);
    K2 (2 < 3): fine 1 < 4 / 2 -> clusternum 2, K2 skipped; K0 emitted (tx 0.25, not
    K2's 0.75); K6 emitted (tx 20.125); K8 (1 < 2): fine 3 >= 2 -> stop.  Identity
    members average to the identity quaternion exactly."""
    cl = _impls(fccf)[impl][1]
    cand = [T_of((0, 0, 0)), T_of((0.5, 0, 0)), T_of((1.0, 0, 0)), T_of((10, 0, 0)), T_of((10.25, 0, 0)),
            T_of((10.5, 0, 0)), T_of((20, 0, 0)), T_of((20.25, 0, 0), "x", 90), T_of((30, 0, 0)),
            T_of((30.25, 0, 0), "z", 90), T_of((40, 0, 0)), T_of((100, 0, 0))]
    fine, ncl = cl(np.stack(cand), 4)
    assert ncl == 7
    assert fine.shape[0] == 3
    assert list(fine[:, 4]) == [10.25, 0.25, 20.125]
    assert np.array_equal(fine[:, 5:7], np.zeros((3, 2), np.float32))
    assert np.array_equal(fine[0, :4], np.array([1, 0, 0, 0], np.float32))
    assert np.array_equal(fine[1, :4], np.array([1, 0, 0, 0], np.float32))
    # K6 averages the identity and a quarter turn about x: y-axes (0,1,0), (0,0,1) ->
    # a 45-degree turn about x
    h = math.radians(22.5)
    assert np.allclose(fine[2, :4], [math.cos(h), math.sin(h), 0, 0], atol=1e-6)
    assert list(fine[:, 7]) == [1.0, 1.0, 1.0]


@pytest.mark.parametrize("impl", IMPLS)
def test_q13_accepts_cluster_num_plus_one(fccf, device_ctx, impl):
    """Six clusters of two candidates each (pairs 0.25 m apart, pairs 10 m apart), plus
    a last isolated candidate: with cluster_num = 2 the loop pushes a cluster and then
    breaks only once fine.size() > cluster_num (:1208): three clusters, not two."""
    cl = _impls(fccf)[impl][1]
    cand = []
    for k in range(6):
        cand += [T_of((10.0 * k, 0, 0)), T_of((10.0 * k + 0.25, 0, 0))]
    cand.append(T_of((500, 0, 0)))
    fine, ncl = cl(np.stack(cand), 2)
    assert ncl == 6
    assert list(fine[:, 4]) == [0.125, 10.125, 20.125]
    fine0, _ = cl(np.stack(cand), 0)  # cluster_num 0: the first push already exceeds it
    assert list(fine0[:, 4]) == [0.125]


@pytest.mark.parametrize("impl", IMPLS)
def test_q13_clusternum_below_two_ends(fccf, device_ctx, impl):
    """Sizes [2, 1, 1, ...]: clusternum = 2; the 2-cluster is emitted, then the first
    1-cluster (1 < 2) with fine 1 < cluster_num / 2 = 5 decrements clusternum to 1 < 2:
    break (:1219-1222), even though the remaining clusters would now qualify."""
    cl = _impls(fccf)[impl][1]
    cand = [T_of((0, 0, 0)), T_of((0.25, 0, 0))] + [T_of((10.0 * k, 0, 0)) for k in range(1, 11)]
    fine, ncl = cl(np.stack(cand), 10)
    assert ncl == 10  # 12 candidates, 2 in the first cluster, the last never seeds
    assert list(fine[:, 4]) == [0.125]


@pytest.mark.parametrize("impl", IMPLS)
def test_q12_few_candidates_pass_through(fccf, device_ctx, impl):
    """<= cluster_number_threshold candidates pass through unchanged and unallocated
    (:1057-1062); none gives the identity, allocated (:1045-1056)."""
    cl = _impls(fccf)[impl][1]
    cand = np.stack([T_of((k, 0, 0)) for k in range(10)])
    fine, _ = cl(cand, 5)
    assert fine.shape[0] == 10 and list(fine[:, 4]) == [float(k) for k in range(10)]
    assert not fine[:, 7].any()
    empty, _ = cl(np.zeros((0, 4, 4), np.float32), 5)
    assert np.array_equal(empty, np.array([[1, 0, 0, 0, 0, 0, 0, 1]], np.float32))


@pytest.mark.parametrize("impl", IMPLS)
def test_q15_fusion_normalises_over_all_types(fccf, device_ctx, impl):
    """Type 0: a (score 4, fine 0.5), b (2, 1.5); type 1: c (3, 1.0); type 2: none.
    score1_sum = 9 and score2_sum = 3 over BOTH types (:1539-1540), so type 0's best is
    b: 2/9 + 1.5/3 = 0.722 (a: 0.611), type 1's c: 3/9 + 1/3 = 0.667, type 2 scores 0
    with the identity (:1551-1595).  Cut 0.8 * 0.722 = 0.578: b and c are fused (:1601)
    with weights score / (0.722 + 0.667) (:1298-1300).  Per-type sums would instead give
    b 1.083 and c 2.0, and the cut 1.6 would keep c alone."""
    fuse = _impls(fccf)[impl][2]
    a, b, c = T_of((5, 5, 5)), T_of((1, 0, 0)), T_of((0, 2, 0))
    T, high = fuse([[(a, 4.0, 0.5), (b, 2.0, 1.5)], [(c, 3.0, 1.0)], []])
    s1, s2 = f32(f32(f32(0) + f32(4)) + f32(2)) + f32(3), f32(f32(f32(0) + f32(0.5)) + f32(1.5)) + f32(1.0)
    bb = f32(f32(f32(2) / s1) + f32(f32(1.5) / s2))
    bc = f32(f32(f32(3) / s1) + f32(f32(1.0) / s2))
    assert high[0, 7] == bb and high[1, 7] == bc and high[2, 7] == 0.0
    assert np.array_equal(high[2, :7], np.array([1, 0, 0, 0, 0, 0, 0], np.float32))
    assert list(high[0, 4:7]) == [1, 0, 0] and list(high[1, 4:7]) == [0, 2, 0]
    S = f32(f32(0) + bb) + bc
    tx = f32(f32(0) + f32(f32(1) * f32(bb / S))) + f32(f32(0) * f32(bc / S))
    ty = f32(f32(0) + f32(f32(0) * f32(bb / S))) + f32(f32(2) * f32(bc / S))
    assert T[0, 3] == tx and T[1, 3] == ty and T[2, 3] == 0.0
    assert np.allclose(T[:3, :3], np.eye(3), atol=1e-6)
    assert list(T[3]) == [0, 0, 0, 1]


@pytest.mark.parametrize("impl", IMPLS)
def test_q15_analyse_max_bounds_the_sums(fccf, device_ctx, impl):
    """Only the first analyse_max candidates of a type enter the sums (:1499-1544): a
    fifth type-0 candidate with a huge score changes nothing at analyse_max = 4."""
    fuse = _impls(fccf)[impl][2]
    base = [(T_of((k, 0, 0)), 1.0 + k, 0.25 * (k + 1)) for k in range(4)]
    T4, h4 = fuse([base, [(T_of((0, 1, 0)), 2.0, 0.5)], []])
    T5, h5 = fuse([base + [(T_of((9, 9, 9)), 1e6, 1e6)], [(T_of((0, 1, 0)), 2.0, 0.5)], []])
    assert np.array_equal(T4, T5) and np.array_equal(h4, h5)
