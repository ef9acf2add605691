"""TEST INFRASTRUCTURE: ctypes loader for the CPU oracle (oracle/build/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this; the
product (fccf-pcr_amd/) never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "build", "liboracle.so")
STABLE, INTROSORT = 0, 1  # within-leaf VoxelGrid order: INTROSORT is the reference's (std::sort)


def _load():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])
    lib = ctypes.CDLL(LIB)
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    lib.orc_register.restype = P
    lib.orc_register.argtypes = [P, I64, P, I64, ctypes.c_float, ctypes.c_int]
    lib.orc_free.argtypes = [P]
    lib.orc_get.restype = I64
    lib.orc_get.argtypes = [P, ctypes.c_char_p, P, I64]
    lib.orc_times.argtypes = [P, P]
    lib.orc_voxel_grid.restype = I64
    lib.orc_voxel_grid.argtypes = [P, I64, ctypes.c_float, ctypes.c_int, P, ctypes.POINTER(ctypes.c_int)]
    lib.orc_sort_adversary.argtypes = [I64, P]
    lib.orc_sort_pairs.restype = I64
    lib.orc_sort_pairs.argtypes = [P, I64, P]
    lib.orc_eigen33.argtypes = [P, P, P]
    lib.orc_normal_angle.restype = ctypes.c_float
    lib.orc_normal_angle.argtypes = [ctypes.c_float] * 6
    lib.orc_quat_from_rot.argtypes = [P, P]
    lib.orc_rot_from_quat.argtypes = [P, P]
    lib.orc_set_acos_mode.restype = ctypes.c_int
    lib.orc_set_acos_mode.argtypes = [ctypes.c_int]
    lib.orc_set_octree_mode.restype = ctypes.c_int
    lib.orc_set_octree_mode.argtypes = [ctypes.c_int]
    lib.orc_acos_audit.argtypes = [P, ctypes.c_int]
    lib.orc_lm_refine.restype = ctypes.c_int
    lib.orc_lm_refine.argtypes = [P, ctypes.c_int, P, P]
    lib.orc_stage_grow.argtypes = [P, I64, ctypes.c_int, P, ctypes.c_int, P, P, P, ctypes.c_int, P]
    lib.orc_stage_cluster.argtypes = [P, I64, ctypes.c_int, P, I64, P, P]
    lib.orc_stage_fuse.argtypes = [P, P, ctypes.c_int, P, P]
    return lib


lib = _load()


class Run:
    """One oracle registration (FCCF.cpp main + computer_transform_guess)."""

    def __init__(self, src, tar, leaf, order=INTROSORT):
        s = np.ascontiguousarray(src, np.float32)
        t = np.ascontiguousarray(tar, np.float32)
        self.h = lib.orc_register(s.ctypes.data, s.shape[0], t.ctypes.data, t.shape[0], float(leaf), int(order))
        if not self.h:
            raise ValueError("orc_register rejected its arguments")

    def get(self, name, dtype=np.float32):
        n = lib.orc_get(self.h, name.encode(), None, 0)
        if n < 0:
            return None
        a = np.zeros(n // np.dtype(dtype).itemsize, dtype)
        lib.orc_get(self.h, name.encode(), a.ctypes.data, n)
        return a

    @property
    def T(self):
        return self.get("T").reshape(4, 4)

    def times(self):
        ms = np.zeros(9)
        lib.orc_times(self.h, ms.ctypes.data)
        return ms

    def __del__(self):
        if getattr(self, "h", None):
            lib.orc_free(self.h)
            self.h = None


def voxel_grid(xyz, leaf, order=INTROSORT):
    a = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    out = np.zeros((max(a.shape[0], 1), 3), np.float32)
    ovf = ctypes.c_int(0)
    m = lib.orc_voxel_grid(a.ctypes.data, a.shape[0], float(leaf), int(order), out.ctypes.data, ctypes.byref(ovf))
    return out[:m].copy(), bool(ovf.value)


def sort_pairs(keys):
    """std::sort order of PCL's (idx, index) pairs for the keys != 0xFFFFFFFF."""
    k = np.ascontiguousarray(keys, np.uint32)
    perm = np.zeros(max(k.size, 1), np.uint32)
    m = lib.orc_sort_pairs(k.ctypes.data, k.size, perm.ctypes.data)
    return perm[:m].copy()


def sort_adversary(n):
    k = np.zeros(max(n, 1), np.uint32)
    lib.orc_sort_adversary(n, k.ctypes.data)
    return k[:n].copy()


def eigen33(cov):
    c = np.ascontiguousarray(cov, np.float32).reshape(9)
    ev = np.zeros(1, np.float32)
    v = np.zeros(3, np.float32)
    lib.orc_eigen33(c.ctypes.data, ev.ctypes.data, v.ctypes.data)
    return float(ev[0]), v


def normal_angle(a, b):
    return lib.orc_normal_angle(*[float(x) for x in list(a) + list(b)])


# acos conventions of FCCF.cpp:374 (see oracle/fccf_oracle.cpp theta_of_cos)
ACOS_CR_FLOAT, ACOS_LIBM_FLOAT, ACOS_DOUBLE = 0, 1, 2
AUDIT_SITES = ("grow", "merge", "rough", "base", "third", "cluster", "verify", "pair")


def set_octree_mode(mode):
    """1: PCL's pointer octree (default), 0: Morton stable sort; returns the previous mode."""
    return lib.orc_set_octree_mode(int(mode))


def set_acos_mode(mode):
    """Select the acos convention; returns the previous one."""
    return lib.orc_set_acos_mode(int(mode))


def acos_audit(reset=True):
    """{site: (evaluations, angles differing in bits, decisions flipping)} since the last reset."""
    a = np.zeros(3 * len(AUDIT_SITES), np.uint64)
    lib.orc_acos_audit(a.ctypes.data, int(bool(reset)))
    n = len(AUDIT_SITES)
    return {s: (int(a[i]), int(a[n + i]), int(a[2 * n + i])) for i, s in enumerate(AUDIT_SITES)}


def quat_from_rot(R):
    r = np.ascontiguousarray(R, np.float32).reshape(9)
    q = np.zeros(4, np.float32)
    lib.orc_quat_from_rot(r.ctypes.data, q.ctypes.data)
    return q


def rot_from_quat(q):
    qq = np.ascontiguousarray(q, np.float32).reshape(4)
    R = np.zeros(9, np.float32)
    lib.orc_rot_from_quat(qq.ctypes.data, R.ctypes.data)
    return R.reshape(3, 3)


def lm_refine(pairs):
    p = np.ascontiguousarray(pairs, np.float32).reshape(-1, 13)
    q = np.zeros(4)
    t = np.zeros(3)
    lib.orc_lm_refine(p.ctypes.data, p.shape[0], q.ctypes.data, t.ctypes.data)
    return q, t


# ---- single host stages (the known-answer tests of tests/test_host_kat.py)
VOXEL_DTYPE = np.dtype([("c", "<f4", 3), ("n", "<f4", 3), ("count", "<i4"), ("curvature", "<f4")])
PLANE_DTYPE = np.dtype([("c", "<f4", 3), ("n", "<f4", 3), ("fps", "<f4"), ("nvox", "<i4")])
BASE_DTYPE = np.dtype([("i1", "<i4"), ("i2", "<i4"), ("angle", "<f4"), ("type", "<i4")])


def stage_grow(vox, side):
    """Growth + selection + select_base (FCCF.cpp:536-677, :429-468): (planes, theta, bases)
    with libfccf's record layouts."""
    v = np.ascontiguousarray(vox, VOXEL_DTYPE)
    pl = np.zeros((64, 8), np.float32)
    th = np.zeros(64, np.float64)
    bs = np.zeros((2080, 4), np.int32)
    nF, nB = ctypes.c_int(), ctypes.c_int()
    rc = lib.orc_stage_grow(v.ctypes.data, len(v), int(side), pl.ctypes.data, 64, ctypes.byref(nF), th.ctypes.data,
                            bs.ctypes.data, 2080, ctypes.byref(nB))
    assert rc == 0
    planes = np.zeros(nF.value, PLANE_DTYPE)
    planes["c"], planes["n"] = pl[: nF.value, 0:3], pl[: nF.value, 3:6]
    planes["fps"], planes["nvox"] = pl[: nF.value, 6], pl[: nF.value, 7].astype(np.int32)
    bases = np.ascontiguousarray(bs[: nB.value]).view(BASE_DTYPE).reshape(-1).copy()
    return planes, th[: nF.value].copy(), bases


def stage_cluster(cand, cluster_num):
    """transform_cluster (FCCF.cpp:1040-1231): (fused float32[m, 8], clusters formed)."""
    a = np.ascontiguousarray(np.asarray(cand, np.float32).reshape(-1, 16))
    out = np.zeros((max(4 * len(a), 16), 8), np.float32)
    nf, ncl = ctypes.c_int64(), ctypes.c_int64()
    rc = lib.orc_stage_cluster(a.ctypes.data, len(a), int(cluster_num), out.ctypes.data, len(out), ctypes.byref(nf),
                               ctypes.byref(ncl))
    assert rc == 0 and nf.value <= len(out)
    return out[: nf.value].copy(), ncl.value


def stage_fuse(lists, analyse_max=4):
    """The fusion (FCCF.cpp:1546-1606): lists of (T, score, score2) per type -> (T, high[3, 8])."""
    recs = []
    ptrs = (ctypes.c_void_p * 3)()
    ns = (ctypes.c_int64 * 3)()
    for t in range(3):
        a = np.zeros((max(len(lists[t]), 1), 18), np.float32)
        for i, (T, s1, s2) in enumerate(lists[t]):
            a[i, :16] = np.asarray(T, np.float32).reshape(16)
            a[i, 16], a[i, 17] = s1, s2
        recs.append(a)
        ptrs[t] = a.ctypes.data
        ns[t] = len(lists[t])
    T = np.zeros(16, np.float32)
    high = np.zeros(24, np.float32)
    assert lib.orc_stage_fuse(ptrs, ns, int(analyse_max), T.ctypes.data, high.ctypes.data) == 0
    return T.reshape(4, 4), high.reshape(3, 8)
