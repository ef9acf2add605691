"""fccf_amd — ctypes binding of libfccf (include/fccf.h) for tests and bench.

This is the Python mirror of the reference's operator surface for the path: the
reference itself is a C++ CLI (`./FCCF src tar voxel`, FCCF.cpp:1646-1689) around
`computer_transform_guess` (FCCF.cpp:1370).  `register()` is that driver plus
main's VoxelGrid pass, on the GPU.  There is no CPU fallback: loading fails loudly
if lib/libfccf.so is missing, and Ctx() raises when no gfx950 device is present.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FCCF_LIB") or os.path.join(_HERE, "lib", "libfccf.so")  # FCCF_LIB: dev builds (lib_kt/)

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libfccf not built: {LIB_PATH} missing (run `make -C fccf-pcr_amd` or __graft_entry__.build())")
_lib = ctypes.CDLL(LIB_PATH)

FCCF_OK = 0
E_ARG, E_HIP, E_RCCL, E_OOM, E_IO, E_INTERNAL, E_NODEVICE = -1, -2, -3, -4, -5, -6, -7
T_NAMES = ["downsample", "voxelfit", "grow", "select", "match", "cluster", "verify", "fine", "fuse", "h2d"]

_P = ctypes.c_void_p
_I64 = ctypes.c_int64


class Params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in (
        "parameter_l1", "parameter_l2", "parameter_k1", "parameter_k2",
        "normal_vector_threshold1", "normal_vector_threshold2", "face_voxel_size",
        "voxel_point_threshold", "curvature_threshold", "select_plane_number",
        "quick_verify_angel_threshold", "quick_verify_distance_threshold", "required_optimize_plane",
        "fine_verify_voxel_size", "fine_verify_number", "included_angle_same_threshold",
        "included_angle_min_threshold", "included_angle_max_threshold", "third_plane_threshold",
        "third_plane_normal_threshold", "cluster_number_threshold", "cluster_angel_threshold",
        "cluster_distance_threshold", "seclct_cluster_number", "rough_threshold_gl")]


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in (
        "n_src", "n_tar", "m_src", "m_tar", "vox1", "vox2", "res1", "res2", "groups1", "groups2",
        "planes1", "planes2", "bases1", "bases2", "K", "K_pass")] + [
        ("cand", ctypes.c_int64 * 3), ("fine", ctypes.c_int64 * 3), ("lm_solves", ctypes.c_int64),
        ("overflow_passthrough", ctypes.c_int32), ("graph_captures", ctypes.c_int32),
        ("ms", ctypes.c_double * 10), ("ms_total", ctypes.c_double),
        ("m1_src", ctypes.c_int64), ("m1_tar", ctypes.c_int64), ("leaves1", ctypes.c_int64), ("leaves2", ctypes.c_int64),
        ("fine_evals", ctypes.c_int64), ("dev_ms", ctypes.c_double * 4), ("stage_redos", ctypes.c_int64),
        ("shard_ranks", ctypes.c_int32), ("sharded", ctypes.c_uint32), ("fine_reruns", ctypes.c_int64),
        ("xch_bytes", ctypes.c_int64 * 3)]
    SHARDED = {"search": 1, "fine": 2, "sort": 4, "faces": 8}  # fccf_stats.sharded bits (FCCF_SHARDED_*)

    def as_dict(self):
        d = {n: getattr(self, n) for n, _ in self._fields_ if n not in ("cand", "fine", "ms", "dev_ms", "xch_bytes")}
        d["xch_bytes"] = dict(zip(("match", "fine", "cloud"), list(self.xch_bytes)))
        d["dev_ms"] = dict(zip(("vg_main", "vg_driver", "faces", "fine"), list(self.dev_ms)))
        d["cand"] = list(self.cand)
        d["fine"] = list(self.fine)
        d["ms"] = dict(zip(T_NAMES, list(self.ms)))
        d["sharded"] = sorted(k for k, b in self.SHARDED.items() if self.sharded & b)
        return d


def _sig(name, res, *args):
    f = getattr(_lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_sig("fccf_params_default", None, ctypes.POINTER(Params))
_sig("fccf_strerror", ctypes.c_char_p, ctypes.c_int)
_sig("fccf_ctx_create", ctypes.c_int, ctypes.POINTER(_P), ctypes.c_int)
_sig("fccf_ctx_destroy", ctypes.c_int, _P)
_sig("fccf_ctx_set_debug", ctypes.c_int, _P, ctypes.c_int)
_sig("fccf_ctx_set_grow_device", ctypes.c_int, _P, ctypes.c_int)
_sig("fccf_ctx_set_lm_device", ctypes.c_int, _P, ctypes.c_int)
_sig("fccf_ctx_set_cluster_device", ctypes.c_int, _P, ctypes.c_int)
_sig("fccf_debug_sincos", ctypes.c_int, _P, _P, _I64, _P, _P, _P)
_sig("fccf_stage_verify", ctypes.c_int, _P, _P, ctypes.c_int, _P, ctypes.c_int, _P, _I64, ctypes.POINTER(Params), _P, _P, _P)
_sig("fccf_ctx_last_error", ctypes.c_char_p, _P)
_sig("fccf_register", ctypes.c_int, _P, _P, _I64, _P, _I64, ctypes.c_float, ctypes.POINTER(Params), _P,
     ctypes.POINTER(Stats))
_sig("fccf_register_device", ctypes.c_int, _P, _P, _I64, _P, _I64, ctypes.c_float, ctypes.POINTER(Params), _P,
     ctypes.POINTER(Stats))
_sig("fccf_register_batch", ctypes.c_int, _P, ctypes.c_int, _P, _P, _P, _P, ctypes.c_int, ctypes.c_float,
     ctypes.POINTER(Params), _P, _P)
_sig("fccf_device_upload", ctypes.c_int, _P, _P, _I64, ctypes.POINTER(_P))
_sig("fccf_device_free", ctypes.c_int, _P, _P)
_sig("fccf_stage_downsample", ctypes.c_int, _P, _P, _I64, ctypes.c_float, _P, ctypes.POINTER(_I64))
_sig("fccf_stage_downsample_presorted", ctypes.c_int, _P, _P, _I64, ctypes.c_float, _P, ctypes.POINTER(_I64))
_sig("fccf_stage_centroid", ctypes.c_int, _P, _P, _I64, _P)
_sig("fccf_stage_seqsum", ctypes.c_int, _P, _P, _I64, _P)
_sig("fccf_stage_voxel_planes", ctypes.c_int, _P, _P, _I64, ctypes.POINTER(Params), _P, _I64, ctypes.POINTER(_I64), _P,
     _I64, ctypes.POINTER(_I64), _P)
_sig("fccf_stage_grow", ctypes.c_int, _P, _P, _I64, ctypes.c_int, ctypes.POINTER(Params), _P, ctypes.c_int,
     ctypes.POINTER(ctypes.c_int), _P, _P, ctypes.c_int, ctypes.POINTER(ctypes.c_int))
_sig("fccf_stage_match", ctypes.c_int, _P, _P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int,
     ctypes.c_int, ctypes.c_int, ctypes.POINTER(Params), ctypes.POINTER(_P), ctypes.POINTER(_I64), ctypes.POINTER(_I64),
     ctypes.POINTER(_I64))
_sig("fccf_stage_cluster", ctypes.c_int, _P, _P, _I64, ctypes.c_int, ctypes.POINTER(Params), _P, _I64,
     ctypes.POINTER(_I64), ctypes.POINTER(_I64))
_sig("fccf_stage_fuse", ctypes.c_int, _P, ctypes.POINTER(_P), ctypes.POINTER(_I64), ctypes.c_int, _P, _P)
_sig("fccf_stage_fine_verify", ctypes.c_int, _P, _P, _I64, _P, _I64, _P, ctypes.c_int, ctypes.c_float, _P)
_sig("fccf_ctx_set_probe", ctypes.c_int, _P, ctypes.c_char_p)
_sig("fccf_probe_read", ctypes.c_int, _P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I64),
     ctypes.POINTER(ctypes.c_double))
_sig("fccf_probe_read_widths", ctypes.c_int, _P, ctypes.c_int, _P, _P, _P)
_sig("fccf_debug_graph_mismatch", ctypes.c_int, _P)
_sig("fccf_debug_group_fail", ctypes.c_int, _P, ctypes.c_int, ctypes.c_int)
_sig("fccf_group_aborted", ctypes.c_int, _P)
_sig("fccf_debug_get", ctypes.c_int, _P, ctypes.c_char_p, _P, _I64, ctypes.POINTER(_I64))
_sig("fccf_debug_sort_keys", ctypes.c_int, _P, _P, _I64, ctypes.c_int, _P)
if hasattr(_lib, "fccf_debug_sort_keys_batch"):  # (dev A/B runs load older builds through FCCF_LIB)
    _sig("fccf_debug_sort_keys_batch", ctypes.c_int, _P, _P, _I64, ctypes.c_int, _P, _P, ctypes.POINTER(ctypes.c_double))
_sig("fccf_debug_sort_stats", ctypes.c_int, _P, _P)
if hasattr(_lib, "fccf_debug_sort_rounds"):  # (dev A/B runs load older builds through FCCF_LIB)
    _sig("fccf_debug_sort_rounds", ctypes.c_int, _P, _P)
_sig("fccf_debug_inject_sort_fault", ctypes.c_int, _P, ctypes.c_uint32)
_sig("fccf_debug_capture_race", ctypes.c_int, _P, ctypes.c_int, ctypes.c_int, _P)
_sig("fccf_ply_read", ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.POINTER(ctypes.c_float)),
     ctypes.POINTER(_I64))
_sig("fccf_ply_write", ctypes.c_int, ctypes.c_char_p, _P, _I64, ctypes.c_int)
_sig("fccf_free", None, _P)
_sig("fccf_ply_load_device", ctypes.c_int, _P, ctypes.c_char_p, ctypes.POINTER(_P), ctypes.POINTER(_I64))
_sig("fccf_device_download", ctypes.c_int, _P, _P, _I64, _P)
_sig("fccf_group_unique_id", ctypes.c_int, _P)
_sig("fccf_group_create", ctypes.c_int, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P))
_sig("fccf_group_create_local", ctypes.c_int, ctypes.POINTER(_P), ctypes.c_int, ctypes.POINTER(_P))
_sig("fccf_group_destroy", ctypes.c_int, _P)
_sig("fccf_group_info", ctypes.c_int, _P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int))
_sig("fccf_group_bytes", ctypes.c_int, _P, ctypes.POINTER(_I64))
_sig("fccf_group_stage_match", ctypes.c_int, _P, _P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int,
     ctypes.POINTER(Params), ctypes.POINTER(_P), ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I64))
_sig("fccf_synth_scene", ctypes.c_int, _I64, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_uint64,
     ctypes.c_double, _P)
_sig("fccf_synth_pair", ctypes.c_int, _I64, ctypes.c_double, ctypes.c_double, ctypes.c_double, _P, _P, _P)


# fccf_voxel {float c[3], n[3]; int32 count; float curvature}
VOXEL_DTYPE = np.dtype([("c", "<f4", 3), ("n", "<f4", 3), ("count", "<i4"), ("curvature", "<f4")])
# fccf_plane {float c[3], n[3], fps; int32 nvox} and fccf_base {int32 i1, i2; float angle; int32 type}
PLANE_DTYPE = np.dtype([("c", "<f4", 3), ("n", "<f4", 3), ("fps", "<f4"), ("nvox", "<i4")])
BASE_DTYPE = np.dtype([("i1", "<i4"), ("i2", "<i4"), ("angle", "<f4"), ("type", "<i4")])


def planes_from_dump(a) -> np.ndarray:
    """fccf_plane records from a "planesN" dump (8 floats per plane, nvox as float)."""
    a = np.asarray(a, np.float32).reshape(-1, 8)
    out = np.zeros(a.shape[0], PLANE_DTYPE)
    out["c"], out["n"], out["fps"], out["nvox"] = a[:, 0:3], a[:, 3:6], a[:, 6], a[:, 7].astype(np.int32)
    return out


def bases_from_dump(a) -> np.ndarray:
    """fccf_base records from a "basesN" dump (i1, i2, angle bits, type as int32)."""
    a = np.ascontiguousarray(np.asarray(a, np.int32).reshape(-1, 4))
    return a.view(BASE_DTYPE).reshape(-1).copy()


class FCCFError(RuntimeError):
    def __init__(self, code, where="", detail=""):
        self.code = code
        super().__init__(f"{where}: {_lib.fccf_strerror(code).decode()} ({code})" + (f": {detail}" if detail else ""))


def _check(rc, where, h=None):
    if rc != FCCF_OK:
        detail = (_lib.fccf_ctx_last_error(h) or b"").decode(errors="replace") if h else ""
        raise FCCFError(rc, where, detail)


def default_params() -> Params:
    p = Params()
    _lib.fccf_params_default(ctypes.byref(p))
    return p


def _f32(a):
    a = np.ascontiguousarray(a, dtype=np.float32).reshape(-1, 3)
    return a


class Ctx:
    """One fccf_ctx (bound to one HIP device and its own streams)."""

    def __init__(self, device: int = 0, debug: bool = False):
        self._h = _P()
        _check(_lib.fccf_ctx_create(ctypes.byref(self._h), int(device)), "fccf_ctx_create")
        if debug:
            _check(_lib.fccf_ctx_set_debug(self._h, 1), "fccf_ctx_set_debug", self._h)

    def set_grow_device(self, on: bool = True):
        """Region growing (FCCF.cpp:536-648) on the GPU (K4) instead of the host."""
        _check(_lib.fccf_ctx_set_grow_device(self._h, int(bool(on))), "fccf_ctx_set_grow_device", self._h)

    def sincos(self, x):
        """Test hook: the device LM's correctly rounded sin/cos of float64 x: (s, c, ok)."""
        a = np.ascontiguousarray(x, np.float64).reshape(-1)
        s, c, ok = np.zeros(max(a.size, 1)), np.zeros(max(a.size, 1)), np.zeros(max(a.size, 1), np.uint32)
        _check(_lib.fccf_debug_sincos(self._h, a.ctypes.data, a.size, s.ctypes.data, c.ctypes.data, ok.ctypes.data),
               "fccf_debug_sincos", self._h)
        return s[:a.size], c[:a.size], ok[:a.size].astype(bool)

    def set_lm_device(self, on: bool = True):
        """quick_verify + LM (FCCF.cpp:680-783, :210-249) on the GPU instead of the host."""
        _check(_lib.fccf_ctx_set_lm_device(self._h, int(bool(on))), "fccf_ctx_set_lm_device", self._h)

    def set_cluster_device(self, on: bool = True):
        """transform_cluster's seeds, sort and averaging (FCCF.cpp:1040-1231) on the GPU."""
        _check(_lib.fccf_ctx_set_cluster_device(self._h, int(bool(on))), "fccf_ctx_set_cluster_device", self._h)

    def verify(self, F1, F2, qt, params: Params | None = None):
        """quick_verify + LM of clustered candidates qt[n, 8] (fccf_stage_verify):
        (T float32[n, 4, 4], score float32[n], npairs int32[n])."""
        F1, F2 = np.ascontiguousarray(F1, PLANE_DTYPE), np.ascontiguousarray(F2, PLANE_DTYPE)
        q = np.ascontiguousarray(np.asarray(qt, np.float32).reshape(-1, 8))
        n = len(q)
        T = np.zeros((max(n, 1), 16), np.float32)
        sc = np.zeros(max(n, 1), np.float32)
        npr = np.zeros(max(n, 1), np.int32)
        p = params if params is not None else default_params()
        _check(_lib.fccf_stage_verify(self._h, F1.ctypes.data, len(F1), F2.ctypes.data, len(F2), q.ctypes.data, n,
                                      ctypes.byref(p), T.ctypes.data, sc.ctypes.data, npr.ctypes.data),
               "fccf_stage_verify", self._h)
        return T[:n].reshape(-1, 4, 4), sc[:n], npr[:n]

    def close(self):
        if self._h:
            _lib.fccf_ctx_destroy(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def register(self, src, tar, leaf: float, params: Params | None = None):
        """T (4x4 float32) mapping src-file points to the tar-file frame, and stats."""
        s, t = _f32(src), _f32(tar)
        T = np.zeros(16, np.float32)
        st = Stats()
        rc = _lib.fccf_register(self._h, s.ctypes.data, s.shape[0], t.ctypes.data, t.shape[0], float(leaf),
                                ctypes.byref(params) if params is not None else None, T.ctypes.data,
                                ctypes.byref(st))
        _check(rc, "fccf_register", self._h)
        return T.reshape(4, 4), st

    def register_device(self, d_src: int, n_src: int, d_tar: int, n_tar: int, leaf: float,
                        params: Params | None = None):
        """Same, with both clouds already resident in HBM (device pointers as ints)."""
        T = np.zeros(16, np.float32)
        st = Stats()
        rc = _lib.fccf_register_device(self._h, _P(d_src), int(n_src), _P(d_tar), int(n_tar), float(leaf),
                                       ctypes.byref(params) if params is not None else None, T.ctypes.data,
                                       ctypes.byref(st))
        _check(rc, "fccf_register_device", self._h)
        return T.reshape(4, 4), st

    def register_batch(self, pairs, leaf: float, params=None, on_device=False):
        """Pipelined registration of [(src, tar), ...] (host arrays, or (ptr, n) device
        pairs when on_device).  Returns (T[n,4,4], [Stats])."""
        n = len(pairs)
        keep, sp, tp, sn, tn = [], [], [], [], []
        for s, t in pairs:
            if on_device:
                (ps, ns_), (pt, nt_) = s, t
            else:
                a, b = _f32(s), _f32(t)
                keep += [a, b]
                ps, ns_, pt, nt_ = a.ctypes.data, a.shape[0], b.ctypes.data, b.shape[0]
            sp.append(ps); tp.append(pt); sn.append(ns_); tn.append(nt_)
        arr_p = (_P * max(n, 1))
        arr_i = (_I64 * max(n, 1))
        T = np.zeros((max(n, 1), 4, 4), np.float32)
        stats = (Stats * max(n, 1))()
        p = params if params is not None else default_params()
        _check(_lib.fccf_register_batch(self._h, n, arr_p(*sp), arr_i(*sn), arr_p(*tp), arr_i(*tn), int(on_device),
                                        float(leaf), ctypes.byref(p), T.ctypes.data, stats), "fccf_register_batch", self._h)
        return T[:n], list(stats)[:n]

    def upload(self, xyz) -> int:
        """Copy xyz into a new HBM buffer of this ctx's device; returns the device pointer."""
        a = _f32(xyz)
        d = _P()
        _check(_lib.fccf_device_upload(self._h, a.ctypes.data, a.shape[0], ctypes.byref(d)), "fccf_device_upload", self._h)
        return int(d.value or 0)

    def ply_load(self, path: str):
        """Stream a PLY file into a new HBM buffer (fccf_ply_load_device): (device ptr, n)."""
        d, n = _P(), _I64()
        _check(_lib.fccf_ply_load_device(self._h, path.encode(), ctypes.byref(d), ctypes.byref(n)),
               f"fccf_ply_load_device({path})", self._h)
        return int(d.value or 0), n.value

    def download(self, dptr: int, n: int) -> np.ndarray:
        """n xyz points of an HBM buffer of this ctx back to the host (test hook)."""
        out = np.zeros((max(n, 1), 3), np.float32)
        _check(_lib.fccf_device_download(self._h, _P(dptr), int(n), out.ctypes.data), "fccf_device_download", self._h)
        return out[:n]

    def free(self, dptr: int):
        _check(_lib.fccf_device_free(self._h, _P(dptr)), "fccf_device_free", self._h)

    def downsample(self, xyz, leaf: float, presorted: bool = False):
        """PCL VoxelGrid on the GPU; presorted=True runs it as the driver's second pass does."""
        a = _f32(xyz)
        out = np.zeros_like(a) if a.shape[0] else np.zeros((1, 3), np.float32)
        m = _I64()
        f = _lib.fccf_stage_downsample_presorted if presorted else _lib.fccf_stage_downsample
        _check(f(self._h, a.ctypes.data, a.shape[0], float(leaf), out.ctypes.data, ctypes.byref(m)),
               "fccf_stage_downsample", self._h)
        return out[: m.value].copy()

    def sort_keys(self, keys, exact_gate: bool = False) -> np.ndarray:
        """K1's sort (std::sort order) of u32 leaf keys on the GPU; returns the input
        positions of the keys != 0xFFFFFFFF in sorted order (test hook)."""
        k = np.ascontiguousarray(keys, np.uint32)
        perm = np.zeros(max(k.size, 1), np.uint32)
        _check(_lib.fccf_debug_sort_keys(self._h, k.ctypes.data, k.size, int(exact_gate), perm.ctypes.data),
               "fccf_debug_sort_keys", self._h)
        return perm[:int(np.count_nonzero(k != 0xFFFFFFFF))].copy()

    def sort_keys_batch(self, keys, copies: int, xyz=None):
        """K1's sort of `copies` copies of keys in one batched launch sequence (the
        stage group's grid), writing sorted points of xyz if given.  Returns (copy 0's
        permutation, device ms)."""
        k = np.ascontiguousarray(keys, np.uint32)
        perm = np.zeros(k.size, np.uint32)
        ms = ctypes.c_double()
        x = None if xyz is None else np.ascontiguousarray(xyz, np.float32)
        _check(_lib.fccf_debug_sort_keys_batch(self._h, k.ctypes.data, k.size, int(copies),
                                               None if x is None else x.ctypes.data, perm.ctypes.data,
                                               ctypes.byref(ms)), "fccf_debug_sort_keys_batch", self._h)
        return perm, ms.value

    def graph_mismatch(self):
        """Test hook: the next cloud-stage graph replay is patched with a wrong layout
        argument; that call must fail (FCCF_E_INTERNAL) before launching anything."""
        _check(_lib.fccf_debug_graph_mismatch(self._h), "fccf_debug_graph_mismatch", self._h)

    def inject_sort_fault(self, bits: int):
        """Test hook: later K1 sorts raise these invariant flags (0 switches it off)."""
        _check(_lib.fccf_debug_inject_sort_fault(self._h, int(bits)), "fccf_debug_inject_sort_fault", self._h)

    def sort_stats(self) -> dict:
        a = np.zeros(32, np.uint32)
        _check(_lib.fccf_debug_sort_stats(self._h, a.ctypes.data), "fccf_debug_sort_stats", self._h)
        # (include/fccf.h, fccf_debug_sort_keys' path counters)
        return dict(n=int(a[0]), flags=int(a[2]), global_parts=int(a[3]), lds_segments=int(a[4]),
                    block_parts=int(a[5]), wave_parts=int(a[6]), heaps=int(a[7]), depth0_distinct=int(a[9]),
                    wave_tasks=int(a[16]) + int(a[18]), raw=a)

    def sort_rounds(self) -> np.ndarray:
        """Round records of the last sort_keys: rows {segments, tiles, owned so far, elements}."""
        a = np.zeros(96, np.uint32)
        _check(_lib.fccf_debug_sort_rounds(self._h, a.ctypes.data), "fccf_debug_sort_rounds", self._h)
        return a.reshape(24, 4)

    def capture_race(self, hold_ms: int = 200, guard: bool = True) -> dict:
        """Test hook: a graph capture held for hold_ms concurrent with another thread's
        wait on an event of the capturing stream (fccf_debug_capture_race)."""
        a = np.zeros(4, np.float64)
        _check(_lib.fccf_debug_capture_race(self._h, int(hold_ms), int(bool(guard)), a.ctypes.data),
               "fccf_debug_capture_race", self._h)
        return dict(wait_ms=float(a[0]), hold_ms=float(a[1]), wait_error=int(a[2]), after_capture=bool(a[3]))

    def voxel_planes(self, xyz, params: Params | None = None):
        """face_extrate's voxel pass (FCCF.cpp:473-534) of one downsampled cloud on the GPU.
        Returns (planar VOXEL_DTYPE[nv], residual float32[nr, 3], centroid float32[4])."""
        a = _f32(xyz)
        p = params if params is not None else default_params()
        cap = max(a.shape[0], 1)
        vox = np.zeros(cap, VOXEL_DTYPE)
        res = np.zeros((cap, 3), np.float32)
        cen = np.zeros(4, np.float32)
        nv, nr = _I64(), _I64()
        _check(_lib.fccf_stage_voxel_planes(self._h, a.ctypes.data, a.shape[0], ctypes.byref(p), vox.ctypes.data, cap,
                                            ctypes.byref(nv), res.ctypes.data, cap, ctypes.byref(nr), cen.ctypes.data),
               "fccf_stage_voxel_planes", self._h)
        return vox[: nv.value].copy(), res[: nr.value].copy(), cen

    def grow(self, vox, side: int, params: Params | None = None):
        """Region growing, plane selection and select_base (FCCF.cpp:536-677, :429-468).
        side 1 = driver source, 2 = target.  Returns (PLANE_DTYPE[F], float64 theta[F], BASE_DTYPE[B])."""
        return stage_grow(vox, side, params, self._h)

    def match(self, F1, B1, F2, B2, b1_lo: int = 0, b1_hi: int = -1, params: Params | None = None):
        """Coplane-pair correspondence search + computer_transform (FCCF.cpp:1410-1428,
        :841-1018) on the GPU for source pairs [b1_lo, b1_hi).  F*: PLANE_DTYPE arrays,
        B*: BASE_DTYPE arrays.  Returns ([cand_t float32[n_t, 4, 4] for t in 0..2], k_pass)."""
        F1, F2 = np.ascontiguousarray(F1, PLANE_DTYPE), np.ascontiguousarray(F2, PLANE_DTYPE)
        B1, B2 = np.ascontiguousarray(B1, BASE_DTYPE), np.ascontiguousarray(B2, BASE_DTYPE)
        p = params if params is not None else default_params()
        ncand, kp = (_I64 * 3)(), _I64()
        args = [self._h, F1.ctypes.data, len(F1), B1.ctypes.data, len(B1), F2.ctypes.data, len(F2),
                B2.ctypes.data, len(B2), int(b1_lo), int(b1_hi), ctypes.byref(p)]
        _check(_lib.fccf_stage_match(*args, None, None, ncand, ctypes.byref(kp)), "fccf_stage_match", self._h)
        out = [np.zeros((max(int(n), 1), 4, 4), np.float32) for n in ncand]
        ptrs = (_P * 3)(*[o.ctypes.data for o in out])
        caps = (_I64 * 3)(*[int(n) for n in ncand])
        _check(_lib.fccf_stage_match(*args, ptrs, caps, ncand, ctypes.byref(kp)), "fccf_stage_match", self._h)
        return [o[: int(n)] for o, n in zip(out, ncand)], kp.value

    def cluster(self, cand, cluster_num: int, params: Params | None = None):
        """transform_cluster (FCCF.cpp:1040-1231) of one type's candidates (float32[n, 4, 4]).
        Returns (fused float32[m, 8] = qw qx qy qz tx ty tz allocated, clusters formed)."""
        return stage_cluster(cand, cluster_num, params, self._h)

    def fuse(self, lists, analyse_max: int = 4):
        """Fusion (FCCF.cpp:1546-1606): see stage_fuse."""
        return stage_fuse(lists, analyse_max, self._h)

    def fine_verify(self, s1, s2, T, voxel: float = 0.5):
        """fine_verify (FCCF.cpp:785-839) of E <= 16 transforms T[E, 4, 4]: float32[E] scores."""
        a, b = _f32(s1), _f32(s2)
        T = np.ascontiguousarray(np.asarray(T, np.float32).reshape(-1, 16))
        sc = np.zeros(max(T.shape[0], 1), np.float32)
        _check(_lib.fccf_stage_fine_verify(self._h, a.ctypes.data, a.shape[0], b.ctypes.data, b.shape[0], T.ctypes.data,
                                           T.shape[0], float(voxel), sc.ctypes.data), "fccf_stage_fine_verify", self._h)
        return sc[: T.shape[0]]

    def set_probe(self, kernel):
        """Time every launch of `kernel` with HIP events (None = off); resets totals."""
        _check(_lib.fccf_ctx_set_probe(self._h, kernel.encode() if kernel else None), "fccf_ctx_set_probe", self._h)

    def probe_read(self):
        """(total_ms, launches, total_algorithmic_bytes) since set_probe."""
        ms, n, b = ctypes.c_double(), _I64(), ctypes.c_double()
        _check(_lib.fccf_probe_read(self._h, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b)), "fccf_probe_read", self._h)
        return ms.value, n.value, b.value

    def probe_read_widths(self, max_width=16):
        """{width: (total_ms, launches, total_algorithmic_bytes)} since set_probe, per
        launch width (clouds per batched launch), widths with launches only."""
        ms = np.zeros(max_width, np.float64)
        n = np.zeros(max_width, np.int64)
        b = np.zeros(max_width, np.float64)
        _check(_lib.fccf_probe_read_widths(self._h, max_width, ms.ctypes.data, n.ctypes.data, b.ctypes.data),
               "fccf_probe_read_widths", self._h)
        return {w + 1: (float(ms[w]), int(n[w]), float(b[w])) for w in range(max_width) if n[w]}

    def centroid(self, xyz):
        """compute3DCentroid (FCCF.cpp:473) of a dense cloud: float32[4] (x, y, z, 1)."""
        a = _f32(xyz)
        out = np.zeros(4, np.float32)
        _check(_lib.fccf_stage_centroid(self._h, a.ctypes.data, a.shape[0], out.ctypes.data), "fccf_stage_centroid", self._h)
        return out

    def seqsum(self, x) -> np.float32:
        """Left-to-right float32 sum ((0 + x0) + x1) + ... (similar_num order, FCCF.cpp:830-835)."""
        a = np.ascontiguousarray(np.asarray(x, np.float32).reshape(-1))
        out = np.zeros(1, np.float32)
        _check(_lib.fccf_stage_seqsum(self._h, a.ctypes.data, a.shape[0], out.ctypes.data), "fccf_stage_seqsum", self._h)
        return out[0]

    def debug(self, name: str, dtype=np.float32):
        n = _I64()
        rc = _lib.fccf_debug_get(self._h, name.encode(), None, 0, ctypes.byref(n))
        if rc != FCCF_OK:
            return None
        buf = np.zeros(n.value // np.dtype(dtype).itemsize, dtype)
        _check(_lib.fccf_debug_get(self._h, name.encode(), buf.ctypes.data, n.value, ctypes.byref(n)), "debug")
        return buf


GROUP_ID_BYTES = 128


def group_unique_id() -> bytes:
    """An RCCL unique id (rank 0 makes it; every rank of the group needs the same bytes)."""
    buf = (ctypes.c_uint8 * GROUP_ID_BYTES)()
    _check(_lib.fccf_group_unique_id(buf), "fccf_group_unique_id")
    return bytes(buf)


class Group:
    """One rank of an RCCL group attached to a Ctx (fccf_group_create): while it is
    open, the ctx's registrations shard the correspondence search across the ranks."""

    def __init__(self, ctx: "Ctx", uid: bytes, n_ranks: int, rank: int):
        if len(uid) != GROUP_ID_BYTES:
            raise ValueError("group id must be 128 bytes")
        self.ctx = ctx
        self._h = _P()
        buf = (ctypes.c_uint8 * GROUP_ID_BYTES).from_buffer_copy(uid)
        _check(_lib.fccf_group_create(ctx._h, buf, int(n_ranks), int(rank), ctypes.byref(self._h)),
               "fccf_group_create", ctx._h)

    @classmethod
    def _wrap(cls, ctx: "Ctx", h) -> "Group":
        g = cls.__new__(cls)
        g.ctx = ctx
        g._h = h
        return g

    def info(self):
        n, r = ctypes.c_int(), ctypes.c_int()
        _check(_lib.fccf_group_info(self._h, ctypes.byref(n), ctypes.byref(r)), "fccf_group_info")
        return n.value, r.value

    def rx_bytes(self):
        """Bytes this rank has received through the group's collectives, per channel
        (candidate gather, fine scores, cloud stage rows D and P), since creation."""
        a = (_I64 * 3)()
        _check(_lib.fccf_group_bytes(self._h, a), "fccf_group_bytes")
        return [int(x) for x in a]

    def aborted(self) -> bool:
        """True once the group was aborted (a failed registration on this rank or a
        peer's failure seen at the group's time limit); destroy and recreate it."""
        r = _lib.fccf_group_aborted(self._h)
        if r < 0:
            _check(r, "fccf_group_aborted")
        return bool(r)

    def inject_failure(self, site: int, silent: bool = False):
        """Test hook: fail this rank at collective site 1 (candidate gather), 2 (fine
        scores) or 3 (sharded sort gather) of its next registration; silent: without
        aborting the transport (a dead peer)."""
        _check(_lib.fccf_debug_group_fail(self._h, int(site), 1 if silent else 0), "fccf_debug_group_fail")

    def match(self, F1, B1, F2, B2, params: Params | None = None):
        """The sharded search (fccf_group_stage_match): same result as Ctx.match over
        all source pairs, on every rank."""
        F1, F2 = np.ascontiguousarray(F1, PLANE_DTYPE), np.ascontiguousarray(F2, PLANE_DTYPE)
        B1, B2 = np.ascontiguousarray(B1, BASE_DTYPE), np.ascontiguousarray(B2, BASE_DTYPE)
        p = params if params is not None else default_params()
        ncand, kp = (_I64 * 3)(), _I64()
        args = [self._h, F1.ctypes.data, len(F1), B1.ctypes.data, len(B1), F2.ctypes.data, len(F2),
                B2.ctypes.data, len(B2), ctypes.byref(p)]
        _check(_lib.fccf_group_stage_match(*args, None, None, ncand, ctypes.byref(kp)), "fccf_group_stage_match",
               self.ctx._h)
        out = [np.zeros((max(int(n), 1), 4, 4), np.float32) for n in ncand]
        ptrs = (_P * 3)(*[o.ctypes.data for o in out])
        caps = (_I64 * 3)(*[int(n) for n in ncand])
        _check(_lib.fccf_group_stage_match(*args, ptrs, caps, ncand, ctypes.byref(kp)), "fccf_group_stage_match",
               self.ctx._h)
        return [o[: int(n)] for o, n in zip(out, ncand)], kp.value

    def close(self):
        """Releases the communicator.  Safe in either order with Ctx.close: a ctx
        destroyed first detaches its group (fccf_ctx_destroy)."""
        if self._h:
            _lib.fccf_group_destroy(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def local_groups(ctxs) -> list:
    """Virtual ranks (fccf_group_create_local, a test hook): one Group per Ctx, all on
    one device, exchanging through host barriers instead of RCCL.  Rank r's calls must
    run on their own thread, concurrently with the other ranks' (ctypes releases the
    GIL inside the library), exactly as one process per GPU would."""
    n = len(ctxs)
    hs = (_P * n)(*[c._h for c in ctxs])
    out = (_P * n)()
    _check(_lib.fccf_group_create_local(hs, n, out), "fccf_group_create_local")
    return [Group._wrap(c, _P(out[i])) for i, c in enumerate(ctxs)]


# The host-only stage exports (fccf_stage_grow / _cluster / _fuse run the product's host
# C++; they need no GPU, so they can be called without a ctx, e.g. by the CPU tests).
def stage_grow(vox, side: int, params: Params | None = None, h=None):
    """Region growing, plane selection and select_base (FCCF.cpp:536-677, :429-468) of
    VOXEL_DTYPE records.  Returns (PLANE_DTYPE[F], float64 theta[F], BASE_DTYPE[B])."""
    v = np.ascontiguousarray(vox, VOXEL_DTYPE)
    p = params if params is not None else default_params()
    planes, theta, bases = np.zeros(64, PLANE_DTYPE), np.zeros(64, np.float64), np.zeros(2080, BASE_DTYPE)
    nF, nB = ctypes.c_int(), ctypes.c_int()
    _check(_lib.fccf_stage_grow(h, v.ctypes.data, len(v), int(side), ctypes.byref(p), planes.ctypes.data,
                                len(planes), ctypes.byref(nF), theta.ctypes.data, bases.ctypes.data, len(bases),
                                ctypes.byref(nB)), "fccf_stage_grow", h)
    return planes[: nF.value].copy(), theta[: nF.value].copy(), bases[: nB.value].copy()


def stage_cluster(cand, cluster_num: int, params: Params | None = None, h=None):
    """transform_cluster (FCCF.cpp:1040-1231) of one type's candidates (float32[n, 4, 4]).
    Returns (fused float32[m, 8] = qw qx qy qz tx ty tz allocated, clusters formed)."""
    a = np.ascontiguousarray(np.asarray(cand, np.float32).reshape(-1, 16))
    p = params if params is not None else default_params()
    nf, ncl = _I64(), _I64()
    _check(_lib.fccf_stage_cluster(h, a.ctypes.data, len(a), int(cluster_num), ctypes.byref(p), None, 0,
                                   ctypes.byref(nf), ctypes.byref(ncl)), "fccf_stage_cluster", h)
    out = np.zeros((max(nf.value, 1), 8), np.float32)
    _check(_lib.fccf_stage_cluster(h, a.ctypes.data, len(a), int(cluster_num), ctypes.byref(p),
                                   out.ctypes.data, nf.value, ctypes.byref(nf), ctypes.byref(ncl)),
           "fccf_stage_cluster", h)
    return out[: nf.value], ncl.value


def stage_fuse(lists, analyse_max: int = 4, h=None):
    """Fusion of computer_transform_guess (FCCF.cpp:1546-1606).  lists: three sequences of
    (T float32[4, 4], quick_verify score, fine_verify score) in score_range order.
    Returns (T float32[4, 4], high float32[3, 8] = per-type best qw qx qy qz tx ty tz score)."""
    recs, ptrs, ns = [], (_P * 3)(), (_I64 * 3)()
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
    _check(_lib.fccf_stage_fuse(h, ptrs, ns, int(analyse_max), T.ctypes.data, high.ctypes.data), "fccf_stage_fuse", h)
    return T.reshape(4, 4), high.reshape(3, 8)


def strerror(code: int) -> str:
    return _lib.fccf_strerror(code).decode()


def ply_read(path: str) -> np.ndarray:
    p = ctypes.POINTER(ctypes.c_float)()
    n = _I64()
    _check(_lib.fccf_ply_read(path.encode(), ctypes.byref(p), ctypes.byref(n)), f"fccf_ply_read({path})")
    try:
        return np.ctypeslib.as_array(p, shape=(n.value * 3,)).reshape(-1, 3).copy() if n.value else np.zeros((0, 3), np.float32)
    finally:
        _lib.fccf_free(p)


def ply_write(path: str, xyz, binary: bool = True):
    a = _f32(xyz)
    _check(_lib.fccf_ply_write(path.encode(), a.ctypes.data, a.shape[0], 1 if binary else 0), "fccf_ply_write")


def synth_scene(n: int, room=(20.0, 15.0, 4.0), seed: int = 1, crop_x_frac: float = 0.0) -> np.ndarray:
    out = np.zeros((max(n, 1), 3), np.float32)
    _check(_lib.fccf_synth_scene(n, *map(float, room), seed, crop_x_frac, out.ctypes.data), "fccf_synth_scene")
    return out[:n]


def synth_pair(n: int, room=(20.0, 15.0, 4.0)):
    """(src, tar, T_gt): tar = scene cropped to x <= 0.8 Lx, src = scene mapped by T_gt^-1."""
    src = np.zeros((max(n, 1), 3), np.float32)
    tar = np.zeros((max(n, 1), 3), np.float32)
    T = np.zeros(16, np.float32)
    _check(_lib.fccf_synth_pair(n, *map(float, room), src.ctypes.data, tar.ctypes.data, T.ctypes.data),
           "fccf_synth_pair")
    return src[:n], tar[:n], T.reshape(4, 4)


# Workloads of BASELINE.json configs[1..4]; configs[0] is the ETH PLY pair.
CONFIGS = {
    "c2": dict(n=100_000, room=(20.0, 15.0, 4.0), leaf=0.1),
    "c3": dict(n=1_000_000, room=(20.0, 15.0, 4.0), leaf=0.05),
    "c4": dict(n=5_000_000, room=(30.0, 24.0, 6.0), leaf=0.05),
    "c5": dict(n=10_000_000, room=(30.0, 24.0, 6.0), leaf=0.02),
}
