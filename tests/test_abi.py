"""CPU-side checks of the C-ABI library: it loads, exports every symbol declared in
include/fccf.h, and its host-only entry points (params, strerror, PLY, synth) work."""
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "fccf.h")).read()
    return sorted(set(re.findall(r"\b(fccf_[a-z_0-9]+)\s*\(", hdr)))


def test_exports_every_declared_symbol(fccf):
    syms = declared_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(fccf._lib, s), s


def test_params_match_reference_defaults(fccf):
    p = fccf.default_params()
    # FCCF.cpp:126-175
    assert (p.parameter_l1, p.parameter_l2, p.parameter_k1, p.parameter_k2) == (0.5, 1.0, 5.0, 2.0)
    assert (p.normal_vector_threshold1, p.normal_vector_threshold2, p.face_voxel_size) == (5.0, 8.0, 1.0)
    assert abs(p.curvature_threshold - 0.05) < 1e-9 and p.select_plane_number == 15
    assert (p.fine_verify_voxel_size, p.fine_verify_number, p.seclct_cluster_number) == (0.5, 4.0, 200.0)
    assert abs(p.cluster_distance_threshold - 0.8) < 1e-7 and p.rough_threshold_gl == 2.0


def test_strerror(fccf):
    assert fccf.strerror(0) == "ok"
    assert "device" in fccf.strerror(fccf.E_NODEVICE)


def test_ply_roundtrip(fccf, tmp_path):
    x = fccf.synth_scene(1000, seed=5)
    for binary in (True, False):
        p = str(tmp_path / f"a{int(binary)}.ply")
        fccf.ply_write(p, x, binary)
        y = fccf.ply_read(p)
        np.testing.assert_array_equal(x, y)


def test_ply_extra_properties_and_bigendian(fccf, tmp_path):
    x = np.arange(12, dtype=np.float32).reshape(4, 3)
    p = tmp_path / "be.ply"
    hdr = ("ply\nformat binary_big_endian 1.0\nelement vertex 4\nproperty double x\nproperty uchar red\n"
           "property float y\nproperty float z\nelement face 1\nproperty list uchar int vertex_indices\nend_header\n")
    body = b"".join(np.array([r[0]], ">f8").tobytes() + b"\x07" + r[1:].astype(">f4").tobytes() for r in x)
    body += b"\x03" + np.array([0, 1, 2], ">i4").tobytes()
    p.write_bytes(hdr.encode() + body)
    np.testing.assert_array_equal(fccf.ply_read(str(p)), x)


def test_ply_missing_file(fccf):
    import pytest
    with pytest.raises(fccf.FCCFError):
        fccf.ply_read("/nonexistent/x.ply")


def test_synth_deterministic(fccf):
    a, b, T = fccf.synth_pair(5000)
    c, d, T2 = fccf.synth_pair(5000)
    np.testing.assert_array_equal(a, c)
    np.testing.assert_array_equal(b, d)
    np.testing.assert_array_equal(T, T2)
    assert np.all(b[:, 0] <= 0.8 * 20 + 0.05)  # tar cropped


def test_no_cpu_fallback_without_device(fccf):
    """Without a gfx950 device the library refuses to run (no silent CPU path)."""
    import torch
    if torch.cuda.is_available():
        import pytest
        pytest.skip("device present")
    import pytest
    with pytest.raises(fccf.FCCFError) as e:
        fccf.Ctx(0)
    assert e.value.code in (fccf.E_NODEVICE, fccf.E_HIP)
