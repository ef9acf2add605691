"""PLY ingest (the reference's pcl::io::loadPLYFile<PointXYZ>,
FCCF.cpp:1655-1665): the decoder behind fccf_ply_read and the streaming upload
fccf_ply_load_device, on every layout the reader accepts.  Expected values are built
with numpy from the same bytes (parity with PCL's ply_parser conversions: binary values
in their declared type, ascii float tokens correctly rounded to float, unparsable
ascii tokens -> NaN)."""
import numpy as np
import pytest


def write_binary(path, header_props, rows, endian="<", before=None, after=None):
    """rows: structured numpy array matching header_props [(name, ply_type, np_type)]."""
    fmt = "binary_little_endian" if endian == "<" else "binary_big_endian"
    lines = ["ply", f"format {fmt} 1.0"]
    if before is not None:
        lines += [f"element camera {len(before)}", "property float a", "property uchar b"]
    lines.append(f"element vertex {len(rows)}")
    lines += [f"property {t} {n}" for n, t, _ in header_props]
    if after is not None:
        lines += [f"element face {len(after)}", "property list uchar int vertex_indices"]
    lines.append("end_header")
    with open(path, "wb") as f:
        f.write(("\n".join(lines) + "\n").encode())
        if before is not None:
            f.write(before.astype([("a", endian + "f4"), ("b", "u1")]).tobytes())
        f.write(rows.tobytes())
        if after is not None:
            for face in after:
                f.write(np.uint8(len(face)).tobytes() + np.asarray(face, endian + "i4").tobytes())


def test_binary_packed_float(fccf, tmp_path):
    rng = np.random.default_rng(1)
    xyz = rng.normal(size=(100_003, 3)).astype(np.float32)
    fccf.ply_write(str(tmp_path / "a.ply"), xyz, True)
    out = fccf.ply_read(str(tmp_path / "a.ply"))
    assert np.array_equal(out.view(np.uint32), xyz.view(np.uint32))


@pytest.mark.parametrize("endian", ["<", ">"])
def test_binary_mixed_types_and_other_elements(fccf, tmp_path, endian):
    rng = np.random.default_rng(2)
    n = 5000
    dt = np.dtype([("nx", endian + "f4"), ("x", endian + "f8"), ("red", "u1"), ("y", endian + "i2"),
                   ("z", endian + "f4"), ("i", endian + "u4")])
    rows = np.zeros(n, dt)
    rows["x"] = rng.normal(size=n) * 10
    rows["y"] = rng.integers(-3000, 3000, n)
    rows["z"] = rng.normal(size=n).astype(np.float32)
    props = [("nx", "float", None), ("x", "double", None), ("red", "uchar", None), ("y", "short", None),
             ("z", "float", None), ("i", "uint", None)]
    before = np.zeros(3, [("a", "f4"), ("b", "u1")])
    write_binary(tmp_path / "m.ply", props, rows, endian, before=before, after=[[0, 1, 2], [2, 3, 4, 5]])
    out = fccf.ply_read(str(tmp_path / "m.ply"))
    exp = np.stack([rows["x"].astype(np.float32), rows["y"].astype(np.float32), rows["z"].astype(np.float32)], 1)
    assert np.array_equal(out.view(np.uint32), exp.view(np.uint32))


def test_binary_list_in_vertex(fccf, tmp_path):
    # a list property inside the vertex element: rows of variable size are walked
    rng = np.random.default_rng(3)
    n = 777
    xyz = rng.normal(size=(n, 3)).astype(np.float32)
    lines = ["ply", "format binary_little_endian 1.0", f"element vertex {n}", "property float x",
             "property list uchar ushort tags", "property float y", "property float z", "end_header"]
    body = bytearray()
    for i in range(n):
        k = i % 4
        body += xyz[i, 0].tobytes() + np.uint8(k).tobytes() + np.arange(k, dtype="<u2").tobytes()
        body += xyz[i, 1].tobytes() + xyz[i, 2].tobytes()
    (tmp_path / "l.ply").write_bytes(("\n".join(lines) + "\n").encode() + bytes(body))
    out = fccf.ply_read(str(tmp_path / "l.ply"))
    assert np.array_equal(out.view(np.uint32), xyz.view(np.uint32))


def test_ascii_tokens_round_like_the_stream_parser(fccf, tmp_path):
    # float tokens are converted straight to float (correctly rounded), not via double:
    # decimal strings that sit near a float rounding boundary distinguish the two
    rng = np.random.default_rng(4)
    base = rng.normal(size=3000).astype(np.float32)
    toks = []
    for v in base:
        lo = np.nextafter(v, np.float32(np.inf))
        mid = (np.float64(v) + np.float64(lo)) / 2  # exactly halfway in double
        toks.append(repr(float(mid)) if np.isfinite(mid) else "0")
    toks = np.array(toks).reshape(-1, 3)
    text = "ply\nformat ascii 1.0\nelement vertex %d\nproperty float x\nproperty float y\nproperty float z\nend_header\n" % len(toks)
    text += "".join(" ".join(r) + "\r\n" for r in toks)
    (tmp_path / "t.ply").write_text(text)
    out = fccf.ply_read(str(tmp_path / "t.ply"))
    exp = np.array([[np.float32(float(t)) for t in r] for r in toks], np.float32)  # strtod then round
    # numpy's float32(float(str)) is double rounding; the correctly rounded value is
    # the float nearest to the decimal: recompute with exact rationals where they differ
    from fractions import Fraction
    for i, j in zip(*np.nonzero(out.view(np.uint32) != exp.view(np.uint32))):
        q = Fraction(toks[i, j])
        a, b = out[i, j], exp[i, j]
        assert abs(Fraction(float(a)) - q) <= abs(Fraction(float(b)) - q)
    assert np.all(np.isfinite(out))


def test_ascii_bad_token_is_nan_and_extra_columns(fccf, tmp_path):
    text = ("ply\nformat ascii 1.0\ncomment x\nelement vertex 4\nproperty float x\nproperty uchar red\n"
            "property double y\nproperty float z\nelement face 1\nproperty list uchar int vertex_indices\nend_header\n"
            "1.5 3 2.25 -4\n+7 0 1e-3 nan\nabc 1 2 3\n0.1 255 0.30000000000000004 1e39\n3 0 1 2\n")
    (tmp_path / "b.ply").write_text(text)
    out = fccf.ply_read(str(tmp_path / "b.ply"))
    assert out.shape == (4, 3)
    assert np.array_equal(out[0], np.float32([1.5, 2.25, -4]))
    assert out[1, 0] == 7 and out[1, 1] == np.float32(np.float64(1e-3)) and np.isnan(out[1, 2])
    assert np.isnan(out[2, 0]) and out[2, 1] == 2 and out[2, 2] == 3
    assert out[3, 0] == np.float32(0.1) and out[3, 1] == np.float32(0.30000000000000004)
    assert np.isnan(out[3, 2])  # out of float range: the stream parser fails -> NaN


def test_ascii_large_parallel_index(fccf, tmp_path):
    rng = np.random.default_rng(5)
    xyz = (rng.normal(size=(300_001, 3)) * 7).astype(np.float32)
    fccf.ply_write(str(tmp_path / "big.ply"), xyz, False)
    out = fccf.ply_read(str(tmp_path / "big.ply"))
    assert np.array_equal(out.view(np.uint32), xyz.view(np.uint32))


@pytest.mark.parametrize("text", [
    "plx\nformat ascii 1.0\nend_header\n",
    "ply\nformat ascii 1.0\nelement vertex 2\nproperty float x\nproperty float y\nend_header\n1 2\n3 4\n",
    "ply\nformat ascii 1.0\nelement vertex 3\nproperty float x\nproperty float y\nproperty float z\nend_header\n1 2 3\n",
    "ply\nformat binary_little_endian 1.0\nelement vertex 3\nproperty float x\nproperty float y\nproperty float z\nend_header\n\0\0",
    "ply\nformat weird 1.0\nelement vertex 0\nproperty float x\nproperty float y\nproperty float z\nend_header\n",
])
def test_rejected_like_loadplyfile(fccf, tmp_path, text):
    (tmp_path / "bad.ply").write_bytes(text.encode())
    with pytest.raises(fccf.FCCFError):
        fccf.ply_read(str(tmp_path / "bad.ply"))


@pytest.mark.gpu
@pytest.mark.parametrize("binary", [True, False])
def test_streaming_load_equals_host_read(fccf, tmp_path, binary):
    rng = np.random.default_rng(6)
    xyz = (rng.normal(size=(1_000_003, 3)) * 5).astype(np.float32)  # > 3 ring slots
    p = str(tmp_path / "s.ply")
    fccf.ply_write(p, xyz, binary)
    with fccf.Ctx(0) as ctx:
        d, n = ctx.ply_load(p)
        try:
            got = ctx.download(d, n)
        finally:
            ctx.free(d)
        assert n == len(xyz)
        assert np.array_equal(got.view(np.uint32), fccf.ply_read(p).view(np.uint32))
        with pytest.raises(fccf.FCCFError):
            ctx.ply_load(str(tmp_path / "missing.ply"))
