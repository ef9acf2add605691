"""Sanitizer builds (SURVEY.md §5 "Race detection / sanitizers"): libfccf's host-only
code -- the PLY reader (ply.cpp), the synthetic scenes (synth.cpp), the host stages
(host_stages.cpp: growth, selection, select_base, transform_cluster, quick_verify +
LM, fusion) -- and the CPU oracle, compiled with AddressSanitizer + UBSan
(tests/san/Makefile, host code only) and run here on CPU: the host stages against
the oracle's own intermediates bit for bit, the PLY reader on valid files and on
crafted headers whose counts overflow the size arithmetic.  Any sanitizer report
aborts the driver, which fails the test."""
import os
import shutil
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SAN = os.path.join(HERE, "san")
DRIVER = os.path.join(SAN, "build", "san_driver")


@pytest.fixture(scope="module")
def driver():
    if not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("make") is None:
        pytest.skip("hipcc / make not available")
    subprocess.run(["make", "-C", SAN, "-s"], check=True, timeout=600)
    return DRIVER


def run(driver, *args):
    env = dict(os.environ, ASAN_OPTIONS="abort_on_error=1:detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    p = subprocess.run([driver, *args], capture_output=True, text=True, timeout=600, env=env)
    out = p.stdout + p.stderr
    assert "Sanitizer" not in out and "runtime error" not in out, out[-4000:]
    return p.returncode, p.stdout


def test_host_stages_and_oracle_under_asan_ubsan(driver):
    rc, out = run(driver, "host")
    assert rc == 0, out
    assert out.count(": ok") == 3, out


def _header(fmt, count, props=("float x", "float y", "float z"), extra=()):
    lines = ["ply", f"format {fmt} 1.0", *extra, f"element vertex {count}"]
    lines += [f"property {p}" for p in props]
    return ("\n".join(lines + ["end_header"]) + "\n").encode()


def test_ply_reader_under_asan_ubsan(driver, fccf, tmp_path):
    rng = np.random.default_rng(7)
    xyz = rng.normal(size=(2001, 3)).astype(np.float32)
    valid, bad = [], []

    def put(name, data, ok):
        p = str(tmp_path / name)
        with open(p, "wb") as f:
            f.write(data)
        (valid if ok else bad).append(p)

    put("le.ply", _header("binary_little_endian", len(xyz)) + xyz.tobytes(), True)
    put("be.ply", _header("binary_big_endian", len(xyz)) + xyz.astype(">f4").tobytes(), True)
    put("ascii.ply", _header("ascii", 3) + b"1 2 3\n4 nan 6\n7 8 x\n", True)
    lst = b"".join(np.uint8(2).tobytes() + np.int32([1, 2]).tobytes() + r.tobytes() for r in xyz[:50])
    put("list.ply", _header("binary_little_endian", 50, ("list uchar int idx", "float x", "float y", "float z")) + lst,
        True)
    # counts that overflow rec * n or 12 * n (wrap to a tiny size) or exceed the data
    for i, cnt in enumerate(["4611686018427387904", "1537228672809129302", "99999999999", "2147483648",
                             "-5", "1e9", "0x10", "2147483647"]):
        put(f"count{i}.ply", _header("binary_little_endian", cnt) + xyz[:4].tobytes(), False)
        put(f"acount{i}.ply", _header("ascii", cnt) + b"1 2 3\n", False)
    put("short.ply", _header("binary_little_endian", 100) + xyz[:10].tobytes(), False)
    put("ashort.ply", _header("ascii", 5) + b"1 2 3\n4 5 6\n", False)
    # a list count that is not an integer (1e30 as a double count type) or negative
    put("lhuge.ply", _header("binary_little_endian", 1, ("list double int idx", "float x", "float y", "float z")) +
        np.float64(1e30).tobytes() + xyz[0].tobytes(), False)
    put("lneg.ply", _header("binary_little_endian", 1, ("list int int idx", "float x", "float y", "float z")) +
        np.int32(-3).tobytes() + xyz[0].tobytes(), False)
    put("alhuge.ply", _header("ascii", 1, ("list uchar int idx", "float x", "float y", "float z")) + b"1e30 1 2 3\n", True)
    put("noheader.ply", b"ply\nformat ascii 1.0\nelement vertex 1\n", False)
    rc, out = run(driver, "ply", *valid, *bad)
    assert rc == 0, out
    res = {ln.split()[0]: (int(ln.split()[1]), int(ln.split()[2])) for ln in out.splitlines()}
    for p in valid:
        code, n = res[p]
        assert code == 0, (p, code)
        assert n == fccf.ply_read(p).shape[0]
    for p in bad:
        assert res[p][0] == -5, (p, res[p])  # FCCF_E_IO, as loadPLYFile rejects the file
