"""Device-side kernel timeline of registrations (development; csrc/ktrace.h).

Usage (GPU box): make -C fccf-pcr_amd KTRACE=1 lib_kt/libfccf.so, then
  FCCF_LIB=fccf-pcr_amd/lib_kt/libfccf.so python tools/ktrace.py [config] [reps] [batch]
Prints, for the last registration, every instrumented kernel's block-(0,0) start
time (s_memrealtime, 100 MHz) relative to the first one, the gap to the next kernel,
and per-kernel totals of those gaps (the start-to-start cost of each kernel).
"""
import ctypes
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fccf-pcr_amd"))
import numpy as np  # noqa: E402
import fccf_amd as F  # noqa: E402


def kernel_map():
    m = {}
    for f in glob.glob(os.path.join(ROOT, "fccf-pcr_amd", "csrc", "*")):
        src = open(f).read().split("\n")
        tu = None
        for ln in src:
            t = re.match(r"#define KT_TU (\d+)", ln)
            if t:
                tu = int(t.group(1))
        if tu is None:
            continue
        name = "?"
        for i, ln in enumerate(src, 1):
            k = re.search(r"\b(k_\w+)\s*\(", ln)
            if k and "__global__" in " ".join(src[max(0, i - 3):i]):
                name = k.group(1)
            if "KT();" in ln:
                m[(tu, i)] = name
    return m


def main():
    cfg = F.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    hip = ctypes.CDLL("libamdhip64.so")
    names = kernel_map()
    src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
    ctx = F.Ctx(0)
    ds, dt = ctx.upload(src), ctx.upload(tar)
    buf = ctx.upload(np.zeros((16384 * 8 // 12 + 1, 3), np.float32))
    F._lib.fccf_ktrace_arm.argtypes = [ctypes.c_void_p]
    batch = len(sys.argv) > 3 and sys.argv[3] == "batch"
    for _ in range(reps):
        F._lib.fccf_ktrace_arm(ctypes.c_void_p(buf))
        if batch:  # pipelined: pair i+1's cloud stage overlaps pair i's phase B
            ctx.register_batch([((ds, src.shape[0]), (dt, tar.shape[0]))] * 4, cfg["leaf"], on_device=True)
        else:
            ctx.register_device(ds, src.shape[0], dt, tar.shape[0], cfg["leaf"])
    F._lib.fccf_ktrace_arm(None)
    out = np.zeros(16384, np.uint64)
    hip.hipDeviceSynchronize()
    hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(buf), ctypes.c_size_t(out.nbytes), 2)
    n = int(out[0])
    rec = out[2:2 + 2 * n].reshape(-1, 2)
    rec = rec[np.argsort(rec[:, 1], kind="stable")]
    t0 = int(rec[0, 1])
    tot = {}
    for i, (tag, ts) in enumerate(rec):
        tag, ts = int(tag), int(ts)
        nm = names.get((tag >> 32, tag & 0xFFFFFFFF), f"{tag >> 32}:{tag & 0xFFFFFFFF}")
        nxt = int(rec[i + 1, 1]) if i + 1 < len(rec) else ts
        gap = (nxt - ts) / 100.0
        print(f"{(ts - t0) / 100.0:9.2f} {gap:7.2f}  {nm}")
        c, g = tot.get(nm, (0, 0.0))
        tot[nm] = (c + 1, g + gap)
    print(f"{n} kernel starts over {(int(rec[-1, 1]) - t0) / 100.0:.1f} us")
    for nm, (c, g) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"  {nm:24s} {c:4d} launches {g:9.1f} us start-to-next")


if __name__ == "__main__":
    main()
