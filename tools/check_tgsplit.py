"""Dev: TG_SPLIT bit (COMPUTE_PGM_RSRC3 bit 16, gfx90a+) of every kernel descriptor in
a gfx950 device code object.  With it clear, all waves of a workgroup run on one CU.
Usage: python tools/check_tgsplit.py <csrc/*.hip source or device code object>
(a .hip source is compiled device-only for gfx950 first, with the library's flags)."""
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin/"


def kernels(path):
    data = open(path, "rb").read()
    sec = subprocess.run([LLVM + "llvm-readelf", "-S", path], capture_output=True, text=True, check=True).stdout
    addr = off = None
    for line in sec.splitlines():
        f = line.split()
        if ".rodata" in f:
            i = f.index(".rodata")
            addr, off = int(f[i + 2], 16), int(f[i + 3], 16)
    syms = subprocess.run([LLVM + "llvm-readelf", "-s", path], capture_output=True, text=True, check=True).stdout
    seen = set()
    for line in syms.splitlines():
        f = line.split()
        if len(f) >= 8 and f[7].endswith(".kd") and f[7] not in seen:
            seen.add(f[7])
            kd = data[off + int(f[1], 16) - addr:][:64]
            rsrc3 = int.from_bytes(kd[0x2C:0x30], "little")
            yield f[7][:-3], (rsrc3 >> 16) & 1


def device_object(path):
    if not path.endswith(".hip"):
        return path
    import os
    import tempfile
    out = os.path.join(tempfile.mkdtemp(), "dev.o")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fno-fast-math", "-I" + os.path.dirname(os.path.abspath(path)), "-c", path,
                    "--offload-device-only", "--no-gpu-bundle-output", "-o", out], check=True)
    return out


if __name__ == "__main__":
    bad = 0
    for name, tg in kernels(device_object(sys.argv[1])):
        print(f"tg_split={tg}  {name}")
        bad |= tg
    sys.exit(bad)
