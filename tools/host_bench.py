"""Dump oracle inputs of the host stages (c3 pair by default) and time libfccf's
host transform_cluster / quick_verify on them on this CPU (development tool).

Usage: python tools/host_bench.py [config] [reps] [threads ...]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fccf-pcr_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import fccf_amd as F  # noqa: E402
import oracle_py as O  # noqa: E402  (test infrastructure: input generator only)

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
reps = sys.argv[2] if len(sys.argv) > 2 else "20"
out = os.path.join(ROOT, "scratch", "hb")
os.makedirs(out, exist_ok=True)
c = F.CONFIGS[cfg]
src, tar, _ = F.synth_pair(c["n"], c["room"])
r = O.Run(src, tar, c["leaf"], O.STABLE)
for k in ("planes1", "planes2", "cand0", "cand1", "cand2", "vox1", "vox2"):
    r.get(k, np.float32).astype(np.float32).tofile(os.path.join(out, k + ".bin"))
exe = os.path.join(ROOT, "scratch", "host_bench")
lib = os.environ.get("HB_LIB", os.path.join(ROOT, "fccf-pcr_amd", "lib"))
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-o", exe,
                os.path.join(ROOT, "tools", "host_bench.cpp"), "-L" + lib, "-lfccf", "-Wl,-rpath," + lib], check=True)
for th in (sys.argv[3:] or ["1", "8"]):
    subprocess.run([exe, out, reps, th], check=True)
