"""Summarise rocprofv3 PMC passes over the bench command into per-launch traffic for
bench.py's roofline.traffic (tools/gpu_pmc_calib.sh writes the passes).

Usage:
  python tools/pmc_traffic.py PMC_DIR CONFIG OUT.json [MIN_FRAC] [WIDTH]

WIDTH (default 2): the clouds per launch of the workload's cloud-stage kernels -- 2 for
single registrations (the bench command with --no-pipeline), 10 for tools/pmc_batch.py
(five pairs per stage, the timed region's shape; 8 in the summaries before r05au); recorded in OUT.json for bench.py.

PMC_DIR holds bench_p1 .. bench_p4, one counter pass per process (rocprofv3 does not
split counters over passes, and a pass holds at most 4 TCC counters):
  p1  TCC_EA0_RDREQ_sum, TCC_EA0_RDREQ_32B_sum, _64B_sum, _128B_sum
  p2  TCC_EA0_WRREQ_sum, TCC_EA0_WRREQ_64B_sum
  p3  FETCH_SIZE            p4  WRITE_SIZE
and bench_p1.json, the bench line of pass 1, whose kernel_table carries each kernel's
algorithmic bytes per launch (SURVEY.md §8(d) figures, bench.py's probe).

Three figures per kernel and launch:
  raw        FETCH_SIZE + WRITE_SIZE (kilobytes x 1024);
  guide      2 x FETCH_SIZE + WRITE_SIZE: MI355X_MICROARCH.md's gfx950 correction, exact
             for wide coalesced reads only (128-B requests tallied at 64 B);
  exact      32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B read bytes plus
             32 x (WRREQ - WRREQ_64B) + 64 x WRREQ_64B write bytes.  Calibrated on known
             byte counts for every access width the sort uses (tools/pmc_calib.hip,
             profiles/r04*/pmc_calib.json): 1.000 of the algorithmic bytes for 2-, 4- and
             16-B coalesced loads and for 4- and 16-B coalesced stores, and exactly one
             128-B line per random 2-, 4- or 12-B load.  hbm_bytes_per_launch is this one.
All three count the L2's memory-side requests, Infinity-Cache hits included (the guide:
"appear to be counted, not excluded"; TCC_EA0_RDREQ_DRAM reads the same as RDREQ in the
calibration), so they are L2-miss traffic, an upper bound on HBM bytes.

Dispatches whose counter stays below MIN_FRAC (default 0.05) of the kernel's largest
dispatch are left out (launches that skip their work), as bench.py's probe times active
launches only.
"""
import csv
import glob
import json
import os
import re
import statistics
import sys


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name


def per_kernel(d):
    """{kernel: {counter: [value per dispatch, in dispatch order]}}"""
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows = sorted(csv.DictReader(fh), key=lambda r: int(r["Dispatch_Id"]))
        for row in rows:
            acc.setdefault(short(row["Kernel_Name"]), {}).setdefault(row["Counter_Name"], []).append(
                float(row["Counter_Value"]))
    return acc


def active_mean(vals, min_frac):
    if not vals:
        return None, 0
    mx = max(vals)
    keep = [v for v in vals if v >= min_frac * mx] if mx > 0 else vals
    return statistics.mean(keep), len(keep)


def main():
    pmc_dir, config, out = sys.argv[1:4]
    min_frac = float(sys.argv[4]) if len(sys.argv) > 4 else 0.05
    width = int(sys.argv[5]) if len(sys.argv) > 5 else 2
    passes = {}
    for i in range(1, 5):
        for k, cs in per_kernel(os.path.join(pmc_dir, f"bench_p{i}")).items():
            passes.setdefault(k, {}).update(cs)
    alg = {}
    bj = os.path.join(pmc_dir, "bench_p1.json")
    if os.path.exists(bj):
        for k, v in json.load(open(bj)).get("kernel_table", {}).items():
            alg[k] = v.get("algorithmic_bytes_per_launch")
    res = {"config": config, "width": width, "units": "bytes per launch (active launches)",
           "hbm_bytes_per_launch": "exact: calibrated request-size buckets (see tools/pmc_traffic.py)",
           "kernels": {}}
    for k, cs in sorted(passes.items()):
        m = {}
        n = {}
        for c, v in cs.items():
            m[c], n[c] = active_mean(v, min_frac)
        need = ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_WRREQ_sum",
                "TCC_EA0_WRREQ_64B_sum", "FETCH_SIZE", "WRITE_SIZE")
        if any(m.get(c) is None for c in need):
            continue
        rd = 32 * m["TCC_EA0_RDREQ_32B_sum"] + 64 * m["TCC_EA0_RDREQ_64B_sum"] + 128 * m["TCC_EA0_RDREQ_128B_sum"]
        wr = 32 * (m["TCC_EA0_WRREQ_sum"] - m["TCC_EA0_WRREQ_64B_sum"]) + 64 * m["TCC_EA0_WRREQ_64B_sum"]
        f_b, w_b = m["FETCH_SIZE"] * 1024.0, m["WRITE_SIZE"] * 1024.0
        a = alg.get(k) or alg.get(k[:-2] if k.endswith("_s") else k)
        e = {"launches": n["FETCH_SIZE"], "raw_bytes": f_b + w_b, "guide_bytes": 2 * f_b + w_b,
             "exact_read_bytes": rd, "exact_write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
             "algorithmic_bytes_per_launch": a,
             "exact_over_algorithmic": (rd + wr) / a if a else None,
             "raw_over_algorithmic": (f_b + w_b) / a if a else None,
             "active_min_frac": min_frac}
        res["kernels"][k] = e
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, e in sorted(res["kernels"].items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"]):
        if e["hbm_bytes_per_launch"] < 1e6:
            continue
        r = e["exact_over_algorithmic"]
        print(f"{k:22s} exact {e['hbm_bytes_per_launch'] / 1e6:9.2f} MB  raw {e['raw_bytes'] / 1e6:9.2f}  "
              f"guide {e['guide_bytes'] / 1e6:9.2f}  alg {(e['algorithmic_bytes_per_launch'] or 0) / 1e6:8.2f}  "
              f"exact/alg {r if r is not None else float('nan'):.2f}")


if __name__ == "__main__":
    main()
