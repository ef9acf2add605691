"""Summarise tools/gpu_pmc_calib.sh: per calibration kernel (known bytes per launch,
tools/pmc_calib.hip) the counters' reading against the algorithmic bytes.

Usage: python tools/pmc_calib.py OUT_DIR [OUT.json]

Read bytes are counted two ways:
  FETCH_SIZE     rocprofv3's derived counter, (TCC_BUBBLE*128 + (RDREQ - BUBBLE - RDREQ_32B)*64
                 + RDREQ_32B*32) / 1024 KB: on gfx950 the 128-byte requests are not in
                 TCC_BUBBLE, so every one of them is tallied as 64 B (the guide's "half");
  exact          32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B from the request-size
                 buckets, which the guide does not use.
Write bytes: WRITE_SIZE, and 32*(WRREQ - WRREQ_64B) + 64*WRREQ_64B.
"""
import csv
import glob
import json
import os
import re
import statistics
import sys


def short(name):
    m = re.search(r"^\s*(?:void\s+)?([A-Za-z_][\w:]*)", name)
    s = m.group(1) if m else name
    return s.split("::")[-1]


def counters(d):
    """{kernel: {counter: [value per dispatch]}} from every counter_collection.csv under d."""
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                acc.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return acc


def merged(out_dir, prefix):
    acc = {}
    for d in sorted(glob.glob(os.path.join(out_dir, prefix + "*"))):
        if not os.path.isdir(d):
            continue
        for k, cs in counters(d).items():
            acc.setdefault(k, {}).update(cs)
    return acc


def exact_bytes(cs):
    """(read, write) bytes per dispatch from the size buckets, or None where a pass is missing."""
    m = {c: statistics.mean(v) for c, v in cs.items()}
    rd = wr = None
    if all(c in m for c in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")):
        rd = 32 * m["TCC_EA0_RDREQ_32B_sum"] + 64 * m["TCC_EA0_RDREQ_64B_sum"] + 128 * m["TCC_EA0_RDREQ_128B_sum"]
    if all(c in m for c in ("TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum")):
        wr = 32 * (m["TCC_EA0_WRREQ_sum"] - m["TCC_EA0_WRREQ_64B_sum"]) + 64 * m["TCC_EA0_WRREQ_64B_sum"]
    return rd, wr, m


def main():
    out_dir = sys.argv[1]
    alg = {}
    for line in open(os.path.join(out_dir, "calib_alg.txt")):
        p = line.split()
        if len(p) == 2 and p[1].isdigit():
            alg[p[0]] = float(p[1])
    acc = merged(out_dir, "calib_p")
    res = {"source": "tools/pmc_calib.hip under tools/gpu_pmc_calib.sh (one counter pass per process)",
           "kernels": {}}
    for k in alg:
        if k not in acc:
            continue
        rd, wr, m = exact_bytes(acc[k])
        a = alg[k]
        is_ld = k.endswith("_ld")
        e = {"algorithmic_bytes": a,
             "FETCH_SIZE_bytes": m.get("FETCH_SIZE", 0.0) * 1024, "WRITE_SIZE_bytes": m.get("WRITE_SIZE", 0.0) * 1024,
             "exact_read_bytes": rd, "exact_write_bytes": wr,
             "req_32B": m.get("TCC_EA0_RDREQ_32B_sum"), "req_64B": m.get("TCC_EA0_RDREQ_64B_sum"),
             "req_128B": m.get("TCC_EA0_RDREQ_128B_sum"), "wrreq": m.get("TCC_EA0_WRREQ_sum"),
             "wrreq_64B": m.get("TCC_EA0_WRREQ_64B_sum"), "rdreq_dram": m.get("TCC_EA0_RDREQ_DRAM_sum"),
             "bubble": m.get("TCC_BUBBLE_sum")}
        main_ctr = e["FETCH_SIZE_bytes"] if is_ld else e["WRITE_SIZE_bytes"]
        main_ex = rd if is_ld else wr
        e["counter_over_algorithmic"] = main_ctr / a if a else None
        e["exact_over_algorithmic"] = main_ex / a if (a and main_ex is not None) else None
        res["kernels"][k] = e
        print(f"{k:12s} alg {a / 1e6:9.2f} MB  {'FETCH' if is_ld else 'WRITE'}_SIZE/alg "
              f"{e['counter_over_algorithmic']:.3f}  exact/alg "
              f"{e['exact_over_algorithmic'] if e['exact_over_algorithmic'] is not None else float('nan'):.3f}  "
              f"req32/64/128 {e['req_32B']}/{e['req_64B']}/{e['req_128B']}  wr {e['wrreq']}/{e['wrreq_64B']}")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
