"""Summarise rocprofv3 PMC passes into per-launch HBM traffic for bench.py.

Usage:
  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json [MIN_FRAC]

FETCH_DIR / WRITE_DIR hold the `*counter_collection.csv` of two separate passes
(`rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv ...` and the same with
WRITE_SIZE; they cannot share a pass on gfx950). Following MI355X_MICROARCH.md
("HBM"): FETCH_SIZE and WRITE_SIZE are kilobytes from the L2 memory-side request
counters, and on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read,
so traffic = 2 * FETCH_SIZE + WRITE_SIZE. The doubling is exact only for
16-B-per-lane streaming loads; narrower patterns are uncalibrated, as the guide warns,
so the raw counters are kept beside the corrected figure.  Dispatches whose
counter stays below MIN_FRAC (default 0.05) of the kernel's largest dispatch are
launches that skipped their work (radix passes past the key width exit at once) and
are left out, matching bench.py's probe, which times active launches only.
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


def per_kernel(d, counter, min_frac):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = short(row["Kernel_Name"])
                v = float(row["Counter_Value"])
                acc.setdefault(k, []).append(v)
    return {k: [x for x in v if x >= min_frac * max(v)] for k, v in acc.items()}


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    min_frac = float(sys.argv[4]) if len(sys.argv) > 4 else 0.05
    fetch = per_kernel(fetch_dir, "FETCH_SIZE", min_frac)
    write = per_kernel(write_dir, "WRITE_SIZE", min_frac)
    res = {"units": "bytes per launch", "correction": "2*FETCH_SIZE (gfx950 wide-read half count) + WRITE_SIZE",
           "kernels": {}}
    for k in sorted(set(fetch) & set(write)):
        if not fetch[k] or not write[k]:
            continue
        f_kb = statistics.mean(fetch[k])
        w_kb = statistics.mean(write[k])
        res["kernels"][k] = {"launches_fetch_pass": len(fetch[k]), "launches_write_pass": len(write[k]),
                             "FETCH_SIZE_KB_mean": f_kb, "WRITE_SIZE_KB_mean": w_kb,
                             "hbm_bytes_per_launch": (2.0 * f_kb + w_kb) * 1024.0, "active_min_frac": min_frac}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
