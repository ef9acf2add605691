"""Dev probe: K1's sort rounds one by one on the c3 first-pass keys of one cloud.

Run:   python tools/round_profile.py [reps]            -> the round records (fccf_debug_sort_rounds)
Under: rocprofv3 --kernel-trace --output-format csv -d DIR -- python tools/round_profile.py 5
then:  python tools/round_profile.py --csv DIR/.../kernel_trace.csv
       -> every launch of the last sort in order, with its duration and the gap before it.
"""
import csv
import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fccf-pcr_amd"), os.path.join(ROOT, "tools")]


def analyze(path):
    rows = []
    for f in glob.glob(path) if "*" in path else [path]:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # the last sort: from the last k_is_prep to the k_is_wave after it
    starts = [i for i, r in enumerate(rows) if "k_is_prep" in r[2]]
    i0 = starts[-1]
    i1 = next(i for i in range(i0, len(rows)) if "k_is_wave" in rows[i][2])
    prev_end = rows[i0][0]
    t0 = rows[i0][0]
    rnd = -1
    for s, e, n in rows[i0:i1 + 1]:
        short = n.split("(")[0].replace("fccf::(anonymous namespace)::", "")
        if "count" in short:
            rnd += 1
        print(f"{(s - t0) / 1e3:9.2f} us  gap {(s - prev_end) / 1e3:6.2f}  dur {(e - s) / 1e3:7.2f}  r{rnd:<3d} {short}")
        prev_end = e
    print(f"sort span {(rows[i1][1] - t0) / 1e3:.1f} us")


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--csv":
        analyze(sys.argv[2])
        return
    import fccf_amd as F
    from is_bench import leaf_keys
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    c = F.CONFIGS[os.environ.get("CFG", "c3")]
    src, _, _ = F.synth_pair(c["n"], c["room"])
    k = leaf_keys(src, c["leaf"])
    with F.Ctx(0) as ctx:
        for _ in range(reps):
            ctx.sort_keys(k)
        rd = ctx.sort_rounds()
        st = ctx.sort_stats()
    print("round  segments  tiles  owned_so_far  elements")
    for r, (ns, nt, no, el) in enumerate(rd):
        if ns or nt or no or el:
            print(f"{r:5d} {ns:9d} {nt:6d} {no:13d} {el:9d}")
    print({k: v for k, v in st.items() if k != "raw"}, "sort ns", int(st["raw"][31]))


if __name__ == "__main__":
    main()
