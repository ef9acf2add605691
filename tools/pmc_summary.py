"""Dev: mean PMC counter values per dispatch of the named kernels, from every
*counter_collection.csv under a rocprofv3 output directory.
Usage: python tools/pmc_summary.py <dir> <kernel substring> ..."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root, names):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            for n in names:
                if n in k:
                    acc[n][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for n in names:
        print(n)
        for c, v in sorted(acc[n].items()):
            print(f"   {c:24s} mean/dispatch {sum(v) / len(v):16.1f}  ({len(v)} rows)")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
