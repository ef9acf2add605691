"""Dev: print the kernel sequence (durations, gaps) of one registration window from a
rocprofv3 kernel trace.  Usage: python tools/trace_seq.py run_kernel_trace.csv [nth] [anchor]"""
import csv
import re
import sys


def short(n):
    n = n.replace('(anonymous namespace)::', '')
    n = (n[5:] if n.startswith('void ') else n).split('(')[0]
    return re.sub(r'.*::', '', n)[:26]


r = list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x: int(x['Start_Timestamp']))
nth = int(sys.argv[2]) if len(sys.argv) > 2 else 150
anchor = sys.argv[3] if len(sys.argv) > 3 else 'k_vg_bbox'
seq = [(short(x['Kernel_Name']), int(x['Start_Timestamp']), int(x['End_Timestamp']), x['Grid_Size_X'], x['Grid_Size_Y'],
        x['Workgroup_Size_X']) for x in r]
idx = [i for i, s in enumerate(seq) if s[0] == anchor]
a, b = idx[nth], idx[nth + 2] if nth + 2 < len(idx) else len(seq)
t0 = prev = seq[a][1]
for s in seq[a:b]:
    print(f"{s[0]:26s} {(s[2]-s[1])/1e3:8.2f} us  start+{(s[1]-t0)/1e3:8.1f}  gap {(s[1]-prev)/1e3:6.2f}  grid {s[3]}x{s[4]} wg {s[5]}")
    prev = max(prev, s[2])
