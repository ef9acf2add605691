#!/bin/bash
# Dev: runtime blit kernels per registration (kernel trace of tools/blit_count.py:
# warm-up batch of 3, steady batch of N) and the centroid's PMC traffic.
# Usage (via gpurun): bash tools/gpu_blits.sh <tag>
TAG=${1:-blits}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 -u tools/blit_count.py 20 > $OUT/blit.log 2>&1 || { tail -5 $OUT/blit.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
c = {r["Name"]: int(r["Calls"]) for r in rows}
reg = 23  # 3 warm-up + 20 steady registrations
for k in sorted(c, key=lambda k: -c[k]):
    if "rocclr" in k: print(f"{k}: {c[k]} calls, {c[k] / reg:.2f} per registration (incl. uploads/warm-up)")
PY
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/fetch -o run -- python3 -u tools/blit_count.py 5 > $OUT/fetch.log 2>&1 || { tail -5 $OUT/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/write -o run -- python3 -u tools/blit_count.py 5 > $OUT/write.log 2>&1 || { tail -5 $OUT/write.log; exit 1; }
python3 tools/pmc_traffic.py $OUT/fetch $OUT/write $OUT/pmc_traffic.json 0.05 > /dev/null && python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); ks=d.get('kernels',d)
v=ks['k_vg_centroid']; print('k_vg_centroid MB/launch %.2f (fetch KB %.0f write KB %.0f)'%(v['hbm_bytes_per_launch']/1e6, v['FETCH_SIZE_KB_mean'], v['WRITE_SIZE_KB_mean']))" $OUT/pmc_traffic.json
