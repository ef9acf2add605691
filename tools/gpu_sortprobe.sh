#!/bin/bash
# Sort probe (development): device time of K1's sort on the c3 (and c5) first-pass
# keys for several round counts, and a per-item trace of the default build.
# Usage (via gpurun): bash tools/gpu_sortprobe.sh <tag> [round counts, default "10 14 17"]
TAG=${1:-sp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for R in ${2:-10 14 17}; do
  FCCF_IS_ROUNDS=$R timeout -k 10 200 python -u tools/is_bench.py c3 5 > $OUT/is_r$R.log 2>&1 || { cat $OUT/is_r$R.log; exit 1; }
  echo "rounds $R"; cat $OUT/is_r$R.log
done
FCCF_IS_TRACE_OUT=$OUT/trace_c3.txt timeout -k 10 200 python -u tools/is_bench.py c3 1 > $OUT/trace.log 2>&1 || { cat $OUT/trace.log; exit 1; }
python tools/sort_trace.py --analyze $OUT/trace_c3.txt
timeout -k 10 200 python -u tools/is_bench.py c5 3 > $OUT/is_c5.log 2>&1 || { cat $OUT/is_c5.log; exit 1; }
cat $OUT/is_c5.log
