#!/bin/bash
# Dev: per-variant kernel durations at the batch's width plus quick_perf timings.
# Usage (via gpurun): bash tools/gpu_var_kt.sh TAG name [name...]   (name "base" = lib/)
set -o pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then L=fccf-pcr_amd/lib/libfccf.so; else L=fccf-pcr_amd/lib_$v/libfccf.so; fi
  FCCF_LIB=$L timeout -k 5 150 python -u tools/quick_perf.py > $OUT/qp_$v.log 2>&1 || { tail -5 $OUT/qp_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/qp_$v.log)"
  FCCF_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d $OUT/kt_$v -o run -- python3 -u tools/pmc_batch.py c3 20 k_is_wave > $OUT/pb_$v.json 2> $OUT/pb_$v.err || { tail -5 $OUT/pb_$v.err; exit 1; }
  python3 tools/kt_batch.py $OUT/kt_$v $OUT/kd_$v.txt
  python3 tools/round_times.py $OUT/kt_$v 10 > $OUT/rt_$v.txt
  rm -rf $OUT/kt_$v
  grep -E "y=10" $OUT/kd_$v.txt | head -8
done
