#!/bin/bash
# Dev: the batched sort in isolation (tools/sort_bench10.py) for the default library and
# variant libraries (lib_<name>), interleaved, with the per-kernel split at width 10.
# Usage (via gpurun): bash tools/gpu_sortvar.sh TAG name...   ("base" = lib/)
set -o pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then L=fccf-pcr_amd/lib/libfccf.so; else L=fccf-pcr_amd/lib_$v/libfccf.so; fi
  FCCF_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/kt_$v -o run -- python3 -u tools/sort_bench10.py 10 ${CHECK:+--check} > $OUT/sb_$v.log 2> $OUT/sb_$v.err || { tail -5 $OUT/sb_$v.err; cat $OUT/sb_$v.log; exit 1; }
  python3 tools/kt_batch.py $OUT/kt_$v $OUT/kd_$v.txt
  python3 tools/round_times.py $OUT/kt_$v 10 > $OUT/rt_$v.txt
  rm -rf $OUT/kt_$v
  echo "$v: $(tail -1 $OUT/sb_$v.log)"
  grep -E "y=10" $OUT/kd_$v.txt | head -5
done
