#!/bin/bash
# Dev: quick_perf of the working build against older builds (tools/build_rev.sh), and
# the two pair-batch forms, interleaved.  Usage: bash tools/bisect_perf.sh "r03 b3" [rounds]
LIBS=${1:-r03}
N=${2:-2}
mkdir -p gpurun_out
for i in $(seq $N); do
  for L in $LIBS; do
    FCCF_LIB=fccf-pcr_amd/lib_$L/libfccf.so timeout -k 10 120 python -u tools/quick_perf.py > gpurun_out/bis_$L.txt 2>&1 || { tail -5 gpurun_out/bis_$L.txt; exit 1; }
    echo "$L: $(tail -1 gpurun_out/bis_$L.txt)"
  done
  timeout -k 10 120 python -u tools/quick_perf.py > gpurun_out/bis_head.txt 2>&1 || { tail -5 gpurun_out/bis_head.txt; exit 1; }
  echo "head pairs2: $(tail -1 gpurun_out/bis_head.txt)"
  FCCF_PAIR_BATCH=1 timeout -k 10 120 python -u tools/quick_perf.py > gpurun_out/bis_head1.txt 2>&1 || { tail -5 gpurun_out/bis_head1.txt; exit 1; }
  echo "head pairs1: $(tail -1 gpurun_out/bis_head1.txt)"
  if [ -n "$HEAD_ENV" ]; then  # one more variant of the working build, e.g. HEAD_ENV=FCCF_WAIT=sync
    env $HEAD_ENV timeout -k 10 120 python -u tools/quick_perf.py > gpurun_out/bis_headv.txt 2>&1 || { tail -5 gpurun_out/bis_headv.txt; exit 1; }
    echo "head $HEAD_ENV: $(tail -1 gpurun_out/bis_headv.txt)"
  fi
done
