#!/bin/bash
# Dev: interleaved quick_perf runs over several values of one environment variable.
# Usage (via gpurun): bash tools/ab_envs.sh VAR "v1 v2 ..." [rounds]
mkdir -p gpurun_out/abe
for i in $(seq ${3:-3}); do
  for v in $2; do
    env "$1=$v" timeout -k 10 120 python -u tools/quick_perf.py > gpurun_out/abe/$v.txt 2>&1 || { cat gpurun_out/abe/$v.txt; exit 1; }
    echo "$1=$v: $(tail -1 gpurun_out/abe/$v.txt)"
  done
done
