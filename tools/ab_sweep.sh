#!/bin/bash
# Dev: interleaved quick_perf over settings of one environment variable.
# Usage: bash tools/ab_sweep.sh VAR "v1 v2 ..." [rounds]   ("-" = unset)
mkdir -p gpurun_out
for i in $(seq ${3:-2}); do
  for v in $2; do
    if [ "$v" = "-" ]; then
      timeout -k 10 120 python -u tools/quick_perf.py > gpurun_out/ab_s.txt 2>&1 || { cat gpurun_out/ab_s.txt; exit 1; }
    else
      env "$1=$v" timeout -k 10 120 python -u tools/quick_perf.py > gpurun_out/ab_s.txt 2>&1 || { cat gpurun_out/ab_s.txt; exit 1; }
    fi
    echo "$1=$v: $(tail -1 gpurun_out/ab_s.txt)"
  done
done
