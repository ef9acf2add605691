#!/bin/bash
# Dev: interleaved tools/quick_perf.py runs, default against one environment setting.
# Usage: bash tools/ab_quick.sh VAR=VALUE [rounds]
mkdir -p gpurun_out
for i in $(seq ${2:-2}); do
  timeout -k 10 200 python -u tools/quick_perf.py 20 > gpurun_out/abq_a.txt 2>&1 || { cat gpurun_out/abq_a.txt; exit 1; }
  echo "default: $(tail -1 gpurun_out/abq_a.txt)"
  env "$1" timeout -k 10 200 python -u tools/quick_perf.py 20 > gpurun_out/abq_b.txt 2>&1 || { cat gpurun_out/abq_b.txt; exit 1; }
  echo "$1: $(tail -1 gpurun_out/abq_b.txt)"
done
