#!/bin/bash
# Dev: interleaved quick_perf with two pairs per cloud stage (default) and one (FCCF_PAIR_BATCH=1).
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/quick_perf.py > gpurun_out/ab_a.txt 2>&1 || { cat gpurun_out/ab_a.txt; exit 1; }
  echo "pairs2: $(tail -1 gpurun_out/ab_a.txt)"
  FCCF_PAIR_BATCH=1 timeout -k 10 120 python -u tools/quick_perf.py > gpurun_out/ab_b.txt 2>&1 || { cat gpurun_out/ab_b.txt; exit 1; }
  echo "pairs1: $(tail -1 gpurun_out/ab_b.txt)"
done
