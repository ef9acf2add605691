#!/bin/bash
# Dev: c3 timing vs the number of global partition rounds of K1's sort (FCCF_IS_ROUNDS).
mkdir -p gpurun_out/rounds
for r in 15 11 13 17 15; do
  FCCF_IS_ROUNDS=$r timeout -k 5 120 python -u tools/quick_perf.py > gpurun_out/rounds/r$r.log 2>&1 || exit 1
  echo "rounds=$r: $(tail -1 gpurun_out/rounds/r$r.log)"
done
