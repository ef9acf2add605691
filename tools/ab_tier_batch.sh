#!/bin/bash
# Dev: K1's round tier (FCCF_IS_TIER: segments longer than this go through the rounds)
# swept at the pipelined batch's width, interleaved with the default.
# Usage (via gpurun): bash tools/ab_tier_batch.sh [tiers...]
mkdir -p gpurun_out/tier
for rep in 1 2; do
  for t in 4096 ${@:-2048 1024}; do
    FCCF_IS_TIER=$t timeout -k 10 120 python -u tools/quick_perf.py 20 > gpurun_out/tier/t${t}_$rep.txt 2>&1 || { tail -5 gpurun_out/tier/t${t}_$rep.txt; exit 1; }
    echo "tier $t: $(tail -1 gpurun_out/tier/t${t}_$rep.txt)"
  done
done
