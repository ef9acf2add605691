#!/bin/bash
# Dev: c3 timing vs K1's round threshold (FCCF_IS_TIER) and round count (FCCF_IS_ROUNDS).
mkdir -p gpurun_out/tier
for tr in 4096:15 8192:14 8192:13 8192:15 6144:14 6144:15 2048:16 2048:17 4096:15; do
  t=${tr%:*}; r=${tr#*:}
  FCCF_IS_TIER=$t FCCF_IS_ROUNDS=$r timeout -k 5 120 python -u tools/quick_perf.py > gpurun_out/tier/t${t}_r$r.log 2>&1 || { tail -5 gpurun_out/tier/t${t}_r$r.log; exit 1; }
  echo "tier=$t rounds=$r: $(tail -1 gpurun_out/tier/t${t}_r$r.log)"
done
