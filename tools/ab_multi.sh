#!/bin/bash
# Dev: interleaved tools/quick_perf.py runs of several environment settings.
# Usage: bash tools/ab_multi.sh rounds "VAR=V ..." "VAR=V ..." ...   ("-" = the defaults)
R=$1
shift
mkdir -p gpurun_out
for i in $(seq $R); do
  for cfg in "$@"; do
    if [ "$cfg" = "-" ]; then e=""; else e="$cfg"; fi
    env $e timeout -k 10 200 python -u tools/quick_perf.py 20 > gpurun_out/abm.txt 2>&1 || { cat gpurun_out/abm.txt; exit 1; }
    echo "$cfg: $(tail -1 gpurun_out/abm.txt)"
  done
done
