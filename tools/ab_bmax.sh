#!/bin/bash
# Dev: interleaved tools/quick_perf.py runs of batch-width variant libraries
# (fccf-pcr_amd/lib_<name>/) at chosen pairs per stage.
# Usage: bash tools/ab_bmax.sh rounds "name:pp" ...   ("default:pp" = the in-tree library)
set -e
R=$1
shift
mkdir -p gpurun_out
for i in $(seq $R); do
  for cfg in "$@"; do
    n=${cfg%%:*}; pp=${cfg##*:}
    if [ "$n" = "default" ]; then lib=""; else lib="FCCF_LIB=fccf-pcr_amd/lib_$n/libfccf.so"; fi
    env $lib FCCF_PAIR_BATCH=$pp timeout -k 10 200 python -u tools/quick_perf.py 20 > gpurun_out/abb.txt 2>&1 || { cat gpurun_out/abb.txt; exit 1; }
    echo "$cfg: $(tail -1 gpurun_out/abb.txt)"
  done
done
