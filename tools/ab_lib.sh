#!/bin/bash
# Dev: interleaved quick_perf of the default build and a variant build (lib_$1).
V=${1:-w9}
mkdir -p gpurun_out
for i in $(seq ${2:-3}); do
  timeout -k 10 120 python -u tools/quick_perf.py 20 > gpurun_out/ab_a.txt 2>&1 || { cat gpurun_out/ab_a.txt; exit 1; }
  echo "default: $(tail -1 gpurun_out/ab_a.txt)"
  FCCF_LIB=fccf-pcr_amd/lib_$V/libfccf.so timeout -k 10 120 python -u tools/quick_perf.py 20 > gpurun_out/ab_b.txt 2>&1 || { cat gpurun_out/ab_b.txt; exit 1; }
  echo "$V: $(tail -1 gpurun_out/ab_b.txt)"
done
