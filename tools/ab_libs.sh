#!/bin/bash
# Dev: interleaved tools/quick_perf.py runs of the default build and variant builds.
# Usage: bash tools/ab_libs.sh rounds name1 [name2 ...]   (fccf-pcr_amd/lib_<name>/)
R=$1
shift
mkdir -p gpurun_out
for i in $(seq $R); do
  timeout -k 10 200 python -u tools/quick_perf.py 20 > gpurun_out/abl.txt 2>&1 || { cat gpurun_out/abl.txt; exit 1; }
  echo "default: $(tail -1 gpurun_out/abl.txt)"
  for v in "$@"; do
    FCCF_LIB=fccf-pcr_amd/lib_$v/libfccf.so timeout -k 10 200 python -u tools/quick_perf.py 20 > gpurun_out/abl.txt 2>&1 || { cat gpurun_out/abl.txt; exit 1; }
    echo "$v: $(tail -1 gpurun_out/abl.txt)"
  done
done
