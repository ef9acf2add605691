#!/bin/bash
# Dev: interleaved tools/stage_ms.py runs of the default build and a variant (lib_$1).
V=${1:-head}
mkdir -p gpurun_out
for i in $(seq ${2:-3}); do
  timeout -k 10 150 python -u tools/stage_ms.py ${REPS:-60} > gpurun_out/abls_a.txt 2>&1 || { cat gpurun_out/abls_a.txt; exit 1; }
  echo "default: $(tail -1 gpurun_out/abls_a.txt)"
  FCCF_LIB=fccf-pcr_amd/lib_$V/libfccf.so timeout -k 10 150 python -u tools/stage_ms.py ${REPS:-60} > gpurun_out/abls_b.txt 2>&1 || { cat gpurun_out/abls_b.txt; exit 1; }
  echo "$V: $(tail -1 gpurun_out/abls_b.txt)"
done
