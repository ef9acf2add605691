#!/bin/bash
# Dev: A/B of development variant builds (make VAR=name) against the default library.
# Usage (via gpurun): bash tools/ab_variant.sh name [name...]
mkdir -p gpurun_out/var
for rep in 1 2; do
  timeout -k 5 120 python -u tools/quick_perf.py > gpurun_out/var/base_$rep.log 2>&1 || exit 1
  echo "base: $(tail -1 gpurun_out/var/base_$rep.log)"
  for v in "$@"; do
    FCCF_LIB=fccf-pcr_amd/lib_$v/libfccf.so timeout -k 5 120 python -u tools/quick_perf.py > gpurun_out/var/${v}_$rep.log 2>&1 || exit 1
    echo "$v: $(tail -1 gpurun_out/var/${v}_$rep.log)"
  done
done
for v in "$@"; do
  FCCF_LIB=fccf-pcr_amd/lib_$v/libfccf.so timeout -k 5 300 python -u -m pytest tests/test_gpu_introsort.py tests/test_gpu_register.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/var/${v}_tests.log 2>&1
  echo "$v tests rc=$?: $(tail -1 gpurun_out/var/${v}_tests.log)"
done
