#!/bin/bash
# Dev: interleaved default bench runs (no CPU baseline, no parity configs) of the in-tree
# library and variant libraries (fccf-pcr_amd/lib_<name>/); prints ms/step per run.
# Usage: bash tools/ab_bench.sh rounds name1 [name2 ...]
R=$1
shift
mkdir -p gpurun_out
for i in $(seq $R); do
  for v in default "$@"; do
    if [ "$v" = default ]; then lib=""; else lib="FCCF_LIB=fccf-pcr_amd/lib_$v/libfccf.so"; fi
    env $lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --parity-configs= > gpurun_out/abbench.json 2> gpurun_out/abbench.err || { tail -20 gpurun_out/abbench.err; exit 1; }
    echo "$v: $(python tools/bench_summary.py gpurun_out/abbench.json | head -1)"
  done
done
