#!/bin/bash
# Dev: c4 / c5 pipelined benches (10 registrations) at the default pairs per stage and at
# FCCF_PAIR_BATCH=$PP_ALT (default 4), one after the other.
# Usage (via gpurun): bash tools/gpu_c45.sh <tag>
TAG=${1:-c45}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for c in c4 c5; do
  for pp in default ${PP_ALT:-4}; do
    if [ $pp = default ]; then e=""; else e="FCCF_PAIR_BATCH=$pp"; fi
    env $e timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --parity-configs= > $OUT/bench_${c}_$pp.json 2> $OUT/bench_${c}_$pp.err || { tail -20 $OUT/bench_${c}_$pp.err; exit 1; }
    echo "$c pp=$pp: $(python tools/bench_summary.py $OUT/bench_${c}_$pp.json 2>/dev/null | head -1)"
  done
done
