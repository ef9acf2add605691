#!/bin/bash
# Interleaved A/B of two libfccf builds on the bench (development).
# Usage (via gpurun): bash tools/gpu_ab_lib.sh <tag> <libA.so> <libB.so> [reps]
TAG=$1; A=$2; B=$3; REPS=${4:-3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in $(seq 1 $REPS); do
  for L in "$A" "$B"; do
    FCCF_LIB=$L timeout -k 5 90 python -u bench.py --no-cpu-baseline --steps 40 > $OUT/b.json 2> $OUT/b.err || { echo "run failed ($L)"; tail -3 $OUT/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/b.json')); print('$(basename $(dirname $L))', 'rep $rep', 'ms/step %.4f e2e %.4f' % (d['ms_per_step'], d['e2e_ms_median']))"
  done
done
