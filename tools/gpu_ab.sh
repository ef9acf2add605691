#!/bin/bash
# A/B of environment settings on the bench (development).  Usage (via gpurun):
#   bash tools/gpu_ab.sh <tag> "VAR=a" "VAR=b" ...
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for kv in "$@"; do
  for rep in 1 2; do
    env $kv timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 30 > $OUT/b.json 2> $OUT/b.err
    python3 -c "import json,sys; d=json.load(open('$OUT/b.json')); print('$kv', 'rep $rep', 'ms/step %.4f e2e %.4f' % (d['ms_per_step'], d['e2e_ms_median']), {k: v for k, v in d['stage_ms'].items() if v})"
  done
done
