#!/bin/bash
# Segment timing of the cloud stage (FCCF_SEG_TIMING) + per-stage ms at c3 and c5,
# after the parity tests.  Usage (via gpurun): bash tools/gpu_seg.sh <tag>
set -e
TAG=${1:-seg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for cfg in c3 c5; do
  FCCF_SEG_TIMING=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-pipeline --steps 8 --config $cfg > $OUT/bench_$cfg.json 2> $OUT/seg_$cfg.err
  python tools/bench_summary.py $OUT/bench_$cfg.json | head -3
  tail -4 $OUT/seg_$cfg.err
done
