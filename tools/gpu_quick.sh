#!/bin/bash
# Quick GPU iteration: parity tests, then the bench without the CPU baseline.
# Usage (via gpurun): bash tools/gpu_quick.sh <tag>
set -e
TAG=${1:-q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
python tools/bench_summary.py $OUT/bench.json
