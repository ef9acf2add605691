#!/bin/bash
# One GPU-box validation pass: parity tests, bench, rocprofv3 kernel stats.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh <tag>
set -e
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "pytest ok"
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
echo "bench ok"; cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --no-cpu-baseline --steps 10 > $OUT/bench_prof.json 2> $OUT/prof.err
echo "rocprof ok"
