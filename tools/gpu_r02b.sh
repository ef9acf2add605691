#!/bin/bash
# Round-2 checkpoint: GPU parity tests, bench, kernel-trace stats, and (last, it may
# hang by design) the capture-race negative control.
# Usage (via gpurun): bash tools/gpu_r02b.sh <tag>
set -e
TAG=${1:-r02b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
python tools/bench_summary.py $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 -u bench.py --no-cpu-baseline --steps 10 > $OUT/prof_bench.json 2> $OUT/prof.err
echo "profile ok"
timeout -k 10 60 python -u tools/capture_race_unguarded.py > $OUT/unguarded.log 2>&1; echo "unguarded exit $?" >> $OUT/unguarded.log
cat $OUT/unguarded.log
