#!/bin/bash
# GPU checkpoint: -m gpu suite, smoke, bench (with CPU baseline), kernel-trace stats.
# Every GPU step has its own time limit; the script stops at the first failure.
# Usage (via gpurun): bash tools/gpu_ckpt.sh <tag> [pytest -k expr]
TAG=${1:-ckpt}
KEXPR=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then KARGS=(-k "$KEXPR"); else KARGS=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${KARGS[@]}" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then tail -60 $OUT/pytest_gpu.log; exit $rc; fi
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"
if [ $rc -ne 0 ]; then tail -30 $OUT/bench.err; exit $rc; fi
python tools/bench_summary.py $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 -u bench.py --no-cpu-baseline --steps 10 > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; echo "rocprof rc=$rc"
exit $rc
