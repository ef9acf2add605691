#!/bin/bash
# Sort iteration (development): K1 sort parity tests first (they stop the run on a
# failure), then the registration parity tests and a bench line.
# Usage (via gpurun): bash tools/gpu_sort.sh <tag> [extra pytest -k expression]
TAG=${1:-s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_introsort.py tests/test_gpu_voxelgrid.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_sort.log 2>&1
rc=$?; echo "sort tests rc=$rc"; tail -4 $OUT/pytest_sort.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest_sort.log | head -20; exit $rc; fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-configs c2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"
if [ $rc -ne 0 ]; then tail -20 $OUT/bench.err; exit $rc; fi
python tools/bench_summary.py $OUT/bench.json
