#!/bin/bash
# Sort iteration (development): K1 sort parity tests, then the sort probe on c3.
# Usage (via gpurun): bash tools/gpu_sortquick.sh <tag> [round counts, default "10 14"]
TAG=${1:-sq}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_introsort.py tests/test_gpu_voxelgrid.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_sort.log 2>&1
rc=$?; echo "sort tests rc=$rc"; tail -2 $OUT/pytest_sort.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest_sort.log | head -20; exit $rc; fi
for R in ${2:-10 14}; do
  FCCF_IS_ROUNDS=$R timeout -k 10 200 python -u tools/is_bench.py c3 5 > $OUT/is_r$R.log 2>&1 || { cat $OUT/is_r$R.log; exit 1; }
  echo "rounds $R"; cat $OUT/is_r$R.log
done
FCCF_IS_TRACE_OUT=$OUT/trace_c3.txt timeout -k 10 200 python -u tools/is_bench.py c3 1 > $OUT/trace.log 2>&1 || { cat $OUT/trace.log; exit 1; }
python tools/sort_trace.py --analyze $OUT/trace_c3.txt
