#!/bin/bash
# Dev: the sort's parity tests on the default library, then interleaved kernel timings
# against variant libraries (lib_<name>).  Usage (via gpurun): bash tools/gpu_ab_sort.sh TAG name...
set -o pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_introsort.py tests/test_gpu_sorted_points.py tests/test_gpu_register.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/gpu_var_kt.sh $TAG "$@" base "$@" base
