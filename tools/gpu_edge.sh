#!/bin/bash
# Sort edge behaviour (via gpurun): the sort parity tests, the adversary timings, then
# the same sort tests once against the workgroup-fence variant (make VAR=wgf
# EXTRA=-DIS_WG_FENCE, lib_wgf/).  Usage: bash tools/gpu_edge.sh <tag>
TAG=${1:-edge}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp

timeout -k 10 300 python -u -m pytest tests/test_gpu_introsort.py tests/test_gpu_voxelgrid.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_sort.log 2>&1
rc=$?; echo "sort tests rc=$rc"; tail -2 $OUT/pytest_sort.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest_sort.log | head -20; exit $rc; fi
timeout -k 10 400 python -u tools/adversary_bench.py ${2:-20000 65536 262144 1048576} > $OUT/adversary.log 2>&1
rc=$?; echo "adversary rc=$rc"; cat $OUT/adversary.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
FCCF_LIB=$PWD/fccf-pcr_amd/lib_wgf/libfccf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_introsort.py tests/test_gpu_voxelgrid.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/pytest_sort_wgfence.log 2>&1
echo "workgroup-fence variant sort tests rc=$?"; tail -3 $OUT/pytest_sort_wgfence.log
