#!/bin/bash
# Dev: K1/VoxelGrid/registration GPU tests, then c3 timing twice.
mkdir -p gpurun_out/quick
timeout -k 5 300 python -u -m pytest tests/test_gpu_introsort.py tests/test_gpu_voxelgrid.py tests/test_gpu_register.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/quick/tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/quick/tests.log; exit $rc; }
for rep in 1 2; do
  timeout -k 5 120 python -u tools/quick_perf.py > gpurun_out/quick/perf_$rep.log 2>&1 || exit 1
  echo "perf: $(tail -1 gpurun_out/quick/perf_$rep.log)"
done
