#!/bin/bash
# Dev: K1 sort with the plan folded into the count kernel vs the separate plan kernel.
mkdir -p gpurun_out/plan
timeout -k 5 300 python -u -m pytest tests/test_gpu_introsort.py tests/test_gpu_voxelgrid.py tests/test_gpu_register.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/plan/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/plan/tests.log)"; [ $rc -eq 0 ] || exit $rc
for v in fused sep fused sep; do
  if [ $v = sep ]; then export FCCF_IS_PLAN=1; else unset FCCF_IS_PLAN; fi
  timeout -k 5 120 python -u tools/quick_perf.py > gpurun_out/plan/$v.log 2>&1 || exit 1
  echo "$v: $(tail -1 gpurun_out/plan/$v.log)"
done
