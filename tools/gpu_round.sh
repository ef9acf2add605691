#!/bin/bash
# One GPU session: the -m gpu suite, smoke, and a short bench; stops after a crash,
# abort or time limit (exit codes other than 0/1 from pytest).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -v --timeout 200 --timeout-method thread -m gpu ${PYTEST_ARGS} > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_all.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
exit $rc
