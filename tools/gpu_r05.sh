#!/bin/bash
# Round-5 iteration on the GPU box (via gpurun): selected GPU tests, quick_perf (c3
# single + pipelined), and a bench line without the CPU baseline.
# Usage: bash tools/gpu_r05.sh <tag> [pytest targets...]   (TESTS=0 skips the tests)
set -o pipefail
TAG=${1:-r05}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
if [ "${TESTS:-1}" = 1 ]; then
  step tests
  T=${@:-tests}
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $OUT/pytest_gpu.log | head -20; exit $rc; }
fi
if [ "${QUICK:-1}" = 1 ]; then
  step quick
  timeout -k 10 300 python -u tools/quick_perf.py 20 > $OUT/quick.txt 2>&1 || { tail -20 $OUT/quick.txt; exit 1; }
  cat $OUT/quick.txt
fi
if [ "${BENCH:-1}" = 1 ]; then
  step bench
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --parity-configs= > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  python3 tools/bench_summary.py $OUT/bench.json 2>/dev/null | head -30
fi
echo done
