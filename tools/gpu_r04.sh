#!/bin/bash
# Round-4 checkpoint (via gpurun): GPU tests, pair-batch A/B, bench lines (c3 with the
# CPU baseline; c4, c5), rocprofv3 kernel stats of the c3 bench, PMC calibration and the
# size-bucketed PMC passes of the c3 bench.  Usage: bash tools/gpu_r04.sh <tag> [steps]
set -o pipefail
TAG=${1:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; exit $rc; }
step ab
bash tools/ab_pairs.sh | tee $OUT/ab_pairs.log || exit 1
step bench_c3
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json 2>/dev/null | head -20
for cfg in c4 c5; do
  step bench_$cfg
  timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --parity-configs= > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { tail -20 $OUT/bench_$cfg.err; exit 1; }
done
step stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats -o run -- python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --parity-configs= > $OUT/stats_bench.json 2> $OUT/stats.err || { tail -5 $OUT/stats.err; exit 1; }
step pmc
BENCH=1 STEPS=5 bash tools/gpu_pmc_calib.sh $TAG/pmc || exit 1
python3 tools/pmc_calib.py $OUT/pmc $OUT/pmc/pmc_calib.json
python3 tools/pmc_traffic.py $OUT/pmc c3 $OUT/pmc/pmc_traffic.json > $OUT/pmc/pmc_traffic.txt
rm -rf $OUT/pmc/bench_p? $OUT/pmc/calib_p? $OUT/stats/run_kernel_trace.csv  # (gpurun returns at most 64 MiB)
echo done
