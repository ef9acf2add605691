#!/bin/bash
# Round-6 roofline evidence (via gpurun): rocprofv3 kernel stats of the
# exact bench command, per-kernel durations split by launch width (Grid_Size_Y = clouds per
# launch), and the size-bucketed PMC traffic passes over tools/pmc_batch.py (pipelined
# batches only: ten clouds per launch, the timed region's shape).
# Usage: bash tools/gpu_prof_r06.sh <tag> [STATS=1] [PMC=1]
set -o pipefail
TAG=${1:-r06final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
if [ "${STATS:-1}" = 1 ]; then
  step stats
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats -o run -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --parity-configs= > $OUT/bench_under_rocprof.json 2> $OUT/stats.err || { tail -5 $OUT/stats.err; exit 1; }
  python3 tools/kt_batch.py $OUT/stats $OUT/kernel_durations_by_width.txt
  cp $OUT/stats/run_kernel_stats.csv $OUT/kernel_stats.csv 2>/dev/null || find $OUT/stats -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
  head -12 $OUT/kernel_durations_by_width.txt
  rm -f $OUT/stats/*kernel_trace.csv
fi
if [ "${PMC:-1}" = 1 ]; then
  step pmc
  CALIB=0 BATCH=1 STEPS=${STEPS:-10} bash tools/gpu_pmc_calib.sh $TAG/pmc || exit 1
  cp $OUT/pmc/bench_p1.json $OUT/pmc/pmc_batch_p1.json
  python3 tools/pmc_traffic.py $OUT/pmc c3 $OUT/pmc/pmc_traffic.json 0.05 10 > $OUT/pmc/pmc_traffic.txt
  cat $OUT/pmc/pmc_traffic.txt | head -12
  rm -rf $OUT/pmc/bench_p?
fi
if [ "${DRAM:-1}" = 1 ]; then
  # the L2 read requests that went to DRAM (not served by the memory-side cache) beside
  # all L2 read requests, per kernel of the same pipelined batches
  step dram
  timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum --kernel-trace -f csv -d $OUT/dram -o run -- python3 -u tools/pmc_batch.py c3 ${STEPS:-10} > $OUT/dram.json 2> $OUT/dram.err || { tail -5 $OUT/dram.err; exit 1; }
  python3 tools/pmc_sq.py $OUT/dram > $OUT/dram_requests.txt
  head -8 $OUT/dram_requests.txt
  rm -rf $OUT/dram
fi
echo done
