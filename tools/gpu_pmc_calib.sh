#!/bin/bash
# PMC calibration: the request-size-bucketed L2->fabric counters
# (TCC_EA0_RDREQ_32B/64B/128B, TCC_EA0_WRREQ/_64B) beside FETCH_SIZE / WRITE_SIZE, over
# tools/pmc_calib (known bytes per access pattern) and over the bench command, one
# counter pass per process.  BATCH=1: the workload is tools/pmc_batch.py (pipelined
# batches only, eight clouds per launch: the timed region's shape) instead of single
# registrations of the bench command.
# Usage (via gpurun): [CFG=c3] [STEPS=5] [CALIB=0] [BENCH=0] [BATCH=1] bash tools/gpu_pmc_calib.sh <tag>
set -e
TAG=${1:-calib}
CFG=${CFG:-c3}
STEPS=${STEPS:-5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
P2="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
P5="TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_BUBBLE_sum"
if [ "${CALIB:-1}" = 1 ]; then
tools/pmc_calib > $OUT/calib_alg.txt
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --kernel-trace -f csv -d $OUT/calib_p$i -o run -- tools/pmc_calib > /dev/null 2> $OUT/calib_p$i.err
  echo "calib pass $i ok"
done
fi
[ "${BENCH:-1}" = 1 ] || exit 0
if [ "${BATCH:-0}" = 1 ]; then
  B="tools/pmc_batch.py $CFG $STEPS"
else
  B="bench.py --config $CFG --no-cpu-baseline --parity-configs= --no-pipeline --no-sharded --steps $STEPS --warmup 2"
fi
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace -f csv -d $OUT/bench_p$i -o run -- python3 -u $B > $OUT/bench_p$i.json 2> $OUT/bench_p$i.err
  ls $OUT/bench_p$i/*counter_collection.csv > /dev/null || { echo "bench pass $i: no counters"; exit 1; }
  echo "bench pass $i ok"
done
