#!/bin/bash
# SQ / SQC counters of the sort kernels (c3 bench, few steps), separate passes.
OUT=gpurun_out/${1:-sqpmc}
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --config ${CFG:-c3} --no-cpu-baseline --parity-configs= --steps 3 --warmup 1 --no-pipeline"
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
         "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -f csv -d $OUT/p$i -o run -- python3 -u $B > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -5 $OUT/p$i.err; }
done
python3 tools/pmc_sq.py $OUT/p1 $OUT/p2 $OUT/p3 > $OUT/sq.txt; cat $OUT/sq.txt | head -30
