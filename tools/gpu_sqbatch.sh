#!/bin/bash
# Dev: SQ counters per kernel over pipelined c3 batches (tools/pmc_batch.py), two passes.
# Usage (via gpurun): bash tools/gpu_sqbatch.sh TAG
OUT=gpurun_out/${1:-sqb}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -f csv -d $OUT/p$i -o run -- python3 -u tools/pmc_batch.py c3 5 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_sq.py $OUT/p1 $OUT/p2 > $OUT/sq.txt
rm -rf $OUT/p1 $OUT/p2
head -40 $OUT/sq.txt
