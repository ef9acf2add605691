#!/bin/bash
# Sort PMC passes (development): SQ counters of the K1 sort kernels on the c3 keys.
# Usage (via gpurun): bash tools/gpu_sortpmc.sh <tag>
TAG=${1:-spmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp FCCF_IS_ROUNDS=${FCCF_IS_ROUNDS:-14}
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
P2="SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o pmc --output-format csv -- python3 tools/is_bench.py c3 2 > $OUT/p$i.log 2>&1 || { tail -20 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT k_is_item k_is_scatter k_is_count_plan
