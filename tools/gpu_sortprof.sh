#!/bin/bash
# Dev: per-round sort durations and the finish kernels' SQ counters at the batch's width
# (ten clouds per launch), for one library (default lib/; FCCF_LIB to override).
# Usage (via gpurun): bash tools/gpu_sortprof.sh TAG [pmc]
set -o pipefail
TAG=${1:-sortprof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d $OUT/kt -o run -- python3 -u tools/pmc_batch.py c3 20 k_is_wave > $OUT/pb.json 2> $OUT/pb.err || { tail -5 $OUT/pb.err; exit 1; }
python3 tools/round_times.py $OUT/kt 10 | tee $OUT/round_times.txt
python3 tools/kt_batch.py $OUT/kt $OUT/kd.txt
rm -rf $OUT/kt
if [ "$2" = pmc ]; then
  i=0
  for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SCRATCH_LOAD_RETIRED SQ_INSTS_SCRATCH_STORE_RETIRED"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -f csv -d $OUT/p$i -o run -- python3 -u tools/pmc_batch.py c3 10 k_is_wave > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -5 $OUT/p$i.err; }
  done
  python3 tools/pmc_sq.py $OUT/p1 $OUT/p2 $OUT/p3 > $OUT/sq.txt
  grep -E "kernel|k_is_" $OUT/sq.txt | head -20
  rm -rf $OUT/p1 $OUT/p2 $OUT/p3
fi
