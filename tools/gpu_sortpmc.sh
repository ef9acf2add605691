#!/bin/bash
# Dev: SQ / SQC counters of the batched sort in isolation (tools/sort_bench10.py, ten
# copies of a c3 cloud per launch), one pass per counter set, per library variant.
# Usage (via gpurun): bash tools/gpu_sortpmc.sh TAG name...   ("base" = lib/)
# SETS="A B;C D" replaces the SQ/SQC counter sets (one pass per ';'-separated set),
# e.g. SETS="FETCH_SIZE;WRITE_SIZE" for the memory-side bytes.
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then L=fccf-pcr_amd/lib/libfccf.so; else L=fccf-pcr_amd/lib_$v/libfccf.so; fi
  i=0
  D=""
  SETS=${SETS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS;SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_VMEM_RD;SQC_ICACHE_REQ SQC_ICACHE_MISSES"}
  IFS=';' read -ra PASSES <<< "$SETS"
  for P in "${PASSES[@]}"; do
    i=$((i+1))
    FCCF_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -f csv -d $OUT/${v}_p$i -o run -- python3 -u tools/sort_bench10.py 3 > $OUT/${v}_p$i.log 2>&1 || { echo "$v pass $i failed"; tail -3 $OUT/${v}_p$i.log; exit 1; }
    D="$D $OUT/${v}_p$i"
  done
  python3 tools/pmc_sq.py $D > $OUT/sq_$v.txt
  rm -rf $D
  echo "== $v"
  grep -E "^(kernel|k_is_wave|k_is_block|k_is_scatter_s|k_is_count_plan_s) " $OUT/sq_$v.txt
done
