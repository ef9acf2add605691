#!/bin/bash
# Interleaved bench of several libfccf builds at one config (development).
# Usage (via gpurun): bash tools/gpu_ab_multi.sh <tag> <cfg> <reps> <steps> lib1.so lib2.so ...
TAG=$1; CFG=$2; REPS=$3; STEPS=$4; shift 4
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in $(seq 1 $REPS); do
  for L in "$@"; do
    FCCF_LIB=$L timeout -k 5 170 python -u bench.py --config $CFG --no-cpu-baseline --parity-configs= --steps $STEPS > $OUT/b.json 2> $OUT/b.err || { echo "run failed ($L)"; tail -3 $OUT/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/b.json')); kt=d['kernel_table']; print('$CFG', '$(basename $(dirname $L))', 'rep $rep', 'ms/step %.4f e2e %.4f vg_main %.3f' % (d['ms_per_step'], d['e2e_ms_median'], d['device_ms']['vg_main']), ' '.join('%s %.1f' % (k[5:], kt[k]['avg_launch_us']) for k in ('k_is_scatter','k_is_count_plan','k_is_block','k_is_wave') if k in kt))"
  done
done
