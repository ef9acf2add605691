#!/bin/bash
# Interleaved A/B of two libfccf builds on the bench at one config (development).
# Usage (via gpurun): bash tools/gpu_ab_cfg.sh <tag> <cfg> <libA.so> <libB.so> [reps] [steps]
TAG=$1; CFG=$2; A=$3; B=$4; REPS=${5:-2}; STEPS=${6:-10}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in $(seq 1 $REPS); do
  for L in "$A" "$B"; do
    FCCF_LIB=$L timeout -k 5 170 python -u bench.py --config $CFG --no-cpu-baseline --parity-configs= --steps $STEPS > $OUT/b.json 2> $OUT/b.err || { echo "run failed ($L)"; tail -3 $OUT/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/b.json')); print('$CFG', '$(basename $(dirname $L))', 'rep $rep', 'ms/step %.4f e2e %.4f vg_main %.3f' % (d['ms_per_step'], d['e2e_ms_median'], d['device_ms']['vg_main']), 'scatter', d['kernel_table'].get('k_is_scatter',{}).get('avg_launch_us'), 'count', d['kernel_table'].get('k_is_count_plan',{}).get('avg_launch_us'))"
  done
done
