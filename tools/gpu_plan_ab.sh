#!/bin/bash
# K1 round form at one config: large (default >= IS_LARGE_MIN) against small (FCCF_IS_PLAN=small), interleaved.
# Usage (via gpurun): bash tools/gpu_plan_ab.sh <tag> <cfg> [reps] [steps]
TAG=$1; CFG=$2; REPS=${3:-2}; STEPS=${4:-8}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for PL in large small; do
    FCCF_IS_PLAN=$PL timeout -k 5 170 python -u bench.py --config $CFG --no-cpu-baseline --parity-configs= --steps $STEPS > $OUT/b.json 2> $OUT/b.err || { echo "run failed ($PL)"; tail -3 $OUT/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$CFG $PL rep $rep', 'ms/step %.4f vg_main %.3f' % (d['ms_per_step'], d['device_ms']['vg_main']))"
  done
done
