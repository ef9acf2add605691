#!/bin/bash
# Finish-kernel grid sizes (FCCF_IS_GRID=ob,wb per cloud) on the c3 bench, interleaved.
OUT=gpurun_out/gridab
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-4}); do
  for G in ${GRIDS:-256,512 124,496 120,480}; do
    FCCF_IS_GRID=$G timeout -k 5 170 python -u bench.py --config ${CFG:-c3} --no-cpu-baseline --parity-configs= --steps ${STEPS:-40} > $OUT/b.json 2> $OUT/b.err || { echo "run failed"; tail -3 $OUT/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); kt=d['kernel_table']; b=d['stage_ms_in_batch']; print('grid $G rep $rep', 'ms/step %.4f e2e %.4f vg_main %.3f' % (d['ms_per_step'], d['e2e_ms_median'], d['device_ms']['vg_main']), 'block %.1f wave %.1f' % (kt['k_is_block']['avg_launch_us'], kt['k_is_wave']['avg_launch_us']), 'match_in_batch %.3f fine_in_batch %.3f' % (b['match'], b['fine']))"
  done
done
