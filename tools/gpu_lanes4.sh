#!/bin/bash
OUT=gpurun_out/${1:-lanes4}
mkdir -p $OUT
for cfg in "conc 4" "lanes 4" "lanes 8" "conc 8" "lanes 16" "conc3 16" "lanes 8" "lanes 4"; do
  set -- $cfg
  echo -n "hwq=$2  " >> $OUT/probe.log
  GPU_MAX_HW_QUEUES=$2 FCCF_HOST_THREADS=4 timeout -k 10 120 python -u tools/lanes_probe.py $1 40 >> $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
done
cat $OUT/probe.log
