#!/bin/bash
# Critical path of one c3 registration (tools/critical_path.py) into gpurun_out/<tag>/.
# Usage: bash tools/gpu_cp.sh <tag>
OUT=gpurun_out/${1:-cp}
mkdir -p $OUT
export TMPDIR=/tmp
FCCF_HOST_TRACE=1 timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d $OUT/cp -o run -- python3 tools/critical_path.py run 8 2> $OUT/host.log > $OUT/run.txt || { tail $OUT/host.log; exit 1; }
python3 tools/critical_path.py report $OUT/cp $OUT/host.log $OUT/critical_path.txt > /dev/null || exit 1
rm -rf $OUT/cp
head -20 $OUT/critical_path.txt
cat $OUT/run.txt
