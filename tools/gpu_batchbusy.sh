#!/bin/bash
# Dev: GPU occupancy and the stage timeline of one pipelined batch of 20 c3 registrations.
set -o pipefail
OUT=gpurun_out/${1:-bb}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d $OUT/kt -o run -- python3 -u tools/batch_busy.py run 20 > $OUT/run.log 2> $OUT/run.err || { tail -5 $OUT/run.err; exit 1; }
cat $OUT/run.log
python3 tools/batch_busy.py report $OUT/kt $OUT/batch_busy.txt > /dev/null; head -40 $OUT/batch_busy.txt
rm -rf $OUT/kt
