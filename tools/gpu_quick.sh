#!/bin/bash
# Quick GPU iteration: parity tests, segment timing, bench without CPU baseline.
# Usage (via gpurun): bash tools/gpu_quick.sh <tag>
set -e
TAG=${1:-q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
FCCF_SEG_TIMING=1 timeout -k 10 120 python -u scratch/hosttrace.py > $OUT/seg.txt 2>&1
tail -4 $OUT/seg.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms/step',d['ms_per_step'],'e2e',d['e2e_ms_median']);print(d['stage_ms']);print(d.get('stage_ms_in_batch'));print(d['roofline'])"
