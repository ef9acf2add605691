#!/bin/bash
# Exact-sum iteration on the GPU box: probe timings on dumped clouds + GPU tests.
# Usage (via gpurun): bash tools/gpu_xs.sh <tag>   (needs scratch/xs_probe, scratch/ds*.f32)
set -e
OUT=gpurun_out/xs_${1:-x}
mkdir -p $OUT
timeout -k 10 60 ./scratch/xs_probe scratch/ds1.f32 > $OUT/probe.txt 2>&1
timeout -k 10 60 ./scratch/xs_probe scratch/ds2.f32 >> $OUT/probe.txt 2>&1
cat $OUT/probe.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
