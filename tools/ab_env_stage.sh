#!/bin/bash
# Dev: interleaved tools/stage_ms.py runs, default against one environment setting.
# Usage: bash tools/ab_env_stage.sh VAR=VALUE [rounds]
mkdir -p gpurun_out
for i in $(seq ${2:-3}); do
  timeout -k 10 120 python -u tools/stage_ms.py ${REPS:-30} > gpurun_out/abs_a.txt 2>&1 || { cat gpurun_out/abs_a.txt; exit 1; }
  echo "default: $(tail -2 gpurun_out/abs_a.txt | tr '\n' ' ')"
  env "$1" timeout -k 10 120 python -u tools/stage_ms.py ${REPS:-30} > gpurun_out/abs_b.txt 2>&1 || { cat gpurun_out/abs_b.txt; exit 1; }
  echo "$1: $(tail -2 gpurun_out/abs_b.txt | tr '\n' ' ')"
done
