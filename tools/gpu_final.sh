#!/bin/bash
# Round checkpoint: PMC traffic first (copied under profiles/<tag>/ so the bench's
# roofline object reads it), then the -m gpu suite, smoke, bench and kernel stats.
# Usage (via gpurun): bash tools/gpu_final.sh <tag>
TAG=${1:-final}
PMC_MIN_FRAC=0.0 bash tools/gpu_pmc.sh ${TAG}_pmc > gpurun_out/${TAG}_pmc.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc.log; exit 1; }
mkdir -p profiles/$TAG && cp gpurun_out/${TAG}_pmc/pmc_traffic.json profiles/$TAG/pmc_traffic.json
bash tools/gpu_ckpt.sh $TAG
