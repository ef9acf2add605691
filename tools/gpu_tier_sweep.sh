#!/bin/bash
# Dev: c3 bench under K1 sort tier / round-count variants (FCCF_IS_TIER, FCCF_IS_ROUNDS).
# Usage (via gpurun): bash tools/gpu_tier_sweep.sh <tag> "tier:rounds ..."
TAG=${1:-tier}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in ${2:-4096:15 8192:13 8192:14 8192:15}; do
  T=${v%%:*}; R=${v##*:}
  FCCF_IS_TIER=$T FCCF_IS_ROUNDS=$R timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --parity-configs= > $OUT/b_${T}_${R}.json 2> $OUT/b_${T}_${R}.err || { tail -5 $OUT/b_${T}_${R}.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'ms/step %.4f'%d['ms_per_step'], 'vg_main %.4f'%d['device_ms']['vg_main'], d['parity'])" $OUT/b_${T}_${R}.json $v
done
