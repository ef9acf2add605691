#!/bin/bash
# HBM traffic per launch from two separate PMC passes over the bench command
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; MI355X_MICROARCH.md "HBM"),
# then the kernel-trace statistics of the same command.
# Usage (via gpurun): [CFG=c3] [STEPS=5] bash tools/gpu_pmc.sh <tag>
set -e
TAG=${1:-pmc}
CFG=${CFG:-c3}
STEPS=${STEPS:-5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --config $CFG --no-cpu-baseline --parity-configs= --steps $STEPS --warmup 2"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/fetch -o run -- python3 -u $B > $OUT/fetch.json 2> $OUT/fetch.err
echo "fetch pass ok"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/write -o run -- python3 -u $B > $OUT/write.json 2> $OUT/write.err
echo "write pass ok"
python3 tools/pmc_traffic.py $OUT/fetch $OUT/write $OUT/pmc_traffic.json ${PMC_MIN_FRAC:-0.05} && python3 -c "import json,sys; p=sys.argv[1]; d=json.load(open(p)); d[\"config\"]=sys.argv[2]; json.dump(d,open(p,\"w\"),indent=1)" $OUT/pmc_traffic.json $CFG
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats -o run -- python3 -u $B > $OUT/bench.json 2> $OUT/bench.err
echo "stats pass ok"
