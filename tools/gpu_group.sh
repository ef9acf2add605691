#!/bin/bash
# Multi-GPU readiness on one GPU: the group tests (virtual ranks, the packed all-gather-v)
# and the c4 x 4 / c5 x 8 projection (tools/group_projection.py).
set -o pipefail
OUT=gpurun_out/${1:-grp}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_host_kat.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 500 python -u tools/group_projection.py > $OUT/projection.jsonl 2> $OUT/projection.err || { tail -20 $OUT/projection.err; exit 1; }
cat $OUT/projection.jsonl
