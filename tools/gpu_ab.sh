#!/bin/bash
# Dev A/B: bench lines of the default library and a variant (FCCF_LIB=lib_<var>) at the
# given configs.  Usage (via gpurun): bash tools/gpu_ab.sh <tag> <var> "c3 c5"
TAG=${1:-ab}; VAR=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in ${3:-c3 c5}; do
  for lib in default $VAR; do
    L=""; [ "$lib" != default ] && L="FCCF_LIB=$PWD/fccf-pcr_amd/lib_$lib/libfccf.so"
    env $L timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --parity-configs= > $OUT/${cfg}_$lib.json 2> $OUT/${cfg}_$lib.err || { tail -5 $OUT/${cfg}_$lib.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); kt=dict(d['kernel_table'])
print(sys.argv[2], sys.argv[3], 'ms/step %.3f'%d['ms_per_step'], 'vg_main %.3f'%d['device_ms']['vg_main'], d['parity'], ' '.join('%s %.1f'%(k[5:],v['avg_launch_us']) for k,v in kt.items() if k.startswith('k_is_')))" $OUT/${cfg}_$lib.json $cfg $lib
  done
done
