# Dev: c4 / c5 bench lines of lib_head against the default build, interleaved.
set -o pipefail
mkdir -p gpurun_out/c45
for cfg in c4 c5; do
for v in head base head base; do
  if [ $v = base ]; then L=fccf-pcr_amd/lib/libfccf.so; else L=fccf-pcr_amd/lib_$v/libfccf.so; fi
  FCCF_LIB=$L timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --parity-configs= --no-sharded > gpurun_out/c45/${cfg}_$v.json 2> gpurun_out/c45/${cfg}_$v.err || { tail -5 gpurun_out/c45/${cfg}_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'ms/step %.3f' % d['ms_per_step'], 'e2e %.3f' % d['e2e_ms_median'], d['device_ms'], d.get('parity'))" gpurun_out/c45/${cfg}_$v.json $cfg $v
done
done
