# Dev: the rounds' two plan forms (FCCF_IS_PLAN=small|large) on the batched sort harness at ten
# clouds per launch, interleaved, with the per-round split.  Usage (via gpurun): bash tools/gpu_plan_ab10.sh
set -o pipefail
OUT=gpurun_out/pl1; mkdir -p $OUT; export TMPDIR=/tmp
for m in small large small large; do
  FCCF_IS_PLAN=$m timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/kt_$m -o run -- python3 -u tools/sort_bench10.py 10 --check > $OUT/sb_$m.log 2>&1 || { tail -5 $OUT/sb_$m.log; exit 1; }
  python3 tools/kt_batch.py $OUT/kt_$m $OUT/kd_$m.txt; python3 tools/round_times.py $OUT/kt_$m 10 > $OUT/rt_$m.txt; rm -rf $OUT/kt_$m
  echo "$m: $(tail -1 $OUT/sb_$m.log)"; grep -E "y=10" $OUT/kd_$m.txt | head -6
done
