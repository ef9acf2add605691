set -o pipefail
STATS=0 PMC=1 bash tools/gpu_prof_r05.sh r05au > gpurun_out/r05au_prof.log 2>&1 || { tail -20 gpurun_out/r05au_prof.log; exit 1; }
mkdir -p profiles/r05au && cp gpurun_out/r05au/pmc/pmc_traffic.json profiles/r05au/pmc_traffic.json
timeout -k 10 400 python -u bench.py > gpurun_out/r05au/bench.json 2> gpurun_out/r05au/bench.err || { tail -30 gpurun_out/r05au/bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/r05au/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r05au/prof -o run -- python3 -u bench.py --no-cpu-baseline > gpurun_out/r05au/prof_bench.json 2> gpurun_out/r05au/prof.err
