#!/bin/bash
# rocprofv3 evidence for bench.py's roofline line (run on the GPU box from the repo root):
#   1. kernel trace + stats of the default bench command,
#   2./3. separate PMC passes for FETCH_SIZE and WRITE_SIZE (never combined with tracing domains),
#   4. tools/pmc_summary.py -> profiles/<prefix>_summary.json + _kernel_stats.csv.
# usage: bash tools/profile_bench.sh <prefix e.g. r01_pm25_bench>
set -e
PREFIX=${1:-r01_pm25_bench}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-stress --no-elbo --no-api --no-hcp --no-ecog --no-kron"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/bench_under_trace.json 2> $OUT/trace.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py $ARGS --no-breakdown > $OUT/bench_under_fetch.json 2> $OUT/fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py $ARGS --no-breakdown > $OUT/bench_under_write.json 2> $OUT/write.err
cd $R
python3 tools/pmc_summary.py $OUT/trace $OUT/fetch $OUT/write gpurun_out/$PREFIX
tail -1 $OUT/bench_under_trace.json > gpurun_out/${PREFIX}_under_rocprof.json
