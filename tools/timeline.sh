#!/bin/bash
# Kernel timeline of one graph-replayed PM2.5 step (rocprofv3 kernel trace of bench.py; GPU box).
# usage: bash tools/timeline.sh <tag>   -> gpurun_out/tl_<tag>/run_kernel_trace.csv + timeline.txt
set -e
TAG=${1:-x}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/tl_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-breakdown --no-elbo --no-api > $OUT/b.json 2> $OUT/err.log
cd $R
python3 tools/step_timeline.py $(find $OUT -name "*kernel_trace.csv" | head -1) 1 > $OUT/timeline.txt
