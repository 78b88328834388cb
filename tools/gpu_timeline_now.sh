#!/bin/bash
# Kernel trace of a short PM2.5 bench run + the per-step timeline (tools/step_timeline.py).  usage: bash tools/gpu_timeline_now.sh <tag>
TAG=${1:-now}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/tl_$TAG
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-stress --no-elbo --no-api --no-hcp --no-ecog --no-breakdown"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl_$TAG/trace -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/tl_$TAG/bench.json 2> $R/gpurun_out/tl_$TAG/trace.err || exit $?
cd $R
python3 tools/step_timeline.py $(find gpurun_out/tl_$TAG/trace -name "*kernel_trace.csv") > gpurun_out/tl_$TAG/timeline.txt 2>&1
head -1 gpurun_out/tl_$TAG/timeline.txt
