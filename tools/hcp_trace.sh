#!/bin/bash
# HCP-shaped step (tools/bench_configs.py hcp): plain timing, then a kernel-trace + stats pass.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/hcp
mkdir -p $OUT
timeout -k 10 300 python3 $R/tools/bench_configs.py ${CONFIGS:-hcp pm25f32 toy} > $OUT/configs.jsonl 2> $OUT/configs.err
cat $OUT/configs.jsonl | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/bench_configs.py hcp > $OUT/trace.log 2>&1
echo traced
