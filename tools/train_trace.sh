#!/bin/bash
# Kernel breakdown of the HCP (configs[2]) and ECoG (configs[3]) training steps: one rocprofv3 --kernel-trace
# --stats pass of tools/train_leg.py per configuration (no counters), summarised per kernel per step by
# tools/train_summary.py -> gpurun_out/<tag>_{hcp,ecog}_train_kernels.json
set -e
TAG=${1:-r04}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/train_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for cfg in hcp ecog; do
  steps=10; [ $cfg = ecog ] && steps=2
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$cfg -o run -- python3 $R/tools/train_leg.py $cfg $steps > $OUT/$cfg.json 2> $OUT/$cfg.err || { tail -20 $OUT/$cfg.err; exit 1; }
  tail -1 $OUT/$cfg.json | cut -c1-300
  (cd $R && python3 tools/train_summary.py $(find $OUT/$cfg -name "*kernel_trace.csv") $OUT/$cfg.json gpurun_out/${TAG}_${cfg}_train_kernels.json)
done
