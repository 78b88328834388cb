#!/bin/bash
# HBM traffic of the HCP (configs[2]) and ECoG (configs[3]) training steps: separate rocprofv3 PMC passes for
# FETCH_SIZE and WRITE_SIZE of tools/train_leg.py per configuration (no tracing domains), summarised by
# tools/train_traffic.py -> gpurun_out/<tag>_{hcp,ecog}_train_traffic.json
set -e
TAG=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/trainpmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for cfg in hcp ecog; do
  steps=4; [ $cfg = ecog ] && steps=1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$cfg/$c -o run -- python3 $R/tools/train_leg.py $cfg $steps > $OUT/${cfg}_$c.json 2> $OUT/${cfg}_$c.err || { tail -20 $OUT/${cfg}_$c.err; exit 1; }
  done
  (cd $R && python3 tools/train_traffic.py $(find $OUT/$cfg/FETCH_SIZE -name "*counter_collection.csv") $(find $OUT/$cfg/WRITE_SIZE -name "*counter_collection.csv") $OUT/${cfg}_FETCH_SIZE.json gpurun_out/${TAG}_${cfg}_train_traffic.json)
done
