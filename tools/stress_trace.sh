#!/bin/bash
# Kernel-level breakdown of the M=4096 stress Cholesky (tools/chol_stress.py) under rocprofv3.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stress
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/chol_stress.py ${1:-4096} > $OUT/stress.log 2>&1
cat $OUT/stress.log
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
