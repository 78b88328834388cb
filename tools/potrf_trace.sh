#!/bin/bash
# Kernel trace of the blocked potrf / chol+inv stress runs (tools/chol_stress.py) for per-launch timing.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ptrace
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/chol_stress.py ${1:-1024} > $OUT/stress.log 2>&1
cat $OUT/stress.log
