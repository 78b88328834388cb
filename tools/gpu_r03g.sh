#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 120 python -u tests/analysis/p64_debug.py > gpurun_out/r03g_debug.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r03g_debug.log | cut -c1-6000
exit $rc
