#!/bin/bash
# Round-end evidence pass: GPU tests + smoke + default bench line + kernel trace / FETCH / WRITE passes +
# MFMA-busy PMC pass for the PM2.5 step.  usage: bash tools/gpu_final.sh <profile prefix>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_check.sh $1
bash tools/pm25_pmc.sh
cp gpurun_out/pm25pmc/pm25_mfma.json gpurun_out/${1}_mfma_src.json
