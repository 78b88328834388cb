#!/bin/bash
# Round-3 pass E: fp64 v sample + fp64 t-prior adjoints of the fp32 engine; whole GPU suite with NMGP_PROJ_FP64=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export NMGP_PROJ_FP64=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_ecog.py -v -s --timeout 600 --timeout-method thread > gpurun_out/r03e_ecog.log 2>&1
rc=$?; grep -E "PARITY|ecog full|passed|failed|FAILED|Error" gpurun_out/r03e_ecog.log | head -40
[ $rc -gt 1 ] && exit $rc
timeout -k 10 540 python -u -m pytest tests -m gpu --deselect tests/test_gpu_ecog.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/r03e_suite.log 2>&1
rc2=$?; tail -25 gpurun_out/r03e_suite.log
exit $(( rc > rc2 ? rc : rc2 ))
