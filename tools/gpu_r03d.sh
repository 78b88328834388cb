#!/bin/bash
# Round-3 pass D: lookahead Cholesky probe/tests/A-B; fp64 projections of the fp32 engine (ECoG / HCP parity)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
NMGP_CHOL_LA=1 timeout -k 10 60 ./tools/bin/chol4_probe 256 4 > gpurun_out/r03d_probe.txt 2>&1 || exit $?
cat gpurun_out/r03d_probe.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -k "chol_inv or potrf_trtri" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03d_chol_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03d_chol_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/chol_ab.py 256:4:f64 256:1:f64 256:1:f32 128:8:f64 > gpurun_out/r03d_chol_ab.jsonl 2>&1 || exit $?
grep -v amdgpu gpurun_out/r03d_chol_ab.jsonl
NMGP_PROJ_FP64=1 timeout -k 10 200 python -u tests/analysis/ecog_fp32_diag.py > gpurun_out/r03d_ecog_diag.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r03d_ecog_diag.log
NMGP_PROJ_FP64=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_ecog.py tests/test_gpu_engine.py tests/test_gpu_distributed.py -k "fp32 or ecog or hcp or elbo" -v -s --timeout 900 --timeout-method thread > gpurun_out/r03d_tests.log 2>&1
rc=$?; grep -E "PARITY|passed|failed|FAILED|Error" gpurun_out/r03d_tests.log | head -40
exit $rc
