#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 60 ./tools/bin/chol4_probe 256 4 > gpurun_out/r03c_probe.txt 2>&1 || exit $?
NMGP_CHOL_LA=0 timeout -k 10 60 ./tools/bin/chol4_probe 256 4 | head -1 >> gpurun_out/r03c_probe.txt 2>&1 || exit $?
cat gpurun_out/r03c_probe.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -k "chol_inv or potrf_trtri" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03c_chol_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03c_chol_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/chol_ab.py 256:4:f64 256:1:f64 256:1:f32 128:8:f64 > gpurun_out/r03c_chol_ab.jsonl 2>&1 || exit $?
cat gpurun_out/r03c_chol_ab.jsonl | grep -v amdgpu
