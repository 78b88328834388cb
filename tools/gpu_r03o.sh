#!/bin/bash
# Round-3 pass O: four-role Cholesky (separate update workgroup): bit identity vs three-role, timeline, A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_primitives.py -k "four_role" -q -x --timeout 100 --timeout-method thread > gpurun_out/r03o_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r03o_tests.log
[ $rc -ne 0 ] && exit $rc
NMGP_CHOL_4ROLE=1 timeout -k 10 60 ./tools/bin/chol4_probe 256 1 > gpurun_out/r03o_probe_4role.txt 2>&1 || exit $?
cat gpurun_out/r03o_probe_4role.txt
timeout -k 10 120 python -u tools/chol_ab.py 256:4:f64 256:1:f64 128:1:f32 128:8:f32 > gpurun_out/r03o_chol_ab.jsonl 2>&1 || exit $?
cat gpurun_out/r03o_chol_ab.jsonl
exit 0
