#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -x -q --timeout 120 --timeout-method thread > gpurun_out/prim_tests.log 2>&1
tail -1 gpurun_out/prim_tests.log
for v in 1 0 1; do
  NMGP_POTRF_LEAF_ROLES=$v timeout -k 10 200 python -u tools/chol_stress.py 4096 > gpurun_out/stress_leaf_$v.log 2>&1
  echo "LEAF_ROLES=$v: $(grep -E 'float32  potrf' gpurun_out/stress_leaf_$v.log | tr '\n' ' ')"
done
