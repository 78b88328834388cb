#!/bin/bash
# f32 multi-role Cholesky check: GPU suite, stress potrf / chol+inv and f32 configs, each with the f32
# role kernels on (default) and off (NMGP_CHOL_F32_ROLES=0).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
tail -2 gpurun_out/gpu_tests.log
for v in 1 0; do
  echo "NMGP_CHOL_F32_ROLES=$v"
  NMGP_CHOL_F32_ROLES=$v timeout -k 10 200 python -u tools/chol_stress.py 4096 > gpurun_out/stress_$v.log 2>&1
  grep -E "float32" gpurun_out/stress_$v.log
  NMGP_CHOL_F32_ROLES=$v timeout -k 10 300 python -u tools/bench_configs.py pm25f32 hcp > gpurun_out/cfg_$v.log 2>&1
  grep -o '"config": "[a-z0-9]*", "metric": "[^"]*", "value": [0-9.]*' gpurun_out/cfg_$v.log
done
