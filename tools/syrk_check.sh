#!/bin/bash
# Quick GPU pass for the large-tile GEMM / SYRK work: its parity tests, the SYRK probe, the stress Cholesky.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/syrk
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "gemm_big or chol_inv or potrf" > gpurun_out/syrk/tests.log 2>&1 || { tail -30 gpurun_out/syrk/tests.log; exit 1; }
tail -2 gpurun_out/syrk/tests.log
timeout -k 10 120 python3 tools/syrk_probe.py > gpurun_out/syrk/probe.jsonl 2> gpurun_out/syrk/probe.err
cat gpurun_out/syrk/probe.jsonl
timeout -k 10 120 python3 tools/chol_stress.py 4096 2048 1024 > gpurun_out/syrk/stress.log 2>&1
cat gpurun_out/syrk/stress.log
