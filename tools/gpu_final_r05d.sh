#!/bin/bash
# Round-5 final evidence in one call: a quick gemm_big parity gate, part B (profiles incl. the fp32 legs' traffic
# passes, then the default bench line), then part A (the whole GPU suite and smoke).
set -e
TAG=${1:-r05zz}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -x -q -k "big" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_big_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_big_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_big_tests.log
bash tools/gpu_final_r05b.sh $TAG
bash tools/gpu_final_r05a.sh $TAG
