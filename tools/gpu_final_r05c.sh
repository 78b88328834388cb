#!/bin/bash
# Round-5 final evidence, part C: a quick gemm_big parity gate, the batched-product phase trace / probe, then
# part B (profiles + the default bench line) on the final code.
set -e
TAG=${1:-r05zz}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -x -q -k "big" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_big_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_big_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_big_tests.log
timeout -k 10 120 ./tools/big_trace_batch.x 256 1024 > gpurun_out/${TAG}_big_trace_batch.jsonl 2>&1 || { cat gpurun_out/${TAG}_big_trace_batch.jsonl; exit 1; }
cut -c1-240 gpurun_out/${TAG}_big_trace_batch.jsonl
timeout -k 10 240 python -u tools/big_probe.py > gpurun_out/${TAG}_big_probe.jsonl 2>&1 || { tail -20 gpurun_out/${TAG}_big_probe.jsonl; exit 1; }
grep variant gpurun_out/${TAG}_big_probe.jsonl | cut -c1-120
bash tools/gpu_final_r05b.sh $TAG
