#!/bin/bash
# Round-3 pass H: fp64 prior adjoints (finalize fix); fp32 parity prints; whole suite; HIP-only graph-edge repro
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ecog.py tests/test_gpu_engine.py -k "fp32 or ecog or hcp" -v -s --timeout 300 --timeout-method thread > gpurun_out/r03h_fp32.log 2>&1
rc=$?; grep -E "PARITY|errors|passed|failed|FAILED|Error" gpurun_out/r03h_fp32.log | cut -c1-1600 | head -40
[ $rc -gt 1 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu --ignore=tests/test_gpu_ecog.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/r03h_suite.log 2>&1
rc2=$?; tail -6 gpurun_out/r03h_suite.log
[ $rc2 -gt 1 ] && exit $rc2
for p in one_way relay ping_pong; do
  timeout -k 10 60 ./tools/bin/graph_edge_repro $p > gpurun_out/r03h_graph_$p.txt 2>&1
  rcg=$?; echo "pattern $p rc=$rcg"; cat gpurun_out/r03h_graph_$p.txt
  [ $rcg -ne 0 ] && break
done
exit $(( rc > rc2 ? rc : rc2 ))
