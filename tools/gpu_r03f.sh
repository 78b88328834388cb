#!/bin/bash
# Round-3 pass F: fp64 L0/L1 prior adjoints; fp64 path on by default; whole suite; bench; graph edge probe
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ecog.py tests/test_gpu_engine.py -k "fp32 or ecog or hcp" -v -s --timeout 300 --timeout-method thread > gpurun_out/r03f_fp32.log 2>&1
rc=$?; grep -E "PARITY|errors|passed|failed|FAILED|Error" gpurun_out/r03f_fp32.log | cut -c1-1500 | head -40
[ $rc -gt 1 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu --ignore=tests/test_gpu_ecog.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/r03f_suite.log 2>&1
rc2=$?; tail -6 gpurun_out/r03f_suite.log
[ $rc2 -gt 1 ] && exit $rc2
timeout -k 10 600 python -u bench.py > gpurun_out/r03f_bench.json 2> gpurun_out/r03f_bench.err
rc3=$?; tail -c 3000 gpurun_out/r03f_bench.json; [ $rc3 -ne 0 ] && { tail -20 gpurun_out/r03f_bench.err; exit $rc3; }
timeout -k 10 300 python -u tools/graph_edge_probe.py > gpurun_out/r03f_graph_edges.jsonl 2>&1
rc4=$?; cat gpurun_out/r03f_graph_edges.jsonl
exit $(( rc > rc2 ? rc : rc2 ))
