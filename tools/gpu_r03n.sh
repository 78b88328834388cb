#!/bin/bash
# Round-3 pass N: per-group GEMM times in isolation (graph-replayed); graph-crash trigger variants (last).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_group_probe.py > gpurun_out/r03n_gemm_groups.jsonl 2> gpurun_out/r03n_gemm_groups.err || { tail -5 gpurun_out/r03n_gemm_groups.err; exit 3; }
cat gpurun_out/r03n_gemm_groups.jsonl
PROBE_OP=hip timeout -k 10 120 python -u tools/graph_edge_probe.py ping_pong > gpurun_out/r03n_graph_hipop.jsonl 2>&1
cat gpurun_out/r03n_graph_hipop.jsonl
timeout -k 10 60 ./tools/bin/graph_edge_repro ping_pong global autofree query > gpurun_out/r03n_graph_query.txt 2>&1
echo "hip ping_pong query rc=$?: $(tr '\n' ' ' < gpurun_out/r03n_graph_query.txt)"
exit 0
