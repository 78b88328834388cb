#!/bin/bash
# Round-3 pass L: lookahead Cholesky with per-4-column table groups, early diagonal tile, setprio:
# bit-identity test vs the three-role kernel, timeline, A/B; predict plan tests; graph repro variants.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_primitives.py -k "lookahead or chol_inv" -q -x --timeout 100 --timeout-method thread > gpurun_out/r03l_chol_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03l_chol_tests.log
[ $rc -ne 0 ] && exit $rc
NMGP_CHOL_LA=1 timeout -k 10 60 ./tools/bin/chol4_probe 256 1 > gpurun_out/r03l_probe_la1_b1.txt 2>&1 || exit $?
cat gpurun_out/r03l_probe_la1_b1.txt
timeout -k 10 120 python -u tools/chol_ab.py 256:4:f64 256:1:f64 128:8:f32 > gpurun_out/r03l_chol_ab.jsonl 2>&1 || exit $?
cat gpurun_out/r03l_chol_ab.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_training_api.py -q -x -k "predict or test_lists" --timeout 200 --timeout-method thread > gpurun_out/r03l_pred_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03l_pred_tests.log
[ $rc -gt 1 ] && exit $rc
B="--no-elbo --no-hcp --no-ecog --no-stress --no-cpu-baseline --no-breakdown --steps 300"
for la in 1 0; do
  NMGP_CHOL_LA=$la timeout -k 10 200 python -u bench.py $B > gpurun_out/r03l_bench_la$la.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r03l_bench_la$la.json').read().strip().splitlines()[-1]);print('LA=$la', d['value'], d['ms_per_step'], json.dumps(d['api_path'])[:600])"
done
for v in "" "global" "autofree" "global autofree"; do
  timeout -k 10 60 ./tools/bin/graph_edge_repro ping_pong $v > gpurun_out/r03l_graph.txt 2>&1
  rcg=$?; echo "ping_pong [$v] rc=$rcg: $(tr '\n' ' ' < gpurun_out/r03l_graph.txt)"
  [ $rcg -ne 0 ] && break
done
PROBE_CAPTURE_MODE=thread_local timeout -k 10 120 python -u tools/graph_edge_probe.py ping_pong > gpurun_out/r03l_graph_edges_tl.jsonl 2>&1
cat gpurun_out/r03l_graph_edges_tl.jsonl
timeout -k 10 120 python -u tools/graph_edge_probe.py ping_pong > gpurun_out/r03l_graph_edges_gl.jsonl 2>&1
cat gpurun_out/r03l_graph_edges_gl.jsonl
exit 0
