#!/bin/bash
# Round-3 pass M: 16-column pivot-chain microbenchmark; P-bar on the latency kernel A/B; graph-crash trigger.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 60 ./tools/bin/chol16_probe 2000 1 > gpurun_out/r03m_chol16_w1.jsonl 2>&1 || exit $?
timeout -k 10 60 ./tools/bin/chol16_probe 2000 2 > gpurun_out/r03m_chol16_w2.jsonl 2>&1 || exit $?
cat gpurun_out/r03m_chol16_w1.jsonl gpurun_out/r03m_chol16_w2.jsonl
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --steps 300"
run() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 150 python -u bench.py $B > gpurun_out/r03m_bench_$tag.json 2>/dev/null || return $?
  python -c "
import json;d=json.loads(open('gpurun_out/r03m_bench_$tag.json').read().strip().splitlines()[-1]);n=d['phase_ms_by_launch']
print('$tag', d['value'], d['ms_per_step'], d['final_loss'], {k: n.get(k) for k in ('bwd_w','bwd_lbar','quad_W','recon')})"
}
run lat0 NMGP_BWD_LAT_WGS=0 || exit $?
run lat4k NMGP_BWD_LAT_WGS=4096 || exit $?
run lat8k NMGP_BWD_LAT_WGS=8192 || exit $?
run lat2k NMGP_BWD_LAT_WGS=2048 || exit $?
run lat0b NMGP_BWD_LAT_WGS=0 || exit $?
PROBE_KEEP_EVENTS=1 timeout -k 10 120 python -u tools/graph_edge_probe.py ping_pong > gpurun_out/r03m_graph_keep.jsonl 2>&1
cat gpurun_out/r03m_graph_keep.jsonl
timeout -k 10 60 ./tools/bin/graph_edge_repro ping_pong global autofree destroy > gpurun_out/r03m_graph_destroy.txt 2>&1
echo "hip ping_pong destroy rc=$?: $(tr '\n' ' ' < gpurun_out/r03m_graph_destroy.txt)"
exit 0
