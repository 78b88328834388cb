#!/bin/bash
# Round-3 pass K: lookahead Cholesky timeline (chol4_probe), backward-GEMM knob A/B with per-launch times,
# torch graph-edge probe (child processes; last).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
NMGP_CHOL_LA=1 timeout -k 10 60 ./tools/bin/chol4_probe 256 1 > gpurun_out/r03k_probe_la1_b1.txt 2>&1 || exit $?
NMGP_CHOL_LA=1 timeout -k 10 60 ./tools/bin/chol4_probe 256 4 > gpurun_out/r03k_probe_la1_b4.txt 2>&1 || exit $?
NMGP_CHOL_LA=0 timeout -k 10 60 ./tools/bin/chol4_probe 256 1 > gpurun_out/r03k_probe_la0_b1.txt 2>&1 || exit $?
cat gpurun_out/r03k_probe_la1_b1.txt; head -1 gpurun_out/r03k_probe_la1_b4.txt gpurun_out/r03k_probe_la0_b1.txt
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --steps 200"
run() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 150 python -u bench.py $B > gpurun_out/r03k_bench_$tag.json 2>/dev/null || return $?
  python -c "
import json;d=json.loads(open('gpurun_out/r03k_bench_$tag.json').read().strip().splitlines()[-1]);n=d['phase_ms_by_launch']
print('$tag', d['value'], d['ms_per_step'], {k: n.get(k) for k in ('bwd_w','bwd_lbar','quad_W','quad_P','chol','chol_G','recon')})"
}
run def NMGP_X=0 || exit $?
run rounds16 NMGP_GEMM_LAT_MAX_ROUNDS=16 || exit $?
run ksplit2 NMGP_KSPLIT_FACTOR=2 || exit $?
run rounds16b NMGP_GEMM_LAT_MAX_ROUNDS=16 || exit $?
run defb NMGP_X=0 || exit $?
timeout -k 10 300 python -u tools/graph_edge_probe.py > gpurun_out/r03k_graph_edges.jsonl 2>&1
cat gpurun_out/r03k_graph_edges.jsonl
exit 0
