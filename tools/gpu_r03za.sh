#!/bin/bash
# Round-3 pass ZA: split-K k-tile caps for the backward P-bar / L-bar groups (NMGP_KT_CAP_WG / _WP / _LBAR),
# step A/B on the PM2.5 bench (300 steps each, interleaved).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 300"
for c in ${CAPS:-0-0-0 16-0-0 20-0-0 0-0-0 16-0-0 20-0-0 0-0-0 16-0-0 20-0-0 16-16-0}; do
  IFS=- read g p l <<< "$c"
  NMGP_KT_CAP_WG=$g NMGP_KT_CAP_WP=$p NMGP_KT_CAP_LBAR=$l timeout -k 10 150 python -u bench.py $B > gpurun_out/r03za_bench_$c.json 2>gpurun_out/r03za_bench_$c.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r03za_bench_$c.json').read().strip().splitlines()[-1]);print('caps WG-WP-LBAR=$c', d['value'], d['ms_per_step'], d['final_loss'])"
done
exit 0
