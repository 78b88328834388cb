#!/bin/bash
# Round-3 pass Z2: isolated per-launch breakdown (recon, bwd_wG, bwd_wP, bwd_lbar) with and without the
# W-hat fold, then a longer interleaved step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --steps 100"
for c in 1 0; do
  NMGP_WHAT_FOLD=$c timeout -k 10 150 python -u bench.py $B > gpurun_out/r03z2_bd_f$c.json 2>/dev/null || exit $?
  python -c "
import json;d=json.loads(open('gpurun_out/r03z2_bd_f$c.json').read().strip().splitlines()[-1])
b=d['phase_ms_by_launch'];print('WHAT_FOLD=$c', d['value'], {k:b[k] for k in b if k in ('recon','bwd_wG','bwd_wP','bwd_lbar','bwd_w')})"
done
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 600"
for c in 0 1 0 1; do
  NMGP_WHAT_FOLD=$c timeout -k 10 150 python -u bench.py $B > gpurun_out/r03z2_bench_f$c.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r03z2_bench_f$c.json').read().strip().splitlines()[-1]);print('WHAT_FOLD=$c', d['value'], d['ms_per_step'])"
done
exit 0
