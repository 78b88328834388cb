#!/bin/bash
# Round-3 pass Z: W-hat fold (recon writes the per-(factor, row) scales, the backward GEMMs scale their W
# operand: NMGP_ASCALE / NMGP_KSCALE) -- GPU suite, then step A/B against the in-place W-hat (NMGP_WHAT_FOLD=0).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r03z_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03z_tests.log
[ $rc -ne 0 ] && exit $rc
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 300"
for c in 1 0 1 0 1 0; do
  NMGP_WHAT_FOLD=$c timeout -k 10 150 python -u bench.py $B > gpurun_out/r03z_bench_f$c.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r03z_bench_f$c.json').read().strip().splitlines()[-1]);print('WHAT_FOLD=$c', d['value'], d['ms_per_step'], d['final_loss'])"
done
exit 0
