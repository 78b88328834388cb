#!/bin/bash
# Round-3 pass X: four-role Cholesky workgroups reserve the whole CU's LDS (NMGP_CHOL_EXCL): step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -k "four_role or chol_inv" tests/test_gpu_engine.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03x_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03x_tests.log
[ $rc -ne 0 ] && exit $rc
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 300"
for c in 1 0 1 0 1 0; do
  NMGP_CHOL_EXCL=$c timeout -k 10 150 python -u bench.py $B > gpurun_out/r03x_bench_c$c.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r03x_bench_c$c.json').read().strip().splitlines()[-1]);print('CHOL_EXCL=$c', d['value'], d['ms_per_step'], d['final_loss'])"
done
exit 0
