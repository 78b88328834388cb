#!/bin/bash
# Round-3 pass P: four-role Cholesky timeline with the MFMA/poll split; whole-step A/B with it on.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
NMGP_CHOL_4ROLE=1 timeout -k 10 60 ./tools/bin/chol4_probe 256 1 > gpurun_out/r03p_probe_4role.txt 2>&1 || exit $?
cat gpurun_out/r03p_probe_4role.txt
timeout -k 10 300 env NMGP_CHOL_4ROLE=1 python -u -m pytest tests/test_gpu_engine.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03p_engine_4role.log 2>&1
rc=$?; tail -3 gpurun_out/r03p_engine_4role.log
[ $rc -ne 0 ] && exit $rc
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --steps 300"
for c in 1 0 1 0; do
  NMGP_CHOL_4ROLE=$c timeout -k 10 150 python -u bench.py $B > gpurun_out/r03p_bench_c$c.json 2>/dev/null || exit $?
  python -c "
import json;d=json.loads(open('gpurun_out/r03p_bench_c$c.json').read().strip().splitlines()[-1]);n=d['phase_ms_by_launch']
print('4ROLE=$c', d['value'], d['ms_per_step'], {k: n.get(k) for k in ('chol','chol_G','chol_side')})"
done
exit 0
