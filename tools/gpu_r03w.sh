#!/bin/bash
# Round-3 pass W: v chain waits g22 directly (NMGP_G22_SIDE) and forms P_t^T tbar inside the v backward
# (NMGP_VT_FUSED): parity + step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_training_api.py tests/test_gpu_pair_shard.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03w_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03w_tests.log
[ $rc -ne 0 ] && exit $rc
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 300"
for c in 11 00 10 11 00 01 11 00; do
  NMGP_G22_SIDE=${c:0:1} NMGP_VT_FUSED=${c:1:1} timeout -k 10 150 python -u bench.py $B > gpurun_out/r03w_bench_c$c.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r03w_bench_c$c.json').read().strip().splitlines()[-1]);print('G22_SIDE,VT_FUSED=$c', d['value'], d['ms_per_step'], d['final_loss'])"
done
exit 0
