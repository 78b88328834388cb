#!/bin/bash
# Round-3 pass ZK: Sigma_v syrk on the main stream (NMGP_V_SIDE=0) instead of a side branch joined before the first Cholesky -- tests + A/B + timeline.

R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
NMGP_V_SIDE=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_training_api.py tests/test_gpu_api.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03zk_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03zk_tests.log
[ $rc -ne 0 ] && exit $rc
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 300"
for c in 0 1 0 1 0 1; do
  NMGP_V_SIDE=$c timeout -k 10 150 python -u bench.py $B > gpurun_out/r03zk_bench_$c.json 2>gpurun_out/r03zk_bench_$c.err || { tail -5 gpurun_out/r03zk_bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r03zk_bench_$c.json').read().strip().splitlines()[-1]);print('V_SIDE=$c', d['value'], d['ms_per_step'], d['final_loss'])"
done
NMGP_V_SIDE=0 bash tools/gpu_timeline_now.sh vside0
