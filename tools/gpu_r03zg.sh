#!/bin/bash
# Round-3 pass ZG: G-prior adjoint chain on the main stream, K_G12 builder backward + t chains on side2 (NMGP_PR_MAIN) -- tests + A/B + timeline.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
NMGP_PR_MAIN=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_training_api.py tests/test_gpu_ecog.py tests/test_gpu_pair_shard.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03zg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03zg_tests.log
[ $rc -ne 0 ] && exit $rc
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 300"
for c in 1 0 1 0 1 0; do
  NMGP_PR_MAIN=$c timeout -k 10 150 python -u bench.py $B > gpurun_out/r03zg_bench_$c.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r03zg_bench_$c.json').read().strip().splitlines()[-1]);print('PR_MAIN=$c', d['value'], d['ms_per_step'], d['final_loss'])"
done
NMGP_PR_MAIN=1 bash tools/gpu_timeline_now.sh prmain
