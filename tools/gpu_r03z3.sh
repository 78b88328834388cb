#!/bin/bash
# Round-3 pass Z3: W-hat fold bit-identity tests (opt-in path) + default step check.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -q -x -k "what_fold or fp32_big or matches_reference" --timeout 200 --timeout-method thread > gpurun_out/r03z3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03z3_tests.log
[ $rc -ne 0 ] && exit $rc
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 300"
timeout -k 10 150 python -u bench.py $B > gpurun_out/r03z3_bench.json 2>/dev/null || exit $?
python -c "import json;d=json.loads(open('gpurun_out/r03z3_bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['final_loss'])"
