#!/bin/bash
# Round-3 pass B: lookahead Cholesky correctness + A/B timing, ECoG fp32 per-term diagnosis, PM2.5 A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -k "chol_inv or potrf_trtri" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03b_chol_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03b_chol_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/chol_ab.py 256:4:f64 256:1:f64 256:1:f32 128:8:f64 > gpurun_out/r03b_chol_ab.jsonl 2>&1 || exit $?
cat gpurun_out/r03b_chol_ab.jsonl
timeout -k 10 200 python -u tests/analysis/ecog_fp32_diag.py > gpurun_out/r03b_ecog_diag.log 2>&1 || exit $?
cat gpurun_out/r03b_ecog_diag.log | grep -v amdgpu.ids
for la in 1 0 1 0; do
  NMGP_CHOL_LA=$la timeout -k 10 120 python -u bench.py --no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --steps 300 > gpurun_out/r03b_bench_la$la.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r03b_bench_la$la.json').read().strip().splitlines()[-1]);print('LA=$la', d['value'], d['ms_per_step'], d['cholesky'])"
done
