#!/bin/bash
# Round-3 pass ZL: symmetric-row pivot chain in the four-role Cholesky (NMGP_CHOL_SYM, default on):
# bit-identity tests, per-launch A/B, step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_engine.py -q -x -k "chol or oracle or mirror" --timeout 200 --timeout-method thread > gpurun_out/r03zl_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03zl_tests.log
[ $rc -ne 0 ] && exit $rc
for c in 1 0 1 0; do
  NMGP_CHOL_SYM=$c timeout -k 10 120 python -u tools/chol_ab.py 256:4:f64 256:1:f64 > gpurun_out/r03zl_chol_$c.jsonl 2>&1 || exit 1
  echo "SYM=$c"; grep -h four gpurun_out/r03zl_chol_$c.jsonl | cut -c1-200
done
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 300"
for c in 1 0 1 0 1 0; do
  NMGP_CHOL_SYM=$c timeout -k 10 150 python -u bench.py $B > gpurun_out/r03zl_bench_$c.json 2>gpurun_out/r03zl_bench_$c.err || { tail -5 gpurun_out/r03zl_bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r03zl_bench_$c.json').read().strip().splitlines()[-1]);print('CHOL_SYM=$c', d['value'], d['ms_per_step'], d['final_loss'])"
done
