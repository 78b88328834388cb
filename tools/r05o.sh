set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_ecog.py -x -q -k "big or potrf or ecog or rec" --timeout 300 --timeout-method thread > gpurun_out/r05o_tests.log 2>&1 || { tail -30 gpurun_out/r05o_tests.log; exit 1; }
tail -2 gpurun_out/r05o_tests.log
timeout -k 10 600 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-elbo --no-api --no-kron --no-breakdown > gpurun_out/r05o_bench.json 2> gpurun_out/r05o_bench.err || { tail -20 gpurun_out/r05o_bench.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/r05o_bench.json').read().strip().splitlines()[-1])
print('pm25', d['value'], d['ms_per_step'])
for k in ('cholesky_stress','hcp_train','ecog_train'):
    v=d.get(k); print(k, json.dumps(v)[:600])
PY
