set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_ecog.py tests/test_gpu_engine.py -x -q -k "big or potrf or ecog or rec or hcp or pair" --timeout 300 --timeout-method thread > gpurun_out/r05u_tests.log 2>&1 || { tail -30 gpurun_out/r05u_tests.log; exit 1; }
tail -2 gpurun_out/r05u_tests.log
timeout -k 10 120 ./tools/big_trace_batch.x 256 1024 > gpurun_out/r05u_big_trace_batch.jsonl 2>&1 || { cat gpurun_out/r05u_big_trace_batch.jsonl; exit 1; }
cat gpurun_out/r05u_big_trace_batch.jsonl
timeout -k 10 240 python -u tools/big_probe.py > gpurun_out/r05u_big_probe.jsonl 2>&1 || { tail -20 gpurun_out/r05u_big_probe.jsonl; exit 1; }
grep variant gpurun_out/r05u_big_probe.jsonl | cut -c1-150
timeout -k 10 600 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-elbo --no-api --no-kron --no-breakdown > gpurun_out/r05u_bench.json 2> gpurun_out/r05u_bench.err || { tail -20 gpurun_out/r05u_bench.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/r05u_bench.json').read().strip().splitlines()[-1])
print('pm25', d['value'], d['ms_per_step'])
for k in ('cholesky_stress','hcp_train','ecog_train'):
    v=d.get(k); print(k, {x: v.get(x) for x in ('potrf_ms','s_per_step','it_per_s','step_tflops','peak_mem_GB')})
PY
