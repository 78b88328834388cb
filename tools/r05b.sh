set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -x -q -k "kron or graph" --timeout 120 --timeout-method thread > gpurun_out/r05b_tests.log 2>&1 || { tail -30 gpurun_out/r05b_tests.log; exit 1; }
tail -2 gpurun_out/r05b_tests.log
timeout -k 10 300 python -u bench.py --no-hcp --no-ecog --no-elbo --no-api --no-cpu-baseline > gpurun_out/r05b_bench.json 2> gpurun_out/r05b_bench.err || { tail -30 gpurun_out/r05b_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05b_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step']); print(json.dumps(d['kron_mv'])); print(json.dumps(d['cholesky_stress'])[:1500]); print(json.dumps(d['roofline'])[:2500])"
bash tools/stress_hbm.sh r05b
