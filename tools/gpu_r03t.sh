#!/bin/bash
# Round-3 pass T: latency-kernel column-tile packing (NMGP_LAT_COLPACK): parity, per-group times, step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_primitives.py tests/test_gpu_api.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03t_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03t_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/gemm_group_probe.py quad_W quad_P proj3 projG inv3 invG > gpurun_out/r03t_groups_on.jsonl 2>/dev/null || exit $?
NMGP_LAT_COLPACK=0 timeout -k 10 200 python -u tools/gemm_group_probe.py quad_W quad_P proj3 projG inv3 invG > gpurun_out/r03t_groups_off.jsonl 2>/dev/null || exit $?
python - <<'PY'
import json
on=[json.loads(l) for l in open('gpurun_out/r03t_groups_on.jsonl')]
off={d['group']: d for d in (json.loads(l) for l in open('gpurun_out/r03t_groups_off.jsonl'))}
for d in on: print(d['group'], 'lat us packed', d['lat']['us'], 'unpacked', off[d['group']]['lat']['us'], 'tiles', d['lat']['tiles'], off[d['group']]['lat']['tiles'])
PY
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 300"
for c in 1 0 1 0; do
  NMGP_LAT_COLPACK=$c timeout -k 10 150 python -u bench.py $B > gpurun_out/r03t_bench_c$c.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r03t_bench_c$c.json').read().strip().splitlines()[-1]);print('COLPACK=$c', d['value'], d['ms_per_step'], d['final_loss'])"
done
exit 0
