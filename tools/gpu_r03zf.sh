#!/bin/bash
# Round-3 pass ZF: workgroup caps for the side-stream L-bar / P-bar_0/1 groups (NMGP_LBAR_GRID / NMGP_WP_GRID):
# parity tests with a cap, then step A/B (300 steps each, interleaved) + timeline.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
NMGP_LBAR_GRID=128 NMGP_WP_GRID=128 timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03zf_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03zf_tests.log
[ $rc -ne 0 ] && exit $rc
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 300"
for c in ${CAPS:-0-0 128-0 192-0 256-0 128-128 0-0 128-0 192-0 256-0 128-128}; do
  IFS=- read l w <<< "$c"
  NMGP_LBAR_GRID=$l NMGP_WP_GRID=$w timeout -k 10 150 python -u bench.py $B > gpurun_out/r03zf_bench_$c.json 2>gpurun_out/r03zf_bench_$c.err || { tail -5 gpurun_out/r03zf_bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r03zf_bench_$c.json').read().strip().splitlines()[-1]);print('LBAR-WP grid=$c', d['value'], d['ms_per_step'], d['final_loss'])"
done
NMGP_LBAR_GRID=${TL_L:-128} NMGP_WP_GRID=${TL_W:-0} bash tools/gpu_timeline_now.sh grid
