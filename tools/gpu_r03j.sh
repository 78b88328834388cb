#!/bin/bash
# Round-3 pass J: critical-path-first capture order (NMGP_CRIT_FIRST) parity + A/B + kernel trace;
# HIP-only graph-edge reproducer (host-side; last, it may segfault in hipGraphInstantiate).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_training_api.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03j_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03j_tests.log
[ $rc -ne 0 ] && exit $rc
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 300"
for c in 1 0 1 0; do
  NMGP_CRIT_FIRST=$c timeout -k 10 120 python -u bench.py $B > gpurun_out/r03j_bench_c$c.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r03j_bench_c$c.json').read().strip().splitlines()[-1]);print('CRIT=$c', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r03j_trace -o run -- python3 $R/bench.py --steps 30 --warmup 5 --no-breakdown --no-cpu-baseline --no-stress --no-elbo --no-api --no-hcp --no-ecog > $R/gpurun_out/r03j_trace.json 2> $R/gpurun_out/r03j_trace.err || exit $?
cd $R
for p in one_way relay ping_pong; do
  timeout -k 10 60 ./tools/bin/graph_edge_repro $p > gpurun_out/r03j_graph_$p.txt 2>&1
  rcg=$?; echo "pattern $p rc=$rcg"; cat gpurun_out/r03j_graph_$p.txt
  [ $rcg -ne 0 ] && break
done
exit 0
