#!/bin/bash
# Round-3 pass ZB: full GPU suite with the P-bar_G k-tile cap default, default bench x2, and one WRITE_SIZE
# pass of the bench with the W-hat fold on (recon's stores per launch).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r03zb
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -s -k "not nothing" > gpurun_out/r03zb_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03zb_tests.log; grep PARITY gpurun_out/r03zb_tests.log > gpurun_out/r03zb_parity.txt
[ $rc -ne 0 ] && exit $rc
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 300"
for i in 1 2; do
  timeout -k 10 150 python -u bench.py $B > gpurun_out/r03zb_bench_$i.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r03zb_bench_$i.json').read().strip().splitlines()[-1]);print('default', d['value'], d['ms_per_step'], d['final_loss'])"
done
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-stress --no-elbo --no-api --no-hcp --no-ecog --no-breakdown"
for f in 1 0; do
  NMGP_WHAT_FOLD=$f timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r03zb/write_f$f -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/r03zb/bench_f$f.json 2> $R/gpurun_out/r03zb/write_f$f.err || exit $?
done
exit 0
