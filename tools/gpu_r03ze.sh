#!/bin/bash
# Round-3 pass ZE: capture the step on a high-priority stream (NMGP_MAIN_PRIO=-1) -- step A/B + timeline.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
python -c "import torch;print('priority range', torch.cuda.Stream.priority_range())"
B="--no-elbo --no-hcp --no-ecog --no-api --no-stress --no-cpu-baseline --no-breakdown --steps 300"
for c in -1 x -1 x -1 x; do
  if [ "$c" = x ]; then unset NMGP_MAIN_PRIO; else export NMGP_MAIN_PRIO=$c; fi
  timeout -k 10 150 python -u bench.py $B > gpurun_out/r03ze_bench_$c.json 2>gpurun_out/r03ze_bench_$c.err || { tail -5 gpurun_out/r03ze_bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r03ze_bench_$c.json').read().strip().splitlines()[-1]);print('MAIN_PRIO=$c', d['value'], d['ms_per_step'], d['final_loss'])"
done
NMGP_MAIN_PRIO=-1 bash tools/gpu_timeline_now.sh prio
