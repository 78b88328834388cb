#!/bin/bash
# A/B of an engine environment toggle on the PM2.5 bench line: alternates VAR=v1 / v2 / ... runs.
# usage: bash tools/ab_env.sh VAR v1 v2 [v3 ...]   (REPS env: repetitions, default 3)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
V=$1; shift
N=${REPS:-3}
ARGS="--steps 300 --warmup 20 --no-cpu-baseline --no-stress --no-elbo --no-api --no-breakdown --no-hcp --no-ecog --no-kron"
for i in $(seq $N); do
  for val in "$@"; do
    env $V=$val timeout -k 10 120 python bench.py $ARGS > gpurun_out/ab_${V}_${val}_$i.json 2> gpurun_out/ab_err.log
    echo "$V=$val rep $i: $(python -c "import json;r=json.loads(open('gpurun_out/ab_${V}_${val}_$i.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")"
  done
done
