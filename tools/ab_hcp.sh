#!/bin/bash
# A/B of environment variants on the HCP training leg (GPU box): each line "<env> it/s", two rounds.
A="--steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-elbo --no-api --no-ecog --no-kron --no-breakdown"
VARIANTS=${VARIANTS:-"NMGP_BIG_ROWS=0|NMGP_BIG_ROWS=1"}
for rep in 1 2; do
IFS='|'; for v in $VARIANTS; do
  unset IFS
  env $v timeout -k 10 200 python bench.py $A 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); print('$v', d['hcp_train']['it_per_s'])" || exit 1
  IFS='|'
done; unset IFS; done
