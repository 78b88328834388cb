#!/bin/bash
# A/B of step-schedule variants on the PM2.5 bench (GPU box): each line "<env> it/s ms/step", two rounds.
A="--steps 300 --warmup 20 --no-cpu-baseline --no-stress --no-elbo --no-api --no-hcp --no-ecog --no-kron --no-breakdown"
VARIANTS=${VARIANTS:-"NMGP_FUSE_TP=0|NMGP_FUSE_TP=1"}
for rep in 1 2; do
IFS='|'; for v in $VARIANTS; do
  unset IFS
  env $v timeout -k 10 120 python bench.py $A 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); print('$v', d['value'], d['ms_per_step'])" || exit 1
  IFS='|'
done; unset IFS; done
