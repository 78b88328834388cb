#!/bin/bash
# A/B of environment variants on a training leg (GPU box): LEG=hcp (default) prints "<env> it/s", LEG=ecog
# "<env> s/step"; two rounds, variants interleaved.  VARIANTS="A=1|A=0".
LEG=${LEG:-hcp}
if [ "$LEG" = ecog ]; then SKIP=--no-hcp; KEY="d['ecog_train']['s_per_step']"; else SKIP=--no-ecog; KEY="d['hcp_train']['it_per_s']"; fi
A="--steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-elbo --no-api --no-kron --no-breakdown $SKIP"
VARIANTS=${VARIANTS:-"NMGP_BIG_ROWS=0|NMGP_BIG_ROWS=1"}
for rep in 1 2; do
IFS='|'; for v in $VARIANTS; do
  unset IFS
  env $v timeout -k 10 300 python bench.py $A 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); print('$v', $KEY)" || exit 1
  IFS='|'
done; unset IFS; done
