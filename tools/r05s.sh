set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for v in cur lat_head latgemm_head; do
  if [ $v = cur ]; then unset NMGP_LIB_OVERRIDE; else export NMGP_LIB_OVERRIDE=$PWD/ab_libs/$v.so; fi
  timeout -k 10 300 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-breakdown --no-stress --no-hcp --no-ecog --no-elbo --no-api --no-kron > gpurun_out/r05s_${v}_${rep}.json 2> gpurun_out/r05s_err.log || { tail -20 gpurun_out/r05s_err.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05s_${v}_${rep}.json').read().strip().splitlines()[-1]); print('$v', $rep, d['value'], d['ms_per_step'])"
done
done
