set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in cur kl1; do
  if [ $v = cur ]; then unset NMGP_LIB_OVERRIDE; else export NMGP_LIB_OVERRIDE=$PWD/ab_libs/kl1.so; fi
  timeout -k 10 240 python -u tools/big_probe.py > gpurun_out/r05ae_big_probe_$v.jsonl 2>&1 || { tail -20 gpurun_out/r05ae_big_probe_$v.jsonl; exit 1; }
  echo $v; grep '"kl_lbar"' gpurun_out/r05ae_big_probe_$v.jsonl | cut -c1-110
done
for rep in 1 2; do
for v in cur kl1; do
  if [ $v = cur ]; then unset NMGP_LIB_OVERRIDE; else export NMGP_LIB_OVERRIDE=$PWD/ab_libs/kl1.so; fi
  timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-breakdown --no-stress --no-elbo --no-api --no-kron --no-hcp > gpurun_out/r05ae_bench_${v}_$rep.json 2> gpurun_out/r05ae_bench.err || { tail -20 gpurun_out/r05ae_bench.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r05ae_bench_${v}_$rep.json').read().strip().splitlines()[-1])
print('$v', $rep, 'ecog', d['ecog_train']['s_per_step'])"
done
done
