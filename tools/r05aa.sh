set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_ecog.py -x -q -k "big or ecog or rec or potrf or chol" --timeout 300 --timeout-method thread > gpurun_out/r05aa_tests.log 2>&1 || { tail -30 gpurun_out/r05aa_tests.log; exit 1; }
tail -1 gpurun_out/r05aa_tests.log
timeout -k 10 120 ./tools/big_trace_batch.x 256 1024 > gpurun_out/r05aa_big_trace_batch.jsonl 2>&1 || { cat gpurun_out/r05aa_big_trace_batch.jsonl; exit 1; }
cut -c1-250 gpurun_out/r05aa_big_trace_batch.jsonl
for v in nb1 nb2; do
  if [ $v = nb1 ]; then unset NMGP_LIB_OVERRIDE; else export NMGP_LIB_OVERRIDE=$PWD/ab_libs/nb2.so; fi
  timeout -k 10 240 python -u tools/big_probe.py > gpurun_out/r05aa_big_probe_$v.jsonl 2>&1 || { tail -20 gpurun_out/r05aa_big_probe_$v.jsonl; exit 1; }
  echo $v; grep variant gpurun_out/r05aa_big_probe_$v.jsonl | cut -c1-110
done
for rep in 1 2; do
for v in nb1 nb2; do
  if [ $v = nb1 ]; then unset NMGP_LIB_OVERRIDE; else export NMGP_LIB_OVERRIDE=$PWD/ab_libs/nb2.so; fi
  timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-breakdown --no-stress --no-elbo --no-api --no-kron > gpurun_out/r05aa_bench_${v}_$rep.json 2> gpurun_out/r05aa_bench.err || { tail -20 gpurun_out/r05aa_bench.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r05aa_bench_${v}_$rep.json').read().strip().splitlines()[-1])
print('$v', $rep, 'pm25', d['value'], 'hcp', d['hcp_train']['it_per_s'], 'ecog', d['ecog_train']['s_per_step'])"
done
done
