set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05n_tests.log 2>&1 || { tail -30 gpurun_out/r05n_tests.log; exit 1; }
tail -2 gpurun_out/r05n_tests.log
for mode in auto bucketed; do
for n in 2 4; do
  NMGP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2955$n bench.py --gpus $n --steps 30 --warmup 5 --no-breakdown --pair-D 32 --elbo-D 32 --dp-allreduce $mode > gpurun_out/r05n_bench_n${n}_${mode}_gloo_rehearsal.json 2> gpurun_out/r05n_bench_n${n}.err || { tail -20 gpurun_out/r05n_bench_n${n}.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05n_bench_n${n}_${mode}_gloo_rehearsal.json').read().strip().splitlines()[-1]); print($n, '$mode', d['value'], d['ms_per_step'], d['config']['dp_allreduce'][:40])"
done
done
