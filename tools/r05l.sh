set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 2 4; do
  NMGP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2953$n bench.py --gpus $n --steps 30 --warmup 5 --no-breakdown --pair-D 32 --elbo-D 32 > gpurun_out/r05l_bench_n${n}_gloo_rehearsal.json 2> gpurun_out/r05l_bench_n${n}.err || { tail -20 gpurun_out/r05l_bench_n${n}.err; exit 1; }
  tail -1 gpurun_out/r05l_bench_n${n}_gloo_rehearsal.json | cut -c1-700
done
