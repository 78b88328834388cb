#!/bin/bash
# Pair-sharding evidence on a one-GPU box: (1) every rank's ECoG-shaped share timed alone (tools/ecog_bench.py
# shard), (2) bench.py's N=2 path rehearsed with gloo ranks sharing cuda:0 (small pair leg, D=32).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ecog_bench.py shard --world 8 --steps 3 > gpurun_out/ecog_shard.log 2>&1
tail -1 gpurun_out/ecog_shard.log | cut -c1-400
NMGP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --no-elbo --no-breakdown --pair-D 32 > gpurun_out/bench_n2_rehearsal.json 2> gpurun_out/bench_n2_rehearsal.err
tail -1 gpurun_out/bench_n2_rehearsal.json | cut -c1-1500
