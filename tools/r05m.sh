set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for mode in "" "--eager"; do
  NMGP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 20 --warmup 3 $mode --no-breakdown --no-elbo --no-pair > gpurun_out/r05m_n2$mode.json 2> gpurun_out/r05m_n2.err || { tail -20 gpurun_out/r05m_n2.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05m_n2$mode.json').read().strip().splitlines()[-1]); print('$mode', d['value'], d['ms_per_step'])"
done
