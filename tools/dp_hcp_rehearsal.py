"""gloo rehearsal of the data-parallel training step at the HCP shape (BASELINE.json configs[2]: D=50, M=512, B=5000,
348 M fp32 parameters): two ranks sharing cuda:0 of a one-GPU box, flat vs bucketed gradient all-reduce
(DsviTrainer.capture_dp / dp_graph_step).  Never a measurement of RCCL over xGMI: gloo moves the 1.4 GB gradient
through host memory, so it shows the schedule (what overlaps what), not the multi-GPU step time.
Rank / world from the environment (RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT); tools/dp_hcp_rehearsal.sh
starts the ranks.  Usage: python tools/dp_hcp_rehearsal.py <flat|bucketed> <steps>"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

mode, steps = sys.argv[1], int(sys.argv[2])
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
m, tr, eng = bench.train_setup(dev, "hcp")
m._noise_seed = 22 + 7919 * rank
dist.broadcast(m._theta, 0)
graphs = tr.capture_dp(eng, world, mode=mode)
assert (graphs[1] is not None) == (mode == "bucketed")
tr.dp_graph_step(eng)                     # warm-up (gloo buffers, comm stream)
torch.cuda.synchronize()
dist.barrier()
t0 = time.time()
for _ in range(steps):
    tr.dp_graph_step(eng)
torch.cuda.synchronize()
dist.barrier()
el = torch.tensor([(time.time() - t0) / steps], dtype=torch.float64)
dist.all_reduce(el, op=dist.ReduceOp.MAX)
theta_sum = m._theta.double().sum().reshape(1).cpu()
sums = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
dist.all_gather(sums, theta_sum)
if rank == 0:
    print(json.dumps({"mode": mode, "world": world, "backend": "gloo (ranks share cuda:0)", "steps": steps,
                      "s_per_step": round(float(el), 4), "grad_bytes": m._grad.numel() * m._grad.element_size(),
                      "loss": float(eng.out[0]), "ranks_in_sync": bool(all(float(s) == float(sums[0]) for s in sums)),
                      "config": "HCP-shaped (D=50, Q=1275, M=512, B=5000, fp32)"}), flush=True)
dist.destroy_process_group()
