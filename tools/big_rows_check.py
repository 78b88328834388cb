"""HCP-shaped training step with the row-segmented products on the 128x128 kernel (NMGP_BIG_ROWS=1) vs the grouped
64x64 kernel (0): loss and gradient of the first step, and the loss after 1, 5 and 22 Adam steps (GPU box).
Usage: python tools/big_rows_check.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
res = {}
for v in ("0", "1"):
    os.environ["NMGP_BIG_ROWS"] = v
    m, tr, eng = bench.train_setup(dev, "hcp")
    g0 = tr.capture(eng, include_update=False)
    g0.replay()
    torch.cuda.synchronize()
    loss0 = float(eng.out[0])
    grad = m._grad.detach().double().cpu().clone()
    g = tr.capture(eng, include_update=True)
    traj = []
    for s in range(22):
        g.replay()
        if s in (0, 4, 21):
            torch.cuda.synchronize()
            traj.append(float(eng.out[0]))
    res[v] = (loss0, grad, traj)
    print(json.dumps({"big_rows": v, "loss0": loss0, "traj": traj, "grad_norm": float(grad.norm())}), flush=True)
    del g0, g, tr, eng, m
    torch.cuda.empty_cache()
d = (res["1"][1] - res["0"][1]).norm() / res["0"][1].norm()
print(json.dumps({"loss0_rel": abs(res["1"][0] - res["0"][0]) / abs(res["0"][0]), "grad_rel": float(d)}))
