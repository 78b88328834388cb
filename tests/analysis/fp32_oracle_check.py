"""The oracle (the reference's algorithm op for op) run in fp32 vs fp64 on a golden fixture: how much of
an fp32 engine's error is inherent to fp32 arithmetic at that conditioning.  Test
infrastructure (CPU).  usage: python tests/analysis/fp32_oracle_check.py hcp_like_forward 8 512"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import nmgp_oracle as O
from tests import _golden as G
torch.set_num_threads(8)
case, D, M = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
g = G.load(case)
xs, ys = G.split_lists(g)
p = G.params(g, D=D, M=M)
res = {}
for dt in (torch.float64, torch.float32):
    O.DT = dt
    _np64 = np.float64
    O.np = type("npshim", (), {"asarray": staticmethod(lambda a, d=None: np.asarray(a, np.float32 if (dt == torch.float32 and d is np.float64) else d)), "float64": np.float64, **{k: getattr(np, k) for k in ("int64", "int32", "hstack", "repeat", "arange", "stack", "concatenate", "cumsum", "zeros", "ones")}})
    q = {k: v.to(dt).clone().requires_grad_() for k, v in p.items()}
    xs_ = [np.asarray(x, np.float64) for x in xs]
    class Tape(O.TapeNoise):
        def __call__(self, n):
            return super().__call__(n).to(dt)
    loss, c = O.forward(q, xs_, ys, g["z"], float(g["N"]), Tape(g["noise"]))
    loss.backward()
    res[dt] = (float(loss), {k: q[k].grad.double().clone() for k in q}, {k: float(c[k]) for k in ("KL_W","KL_v","KL_U") if k in c})
    print(dt, float(loss), res[dt][2], float(g["loss"]))
l64, g64, _ = res[torch.float64]; l32, g32, _ = res[torch.float32]
print("loss rel", abs(l32-l64)/abs(l64))
full = lambda gg: torch.cat([gg[k].reshape(-1) for k in O.PARAM_NAMES])
print("grad rel-norm", float((full(g32)-full(g64)).norm()/full(g64).norm()))
