"""Print the GEMM groups of the PM2.5-shaped step plan (kernel, split-K, tiles per problem).  GPU box only:
the engine has no CPU path.  usage: python tools/plan_dump.py [names...]"""
import sys

import numpy as np
import torch

from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H

D, M, B = 5, 256, 2000
eng = DsviEngine(D, M, B, np.linspace(0, 1, M))
theta = torch.zeros(eng.nparam, dtype=torch.float64, device="cuda")
eng.bind(theta, torch.zeros_like(theta))
p = eng._plan(0)
names = sys.argv[1:] or ["quad_W", "quad_P", "bwd_wG", "bwd_wP", "bwd_lbar", "kl_lbar", "bwd_R", "bwd_R_L", "bwd_pr",
                         "bwd_pr_L", "invG", "projG"]
for name in names:
    g = p.get(name)
    if not isinstance(g, H.GemmGroup):
        print(name, type(g).__name__)
        continue
    print(name, "lat" if g.lat else "tile", "total", g.total, "grid", g.grid, "plan", g.plan is not None)
    for d in g.descs:
        print("   m %5d n %4d k %5d ksplit %2d tiles %3d x %d row_seg %2d k_seg %2d span %d flags %d" %
              (d.m, d.n, d.k, d.ksplit, d.tiles_m, d.tiles_n, d.row_seg, d.k_seg, d.seg_span, d.flags))
