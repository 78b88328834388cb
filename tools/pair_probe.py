"""Isolated timing of the pair streaming kernels (csrc/pairs.hip) at the ECoG shape: Q pairs of M x M fp32 blocks,
D outputs with R rows each (python tools/pair_probe.py [D] [M] [R]).  Prints per kernel: us per launch and the
algorithmic HBM rate (quad / dot: the lower triangles read once; rank: read + written)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 128
M = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
R = int(sys.argv[3]) if len(sys.argv) > 3 else 4
dev = torch.device("cuda", 0)
pairs = [(i, j) for i in range(D) for j in range(i + 1)]
Q, B = len(pairs), D * R
BM, MM = B * M, M * M
seg = torch.tensor(np.arange(D + 1) * R, dtype=torch.int32, device=dev)
L = torch.randn(Q * MM, device=dev)
P = torch.randn(3 * BM, device=dev)
W = torch.randn(D * BM, device=dev)
C = torch.zeros(D * BM, device=dev)
typ = lambda i, j: 2 if i == j else 1
ops = {
    "quad": H.PairStream("quad", P, L, C, [(typ(i, j) * BM, p * MM, j * BM, i) for p, (i, j) in enumerate(pairs)], seg, M),
    "dot": H.PairStream("dot", W, L, C, [(j * BM, p * MM, j * BM, i) for p, (i, j) in enumerate(pairs)], seg, M),
    "rank": H.PairStream("rank", P, L, W, [(typ(i, j) * BM, p * MM, j * BM, i) for p, (i, j) in enumerate(pairs)],
                         seg, M),
}
tri = Q * M * (M + 1) / 2 * 4
out = {"D": D, "M": M, "R": R, "Q": Q}
for name, op in ops.items():
    op()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        op()
    e1.record()
    torch.cuda.synchronize()
    us = 1000 * e0.elapsed_time(e1) / 3
    nb = tri * (2 if name == "rank" else 1)
    out[name] = {"us": round(us, 1), "GBs": round(nb / us / 1e3, 1)}
print(json.dumps(out))
