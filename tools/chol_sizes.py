"""Time the fused factor+inverse (H.chol_inv_) of one SPD matrix per size, fp32 and fp64 (GPU box).
Usage: python tools/chol_sizes.py [n ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [int(a) for a in sys.argv[1:]] or [64, 128, 256, 512, 1024, 2048, 4096]
for M in sizes:
    g = torch.Generator(device=dev).manual_seed(0)
    G = torch.randn(M, M, generator=g, dtype=torch.float64, device=dev)
    A64 = G @ G.t() / M + torch.eye(M, dtype=torch.float64, device=dev)
    for dt in (torch.float32, torch.float64):
        A0 = A64.to(dt).contiguous()
        work = A0.clone()
        X = torch.empty_like(work)
        info = torch.zeros(1, dtype=torch.int32, device=dev)
        reps = 10
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            work.copy_(A0)
            H.chol_inv_(work, out=X, info=info)
        torch.cuda.current_stream().wait_stream(s)
        gr, gc = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(reps):
                work.copy_(A0)
                H.chol_inv_(work, out=X, info=info)
        with torch.cuda.graph(gc):
            for _ in range(reps):
                work.copy_(A0)
        gr.replay(); gc.replay()
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record(); gr.replay(); e[1].record(); e[2].record(); gc.replay(); e[3].record()
        torch.cuda.synchronize()
        ms = (e[0].elapsed_time(e[1]) - e[2].elapsed_time(e[3])) / reps
        print(f"n={M:5d} {str(dt)[6:]:8s} chol_inv {ms * 1000:9.1f} us  {M ** 3 / 3 / ms / 1e9:8.3f} TF/s (M^3/3)", flush=True)
