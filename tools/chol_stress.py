"""Stress configuration (BASELINE.json configs[4]): one M=4096 SPD matrix, blocked Cholesky +
inverse on the MI355X, fp32 and fp64 (GPU box).  A = G G^T / M + I with G ~ N(0,1), seed 0.
Prints time, GFLOP/s (M^3/3 for the factorization, 2 M^3/3 with the inverse) and residuals."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [int(a) for a in sys.argv[1:]] or [4096]
for M in sizes:
    g = torch.Generator(device=dev).manual_seed(0)
    G = torch.randn(M, M, generator=g, dtype=torch.float64, device=dev)
    A64 = G @ G.t() / M + torch.eye(M, dtype=torch.float64, device=dev)
    for dt in (torch.float32, torch.float64):
        A0 = A64.to(dt).contiguous()
        Ad = A0.clone()
        X, info = H.chol_inv_(Ad)
        torch.cuda.synchronize()
        assert int(info.abs().sum()) == 0, info
        idx = torch.randperm(M, device=dev)[:256]
        Ld, Xd = Ad.double(), X.double()
        res = float((Ld[idx] @ Ld.t() - A64[idx]).norm() / A64[idx].norm())
        resx = float((Xd[idx] @ Ld - torch.eye(M, dtype=torch.float64, device=dev)[idx]).norm() / 16.0)
        work = A0.clone()
        Xw = torch.empty_like(work)
        infow = torch.zeros(1, dtype=torch.int32, device=dev)
        reps = 5
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            work.copy_(A0)
            H.chol_inv_(work, out=Xw, info=infow)
        torch.cuda.current_stream().wait_stream(s)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(reps):
                work.copy_(A0)
                H.chol_inv_(work, out=Xw, info=infow)
        gr.replay()
        torch.cuda.synchronize()
        # copy cost measured separately and subtracted
        gc = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gc):
            for _ in range(reps):
                work.copy_(A0)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record(); gr.replay(); e[1].record(); e[2].record(); gc.replay(); e[3].record()
        torch.cuda.synchronize()
        ms = (e[0].elapsed_time(e[1]) - e[2].elapsed_time(e[3])) / reps
        f1, f2 = M ** 3 / 3.0, 2.0 * M ** 3 / 3.0
        # blocked right-looking factorization alone (potrf semantics, lookahead + side-stream SYRK)
        Wp = A0.clone()
        infop = torch.zeros(1, dtype=torch.int32, device=dev)
        with torch.cuda.stream(s):
            Wp.copy_(A0)
            H.potrf_blocked_(Wp, info=infop)
        torch.cuda.current_stream().wait_stream(s)
        gp = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gp):
            for _ in range(reps):
                Wp.copy_(A0)
                H.potrf_blocked_(Wp, info=infop)
        gp.replay()
        torch.cuda.synchronize()
        e2 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e2[0].record(); gp.replay(); e2[1].record()
        torch.cuda.synchronize()
        msp = (e2[0].elapsed_time(e2[1]) - e[2].elapsed_time(e[3])) / reps
        assert int(infop.item()) == 0
        Lp = Wp.double()
        resp = float((Lp[idx] @ Lp.t() - A64[idx]).norm() / A64[idx].norm())
        # the same launches issued eagerly (no graph): one hardware queue per stream
        torch.cuda.synchronize()
        ee = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ee[0].record()
        for _ in range(reps):
            Wp.copy_(A0)
            H.potrf_blocked_(Wp, info=infop)
        ee[1].record()
        torch.cuda.synchronize()
        mse = ee[0].elapsed_time(ee[1]) / reps - (e[2].elapsed_time(e[3])) / reps
        print(f"M={M} {str(dt)[6:]:8s} potrf    {mse:8.3f} ms  eager launches (no graph)", flush=True)
        print(f"M={M} {str(dt)[6:]:8s} potrf    {msp:8.3f} ms  {M ** 3 / 3.0 / msp / 1e9:7.2f} TF/s (M^3/3)  "
              f"|LL^T-A|/|A| {resp:.2e}  [blocked right-looking, lookahead]", flush=True)
        print(f"M={M} {str(dt)[6:]:8s} chol+inv {ms:8.3f} ms  {f2 / ms / 1e9:7.2f} TF/s (2M^3/3)  "
              f"[{f1 / ms / 1e6:8.1f} GFLOP/s counting M^3/3]  |LL^T-A|/|A| {res:.2e}  |XL-I| {resx:.2e}",
              flush=True)
