"""Stress potrf timing probe (GPU box): bench.py's M=4096 fp32 blocked Cholesky alone, graph-replayed,
plus the residual (run once per tree for an A/B: the round-3/4 step-kernel knobs it was written for are removed).
usage: python tools/potrf_ab.py [n ...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H  # noqa: E402

dev = torch.device("cuda", 0)
for n in [int(a) for a in sys.argv[1:]] or [4096]:
    g = torch.Generator(device=dev).manual_seed(0)
    G = torch.randn(n, n, generator=g, dtype=torch.float64, device=dev)
    A0 = (G @ G.t() / n + torch.eye(n, dtype=torch.float64, device=dev)).float().contiguous()
    W = A0.clone()
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        H.potrf_blocked_(W, info=info)
    torch.cuda.current_stream().wait_stream(s)
    ref = W.clone()
    reps = 10

    def graph_ms(body):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(reps):
                body()
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            e0.record()
            gr.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / reps)
        return best

    def fac():
        W.copy_(A0)
        H.potrf_blocked_(W, info=info)

    t = graph_ms(fac) - graph_ms(lambda: W.copy_(A0))
    fac()
    torch.cuda.synchronize()
    idx = torch.arange(0, n, 16, device=dev)
    Ld = W.double()
    res = float((Ld[idx] @ Ld.t() - A0.double()[idx]).norm() / A0.double()[idx].norm())
    print(json.dumps({"n": n, "potrf_ms": round(t, 4), "tflops": round(n ** 3 / 3 / (t * 1e-3) / 1e12, 2),
                      "residual": res, "info": int(info.item()), "replay_equal": bool(torch.equal(W, ref)),
                      "env": {k: v for k, v in os.environ.items() if k.startswith("NMGP_")}}), flush=True)
