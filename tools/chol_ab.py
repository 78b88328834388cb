"""A/B timing of the fused factor+inverse launch (H.chol_inv_) at the DSVI step's shapes (GPU box):
NMGP_CHOL_4ROLE=1 (four-role kernel: separate update workgroup, chol_inv7_kernel) and =0 (the three-role
chol_inv3_kernel).  (The round-3 lookahead variant, chol_inv4_kernel, was removed in round 4.)
Each variant is captured in a HIP graph of `reps` launches (plus the restore copies, timed separately
and subtracted).  Usage: python tools/chol_ab.py [n:batch:dtype ...]  (default 256:4:f64 256:1:f64)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H  # noqa: E402

dev = torch.device("cuda", 0)


def time_one(n, batch, dt, reps=20):
    g = torch.Generator(device=dev).manual_seed(n + batch)
    G = torch.randn(batch, n, n, generator=g, dtype=torch.float64, device=dev)
    A0 = (G @ G.transpose(-1, -2) / n + torch.eye(n, dtype=torch.float64, device=dev)).to(dt).contiguous()
    work = A0.clone()
    X = torch.empty_like(work)
    info = torch.zeros(batch, dtype=torch.int32, device=dev)
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
    best = None
    for _ in range(5):
        gr.replay(); gc.replay()
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record(); gr.replay(); e[1].record(); e[2].record(); gc.replay(); e[3].record()
        torch.cuda.synchronize()
        us = 1000.0 * (e[0].elapsed_time(e[1]) - e[2].elapsed_time(e[3])) / reps
        best = us if best is None else min(best, us)
    assert int(info.abs().sum()) == 0
    L = work.double()
    resid = float((L @ L.transpose(-1, -2) - A0.double()).norm() / A0.double().norm())
    inv_err = float((X.double() @ L - torch.eye(n, dtype=torch.float64, device=dev)).norm() / n ** 0.5)
    return best, resid, inv_err


cases = sys.argv[1:] or ["256:4:f64", "256:1:f64"]
for c in cases:
    n, b, d = c.split(":")
    dt = torch.float64 if d == "f64" else torch.float32
    rec = {"n": int(n), "batch": int(b), "dtype": d}
    for four, tag in (("1", "four_role"), ("0", "three_role")):
        os.environ["NMGP_CHOL_4ROLE"] = four
        us, resid, ie = time_one(int(n), int(b), dt)
        os.environ.pop("NMGP_CHOL_4ROLE")
        rec[f"{tag}_us"] = round(us, 2)
        rec[f"{tag}_inv_err"] = ie
    print(json.dumps(rec), flush=True)
