"""Timing of the fused prior launch (nmgp_chol_tp_f64) alone on the GPU box, at the PM2.5 step's shapes (n = 256,
B = 2000): the [v | t | L0 | L1]-shaped launch and the Gibbs launch, each with and without its row workgroups
(rows = 0: factor + inverse only), beside the plain four-role chol_inv_ on the same matrices; graph-replayed (20
launches per graph, best of 5, the K22 restore copies timed alone and subtracted).  NMGP_TP_DBG=16: per-workgroup
phase stamps of one launch instead.  Usage: python tools/chol_tp_probe.py [B]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H  # noqa: E402

dev = torch.device("cuda", 0)
F = torch.float64
n = 256
B = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
g = torch.Generator(device=dev).manual_seed(3)
Z = torch.linspace(0, 1, n, dtype=F, device=dev)
x = torch.rand(B, generator=g, dtype=F, device=dev)
hyp = torch.tensor([0.0, -1.0, 0.0, -1.0, 0.0, -1.0, 0.0, -1.0], dtype=F, device=dev)
A = torch.zeros(4, n, n, dtype=F, device=dev)
X = torch.zeros_like(A)
info = torch.zeros(4, dtype=torch.int32, device=dev)
K12, T, P = (torch.zeros(4, B, n, dtype=F, device=dev) for _ in range(3))
v = -1.0 + 0.2 * torch.randn(n, generator=g, dtype=F, device=dev)
ellZ = torch.exp(v)
trow = dict(Pt=0.01 * torch.randn(B, n, generator=g, dtype=F, device=dev),
            Tt=0.01 * torch.randn(B, n, generator=g, dtype=F, device=dev), v=v,
            zt=torch.randn(B, generator=g, dtype=F, device=dev), hyp_t=hyp[:1], ellX=torch.zeros(B, dtype=F, device=dev),
            var_t=torch.zeros(B, dtype=F, device=dev))


def _prefill():
    A0 = torch.zeros(4, n, n, dtype=F, device=dev)
    for k in range(3):
        ls = float(torch.exp(hyp[2 * k + 1]))
        A0[k] = torch.exp(-0.5 * (Z[:, None] / ls - Z[None, :] / ls) ** 2) + 1e-4 * torch.eye(n, dtype=F, device=dev)
    S = ellZ[:, None] ** 2 + ellZ[None, :] ** 2
    A0[3] = torch.sqrt(2 * ellZ[:, None] * ellZ[None, :] / S) * torch.exp(-(Z[:, None] - Z[None, :]) ** 2 / S) \
        + 1e-4 * torch.eye(n, dtype=F, device=dev)
    return A0


A0 = _prefill()
A0m = A0[[0, 0, 1, 2]].clone()    # [Sigma-like | t | L0 | L1] slots


def main_op(rows):
    # [Sigma-like | t | L0 | L1]: the K22 slots restored before each launch (its copy is timed separately)
    mats = [dict()] + [dict(rows=rows, hyp=hyp[2 * k:], K12=K12[k], T=T[k], P=P[k]) for k in range(1, 4)]
    op = H.CholTp(A[0], X[0], info, n, mats, jitter=1e-4, Z=Z, x=x, B=B)

    def run():
        A.copy_(A0m)
        op()
    return run


def g_op(rows):
    op = H.CholTp(A[3], X[3], info[3:], n, [dict(rows=rows, K12=K12[3], T=T[3], P=P[3])], jitter=1e-4, Z=Z,
                  ellZ=ellZ, x=x, B=B, trow=trow)

    def run():
        A[3].copy_(A0[3])
        op()
    A[3].copy_(A0[3])
    return run


def time_op(op, reps=20):
    op()
    torch.cuda.synchronize()
    gr = H.HipGraph(dev)
    with gr.capture():
        for _ in range(reps):
            op()
    best = None
    for _ in range(5):
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        us = 1000.0 * e0.elapsed_time(e1) / reps
        best = us if best is None else min(best, us)
    assert int(info.abs().sum()) == 0
    return round(best, 2)


def read_op():
    # the plain four-role launch on the same four matrices (restored before each launch)
    W = A0m.clone()
    Wg = A0[3:].clone()

    def run():
        W.copy_(A0m)
        H.chol_inv_(W, out=X, info=info)

    def run_g():
        Wg.copy_(A0[3:])
        H.chol_inv_(Wg, out=X[3:], info=info[3:])
    return run, (lambda: W.copy_(A0m)), run_g, (lambda: Wg.copy_(A0[3:]))


def trace(op, nwg, label):
    """One eager launch with phase stamps (NMGP_TP_DBG bit 16): per workgroup [start, end, phase2, phase3, phase4]
    in us from the earliest start (wall clock 100 MHz)."""
    import ctypes
    import numpy as np
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    for _ in range(3):
        op()
    torch.cuda.synchronize()
    buf = np.zeros(8 * 512, dtype=np.uint64)
    op()
    torch.cuda.synchronize()
    L.lib().nmgp_chol_tp_trace(ctypes.c_void_p(buf.ctypes.data), buf.size)
    t = buf.reshape(512, 8)[:nwg].astype(np.int64)
    t0 = t[:, 0].min()
    rel = lambda v: round((int(v) - int(t0)) / 100.0, 2) if v > 0 else None
    rows = [[rel(v) for v in t[w, :5]] for w in range(nwg)]
    print(json.dumps({"trace": label, "workgroups": rows}))


if os.environ.get("NMGP_TP_DBG") == "16":
    trace(main_op(1), 16 + 3 * ((B + 31) // 32), "main")
    trace(g_op(2), 4 + (B + 31) // 32, "gibbs")
    sys.exit(0)
rd, cp, rdg, cpg = read_op()
rec = {"n": n, "B": B, "plain_4_us": round(time_op(rd) - time_op(cp), 2), "plain_1_us": round(time_op(rdg) - time_op(cpg), 2),
       "fused_main_us": round(time_op(main_op(1)) - time_op(cp), 2),
       "fused_main_no_rows_us": round(time_op(main_op(0)) - time_op(cp), 2),
       "fused_gibbs_us": round(time_op(g_op(2)) - time_op(cpg), 2),
       "fused_gibbs_no_rows_us": round(time_op(g_op(0)) - time_op(cpg), 2)}
from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L  # noqa: E402
rec["device_status"] = L.device_status(clear=True)
print(json.dumps(rec))
