"""Timing of the fused prior launch (nmgp_chol_tp_f64) alone on the GPU box, at the PM2.5 step's shapes (n = 256,
B = 2000): the [v | t | L0 | L1]-shaped launch and the Gibbs launch, each with and without its row workgroups
(rows = 0: factor + inverse only, K22 still built), graph-replayed (20 launches per graph, best of 5).  What the row
workgroups add to a launch is the difference.  Usage: python tools/chol_tp_probe.py [B]"""
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


def main_op(rows):
    mats = [dict(build=1, rows=0, hyp=hyp[0:])] + [dict(build=1, rows=rows, hyp=hyp[2 * k:], K12=K12[k], T=T[k],
                                                        P=P[k]) for k in range(1, 4)]
    return H.CholTp(A[0], X[0], info, n, mats, jitter=1e-4, Z=Z, x=x, B=B)


def g_op(rows):
    return H.CholTp(A[3], X[3], info[3:], n, [dict(build=2, rows=rows, K12=K12[3], T=T[3], P=P[3])], jitter=1e-4, Z=Z,
                    ellZ=ellZ, x=x, B=B, trow=trow)


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
    # the plain four-role launch on the same matrices (K22 read from A, restored before each launch)
    A0 = torch.zeros(4, n, n, dtype=F, device=dev)
    for k in range(4):
        ls = float(torch.exp(hyp[2 * k + 1]))
        A0[k] = torch.exp(-0.5 * (Z[:, None] / ls - Z[None, :] / ls) ** 2) + 1e-4 * torch.eye(n, dtype=F, device=dev)
    W = A0.clone()

    def run():
        W.copy_(A0)
        H.chol_inv_(W, out=X, info=info)
    return run, (lambda: W.copy_(A0))


def main_prefilled(rows):
    # the fused launch with every K22 already in A (restored before each launch): with NMGP_TP_DBG=1/2/3 the
    # factor / update roles read it instead of building
    A0 = torch.zeros(4, n, n, dtype=F, device=dev)
    for k in range(4):
        ls = float(torch.exp(hyp[2 * k + 1]))
        A0[k] = torch.exp(-0.5 * (Z[:, None] / ls - Z[None, :] / ls) ** 2) + 1e-4 * torch.eye(n, dtype=F, device=dev)
    op = main_op(rows)

    def run():
        A.copy_(A0)
        op()
    return run


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
    L.lib().nmgp_chol_tp_trace(ctypes.c_void_p(buf.ctypes.data), 0)
    zero = np.zeros(8 * 512, dtype=np.uint64)
    op()
    torch.cuda.synchronize()
    L.lib().nmgp_chol_tp_trace(ctypes.c_void_p(buf.ctypes.data), buf.size)
    t = buf.reshape(512, 8)[:nwg].astype(np.int64)
    t0 = t[:, 0].min()
    rel = lambda v: round((int(v) - int(t0)) / 100.0, 2) if v > 0 else None
    rows = [[rel(v) for v in t[w, :5]] for w in range(nwg)]
    print(json.dumps({"trace": label, "workgroups": rows}))


if os.environ.get("NMGP_TP_DBG") == "16":
    trace(main_op(1), 16 + 3 * ((B + 63) // 64), "main")
    trace(g_op(2), 4 + (B + 63) // 64, "gibbs")
    sys.exit(0)
if os.environ.get("NMGP_TP_DBG"):
    dbg = int(os.environ["NMGP_TP_DBG"])
    print(json.dumps({"dbg": dbg, "main_rows_prefilled_us": time_op(main_prefilled(1)) if not dbg & 4 else None,
                      "main_no_rows_prefilled_us": time_op(main_prefilled(0))}))
    sys.exit(0)
rd, cp = read_op()
rec = {"n": n, "B": B, "chol_inv7_4_us_incl_copy": time_op(rd), "copy_us": time_op(cp),
       "main_rows_us": time_op(main_op(1)), "main_no_rows_us": time_op(main_op(0)),
       "gibbs_rows_us": time_op(g_op(2)), "gibbs_no_rows_us": time_op(g_op(0))}
from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L  # noqa: E402
rec["device_status"] = L.device_status(clear=True)
print(json.dumps(rec))
