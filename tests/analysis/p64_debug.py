"""Intermediates of the fp32 engine's fp64 prior-adjoint chains vs the all-fp32 path (GPU; analysis only)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import nmgp_oracle as O  # noqa: E402
from tests import _golden as G  # noqa: E402
from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine  # noqa: E402

case, D, M = "mid_forward", 3, 64
g = G.load(case)
p = G.params(g, D=D, M=M)
sizes = [int(s) for s in g["sizes"]] if "sizes" in g else [len(x) for x in G.split_lists(g)[0]]
out = {}
for flag in ("0", "1"):
    os.environ["NMGP_PROJ_FP64"] = flag
    eng = DsviEngine(D, M, sum(sizes), g["z"], dtype=torch.float32)
    th = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda", torch.float32)
    gr = torch.zeros_like(th)
    eng.bind(th, gr, N=float(g["N"]))
    eng.load_batch(g["x"], g["y"], sizes, noise=g["noise"])
    eng.forward_backward()
    torch.cuda.synchronize()
    so = [int(v) for v in eng.scal_off]
    nrm = lambda t: float(t.double().norm())
    if flag == "0":
        sp = eng.scal_part.double().cpu().numpy()
        r = {"Pbar_L": nrm(eng.Pbar[1:3]), "R_L": nrm(eng.R[1:3]), "Abar_L": nrm(eng.Abar[1:3]),
             "c0c1": nrm(eng.rowbuf[2 * D + 1:2 * D + 3])}
    else:
        sp = eng.scal64.double().cpu().numpy()
        r = {"Pbar_L": nrm(eng.PbL64), "R_L": nrm(eng.RL64), "Abar_L": nrm(eng.AbL64), "c0c1": nrm(eng.rcL64),
             "p64": eng.p64}
    for q in range(6):
        r[f"scal{q}"] = (float(sp[2 * so[q]:2 * so[q + 1]:2].sum()), float(sp[2 * so[q] + 1:2 * so[q + 1]:2].sum()))
    r["hyp_grad"] = gr[eng.offs["sigma2_tildeell_log"][0]:][:7].double().cpu().numpy().round(6).tolist()
    print("NMGP_PROJ_FP64=" + flag, r, flush=True)
    del eng
os.environ["NMGP_PROJ_FP64"] = "1"
eng = DsviEngine(D, M, sum(sizes), g["z"], dtype=torch.float32)
th = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda", torch.float32)
eng.bind(th, torch.zeros_like(th), N=float(g["N"]))
eng.load_batch(g["x"], g["y"], sizes, noise=g["noise"])
eng.forward_backward()
print([(it[0], it[-1]) if len(it) == 4 else it for it in eng._sched], flush=True)

torch.cuda.synchronize()
gr = eng._grad
o = eng.offs["sigma2_tildeell_log"][0]
print("graph-order eager run  hyp grad", gr[o:o + 7].double().cpu().numpy().round(4).tolist(), flush=True)
import ctypes  # noqa: E402
from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as LL  # noqa: E402
a = eng._keep_args[(0, True)]
LL.check(LL.lib().nmgp_dsvi_finalize_f32(ctypes.byref(a), LL.stream_handle()), "fin")
torch.cuda.synchronize()
print("finalize re-run         hyp grad", gr[o:o + 7].double().cpu().numpy().round(4).tolist(), flush=True)


class Serial:
    concurrent = False

    def start(self, *a):
        pass

    def stop(self, *a):
        pass


eng.scal64.zero_()
eng.forward_backward(timer=Serial())
torch.cuda.synchronize()
print("serial one-stream run   hyp grad", gr[o:o + 7].double().cpu().numpy().round(4).tolist(), flush=True)
