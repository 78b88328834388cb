"""Diagnostic: on the model.pt golden case, compare the fused chol_inv kernel with potrf+trtri and
with CPU LAPACK on the exact matrices the engine factorizes (run on the GPU box)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests.test_gpu_engine import _setup
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H

case = sys.argv[1] if len(sys.argv) > 1 else "modelpt_forward"
g, xs, ys, p, eng, theta, grad = _setup(case)
saved = {}
sched = eng._schedule(0)
new = []
for it in sched:
    if len(it) > 1 and it[1] == "chol":
        name, kind, fn, where = it

        def wrap(s, fn=fn, name=name):
            saved[name] = eng.Afac.clone()   # all slots; the factorized ones are selected below
            fn(s)
        new.append((name, kind, wrap, where))
    else:
        new.append(it)
eng._sched = new
eng._run(new, None, None)
torch.cuda.synchronize()
NF = eng.NF
FV = NF - 1
ranges = {"chol_side": range(0, FV), "chol": range(FV, FV + 4), "chol_G": range(NF + 3, NF + 4)}
for name, rg in ranges.items():
    if name not in saved:
        continue
    for i in rg:
        A = saved[name][i].double()
        Acpu = A.cpu()
        Lref = torch.linalg.cholesky(Acpu)
        Xref = torch.linalg.inv(Lref)
        cond = torch.linalg.cond(Acpu).item()
        L1 = A.clone().contiguous()
        X1, info1 = H.chol_inv_(L1)
        L2 = A.clone().contiguous()
        H.potrf_(L2)
        X2 = H.trtri(L2)
        rel = lambda a, b: float((a.cpu() - b).norm() / b.norm())
        print(f"{name}[{i}] cond {cond:.3e}  fused L {rel(L1, Lref):.2e} X {rel(X1, Xref):.2e} | "
              f"old L {rel(L2, Lref):.2e} X {rel(X2, Xref):.2e}", flush=True)
        E = (L1.cpu() - Lref).abs() / Lref.abs().max()
        idx = int(E.argmax())
        print("   worst L entry", divmod(idx, A.shape[0]), f"{float(E.max()):.2e}",
              "diag rel err", [f"{v:.1e}" for v in ((L1.cpu().diagonal() - Lref.diagonal()) / Lref.diagonal()).abs().tolist()[:20]])
