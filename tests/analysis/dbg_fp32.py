import sys, numpy as np, torch
sys.path.insert(0, '.')
from oracle import nmgp_oracle as O
from tests import _golden as G
from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
g = G.load("toy_forward"); xs, ys = G.split_lists(g); p = G.params(g, D=2, M=20)
sizes = [len(x) for x in xs]
for dt in (torch.float64, torch.float32):
    eng = DsviEngine(2, 20, sum(sizes), g["z"], dtype=dt)
    theta = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda", dt)
    grad = torch.zeros_like(theta)
    eng.bind(theta, grad, frozen_mask=0, N=float(g["N"]))
    eng.load_batch(g["x"], g["y"], sizes, noise=g["noise"])
    class T:
        def start(self, n, k): pass
        def stop(self, n, k):
            torch.cuda.synchronize()
            bad = [b for b in ["Afac","Cinv","Ainv","K12","P","Pbar","R","Abar","WG","WP","Y","Xs","v","ellZ","ellX","var_t","rowbuf","facbuf","red","out"] if not torch.isfinite(getattr(eng, b)).all()]
            if bad and not getattr(self, "done", False):
                print(dt, "first non-finite after", n, bad); self.done = True
    eng.forward_backward(timer=T())
    torch.cuda.synchronize()
    print(dt, "loss", float(eng.out[0]), "grad finite", bool(torch.isfinite(grad).all()))
