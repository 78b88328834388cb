"""One tiny DSVI forward+backward on cuda:0 through the HIP engine, checked against the CPU oracle."""
import numpy as np
import torch

from oracle import nmgp_oracle as O
from tests import _golden as G


def run_smoke():
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
    g = G.load("toy_forward")
    xs, ys = G.split_lists(g)
    p = G.params(g)
    sizes = [len(x) for x in xs]
    eng = DsviEngine(2, 20, sum(sizes), g["z"], device="cuda:0")
    theta = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda:0")
    grad = torch.zeros_like(theta)
    eng.bind(theta, grad, N=float(g["N"]))
    eng.load_batch(g["x"], g["y"], sizes, noise=g["noise"])
    out = eng.forward_backward()
    torch.cuda.synchronize()
    q = {k: v.clone().requires_grad_() for k, v in p.items()}
    loss, _ = O.forward(q, xs, ys, g["z"], float(g["N"]), O.TapeNoise(g["noise"]))
    loss.backward()
    ref_grad = torch.cat([q[k].grad.reshape(-1) for k in O.PARAM_NAMES])
    lrel = abs(float(out[0]) - float(loss)) / abs(float(loss))
    grel = float((grad.cpu() - ref_grad).norm() / ref_grad.norm())
    print(f"smoke: loss {float(out[0]):.12g} (oracle {float(loss):.12g}, rel {lrel:.2e}), grad rel {grel:.2e}")
    assert lrel < 1e-10 and grel < 1e-8, (lrel, grel)
