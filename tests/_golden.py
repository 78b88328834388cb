"""Helpers that turn a golden ``.npz`` fixture into oracle / engine inputs (test infrastructure)."""
import os

import numpy as np
import torch

from oracle import nmgp_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def split_lists(g, xkey="x", ykey="y", skey="sizes"):
    sizes = [int(s) for s in g[skey]]
    offs = np.concatenate([[0], np.cumsum(sizes)])
    xs = [g[xkey][offs[i]:offs[i + 1]] for i in range(len(sizes))]
    ys = [g[ykey][offs[i]:offs[i + 1]] for i in range(len(sizes))]
    return xs, ys


def params(g, D=None, M=None, requires_grad=False):
    """The 13 parameters of a forward fixture; big ones regenerated from NMGP(seed=22) if absent."""
    p = {}
    missing = [k for k in O.PARAM_NAMES if "p_" + k not in g]
    if missing:
        base = O.new_params(D, M, seed=22)
        for k in missing:
            p[k] = base[k]
    for k in O.PARAM_NAMES:
        if "p_" + k in g:
            p[k] = torch.from_numpy(np.asarray(g["p_" + k], np.float64).copy())
    if requires_grad:
        p = {k: v.clone().requires_grad_() for k, v in p.items()}
    return p
