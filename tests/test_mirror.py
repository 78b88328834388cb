"""The closed-form (engine) gradients equal the oracle's autograd gradients (CPU)."""
import numpy as np
import pytest
import torch

from oracle import nmgp_oracle as O
from tests import _golden as G
from tests import dsvi_mirror as MR


def _rel(a, b):
    a, b = a.detach().reshape(-1), b.detach().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


@pytest.mark.parametrize("case,D,M", [("toy_forward", 2, 20), ("mid_forward", 3, 64), ("pm25_forward", 5, 256)])
def test_mirror_matches_oracle(case, D, M):
    g = G.load(case)
    xs, ys = G.split_lists(g)
    p = G.params(g, D=D, M=M, requires_grad=True)
    loss, _ = O.forward(p, xs, ys, g["z"], float(g["N"]), O.TapeNoise(g["noise"]))
    loss.backward()
    q = {k: v.detach().clone() for k, v in p.items()}
    x = torch.from_numpy(g["x"]); y = torch.from_numpy(g["y"]); z = torch.from_numpy(g["z"])
    l2, gr, _ = MR.forward_backward(q, x, y, [int(s) for s in g["sizes"]], z, float(g["N"]), torch.from_numpy(g["noise"]))
    assert float(l2) == pytest.approx(float(loss), rel=1e-9)
    for k in O.PARAM_NAMES:
        ref = p[k].grad
        if float(ref.norm()) == 0:
            assert float(gr[k].norm()) == 0, k
            continue
        assert _rel(gr[k], ref) < 1e-7, (k, _rel(gr[k], ref))
