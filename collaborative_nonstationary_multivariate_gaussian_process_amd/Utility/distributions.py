"""Kronecker Gaussian log-density of ``code/SIM_code/Utility/distributions.py:26-52``."""
import torch

from . import kronecker_operation as KO

F64 = torch.float64


def multivariate_normal_logpdf0(y, mu, B, K, sigma2):
    """Unnormalised log N(y; mu, B kron K + sigma2 I) via the two eigendecompositions (distributions.py:26-52)."""
    wB, vB = torch.linalg.eigh(KO._dev(B))
    wK, vK = torch.linalg.eigh(KO._dev(K))
    a = KO.kron_mv(vB.t(), vK.t(), KO._dev(y) - KO._dev(mu))
    t = KO.kronecker_product_diag(wB, wK)
    w = 1. / (KO._dev(sigma2) + t)
    return -0.5 * torch.log(t + KO._dev(sigma2)).sum() - 0.5 * torch.dot(a * w, a)
