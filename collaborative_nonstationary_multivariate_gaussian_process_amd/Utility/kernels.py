"""Drop-in for ``code/SIM_code/Utility/kernels.py`` on the HIP pairwise builder.

Same signatures and semantics: expanded distance ``||x||^2 + ||y||^2 - 2 x.y`` (:5-21), ``+ jitter I``
only when ``X2 is None`` (:35, :64), per-point sigma in the nonstationary kernel (:71).  Inputs may be
CPU tensors; results are device tensors (float64).
"""
import torch

from .. import _lib as L
from .. import hip_ops as H
from . import settings

F64 = torch.float64


def _dev(t):
    dev = torch.device("cuda", torch.cuda.current_device())
    return t.to(device=dev, dtype=F64).contiguous() if t is not None else None


def pairwise_distances(x, y=None):
    """SIM_code/Utility/kernels.py:5-21: ||x||^2 + ||y||^2 - 2 x.y (the x.y product on the MFMA GEMM)."""
    x = _dev(x)
    y = x if y is None else _dev(y)
    xn = (x ** 2).sum(1).view(-1, 1)
    yn = (y ** 2).sum(1).view(1, -1)
    return xn + yn - 2.0 * H.matmul(x, y, transB=True)


def RBF_cov(X1, X2=None, alpha=1., beta=1.):
    """SIM_code/Utility/kernels.py:24-43."""
    X1 = _dev(X1)
    same = X2 is None
    X2 = X1 if same else _dev(X2)
    return H.pairwise(X1, X2, mode=L.RBF, dist=L.DIST_EXPAND, scale2=float(alpha) ** 2, length_scale=float(beta),
                      diag_add=settings.jitter if same else 0.0)


def Nonstationary_RBF_cov(X1, sigma1=None, ell1=None, X2=None, sigma2=None, ell2=None):
    """SIM_code/Utility/kernels.py:46-73."""
    X1 = _dev(X1)
    n1 = X1.shape[0]
    dev = X1.device
    sigma1 = torch.ones(n1, dtype=F64, device=dev) if sigma1 is None else _dev(sigma1)
    ell1 = torch.ones(n1, dtype=F64, device=dev) if ell1 is None else _dev(ell1)
    same = X2 is None
    if same:
        X2, sigma2, ell2 = X1, sigma1, ell1
    else:
        X2, sigma2, ell2 = _dev(X2), _dev(sigma2), _dev(ell2)
    return H.pairwise(X1, X2, mode=L.GIBBS, dist=L.DIST_EXPAND, ellX=ell1, ellZ=ell2, sigX=sigma1, sigZ=sigma2,
                      diag_add=settings.jitter if same else 0.0)
