"""Kronecker Gaussian log-density of ``code/SIM_code/Utility/distributions.py:26-52``."""
import torch

from .. import hip_ops as H
from . import kronecker_operation as KO

F64 = torch.float64


def multivariate_normal_logpdf0(y, mu, B, K, sigma2):
    """Unnormalised log N(y; mu, B kron K + sigma2 I) via the two eigendecompositions (distributions.py:26-52)."""
    wB, vB = H.syevj(KO._dev(B))
    wK, vK = H.syevj(KO._dev(K))
    a = KO.kron_mv(vB.t(), vK.t(), KO._dev(y) - KO._dev(mu))
    t = KO.kronecker_product_diag(wB, wK)
    w = 1. / (KO._dev(sigma2) + t)
    return -0.5 * torch.log(t + KO._dev(sigma2)).sum() - 0.5 * torch.dot(a * w, a)


def multivariate_normal_logpdf(y, mu, logdetSigma, invSigma):
    """Unnormalised dense log-density (distributions.py:10-23): -1/2 logdet - 1/2 (y-mu)^T Sigma^{-1} (y-mu)."""
    yb = KO._dev(y) - KO._dev(mu)
    return -0.5 * KO._dev(logdetSigma) - 0.5 * torch.dot(yb, H.matmul(KO._dev(invSigma), yb.view(-1, 1)).view(-1))


def multivariate_normal_logpdf1(y, mu, B, K, sigma2):
    """Robust variant (distributions.py:55-96): the reference adds torch.rand(n) * precision to the
    diagonals of B and K (host generator, B first) before the two eigendecompositions."""
    from . import settings
    jB = torch.rand(B.size(0)).type(settings.torchType) * settings.precision
    jK = torch.rand(K.size(0)).type(settings.torchType) * settings.precision
    B = KO._dev(B) + torch.diag(KO._dev(jB))
    K = KO._dev(K) + torch.diag(KO._dev(jK))
    return multivariate_normal_logpdf0(y, mu, B, K, sigma2)


def multivariate_normal_logpdf2(y, mu, B, K, sigma2):
    """Dense reference form (distributions.py:99-113): Sigma = B kron K + sigma2 I, logdet and inverse
    from the fused HIP Cholesky + inverse (Sigma is SPD) instead of torch.logdet / torch.inverse."""
    S = KO.kronecker_product(B, K)
    S = S + KO._dev(sigma2) * torch.eye(S.shape[0], dtype=F64, device=S.device)
    Lm = S.contiguous().clone()
    X, info = H.chol_inv_(Lm)
    if int(info[0]) != 0:
        raise torch.linalg.LinAlgError("multivariate_normal_logpdf2: B kron K + sigma2 I is not positive definite")
    logdet = 2.0 * torch.log(torch.diagonal(Lm)).sum()
    inv = H.matmul(X, X, transA=True)
    return multivariate_normal_logpdf(y, mu, logdet, inv)
