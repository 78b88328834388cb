"""Drop-in for ``code/SIM_code/Utility/kronecker_operation.py`` on the HIP Kronecker kernels.

``kronecker_product`` / ``kronecker_product_diag`` are bit-exact (one multiply per element, the
reference's operand order); ``kron_mv`` is (B kron K) y without forming the product (two MFMA GEMMs,
reference reshape order).  ``kron_inv`` / ``kron_logdet`` take the eigendecompositions the reference
takes with the removed ``torch.symeig`` on the HIP Jacobi eigensolver (``eig.hip``:
in-LDS parallel Jacobi for n <= 64, block Jacobi above).  Eigenvector signs are arbitrary, as
LAPACK's are; every output here is invariant to them.
"""
import torch

from .. import hip_ops as H

F64 = torch.float64


def _dev(t):
    dev = torch.device("cuda", torch.cuda.current_device())
    if not torch.is_tensor(t):
        t = torch.tensor(t, dtype=F64)
    return t.to(device=dev, dtype=F64).contiguous()


def kronecker_product(t1, t2):
    """kronecker_operation.py:5-22."""
    return H.kron_product(_dev(t1), _dev(t2))


def kronecker_product_diag(d1, d2):
    """kronecker_operation.py:25-33."""
    return H.kron_product(_dev(d1).view(-1, 1), _dev(d2).view(-1, 1)).view(-1)


def kron_mv(B, K, y):
    """kronecker_operation.py:72-85."""
    return H.kron_mv(_dev(B), _dev(K), _dev(y))


def kron_inv(sigma2, B, K):
    """kronecker_operation.py:36-53."""
    wB, vB = H.syevj(_dev(B))
    wK, vK = H.syevj(_dev(K))
    U = kronecker_product(vB, vK)
    t = kronecker_product_diag(wB, wK)
    Us = U * (1.0 / (t + _dev(sigma2)))[None, :]
    return H.matmul(Us, U, transB=True)


def kron_logdet(sigma2, B, K):
    """kronecker_operation.py:56-69."""
    wB = H.syevj(_dev(B))[0]
    wK = H.syevj(_dev(K))[0]
    return torch.log(kronecker_product_diag(wB, wK) + _dev(sigma2)).sum()
