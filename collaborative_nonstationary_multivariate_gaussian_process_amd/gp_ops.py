"""HIP-backed, autograd-capable versions of the reference GP helpers (code/utils.py:15-351).

The dense pieces -- kernel-matrix builds, Cholesky, SPD solves, triangular inverses, matrix
products -- are torch.autograd.Functions whose forward AND backward run libnmgp_hip.so kernels;
only O(n) elementwise glue (exp, sqrt, sums) is left to torch on the device.  Inputs may be CPU
tensors (they are moved to the HIP device) so reference driver code runs unchanged.

These drop-ins serve user code that calls the helpers directly.  The training step itself does not
go through them: NMGP.forward uses the fused closed-form engine (engine.py).
"""
import math

import torch

from . import _lib as L
from . import hip_ops as H

F64 = torch.float64
JITTER = 1e-4


def _dev():
    if not torch.cuda.is_available():
        raise RuntimeError("HIP device required (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def _on(t):
    if t is None:
        return None
    if not torch.is_tensor(t):
        return torch.tensor(float(t), dtype=F64, device=_dev())
    return t.to(device=_dev(), dtype=F64) if (not t.is_cuda or t.dtype != F64) else t


# ===================================================================== autograd primitives
def _mm(A, B, tA=False, tB=False, alpha=1.0):
    return H.matmul(A.contiguous(), B.contiguous(), transA=tA, transB=tB, alpha=alpha)


class _MatMul(torch.autograd.Function):
    """C = A @ B for 2-D device tensors on the MFMA GEMM."""

    @staticmethod
    def forward(ctx, A, B):
        ctx.save_for_backward(A, B)
        return _mm(A, B)

    @staticmethod
    def backward(ctx, G):
        A, B = ctx.saved_tensors
        gA = _mm(G, B, tB=True) if ctx.needs_input_grad[0] else None
        gB = _mm(A, G, tA=True) if ctx.needs_input_grad[1] else None
        return gA, gB


def matmul(A, B):
    """torch.matmul semantics for the shapes the reference uses: (m,k)@(k,n), batched (...,m,k)@(...,k,n)
    with broadcasting of a 2-D operand, and matrix @ (...,k,1) vectors."""
    A, B = _on(A), _on(B)
    if A.dim() == 2 and B.dim() == 2:
        return _MatMul.apply(A, B)
    if A.dim() == 2 and B.dim() >= 3:          # P (n,k) @ mu (..., k, 1) -> (..., n, 1)
        Bf = B.reshape(-1, B.shape[-2], B.shape[-1])
        cat = Bf.transpose(0, 1).reshape(B.shape[-2], -1)          # (k, batch*c)
        out = _MatMul.apply(A, cat)                                 # (n, batch*c)
        return out.reshape(A.shape[0], Bf.shape[0], B.shape[-1]).transpose(0, 1).reshape(*B.shape[:-2], A.shape[0], B.shape[-1])
    if A.dim() >= 3 and B.dim() == 2:          # (..., m, k) @ (k, n)
        return _MatMul.apply(A.reshape(-1, A.shape[-1]), B).reshape(*A.shape[:-1], B.shape[-1])
    bs = torch.broadcast_shapes(A.shape[:-2], B.shape[:-2])
    Ab = A.expand(*bs, *A.shape[-2:]).reshape(-1, *A.shape[-2:])
    Bb = B.expand(*bs, *B.shape[-2:]).reshape(-1, *B.shape[-2:])
    outs = [_MatMul.apply(Ab[i], Bb[i]) for i in range(Ab.shape[0])]
    return torch.stack(outs).reshape(*bs, A.shape[-2], B.shape[-1])


class _Cholesky(torch.autograd.Function):
    """Lower Cholesky of (..., n, n) on the HIP potrf; backward L^-T Phi(L^T Lbar) L^-1, symmetrised."""

    @staticmethod
    def forward(ctx, A):
        Lc = A.detach().contiguous().clone()
        info = H.potrf_(Lc)
        if int(info.abs().sum().cpu()) != 0:
            raise torch.linalg.LinAlgError("cholesky: the input is not positive-definite")
        ctx.save_for_backward(Lc)
        return Lc

    @staticmethod
    def backward(ctx, Lbar):
        Lc, = ctx.saved_tensors
        n = Lc.shape[-1]
        Lf = Lc.reshape(-1, n, n)
        Gf = Lbar.contiguous().reshape(-1, n, n)
        Xi = H.trtri(Lf)
        out = []
        for b in range(Lf.shape[0]):
            Pm = _mm(Lf[b], Gf[b], tA=True)
            Pm = torch.tril(Pm)
            Pm.diagonal().mul_(0.5)
            Ab = _mm(_mm(Xi[b], Pm, tA=True), Xi[b])
            out.append(0.5 * (Ab + Ab.t()))
        return torch.stack(out).reshape(Lc.shape)


def cholesky(A):
    return _Cholesky.apply(_on(A))


class _SolveSPD(torch.autograd.Function):
    """X = A^{-1} B for SPD A (n,n), B (n,k): Cholesky + triangular inverse + GEMMs.
    Replaces torch.solve(A=K22_err, input=K21) (LU) of code/utils.py:119 (same solution up to rounding)."""

    @staticmethod
    def forward(ctx, A, B):
        C = A.detach().contiguous().clone()
        Ci, info = H.chol_inv_(C)
        if int(info.cpu()[0]) != 0:
            raise torch.linalg.LinAlgError("solve: A is not positive-definite")
        Ainv = H.matmul(Ci, Ci, transA=True, maskA=L.A_UPPER, maskB=L.B_LOWER)
        X = _mm(Ainv, B)
        ctx.save_for_backward(Ainv, X)
        return X

    @staticmethod
    def backward(ctx, Xbar):
        Ainv, X = ctx.saved_tensors
        Bbar = _mm(Ainv, Xbar)
        Abar = _mm(Bbar, X, tB=True, alpha=-1.0) if ctx.needs_input_grad[0] else None
        return Abar, Bbar


def solve_spd(A, B):
    return _SolveSPD.apply(_on(A), _on(B))


class _TriInv(torch.autograd.Function):
    """X = L^{-1} for lower-triangular (..., n, n) L; backward Lbar = -tril(X^T Xbar X^T)."""

    @staticmethod
    def forward(ctx, Lm):
        X = H.trtri(Lm.detach().contiguous())
        ctx.save_for_backward(X)
        return X

    @staticmethod
    def backward(ctx, Xbar):
        X, = ctx.saved_tensors
        n = X.shape[-1]
        Xf, Gf = X.reshape(-1, n, n), Xbar.contiguous().reshape(-1, n, n)
        out = [torch.tril(_mm(_mm(Xf[b], Gf[b], tA=True), Xf[b], tB=True, alpha=-1.0)) for b in range(Xf.shape[0])]
        return torch.stack(out).reshape(X.shape)


class _RBF(torch.autograd.Function):
    """s2 * exp(-0.5 ||x/ls - z/ls||^2) on the HIP builder; grads w.r.t. s2 and ls (code/utils.py:91-94)."""

    @staticmethod
    def forward(ctx, X, X2, s2, ls):
        K = H.pairwise(X, X2, mode=L.RBF, scale2=float(s2), length_scale=float(ls))
        ctx.save_for_backward(X, X2, K)
        ctx.s2, ctx.ls = float(s2), float(ls)
        return K

    @staticmethod
    def backward(ctx, Kbar):
        X, X2, K = ctx.saved_tensors
        n, m = K.shape
        tiles, _, _ = H.bwd_tiles(n, m)
        sp = torch.zeros(tiles * 2, dtype=F64, device=K.device)
        Kb = Kbar.contiguous()
        d = H.pairwise_bwd_desc(X, X2, K, Kb, mode=L.RBF, ld=m, scale2=ctx.s2, length_scale=ctx.ls, scal_part=sp)
        grp = H.PairwiseBwdGroup([d], K.device)
        grp(F64)
        s = sp.view(tiles, 2).sum(0)
        return None, None, s[0] / ctx.s2, s[1] / ctx.ls


class _Gibbs(torch.autograd.Function):
    """Nonstationary Gibbs kernel (code/utils.py:97-103); grads w.r.t. ell_X, ell_X2, scale2."""

    @staticmethod
    def forward(ctx, X, X2, ex, ez, s2):
        K = H.pairwise(X, X2, mode=L.GIBBS, scale2=float(s2), ellX=ex.detach().contiguous(),
                       ellZ=ez.detach().contiguous())
        ctx.save_for_backward(X, X2, ex, ez, K)
        ctx.s2 = float(s2)
        return K

    @staticmethod
    def backward(ctx, Kbar):
        X, X2, ex, ez, K = ctx.saved_tensors
        n, m = K.shape
        tiles, nct, nrt = H.bwd_tiles(n, m)
        rp = torch.zeros(nct, n, dtype=F64, device=K.device)
        cp = torch.zeros(nrt, m, dtype=F64, device=K.device)
        sp = torch.zeros(tiles * 2, dtype=F64, device=K.device)
        exd, ezd, Kb = ex.detach().contiguous(), ez.detach().contiguous(), Kbar.contiguous()
        d = H.pairwise_bwd_desc(X, X2, K, Kb, mode=L.GIBBS, ld=m, ellX=exd, ellZ=ezd, scale2=ctx.s2,
                                row_part=rp, col_part=cp, scal_part=sp)
        grp = H.PairwiseBwdGroup([d], K.device)
        grp(F64)
        gx, gz = rp.sum(0), cp.sum(0)
        return None, None, gx, gz, sp.view(tiles, 2)[:, 0].sum() / ctx.s2


# ===================================================================== code/utils.py API
def reparameterize(mean, var, z, full_cov=False, use_std=False):
    """code/utils.py:15-65."""
    if var is None:
        return mean
    mean, var, z = _on(mean), _on(var), _on(z)
    if full_cov is False:
        return mean + z * (var + JITTER) ** 0.5
    n = mean.shape[-1]
    chol = var if use_std else cholesky(var + JITTER * torch.eye(n, dtype=F64, device=var.device))
    return mean + matmul(chol, z.unsqueeze(-1))[..., 0]


def mat2ltri(X):
    """code/utils.py:68-72."""
    return torch.tril(_on(X))


def squared_distance(X, X2):
    """code/utils.py:75-81."""
    X, X2 = _on(X), _on(X2)
    diff = X.unsqueeze(1) - X2.unsqueeze(0)
    return torch.sum(diff * diff, -1)


def squared_dist(X, X2, length_scales):
    """code/utils.py:84-88."""
    X = _on(X)
    if X2 is None:
        return squared_distance(X / length_scales, X / length_scales)
    return squared_distance(X / length_scales, _on(X2) / length_scales)


def create_RBF(X, X2=None, scale2=1., length_scales=1.):
    """code/utils.py:91-94 on the HIP builder (differentiable in scale2 / length_scales)."""
    X = _on(X).contiguous()
    X2 = X if X2 is None else _on(X2).contiguous()
    return _RBF.apply(X, X2, _on(scale2).reshape(()), _on(length_scales).reshape(()))


def create_Gibbs(X, X2, ell_X, ell_X2, scale2=1.):
    """code/utils.py:97-103 on the HIP builder (differentiable in ell_X, ell_X2, scale2)."""
    X, X2 = _on(X).contiguous(), _on(X2).contiguous()
    return _Gibbs.apply(X, X2, _on(ell_X), _on(ell_X2), _on(scale2).reshape(()))


def _projection(K12, K22):
    K12, K22 = _on(K12), _on(K22)
    A = K22 + JITTER * torch.eye(K22.shape[0], K22.shape[1], dtype=F64, device=K22.device)
    return solve_spd(A, K12.t()).t(), K12


def _marginal(P, K12, d11, mu, Sigma):
    mu, Sigma = _on(mu), _on(Sigma)
    mu_Y = matmul(P, mu.unsqueeze(-1))[..., 0]
    PS = matmul(P, Sigma)
    s2 = _on(d11) - torch.mul(P, K12).sum(-1) + torch.mul(PS, P).sum(-1)
    return mu_Y, s2


def _randn_like_ref(shape, device):
    """The reference's noise: float32 torch.randn on the CPU generator, cast to float64."""
    return torch.randn(shape).to(F64).to(device)


def MGP_d(K12, K22, d11, mu, Sigma):
    """code/utils.py:106-125."""
    P, K12 = _projection(K12, K22)
    mu_Y, s2 = _marginal(P, K12, d11, mu, Sigma)
    z = _randn_like_ref(mu_Y.size(), mu_Y.device)
    return reparameterize(mu_Y, s2, z, full_cov=False)


def MGP_mu_sigma2(K12, K22, d11, mu, Sigma):
    """code/utils.py:128-146."""
    P, K12 = _projection(K12, K22)
    return _marginal(P, K12, d11, mu, Sigma)


def MGP_mu(K12, K22, mu, device0=None):
    """code/utils.py:149-157."""
    P, _ = _projection(K12, K22)
    return matmul(P, _on(mu).unsqueeze(-1))[..., 0]


def MGP(K12, K22, K11, mu, Sigma):
    """code/utils.py:160-186 (including its double jitter on K22)."""
    K22 = _on(K22) + torch.eye(_on(K22).shape[-1], dtype=F64, device=_dev()) * JITTER
    P, K12 = _projection(K12, K22)
    mu, Sigma = _on(mu), _on(Sigma)
    mu_Y = matmul(P, mu.unsqueeze(-1))[..., 0]
    Sigma_Y = _on(K11) - matmul(P, K12.t()) + matmul(matmul(P, Sigma), P.t())
    z = _randn_like_ref(mu_Y.size(), mu_Y.device)
    return reparameterize(mu_Y, Sigma_Y, z, full_cov=True)


def JGP(K12, K22, K11, mu, Sigma):
    """code/utils.py:189-213."""
    P, K12 = _projection(K12, K22)
    mu, Sigma = _on(mu), _on(Sigma)
    mu_Y = torch.cat([matmul(P, mu.unsqueeze(-1))[..., 0], mu])
    Bm = _on(K11) - matmul(P, K12.t())
    S12 = matmul(P, Sigma)
    S11 = matmul(S12, P.t()) + Bm
    Sigma_Y = torch.cat([torch.cat([S11, S12], 1), torch.cat([S12.t(), Sigma], 1)], 0)
    z = _randn_like_ref(mu_Y.size(), mu_Y.device)
    return reparameterize(mu_Y, Sigma_Y, z, full_cov=True)


def JGP_S(K11_diag, K12, K22, mu, Sigma):
    """code/utils.py:216-237: v ~ N(mu, Sigma) then the independent rows given v."""
    mu = _on(mu)
    z_v = _randn_like_ref(mu.size(), mu.device)
    v = reparameterize(mu, Sigma, z_v, full_cov=True)
    P, K12 = _projection(K12, K22)
    mu_Y = matmul(P, v.unsqueeze(-1))[..., 0]
    s2 = _on(K11_diag) - torch.sum(torch.mul(P, K12), 1)
    z = _randn_like_ref(mu_Y.size(), mu_Y.device)
    return torch.cat([reparameterize(mu_Y, s2, z, full_cov=False), v])


def CGP(K12, K22, K11, X):
    """code/utils.py:240-265."""
    P, K12 = _projection(K12, K22)
    mu_Y = matmul(P, _on(X).unsqueeze(-1))[..., 0]
    Sigma_Y = _on(K11) - matmul(P, K12.t())
    z = _randn_like_ref(mu_Y.size(), mu_Y.device)
    return reparameterize(mu_Y, Sigma_Y, z, full_cov=True)


def Normal_logprob(loc, scale, y):
    """code/utils.py:268-272."""
    loc, scale, y = _on(loc), _on(scale), _on(y)
    var = scale ** 2
    return torch.sum(-((y - loc) ** 2) / (2 * var) - torch.log(scale) - math.log(math.sqrt(2 * math.pi)))


def log_determinant_halfpower(K):
    """code/utils.py:275-277."""
    return cholesky(_on(K)).diagonal(dim1=-2, dim2=-1).log().sum(-1)


def batch_trace_XXT(bmat):
    """code/utils.py:280-287."""
    n, m = bmat.size(-1), bmat.size(-2)
    return bmat.reshape(-1, m * n).pow(2).sum(-1).reshape(bmat.shape[:-2])


def batch_mahalanobis(bL, bx):
    """code/utils.py:290-329 for one (n,n) factor broadcast over a batch of vectors: ||L^{-1} x||^2."""
    bL, bx = _on(bL), _on(bx)
    if bL.dim() != 2:
        raise NotImplementedError("batch_mahalanobis: only a single (n, n) factor is used on the DSVI path")
    Li = _TriInv.apply(bL)
    flat = bx.reshape(-1, bx.shape[-1])
    sol = matmul(Li, flat.t().contiguous())
    return sol.pow(2).sum(0).reshape(bx.shape[:-1])


def KL_Gaussian(X_mu, X_Sigma, X2_mu, X2_Sigma, device0=None):
    """code/utils.py:332-351, with the reference's upper=True trace quirk: triangular_solve reads
    only diag(L2) of the lower factor, so term2 = sum (L1[i,k] / L2[i,i])^2 (code/utils.py:349)."""
    X_mu, X_Sigma, X2_mu, X2_Sigma = _on(X_mu), _on(X_Sigma), _on(X2_mu), _on(X2_Sigma)
    n = X_mu.shape[-1]
    I = torch.eye(n, dtype=F64, device=X_mu.device)
    A1 = X_Sigma + I * JITTER
    A2 = X2_Sigma + I * JITTER
    L1 = cholesky(A1)
    L2 = cholesky(A2)
    half1 = L2.diagonal(dim1=-2, dim2=-1).log().sum(-1) - L1.diagonal(dim1=-2, dim2=-1).log().sum(-1)
    term2 = batch_trace_XXT(L1 / L2.diagonal(dim1=-2, dim2=-1).unsqueeze(-1))
    term3 = batch_mahalanobis(L2, X2_mu - X_mu)
    return half1 + 0.5 * (term2 + term3 - n)
