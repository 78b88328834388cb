"""Posterior-mean prediction on the MI355X (reference NMGP.predict_Y, code/nmgp_dsvi.py:666-722).

All kernel matrices come from the HIP builder, the four solves K12 (K22 + 1e-4 I)^{-1} mu go
through the HIP Cholesky / triangular inverse / MFMA GEMM; only the final per-row gather
(est_Y[n] = sum_j L[I_n, j, n] G[j, n], the reference's permute + index, :721-722) is a small
elementwise reduction.
"""
import numpy as np
import torch

from . import _lib as L
from . import hip_ops as H

F64 = torch.float64
JIT = 1e-4


def _solve_rows(K12, K22, rhs):
    """K12 (K22 + 1e-4 I)^{-1} rhs  for rhs (M, k): Cholesky -> inverse -> two GEMMs."""
    A = K22.clone()
    A.diagonal().add_(JIT)
    Ci, info = H.chol_inv_(A)
    if int(info.cpu()[0]) != 0:
        raise torch.linalg.LinAlgError("cholesky: K22 + 1e-4 I is not positive-definite")
    Ainv = H.matmul(Ci, Ci, transA=True, maskA=L.A_UPPER, maskB=L.B_LOWER)
    return H.matmul(K12, H.matmul(Ainv, rhs))


def predict_mean(model, inputs_list, index=None):
    dev = model.device_
    D, M = model.D, model.M
    xs = [torch.as_tensor(x).reshape(-1).to(F64) for x in inputs_list]
    ids = list(range(len(xs))) if index is None else list(index)
    I = torch.cat([torch.full((x.shape[0],), int(j), dtype=torch.long) for x, j in zip(xs, ids)]).to(dev)
    x = torch.cat(xs).to(dev).reshape(-1, 1).contiguous()
    Z = model.Z
    th = {k: getattr(model, k).detach() for k in ["mu_W", "mu_v", "mu_U"]}
    hyp = {k: float(torch.exp(getattr(model, k).detach())) for k in
           ["sigma2_tildeell_log", "length_scales_tildeell_log", "sigma2_L0_log", "length_scales_L0_log",
            "sigma2_L1_log", "length_scales_L1_log"]}

    def rbf(a, b, s2, ls):
        return H.pairwise(a, b, mode=L.RBF, scale2=s2, length_scale=ls)

    Kt12 = rbf(x, Z, hyp["sigma2_tildeell_log"], hyp["length_scales_tildeell_log"])
    Kt22 = rbf(Z, Z, hyp["sigma2_tildeell_log"], hyp["length_scales_tildeell_log"])
    v = th["mu_v"].reshape(-1, 1).contiguous()
    t_ell = _solve_rows(Kt12, Kt22, v).reshape(-1)
    ellZ, ellX = torch.exp(v.reshape(-1)), torch.exp(t_ell)
    K012 = rbf(x, Z, hyp["sigma2_L0_log"], hyp["length_scales_L0_log"])
    K022 = rbf(Z, Z, hyp["sigma2_L0_log"], hyp["length_scales_L0_log"])
    K112 = rbf(x, Z, hyp["sigma2_L1_log"], hyp["length_scales_L1_log"])
    K122 = rbf(Z, Z, hyp["sigma2_L1_log"], hyp["length_scales_L1_log"])
    muU = th["mu_U"].reshape(D * D, M).t().contiguous()                 # (M, D*D)
    L0 = _solve_rows(K012, K022, muU)                                   # (B, D*D)
    L1 = _solve_rows(K112, K122, muU)
    KG12 = H.pairwise(x, Z, mode=L.GIBBS, ellX=ellX, ellZ=ellZ)
    KG22 = H.pairwise(Z, Z, mode=L.GIBBS, ellX=ellZ, ellZ=ellZ)
    Gm = _solve_rows(KG12, KG22, th["mu_W"].t().contiguous())          # (B, D)
    Bn = x.shape[0]
    Lr = torch.where(torch.eye(D, dtype=torch.bool, device=dev).reshape(-1), torch.exp(L1), L0).reshape(Bn, D, D)
    Lr = torch.tril(Lr)                                                 # est_L[i, j] for j <= i
    rowsL = Lr[torch.arange(Bn, device=dev), I]                          # (B, D): row I_n of L at n
    return (rowsL * Gm).sum(1)


def sample_Y(model, X_list, n_sample=1000):
    raise NotImplementedError("sample_Y is SURVEY §8f row f1 (next): not in this round")


def sample_FY(model, x, n_sample=1000):
    raise NotImplementedError("sample_FY is SURVEY §8f row f1 (next): not in this round")
