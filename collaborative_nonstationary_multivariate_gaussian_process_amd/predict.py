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


def _solve_rows(K12, K22, rhs, infos):
    """K12 (K22 + 1e-4 I)^{-1} rhs  for rhs (M, k): Cholesky -> inverse -> two GEMMs.  The Cholesky
    info word is appended to `infos` (checked by the caller: no host synchronisation here)."""
    A = K22.clone()
    A.diagonal().add_(JIT)
    Ci, info = H.chol_inv_(A)
    infos.append(info)
    Ainv = H.matmul(Ci, Ci, transA=True, maskA=L.A_UPPER, maskB=L.B_LOWER)
    return H.matmul(K12, H.matmul(Ainv, rhs))


def prepare_inputs(model, inputs_list, index=None):
    """Device copies of the prediction inputs (x as a column, the output id of every row): made once
    when the same test inputs are predicted every iteration (inference(X_test_list=...))."""
    dev = model.device_
    xs = [torch.as_tensor(x).reshape(-1).to(F64) for x in inputs_list]
    ids = list(range(len(xs))) if index is None else list(index)
    I = torch.cat([torch.full((x.shape[0],), int(j), dtype=torch.long) for x, j in zip(xs, ids)]).to(dev)
    x = torch.cat([t.to(dev) for t in xs]).reshape(-1, 1).contiguous()
    return x, I


def _rbf(model, hyp64, a, b, k):
    """RBF kernel of prior k (0: tilde-ell, 1: L0, 2: L1) with its hyper-parameters read ON THE DEVICE
    (log scale, from the fp64 copy of theta's 7 hyper-parameters): no host round trip."""
    out = torch.empty(a.shape[0], b.shape[0], dtype=F64, device=a.device)
    H.PairwiseGroup([H.pairwise_desc(out, a, b, mode=L.RBF, hyp=hyp64, hyp_off=2 * k, hyp_log=True)],
                    a.device)(F64)
    return out


def predict_mean(model, inputs_list, index=None, prepared=None, defer_check=False):
    """NMGP.predict_Y (code/nmgp_dsvi.py:666-722) -> (N,) device tensor, computed in fp64.

    Sync-free: hyper-parameters are read on the device and the four Cholesky info words are checked
    at the end -- or, with defer_check=True, left to the model's next check_numerics() (the caller's
    existing synchronisation point; inference() predicts every iteration this way).  `prepared`: the
    (x, I) of prepare_inputs for repeated predictions on the same inputs."""
    dev = model.device_
    D, M = model.D, model.M
    x, I = prepared if prepared is not None else prepare_inputs(model, inputs_list, index)
    Z = model.Z
    th = {k: getattr(model, k).detach().to(F64) for k in ["mu_W", "mu_v", "mu_U"]}   # predicts in fp64
    o = model._offs["sigma2_tildeell_log"][0]
    hyp64 = model._theta.detach()[o:o + 7].to(F64)
    infos = []
    Kt12, Kt22 = _rbf(model, hyp64, x, Z, 0), _rbf(model, hyp64, Z, Z, 0)
    v = th["mu_v"].reshape(-1, 1).contiguous()
    t_ell = _solve_rows(Kt12, Kt22, v, infos).reshape(-1)
    ellZ, ellX = torch.exp(v.reshape(-1)), torch.exp(t_ell)
    K012, K022 = _rbf(model, hyp64, x, Z, 1), _rbf(model, hyp64, Z, Z, 1)
    K112, K122 = _rbf(model, hyp64, x, Z, 2), _rbf(model, hyp64, Z, Z, 2)
    muU = model.mu_U_dense().to(F64).reshape(D * D, M).t().contiguous()   # (M, D*D)
    L0 = _solve_rows(K012, K022, muU, infos)                            # (B, D*D)
    L1 = _solve_rows(K112, K122, muU, infos)
    KG12 = H.pairwise(x, Z, mode=L.GIBBS, ellX=ellX, ellZ=ellZ)
    KG22 = H.pairwise(Z, Z, mode=L.GIBBS, ellX=ellZ, ellZ=ellZ)
    Gm = _solve_rows(KG12, KG22, th["mu_W"].t().contiguous(), infos)   # (B, D)
    Bn = x.shape[0]
    Lr = torch.where(torch.eye(D, dtype=torch.bool, device=dev).reshape(-1), torch.exp(L1), L0).reshape(Bn, D, D)
    Lr = torch.tril(Lr)                                                 # est_L[i, j] for j <= i
    rowsL = Lr[torch.arange(Bn, device=dev), I]                          # (B, D): row I_n of L at n
    info = torch.cat(infos)
    if defer_check:
        model._pending_info.append(info)
    elif int(info.abs().max().cpu()) != 0:
        raise torch.linalg.LinAlgError("cholesky: K22 + 1e-4 I is not positive-definite")
    return (rowsL * Gm).sum(1)


# ==================================================================================== sampling (§8f f1)
class _Draws:
    """Standard normals in the reference's call order per sample (code/nmgp_dsvi.py:436-476):
    z_v (M), z_t (N), Q x (N) pair noise in (i, j <= i) order, G (D, N), then z_F.  ``tape`` (a flat
    float64 vector, tests only) replays recorded reference noise; otherwise draws come from the
    HIP Philox generator seeded from torch's CPU generator (so ``torch.manual_seed`` makes runs
    reproducible; the stream itself is not the reference's float32 CPU stream)."""

    def __init__(self, dev, tape=None):
        self.dev, self.pos = dev, 0
        self.tape = None if tape is None else torch.as_tensor(np.asarray(tape, np.float64)).to(dev)
        self.seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if tape is None else 0

    def take(self, S, per_sample):
        """(S, per_sample) block: the next S samples' noise."""
        n = S * per_sample
        if self.tape is not None:
            out = self.tape[self.pos:self.pos + n]
            assert out.numel() == n, "noise tape exhausted"
        else:
            out = H.normal_(torch.empty(n, dtype=F64, device=self.dev), self.seed, offset=self.pos)
        self.pos += n
        return out.reshape(S, per_sample)


def _tril(t):
    return torch.tril(t)


def _chol_inv_checked(A, what):
    Ci, info = H.chol_inv_(A)
    if int(info.max().cpu()) != 0:
        raise torch.linalg.LinAlgError(f"cholesky: {what} + 1e-4 I is not positive-definite")
    return A, Ci                                                         # A now holds L


def _proj_var(K12, K22, d11):
    """P = K12 (K22 + 1e-4 I)^-1 and d11 - rowsum(P o K12) (code/utils.py:117-120)."""
    A = K22.clone()
    A.diagonal().add_(JIT)
    _, Ci = _chol_inv_checked(A, "K22")
    Ainv = H.matmul(Ci, Ci, transA=True, maskA=L.A_UPPER, maskB=L.B_LOWER)
    P = H.matmul(K12, Ainv)
    return P, d11 - (P * K12).sum(1)


def _sampling_setup(model, x):
    """Everything the samples share: P, means and variances of the three RBF-prior GPs (the pair
    marginals do not depend on the sample), the Cholesky factor of Sigma_v, tril(sqrt_W)."""
    dev = model.device_
    D, M = model.D, model.M
    Z = model.Z
    p = {k: getattr(model, k).detach().to(F64) for k in ["mu_W", "sqrt_W", "mu_v", "sqrt_v"]}
    p["mu_U"] = model.mu_U_dense().to(F64)
    hyp = {k: float(torch.exp(getattr(model, k).detach().to(F64))) for k in
           ["sigma2_tildeell_log", "length_scales_tildeell_log", "sigma2_L0_log", "length_scales_L0_log",
            "sigma2_L1_log", "length_scales_L1_log", "sigma2_err_log"]}
    N = x.shape[0]

    def rbf(a, b, s2, ls):
        return H.pairwise(a, b, mode=L.RBF, scale2=s2, length_scale=ls)

    st = {"N": N, "D": D, "M": M, "Z": Z, "x": x, "mu_W": p["mu_W"], "s2_err": hyp["sigma2_err_log"]}
    Kt12 = rbf(x, Z, hyp["sigma2_tildeell_log"], hyp["length_scales_tildeell_log"])
    Kt22 = rbf(Z, Z, hyp["sigma2_tildeell_log"], hyp["length_scales_tildeell_log"])
    st["Pt"], st["var_t"] = _proj_var(Kt12, Kt22, torch.full((N,), hyp["sigma2_tildeell_log"], dtype=F64,
                                                              device=dev))
    # v ~ N(mu_v, Sigma_v): chol(Sigma_v + 1e-4 I) (code/utils.py:40-47, 225-226)
    lv = _tril(p["sqrt_v"])
    Sv = H.matmul(lv, lv, transB=True, maskA=L.A_LOWER, maskB=L.B_UPPER)
    Sv.diagonal().add_(JIT)
    st["Cv"], _ = _chol_inv_checked(Sv, "Sigma_v")
    st["mu_v"] = p["mu_v"]
    # pair marginals (code/utils.py:106-125): mean P mu_ij, variance d - rowsum(P o K12) +
    # rowsum((P tril(S_ij))^2)  (= rowsum((P Sigma_ij) o P) since Sigma_ij = tril(S) tril(S)^T)
    K012 = rbf(x, Z, hyp["sigma2_L0_log"], hyp["length_scales_L0_log"])
    K022 = rbf(Z, Z, hyp["sigma2_L0_log"], hyp["length_scales_L0_log"])
    K112 = rbf(x, Z, hyp["sigma2_L1_log"], hyp["length_scales_L1_log"])
    K122 = rbf(Z, Z, hyp["sigma2_L1_log"], hyp["length_scales_L1_log"])
    P0, b0 = _proj_var(K012, K022, torch.full((N,), hyp["sigma2_L0_log"], dtype=F64, device=dev))
    P1, b1 = _proj_var(K112, K122, torch.full((N,), hyp["sigma2_L1_log"], dtype=F64, device=dev))
    pairs = [(i, j) for i in range(D) for j in range(i + 1)]
    mus, sds = [], []
    for (i, j) in pairs:
        P, base = (P1, b1) if i == j else (P0, b0)
        mus.append(H.matmul(P, p["mu_U"][i, j].reshape(M, 1).contiguous()).reshape(N))
        PL = H.matmul(P, _tril(model.sqrt_U_pair(i, j).detach().to(F64)).contiguous(), maskB=L.B_LOWER)
        sds.append(torch.sqrt(base + (PL * PL).sum(1) + JIT))
    st["pairs"], st["pair_mu"], st["pair_sd"] = pairs, torch.stack(mus), torch.stack(sds)   # (Q, N)
    st["lW"] = _tril(p["sqrt_W"]).contiguous()                           # (D, M, M)
    return st


def _sample_chunk(st, zc, fy):
    """S samples from their noise block zc (S, per-sample noise).  Returns t (S,N), Lfull (S,D,D,N),
    G (S,D,N) and the F-noise (S, N) or (S, N, D)."""
    N, D, M = st["N"], st["D"], st["M"]
    Q = len(st["pairs"])
    S = zc.shape[0]
    o = 0
    z_v = zc[:, o:o + M]; o += M
    z_t = zc[:, o:o + N]; o += N
    z_p = zc[:, o:o + Q * N].reshape(S, Q, N); o += Q * N
    z_g = zc[:, o:o + D * N].reshape(S, D, N); o += D * N
    z_f = zc[:, o:].reshape(S, N, D) if fy else zc[:, o:o + N]
    # v = mu_v + chol(Sigma_v + 1e-4 I) z_v ; t = P_t v + sqrt(var_t + 1e-4) z_t   (JGP_S)
    V = st["mu_v"].reshape(1, M) + H.matmul(z_v.contiguous(), st["Cv"], transB=True, maskB=L.B_UPPER)
    T = H.matmul(V, st["Pt"], transB=True) + torch.sqrt(st["var_t"] + JIT).reshape(1, N) * z_t
    # pair samples (S, Q, N); the diagonal pairs are log L_ii
    Ls = st["pair_mu"].unsqueeze(0) + st["pair_sd"].unsqueeze(0) * z_p
    Lfull = torch.zeros(S, D, D, N, dtype=F64, device=V.device)
    for q, (i, j) in enumerate(st["pairs"]):
        Lfull[:, i, j] = torch.exp(Ls[:, q]) if i == j else Ls[:, q]
    # G | ell  (MGP_d with the sample's Gibbs kernel; code/nmgp_dsvi.py:468-472)
    ellZ, ellX = torch.exp(V), torch.exp(T)
    KG12 = torch.empty(S, N, M, dtype=F64, device=V.device)
    KG22 = torch.empty(S, M, M, dtype=F64, device=V.device)
    descs = []
    for s_ in range(S):
        descs.append(H.pairwise_desc(KG12[s_], st["x"], st["Z"], mode=L.GIBBS, ellX=ellX[s_], ellZ=ellZ[s_]))
        descs.append(H.pairwise_desc(KG22[s_], st["Z"], st["Z"], mode=L.GIBBS, ellX=ellZ[s_], ellZ=ellZ[s_]))
    H.PairwiseGroup(descs, V.device)(F64)
    A = KG22.clone()
    A.diagonal(dim1=1, dim2=2).add_(JIT)
    _, Ci = _chol_inv_checked(A, "K_G22")
    Ainv = H.bmm(Ci, Ci, transA=True, maskA=L.A_UPPER, maskB=L.B_LOWER)
    PG = H.bmm(KG12, Ainv)                                               # (S, N, M)
    mu_g = H.bmm(PG, st["mu_W"].contiguous(), transB=True)              # (S, N, D)
    var0 = 1.0 - (PG * KG12).sum(2)                                      # (S, N)
    var_g = torch.empty(S, D, N, dtype=F64, device=V.device)
    for d in range(D):
        PL = H.bmm(PG, st["lW"][d], maskB=L.B_LOWER)
        var_g[:, d] = var0 + (PL * PL).sum(2)
    G = mu_g.transpose(1, 2) + torch.sqrt(var_g + JIT) * z_g           # (S, D, N)
    return T, Lfull, G, z_f


def _chunk_size(n_sample, N, M):
    return max(1, min(n_sample, (1 << 25) // max(1, N * M)))


def sample_Y(model, X_list, n_sample=1000, index=None, noise_tape=None):
    """NMGP.sample_Y (code/nmgp_dsvi.py:406-490) on the device -> (Ys (S, N), Ls (S, N, D),
    Gs (S, D, N), tilde_ells (S, N)), torch tensors on the model's device."""
    dev = model.device_
    xs = [torch.as_tensor(x).reshape(-1).to(F64) for x in X_list]
    ids = list(range(len(xs))) if index is None else list(index)
    I = torch.cat([torch.full((x.shape[0],), int(j), dtype=torch.long) for x, j in zip(xs, ids)]).to(dev)
    x = torch.cat(xs).to(dev).reshape(-1, 1).contiguous()
    st = _sampling_setup(model, x)
    N, D, M = st["N"], st["D"], st["M"]
    per = M + N + len(st["pairs"]) * N + D * N + N
    draws = _Draws(dev, noise_tape)
    sd_err = (st["s2_err"] + JIT) ** 0.5
    rows = torch.arange(N, device=dev)
    Ys, Ls, Gs, Ts = [], [], [], []
    done = 0
    while done < n_sample:
        S = min(_chunk_size(n_sample, N, M), n_sample - done)
        T, Lfull, G, z_f = _sample_chunk(st, draws.take(S, per), fy=False)
        l = Lfull.permute(0, 3, 1, 2)[:, rows, I]                       # (S, N, D): row I_n of L
        F = (l * G.transpose(1, 2)).sum(2)
        Ys.append(F + sd_err * z_f), Ls.append(l), Gs.append(G), Ts.append(T)
        done += S
    return torch.cat(Ys), torch.cat(Ls), torch.cat(Gs), torch.cat(Ts)


def sample_FY(model, x, n_sample=1000, noise_tape=None):
    """NMGP.sample_FY (code/nmgp_dsvi.py:492-580) on the device -> (tilde_ells (S, N),
    Ys (S, N, D), corrs (S, N, D, D))."""
    dev = model.device_
    x = torch.as_tensor(x).reshape(-1, 1).to(F64).to(dev).contiguous()
    st = _sampling_setup(model, x)
    N, D, M = st["N"], st["D"], st["M"]
    per = M + N + len(st["pairs"]) * N + D * N + N * D
    draws = _Draws(dev, noise_tape)
    sd_err = (st["s2_err"] + JIT) ** 0.5
    Ts, Ys, Cs = [], [], []
    done = 0
    while done < n_sample:
        S = min(_chunk_size(n_sample, N, M), n_sample - done)
        T, Lfull, G, z_f = _sample_chunk(st, draws.take(S, per), fy=True)
        Ln = Lfull.permute(0, 3, 1, 2)                                   # (S, N, D, D)
        F = torch.matmul(Ln, G.transpose(1, 2).unsqueeze(3))[..., 0]     # (S, N, D)
        cov = torch.matmul(Ln, Ln.transpose(2, 3))
        invstd = torch.sqrt(torch.diag_embed(1.0 / torch.diagonal(cov, dim1=-2, dim2=-1)))
        Ts.append(T), Ys.append(F + sd_err * z_f), Cs.append(torch.matmul(torch.matmul(invstd, cov), invstd))
        done += S
    return torch.cat(Ts), torch.cat(Ys), torch.cat(Cs)
