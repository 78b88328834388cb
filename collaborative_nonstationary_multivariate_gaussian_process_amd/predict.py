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


def prepare_inputs(model, inputs_list, index=None):
    """Device copies of the prediction inputs (x as a column, the output id of every row): made once
    when the same test inputs are predicted every iteration (inference(X_test_list=...))."""
    dev = model.device_
    xs = [torch.as_tensor(x).reshape(-1).to(F64) for x in inputs_list]
    ids = list(range(len(xs))) if index is None else list(index)
    I = torch.cat([torch.full((x.shape[0],), int(j), dtype=torch.long) for x, j in zip(xs, ids)]).to(dev)
    x = torch.cat([t.to(dev) for t in xs]).reshape(-1, 1).contiguous()
    return x, I


class PredictPlan:
    """NMGP.predict_Y (code/nmgp_dsvi.py:666-722) for one fixed set of prediction inputs, in fp64.

    The four GP systems of the prediction -- the three RBF priors (tilde-ell, L0, L1) and the Gibbs prior,
    whose K22 needs only ell_Z = exp(mu_v) -- are built by ONE pairwise launch (K22 + 1e-4 I and the three
    RBF cross kernels) and factored by ONE batched fused Cholesky + inverse launch; each solve
    K12 (K22 + 1e-4 I)^{-1} rhs is K12 (C^-T (C^-1 rhs)).  Buffers and kernel descriptors are made once, the
    hyper-parameters and means are read from theta on the device when the plan runs, so with graph=True the
    whole prediction is one HIP graph replay (inference(X_test_list=...) predicts after every iteration,
    code/nmgp_dsvi.py:865-868).  `info_acc` keeps the largest Cholesky info word of every run since the
    plan was made (0: all factorizations succeeded)."""

    def __init__(self, model, prepared, graph=False):
        self.model = model
        self.x, self.I = prepared
        dev, D, M = model.device_, model.D, model.M
        Bn = self.x.shape[0]
        Z = model.Z.to(F64)
        self.Z = Z
        e = lambda *shape: torch.empty(*shape, dtype=F64, device=dev)
        self.K22, self.Ci, self.K12 = e(4, M, M), e(4, M, M), e(3, Bn, M)
        self.KG12, self.ellZ, self.ellX, self.hyp64 = e(Bn, M), e(M), e(Bn), e(7)
        self.info = torch.zeros(4, dtype=torch.int32, device=dev)
        self.info_acc = torch.zeros(4, dtype=torch.int32, device=dev)
        descs = [H.pairwise_desc(self.K22[k], Z, Z, mode=L.RBF, hyp=self.hyp64, hyp_off=2 * k, hyp_log=True,
                                 diag_add=JIT) for k in range(3)]
        descs.append(H.pairwise_desc(self.K22[3], Z, Z, mode=L.GIBBS, ellX=self.ellZ, ellZ=self.ellZ, diag_add=JIT))
        descs += [H.pairwise_desc(self.K12[k], self.x, Z, mode=L.RBF, hyp=self.hyp64, hyp_off=2 * k, hyp_log=True)
                  for k in range(3)]
        self.build = H.PairwiseGroup(descs, dev)
        self.build_g12 = H.PairwiseGroup([H.pairwise_desc(self.KG12, self.x, Z, mode=L.GIBBS, ellX=self.ellX,
                                                          ellZ=self.ellZ)], dev)
        self.rows = torch.arange(Bn, device=dev)
        self.diag = torch.eye(D, dtype=torch.bool, device=dev).reshape(-1)
        if model.packed:
            ii, jj = np.tril_indices(D)
            self.pair_ij = (torch.from_numpy(ii).to(dev), torch.from_numpy(jj).to(dev))
        self.graph, self.est = None, None
        if graph:
            cur = torch.cuda.current_stream(dev)
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                self._body()                    # warm-up: library load, GEMM paths, allocator pool
            cur.wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.est = self._body()

    def _solve(self, k, K12, rhs):
        """K12 (K22_k + 1e-4 I)^{-1} rhs = K12 C_k^-T (C_k^-1 rhs), C_k^-1 lower triangular."""
        Ck = self.Ci[k]
        y = H.matmul(Ck, rhs, maskA=L.A_LOWER)
        y = H.matmul(Ck, y, transA=True, maskA=L.A_UPPER)
        return H.matmul(K12, y)

    def _body(self):
        m = self.model
        D, M = m.D, m.M
        o = m._offs["sigma2_tildeell_log"][0]
        self.hyp64.copy_(m._theta.detach()[o:o + 7])
        mu_v = m.mu_v.detach().to(F64).reshape(-1)
        torch.exp(mu_v, out=self.ellZ)
        self.build(F64)                                                   # K22 + 1e-4 I (x4), K12 (x3)
        H.chol_inv_(self.K22, out=self.Ci, info=self.info)                 # one batched launch
        torch.maximum(self.info_acc, self.info, out=self.info_acc)
        t_ell = self._solve(0, self.K12[0], mu_v.reshape(-1, 1).contiguous()).reshape(-1)
        torch.exp(t_ell, out=self.ellX)
        if m.packed:
            muU = torch.zeros(D, D, M, dtype=F64, device=m.device_)
            muU[self.pair_ij] = m.mu_U.detach().to(F64)
        else:
            muU = m.mu_U.detach().to(F64)
        muU = muU.reshape(D * D, M).t().contiguous()                      # (M, D*D)
        L0 = self._solve(1, self.K12[1], muU)                             # (B, D*D)
        L1 = self._solve(2, self.K12[2], muU)
        self.build_g12(F64)                                               # K_G12 from ell_X, ell_Z
        Gm = self._solve(3, self.KG12, m.mu_W.detach().to(F64).t().contiguous())   # (B, D)
        Bn = self.x.shape[0]
        Lr = torch.where(self.diag, torch.exp(L1), L0).reshape(Bn, D, D)
        Lr = torch.tril(Lr)                                               # est_L[i, j] for j <= i
        rowsL = Lr[self.rows, self.I]                                     # (B, D): row I_n of L at n
        return (rowsL * Gm).sum(1)

    def __call__(self):
        """The posterior means (N,) of the current parameters (no host synchronisation)."""
        if self.graph is not None:
            self.graph.replay()
            return self.est
        return self._body()


def predict_mean(model, inputs_list, index=None, prepared=None, defer_check=False):
    """NMGP.predict_Y (code/nmgp_dsvi.py:666-722) -> (N,) device tensor, computed in fp64 (PredictPlan).

    The four Cholesky info words are checked at the end -- or, with defer_check=True, left to the model's
    next check_numerics() (the caller's existing synchronisation point).  `prepared`: the (x, I) of
    prepare_inputs."""
    plan = PredictPlan(model, prepared if prepared is not None else prepare_inputs(model, inputs_list, index))
    est = plan()
    if defer_check:
        model._pending_info.append(plan.info_acc)
    elif int(plan.info_acc.max().cpu()) != 0:
        raise torch.linalg.LinAlgError("cholesky: K22 + 1e-4 I is not positive-definite")
    return est


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
