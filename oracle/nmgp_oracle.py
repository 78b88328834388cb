"""CPU ORACLE for the DSVI hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity checker and the CPU baseline, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it; the shipped
package (``collaborative_nonstationary_multivariate_gaussian_process_amd``) never does, and it
fails loudly when its HIP library is missing instead of falling back to anything here.

What it is: a torch-CPU float64 restatement of the reference's DSVI step, written op for op in
the same order and with the same redundancy as the reference (per-pair LU solves, all D*D
blocks of Sigma_U, every pair sampled at every row), so that (a) it reproduces the reference to
~1e-13 relative and (b) its CPU speed stands in for the reference's on the GPU box, where the
reference itself cannot travel.  Every function cites the reference file:line it restates.
It is pinned against the golden vectors in ``tests/golden/*.npz`` (generated from the real
reference by ``tests/golden/make_golden.py``) by ``tests/test_oracle_golden.py``.

Reference quirks reproduced on purpose:
  * KL term2 uses ``triangular_solve(..., upper=True)`` on a LOWER factor -> only diag(L2) used
    (``code/utils.py:349``);
  * ``compute_ELBO`` gathers a COLUMN of L (``permute(2,1,0)``, ``code/nmgp_dsvi.py:361``) and
    takes KL_W from the last sample's K_G22 (``:385``);
  * LU solve (``torch.solve`` -> ``torch.linalg.solve``) on the SPD K22 (``code/utils.py:119``);
  * noise drawn as float32 ``torch.randn`` then cast to float64 (``code/utils.py:123,226,234``).
"""
import math

import numpy as np
import torch

DT = torch.float64
JITTER = 1e-4            # code/utils.py:7  tridiagonal_jitter
LEGACY_JITTER = 1e-6     # code/SIM_code/Utility/settings.py:3

PARAM_NAMES = ["mu_W", "sqrt_W", "mu_v", "sqrt_v", "mu_U", "sqrt_U",
               "sigma2_tildeell_log", "length_scales_tildeell_log", "sigma2_L0_log",
               "length_scales_L0_log", "sigma2_L1_log", "length_scales_L1_log", "sigma2_err_log"]


# ============================================================================ noise sources
class TorchNoise:
    """The reference's own stream: float32 ``torch.randn(size)`` cast to float64."""

    def __call__(self, n):
        return torch.randn(n).to(DT)


class TapeNoise:
    """Replays a flat float64 vector of injected noise in call order."""

    def __init__(self, flat):
        self.flat = torch.as_tensor(np.asarray(flat, np.float64))
        self.pos = 0

    def __call__(self, n):
        out = self.flat[self.pos:self.pos + n].clone()
        assert out.numel() == n, "noise tape exhausted"
        self.pos += n
        return out

    def done(self):
        return self.pos == self.flat.numel()


# ============================================================================ code/utils.py
def eye_jitter(n, jitter=JITTER):
    return torch.eye(n, dtype=DT) * jitter


def reparameterize(mean, var, z, full_cov=False, use_std=False):
    """code/utils.py:15-65."""
    if var is None:
        return mean
    if not full_cov:
        return mean + z * (var + JITTER) ** 0.5
    n = mean.shape[-1]
    chol = var if use_std else torch.linalg.cholesky(var + eye_jitter(n))
    return mean + torch.matmul(chol, z.unsqueeze(-1))[..., 0]


def mat2ltri(X):
    """code/utils.py:68-72: zero the strict upper triangle of the trailing two dims."""
    return torch.tril(X)


def _sqdist(X, X2):
    """code/utils.py:75-81 (difference form, summed over the feature dim)."""
    diff = X.unsqueeze(1) - X2.unsqueeze(0)
    return (diff * diff).sum(-1)


def create_RBF(X, X2=None, scale2=1., length_scales=1.):
    """code/utils.py:84-94: divide by the length scale, then difference."""
    Xs = X / length_scales
    X2s = Xs if X2 is None else X2 / length_scales
    return scale2 * torch.exp(-0.5 * _sqdist(Xs, X2s))


def create_Gibbs(X, X2, ell_X, ell_X2, scale2=1.):
    """code/utils.py:97-103: Gibbs / nonstationary RBF."""
    r2 = _sqdist(X, X2)
    S = (ell_X ** 2).unsqueeze(1) + (ell_X2 ** 2).unsqueeze(0)
    C = torch.sqrt(2 * (ell_X.unsqueeze(1) * ell_X2.unsqueeze(0)) / S)
    return scale2 * C * torch.exp(-r2 / S)


def _proj(K12, K22):
    """P = K12 (K22 + 1e-4 I)^-1 by LU, as code/utils.py:117-119."""
    A = K22 + eye_jitter(K22.shape[0])
    return torch.linalg.solve(A, K12.t()).t()


def MGP_d(K12, K22, d11, mu, Sigma, noise):
    """code/utils.py:106-125: sample the marginalised element-wise GP."""
    P = _proj(K12, K22)
    mu_Y = torch.matmul(P, mu.unsqueeze(-1))[..., 0]
    s2 = d11 - (P * K12).sum(-1) + (P.matmul(Sigma) * P).sum(-1)
    z = noise(mu_Y.numel()).reshape(mu_Y.shape)
    return reparameterize(mu_Y, s2, z)


def MGP_mu_sigma2(K12, K22, d11, mu, Sigma):
    """code/utils.py:128-146."""
    P = _proj(K12, K22)
    mu_Y = torch.matmul(P, mu.unsqueeze(-1))[..., 0]
    s2 = d11 - (P * K12).sum(-1) + (P.matmul(Sigma) * P).sum(-1)
    return mu_Y, s2


def MGP_mu(K12, K22, mu):
    """code/utils.py:149-157."""
    return torch.matmul(_proj(K12, K22), mu.unsqueeze(-1))[..., 0]


def JGP_S(K11_diag, K12, K22, mu, Sigma, noise):
    """code/utils.py:216-237: sample v ~ N(mu, Sigma), then independent rows given v."""
    z_v = noise(mu.numel())
    v = reparameterize(mu, Sigma, z_v, full_cov=True)
    P = _proj(K12, K22)
    mu_Y = torch.matmul(P, v.unsqueeze(-1))[..., 0]
    s2 = K11_diag - torch.sum(P * K12, 1)
    z = noise(mu_Y.numel())
    return torch.cat([reparameterize(mu_Y, s2, z), v])


def Normal_logprob(loc, scale, y):
    """code/utils.py:268-272."""
    var = scale ** 2
    return torch.sum(-((y - loc) ** 2) / (2 * var) - torch.log(scale) - math.log(math.sqrt(2 * math.pi)))


def KL_Gaussian(X_mu, X_Sigma, X2_mu, X2_Sigma):
    """code/utils.py:275-351, including the upper=True quirk of the trace term (:349)."""
    n = X_mu.shape[-1]
    A1 = X_Sigma + eye_jitter(n)
    A2 = X2_Sigma + eye_jitter(n)
    half1 = torch.linalg.cholesky(A2).diagonal(dim1=-2, dim2=-1).log().sum(-1) - \
        torch.linalg.cholesky(A1).diagonal(dim1=-2, dim2=-1).log().sum(-1)
    L1 = torch.linalg.cholesky(A1)
    L2 = torch.linalg.cholesky(A2)
    # triangular_solve(input=L1, A=L2) with the default upper=True: only triu(L2) = diag(L2) is read
    X = torch.linalg.solve_triangular(torch.triu(L2).expand(L1.shape), L1, upper=True)
    term2 = X.pow(2).sum((-2, -1))
    diff = (X2_mu - X_mu).reshape(-1, n)          # batch_mahalanobis (code/utils.py:290-329), one L
    sol = torch.linalg.solve_triangular(L2, diff.t(), upper=False)
    term3 = sol.pow(2).sum(-2).reshape(X_mu.shape[:-1])
    return half1 + 0.5 * (term2 + term3 - n)


# ============================================================================ code/nmgp_dsvi.py
def new_params(D, M, seed=22):
    """NMGP.__init__ defaults (code/nmgp_dsvi.py:115-155): torch seed, then randn in order."""
    torch.random.manual_seed(seed)
    p = {"mu_W": 0.1 * torch.randn(D, M).to(DT), "sqrt_W": 0.1 * torch.randn(D, M, M).to(DT),
         "mu_v": -4 * torch.ones(M, dtype=DT), "sqrt_v": 0.1 * torch.randn(M, M).to(DT),
         "mu_U": 0.1 * torch.randn(D, D, M).to(DT), "sqrt_U": 0.1 * torch.randn(D, D, M, M).to(DT),
         "sigma2_tildeell_log": torch.tensor(0., dtype=DT), "length_scales_tildeell_log": torch.tensor(-4., dtype=DT),
         "sigma2_L0_log": torch.tensor(0., dtype=DT), "length_scales_L0_log": torch.tensor(-4., dtype=DT),
         "sigma2_L1_log": torch.tensor(0., dtype=DT), "length_scales_L1_log": torch.tensor(-4., dtype=DT),
         "sigma2_err_log": torch.tensor(-2., dtype=DT)}
    return p


def _covs(p):
    """code/nmgp_dsvi.py:172-177."""
    lW, lv, lU = mat2ltri(p["sqrt_W"]), mat2ltri(p["sqrt_v"]), mat2ltri(p["sqrt_U"])
    return (torch.matmul(lW, lW.permute(0, 2, 1)), torch.matmul(lv, lv.permute(1, 0)),
            torch.matmul(lU, lU.permute(0, 1, 3, 2)))


def _hyper(p):
    """code/nmgp_dsvi.py:180-188."""
    e = torch.exp
    return {"s2_t": e(p["sigma2_tildeell_log"]), "ls_t": e(p["length_scales_tildeell_log"]),
            "s2_0": e(p["sigma2_L0_log"]), "ls_0": e(p["length_scales_L0_log"]),
            "s2_1": e(p["sigma2_L1_log"]), "ls_1": e(p["length_scales_L1_log"]), "s2_err": e(p["sigma2_err_log"])}


def output_ids(sizes, index=None):
    """code/nmgp_dsvi.py:163-167: the output id of every concatenated row (bit-exact int64)."""
    ids = range(len(sizes)) if index is None else index
    return np.hstack([np.repeat(j, n) for n, j in zip(sizes, ids)]).astype(np.int64)


def _sample_core(p, Sigma_v, Sigma_U, h, Z, inputs, D, noise, n11_t):
    """The shared sampling body of forward / compute_ELBO (code/nmgp_dsvi.py:198-237, :334-360)."""
    B = inputs.shape[0]
    K_t11 = torch.ones(int(n11_t), dtype=DT) * h["s2_t"]
    K_t12 = create_RBF(inputs, Z, scale2=h["s2_t"], length_scales=h["ls_t"])
    K_t22 = create_RBF(Z, scale2=h["s2_t"], length_scales=h["ls_t"])
    vt = JGP_S(K_t11, K_t12, K_t22, p["mu_v"], Sigma_v, noise)
    t_ell, v = vt[:B], vt[B:]
    ell_Z, ell_X = torch.exp(v), torch.exp(t_ell)
    K_L0_11 = torch.ones(B, dtype=DT) * h["s2_0"]
    K_L0_12 = create_RBF(inputs, Z, scale2=h["s2_0"], length_scales=h["ls_0"])
    K_L0_22 = create_RBF(Z, scale2=h["s2_0"], length_scales=h["ls_0"])
    K_L1_11 = torch.ones(B, dtype=DT) * h["s2_1"]
    K_L1_12 = create_RBF(inputs, Z, scale2=h["s2_1"], length_scales=h["ls_1"])
    K_L1_22 = create_RBF(Z, scale2=h["s2_1"], length_scales=h["ls_1"])
    L = torch.zeros(D, D, B, dtype=DT)
    pair_samples = []
    for i in range(D):
        for j in range(i + 1):
            if i == j:
                s = MGP_d(K_L1_12, K_L1_22, K_L1_11, p["mu_U"][i, j], Sigma_U[i, j], noise)
                L[i, j, :] = torch.exp(s)
            else:
                s = MGP_d(K_L0_12, K_L0_22, K_L0_11, p["mu_U"][i, j], Sigma_U[i, j], noise)
                L[i, j, :] = s
            pair_samples.append(s)
    return dict(K_t12=K_t12, K_t22=K_t22, t_ell=t_ell, v=v, ell_Z=ell_Z, ell_X=ell_X, K_L0_12=K_L0_12,
                K_L0_22=K_L0_22, K_L1_12=K_L1_12, K_L1_22=K_L1_22, L=L, pair_samples=pair_samples)


def _kl_terms(p, Sigma_W, Sigma_v, Sigma_U, K_G22, K_t22, K_L0_22, K_L1_22, D, M):
    """code/nmgp_dsvi.py:266-295 (and :385-402)."""
    zero = torch.zeros(M, dtype=DT)
    KL_W = KL_Gaussian(p["mu_W"], Sigma_W, zero, K_G22).sum()
    KL_v = KL_Gaussian(p["mu_v"], Sigma_v, zero, K_t22)
    mu1 = torch.stack([p["mu_U"][i, i] for i in range(D)])
    S1 = torch.stack([Sigma_U[i, i] for i in range(D)])
    mu0 = torch.cat([p["mu_U"][i, :i].reshape(i, M) for i in range(1, D)])
    S0 = torch.cat([Sigma_U[i, :i].reshape(i, M, M) for i in range(1, D)])
    KL_U = KL_Gaussian(mu1, S1, zero, K_L1_22).sum() + KL_Gaussian(mu0, S0, zero, K_L0_22).sum()
    return KL_W, KL_v, KL_U


def forward(p, x_list, y_list, z, N, noise, index=None):
    """NMGP.forward (code/nmgp_dsvi.py:157-301): returns (-SELBO, intermediates).

    ``p`` maps the 13 parameter names to float64 tensors (leaf tensors with requires_grad for
    gradients); ``x_list``/``y_list`` are per-output 1-D arrays; ``noise`` a TorchNoise/TapeNoise.
    """
    D, M = p["mu_W"].shape
    sizes = [int(np.asarray(x).reshape(-1).shape[0]) for x in x_list]
    I = output_ids(sizes, index)
    rows = torch.from_numpy(np.arange(I.shape[0]))
    cols = torch.from_numpy(I)
    inputs = torch.cat([torch.as_tensor(np.asarray(x, np.float64)).reshape(-1) for x in x_list]).view(-1, 1)
    outputs = torch.cat([torch.as_tensor(np.asarray(y, np.float64)).reshape(-1) for y in y_list]).view(-1, 1)
    Z = torch.as_tensor(np.asarray(z, np.float64)).reshape(-1, 1)
    Sigma_W, Sigma_v, Sigma_U = _covs(p)
    h = _hyper(p)
    B = inputs.shape[0]
    c = _sample_core(p, Sigma_v, Sigma_U, h, Z, inputs, D, noise, B)
    l = c["L"].permute(2, 0, 1)[rows, cols]                      # row I_n of L  (nmgp_dsvi.py:238)
    K_G12 = create_Gibbs(inputs, Z, c["ell_X"], c["ell_Z"], scale2=1)
    K_G22 = create_Gibbs(Z, Z, c["ell_Z"], c["ell_Z"], scale2=1)
    mu_g, s2_g = MGP_mu_sigma2(K_G12, K_G22, torch.ones(B, dtype=DT), p["mu_W"], Sigma_W)
    F = torch.sum(l * mu_g.t(), 1).view(-1, 1)
    R = Normal_logprob(F, torch.sqrt(h["s2_err"]), outputs)
    R = R - 0.5 / h["s2_err"] * (l ** 2 * s2_g.t()).sum()
    KL_W, KL_v, KL_U = _kl_terms(p, Sigma_W, Sigma_v, Sigma_U, K_G22, c["K_t22"], c["K_L0_22"], c["K_L1_22"], D, M)
    selbo = N / B * R - KL_W - KL_v - KL_U
    c.update(l=l, K_G12=K_G12, K_G22=K_G22, mu_g=mu_g, sigma2_g=s2_g, SELBO_R=R, KL_W=KL_W, KL_v=KL_v, KL_U=KL_U)
    return -selbo, c


def compute_ELBO(p, x_list, y_list, z, N, noise, n_sample=1000, index=None):
    """NMGP.compute_ELBO (code/nmgp_dsvi.py:303-404), detached, with the column-gather quirk."""
    with torch.no_grad():
        D, M = p["mu_W"].shape
        sizes = [int(np.asarray(x).reshape(-1).shape[0]) for x in x_list]
        I = output_ids(sizes, index)
        rows, cols = torch.from_numpy(np.arange(I.shape[0])), torch.from_numpy(I)
        inputs = torch.cat([torch.as_tensor(np.asarray(x, np.float64)).reshape(-1) for x in x_list]).view(-1, 1)
        outputs = torch.cat([torch.as_tensor(np.asarray(y, np.float64)).reshape(-1) for y in y_list]).view(-1, 1)
        Z = torch.as_tensor(np.asarray(z, np.float64)).reshape(-1, 1)
        Sigma_W, Sigma_v, Sigma_U = _covs(p)
        h = _hyper(p)
        B = inputs.shape[0]
        lps = []
        for _ in range(n_sample):
            c = _sample_core(p, Sigma_v, Sigma_U, h, Z, inputs, D, noise, N)
            l = c["L"].permute(2, 1, 0)[rows, cols]                  # COLUMN I_n (nmgp_dsvi.py:361)
            K_G12 = create_Gibbs(inputs, Z, c["ell_X"], c["ell_Z"])
            K_G22 = create_Gibbs(Z, Z, c["ell_Z"], c["ell_Z"])
            mu_g, s2_g = MGP_mu_sigma2(K_G12, K_G22, torch.ones(B, dtype=DT), p["mu_W"], Sigma_W)
            F = torch.sum(l * mu_g.t(), 1).view(-1, 1)
            R = Normal_logprob(F, torch.sqrt(h["s2_err"]), outputs)
            R = R - 0.5 / h["s2_err"] * (l ** 2 * s2_g.t()).sum()
            lps.append(R)
        lps = torch.stack(lps)
        KL_W, KL_v, KL_U = _kl_terms(p, Sigma_W, Sigma_v, Sigma_U, K_G22, c["K_t22"], c["K_L0_22"], c["K_L1_22"], D, M)
        return torch.mean(lps) - KL_W - KL_v - KL_U, lps


def predict_Y(p, x_list, z, index=None):
    """NMGP.predict_Y (code/nmgp_dsvi.py:666-722): posterior-mean prediction."""
    with torch.no_grad():
        D, M = p["mu_W"].shape
        sizes = [int(np.asarray(x).reshape(-1).shape[0]) for x in x_list]
        I = output_ids(sizes, index)
        rows, cols = torch.from_numpy(np.arange(I.shape[0])), torch.from_numpy(I)
        inputs = torch.cat([torch.as_tensor(np.asarray(x, np.float64)).reshape(-1) for x in x_list]).view(-1, 1)
        Z = torch.as_tensor(np.asarray(z, np.float64)).reshape(-1, 1)
        h = _hyper(p)
        B = inputs.shape[0]
        K_t12 = create_RBF(inputs, Z, scale2=h["s2_t"], length_scales=h["ls_t"])
        K_t22 = create_RBF(Z, scale2=h["s2_t"], length_scales=h["ls_t"])
        v = p["mu_v"]
        t_ell = MGP_mu(K_t12, K_t22, v)
        ell_Z, ell_X = torch.exp(v), torch.exp(t_ell)
        K_L0_12 = create_RBF(inputs, Z, scale2=h["s2_0"], length_scales=h["ls_0"])
        K_L0_22 = create_RBF(Z, scale2=h["s2_0"], length_scales=h["ls_0"])
        K_L1_12 = create_RBF(inputs, Z, scale2=h["s2_1"], length_scales=h["ls_1"])
        K_L1_22 = create_RBF(Z, scale2=h["s2_1"], length_scales=h["ls_1"])
        L = torch.zeros(D, D, B, dtype=DT)
        for i in range(D):
            for j in range(i + 1):
                if i == j:
                    L[i, j] = torch.exp(MGP_mu(K_L1_12, K_L1_22, p["mu_U"][i, j]))
                else:
                    L[i, j] = MGP_mu(K_L0_12, K_L0_22, p["mu_U"][i, j])
        K_G12 = create_Gibbs(inputs, Z, ell_X, ell_Z)
        K_G22 = create_Gibbs(Z, Z, ell_Z, ell_Z)
        G = MGP_mu(K_G12, K_G22, p["mu_W"])
        Y = torch.matmul(L.permute(2, 0, 1), G.permute(1, 0).unsqueeze(2))[:, :, 0]
        return Y[rows, cols]


def sample_Y(p, x_list, z, noise, n_sample=1000, index=None):
    """NMGP.sample_Y (code/nmgp_dsvi.py:406-490): posterior-predictive samples of the observed
    outputs -> (Ys (S, N), Ls (S, N, D): row I_n of L, Gs (S, D, N), tilde_ells (S, N))."""
    with torch.no_grad():
        D, M = p["mu_W"].shape
        sizes = [int(np.asarray(x).reshape(-1).shape[0]) for x in x_list]
        I = output_ids(sizes, index)
        rows, cols = torch.from_numpy(np.arange(I.shape[0])), torch.from_numpy(I)
        inputs = torch.cat([torch.as_tensor(np.asarray(x, np.float64)).reshape(-1) for x in x_list]).view(-1, 1)
        Z = torch.as_tensor(np.asarray(z, np.float64)).reshape(-1, 1)
        Sigma_W, Sigma_v, Sigma_U = _covs(p)
        h = _hyper(p)
        N = inputs.shape[0]
        Ys, Ls, Gs, Ts = [], [], [], []
        for _ in range(n_sample):
            c = _sample_core(p, Sigma_v, Sigma_U, h, Z, inputs, D, noise, N)
            l = c["L"].permute(2, 0, 1)[rows, cols]                  # row I_n (nmgp_dsvi.py:466)
            K_G12 = create_Gibbs(inputs, Z, c["ell_X"], c["ell_Z"])
            K_G22 = create_Gibbs(Z, Z, c["ell_Z"], c["ell_Z"])
            G = MGP_d(K_G12, K_G22, torch.ones(N, dtype=DT), p["mu_W"], Sigma_W, noise)
            F = torch.sum(l * G.t(), 1)
            Y = reparameterize(F, torch.ones_like(F) * h["s2_err"], noise(N))
            Ys.append(Y), Ls.append(l), Gs.append(G), Ts.append(c["t_ell"])
        return torch.stack(Ys), torch.stack(Ls), torch.stack(Gs), torch.stack(Ts)


def sample_FY(p, x, z, noise, n_sample=1000):
    """NMGP.sample_FY (code/nmgp_dsvi.py:492-580): samples of all D outputs at x plus the implied
    correlation matrices -> (tilde_ells (S, N), Ys (S, N, D), corrs (S, N, D, D))."""
    with torch.no_grad():
        D, M = p["mu_W"].shape
        inputs = torch.as_tensor(np.asarray(x, np.float64)).reshape(-1, 1)
        Z = torch.as_tensor(np.asarray(z, np.float64)).reshape(-1, 1)
        Sigma_W, Sigma_v, Sigma_U = _covs(p)
        h = _hyper(p)
        N = inputs.shape[0]
        Ts, Ys, Cs = [], [], []
        for _ in range(n_sample):
            c = _sample_core(p, Sigma_v, Sigma_U, h, Z, inputs, D, noise, N)
            K_G12 = create_Gibbs(inputs, Z, c["ell_X"], c["ell_Z"])
            K_G22 = create_Gibbs(Z, Z, c["ell_Z"], c["ell_Z"])
            G = MGP_d(K_G12, K_G22, torch.ones(N, dtype=DT), p["mu_W"], Sigma_W, noise)
            Ln = c["L"].permute(2, 0, 1)                               # (N, D, D)
            F = torch.matmul(Ln, G.permute(1, 0).unsqueeze(2))[:, :, 0]
            Y = reparameterize(F, torch.ones_like(F) * h["s2_err"], noise(F.numel()).reshape(F.shape))
            cov = torch.matmul(Ln, c["L"].permute(2, 1, 0))
            invstd = torch.sqrt(torch.diag_embed(1. / torch.diagonal(cov, dim1=-2, dim2=-1)))
            Ts.append(c["t_ell"]), Ys.append(Y), Cs.append(torch.matmul(torch.matmul(invstd, cov), invstd))
        return torch.stack(Ts), torch.stack(Ys), torch.stack(Cs)


def adam_step(params, grads, state, lr, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam default update (code/nmgp_dsvi.py:777, :854), restated."""
    b1, b2 = betas
    state["step"] = state.get("step", 0) + 1
    t = state["step"]
    for k, g in grads.items():
        m = state.setdefault("m_" + k, torch.zeros_like(g))
        v = state.setdefault("v_" + k, torch.zeros_like(g))
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        params[k].data.addcdiv_(m, denom, value=-lr / bc1)


# ============================================================================ SIM_code/Utility
def pairwise_distances(x, y=None):
    """SIM_code/Utility/kernels.py:5-21 (expand form x^2 + y^2 - 2 x.y)."""
    xn = (x ** 2).sum(1).view(-1, 1)
    if y is None:
        y, yn = x, xn.view(1, -1)
    else:
        yn = (y ** 2).sum(1).view(1, -1)
    return xn + yn - 2.0 * torch.mm(x, y.t())


def RBF_cov(X1, X2=None, alpha=1., beta=1.):
    """SIM_code/Utility/kernels.py:24-43 (+1e-6 I when X2 is None)."""
    if X2 is None:
        X2 = X1
        cov = torch.eye(X1.shape[0], dtype=DT) * LEGACY_JITTER
    else:
        cov = torch.zeros(X1.shape[0], X2.shape[0], dtype=DT)
    return cov + torch.exp(-0.5 * pairwise_distances(X1 / beta, X2 / beta)) * alpha ** 2


def Nonstationary_RBF_cov(X1, sigma1=None, ell1=None, X2=None, sigma2=None, ell2=None):
    """SIM_code/Utility/kernels.py:46-73."""
    n1 = X1.shape[0]
    sigma1 = torch.ones(n1, dtype=DT) if sigma1 is None else sigma1
    ell1 = torch.ones(n1, dtype=DT) if ell1 is None else ell1
    if X2 is None:
        X2, sigma2, ell2 = X1, sigma1, ell1
        cov = torch.eye(n1, dtype=DT) * LEGACY_JITTER
    else:
        cov = torch.zeros(n1, X2.shape[0], dtype=DT)
    dist = pairwise_distances(X1, X2)
    A = (ell1 ** 2).view(-1, 1) + (ell2 ** 2).view(1, -1)
    Bm = ell1.view(-1, 1) * ell2.view(1, -1)
    C = sigma1.view(-1, 1) * sigma2.view(1, -1)
    return cov + C * torch.sqrt(2. * Bm / A) * torch.exp(-dist / A)


def kronecker_product(t1, t2):
    """SIM_code/Utility/kronecker_operation.py:5-22: out[i*r2+k, j*c2+l] = t1[i,j] * t2[k,l]."""
    r1, c1 = t1.shape
    r2, c2 = t2.shape
    return (t1[:, None, :, None] * t2[None, :, None, :]).reshape(r1 * r2, c1 * c2)


def kronecker_product_diag(d1, d2):
    """SIM_code/Utility/kronecker_operation.py:25-33."""
    return kronecker_product(d1.view(-1, 1), d2.view(-1, 1)).view(-1)


def kron_mv(B, K, y):
    """SIM_code/Utility/kronecker_operation.py:72-85: (B kron K) y via two GEMMs."""
    m, n = B.shape[1], K.shape[1]
    Y = y.view(m, n).t()
    return torch.mm(torch.mm(K, Y), B.t()).t().contiguous().view(-1)


def kron_inv(sigma2, B, K):
    """SIM_code/Utility/kronecker_operation.py:36-53 (symeig -> eigh)."""
    wB, vB = torch.linalg.eigh(B)
    wK, vK = torch.linalg.eigh(K)
    U = kronecker_product(vB, vK)
    t = kronecker_product_diag(wB, wK)
    return torch.mm(torch.mm(U, torch.diag(1. / (t + sigma2))), U.t())


def kron_logdet(sigma2, B, K):
    """SIM_code/Utility/kronecker_operation.py:56-69."""
    wB, _ = torch.linalg.eigh(B)
    wK, _ = torch.linalg.eigh(K)
    return torch.log(kronecker_product_diag(wB, wK) + sigma2).sum()


def multivariate_normal_logpdf0(y, mu, B, K, sigma2):
    """SIM_code/Utility/distributions.py:26-52 (unnormalised)."""
    wB, vB = torch.linalg.eigh(B)
    wK, vK = torch.linalg.eigh(K)
    a = kron_mv(vB.t(), vK.t(), y - mu)
    t = kronecker_product_diag(wB, wK)
    w = 1. / (sigma2 + t)
    return -0.5 * torch.log(t + sigma2).sum() - 0.5 * torch.dot(a * w, a)
