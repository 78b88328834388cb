"""Torch-CPU mirror of the HIP DSVI engine's closed-form forward/backward (test infrastructure).

The HIP engine does not run autograd: it evaluates -SELBO and ALL 13 parameter gradients in
closed form, deduplicated (4 prior factorisations instead of Q+2 LU solves, only the Q lower
coefficient pairs, quadratic forms only on the rows that use them).  This file is that exact
algorithm written with dense torch ops, step for step in the order of the engine's kernels, so
that (1) tests pin the math against the oracle's autograd gradients on CPU, and (2) GPU tests can
compare the engine's intermediates one kernel at a time.

Symbols (reference code/nmgp_dsvi.py:157-301): D outputs, M inducing points, B rows (grouped by
output), Q = D(D+1)/2 pairs (i, j<=i), lam = 1e-4 jitter, c = -N/B.
"""
import math

import numpy as np
import torch

LAM = 1e-4
DT = torch.float64


def pair_list(D):
    return [(i, j) for i in range(D) for j in range(i + 1)]


def rbf(x, z, s2, ls):
    d = x[:, None] / ls - z[None, :] / ls
    return s2 * torch.exp(-0.5 * d * d), d * d


def gibbs(x, z, ex, ez):
    r2 = (x[:, None] - z[None, :]) ** 2
    S = ex[:, None] ** 2 + ez[None, :] ** 2
    C = torch.sqrt(2 * (ex[:, None] * ez[None, :]) / S)
    return C * torch.exp(-r2 / S), r2, S


def gibbs_bwd(Kbar, K, r2, S, ex, ez):
    W = Kbar * K
    gx = (W * (1 / (2 * ex[:, None]) - ex[:, None] / S + 2 * ex[:, None] * r2 / S ** 2)).sum(1)
    gz = (W * (1 / (2 * ez[None, :]) - ez[None, :] / S + 2 * ez[None, :] * r2 / S ** 2)).sum(0)
    return gx, gz


def forward_backward(p, x, y, sizes, z, N, noise, pair_range=None, kl_owner=True):
    """Return (loss, grads dict, intermediates dict) with the engine's closed-form algorithm.

    p: dict of the 13 parameters (float64 tensors); x, y: (B,) concatenated rows grouped by output;
    sizes: rows per output; noise: flat (M + B + Q*B) in reference call order.
    pair_range=(i0, i1), kl_owner: one rank's share under pair sharding (engine.DsviEngine): rows only
    of outputs [i0, i1) (sizes of the others 0), only their pairs (noise Q_r x B in their order), and
    KL_W / KL_v only when kl_owner.  The shares' losses and gradients sum to the whole model's.
    """
    D, M = p["mu_W"].shape
    B = x.shape[0]
    i0, i1 = (0, D) if pair_range is None else pair_range
    pairs = [(i, j) for i in range(i0, i1) for j in range(i + 1)]
    Q = len(pairs)
    assert all(sizes[d] == 0 for d in range(D) if not i0 <= d < i1)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(int)
    I = np.concatenate([np.full(n, i) for i, n in enumerate(sizes)]).astype(int)
    z_v = noise[:M]
    z_t = noise[M:M + B]
    z_p = noise[M + B:].reshape(Q, B)
    c = -N / B
    eye = torch.eye(M, dtype=DT)
    # ---------------------------------------------------------------- F0 hyper-parameters
    e = lambda k: torch.exp(p[k])
    s2t, lst, s20, ls0, s21, ls1, s2e = (e("sigma2_tildeell_log"), e("length_scales_tildeell_log"), e("sigma2_L0_log"),
                                        e("length_scales_L0_log"), e("sigma2_L1_log"), e("length_scales_L1_log"),
                                        e("sigma2_err_log"))
    # ---------------------------------------------------------------- F1 RBF builders
    Kt12, rt12 = rbf(x, z, s2t, lst)
    Kt22, rt22 = rbf(z, z, s2t, lst)
    K012, r012 = rbf(x, z, s20, ls0)
    K022, r022 = rbf(z, z, s20, ls0)
    K112, r112 = rbf(x, z, s21, ls1)
    K122, r122 = rbf(z, z, s21, ls1)
    # ---------------------------------------------------------------- F2 variational factors
    LW = torch.tril(p["sqrt_W"])
    Lv = torch.tril(p["sqrt_v"])
    LU = torch.tril(p["sqrt_U"])
    facs = [LW[d] for d in range(D)] + [Lv] + [LU[i, j] for (i, j) in pairs]        # NF = D+1+Q
    mus = [p["mu_W"][d] for d in range(D)] + [p["mu_v"]] + [p["mu_U"][i, j] for (i, j) in pairs]
    A1 = torch.stack([L @ L.t() + LAM * eye for L in facs])
    # ---------------------------------------------------------------- F3/F4/F5 factorisations
    C1 = torch.linalg.cholesky(A1)
    C1inv = torch.linalg.inv(C1)
    A2 = {"t": Kt22 + LAM * eye, "0": K022 + LAM * eye, "1": K122 + LAM * eye}
    C2 = {k: torch.linalg.cholesky(v) for k, v in A2.items()}
    C2inv = {k: torch.linalg.inv(v) for k, v in C2.items()}
    Ainv = {k: C2inv[k].t() @ C2inv[k] for k in C2}
    # ---------------------------------------------------------------- F6 projections
    P = {"t": Kt12 @ Ainv["t"], "0": K012 @ Ainv["0"], "1": K112 @ Ainv["1"]}
    # ---------------------------------------------------------------- F7 v, ell_Z
    Cv = C1[D]
    v = p["mu_v"] + Cv @ z_v
    ellZ = torch.exp(v)
    # ---------------------------------------------------------------- F8 t-row
    mean_t = P["t"] @ v
    q_t = (P["t"] * Kt12).sum(1)
    var_t = s2t - q_t
    sd_t = torch.sqrt(var_t + LAM)
    ellX = torch.exp(mean_t + z_t * sd_t)
    # ---------------------------------------------------------------- F9 Gibbs prior
    KG22, rg22, Sg22 = gibbs(z, z, ellZ, ellZ)
    KG12, rg12, Sg12 = gibbs(x, z, ellX, ellZ)
    A2["G"] = KG22 + LAM * eye
    C2["G"] = torch.linalg.cholesky(A2["G"])
    C2inv["G"] = torch.linalg.inv(C2["G"])
    Ainv["G"] = C2inv["G"].t() @ C2inv["G"]
    P["G"] = KG12 @ Ainv["G"]
    # ---------------------------------------------------------------- F10 W GEMMs + Y
    WG = torch.stack([P["G"] @ LW[d] for d in range(D)])                        # (D,B,M)
    WP = torch.zeros(D, B, M, dtype=DT)                                           # WP[j][r] for pair (I_r, j)
    for (i, j) in pairs:
        typ = "1" if i == j else "0"
        rs = slice(off[i], off[i + 1])
        WP[j, rs] = P[typ][rs] @ LU[i, j]
    Y = {"G": Ainv["G"] @ p["mu_W"].t(), "t": Ainv["t"] @ p["mu_v"],
         "0": Ainv["0"] @ p["mu_U"].reshape(D * D, M).t(), "1": Ainv["1"] @ p["mu_U"].reshape(D * D, M).t()}
    # ---------------------------------------------------------------- F11 recon (per row)
    qG = (P["G"] * KG12).sum(1)
    q0 = (P["0"] * K012).sum(1)
    q1 = (P["1"] * K112).sum(1)
    m = P["G"] @ p["mu_W"].t()                                  # (B,D)
    g = 1 - qG[:, None] + (WG ** 2).sum(2).t()                  # (B,D)
    l = torch.zeros(B, D, dtype=DT)
    mup = torch.zeros(B, D, dtype=DT)
    s2p = torch.zeros(B, D, dtype=DT)
    sdp = torch.zeros(B, D, dtype=DT)
    zp = torch.zeros(B, D, dtype=DT)
    ptype1 = torch.zeros(B, D, dtype=torch.bool)
    for (i, j) in pairs:
        rs = slice(off[i], off[i + 1])
        typ = "1" if i == j else "0"
        mu_ij = p["mu_U"][i, j]
        mup[rs, j] = P[typ][rs] @ mu_ij
        s2k, qk = (s21, q1) if i == j else (s20, q0)
        s2p[rs, j] = s2k - qk[rs] + (WP[j, rs] ** 2).sum(1)
        sdp[rs, j] = torch.sqrt(s2p[rs, j] + LAM)
        zp[rs, j] = z_p[pairs.index((i, j)), rs]
        smp = mup[rs, j] + zp[rs, j] * sdp[rs, j]
        l[rs, j] = torch.exp(smp) if i == j else smp
        ptype1[rs, j] = i == j
    F = (l * m).sum(1)
    sc = torch.sqrt(s2e)
    var = sc * sc
    res = y - F
    R = (-(res ** 2) / (2 * var) - torch.log(sc) - math.log(math.sqrt(2 * math.pi))).sum() \
        - 0.5 / s2e * (l ** 2 * g).sum()
    # ---------------------------------------------------------------- F12 KL
    prior_of = ["G"] * D + ["t"] + ["1" if i == j else "0" for (i, j) in pairs]
    ycol = list(range(D)) + [None] + [i * D + j for (i, j) in pairs]
    wkl = [1.0 if kl_owner else 0.0] * (D + 1) + [1.0] * Q        # whose KL this share adds
    KL = []
    evec = []
    for f in range(len(facs)):
        k = prior_of[f]
        Cf = C1[f]
        a1d = (facs[f] ** 2).sum(1) + LAM
        c2d = torch.diagonal(C2[k])
        yf = Y[k] if ycol[f] is None else Y[k][:, ycol[f]]
        term3 = mus[f] @ yf
        KL.append(torch.log(c2d).sum() - torch.log(torch.diagonal(Cf)).sum() + 0.5 * ((a1d / c2d ** 2).sum() + term3 - M))
        evec.append(0.5 - 0.5 * a1d / c2d ** 2)
    KL = torch.stack(KL) * torch.tensor(wkl, dtype=DT)
    loss = c * R + KL.sum()
    # ================================================================= backward
    grads = {}
    Fbar = c * res / var
    mbar = Fbar[:, None] * l                                    # (B,D)
    gbar = c * (-(l ** 2) / (2 * s2e))
    lbar = Fbar[:, None] * m + c * (-(l * g) / s2e)
    sbar = torch.where(ptype1, lbar * l, lbar)                  # only j <= I_r meaningful
    s2pbar = sbar * zp / (2 * sdp.clamp_min(1e-300))
    valid = torch.zeros(B, D, dtype=torch.bool)
    for (i, j) in pairs:
        valid[off[i]:off[i + 1], j] = True
    sbar = torch.where(valid, sbar, torch.zeros_like(sbar))
    s2pbar = torch.where(valid, s2pbar, torch.zeros_like(s2pbar))
    # s2e adjoint
    dR_dsc = ((res ** 2) / sc ** 3 - 1 / sc).sum()
    dR_ds2e = dR_dsc / (2 * sc) + 0.5 / s2e ** 2 * (l ** 2 * g).sum()
    ebar = c * dR_ds2e * s2e
    # W-hat (in place scaling of the W rows) and P-bar initial rows
    WGh = 2 * gbar.t()[:, :, None] * WG
    WPh = 2 * s2pbar.t()[:, :, None] * WP
    cG = gbar.sum(1)
    c1 = torch.where(ptype1, s2pbar, torch.zeros_like(s2pbar)).sum(1)
    c0 = torch.where(ptype1, torch.zeros_like(s2pbar), s2pbar).sum(1)
    Pbar = {"G": mbar @ p["mu_W"] - cG[:, None] * KG12}
    Pbar["1"] = torch.zeros(B, M, dtype=DT)
    Pbar["0"] = torch.zeros(B, M, dtype=DT)
    for (i, j) in pairs:
        rs = slice(off[i], off[i + 1])
        typ = "1" if i == j else "0"
        Pbar[typ][rs] += sbar[rs, j][:, None] * p["mu_U"][i, j][None, :]
    Pbar["1"] -= c1[:, None] * K112
    Pbar["0"] -= c0[:, None] * K012
    # B2: GEMM1 + L-bar + mu-bar
    Pbar["G"] = Pbar["G"] + sum(WGh[d] @ LW[d].t() for d in range(D))
    for (i, j) in pairs:
        rs = slice(off[i], off[i + 1])
        typ = "1" if i == j else "0"
        Pbar[typ][rs] += WPh[j, rs] @ LU[i, j].t()
    gsW = torch.stack([P["G"].t() @ WGh[d] for d in range(D)])
    gsU = torch.zeros(D, D, M, M, dtype=DT)
    gmU = torch.zeros(D, D, M, dtype=DT)
    for (i, j) in pairs:
        rs = slice(off[i], off[i + 1])
        typ = "1" if i == j else "0"
        gsU[i, j] = P[typ][rs].t() @ WPh[j, rs]
        gmU[i, j] = P[typ][rs].t() @ sbar[rs, j]
    gmW = (P["G"].t() @ mbar).t()
    # B1: prior adjoints from KL
    Abar = {}
    for k in ["G", "t", "0", "1"]:
        fs = [f for f in range(len(facs)) if prior_of[f] == k and wkl[f]]
        if not fs:
            Abar[k] = torch.zeros(M, M, dtype=DT)
            continue
        delta = sum(evec[f] for f in fs)
        Ys = torch.stack([(Y[k] if ycol[f] is None else Y[k][:, ycol[f]]) for f in fs], 1)
        Abar[k] = C2inv[k].t() @ torch.diag(delta) @ C2inv[k] - 0.5 * Ys @ Ys.t()
    # B3/B4: solve backward
    Rm = {k: Pbar[k] @ Ainv[k] for k in ["G", "0", "1"]}
    for k in ["G", "0", "1"]:
        Abar[k] = Abar[k] - P[k].t() @ Rm[k]
    # B5: builder backward
    Kbar_G12 = Rm["G"] - cG[:, None] * P["G"]
    gx, gz1 = gibbs_bwd(Kbar_G12, KG12, rg12, Sg12, ellX, ellZ)
    gz2a, gz2b = gibbs_bwd(Abar["G"], KG22, rg22, Sg22, ellZ, ellZ)
    ellZbar = gz1 + gz2a + gz2b
    Kbar_012 = Rm["0"] - c0[:, None] * P["0"]
    Kbar_112 = Rm["1"] - c1[:, None] * P["1"]
    a0 = (Kbar_012 * K012).sum() + (Abar["0"] * K022).sum() + s20 * s2pbar[~ptype1].sum()
    b0 = (Kbar_012 * K012 * r012).sum() + (Abar["0"] * K022 * r022).sum()
    a1 = (Kbar_112 * K112).sum() + (Abar["1"] * K122).sum() + s21 * s2pbar[ptype1].sum()
    b1 = (Kbar_112 * K112 * r112).sum() + (Abar["1"] * K122 * r122).sum()
    # B6: t-row backward
    tbar = gx * ellX
    varbar = tbar * z_t / (2 * sd_t)
    Pbar["t"] = tbar[:, None] * v[None, :] - varbar[:, None] * Kt12
    vbar = P["t"].t() @ tbar
    # B7/B8
    Rm["t"] = Pbar["t"] @ Ainv["t"]
    Abar["t"] = Abar["t"] - P["t"].t() @ Rm["t"]
    Kbar_t12 = Rm["t"] - varbar[:, None] * P["t"]
    at = (Kbar_t12 * Kt12).sum() + (Abar["t"] * Kt22).sum() + s2t * varbar.sum()
    bt = (Kbar_t12 * Kt12 * rt12).sum() + (Abar["t"] * Kt22 * rt22).sum()
    # B9: v backward through reparameterisation + Cholesky of Sigma_v + lam I
    vbar = vbar + ellZbar * ellZ
    Cvinv = C1inv[D]
    w = Cv.t() @ vbar
    Phi = torch.tril(w[:, None] * z_v[None, :])
    Phi = Phi - 0.5 * torch.diag(torch.diagonal(Phi))
    Av = Cvinv.t() @ Phi @ Cvinv
    Lvbar = (Av + Av.t()) @ Lv
    # B10: KL gradients of the variational factors
    Lbar_kl = []
    for f in range(len(facs)):
        k = prior_of[f]
        Xf = C1inv[f] @ facs[f]
        wv = 1 / torch.diagonal(C2[k]) ** 2
        Lbar_kl.append(wkl[f] * (-C1inv[f].t() @ Xf + wv[:, None] * facs[f]))
    gsW = gsW + torch.stack(Lbar_kl[:D])
    gsv = Lvbar + Lbar_kl[D]
    for n_, (i, j) in enumerate(pairs):
        gsU[i, j] += Lbar_kl[D + 1 + n_]
        gmU[i, j] += Y["1" if i == j else "0"][:, i * D + j]
    gmW = gmW + Y["G"].t() if kl_owner else gmW
    gmv = vbar + Y["t"] if kl_owner else vbar
    grads = {"mu_W": gmW, "sqrt_W": torch.tril(gsW), "mu_v": gmv, "sqrt_v": torch.tril(gsv), "mu_U": gmU,
             "sqrt_U": torch.tril(gsU), "sigma2_tildeell_log": at, "length_scales_tildeell_log": bt,
             "sigma2_L0_log": a0, "length_scales_L0_log": b0, "sigma2_L1_log": a1, "length_scales_L1_log": b1,
             "sigma2_err_log": ebar}
    inter = dict(P=P, Ainv=Ainv, C2=C2, v=v, ellX=ellX, ellZ=ellZ, var_t=var_t, WG=WG, WP=WP, l=l, m=m, g=g,
                 KL=KL, R=R, Pbar=Pbar, Rm=Rm, Abar=Abar, ellZbar=ellZbar, tbar=tbar, KG12=KG12, KG22=KG22,
                 mbar=mbar, gbar=gbar, sbar=sbar, s2pbar=s2pbar, Y=Y)
    return loss, grads, inter
