"""Where fp32 arithmetic loses the ECoG-like fixture (M = 1024, length scales 3/M): CPU emulations on the
oracle (analysis only, ~5 min; run by hand: python tests/analysis/ecog_hyper_sensitivity.py).

Each experiment re-runs the oracle's fp64 forward/backward (or compute_ELBO) with ONE quantity rounded to
fp32 and prints the relative error against the reference's fixture:

  inputs      parameters, data, z and noise rounded to fp32, all arithmetic fp64: the error any fp32
              engine inherits (loss 7.6e-7, hyper-gradients <= 7e-5, ELBO samples <= 8e-5);
  adjoints    the gradient of one prior kernel matrix (K_t12, K_t22, K_G12, K_G22, K_L*) rounded to fp32
              before the hyper-parameter contraction: K_t12 alone leaves sigma2_tildeell_log 14% off,
              K_t22 6% -- the sums of K-bar o dK/dtheta over K12 and K22 cancel to ~1e-7 of their terms
              (K12 - P K22 = 1e-4 P), so the t prior's adjoint chain must be fp64 (engine: t64 path);
              K_G12 / K_G22 / the L priors stay below 1e-3;
  v sample    Sigma_v + 1e-4 I factored and applied in fp32: compute_ELBO samples 1.3e-3 off (exp(v)
              turns v's absolute error into relative error of every Gibbs length scale) -- the fp32
              engine samples v from an fp64 factor;
  products    P rounded to fp32 and P mu, P Sigma P^T in fp32: 1.5e-7 (harmless).
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import nmgp_oracle as O  # noqa: E402
from tests import _golden as G  # noqa: E402

HYP = ["sigma2_tildeell_log", "length_scales_tildeell_log", "sigma2_L0_log", "length_scales_L0_log",
       "sigma2_L1_log", "length_scales_L1_log", "sigma2_err_log"]
g = G.load("ecog_like_forward")
xs, ys = G.split_lists(g)
N = float(g["N"])
r32 = lambda a: np.asarray(a, np.float64).astype(np.float32).astype(np.float64)
f32 = lambda t: t.float().double()
_orig = {k: getattr(O, k) for k in ("create_RBF", "create_Gibbs", "JGP_S")}


def restore():
    for k, v in _orig.items():
        setattr(O, k, v)


def grad_errors(round_inputs=False):
    p = G.params(g, D=4, M=1024, requires_grad=True)
    xx, yy, z, nz = xs, ys, g["z"], g["noise"]
    if round_inputs:
        with torch.no_grad():
            for k in p:
                p[k].copy_(f32(p[k]))
        xx, yy, z, nz = [r32(x) for x in xs], [r32(y) for y in ys], r32(z), r32(nz)
    loss, _ = O.forward(p, xx, yy, z, N, O.TapeNoise(nz))
    loss.backward()
    out = {"loss": abs(float(loss.detach()) - float(g["loss"])) / abs(float(g["loss"]))}
    for k in HYP:
        out[k] = abs(abs(float(p[k].grad.reshape(-1)[0])) - float(g["gnorm_" + k])) / float(g["gnorm_" + k])
    return out


def elbo_errors(round_inputs=False):
    p = G.params(g, D=4, M=1024)
    xx, yy, z, nz = xs, ys, g["z"], g["elbo_noise"]
    if round_inputs:
        p = {k: f32(v) for k, v in p.items()}
        xx, yy, z, nz = [r32(x) for x in xs], [r32(y) for y in ys], r32(z), r32(nz)
    with torch.no_grad():
        _, lps = O.compute_ELBO(p, xx, yy, z, N, O.TapeNoise(nz), n_sample=int(g["elbo_n_sample"]))
    ref = g["elbo_logprob_per_sample"]
    return {"elbo_samples": list(np.abs(lps.numpy() - ref) / np.abs(ref))}


def fmt(d):
    return {k: ([f"{u:.2e}" for u in v] if isinstance(v, list) else f"{v:.2e}") for k, v in d.items()}


def round_adjoint(which):
    """Round the adjoint of the named kernel matrices to fp32 (gradient hook on the builder output)."""
    names_rbf = ["t12", "t22", "L012", "L022", "L112", "L122"]
    cnt = {"rbf": 0}

    def rbf(*a, **k):
        K = _orig["create_RBF"](*a, **k)
        nm = names_rbf[cnt["rbf"] % 6]
        cnt["rbf"] += 1
        if nm in which and K.requires_grad:
            K.register_hook(f32)
        return K

    def gib(X, X2, *a, **k):
        K = _orig["create_Gibbs"](X, X2, *a, **k)
        nm = "G22" if X is X2 else "G12"
        if nm in which and K.requires_grad:
            K.register_hook(f32)
        return K
    O.create_RBF, O.create_Gibbs = rbf, gib


def v_sample_fp32():
    def JGP_S(K11_diag, K12, K22, mu, Sigma, noise):
        z_v = noise(mu.numel())
        C = torch.linalg.cholesky(Sigma.float() + O.eye_jitter(Sigma.shape[0]).float())
        v = (mu.float() + (C @ z_v.float().unsqueeze(-1))[..., 0]).double()
        P = O._proj(K12, K22)
        mu_Y = (P @ v.unsqueeze(-1))[..., 0]
        s2 = K11_diag - torch.sum(P * K12, 1)
        z = noise(mu_Y.numel())
        return torch.cat([O.reparameterize(mu_Y, s2, z), v])
    O.JGP_S = JGP_S


if __name__ == "__main__":
    print("exact (oracle vs reference)", fmt(grad_errors()), flush=True)
    print("inputs rounded to fp32", fmt({**grad_errors(True), **elbo_errors(True)}), flush=True)
    for which in ({"t12"}, {"t22"}, {"G12"}, {"G22"}, {"L012", "L022", "L112", "L122"}):
        round_adjoint(which)
        print("adjoint of", sorted(which), "in fp32", fmt(grad_errors()), flush=True)
        restore()
    v_sample_fp32()
    print("v sample in fp32", fmt(elbo_errors()), flush=True)
    restore()
