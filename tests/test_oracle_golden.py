"""Pin the CPU oracle against the golden vectors generated from the real reference (CPU only)."""
import numpy as np
import pytest
import torch

from oracle import nmgp_oracle as O
from tests import _golden as G

FWD_CASES = ["toy_forward", "modelpt_forward", "mid_forward", "driver_hyper_forward"]


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm((a - b).reshape(-1)) / max(np.linalg.norm(b.reshape(-1)), 1e-300)


@pytest.mark.parametrize("case", FWD_CASES)
def test_forward_loss_grads_intermediates(case):
    g = G.load(case)
    xs, ys = G.split_lists(g)
    p = G.params(g, requires_grad=True)
    tape = O.TapeNoise(g["noise"])
    loss, c = O.forward(p, xs, ys, g["z"], float(g["N"]), tape)
    assert tape.done()
    loss.backward()
    assert abs(float(loss) - float(g["loss"])) <= 1e-12 * abs(float(g["loss"]))
    for k in O.PARAM_NAMES:
        assert _rel(p[k].grad, g["grad_" + k]) <= 1e-10 or np.linalg.norm(g["grad_" + k]) < 1e-300, k
    if "K_G12" in g:
        for k, ck in [("K_t12", "K_t12"), ("K_L0_22", "K_L0_22"), ("K_G12", "K_G12"), ("K_G22", "K_G22"),
                      ("mu_g", "mu_g"), ("sigma2_g", "sigma2_g"), ("sampled_tilde_ell", "t_ell"), ("sampled_v", "v")]:
            assert _rel(c[ck].detach(), g[k]) <= 1e-12, k
        assert _rel(torch.stack(c["pair_samples"]).detach(), g["pair_samples"]) <= 1e-12
        for k in ["KL_W", "KL_v", "KL_U"]:
            assert abs(float(c[k]) - float(g[k])) <= 1e-11 * max(1.0, abs(float(g[k]))), k


def test_modelpt_known_answer_with_reference_rng():
    """model.pt state + torch.manual_seed(123) + the reference's own float32 randn stream."""
    g = G.load("modelpt_forward")
    xs, ys = G.split_lists(g)
    p = G.params(g)
    torch.manual_seed(123)
    loss, _ = O.forward(p, xs, ys, g["z"], 200.0, O.TorchNoise())
    assert float(loss) == pytest.approx(147.88397067775404, rel=1e-13)
    assert float(loss) == pytest.approx(float(g["loss"]), rel=1e-13)


@pytest.mark.parametrize("case,D,M", [("pm25_forward", 5, 256), ("hcp_like_forward", 8, 512),
                                      ("ecog_like_forward", 4, 1024)])
def test_big_shape_digests(case, D, M):
    """Loss, per-parameter gradient norms and strided gradient samples of the PM2.5-shaped and the
    HCP-like (D=8, M=512, B=5000) reference runs."""
    g = G.load(case)
    xs, ys = G.split_lists(g)
    p = G.params(g, D=D, M=M, requires_grad=True)
    loss, _ = O.forward(p, xs, ys, g["z"], float(g["N"]), O.TapeNoise(g["noise"]))
    loss.backward()
    assert float(loss) == pytest.approx(float(g["loss"]), rel=1e-11)
    for k in O.PARAM_NAMES:
        gr = p[k].grad.reshape(-1).numpy()
        assert np.linalg.norm(gr) == pytest.approx(float(g["gnorm_" + k]), rel=1e-8, abs=1e-300), k
        samp = gr[:: max(1, gr.size // 997)]
        assert _rel(samp, g["gsample_" + k]) <= 1e-8 or np.linalg.norm(g["gsample_" + k]) == 0, k


def test_compute_elbo_ecog_like():
    """The M = 1024 (ECoG length scales) fixture's 2-sample compute_ELBO."""
    g = G.load("ecog_like_forward")
    xs, ys = G.split_lists(g)
    p = G.params(g, D=4, M=1024)
    tape = O.TapeNoise(g["elbo_noise"])
    elbo, lps = O.compute_ELBO(p, xs, ys, g["z"], float(g["N"]), tape, n_sample=int(g["elbo_n_sample"]))
    assert tape.done()
    assert float(elbo) == pytest.approx(float(g["elbo"]), rel=1e-11)
    np.testing.assert_allclose(lps.numpy(), g["elbo_logprob_per_sample"], rtol=1e-11)


def test_compute_elbo():
    g = G.load("toy_elbo")
    xs, ys = G.split_lists(g)
    p = G.params(g)
    tape = O.TapeNoise(g["noise"])
    elbo, lps = O.compute_ELBO(p, xs, ys, g["z"], float(g["N"]), tape, n_sample=int(g["n_sample"]))
    assert tape.done()
    assert float(elbo) == pytest.approx(float(g["elbo"]), rel=1e-12)
    np.testing.assert_allclose(lps.numpy(), g["logprob_per_sample"], rtol=1e-12)


def test_utils_cases():
    g = G.load("utils_cases")
    X, Z = torch.from_numpy(g["X"]), torch.from_numpy(g["Z"])
    s2 = torch.tensor(1.3, dtype=torch.float64, requires_grad=True)
    ls = torch.tensor(0.2, dtype=torch.float64, requires_grad=True)
    K = O.create_RBF(X, Z, s2, ls)
    (K * torch.from_numpy(g["rbf_Kbar"])).sum().backward()
    np.testing.assert_allclose(K.detach().numpy(), g["rbf_K"], rtol=1e-13)
    assert float(s2.grad) == pytest.approx(float(g["rbf_gs2"]), rel=1e-12)
    assert float(ls.grad) == pytest.approx(float(g["rbf_gls"]), rel=1e-12)
    np.testing.assert_allclose(O.create_RBF(Z, None, 1.3, 0.2).numpy(), g["rbf_K22"], rtol=1e-13)
    eX = torch.from_numpy(g["ellX"]).requires_grad_()
    eZ = torch.from_numpy(g["ellZ"]).requires_grad_()
    Gm = O.create_Gibbs(X, Z, eX, eZ, 0.7)
    (Gm * torch.from_numpy(g["rbf_Kbar"])).sum().backward()
    np.testing.assert_allclose(Gm.detach().numpy(), g["gibbs_K"], rtol=1e-13)
    np.testing.assert_allclose(eX.grad.numpy(), g["gibbs_gellX"], rtol=1e-11)
    np.testing.assert_allclose(eZ.grad.numpy(), g["gibbs_gellZ"], rtol=1e-11)
    K12 = torch.from_numpy(g["mgp_K12"]).requires_grad_()
    K22 = torch.from_numpy(g["mgp_K22"]).requires_grad_()
    mu = torch.from_numpy(g["mgp_mu"]).requires_grad_()
    Sig = torch.from_numpy(g["mgp_Sigma"]).requires_grad_()
    muY, s2Y = O.MGP_mu_sigma2(K12, K22, torch.ones(K12.shape[0], dtype=torch.float64), mu, Sig)
    ((muY * torch.from_numpy(g["mgp_wm"])).sum() + (s2Y * torch.from_numpy(g["mgp_ws"])).sum()).backward()
    for a, k in [(muY, "mgp_muY"), (s2Y, "mgp_s2Y"), (K12.grad, "mgp_gK12"), (K22.grad, "mgp_gK22"),
                 (mu.grad, "mgp_gmu"), (Sig.grad, "mgp_gSigma")]:
        assert _rel(a.detach(), g[k]) <= 1e-11, k
    d11 = torch.ones(K12.shape[0], dtype=torch.float64)
    smp = O.MGP_d(K12.detach(), K22.detach(), d11, mu.detach()[0], Sig.detach()[0], O.TapeNoise(g["mgpd_z"]))
    assert _rel(smp, g["mgpd_sample"]) <= 1e-12
    js = O.JGP_S(d11, K12.detach(), K22.detach(), mu.detach()[1], Sig.detach()[1],
                 O.TapeNoise(np.concatenate([g["jgp_zv"], g["jgp_zt"]])))
    assert _rel(js, g["jgp_sample"]) <= 1e-12
    muk, Sk, K22k = mu.detach().clone().requires_grad_(), Sig.detach().clone().requires_grad_(), K22.detach().clone().requires_grad_()
    kl = O.KL_Gaussian(muk, Sk, torch.zeros(muk.shape[-1], dtype=torch.float64), K22k)
    kl.sum().backward()
    assert _rel(kl.detach(), g["kl"]) <= 1e-12
    for a, k in [(muk.grad, "kl_gmu"), (Sk.grad, "kl_gSigma"), (K22k.grad, "kl_gK22")]:
        assert _rel(a, g[k]) <= 1e-9, k
    rep = O.reparameterize(mu.detach()[2], Sig.detach()[2], torch.from_numpy(g["rep_z"]), full_cov=True)
    assert _rel(rep, g["rep_full"]) <= 1e-13
    nl = O.Normal_logprob(torch.from_numpy(g["nl_loc"]), torch.tensor(0.37, dtype=torch.float64), torch.from_numpy(g["nl_y"]))
    assert float(nl) == pytest.approx(float(g["nl_val"]), rel=1e-14)
    np.testing.assert_array_equal(O.mat2ltri(torch.from_numpy(g["m2l_in"])).numpy(), g["m2l_out"])


def test_legacy_cases():
    g = G.load("legacy_cases")
    t1, t2 = torch.from_numpy(g["X1"]), torch.from_numpy(g["X2"])
    np.testing.assert_allclose(O.pairwise_distances(t1, t2).numpy(), g["pd_12"], rtol=1e-13, atol=1e-14)
    np.testing.assert_allclose(O.pairwise_distances(t1).numpy(), g["pd_11"], rtol=1e-13, atol=1e-14)
    np.testing.assert_allclose(O.RBF_cov(t1, t2, 1.7, 0.8).numpy(), g["rbf_12"], rtol=1e-13)
    np.testing.assert_allclose(O.RBF_cov(t1, None, 1.7, 0.8).numpy(), g["rbf_11"], rtol=1e-13)
    f = lambda k: torch.from_numpy(g[k])
    np.testing.assert_allclose(O.Nonstationary_RBF_cov(t1, f("sig1"), f("ell1"), t2, f("sig2"), f("ell2")).numpy(),
                               g["ns_12"], rtol=1e-13)
    np.testing.assert_allclose(O.Nonstationary_RBF_cov(t1, f("sig1"), f("ell1")).numpy(), g["ns_11"], rtol=1e-13)
    np.testing.assert_allclose(O.Nonstationary_RBF_cov(t1).numpy(), g["ns_11_default"], rtol=1e-13)
    np.testing.assert_array_equal(O.kronecker_product(f("kp_A"), f("kp_B")).numpy(), g["kp_AB"])
    np.testing.assert_array_equal(O.kronecker_product_diag(f("kd_1"), f("kd_2")).numpy(), g["kd_out"])
    np.testing.assert_allclose(O.kron_mv(f("mv_B"), f("mv_K"), f("mv_y")).numpy(), g["mv_out"], rtol=1e-13)
    np.testing.assert_allclose(O.kron_inv(0.3, f("ki_B"), f("ki_K")).numpy(), g["ki_inv"], rtol=1e-10)
    assert float(O.kron_logdet(0.3, f("ki_B"), f("ki_K"))) == pytest.approx(float(g["ki_logdet"]), rel=1e-12)
    lp = O.multivariate_normal_logpdf0(f("lp_y"), torch.zeros(12, dtype=torch.float64), f("ki_B"), f("ki_K"), 0.3)
    assert float(lp) == pytest.approx(float(g["lp_val"]), rel=1e-12)


def test_inference_two_adam_steps():
    """Replays the reference `inference` loop (2 full-batch Adam steps, lr 0.005) from its recorded batches."""
    g = G.load("toy_inference")
    p = {k: torch.from_numpy(np.asarray(g["init_" + k], np.float64).copy()).requires_grad_() for k in O.PARAM_NAMES}
    frozen = {"length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"}
    state = {}
    losses = []
    for it in range(2):
        xs, ys = G.split_lists(g, f"it{it}_x", f"it{it}_y", f"it{it}_sizes")
        for v in p.values():
            v.grad = None
        loss, _ = O.forward(p, xs, ys, g["z"], 200.0, O.TapeNoise(g[f"it{it}_noise"]))
        loss.backward()
        losses.append(float(loss))
        O.adam_step(p, {k: v.grad for k, v in p.items() if k not in frozen}, state, float(g["lr"]))
    np.testing.assert_allclose(losses, g["loss_list"], rtol=1e-12)
    for k in O.PARAM_NAMES:
        np.testing.assert_allclose(p[k].detach().numpy(), g["final_" + k], rtol=1e-10, atol=1e-13, err_msg=k)


# ------------------------------------------------------------------- sample_Y / sample_FY (§8f f1)
def test_oracle_sample_Y_and_sample_FY_match_reference():
    g = G.load("sample_cases")
    p = G.params(g)
    S = int(g["n_sample"])
    ys, ls, gs, ts = O.sample_Y(p, [g["x0"], g["x1"]], g["z"], O.TapeNoise(g["noise_y"]), n_sample=S)
    for got, key in [(ys, "Ys"), (ls, "Ls"), (gs, "Gs"), (ts, "tilde_ells")]:
        ref = g[key]
        assert got.shape == ref.shape
        assert np.max(np.abs(got.numpy() - ref)) <= 1e-10 * max(1.0, np.max(np.abs(ref))), key
    tf, yf, cf = O.sample_FY(p, g["xf"], g["z"], O.TapeNoise(g["noise_f"]), n_sample=S)
    for got, key in [(tf, "fy_tilde_ells"), (yf, "fy_Ys"), (cf, "fy_corrs")]:
        ref = g[key]
        assert got.shape == ref.shape
        assert np.max(np.abs(got.numpy() - ref)) <= 1e-10 * max(1.0, np.max(np.abs(ref))), key
