"""The drop-in Python surface (NMGP / inference / utils / Utility) on the MI355X vs golden vectors."""
import numpy as np
import pytest
import torch

from oracle import nmgp_oracle as O
from tests import _golden as G

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu().reshape(-1)
    b = torch.as_tensor(b).detach().double().cpu().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


def _model_from(g, D, M, N, **kw):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP
    m = NMGP(N, D, g["z"], **kw)
    with torch.no_grad():
        for k in O.PARAM_NAMES:
            if "p_" + k in g:
                getattr(m, k).data.copy_(torch.from_numpy(np.asarray(g["p_" + k])))
    return m


def test_state_dict_layout_matches_reference():
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP
    m = NMGP(200, 2, np.linspace(0, 1, 20))
    assert list(m.state_dict().keys()) == O.PARAM_NAMES
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert shapes["sqrt_U"] == (2, 2, 20, 20) and shapes["sigma2_err_log"] == ()
    # reference initialisation stream (NMGP.__init__ with seed 22)
    ref = O.new_params(2, 20, seed=22)
    for k in O.PARAM_NAMES:
        np.testing.assert_array_equal(getattr(m, k).detach().cpu().numpy(), ref[k].numpy())


def test_forward_known_answer_reference_rng_and_backward():
    """model.pt state + torch.manual_seed(123): the reference's own float32 randn stream, through the
    drop-in NMGP.forward / loss.backward()."""
    g = G.load("modelpt_forward")
    xs, ys = G.split_lists(g)
    m = _model_from(g, 2, 20, 200)
    torch.manual_seed(123)
    loss = m([torch.from_numpy(x)[:, None] for x in xs], [torch.from_numpy(y)[:, None] for y in ys])
    assert float(loss) == pytest.approx(147.88397067775404, rel=1e-9)
    loss.backward()
    for k in O.PARAM_NAMES:
        ref = g["grad_" + k]
        if np.linalg.norm(ref) > 0:
            assert _rel(getattr(m, k).grad, ref) < 1e-6, k   # trained state: cancelling scalar grads


def test_inference_two_adam_steps_replays_reference_loop():
    """inference(...) with the reference RNG reproduces the reference loop's losses and parameters."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import inference
    g = G.load("toy_inference")
    xs, ys = G.split_lists(g)
    hyper = {"sigma2_L0_log": 0., "length_scales_L0_log": 2., "sigma2_L1_log": 0., "length_scales_L1_log": 2.,
             "sigma2_tildeell_log": 0., "length_scales_tildeell_log": 0., "sigma2_err_log": -2.}
    torch.manual_seed(0)
    model, loss_list, time_list = inference([x[:, None] for x in xs], [y[:, None] for y in ys], g["z"], 200, 2,
                                            hyperpars=hyper, lr=0.005, itnum=2, show_ELBO=False, seed=22)
    np.testing.assert_allclose([float(v) for v in loss_list], g["loss_list"], rtol=1e-10)
    for k in O.PARAM_NAMES:
        np.testing.assert_allclose(getattr(model, k).detach().cpu().numpy(), g["final_" + k], rtol=1e-8, atol=1e-11,
                                   err_msg=k)
    assert len(time_list) == 2


def test_compute_elbo_through_api():
    g = G.load("toy_elbo")
    xs, ys = G.split_lists(g)
    m = _model_from(g, 2, 20, int(g["N"]))
    tape = O.TapeNoise(g["noise"])
    m._torch_noise = lambda B, n_pairs: tape(20 + B + n_pairs * B)
    elbo = m.compute_ELBO([torch.from_numpy(x) for x in xs], [torch.from_numpy(y) for y in ys],
                          n_sample=int(g["n_sample"]))
    assert float(elbo) == pytest.approx(float(g["elbo"]), rel=1e-10)


def test_compute_elbo_unsorted_index_matches_oracle():
    """compute_ELBO(..., index=[2, 0, 1]) with 3 reference-RNG samples: the engine regroups rows by output,
    and every sample's per-row noise (the first AND the cached later ones, engine.load_noise) must be
    regrouped the same way; equals the oracle run with the same lists, index and noise."""
    g = G.load("mid_forward")
    xs, ys = G.split_lists(g)
    order = [2, 0, 1]
    xl, yl = [xs[k] for k in order], [ys[k] for k in order]
    N = sum(len(x) for x in xl)
    S, M, Q = 3, 64, 6
    rng = np.random.default_rng(23)
    noise = rng.standard_normal(S * (M + N + Q * N)).astype(np.float32).astype(np.float64)
    m = _model_from(g, 3, M, N)
    tape = O.TapeNoise(noise)
    m._torch_noise = lambda B, n_pairs: tape(M + B + n_pairs * B)
    elbo = m.compute_ELBO([torch.from_numpy(x) for x in xl], [torch.from_numpy(y) for y in yl], index=order,
                          n_sample=S)
    ref, _ = O.compute_ELBO(G.params(g), xl, yl, g["z"], N, O.TapeNoise(noise), n_sample=S, index=order)
    assert float(elbo) == pytest.approx(float(ref), rel=1e-10)


def test_predict_Y_matches_oracle():
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import predict_Y
    g = G.load("mid_forward")
    xs, _ = G.split_lists(g)
    m = _model_from(g, 3, 64, 4096)
    est = predict_Y(m, xs)
    ref = O.predict_Y(G.params(g), xs, g["z"])
    assert _rel(est, ref) < 1e-9


def test_utils_dropins_vs_golden():
    from collaborative_nonstationary_multivariate_gaussian_process_amd import utils as U
    from collaborative_nonstationary_multivariate_gaussian_process_amd import gp_ops
    g = G.load("utils_cases")
    dev = "cuda"
    X, Z = torch.from_numpy(g["X"]), torch.from_numpy(g["Z"])
    s2 = torch.tensor(1.3, dtype=torch.float64, device=dev, requires_grad=True)
    ls = torch.tensor(0.2, dtype=torch.float64, device=dev, requires_grad=True)
    K = U.create_RBF(X, Z, scale2=s2, length_scales=ls)
    (K * torch.from_numpy(g["rbf_Kbar"]).to(dev)).sum().backward()
    assert _rel(K, g["rbf_K"]) < 1e-14
    assert float(s2.grad) == pytest.approx(float(g["rbf_gs2"]), rel=1e-12)
    assert float(ls.grad) == pytest.approx(float(g["rbf_gls"]), rel=1e-12)
    eX = torch.from_numpy(g["ellX"]).to(dev).requires_grad_()
    eZ = torch.from_numpy(g["ellZ"]).to(dev).requires_grad_()
    Gm = U.create_Gibbs(X, Z, eX, eZ, scale2=0.7)
    (Gm * torch.from_numpy(g["rbf_Kbar"]).to(dev)).sum().backward()
    assert _rel(Gm, g["gibbs_K"]) < 1e-14
    assert _rel(eX.grad, g["gibbs_gellX"]) < 1e-11 and _rel(eZ.grad, g["gibbs_gellZ"]) < 1e-11
    K12 = torch.from_numpy(g["mgp_K12"]).to(dev).requires_grad_()
    K22 = torch.from_numpy(g["mgp_K22"]).to(dev).requires_grad_()
    mu = torch.from_numpy(g["mgp_mu"]).to(dev).requires_grad_()
    Sig = torch.from_numpy(g["mgp_Sigma"]).to(dev).requires_grad_()
    d11 = torch.ones(K12.shape[0], dtype=torch.float64, device=dev)
    muY, s2Y = U.MGP_mu_sigma2(K12, K22, d11, mu, Sig)
    ((muY * torch.from_numpy(g["mgp_wm"]).to(dev)).sum() + (s2Y * torch.from_numpy(g["mgp_ws"]).to(dev)).sum()).backward()
    for a, k in [(muY, "mgp_muY"), (s2Y, "mgp_s2Y"), (K12.grad, "mgp_gK12"), (K22.grad, "mgp_gK22"),
                 (mu.grad, "mgp_gmu"), (Sig.grad, "mgp_gSigma")]:
        assert _rel(a, g[k]) < 1e-9, k
    muk = torch.from_numpy(g["mgp_mu"]).to(dev).requires_grad_()
    Sk = torch.from_numpy(g["mgp_Sigma"]).to(dev).requires_grad_()
    K22k = torch.from_numpy(g["mgp_K22"]).to(dev).requires_grad_()
    kl = U.KL_Gaussian(muk, Sk, torch.zeros(muk.shape[-1], dtype=torch.float64), K22k)
    kl.sum().backward()
    assert _rel(kl, g["kl"]) < 1e-10
    for a, k in [(muk.grad, "kl_gmu"), (Sk.grad, "kl_gSigma"), (K22k.grad, "kl_gK22")]:
        assert _rel(a, g[k]) < 1e-7, k
    # MGP_d / JGP_S with the fixture's injected noise
    zs = [torch.from_numpy(g["mgpd_z"]), torch.from_numpy(g["jgp_zv"]), torch.from_numpy(g["jgp_zt"])]
    orig = gp_ops._randn_like_ref
    try:
        gp_ops._randn_like_ref = lambda shape, device: zs.pop(0).to(device)
        smp = U.MGP_d(K12.detach(), K22.detach(), d11, mu.detach()[0], Sig.detach()[0])
        assert _rel(smp, g["mgpd_sample"]) < 1e-9
        js = U.JGP_S(d11, K12.detach(), K22.detach(), mu.detach()[1], Sig.detach()[1])
        assert _rel(js, g["jgp_sample"]) < 1e-9
    finally:
        gp_ops._randn_like_ref = orig
    rep = U.reparameterize(mu.detach()[2], Sig.detach()[2], torch.from_numpy(g["rep_z"]), full_cov=True)
    assert _rel(rep, g["rep_full"]) < 1e-12
    nl = U.Normal_logprob(torch.from_numpy(g["nl_loc"]), torch.tensor(0.37, dtype=torch.float64),
                          torch.from_numpy(g["nl_y"]))
    assert float(nl) == pytest.approx(float(g["nl_val"]), rel=1e-13)
    assert torch.equal(U.mat2ltri(torch.from_numpy(g["m2l_in"])).cpu(), torch.from_numpy(g["m2l_out"]))


def test_legacy_kernels_and_kronecker_vs_golden():
    from collaborative_nonstationary_multivariate_gaussian_process_amd.Utility import kernels as K
    from collaborative_nonstationary_multivariate_gaussian_process_amd.Utility import kronecker_operation as KO
    from collaborative_nonstationary_multivariate_gaussian_process_amd.Utility import distributions as DI
    g = G.load("legacy_cases")
    f = lambda k: torch.from_numpy(g[k])
    assert _rel(K.pairwise_distances(f("X1"), f("X2")), g["pd_12"]) < 1e-13
    assert _rel(K.pairwise_distances(f("X1")), g["pd_11"]) < 1e-13
    assert _rel(K.RBF_cov(f("X1"), f("X2"), alpha=1.7, beta=0.8), g["rbf_12"]) < 1e-13
    assert _rel(K.RBF_cov(f("X1"), alpha=1.7, beta=0.8), g["rbf_11"]) < 1e-13
    assert _rel(K.Nonstationary_RBF_cov(f("X1"), f("sig1"), f("ell1"), f("X2"), f("sig2"), f("ell2")), g["ns_12"]) < 1e-13
    assert _rel(K.Nonstationary_RBF_cov(f("X1"), f("sig1"), f("ell1")), g["ns_11"]) < 1e-13
    assert _rel(K.Nonstationary_RBF_cov(f("X1")), g["ns_11_default"]) < 1e-13
    assert torch.equal(KO.kronecker_product(f("kp_A"), f("kp_B")).cpu(), f("kp_AB"))          # bit-exact
    assert torch.equal(KO.kronecker_product_diag(f("kd_1"), f("kd_2")).cpu(), f("kd_out"))    # bit-exact
    assert _rel(KO.kron_mv(f("mv_B"), f("mv_K"), f("mv_y")), g["mv_out"]) < 1e-13
    assert _rel(KO.kron_inv(0.3, f("ki_B"), f("ki_K")), g["ki_inv"]) < 1e-10
    assert float(KO.kron_logdet(0.3, f("ki_B"), f("ki_K"))) == pytest.approx(float(g["ki_logdet"]), rel=1e-12)
    lp = DI.multivariate_normal_logpdf0(f("lp_y"), torch.zeros(12, dtype=torch.float64), f("ki_B"), f("ki_K"), 0.3)
    assert float(lp) == pytest.approx(float(g["lp_val"]), rel=1e-11)


def test_device_noise_graph_step_is_finite_and_matches_eager():
    """The HIP-graph replay of a full step equals the eager step (same Philox stream), and capturing
    the graph has no side effects: k replays after the capture == k eager steps."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
    g = G.load("mid_forward")
    xs, ys = G.split_lists(g)
    for k in (1, 3):
        res = []
        for use_graph in (False, True):
            m = _model_from(g, 3, 64, 4096, noise="device")
            tr = DsviTrainer(m, lr=0.01)
            eng = m.engine(sum(len(x) for x in xs))
            eng.load_batch(g["x"], g["y"], [len(x) for x in xs])
            if use_graph:
                gr = tr.capture(eng)              # warm-up + capture: no parameter / RNG change
                for _ in range(k):
                    gr.replay()
            else:
                for _ in range(k):
                    tr.step(eng)
            torch.cuda.synchronize()
            res.append((float(eng.out[0]), m._theta.clone(), int(tr.step_count.item()), int(m._noise_counter.item())))
        assert np.isfinite(res[0][0])
        assert res[0][0] == pytest.approx(res[1][0], rel=1e-12)
        assert _rel(res[1][1], res[0][1]) < 1e-12
        assert res[0][2] == res[1][2] == k and res[0][3] == res[1][3] == k


def test_sample_Y_and_sample_FY_replay_reference_noise():
    """§8f f1: NMGP sampling on the device with the reference's recorded noise (model.pt state).
    Tolerance 1e-7 relative: Cholesky solves replace the reference's LU and (P Sigma) o P becomes
    (P tril S)^2 on a trained state whose K22 + 1e-4 I has cond ~1e6 (measured 2.4e-9)."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd import predict
    g = G.load("sample_cases")
    S = int(g["n_sample"])
    m = _model_from(g, 2, 20, 200)
    ys, ls, gs, ts = predict.sample_Y(m, [torch.from_numpy(g["x0"]), torch.from_numpy(g["x1"])], n_sample=S,
                                      noise_tape=g["noise_y"])
    for got, key in [(ys, "Ys"), (ls, "Ls"), (gs, "Gs"), (ts, "tilde_ells")]:
        assert tuple(got.shape) == g[key].shape, key
        assert _rel(got, g[key]) < 1e-7, (key, _rel(got, g[key]))
    tf, yf, cf = predict.sample_FY(m, torch.from_numpy(g["xf"]), n_sample=S, noise_tape=g["noise_f"])
    for got, key in [(tf, "fy_tilde_ells"), (yf, "fy_Ys"), (cf, "fy_corrs")]:
        assert tuple(got.shape) == g[key].shape, key
        assert _rel(got, g[key]) < 1e-7, (key, _rel(got, g[key]))


def test_sample_Y_module_api_shapes_and_moments():
    """Module-level sample_Y / sample_FY (numpy out, device Philox noise): shapes as the reference's,
    sample means near predict_Y's posterior mean, correlation matrices with unit diagonal."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd import nmgp_dsvi as NM
    g = G.load("sample_cases")
    m = _model_from(g, 2, 20, 200)
    torch.manual_seed(0)
    X = [g["x0"], g["x1"]]
    ys, ls, gs, ts = NM.sample_Y(m, X, n_sample=400)
    N = sum(x.shape[0] for x in X)
    assert ys.shape == (400, N) and ls.shape == (400, N, 2) and gs.shape == (400, 2, N) and ts.shape == (400, N)
    assert np.all(np.isfinite(ys))
    mean = NM.predict_Y(m, X)
    # the predictive mean of l*G is not l_mean*G_mean, but on this trained state they are close
    assert np.max(np.abs(ys.mean(0) - mean)) < 0.5
    tf, yf, cf = NM.sample_FY(m, g["xf"], n_sample=50)
    assert tf.shape == (50, 11) and yf.shape == (50, 11, 2) and cf.shape == (50, 11, 2, 2)
    np.testing.assert_allclose(np.diagonal(cf, axis1=2, axis2=3), 1.0, rtol=0, atol=1e-12)
