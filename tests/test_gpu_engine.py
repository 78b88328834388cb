"""The HIP DSVI engine vs the CPU oracle (autograd) and the closed-form mirror, on golden inputs.

Tolerances (stated per case): the engine solves with Cholesky-based explicit inverses where the
reference uses LU, and the PM2.5-shaped case is ill-conditioned by construction (length scale
e^-1 on 256 inducing points: cond(K22 + 1e-4 I) ~ 1e6), so its gradient gate is looser.
"""
import numpy as np
import pytest
import torch

from oracle import nmgp_oracle as O
from tests import _golden as G
from tests import dsvi_mirror as MR

pytestmark = pytest.mark.gpu

# name: (D, M, loss rtol, per-parameter gradient rel-norm tol).  Gates are ~10x the errors measured
# on the MI355X (round 2, printed as "PARITY ..." by the test; VERDICT r1 asked for measured-based
# gates); every fp64 case must also meet SURVEY §8c's fp64 gate: loss 1e-10 and whole-gradient
# rel-norm 1e-8.  Measured: toy 2.3e-13 / 5.2e-11, model.pt 1.3e-12 / 7.5e-10, mid 5.7e-13 / 2.7e-11,
# PM2.5 6.5e-12 / 3.4e-9 (whole gradient 7.0e-10), driver hyper-parameters 3.4e-13 / 2.4e-10.
CASES = {
    "toy_forward": (2, 20, 3e-12, 1e-9),
    "modelpt_forward": (2, 20, 2e-11, 1e-8),    # trained state: larger cond(K22), cancelling d/dsigma2_L1
    "mid_forward": (3, 64, 1e-11, 5e-10),
    "pm25_forward": (5, 256, 1e-10, 5e-8),      # length scale e^-1 on 256 points: cond(K22 + 1e-4 I) ~ 1e6
    # the reference drivers' hyper-parameters (length-scale logs 10 on an hour axis, mu_v = 1,
    # code/NMGP_PM25.py:63-64): nearly rank-one RBF priors held PD by the 1e-4 jitter only
    "driver_hyper_forward": (3, 64, 5e-12, 3e-9),
}
SURVEY_FP64_LOSS, SURVEY_FP64_GRAD = 1e-10, 1e-8


def _rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu().reshape(-1)
    b = torch.as_tensor(b).detach().double().cpu().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


def _setup(case):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
    D, M = CASES[case][:2]
    g = G.load(case)
    xs, ys = G.split_lists(g)
    p = G.params(g, D=D, M=M)
    sizes = [len(x) for x in xs]
    B = sum(sizes)
    eng = DsviEngine(D, M, B, g["z"])
    theta = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda")
    grad = torch.zeros_like(theta)
    eng.bind(theta, grad, frozen_mask=0, N=float(g["N"]))
    eng.load_batch(g["x"], g["y"], sizes, noise=g["noise"])
    return g, xs, ys, p, eng, theta, grad


def _unflatten(eng, flat):
    out = {}
    for k in O.PARAM_NAMES:
        o, shp = eng.offs[k]
        n = int(np.prod(shp)) if shp else 1
        out[k] = flat[o:o + n].reshape(shp).cpu()
    return out


@pytest.mark.parametrize("case", list(CASES))
def test_engine_matches_oracle(case):
    g, xs, ys, p, eng, theta, grad = _setup(case)
    _, _, ltol, gtol = CASES[case]
    out = eng.forward_backward()
    torch.cuda.synchronize()
    eng.check_info()
    # oracle (reference op-for-op, autograd)
    q = {k: v.clone().requires_grad_() for k, v in p.items()}
    loss, _ = O.forward(q, xs, ys, g["z"], float(g["N"]), O.TapeNoise(g["noise"]))
    loss.backward()
    gd = _unflatten(eng, grad)
    errs = {k: _rel(gd[k], q[k].grad) for k in O.PARAM_NAMES if float(q[k].grad.norm()) > 0}
    lerr = abs(float(out[0]) - float(loss)) / abs(float(loss))
    print(f"PARITY {case}: loss rel {lerr:.3e}  max grad rel-norm {max(errs.values()):.3e}  "
          f"whole-gradient rel-norm {_rel(torch.cat([gd[k].reshape(-1) for k in O.PARAM_NAMES]), torch.cat([q[k].grad.reshape(-1) for k in O.PARAM_NAMES])):.3e}")
    whole = _rel(torch.cat([gd[k].reshape(-1) for k in O.PARAM_NAMES]),
                 torch.cat([q[k].grad.reshape(-1) for k in O.PARAM_NAMES]))
    assert lerr <= min(ltol, SURVEY_FP64_LOSS) and whole <= SURVEY_FP64_GRAD, (lerr, whole)
    bad = {k: e for k, e in errs.items() if e > gtol}
    assert not bad, f"gradient mismatch {bad} (all: {errs})"


def test_engine_intermediates_vs_mirror():
    """Kernel-by-kernel comparison on the mid case (localises a failing kernel)."""
    case = "mid_forward"
    g, xs, ys, p, eng, theta, grad = _setup(case)
    eng.forward_backward()
    torch.cuda.synchronize()
    x = torch.from_numpy(g["x"]); y = torch.from_numpy(g["y"]); z = torch.from_numpy(g["z"])
    loss, gr, it = MR.forward_backward({k: v.clone() for k, v in p.items()}, x, y, [int(s) for s in g["sizes"]], z,
                                       float(g["N"]), torch.from_numpy(g["noise"]))
    D = eng.D
    checks = {
        "P_t": (eng.P[0], it["P"]["t"]), "P_0": (eng.P[1], it["P"]["0"]), "P_1": (eng.P[2], it["P"]["1"]),
        "Ainv_t": (eng.Ainv[0], it["Ainv"]["t"]), "v": (eng.v, it["v"]), "ellX": (eng.ellX, it["ellX"]),
        "K_G12": (eng.K12[3], it["KG12"]), "Ainv_G": (eng.Ainv[3], it["Ainv"]["G"]), "P_G": (eng.P[3], it["P"]["G"]),
        "KL": (eng.facbuf[:eng.NF], torch.cat([it["KL"][:D], it["KL"][D + 1:], it["KL"][D:D + 1]])), "R_G": (eng.R[3], it["Rm"]["G"]), "R_0": (eng.R[1], it["Rm"]["0"]),
        "R_t": (eng.R[0], it["Rm"]["t"]), "Abar_G": (eng.Abar[3], it["Abar"]["G"]), "Abar_0": (eng.Abar[1], it["Abar"]["0"]),
        "Abar_t": (eng.Abar[0], it["Abar"]["t"]), "Pbar_G": (eng.Pbar[3], it["Pbar"]["G"]),
        "Pbar_0": (eng.Pbar[1], it["Pbar"]["0"]), "Pbar_t": (eng.Pbar[0], it["Pbar"]["t"]),
        "mbar": (eng.rowbuf[:D].t(), it["mbar"]), "sbar": (eng.rowbuf[D:2 * D].t(), it["sbar"]),
        "vbar": (eng.vbar, None),
    }
    errs = {}
    for k, (a, b) in checks.items():
        if b is None:
            continue
        errs[k] = _rel(a, b)
    gd = _unflatten(eng, grad)
    for k in O.PARAM_NAMES:
        if float(gr[k].norm()) > 0:
            errs["grad_" + k] = _rel(gd[k], gr[k])
    errs["loss"] = abs(float(eng.out[0]) - float(loss)) / abs(float(loss))
    bad = {k: e for k, e in errs.items() if not e < 1e-7}
    assert not bad, f"mismatching intermediates {bad}; all {errs}"


def test_engine_elbo_sample_matches_oracle():
    """compute_ELBO's column-gather sample + last-sample KL on the toy fixture (8 samples)."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
    g = G.load("toy_elbo")
    xs, ys = G.split_lists(g)
    p = G.params(g)
    sizes = [len(x) for x in xs]
    N, S, D, M = int(g["N"]), int(g["n_sample"]), 2, 20
    eng = DsviEngine(D, M, N, g["z"])
    theta = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda")
    eng.bind(theta, torch.zeros_like(theta), N=N)
    noise = g["noise"]
    per = M + N + D * (D + 1) // 2 * N
    lps = []
    for s in range(S):
        eng.load_batch(g["x"], g["y"], sizes, noise=noise[s * per:(s + 1) * per])
        out = eng.elbo_sample(with_kl=(s == S - 1))
        lps.append(float(out[1]))
    kl = float(out[2] + out[3] + out[4])
    np.testing.assert_allclose(lps, g["logprob_per_sample"], rtol=1e-10)
    assert np.mean(lps) - kl == pytest.approx(float(g["elbo"]), rel=1e-10)


# ------------------------------------------------------------------------ fp32 engine (SURVEY §8d HCP/ECoG)
FP32_CASES = {  # fp32 gates from SURVEY §8c: loss rtol 1e-3, gradient rel-norm 2e-2 (vs the fp64 oracle)
    "toy_forward": (2, 20),
    "mid_forward": (3, 64),
}


@pytest.mark.parametrize("case", list(FP32_CASES))
def test_fp32_engine_within_fp32_gates(case):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
    D, M = FP32_CASES[case]
    g = G.load(case)
    xs, ys = G.split_lists(g)
    p = G.params(g, D=D, M=M)
    sizes = [len(x) for x in xs]
    eng = DsviEngine(D, M, sum(sizes), g["z"], dtype=torch.float32)
    theta = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda", torch.float32)
    grad = torch.zeros_like(theta)
    eng.bind(theta, grad, frozen_mask=0, N=float(g["N"]))
    eng.load_batch(g["x"], g["y"], sizes, noise=g["noise"])
    out = eng.forward_backward()
    torch.cuda.synchronize()
    eng.check_info()
    q = {k: v.clone().requires_grad_() for k, v in p.items()}
    loss, _ = O.forward(q, xs, ys, g["z"], float(g["N"]), O.TapeNoise(g["noise"]))
    loss.backward()
    assert float(out[0]) == pytest.approx(float(loss), rel=1e-3)
    # SURVEY §8c fp32 gate on the whole gradient vector (rel-norm 2e-2), and per parameter too: the small
    # scalar gradients (sigma2 logs) come from cancelling sums (cond(K22 + 1e-4 I) ~ 2e5 on the toy
    # fixture's smooth prior), which the fp32 engine forms in fp64 (fp64 projections and prior adjoints)
    gd = _unflatten(eng, grad)
    full_g = torch.cat([gd[k].reshape(-1).double() for k in O.PARAM_NAMES])
    full_r = torch.cat([q[k].grad.reshape(-1) for k in O.PARAM_NAMES])
    assert _rel(full_g, full_r) < 2e-2, _rel(full_g, full_r)
    errs = {k: _rel(gd[k], q[k].grad) for k in O.PARAM_NAMES if float(q[k].grad.norm()) > 0}
    print(f"PARITY {case} fp32 per-parameter:", {k: f"{e:.2e}" for k, e in errs.items()})
    bad = {k: e for k, e in errs.items() if e > 2e-2}
    assert not bad, f"fp32 gradient mismatch {bad} (all: {errs})"


def test_fp32_hcp_like_step_trains():
    """A scaled-down HCP-shaped run (D=12 outputs, M=128, B=1200, fp32, device noise, graph replay):
    finite losses that decrease over 30 Adam steps, every Cholesky positive-definite."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import inference
    rng = np.random.default_rng(4)
    D, n = 12, 400
    X = [np.sort(rng.uniform(0, 1, n)).reshape(-1, 1) for _ in range(D)]
    Y = [np.sin(6 * x + d) + 0.1 * rng.standard_normal(x.shape) for d, x in enumerate(X)]
    hyper = {"sigma2_L0_log": 0., "length_scales_L0_log": -2.5, "sigma2_L1_log": 0., "length_scales_L1_log": -2.5,
             "sigma2_tildeell_log": 0., "length_scales_tildeell_log": -2.5, "sigma2_err_log": -2.}
    torch.manual_seed(0)
    model, losses, _ = inference(X, Y, np.linspace(0, 1, 128), 1200, D, hyperpars=hyper, fix_hyperpars=True,
                                 lr=0.01, itnum=10, show_ELBO=False, device="cuda:0", noise="device",
                                 use_graph=True, dtype=torch.float32)
    L = np.array([float(v) for v in losses])
    assert model._theta.dtype == torch.float32
    assert np.all(np.isfinite(L)) and len(L) == 40
    assert L[-5:].mean() < L[:5].mean()


def test_fp32_big_side_products_match_grouped(monkeypatch):
    """M >= 512 fp32 engines run the D+Q factor products (Sigma_f = tril(S_f) tril(S_f)^T + jitter,
    Xs_f = C_f^-1 L_f, the KL L-bar) on the 128x128 kernel at per-factor offsets; same loss and
    gradients as the 64x64 grouped path (NMGP_BIG_SIDE=0) within fp32 rounding (D=3, M=512, device
    noise, HCP-style length scales).  Sigma_v stays on the grouped kernel in both: it feeds
    ell_Z = exp(v), where a change of fp32 summation order moves this loss (~7e6) by 1e-3."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP
    rng = np.random.default_rng(12)
    D, n, M = 3, 300, 512
    X = [np.sort(rng.uniform(0, 1, n)).reshape(-1, 1) for _ in range(D)]
    Y = [np.sin(6 * x + d) + 0.3 * rng.standard_normal(x.shape) for d, x in enumerate(X)]
    res = []
    for big in ("1", "0"):
        monkeypatch.setenv("NMGP_BIG_SIDE", big)
        model = NMGP(number_observations=D * n, dim_outputs=D, Z=np.linspace(0, 1, M), seed=22,
                     device="cuda:0", noise="device", dtype=torch.float32)
        for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
            getattr(model, k).data.fill_(float(np.log(3.0 / M)))
        loss = model(X, Y)
        loss.backward()
        torch.cuda.synchronize()
        res.append((float(loss), torch.cat([p.grad.reshape(-1).double() for p in model.parameters()]).cpu()))
    assert np.isfinite(res[0][0])
    assert res[0][0] == pytest.approx(res[1][0], rel=1e-4)
    assert _rel(res[0][1], res[1][1]) < 1e-3


@pytest.mark.parametrize("M", [512, 640])
def test_kl_solve_form_matches_explicit_inverse(monkeypatch, M):
    """The KL L-bar of the variational factors in the solve form (factor + diagonal-block inverses, W = C^-1 L and
    C^-T W applied by blocks; nmgp_chol_blockinv_batched_f32 + the dual-store product) vs the explicit-inverse form
    (NMGP_KL_SOLVE=0): same loss and gradients within fp32 rounding -- the variational factors' rows
    (sqrt_W, sqrt_U) compared on their own.  M = 640 splits unevenly (384 + 256: the diagonal blocks in two
    launches).  Reference: code/utils.py:339-351."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP
    rng = np.random.default_rng(31)
    D, n = 3, 200
    X = [np.sort(rng.uniform(0, 1, n)).reshape(-1, 1) for _ in range(D)]
    Y = [np.sin(6 * x + d) + 0.3 * rng.standard_normal(x.shape) for d, x in enumerate(X)]
    res = []
    for ks in ("1", "0"):
        monkeypatch.setenv("NMGP_KL_SOLVE", ks)
        model = NMGP(number_observations=D * n, dim_outputs=D, Z=np.linspace(0, 1, M), seed=23,
                     device="cuda:0", noise="device", dtype=torch.float32, pair_layout="packed")
        for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
            getattr(model, k).data.fill_(float(np.log(3.0 / M)))
        loss = model(X, Y)
        loss.backward()
        torch.cuda.synchronize()
        assert model.engine(D * n).kl_solve == (ks == "1")
        g = {nm: p.grad.reshape(-1).double().cpu() for nm, p in model.named_parameters()}
        res.append((float(loss), g))
    (l1, g1), (l0, g0) = res
    print(f"KL_SOLVE M={M}: loss rel {abs(l1 - l0) / abs(l0):.3e}  " +
          "  ".join(f"{nm} {_rel(g1[nm], g0[nm]):.2e}" for nm in g0 if g0[nm].abs().max() > 0))
    assert np.isfinite(l1)
    assert l1 == pytest.approx(l0, rel=1e-5)
    for nm in ("sqrt_W", "sqrt_U"):
        assert _rel(g1[nm], g0[nm]) < 1e-4, nm
    assert _rel(torch.cat(list(g1.values())), torch.cat(list(g0.values()))) < 1e-4


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_pair_stream_products_match_grouped(monkeypatch, dtype):
    """Few rows per output (D = 16 outputs, 4 rows each on average, M = 512): the per-pair quadratic-form factors,
    their P-bar and the pair L-bar on the pair streaming kernels (csrc/pairs.hip) vs the grouped / batched MFMA
    products (NMGP_PAIR_STREAM=0): same loss and gradient within rounding (fp32: the 128x128 batched path with
    big_side; fp64: the grouped path)."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP
    rng = np.random.default_rng(5)
    D, M = 16, 512
    n = [int(v) for v in rng.integers(0, 9, D)]
    n[3] = 0
    n[7] = 13
    X = [np.sort(rng.uniform(0, 1, k)).reshape(-1, 1) for k in n]
    Y = [np.sin(6 * x + d) + 0.3 * rng.standard_normal(x.shape) for d, x in enumerate(X)]
    res = []
    for ps in ("1", "0"):
        monkeypatch.setenv("NMGP_PAIR_STREAM", ps)
        model = NMGP(number_observations=10 * sum(n), dim_outputs=D, Z=np.linspace(0, 1, M), seed=22,
                     device="cuda:0", noise="device", dtype=dtype, pair_layout="packed")
        for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
            getattr(model, k).data.fill_(float(np.log(3.0 / M)))
        loss = model(X, Y)
        loss.backward()
        torch.cuda.synchronize()
        assert model.engine(sum(n)).pair_stream == (ps == "1")
        res.append((float(loss), torch.cat([p.grad.reshape(-1).double() for p in model.parameters()]).cpu()))
    lt, gt = (1e-4, 1e-3) if dtype == torch.float32 else (1e-12, 1e-10)
    print(f"PAIR_STREAM {dtype}: loss rel {abs(res[0][0] - res[1][0]) / abs(res[1][0]):.3e}  "
          f"grad rel {_rel(res[0][1], res[1][1]):.3e}")
    assert np.isfinite(res[0][0])
    assert res[0][0] == pytest.approx(res[1][0], rel=lt)
    assert _rel(res[0][1], res[1][1]) < gt


def test_step_begin_matches_separate_launches():
    """nmgp_step_begin (one launch) == batch gather + Philox noise + noise-counter advance + grad
    zeroing as separate launches: bit-identical minibatch, segment table, noise, counters."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
    from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as Hx
    D, M, B, nb = 3, 24, 150, 3
    eng = DsviEngine(D, M, B, np.linspace(0, 1, M))
    theta = torch.zeros(eng.nparam, dtype=torch.float64, device="cuda")
    grad = torch.full_like(theta, 7.0)
    eng.bind(theta, grad)
    g = torch.Generator().manual_seed(3)
    Xb = torch.rand(nb, B, generator=g, dtype=torch.float64).cuda()
    Yb = torch.randn(nb, B, generator=g, dtype=torch.float64).cuda()
    Ib = torch.sort(torch.randint(0, D, (nb, B), generator=g), dim=1).values.to(torch.int32).cuda()
    Sb = torch.stack([torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(torch.bincount(r, minlength=D), 0)])
                      for r in Ib.cpu().long()]).to(torch.int32).cuda()
    bctr = eng.bind_dataset(Xb, Yb, Ib, Sb)
    nctr = torch.zeros(1, dtype=torch.int64, device="cuda")
    outs = []
    for fused in (False, True):
        bctr.fill_(1)
        nctr.fill_(5)
        grad.fill_(7.0)
        if fused:
            eng.begin_step(1234, nctr)
        else:
            eng.gather_batch()
            eng.device_noise(1234, nctr)
            Hx.counter_add_(nctr, 1)
            grad.zero_()
        torch.cuda.synchronize()
        outs.append([t.clone() for t in (eng.x, eng.y, eng.row_out, eng.seg, eng.noise, bctr, nctr, grad)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert int(outs[1][5]) == 2 and int(outs[1][6]) == 6 and int(eng._begin_done.item()) == 0


# ------------------------------------------------------------------------ HCP-shaped
def _digest_errs(eng, grad, g):
    """Loss / per-parameter gradient-norm / strided-sample errors against a digest fixture."""
    gd = _unflatten(eng, grad)
    out = {"loss": abs(float(eng.out[0]) - float(g["loss"])) / abs(float(g["loss"]))}
    for k in O.PARAM_NAMES:
        ref_n = float(g["gnorm_" + k])
        if ref_n == 0:
            continue
        gr = gd[k].reshape(-1).double()
        out["norm_" + k] = abs(float(gr.norm()) - ref_n) / ref_n
        out["sample_" + k] = _rel(gr[:: max(1, gr.numel() // 997)], g["gsample_" + k])
    return out


HYPER = ("sigma2_", "length_scales_")


def _hcp_like_engine(dtype):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
    g = G.load("hcp_like_forward")
    p = G.params(g, D=8, M=512)
    sizes = [int(s) for s in g["sizes"]]
    eng = DsviEngine(8, 512, sum(sizes), g["z"], dtype=dtype)
    theta = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda", dtype)
    grad = torch.zeros_like(theta)
    eng.bind(theta, grad, frozen_mask=0, N=float(g["N"]))
    eng.load_batch(g["x"], g["y"], sizes, noise=g["noise"])
    eng.forward_backward()
    torch.cuda.synchronize()
    eng.check_info()
    return g, eng, grad


def test_hcp_like_fp32_engine_within_fp32_gates():
    """D=8 outputs, M=512, B=5000, length scales 3/M (reference-generated, tests/golden/make_golden.py
    case_hcp_like): the fp32 engine -- the HCP configuration's arithmetic -- against the fp64 reference
    at SURVEY §8c's fp32 gates (loss 1e-3, gradient norms / samples 2e-2)."""
    g, eng, grad = _hcp_like_engine(torch.float32)
    errs = _digest_errs(eng, grad, g)
    print("hcp_like fp32 errors", errs)
    # measured (round 2): loss 6.1e-4, vector-parameter samples <= 7.4e-3, concatenated samples ~5e-3;
    # the reference's own algorithm run in fp32 on the CPU is off by 1.8e-3 (loss) / 6.0e-3 (gradient)
    assert errs["loss"] < 1e-3, errs
    vec = {k: e for k, e in errs.items() if k != "loss" and not any(h in k for h in HYPER)}
    bad = {k: e for k, e in vec.items() if e > 2e-2}
    assert not bad, f"fp32 gradient digest mismatch {bad} (all {errs})"
    # scalar hyper-parameter gradients are sums whose terms cancel to ~1e-7 of their size (K12 - P K22 ~
    # 1e-4 P at these length scales): with fp32 adjoints d/d sigma2_tildeell_log was 0.13 off (round 2);
    # the fp32 engine forms the prior adjoint chains and these sums in fp64, so they meet the
    # vector parameters' 2e-2
    assert max(e for k, e in errs.items() if any(h in k for h in HYPER)) < 2e-2, errs
    gd = _unflatten(eng, grad)
    samp = torch.cat([gd[k].reshape(-1).double()[:: max(1, gd[k].numel() // 997)] for k in O.PARAM_NAMES])
    ref = torch.cat([torch.as_tensor(g["gsample_" + k]).reshape(-1) for k in O.PARAM_NAMES])
    assert _rel(samp, ref) < 2e-2


def test_hcp_like_fp64_engine_matches_reference():
    g, eng, grad = _hcp_like_engine(torch.float64)
    errs = _digest_errs(eng, grad, g)
    print("hcp_like fp64 errors", errs)
    assert errs["loss"] < 1e-10, errs            # SURVEY §8c fp64 gate; measured 6.6e-11
    bad = {k: e for k, e in errs.items() if k != "loss" and e > 3e-9}    # measured <= 2.9e-10
    assert not bad, f"fp64 gradient digest mismatch {bad} (all {errs})"


def test_hcp_full_size_fp32_step_tracks_fp64():
    """The full HCP shape (D=50 outputs, Q=1275 pairs, M=512, B=5000; 670 M parameters): one fp32
    step has finite loss, every factor positive-definite, and stays within the fp32 gates of the
    fp64 engine on the same inputs (no reference run exists at this size: DNF on the CPU)."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine, param_layout
    D, M, B = 50, 512, 5000
    rng = np.random.default_rng(50)
    sizes = [B // D] * D
    x = np.concatenate([np.sort(rng.uniform(0, 1, n)) for n in sizes])
    y = np.sin(6 * x) + 0.3 * rng.standard_normal(x.shape)
    z = np.linspace(0, 1, M)
    offs, n = param_layout(D, M)
    gen = torch.Generator(device="cuda").manual_seed(50)
    theta64 = 0.1 * torch.randn(n, generator=gen, dtype=torch.float64, device="cuda")
    o = offs["mu_v"][0]
    theta64[o:o + M] = -4.0 + 0.1 * theta64[o:o + M]
    hyp = offs["sigma2_tildeell_log"][0]
    theta64[hyp:hyp + 7] = torch.tensor([0., np.log(3.0 / M), 0., np.log(3.0 / M), 0., np.log(3.0 / M), -2.],
                                        dtype=torch.float64)
    Q = D * (D + 1) // 2
    noise = np.random.default_rng(51).standard_normal(M + B + Q * B).astype(np.float32)
    res = {}
    for dt in (torch.float64, torch.float32):
        eng = DsviEngine(D, M, B, z, dtype=dt)
        th = theta64.to(dt)
        gr = torch.zeros_like(th)
        eng.bind(th, gr, frozen_mask=0b0101010, N=500000.0)
        eng.load_batch(x, y, sizes, noise=noise)
        eng.forward_backward()
        torch.cuda.synchronize()
        eng.check_info()
        res[dt] = (float(eng.out[0]), gr.double())
        del eng
        torch.cuda.empty_cache()
    l64, g64 = res[torch.float64]
    l32, g32 = res[torch.float32]
    assert np.isfinite(l64) and np.isfinite(l32)
    print("hcp full size: loss rel", abs(l32 - l64) / abs(l64), "grad rel-norm", _rel(g32, g64))
    assert abs(l32 - l64) / abs(l64) < 1e-3
    assert _rel(g32, g64) < 2e-2


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_cached_elbo_samples_equal_full_samples(dtype):
    """compute_ELBO's later samples reuse the sample-independent work of the first one (RBF priors,
    chol(Sigma_v), pair quadratic forms): per-sample reconstruction terms and the last sample's KL are
    bit-identical to recomputing everything per sample."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
    g = G.load("mid_forward")
    p = G.params(g, D=3, M=64)
    sizes = [int(s) for s in g["sizes"]]
    B = sum(sizes)
    eng = DsviEngine(3, 64, B, g["z"], dtype=dtype)
    theta = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda", dtype)
    eng.bind(theta, torch.zeros_like(theta), N=float(g["N"]))
    per = 64 + B + 6 * B
    rng = np.random.default_rng(9)
    noises = [rng.standard_normal(per).astype(np.float32) for _ in range(4)]
    res = []
    for cached in (False, True):
        vals = []
        for s, nz in enumerate(noises):
            eng.load_batch(g["x"], g["y"], sizes, noise=nz)
            out = eng.elbo_sample(with_kl=(s == 3), cached=cached and s > 0)
            torch.cuda.synchronize()
            vals.append(float(out[1]))
        res.append((vals, [float(v) for v in out[2:5]]))
    assert res[0] == res[1]


def test_index_argument_any_order_matches_oracle():
    """forward(..., index=[...]) with the lists in any output order (code/nmgp_dsvi.py:163-169): rows and
    their injected noise are regrouped by output on the host; loss and gradients match the oracle run
    with the same lists, index and noise."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
    g = G.load("mid_forward")
    xs, ys = G.split_lists(g)
    p = G.params(g, D=3, M=64)
    order = [2, 0, 1]
    xl, yl = [xs[k] for k in order], [ys[k] for k in order]
    sizes = [len(x) for x in xl]
    B = sum(sizes)
    rng = np.random.default_rng(17)
    noise = rng.standard_normal(64 + B + 6 * B).astype(np.float32).astype(np.float64)
    eng = DsviEngine(3, 64, B, g["z"])
    theta = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda")
    grad = torch.zeros_like(theta)
    eng.bind(theta, grad, N=float(g["N"]))
    eng.load_batch(np.concatenate(xl), np.concatenate(yl), sizes, noise=noise, index=order)
    eng.forward_backward()
    torch.cuda.synchronize()
    q = {k: v.clone().requires_grad_() for k, v in p.items()}
    loss, _ = O.forward(q, xl, yl, g["z"], float(g["N"]), O.TapeNoise(noise), index=order)
    loss.backward()
    assert float(eng.out[0]) == pytest.approx(float(loss), rel=1e-11)
    gd = _unflatten(eng, grad)
    whole = _rel(torch.cat([gd[k].reshape(-1) for k in O.PARAM_NAMES]), torch.cat([q[k].grad.reshape(-1) for k in O.PARAM_NAMES]))
    assert whole < 1e-9


RAGGED = [("mid_forward", [5, 0, 7]), ("mid_forward", [0, 9, 3]), ("mid_forward", [40, 1, 0]),
          ("pm25_forward", [120, 0, 95, 1, 64]), ("hcp_like_forward", [60, 0, 1, 45, 0, 30, 22, 12]),
          # few rows per output (B / D <= 32): the per-pair products run on the pair streaming kernels
          # (csrc/pairs.hip), incl. an empty output and outputs with more rows than one pass holds (RB = 4 / 8)
          ("hcp_like_forward", [3, 0, 1, 8, 9, 4, 2, 5])]
RAGGED_DM = {"mid_forward": (3, 64), "pm25_forward": (5, 256), "hcp_like_forward": (8, 512)}


def _ragged_run(case, sizes, dtype):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
    D, M = RAGGED_DM[case]
    g = G.load(case)
    p = G.params(g, D=D, M=M)
    rng = np.random.default_rng(sum(sizes) * 7 + len(sizes))
    xl = [np.sort(rng.uniform(0, 1, s)) for s in sizes]
    yl = [rng.standard_normal(s) for s in sizes]
    B = sum(sizes)
    noise = rng.standard_normal(M + B + D * (D + 1) // 2 * B)
    eng = DsviEngine(D, M, B, g["z"], dtype=dtype)
    theta = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda", dtype)
    grad = torch.zeros_like(theta)
    eng.bind(theta, grad, N=float(g["N"]))
    eng.load_batch(np.concatenate(xl), np.concatenate(yl), sizes, noise=noise)
    eng.forward_backward()
    torch.cuda.synchronize()
    eng.check_info()
    q = {k: v.clone().requires_grad_() for k, v in p.items()}
    tape = O.TapeNoise(noise)
    loss, _ = O.forward(q, xl, yl, g["z"], float(g["N"]), tape)
    loss.backward()
    assert tape.done()
    gd = _unflatten(eng, grad)
    lerr = abs(float(eng.out[0]) - float(loss)) / abs(float(loss))
    whole = _rel(torch.cat([gd[k].reshape(-1).double() for k in O.PARAM_NAMES]),
                 torch.cat([q[k].grad.reshape(-1) for k in O.PARAM_NAMES]))
    return eng, lerr, whole


@pytest.mark.parametrize("case,sizes", RAGGED)
def test_ragged_minibatch_with_empty_outputs_matches_oracle(case, sizes):
    """Minibatches whose outputs have very different row counts, some none at all (the DataLoader draw of
    code/nmgp_dsvi.py:829-837 can leave an output empty): every row- and k-segmented product then runs on empty
    or one-row segments -- the per-(output, factor) L-bar slots of an empty output must come out as zeros, the
    per-factor P-bar reduction must skip it (M = 512: the one-product-per-factor L-bar form).  Loss and gradient
    against the oracle at SURVEY's fp64 gates."""
    _, lerr, whole = _ragged_run(case, sizes, torch.float64)
    print(f"PARITY ragged {case} {sizes}: loss rel {lerr:.3e}  whole-gradient rel-norm {whole:.3e}")
    assert lerr <= SURVEY_FP64_LOSS and whole <= SURVEY_FP64_GRAD, (lerr, whole)


@pytest.mark.parametrize("case,sizes", [RAGGED[0], RAGGED[2], RAGGED[4], RAGGED[5]])
def test_fp32_ragged_minibatch_with_empty_outputs(case, sizes):
    """The fp32 engine on the same ragged minibatches (M = 512: the 128x128 batched factor products with
    per-problem k segments, several of them empty) at SURVEY's fp32 gates: loss 1e-3, whole gradient 2e-2."""
    eng, lerr, whole = _ragged_run(case, sizes, torch.float32)
    print(f"PARITY ragged fp32 {case} {sizes} (big_side {eng.big_side}): loss rel {lerr:.3e}  "
          f"whole-gradient rel-norm {whole:.3e}")
    assert lerr <= 1e-3 and whole <= 2e-2, (lerr, whole)


@pytest.mark.parametrize("case", ["mid_forward", "pm25_forward"])
def test_step_is_deterministic_run_to_run(case):
    """The fused step (grouped / latency-kernel GEMMs with their split-K combines, the multi-workgroup
    Cholesky, every reduction) is bit-reproducible: the same batch twice gives identical loss and
    gradient bits."""
    if case not in CASES:
        pytest.skip(case)
    g, xs, ys, p, eng, theta, grad = _setup(case)
    outs = []
    for _ in range(3):
        eng.forward_backward()           # (zeroes the gradient first; the host noise stays loaded)
        torch.cuda.synchronize()
        outs.append((eng.out.clone().cpu(), grad.clone().cpu()))
    for o, gr in outs[1:]:
        assert torch.equal(o[:1], outs[0][0][:1]) and torch.equal(gr, outs[0][1])


@pytest.mark.parametrize("sizes", [None, [120, 0, 95, 1, 64]])
def test_fused_prior_launches_match_separate_launches(monkeypatch, sizes):
    """Round 6: at M = 256 fp64 the engine runs the GP priors as two fused launches (nmgp_chol_tp_f64: builders,
    factor + inverse, T = K12 L^-T, P = T L^-1 and the t-row in the launch).  Same step with NMGP_FUSE_TP=0 (the
    separate builder / invG / projG / t-row launches): loss, every gradient and the projections agree to rounding
    (T / P by substitution instead of explicit-inverse products), on the golden PM2.5 minibatch and a ragged one
    with empty outputs (B = 280: a partial last row workgroup)."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
    g = G.load("pm25_forward")
    D, M = 5, 256
    p = G.params(g, D=D, M=M)
    theta = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda")
    if sizes is None:
        x, y, sz, noise = g["x"], g["y"], [int(s) for s in g["sizes"]], g["noise"]
    else:
        rng = np.random.default_rng(5)
        sz = sizes
        B = sum(sz)
        x, y = np.sort(rng.random(B)), rng.standard_normal(B)
        Q = D * (D + 1) // 2
        noise = rng.standard_normal(M + B + Q * B)
    B = sum(sz)
    res = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("NMGP_FUSE_TP", fuse)
        eng = DsviEngine(D, M, B, g["z"])
        assert eng.fuse_tp == (fuse == "1")
        grad = torch.zeros_like(theta)
        eng.bind(theta, grad, frozen_mask=0, N=float(g["N"]))
        eng.load_batch(x, y, sz, noise=noise)
        eng.forward_backward()
        torch.cuda.synchronize()
        eng.check_info()
        res[fuse] = (float(eng.out[0]), grad.clone(), eng.T.clone(), eng.P.clone(), eng.K12.clone(), eng.ellX.clone())
    (l1, g1, T1, P1, K1, e1), (l0, g0, T0, P0, K0, e0) = res["1"], res["0"]
    print(f"FUSED-TP sizes={sizes}: loss {abs(l1 - l0) / abs(l0):.2e} grad {_rel(g1, g0):.2e} T {_rel(T1, T0):.2e} "
          f"P {_rel(P1, P0):.2e} K12 {_rel(K1, K0):.2e} ellX {_rel(e1, e0):.2e}")
    # the separate launches' explicit-inverse products carry ~20x the fused substitution's error against exact
    # triangular solves (tests/test_gpu_primitives.py::test_chol_tp_fused_priors_vs_torch: P 3e-9 vs 1.5e-10 at
    # cond ~1e6); ell_X (P_t v) and K_G12 inherit that difference, the RBF K12 rows are the same arithmetic
    assert abs(l1 - l0) / abs(l0) < 5e-11 and _rel(g1, g0) < 1e-8
    assert _rel(K1[:3], K0[:3]) < 1e-14 and _rel(K1[3], K0[3]) < 1e-8 and _rel(e1, e0) < 1e-8
    assert _rel(T1, T0) < 1e-8 and _rel(P1, P0) < 1e-7


def test_fused_gibbs_k22_matches_its_own_launch(monkeypatch):
    """Round 6: the training step forms v, ell_Z and the Gibbs prior's K22 in extra workgroups of the fused prior launch
    that factors Sigma_v (NMGP_FUSE_VG=1) instead of the dsvi_vg22 launch after it: the same sums in the same order,
    so v, ell_Z, K_G22 (its lower triangle, before the Gibbs factorization overwrote it: read back as L L^T), the
    loss and the gradient are bit-identical."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
    g = G.load("pm25_forward")
    D, M = 5, 256
    p = G.params(g, D=D, M=M)
    theta = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda")
    x, y, sz, noise = g["x"], g["y"], [int(s) for s in g["sizes"]], g["noise"]
    B = sum(sz)
    res = {}
    for vg in ("1", "0"):
        monkeypatch.setenv("NMGP_FUSE_TP", "1")
        monkeypatch.setenv("NMGP_FUSE_VG", vg)
        eng = DsviEngine(D, M, B, g["z"])
        assert eng.fuse_tp and eng.fuse_vg == (vg == "1")
        grad = torch.zeros_like(theta)
        eng.bind(theta, grad, frozen_mask=0, N=float(g["N"]))
        eng.load_batch(x, y, sz, noise=noise)
        for _ in range(2):                     # (a second step re-arms the launch's progress words)
            eng.forward_backward()
        torch.cuda.synchronize()
        eng.check_info()
        Lg = torch.tril(eng.Afac[eng.NF + 3].clone())
        res[vg] = (eng.out[:1].clone(), grad.clone(), eng.v.clone(), eng.ellZ.clone(), Lg, eng.T.clone(),
                   eng.P.clone())
    for a, b in zip(res["1"], res["0"]):
        assert torch.equal(a, b)
