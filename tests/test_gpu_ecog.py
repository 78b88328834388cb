"""The ECoG-full configuration (BASELINE.json configs[3]; SURVEY §8d: D=128 channels, M=1024 inducing
points, fp32, packed Q-pair layout, compute_ELBO sharded over Monte-Carlo samples) on the HIP path.

At M = 1024 the fp32 engine runs a different code path from the PM2.5 / HCP shapes: the recursive
batched Cholesky (chol_inv_rec: 128-multiple splits, fused leaves, L21 / Schur / X21 products on the
128x128 MFMA kernel), the per-factor offsets products (BigBatch: Sigma_f, Xs_f, the KL and pair L-bar
products) and, with pair_layout="packed", the packed pair layout.  Pinned here by

* a reference-generated fixture at M = 1024 (tests/golden/make_golden.py case_ecog_like: D = 4,
  B = N = 2000, length scales 3/M as code/NMGP_ECoG_full.py trains): one training-step gradient and a
  2-sample compute_ELBO (code/nmgp_dsvi.py:303-404), fp32 packed at SURVEY §8c's fp32 gates and fp64 at
  the fp64 gates;
* pair-sharded shares at M = 1024 (D = 16, 2 ranks) summing to the whole model's loss and gradient;
* the full ECoG shape (D = 128, M = 1024, N = 50,048): one compute_ELBO sample and one training step
  (finite, every factor positive-definite, device status clean) and the packed -> dense state_dict
  round trip.
"""
import gc

import numpy as np
import pytest
import torch

from oracle import nmgp_oracle as O
from tests import _golden as G

pytestmark = pytest.mark.gpu

D4, M4 = 4, 1024
HYPER = ("sigma2_", "length_scales_")


def _rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu().reshape(-1)
    b = torch.as_tensor(b).detach().double().cpu().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


def _pack(t, D):
    ii, jj = np.tril_indices(D)
    return t[torch.from_numpy(ii), torch.from_numpy(jj)]


def _theta(p, D, M, dtype, packed):
    parts = []
    for k in O.PARAM_NAMES:
        v = p[k]
        if packed and k in ("mu_U", "sqrt_U"):
            v = _pack(v, D)
        parts.append(v.reshape(-1))
    return torch.cat(parts).to("cuda", dtype)


def _dense_grads(eng, grad, D):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import _unpack_pairs_host
    out = {}
    for k in O.PARAM_NAMES:
        o, shp = eng.offs[k]
        n = int(np.prod(shp)) if shp else 1
        v = grad[o:o + n].reshape(shp)
        out[k] = (_unpack_pairs_host(v, D) if eng.packed and k in ("mu_U", "sqrt_U") else v.cpu()).double()
    return out


def _digest(gd, loss, g):
    errs = {"loss": abs(loss - float(g["loss"])) / abs(float(g["loss"]))}
    for k in O.PARAM_NAMES:
        ref_n = float(g["gnorm_" + k])
        if ref_n == 0:
            continue
        gr = gd[k].reshape(-1)
        errs["norm_" + k] = abs(float(gr.norm()) - ref_n) / ref_n
        errs["sample_" + k] = _rel(gr[:: max(1, gr.numel() // 997)], g["gsample_" + k])
    return errs


def _ecog_like_engine(dtype, packed):
    from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
    g = G.load("ecog_like_forward")
    p = G.params(g, D=D4, M=M4)
    sizes = [int(s) for s in g["sizes"]]
    eng = DsviEngine(D4, M4, sum(sizes), g["z"], dtype=dtype, packed=packed)
    theta = _theta(p, D4, M4, dtype, packed)
    grad = torch.zeros_like(theta)
    eng.bind(theta, grad, frozen_mask=0, N=float(g["N"]))
    if dtype == torch.float32:
        # the large-M fp32 path: per-factor offsets products on the 128x128 kernel (the KL L-bar in the solve form:
        # a sequence of block products, each a BigBatch)
        plan = eng._plan(0)
        assert isinstance(plan["syrk_side"], H.BigBatch)
        kl = plan["kl_lbar"]
        assert isinstance(kl, H.BigBatch) or (eng.kl_solve and all(isinstance(q, H.BigBatch) for q in kl.parts))
    eng.load_batch(g["x"], g["y"], sizes, noise=g["noise"])
    eng.forward_backward()
    torch.cuda.synchronize()
    eng.check_info()
    return g, eng, grad


def test_ecog_like_fp32_packed_engine_within_fp32_gates():
    """The ECoG configuration's arithmetic (fp32, packed pairs, M = 1024) against the fp64 reference at
    SURVEY §8c's fp32 gates: loss 1e-3, vector-parameter gradient norms / strided samples 2e-2."""
    g, eng, grad = _ecog_like_engine(torch.float32, packed=True)
    gd = _dense_grads(eng, grad, D4)
    errs = _digest(gd, float(eng.out[0]), g)
    print("PARITY ecog_like fp32 packed:", {k: f"{v:.2e}" for k, v in errs.items()})
    assert errs["loss"] < 1e-3, errs
    vec = {k: e for k, e in errs.items() if k != "loss" and not any(h in k for h in HYPER)}
    bad = {k: e for k, e in vec.items() if e > 2e-2}
    assert not bad, f"fp32 gradient digest mismatch {bad} (all {errs})"
    # (hyper-parameter gradients: fp64 prior adjoint chains; 0.26-0.30 with fp32 ones)
    assert max(e for k, e in errs.items() if any(h in k for h in HYPER)) < 2e-2, errs
    samp = torch.cat([gd[k].reshape(-1)[:: max(1, gd[k].numel() // 997)] for k in O.PARAM_NAMES])
    ref = torch.cat([torch.as_tensor(g["gsample_" + k]).reshape(-1) for k in O.PARAM_NAMES])
    assert _rel(samp, ref) < 2e-2


@pytest.mark.parametrize("packed", [False, True])
def test_ecog_like_fp64_engine_matches_reference(packed):
    """Same fixture, fp64 engine (recursive fp64 Cholesky at M = 1024): SURVEY's fp64 gates."""
    g, eng, grad = _ecog_like_engine(torch.float64, packed=packed)
    errs = _digest(_dense_grads(eng, grad, D4), float(eng.out[0]), g)
    print(f"PARITY ecog_like fp64 packed={packed}:", {k: f"{v:.2e}" for k, v in errs.items()})
    assert errs["loss"] < 1e-10, errs
    # vector parameters at SURVEY's 1e-8; the scalar hyper-parameter gradients are sums whose terms cancel
    # to ~1e-7 of their size at these length scales (K12 - P K22 ~ 1e-4 P): the CPU oracle itself, the
    # reference's algorithm in another fp64 summation order, is 3.6e-9 off the reference on
    # length_scales_tildeell_log (tests/analysis/ecog_hyper_sensitivity.py), so they get 1e-7
    bad = {k: e for k, e in errs.items()
           if k != "loss" and e > (1e-7 if any(h in k for h in HYPER) else 1e-8)}
    assert not bad, f"fp64 gradient digest mismatch {bad} (all {errs})"


@pytest.mark.parametrize("dtype,layout,rtol", [(torch.float64, "dense", 1e-10), (torch.float32, "packed", 1e-3)])
def test_ecog_like_compute_elbo_through_api(dtype, layout, rtol):
    """NMGP.compute_ELBO at M = 1024 with the reference's injected noise (2 samples, column gather,
    last-sample K_G22 KL): per-sample reconstruction terms and the ELBO against the reference."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP
    g = G.load("ecog_like_forward")
    p = G.params(g, D=D4, M=M4)
    xs, ys = G.split_lists(g)
    N = int(g["N"])
    m = NMGP(N, D4, g["z"], device="cuda:0", dtype=dtype, pair_layout=layout,
             **{k: p[k].numpy() for k in ["mu_W", "sqrt_W", "mu_v", "sqrt_v", "mu_U", "sqrt_U"]})
    with torch.no_grad():
        for k in O.PARAM_NAMES[6:]:
            getattr(m, k).data.fill_(float(p[k]))
    assert m.packed == (layout == "packed")
    tape = O.TapeNoise(g["elbo_noise"])
    m._torch_noise = lambda B, n_pairs: tape(M4 + B + n_pairs * B)
    lps = []
    eng_fn = m.engine

    def engine(B, N=None):                   # record every sample's reconstruction term
        e = eng_fn(B, N)
        if not getattr(e, "_rec_wrapped", False):
            orig = e.elbo_sample

            def rec(*a, **k):
                out = orig(*a, **k)
                lps.append(float(out[1]))
                return out
            e.elbo_sample, e._rec_wrapped = rec, True
        return e
    m.engine = engine
    elbo = m.compute_ELBO([torch.from_numpy(x) for x in xs], [torch.from_numpy(y) for y in ys],
                          n_sample=int(g["elbo_n_sample"]))
    print(f"PARITY ecog_like compute_ELBO {dtype} {layout}: elbo rel "
          f"{abs(float(elbo) - float(g['elbo'])) / abs(float(g['elbo'])):.2e}, per-sample "
          f"{[abs(a - b) / abs(b) for a, b in zip(lps, g['elbo_logprob_per_sample'])]}")
    assert tape.done()
    np.testing.assert_allclose(lps, g["elbo_logprob_per_sample"], rtol=rtol)
    assert float(elbo) == pytest.approx(float(g["elbo"]), rel=rtol)


# (fp32: the replicated gradient is dominated by the hyper-parameter scalars, sums of B*M + M*M partials
#  whose terms cancel; the shards' and the whole model's fp32 partial sums differ in order -> 1e-3)
@pytest.mark.parametrize("dtype,ltol,gtol", [(torch.float64, 1e-11, 1e-9), (torch.float32, 1e-5, 1e-3)])
def test_ecog_pair_shares_sum_to_whole_model(dtype, ltol, gtol):
    """Pair sharding at M = 1024 (SURVEY §8e axis 3, the ECoG configuration's training layout): D = 16
    outputs over 2 ranks (shares evaluated in turn in one process) -- the summed loss and replicated
    gradients equal the whole packed model's on the same noise, and each share's pair gradients equal
    the whole model's pair rows."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine
    from collaborative_nonstationary_multivariate_gaussian_process_amd.pair_shard import PairShard, pair_shard_ranges
    D, M, n = 16, 1024, 40
    Q = D * (D + 1) // 2
    rng = np.random.default_rng(16)
    xs = [np.sort(rng.uniform(0, 1, n)) for _ in range(D)]
    ys = [np.sin(6 * x + 0.2 * d) + 0.3 * rng.standard_normal(n) for d, x in enumerate(xs)]
    z = np.linspace(0, 1, M)
    gen = torch.Generator().manual_seed(16)
    p = {"mu_W": 0.1 * torch.randn(D, M, generator=gen, dtype=torch.float64),
         "sqrt_W": 0.1 * torch.randn(D, M, M, generator=gen, dtype=torch.float64),
         "mu_v": -4.0 + 0.1 * torch.randn(M, generator=gen, dtype=torch.float64),
         "sqrt_v": 0.1 * torch.randn(M, M, generator=gen, dtype=torch.float64),
         "mu_U": 0.1 * torch.randn(Q, M, generator=gen, dtype=torch.float64),
         "sqrt_U": 0.1 * torch.randn(Q, M, M, generator=gen, dtype=torch.float64)}
    ls = float(np.log(3.0 / M))
    for k, v in zip(O.PARAM_NAMES[6:], [0., ls, 0., ls, 0., ls, -2.]):
        p[k] = torch.tensor(v, dtype=torch.float64)
    B = D * n
    N = 50.0 * B
    noise = np.random.default_rng(17).standard_normal(M + B + Q * B)
    whole = DsviEngine(D, M, B, z, dtype=dtype, packed=True)
    th = torch.cat([p[k].reshape(-1) for k in O.PARAM_NAMES]).to("cuda", dtype)
    gw = torch.zeros_like(th)
    whole.bind(th, gw, frozen_mask=0, N=N)
    whole.load_batch(np.concatenate(xs), np.concatenate(ys), [n] * D, noise=noise)
    whole.forward_backward()
    torch.cuda.synchronize()
    whole.check_info()
    lw = float(whole.out[0])
    gwd = {k: gw[whole.offs[k][0]:whole.offs[k][0] + (int(np.prod(whole.offs[k][1])) if whole.offs[k][1] else 1)]
           .double().cpu() for k in O.PARAM_NAMES}
    del whole
    torch.cuda.empty_cache()
    z_v, z_t, z_p = noise[:M], noise[M:M + B], noise[M + B:].reshape(Q, B)
    tot, rep, pair_err = 0.0, None, 0.0
    for r, (i0, i1) in enumerate(pair_shard_ranges(D, 2)):
        rows = np.arange(i0 * n, i1 * n)
        q0, q1 = i0 * (i0 + 1) // 2, i1 * (i1 + 1) // 2
        nz = np.concatenate([z_v, z_t[rows], z_p[q0:q1][:, rows].reshape(-1)])
        sh = PairShard(p, z, B_r=len(rows), N_r=N * len(rows) / B, rank=r, world=2, dtype=dtype, device="cuda")
        sh.load(xs[i0:i1], ys[i0:i1], noise=nz)
        tot += float(sh.grad_step(reduce=False))
        torch.cuda.synchronize()
        sh.check()
        g_r = torch.cat([sh.local_grad(k).reshape(-1).double().cpu() for k in ("mu_W", "sqrt_W", "mu_v", "sqrt_v")]
                        + [sh.local_grad(k).reshape(-1).double().cpu() for k in O.PARAM_NAMES[6:]])
        rep = g_r if rep is None else rep + g_r
        for k in ("mu_U", "sqrt_U"):
            per = int(np.prod(p[k].shape[1:]))
            ref = gwd[k][q0 * per:q1 * per]
            pair_err = max(pair_err, _rel(sh.local_grad(k).reshape(-1), ref))
        del sh
        gc.collect()
        torch.cuda.empty_cache()
    rep_w = torch.cat([gwd[k].reshape(-1) for k in ("mu_W", "sqrt_W", "mu_v", "sqrt_v")] +
                      [gwd[k].reshape(-1) for k in O.PARAM_NAMES[6:]])
    lerr, rerr = abs(tot - lw) / abs(lw), _rel(rep, rep_w)
    print(f"PARITY ecog pair shares D={D} M={M} {dtype}: loss rel {lerr:.2e}  replicated grad rel-norm {rerr:.2e}  "
          f"pair grad rel-norm {pair_err:.2e}")
    assert lerr < ltol and rerr < gtol and pair_err < gtol, (lerr, rerr, pair_err)


def _checksum(t, chunk=1 << 28):
    """fp64 sum of a huge fp32 vector in fixed chunks (no full-size fp64 temporary)."""
    return float(sum(float(t[i:i + chunk].sum(dtype=torch.float64)) for i in range(0, t.numel(), chunk)))


@pytest.mark.timeout(900)
def test_ecog_full_size_elbo_sample_training_step_and_state_roundtrip():
    """The full ECoG shape: D = 128 (Q = 8256 pairs), M = 1024, N = 50,048 rows, fp32, pair_layout auto
    (-> packed: 35 GB of parameters).  One compute_ELBO sample over all rows (the bench's sharded leg) and
    one training step on B = 512 rows with Adam: finite values, every factor positive-definite, device
    status clean, parameters moved.  Then the reference-shaped dense state_dict (host, 69 GB sqrt_U)
    round-trips into the packed model bit for bit.  No reference run exists at this size (DNF on the
    CPU); the M = 1024 arithmetic is pinned by the fixture tests above."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as Lb
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
    D, M, rows, B = 128, 1024, 391, 512
    rng = np.random.default_rng(7)
    xs = [np.sort(rng.uniform(0, 1, rows)) for _ in range(D)]
    ys = [np.sin(6 * x + 0.1 * d) + 0.3 * rng.standard_normal(rows) for d, x in enumerate(xs)]
    m = NMGP(D * rows, D, np.linspace(0, 1, M), seed=22, device="cuda:0", noise="device", dtype=torch.float32)
    assert m.packed
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        getattr(m, k).data.fill_(float(np.log(3.0 / M)))
    elbo = float(m.compute_ELBO([torch.from_numpy(x) for x in xs], [torch.from_numpy(y) for y in ys], n_sample=1))
    assert np.isfinite(elbo), elbo
    Lb.check_device_status()
    m._engines.clear()                       # the N-row ELBO engine (52 GB of row factors) before training
    gc.collect()
    torch.cuda.empty_cache()
    tr = DsviTrainer(m, lr=0.01)
    eng = m.engine(B)
    pick = np.sort(np.random.default_rng(8).choice(D * rows, B, replace=False))
    out_id = pick // rows
    xb = np.concatenate(xs)[pick]
    yb = np.concatenate(ys)[pick]
    sizes = np.bincount(out_id, minlength=D)
    eng.load_batch(xb, yb, sizes)
    th_before = m._theta[::4099].clone()
    loss = float(tr.step(eng))
    torch.cuda.synchronize()
    m.check_numerics()
    assert np.isfinite(loss), loss
    # (fp32 sums: a float64 sum of the 8.8 G-element vectors would materialise a 70 GB fp64 copy)
    assert np.isfinite(float(m._grad.sum()))
    assert np.isfinite(float(m._theta.sum()))
    assert not torch.equal(th_before, m._theta[::4099])
    print(f"ecog full size: elbo {elbo:.6e}  step loss {loss:.6e}  peak {torch.cuda.max_memory_allocated() / 1e9:.1f} GB")
    # packed -> dense (host) -> packed
    del tr, eng
    m._engines.clear()
    gc.collect()
    torch.cuda.empty_cache()
    chk = (_checksum(m._theta), m._theta[::7919].clone())
    sd = m.state_dict()
    assert tuple(sd["sqrt_U"].shape) == (D, D, M, M) and sd["sqrt_U"].device.type == "cpu"
    assert float(sd["sqrt_U"][3, 100].abs().sum()) == 0.0                # a dead upper pair block
    assert torch.equal(sd["sqrt_U"][100, 3], m.sqrt_U_pair(100, 3).detach().cpu())
    with torch.no_grad():
        m.sqrt_U.zero_()
        m.mu_U.zero_()
    m.load_state_dict(sd)
    del sd
    gc.collect()
    assert _checksum(m._theta) == chk[0]
    assert torch.equal(m._theta[::7919], chk[1])
