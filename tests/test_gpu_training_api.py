"""Training-loop surface on the MI355X: loud failures, checkpoint formats (f3), the on-device input
pipeline (f4), the drivers' VTVLCM entry points, and the optimizer-state semantics of
torch.optim.Adam that `continuous_training` relies on."""
import os
import pickle

import numpy as np
import pytest
import torch

from oracle import nmgp_oracle as O
from tests import _golden as G

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu().reshape(-1)
    b = torch.as_tensor(b).detach().double().cpu().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


def _toy():
    g = G.load("toy_forward")
    xs, ys = G.split_lists(g)
    return g, [x[:, None] for x in xs], [y[:, None] for y in ys]


TOY_HYPER = {"sigma2_L0_log": 0., "length_scales_L0_log": 2., "sigma2_L1_log": 0., "length_scales_L1_log": 2.,
             "sigma2_tildeell_log": 0., "length_scales_tildeell_log": 0., "sigma2_err_log": -2.}


# ------------------------------------------------------------------------------ loud failures
def test_non_pd_factor_raises_linalg_error():
    """A NaN in sqrt_v makes Sigma_v + 1e-4 I non-PD: the reference's torch.cholesky raises
    (code/utils.py:46); NMGP.forward raises torch.linalg.LinAlgError from the device info word."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP
    g, xs, ys = _toy()
    m = NMGP(200, 2, g["z"], device="cuda:0")
    with torch.no_grad():
        m.sqrt_v.data[3, 2] = float("nan")
    torch.manual_seed(0)
    with pytest.raises(torch.linalg.LinAlgError, match="positive-definite"):
        m(xs, ys)
    # a healthy state afterwards: the info words are reset by the next factorization
    with torch.no_grad():
        m.sqrt_v.data[3, 2] = 0.0
    loss = m(xs, ys)
    assert np.isfinite(float(loss))


def test_non_pd_inside_inference_raises():
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import inference
    g, xs, ys = _toy()
    sv = 0.1 * np.random.default_rng(0).standard_normal((20, 20))
    sv[5, 5] = np.nan
    for noise in ("torch", "device"):
        torch.manual_seed(0)
        with pytest.raises(torch.linalg.LinAlgError):
            inference(xs, ys, g["z"], 100, 2, hyperpars=dict(TOY_HYPER), sqrt_v=sv, lr=0.005, itnum=2,
                      show_ELBO=False, device="cuda:0", noise=noise)


def test_device_status_is_clean_after_work():
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H
    A = torch.randn(8, 64, 64, dtype=torch.float64, device="cuda")
    A = A @ A.transpose(1, 2) + 64 * torch.eye(64, dtype=torch.float64, device="cuda")
    X, info = H.chol_inv_(A.clone())
    H.bmm(A, A)
    assert L.device_status(clear=True) == 0
    L.check_device_status()                 # does not raise


# ------------------------------------------------------------------------------ f3 formats
def test_reference_model_pt_loads_through_load_state_dict():
    """code/notebook/model.pt (re-saved tensors, tests/golden/model_pt.pt) through the drop-in's
    load_state_dict (weights-only load) reproduces the known answer of SURVEY §8c (manual_seed 123)."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
    ck = torch.load(os.path.join(ROOT, "tests", "golden", "model_pt.pt"), weights_only=True)
    g, xs, ys = _toy()
    m = NMGP(200, 2, g["z"], device="cuda:0")
    m.load_state_dict(ck["model_state_dict"])
    for k, v in ck["model_state_dict"].items():
        assert torch.equal(getattr(m, k).detach().cpu(), v), k
    m._assert_views()                       # still one flat device vector
    torch.manual_seed(123)
    loss = m([torch.from_numpy(x) for x in xs], [torch.from_numpy(y) for y in ys])
    assert float(loss) == pytest.approx(147.88397067775404, rel=1e-9)
    # the old-torch optimizer state (object-id keys, frozen length scales absent) is adopted
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        getattr(m, k).requires_grad = False
    tr = DsviTrainer(m, lr=0.123)
    tr.load_optimizer_state(ck["optimizer_state_dict"])
    assert tr.lr == 0.005 and int(tr.step_count.item()) == 2000
    o, shp = m._offs["sqrt_U"]
    n = int(np.prod(shp))
    pid = ck["optimizer_state_dict"]["param_groups"][0]["params"][5]
    assert torch.equal(tr.m[o:o + n].cpu().reshape(shp), ck["optimizer_state_dict"]["state"][pid]["exp_avg"])


def test_adam_state_semantics_match_torch_adam():
    """DsviTrainer.load_optimizer_state + update == torch.optim.Adam.load_state_dict + step on the same
    gradients, including the checkpoint's lr replacing the constructor's and frozen parameters."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer, \
        _adam_state_dict
    g, xs, ys = _toy()
    m = NMGP(200, 2, g["z"], device="cuda:0")
    frozen = ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]
    for k in frozen:
        getattr(m, k).requires_grad = False
    params = [torch.nn.Parameter(getattr(m, k).detach().cpu().clone(), requires_grad=getattr(m, k).requires_grad)
              for k in O.PARAM_NAMES]
    opt = torch.optim.Adam(params, lr=0.02)
    rng = np.random.default_rng(3)
    grads = [[torch.from_numpy(rng.standard_normal(tuple(p.shape))) if p.requires_grad else None for p in params]
             for _ in range(3)]
    for s in range(2):
        for p, gr in zip(params, grads[s]):
            p.grad = gr
        opt.step()
    sd = opt.state_dict()
    with torch.no_grad():
        for k, p in zip(O.PARAM_NAMES, params):
            getattr(m, k).data.copy_(p.detach())
    tr = DsviTrainer(m, lr=0.5)                       # the checkpoint's lr (0.02) must win
    tr.load_optimizer_state(sd)
    assert tr.lr == 0.02
    for p, gr in zip(params, grads[2]):
        p.grad = gr
    opt.step()
    with torch.no_grad():
        m._grad.zero_()
        for k, gr in zip(O.PARAM_NAMES, grads[2]):
            if gr is not None:
                o, shp = m._offs[k]
                n = int(np.prod(shp)) if shp else 1
                m._grad[o:o + n] = gr.reshape(-1).to(m._grad.device)
    tr.update()
    torch.cuda.synchronize()
    for k, p in zip(O.PARAM_NAMES, params):
        np.testing.assert_allclose(getattr(m, k).detach().cpu().numpy(), p.detach().numpy(), rtol=1e-13, atol=1e-15,
                                   err_msg=k)
    # and our state_dict loads into torch Adam and continues identically
    opt2 = torch.optim.Adam([torch.nn.Parameter(p.detach().clone(), requires_grad=p.requires_grad) for p in params])
    opt2.load_state_dict(_adam_state_dict(m, tr))
    assert opt2.param_groups[0]["lr"] == 0.02
    # mixed step counts are rejected, not silently bias-corrected
    sd_bad = {"state": dict(sd["state"]), "param_groups": sd["param_groups"]}
    sd_bad["state"][0] = dict(sd_bad["state"][0], step=torch.tensor(7.0))
    with pytest.raises(NotImplementedError):
        DsviTrainer(m, lr=0.1).load_optimizer_state(sd_bad)


def test_save_model_then_continuous_training(tmp_path):
    """inference(save_model=True) writes the reference's checkpoint dict (code/nmgp_dsvi.py:893-899);
    continuous_training=True (:789-792) resumes from it: parameters, lr and the Adam step count."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import inference
    g, xs, ys = _toy()
    path = str(tmp_path / "model.pt")
    torch.manual_seed(0)
    m1, l1, _ = inference(xs, ys, g["z"], 200, 2, hyperpars=dict(TOY_HYPER), lr=0.005, itnum=2, show_ELBO=False,
                          save_model=True, PATH=path, device="cuda:0")
    ck = torch.load(path, weights_only=True)
    assert set(ck) == {"epoch", "model_state_dict", "optimizer_state_dict", "loss"}
    assert list(ck["model_state_dict"]) == O.PARAM_NAMES
    assert len(ck["optimizer_state_dict"]["state"]) == 10          # 3 frozen length scales: no state
    assert float(ck["loss"]) == pytest.approx(float(l1[-1]))
    torch.manual_seed(1)
    m2, l2, _ = inference(xs, ys, g["z"], 200, 2, hyperpars=dict(TOY_HYPER), lr=0.9, itnum=1, show_ELBO=False,
                          continuous_training=True, PATH=path, device="cuda:0")
    assert np.isfinite(float(l2[0]))
    # the resumed run started from the saved parameters and did exactly one Adam step of lr 0.005
    moved = float((m2._theta - m1._theta).abs().max())
    assert 0 < moved < 0.05                 # lr 0.9 from the call would move parameters by ~0.9


def test_whole_model_pickle_roundtrip(tmp_path):
    """The drivers pickle whole NMGP objects (code/NMGP_PM25.py:101-106)."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP
    g, xs, ys = _toy()
    m = NMGP(200, 2, g["z"], device="cuda:0")
    m.length_scales_L0_log.requires_grad = False
    p = tmp_path / "m.pickle"
    with open(p, "wb") as fh:
        pickle.dump([m, [1.0, 2.0]], fh)
    with open(p, "rb") as fh:
        m2, lst = pickle.load(fh)
    assert torch.equal(m2._theta, m._theta) and lst == [1.0, 2.0]
    assert not m2.length_scales_L0_log.requires_grad
    m2._assert_views()
    torch.manual_seed(4)
    a = float(m(xs, ys))
    torch.manual_seed(4)
    b = float(m2(xs, ys))
    assert a == b


# ------------------------------------------------------------------------------ f4 pipeline
def _hcp_like(D=4, n=300, seed=2):
    rng = np.random.default_rng(seed)
    X = [np.sort(rng.uniform(0, 1, n)).reshape(-1, 1) for _ in range(D)]
    Y = [np.sin(6 * x + d) + 0.1 * rng.standard_normal(x.shape) for d, x in enumerate(X)]
    return X, Y


@pytest.mark.parametrize("bs", [400, 350])          # 350: a ragged last minibatch of 150 rows
def test_device_pipeline_graph_equals_eager(bs):
    """noise="device": the on-device pipeline with one graph replay per step gives the same
    parameters and losses as the same pipeline launched eagerly."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import inference
    X, Y = _hcp_like()
    hyper = {"length_scales_L0_log": -2.0, "length_scales_L1_log": -2.0, "length_scales_tildeell_log": -2.0}
    res = []
    for use_graph in (False, True):
        torch.manual_seed(0)
        m, losses, times = inference(X, Y, np.linspace(0, 1, 32), bs, 4, hyperpars=hyper, lr=0.01, itnum=3,
                                     show_ELBO=False, device="cuda:0", noise="device", use_graph=use_graph)
        res.append((m._theta.detach().cpu().clone(), np.array([float(v) for v in losses]), times))
    nb = -(-1200 // bs)
    assert len(res[0][1]) == len(res[1][1]) == 3 * nb
    np.testing.assert_allclose(res[1][1], res[0][1], rtol=1e-12)
    assert _rel(res[1][0], res[0][0]) < 1e-12
    assert all(np.diff(res[1][2]) >= 0) and len(res[1][2]) == 3 * nb


def test_device_pipeline_batches_are_the_reference_minibatches():
    """The first step of the device pipeline sees the reference DataLoader's first minibatch, grouped
    by output as vec2list makes it (seeded global generator)."""
    from torch.utils.data import DataLoader
    from collaborative_nonstationary_multivariate_gaussian_process_amd import nmgp_dsvi as NM
    X, Y = _hcp_like(D=3, n=100)
    torch.manual_seed(11)
    Xv = torch.from_numpy(np.concatenate(X)); Yv = torch.from_numpy(np.concatenate(Y))
    Iv = torch.from_numpy(np.concatenate([np.full((100, 1), d) for d in range(3)])).double()
    xb, yb, ib = next(iter(DataLoader(NM.trainData(Xv, Yv, Iv), batch_size=64, shuffle=True)))
    xl, yl = NM.vec2list(xb, yb, ib, dim=3)
    torch.manual_seed(11)
    m = NM.NMGP(300, 3, np.linspace(0, 1, 16), device="cuda:0", noise="device")
    tr = NM.DsviTrainer(m, 0.01)
    pipe = NM._DevicePipeline(m, tr, Xv.reshape(-1), Yv.reshape(-1), Iv.reshape(-1), 64, 0, 1, False, True)
    torch.manual_seed(11)
    plan = pipe.epoch(list(NM._index_loader(300, 64)))
    eng = plan[0]["eng"]
    tr.grad_step(eng)
    torch.cuda.synchronize()
    assert torch.equal(eng.x.cpu(), torch.cat(xl).reshape(-1))
    assert torch.equal(eng.y.cpu(), torch.cat(yl).reshape(-1))
    seg = np.concatenate([[0], np.cumsum([len(x) for x in xl])])
    assert np.array_equal(eng.seg.cpu().numpy(), seg)


# ------------------------------------------------------------------------------ drivers
def test_drivers_vtvlcm_run_and_reload(tmp_path):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.drivers import NMGP_HCP, NMGP_PM25, \
        synthetic_data
    NMGP_PM25.set_data(*synthetic_data(3, 120, 30, t_max=24.0, seed=1))
    model, losses, rmse, times = NMGP_PM25.VTVLCM("PM25", 16, batchsize=100, lr=0.01, itnum=2, do_test=True,
                                                  res_dir=str(tmp_path), verbose=False, device="cuda:0")
    nb = -(-360 // 100)
    assert len(losses) == len(rmse) == len(times) == 2 * nb
    assert np.all(np.isfinite([float(v) for v in losses]))
    assert float(model.length_scales_L0_log) == 10 and not model.length_scales_L0_log.requires_grad
    assert not torch.allclose(model.mu_v.detach().cpu(), torch.ones(16, dtype=torch.float64))   # trained from 1
    again = NMGP_PM25.VTVLCM("PM25", 16, batchsize=100, do_inference=False, do_test=True, res_dir=str(tmp_path))
    assert torch.equal(again[0]._theta.cpu(), model._theta.cpu()) and again[1] == losses
    NMGP_HCP.set_data(*synthetic_data(4, 80, 0, t_max=1.0, seed=2))
    model, losses, times = NMGP_HCP.VTVLCM("HCP", 16, batchsize=0, itnum=3, res_dir=None, verbose=False,
                                           device="cuda:0", noise="device", dtype=torch.float32)
    assert model._theta.dtype == torch.float32 and len(losses) == 3
    assert float(model.length_scales_tildeell_log) == 5


# ------------------------------------------------------------------------------ packed pair layout
def test_packed_pair_layout_matches_dense():
    """pair_layout="packed" (the ECoG memory layout: Q live pairs instead of D^2 blocks) gives the same
    loss and gradients as the reference's dense layout; state_dict exports / accepts dense shapes."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
    g = G.load("mid_forward")
    xs, ys = G.split_lists(g)
    p = G.params(g, D=3, M=64)
    res = {}
    for layout in ("dense", "packed"):
        m = NMGP(4096, 3, g["z"], device="cuda:0", noise="device", pair_layout=layout,
                 **{k: p[k].numpy() for k in ["mu_W", "sqrt_W", "mu_v", "sqrt_v", "mu_U", "sqrt_U"]})
        with torch.no_grad():
            for k in O.PARAM_NAMES[6:]:
                getattr(m, k).data.fill_(float(p[k]))
        assert m.packed == (layout == "packed")
        sd = m.state_dict()
        assert tuple(sd["sqrt_U"].shape) == (3, 3, 64, 64) and tuple(sd["mu_U"].shape) == (3, 3, 64)
        eng = m.engine(sum(len(x) for x in xs))
        eng.load_batch(g["x"], g["y"], [len(x) for x in xs], noise=g["noise"])
        tr = DsviTrainer(m, lr=0.01)
        tr.grad_step(eng, noise=g["noise"])
        torch.cuda.synchronize()
        eng.check_info()
        grads = {k: v.clone() for k, v in zip(O.PARAM_NAMES, m._grad_views)}
        if m.packed:
            from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import _unpack_pairs
            grads = {k: (_unpack_pairs(v, 3) if k in ("mu_U", "sqrt_U") else v) for k, v in grads.items()}
        res[layout] = (float(eng.out[0]), grads, m)
    (ld, gd, md), (lp, gp, mp) = res["dense"], res["packed"]
    assert lp == pytest.approx(ld, rel=1e-13)
    # (the layouts order the pair columns differently -- dense (0,0),(0,1),..., packed (0,0),(1,0),(1,1),...
    # -- so sums over pairs, e.g. the KL mean products over the Y columns, round differently: the scalar
    # hyper-parameter gradients, sums with cancellation, differ at ~1e-12 relative; the step itself is
    # bit-reproducible, tests/test_gpu_engine.py::test_step_is_deterministic_run_to_run)
    for k in O.PARAM_NAMES:
        if float(gd[k].norm()) > 0:
            assert _rel(gp[k], gd[k]) < 1e-11, k
    # the packed model's dense export holds the live pairs; a dense state_dict loads into it
    ii, jj = np.tril_indices(3)
    for k in ("mu_U", "sqrt_U"):
        assert torch.equal(mp.state_dict()[k][ii, jj].cpu(), md.state_dict()[k][ii, jj].cpu())
    mp.load_state_dict(md.state_dict())
    assert torch.equal(mp.sqrt_U.detach(), md.sqrt_U.detach()[ii, jj])


def test_packed_export_allocates_no_device_memory():
    """state_dict() and the Adam state export of a packed model build the reference's dense mu_U / sqrt_U
    on the host (at the ECoG shape one dense fp32 sqrt_U is 69 GB): device memory in use is unchanged
    across the exports, and the exported pairs equal the device's packed pairs."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import (
        NMGP, DsviTrainer, _adam_state_dict)
    D, M = 6, 96
    m = NMGP(1000, D, np.linspace(0, 1, M), device="cuda:0", noise="device", pair_layout="packed",
             dtype=torch.float32)
    tr = DsviTrainer(m, lr=0.01)
    tr.m.normal_()
    torch.cuda.synchronize()
    before = torch.cuda.memory_allocated()
    sd = m.state_dict()
    opt = _adam_state_dict(m, tr)
    torch.cuda.synchronize()
    assert torch.cuda.memory_allocated() == before
    assert sd["sqrt_U"].device.type == "cpu" and tuple(sd["sqrt_U"].shape) == (D, D, M, M)
    ii, jj = np.tril_indices(D)
    assert torch.equal(sd["sqrt_U"][ii, jj], m.sqrt_U.detach().cpu())
    assert float(sd["sqrt_U"][0, 1].abs().sum()) == 0.0
    o, _ = m._offs["sqrt_U"]
    ea = opt["state"][5]["exp_avg"]
    assert tuple(ea.shape) == (D, D, M, M)
    assert torch.equal(ea[ii, jj].reshape(-1), tr.m[o:o + ea[ii, jj].numel()].cpu())


def test_inference_with_test_lists_rmse_matches_predict_after_training():
    """inference(X_test_list=...) predicts every iteration on the device (code/nmgp_dsvi.py:865-868) without
    host synchronisation: one RMSE per step, the last equal to predict_Y on the trained model (same
    parameters), numpy floats like the reference's."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import inference, predict_Y
    rng = np.random.default_rng(21)
    D, n, M = 3, 150, 32
    X = [np.sort(rng.uniform(0, 1, n))[:, None] for _ in range(D)]
    Y = [np.sin(5 * x + d) + 0.1 * rng.standard_normal(x.shape) for d, x in enumerate(X)]
    Xt = [np.sort(rng.uniform(0, 1, 40))[:, None] for _ in range(D)]
    Yt = [np.sin(5 * x + d) for d, x in enumerate(Xt)]
    hyper = {"length_scales_tildeell_log": -1.5, "length_scales_L0_log": -1.5, "length_scales_L1_log": -1.5}
    for noise in ("device", "torch"):
        torch.manual_seed(0)
        model, losses, rmse, times = inference(X, Y, np.linspace(0, 1, M), 150, D, hyperpars=hyper, itnum=3,
                                               show_ELBO=False, device="cuda:0", noise=noise,
                                               X_test_list=Xt, Y_test_list=Yt)
        assert len(rmse) == len(losses) == len(times) == 9
        assert all(isinstance(r, np.floating) and np.isfinite(r) for r in rmse)
        est = predict_Y(model, Xt)
        ref = np.sqrt(np.mean((est[:, None] - np.concatenate(Yt)) ** 2))
        assert float(rmse[-1]) == pytest.approx(float(ref), rel=1e-12)


@pytest.mark.parametrize("M,dt", [(514, torch.float32), (513, torch.float64)])
def test_unaligned_M_trains_with_the_dense_adam(M, dt):
    """from M = 512 the trainer updated the sqrt blocks with nmgp_adam_lower, which needs M (and every
    block offset) to be a multiple of 16 / element size -- fp32 M = 514 or fp64 M = 513 raised at the first
    optimizer step.  Such shapes now take the dense Adam: inference runs and its update equals
    torch.optim.Adam's first step on the same gradient."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer, inference
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import use_adam_lower
    g, xs, ys = _toy()
    z = np.linspace(0, 1, M)
    m = NMGP(200, 2, z, device="cuda:0", noise="device", dtype=dt)
    assert not use_adam_lower(M, dt, m._offs)
    tr = DsviTrainer(m, lr=0.01)
    gen = torch.Generator(device="cuda:0").manual_seed(3)
    m._grad.copy_(torch.randn(m._grad.shape, generator=gen, device="cuda:0", dtype=dt))
    ref = m._theta.detach().clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=0.01)
    ref.grad = m._grad.clone()
    opt.step()
    tr.update()
    assert _rel(m._theta, ref) < (1e-6 if dt == torch.float32 else 1e-14)
    model, losses, _ = inference(xs, ys, z, 200, 2, hyperpars=dict(TOY_HYPER), lr=0.005, itnum=2, show_ELBO=False,
                                 device="cuda:0", noise="device", dtype=dt)
    assert len(losses) == 2 and all(np.isfinite(losses))
