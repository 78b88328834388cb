"""Generate the golden parity fixtures under tests/golden/ from the REAL reference.

Runs ONLY in the build container, where the read-only reference tree is mounted at
/root/reference.  It imports the reference Python (`code/nmgp_dsvi.py`, `code/utils.py`,
`code/SIM_code/Utility/*`), feeds it seeded inputs / parameters / injected noise and
records inputs, intermediates, outputs and gradients into small ``.npz`` files.  Only those
data files travel to the GPU box; the reference source never leaves this container and
nothing in this repository copies it.

torch 2.x removed ``torch.solve`` and ``torch.symeig`` that the reference calls
(``code/utils.py:119,142,154,230``; ``SIM_code/Utility/kronecker_operation.py:45,47,66,67``;
``SIM_code/Utility/distributions.py:37,40``).  Before importing the reference this script
installs a two-symbol shim (LU solve via ``torch.linalg.solve``, ``eigh``); the golden values
therefore reflect torch-2.10 LAPACK.

The toy data come from ``data/simulation/sim_illustration_*_freq.pickle``.  Those pickles are
NOT unpickled: ``_pickle_arrays`` walks the opcode stream with ``pickletools.genops`` (a
disassembler that executes nothing) and copies out the raw little-endian float64 payloads.

Usage:  python tests/golden/make_golden.py     (writes tests/golden/*.npz)
"""
import collections
import os
import pickletools
import sys

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

# ----------------------------------------------------------------------------- shim + import
_Sol = collections.namedtuple("solve", ["solution", "LU"])
torch.solve = lambda input, A: _Sol(torch.linalg.solve(A, input), None)
torch.symeig = lambda A, eigenvectors=False, upper=True: torch.linalg.eigh(A, UPLO="U" if upper else "L")
os.environ.setdefault("MPLBACKEND", "Agg")
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(REF, "code"))
sys.path.insert(0, os.path.join(REF, "code", "SIM_code"))
import nmgp_dsvi as R  # noqa: E402
import utils as RU  # noqa: E402
from Utility import kernels as RK  # noqa: E402
from Utility import kronecker_operation as RKO  # noqa: E402
from Utility import distributions as RDIST  # noqa: E402

DT = torch.float64


# ----------------------------------------------------------------------------- helpers
def _pickle_arrays(path):
    """Copy the ndarray payloads out of a protocol-3 pickle WITHOUT unpickling it."""
    data = open(path, "rb").read()
    out, ints, marked, shape, descr, want_descr = [], [], False, None, None, False
    for op, arg, _ in pickletools.genops(data):
        n = op.name
        if n in ("BININT1", "BININT", "BININT2"):
            ints.append(arg)
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = {"TUPLE1": 1, "TUPLE2": 2, "TUPLE3": 3}[n]
            if marked and len(ints) == k + 1:
                shape = tuple(ints[1:])
            ints, marked = [], False
        elif n == "GLOBAL" and arg == "numpy dtype":
            want_descr = True
        elif n in ("BINUNICODE", "SHORT_BINUNICODE") and want_descr:
            descr, want_descr = arg, False
        elif n in ("BINBYTES", "SHORT_BINBYTES", "BINBYTES8") and len(arg) > 1:
            out.append(np.frombuffer(arg, dtype="<" + descr).reshape(shape).copy())
            shape = None
        elif n == "MARK":
            ints, marked = [], True
    return out


def toy_data(kind="low"):
    a = _pickle_arrays(os.path.join(REF, "data", "simulation", f"sim_illustration_{kind}_freq.pickle"))
    assert len(a) == 8
    return a[0:2], a[2:4], a[4:6], a[6:8]   # X_list, Y_list, Xt_list, Yt_list  each (100,1)


class NoiseTape:
    """Replaces torch.randn: 'inject' pops queued arrays, 'record' draws and records."""

    def __init__(self):
        self.orig = torch.randn
        self.mode = None
        self.queue = []
        self.rec = []

    def __call__(self, *size, **kw):
        if self.mode == "inject":
            a = self.queue.pop(0)
            shp = tuple(size[0]) if len(size) == 1 and not isinstance(size[0], int) else tuple(size)
            assert tuple(a.shape) == shp, (a.shape, shp)
            return torch.from_numpy(np.asarray(a, dtype=np.float32).copy())
        t = self.orig(*size, **kw)
        if self.mode == "record":
            self.rec.append(t.detach().clone().numpy())
        return t

    def inject(self, arrays):
        self.mode, self.queue = "inject", list(arrays)

    def record(self):
        self.mode, self.rec = "record", []

    def off(self):
        assert not self.queue, "unconsumed injected noise"
        self.mode = None


TAPE = NoiseTape()
torch.randn = TAPE


class Spy:
    """Wraps the helper names bound in nmgp_dsvi's namespace to record their outputs in call order."""

    NAMES = ["create_RBF", "create_Gibbs", "JGP_S", "MGP_d", "MGP_mu_sigma2", "KL_Gaussian", "Normal_logprob"]

    def __init__(self):
        self.log = []
        self.orig = {n: getattr(R, n) for n in self.NAMES}

    def __enter__(self):
        for n in self.NAMES:
            f = self.orig[n]

            def w(*a, _n=n, _f=f, **k):
                r = _f(*a, **k)
                self.log.append((_n, r))
                return r
            setattr(R, n, w)
        return self

    def __exit__(self, *exc):
        for n, f in self.orig.items():
            setattr(R, n, f)

    def get(self, name):
        return [r for n, r in self.log if n == name]


def np64(t):
    if isinstance(t, (tuple, list)):
        return [np64(x) for x in t]
    return t.detach().cpu().to(DT).numpy() if torch.is_tensor(t) else np.asarray(t)


PARAM_NAMES = ["mu_W", "sqrt_W", "mu_v", "sqrt_v", "mu_U", "sqrt_U",
               "sigma2_tildeell_log", "length_scales_tildeell_log", "sigma2_L0_log",
               "length_scales_L0_log", "sigma2_L1_log", "length_scales_L1_log", "sigma2_err_log"]


def build_model(N, D, z, params=None, seed=22):
    Z = torch.from_numpy(np.asarray(z, np.float64)).type(DT).unsqueeze(1)
    kw = {}
    if params is not None:
        for k in ["mu_v", "mu_W", "mu_U", "sqrt_v", "sqrt_W", "sqrt_U"]:
            kw[k] = params[k]
    m = R.NMGP(number_observations=N, dim_outputs=D, Z=Z, seed=seed, **kw)
    if params is not None:
        for k in PARAM_NAMES[6:]:
            getattr(m, k).data.fill_(float(params[k]))
    return m


def model_params(m):
    return {k: np64(getattr(m, k)) for k in PARAM_NAMES}


def forward_noise(rng, D, M, B):
    Q = D * (D + 1) // 2
    return [rng.standard_normal(M).astype(np.float32), rng.standard_normal(B).astype(np.float32)] + \
           [rng.standard_normal(B).astype(np.float32) for _ in range(Q)]


def run_forward(m, X_list, Y_list, noise, full=True):
    """One reference NMGP.forward + backward with injected noise; returns a fixture dict."""
    Xt = [torch.from_numpy(np.asarray(x, np.float64)).type(DT) for x in X_list]
    Yt = [torch.from_numpy(np.asarray(y, np.float64)).type(DT) for y in Y_list]
    m.zero_grad()
    TAPE.inject(noise)
    with Spy() as spy:
        loss = m(Xt, Yt)
    TAPE.off()
    loss.backward()
    D = m.D
    out = {"loss": np64(loss)}
    for k in PARAM_NAMES:
        g = getattr(m, k).grad
        out["grad_" + k] = np64(g) if g is not None else np.zeros_like(np64(getattr(m, k)))
    if full:
        rbf = spy.get("create_RBF")
        out.update({"K_t12": np64(rbf[0]), "K_t22": np64(rbf[1]), "K_L0_12": np64(rbf[2]),
                    "K_L0_22": np64(rbf[3]), "K_L1_12": np64(rbf[4]), "K_L1_22": np64(rbf[5])})
        jgp = np64(spy.get("JGP_S")[0])
        B = out["K_t12"].shape[0]
        out["sampled_tilde_ell"], out["sampled_v"] = jgp[:B], jgp[B:]
        out["pair_samples"] = np.stack(np64(spy.get("MGP_d")))      # (Q,B) in (i, j<=i) order
        gib = spy.get("create_Gibbs")
        out["K_G12"], out["K_G22"] = np64(gib[0]), np64(gib[1])
        mu_g, s2_g = spy.get("MGP_mu_sigma2")[0]
        out["mu_g"], out["sigma2_g"] = np64(mu_g), np64(s2_g)
        kls = spy.get("KL_Gaussian")
        out["KL_W"] = np64(kls[0].sum())
        out["KL_v"] = np64(kls[1])
        out["KL_U"] = np64(kls[2].sum() + kls[3].sum())
        out["SELBO_logprob"] = np64(spy.get("Normal_logprob")[0])
    return out


def pack_inputs(prefix_dict, X_list, Y_list, z, params, noise):
    d = dict(prefix_dict)
    d["x"] = np.concatenate([np.asarray(x, np.float64).reshape(-1) for x in X_list])
    d["y"] = np.concatenate([np.asarray(y, np.float64).reshape(-1) for y in Y_list])
    d["sizes"] = np.array([np.asarray(x).reshape(-1).shape[0] for x in X_list], np.int64)
    d["z"] = np.asarray(z, np.float64)
    for k, v in params.items():
        d["p_" + k] = np.asarray(v, np.float64)
    d["noise"] = np.concatenate([np.asarray(a, np.float64).reshape(-1) for a in noise])
    return d


def save(name, d):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **d)
    print(f"wrote {path}  ({os.path.getsize(path) / 1024:.1f} KiB)")


TOY_HYPER = {"sigma2_L0_log": 0., "length_scales_L0_log": 2., "sigma2_L1_log": 0., "length_scales_L1_log": 2.,
             "sigma2_tildeell_log": 0., "length_scales_tildeell_log": 0., "sigma2_err_log": -2.}


# ----------------------------------------------------------------------------- cases
def case_toy():
    X_list, Y_list, _, _ = toy_data("low")
    M, D = 20, 2
    z = np.linspace(0, 1, M)
    m = build_model(200, D, z, seed=22)
    for k, v in TOY_HYPER.items():
        getattr(m, k).data.fill_(v)
    params = model_params(m)
    noise = forward_noise(np.random.default_rng(1), D, M, 200)
    out = run_forward(m, X_list, Y_list, noise)
    save("toy_forward", {**pack_inputs({"N": 200}, X_list, Y_list, z, params, noise), **out})


def case_modelpt():
    """Known-answer: the shipped checkpoint state, torch.manual_seed(123), reference's own RNG."""
    X_list, Y_list, _, _ = toy_data("low")
    ck = torch.load(os.path.join(REF, "code", "notebook", "model.pt"), weights_only=True)
    M, D = 20, 2
    z = np.linspace(0, 1, M)
    m = build_model(200, D, z, seed=22)
    m.load_state_dict(ck["model_state_dict"])
    params = model_params(m)
    Xt = [torch.from_numpy(x).type(DT) for x in X_list]
    Yt = [torch.from_numpy(y).type(DT) for y in Y_list]
    torch.manual_seed(123)
    TAPE.record()
    loss = m(Xt, Yt)
    noise = list(TAPE.rec)
    TAPE.off()
    loss.backward()
    out = {"loss": np64(loss)}
    for k in PARAM_NAMES:
        out["grad_" + k] = np64(getattr(m, k).grad)
    print("model.pt known-answer loss", float(loss))
    save("modelpt_forward", {**pack_inputs({"N": 200, "seed": 123}, X_list, Y_list, z, params, noise), **out})


def case_modelpt_file():
    """The shipped checkpoint code/notebook/model.pt, loaded weights-only and re-saved as plain tensors
    (same dict layout: epoch, model_state_dict, optimizer_state_dict with the old torch's object-id
    keys, loss) so the GPU box -- where the reference tree does not exist -- can load it through
    NMGP.load_state_dict / the optimizer-state path."""
    ck = torch.load(os.path.join(REF, "code", "notebook", "model.pt"), weights_only=True, map_location="cpu")
    out = {"epoch": int(ck["epoch"]), "loss": ck["loss"].detach().clone(),
           "model_state_dict": {k: v.detach().clone() for k, v in ck["model_state_dict"].items()},
           "optimizer_state_dict": {
               "state": {int(k): {"step": torch.tensor(float(v["step"])), "exp_avg": v["exp_avg"].detach().clone(),
                                  "exp_avg_sq": v["exp_avg_sq"].detach().clone()}
                         for k, v in ck["optimizer_state_dict"]["state"].items()},
               "param_groups": [dict(g) for g in ck["optimizer_state_dict"]["param_groups"]]}}
    path = os.path.join(OUT, "model_pt.pt")
    torch.save(out, path)
    print(f"wrote {path}  ({os.path.getsize(path) / 1024:.1f} KiB)")


def synth_case(D, M, sizes, seed, mu_v0, hyper):
    rng = np.random.default_rng(seed)
    X_list = [np.sort(rng.uniform(0, 1, n))[:, None] for n in sizes]
    Y_list = [rng.standard_normal(n)[:, None] for n in sizes]
    z = np.linspace(0, 1, M)
    params = {"mu_W": 0.1 * rng.standard_normal((D, M)), "sqrt_W": 0.1 * rng.standard_normal((D, M, M)),
              "mu_v": mu_v0 + 0.1 * rng.standard_normal(M), "sqrt_v": 0.1 * rng.standard_normal((M, M)),
              "mu_U": 0.1 * rng.standard_normal((D, D, M)), "sqrt_U": 0.1 * rng.standard_normal((D, D, M, M))}
    params.update(hyper)
    return X_list, Y_list, z, params, rng


def case_mid():
    D, M, sizes = 3, 64, [150, 170, 192]
    hyper = {"sigma2_tildeell_log": 0.1, "length_scales_tildeell_log": -2.0, "sigma2_L0_log": -0.2,
             "length_scales_L0_log": -2.0, "sigma2_L1_log": 0.3, "length_scales_L1_log": -1.5, "sigma2_err_log": -1.0}
    X_list, Y_list, z, params, rng = synth_case(D, M, sizes, 7, -3.0, hyper)
    m = build_model(4096, D, z, params)
    noise = forward_noise(rng, D, M, sum(sizes))
    out = run_forward(m, X_list, Y_list, noise)
    save("mid_forward", {**pack_inputs({"N": 4096}, X_list, Y_list, z, params, noise), **out})


def case_pm25():
    """PM2.5-shaped: D=5, M=256, B=2000, NMGP(seed=22) init, length-scale logs -1."""
    D, M, sizes = 5, 256, [400] * 5
    rng = np.random.default_rng(0)
    X_list = [np.sort(rng.uniform(0, 1, n))[:, None] for n in sizes]
    Y_list = [rng.standard_normal(n)[:, None] for n in sizes]
    z = np.linspace(0, 1, M)
    m = build_model(10000, D, z, seed=22)
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        getattr(m, k).data.fill_(-1.0)
    params = model_params(m)
    noise = forward_noise(rng, D, M, sum(sizes))
    out = run_forward(m, X_list, Y_list, noise, full=False)
    small = {"loss": out["loss"]}
    for k in PARAM_NAMES:
        g = out["grad_" + k]
        small["gnorm_" + k] = np.linalg.norm(g.reshape(-1))
        small["gsample_" + k] = g.reshape(-1)[:: max(1, g.size // 997)]
    # the big parameters are regenerated from seed 22 on load (NMGP init), keep only scalars+small
    keep = {k: v for k, v in params.items() if k not in ("sqrt_W", "sqrt_U", "sqrt_v")}
    d = pack_inputs({"N": 10000}, X_list, Y_list, z, keep, noise)
    save("pm25_forward", {**d, **small})


def _grad_digest(out):
    """Per-parameter gradient norms + a strided sample of every gradient (big fixtures)."""
    small = {"loss": out["loss"]}
    for k in PARAM_NAMES:
        g = out["grad_" + k]
        small["gnorm_" + k] = np.linalg.norm(g.reshape(-1))
        small["gsample_" + k] = g.reshape(-1)[:: max(1, g.size // 997)]
    return small


def case_hcp_like():
    """HCP-shaped at a size the reference finishes on the CPU: D=8 outputs,
    M=512 inducing points, B=5000 rows (625 per output), N=50000, length scales 3/M of the input
    range (cond(K22 + 1e-4 I) moderate), NMGP(seed=22) initialisation.  The fp32 engine
    is gated against this fp64 reference at SURVEY §8c's fp32 tolerances."""
    D, M, sizes = 8, 512, [625] * 8
    rng = np.random.default_rng(21)
    X_list = [np.sort(rng.uniform(0, 1, n))[:, None] for n in sizes]
    Y_list = [(np.sin(6 * x + 0.5 * d) + 0.3 * rng.standard_normal(x.shape)) for d, x in enumerate(X_list)]
    z = np.linspace(0, 1, M)
    m = build_model(50000, D, z, seed=22)
    ls = float(np.log(3.0 / M))
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        getattr(m, k).data.fill_(ls)
    params = model_params(m)
    noise = forward_noise(rng, D, M, sum(sizes))
    out = run_forward(m, X_list, Y_list, noise, full=False)
    keep = {k: v for k, v in params.items() if k not in ("sqrt_W", "sqrt_U", "sqrt_v")}
    d = pack_inputs({"N": 50000}, X_list, Y_list, z, keep, noise)
    save("hcp_like_forward", {**d, **_grad_digest(out)})


def case_driver_hyper():
    """The reference drivers' own hyper-parameters (code/NMGP_PM25.py:63-64): length-scale logs 10
    and mu_v = 1 on an hour-indexed axis (z = linspace(0, t_max, M), t_max = 5000 h), where the RBF
    priors are nearly rank one and only the 1e-4 jitter keeps K22 positive-definite."""
    D, M, sizes = 3, 64, [190, 210, 200]
    rng = np.random.default_rng(31)
    t_max = 5000.0
    X_list = [np.sort(rng.uniform(0, t_max, n))[:, None] for n in sizes]
    Y_list = [(np.sin(x / 700.0 + d) + 0.3 * rng.standard_normal(x.shape)) for d, x in enumerate(X_list)]
    z = np.linspace(0, t_max, M)
    m = build_model(6000, D, z, params={"mu_v": np.ones(M), "mu_W": None, "mu_U": None, "sqrt_v": None,
                                        "sqrt_W": None, "sqrt_U": None, **{k: 0.0 for k in PARAM_NAMES[6:]}},
                    seed=22)
    for k, v in {"length_scales_L0_log": 10., "length_scales_L1_log": 10., "length_scales_tildeell_log": 10.,
                 "sigma2_tildeell_log": 0., "sigma2_L0_log": 0., "sigma2_L1_log": 0., "sigma2_err_log": -2.}.items():
        getattr(m, k).data.fill_(v)
    params = model_params(m)
    noise = forward_noise(rng, D, M, sum(sizes))
    out = run_forward(m, X_list, Y_list, noise, full=False)
    save("driver_hyper_forward", {**pack_inputs({"N": 6000}, X_list, Y_list, z, params, noise), **out})


def case_ecog_like():
    """ECoG-full-shaped at a size the reference finishes on the CPU: M = 1024
    inducing points with the ECoG configuration's length scales 3/M (code/NMGP_ECoG_full.py trains at
    M = 1024), D = 4 outputs, B = N = 2000 rows (500 per output), NMGP(seed=22) initialisation.
    Records (1) one forward + backward with injected noise (gradient digest) and (2) compute_ELBO over
    the same data with 2 injected-noise samples (per-sample reconstruction terms + ELBO).  At M = 1024
    the fp32 engine takes its large-M path: recursive chol_inv_rec, the 128x128 offsets products and
    (with pair_layout="packed") the packed pair layout -- this fixture pins that path."""
    D, M, sizes = 4, 1024, [500] * 4
    N = sum(sizes)
    rng = np.random.default_rng(41)
    X_list = [np.sort(rng.uniform(0, 1, n))[:, None] for n in sizes]
    Y_list = [(np.sin(6 * x + 0.7 * d) + 0.3 * rng.standard_normal(x.shape)) for d, x in enumerate(X_list)]
    z = np.linspace(0, 1, M)
    m = build_model(N, D, z, seed=22)
    ls = float(np.log(3.0 / M))
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        getattr(m, k).data.fill_(ls)
    params = model_params(m)
    noise = forward_noise(rng, D, M, N)
    out = run_forward(m, X_list, Y_list, noise, full=False)
    keep = {k: v for k, v in params.items() if k not in ("sqrt_W", "sqrt_U", "sqrt_v")}
    d = pack_inputs({"N": N}, X_list, Y_list, z, keep, noise)
    S = 2
    enoise = []
    for _ in range(S):
        enoise += forward_noise(rng, D, M, N)
    Xt = [torch.from_numpy(x).type(DT) for x in X_list]
    Yt = [torch.from_numpy(y).type(DT) for y in Y_list]
    TAPE.inject(enoise)
    with Spy() as spy, torch.no_grad():
        elbo = m.compute_ELBO(Xt, Yt, n_sample=S)
    TAPE.off()
    lp = np64(spy.get("Normal_logprob"))
    d.update({"elbo_n_sample": S, "elbo_noise": np.concatenate([np.asarray(a, np.float64).reshape(-1) for a in enoise]),
              "elbo": np64(elbo), "elbo_logprob_per_sample": np.array(lp)})
    print("ecog_like loss", float(out["loss"]), "elbo", float(elbo))
    save("ecog_like_forward", {**d, **_grad_digest(out)})


def case_elbo():
    X_list, Y_list, _, _ = toy_data("low")
    M, D, N, S = 20, 2, 200, 8
    z = np.linspace(0, 1, M)
    m = build_model(N, D, z, seed=22)
    for k, v in TOY_HYPER.items():
        getattr(m, k).data.fill_(v)
    params = model_params(m)
    rng = np.random.default_rng(3)
    noise = []
    for _ in range(S):
        noise += forward_noise(rng, D, M, N)
    Xt = [torch.from_numpy(x).type(DT) for x in X_list]
    Yt = [torch.from_numpy(y).type(DT) for y in Y_list]
    TAPE.inject(noise)
    with Spy() as spy:
        elbo = m.compute_ELBO(Xt, Yt, n_sample=S)
    TAPE.off()
    lp = np64(spy.get("Normal_logprob"))
    save("toy_elbo", {**pack_inputs({"N": N, "n_sample": S}, X_list, Y_list, z, params, noise),
                      "elbo": np64(elbo), "logprob_per_sample": np.array(lp)})


def case_utils():
    rng = np.random.default_rng(11)
    d = {}
    n, mm = 37, 23
    X = rng.uniform(0, 1, (n, 1)); Z = np.linspace(0, 1, mm)[:, None]
    d["X"], d["Z"] = X, Z
    Xt, Zt = torch.from_numpy(X), torch.from_numpy(Z)
    s2 = torch.tensor(1.3, dtype=DT, requires_grad=True); ls = torch.tensor(0.2, dtype=DT, requires_grad=True)
    K = RU.create_RBF(Xt, Zt, scale2=s2, length_scales=ls)
    Kbar = rng.standard_normal((n, mm)); d["rbf_Kbar"] = Kbar
    (K * torch.from_numpy(Kbar)).sum().backward()
    d["rbf_K"], d["rbf_gs2"], d["rbf_gls"] = np64(K), np64(s2.grad), np64(ls.grad)
    K22 = RU.create_RBF(Zt, scale2=1.3, length_scales=0.2); d["rbf_K22"] = np64(K22)
    ellX = torch.from_numpy(np.exp(rng.normal(-2, 0.3, n))).requires_grad_()
    ellZ = torch.from_numpy(np.exp(rng.normal(-2, 0.3, mm))).requires_grad_()
    d["ellX"], d["ellZ"] = np64(ellX), np64(ellZ)
    G = RU.create_Gibbs(Xt, Zt, ellX, ellZ, scale2=0.7)
    (G * torch.from_numpy(Kbar)).sum().backward()
    d["gibbs_K"], d["gibbs_gellX"], d["gibbs_gellZ"] = np64(G), np64(ellX.grad), np64(ellZ.grad)
    # MGP_d / MGP_mu_sigma2 / KL_Gaussian with grads
    K12 = RU.create_RBF(Xt, Zt, scale2=1.0, length_scales=0.15).requires_grad_()
    K22 = RU.create_RBF(Zt, scale2=1.0, length_scales=0.15).requires_grad_()
    Lm = torch.from_numpy(np.tril(0.2 * rng.standard_normal((3, mm, mm))))
    Sig = (Lm @ Lm.transpose(-1, -2)).requires_grad_()
    mu = torch.from_numpy(0.3 * rng.standard_normal((3, mm))).requires_grad_()
    d11 = torch.ones(n, dtype=DT)
    d["mgp_K12"], d["mgp_K22"], d["mgp_Sigma"], d["mgp_mu"] = np64(K12), np64(K22), np64(Sig), np64(mu)
    mu_Y, s2_Y = RU.MGP_mu_sigma2(K12, K22, d11, mu, Sig)
    wm, ws = rng.standard_normal(mu_Y.shape), rng.standard_normal(s2_Y.shape)
    d["mgp_wm"], d["mgp_ws"] = wm, ws
    ((mu_Y * torch.from_numpy(wm)).sum() + (s2_Y * torch.from_numpy(ws)).sum()).backward()
    d["mgp_muY"], d["mgp_s2Y"] = np64(mu_Y), np64(s2_Y)
    d["mgp_gK12"], d["mgp_gK22"], d["mgp_gmu"], d["mgp_gSigma"] = np64(K12.grad), np64(K22.grad), np64(mu.grad), np64(Sig.grad)
    # MGP_d with injected noise (single pair)
    zd = rng.standard_normal(n).astype(np.float32); d["mgpd_z"] = zd.astype(np.float64)
    TAPE.inject([zd])
    smp = RU.MGP_d(K12.detach(), K22.detach(), d11, mu.detach()[0], Sig.detach()[0])
    TAPE.off()
    d["mgpd_sample"] = np64(smp)
    # JGP_S with injected noise
    zv = rng.standard_normal(mm).astype(np.float32); zt = rng.standard_normal(n).astype(np.float32)
    d["jgp_zv"], d["jgp_zt"] = zv.astype(np.float64), zt.astype(np.float64)
    TAPE.inject([zv, zt])
    js = RU.JGP_S(torch.ones(n, dtype=DT) * 1.0, K12.detach(), K22.detach(), mu.detach()[1], Sig.detach()[1])
    TAPE.off()
    d["jgp_sample"] = np64(js)
    # KL_Gaussian (batched, quirky term2) with grads
    muk = mu.detach().clone().requires_grad_(); Sk = Sig.detach().clone().requires_grad_()
    K22k = K22.detach().clone().requires_grad_()
    kl = RU.KL_Gaussian(muk, Sk, torch.zeros(mm, dtype=DT), K22k)
    kl.sum().backward()
    d["kl"], d["kl_gmu"], d["kl_gSigma"], d["kl_gK22"] = np64(kl), np64(muk.grad), np64(Sk.grad), np64(K22k.grad)
    # reparameterize full_cov, Normal_logprob, mat2ltri
    zr = rng.standard_normal(mm); d["rep_z"] = zr
    d["rep_full"] = np64(RU.reparameterize(mu.detach()[2], Sig.detach()[2], torch.from_numpy(zr), full_cov=True))
    yy = rng.standard_normal((n, 1)); loc = rng.standard_normal((n, 1)); d["nl_y"], d["nl_loc"] = yy, loc
    d["nl_val"] = np64(RU.Normal_logprob(torch.from_numpy(loc), torch.tensor(0.37, dtype=DT), torch.from_numpy(yy)))
    Sm = rng.standard_normal((2, 3, 5, 5)); d["m2l_in"] = Sm; d["m2l_out"] = np64(RU.mat2ltri(torch.from_numpy(Sm)))
    save("utils_cases", d)


def case_legacy():
    rng = np.random.default_rng(5)
    d = {}
    X1 = rng.standard_normal((31, 3)); X2 = rng.standard_normal((17, 3))
    d["X1"], d["X2"] = X1, X2
    t1, t2 = torch.from_numpy(X1), torch.from_numpy(X2)
    d["pd_12"], d["pd_11"] = np64(RK.pairwise_distances(t1, t2)), np64(RK.pairwise_distances(t1))
    d["rbf_12"] = np64(RK.RBF_cov(t1, t2, alpha=1.7, beta=0.8))
    d["rbf_11"] = np64(RK.RBF_cov(t1, alpha=1.7, beta=0.8))
    s1, s2 = np.exp(rng.normal(0, .3, 31)), np.exp(rng.normal(0, .3, 17))
    e1, e2 = np.exp(rng.normal(0, .3, 31)), np.exp(rng.normal(0, .3, 17))
    d["sig1"], d["sig2"], d["ell1"], d["ell2"] = s1, s2, e1, e2
    d["ns_12"] = np64(RK.Nonstationary_RBF_cov(t1, torch.from_numpy(s1), torch.from_numpy(e1), t2,
                                               torch.from_numpy(s2), torch.from_numpy(e2)))
    d["ns_11"] = np64(RK.Nonstationary_RBF_cov(t1, torch.from_numpy(s1), torch.from_numpy(e1)))
    d["ns_11_default"] = np64(RK.Nonstationary_RBF_cov(t1))
    A = rng.standard_normal((3, 4)); Bm = rng.standard_normal((5, 2))
    d["kp_A"], d["kp_B"] = A, Bm
    d["kp_AB"] = np64(RKO.kronecker_product(torch.from_numpy(A), torch.from_numpy(Bm)))
    d1, d2 = rng.standard_normal(6), rng.standard_normal(7)
    d["kd_1"], d["kd_2"] = d1, d2
    d["kd_out"] = np64(RKO.kronecker_product_diag(torch.from_numpy(d1), torch.from_numpy(d2)))
    Bk = rng.standard_normal((4, 6)); Kk = rng.standard_normal((9, 5)); yk = rng.standard_normal(6 * 5)
    d["mv_B"], d["mv_K"], d["mv_y"] = Bk, Kk, yk
    d["mv_out"] = np64(RKO.kron_mv(torch.from_numpy(Bk), torch.from_numpy(Kk), torch.from_numpy(yk)))
    LB = rng.standard_normal((3, 3)); LK = rng.standard_normal((4, 4))
    SB, SK = LB @ LB.T + 0.5 * np.eye(3), LK @ LK.T + 0.5 * np.eye(4)
    d["ki_B"], d["ki_K"] = SB, SK
    d["ki_inv"] = np64(RKO.kron_inv(torch.tensor(0.3, dtype=DT), torch.from_numpy(SB), torch.from_numpy(SK)))
    d["ki_logdet"] = np64(RKO.kron_logdet(torch.tensor(0.3, dtype=DT), torch.from_numpy(SB), torch.from_numpy(SK)))
    yl = rng.standard_normal(12); d["lp_y"] = yl
    d["lp_val"] = np64(RDIST.multivariate_normal_logpdf0(torch.from_numpy(yl), torch.zeros(12, dtype=DT),
                                                         torch.from_numpy(SB), torch.from_numpy(SK),
                                                         torch.tensor(0.3, dtype=DT)))
    save("legacy_cases", d)


def case_inference():
    """Two full-batch training iterations through the reference `inference` loop (Adam, lr 0.005)."""
    X_list, Y_list, _, _ = toy_data("low")
    M, D = 20, 2
    z = np.linspace(0, 1, M)
    rec_batches, rec_noise = [], []
    orig_fwd = R.NMGP.forward

    def fwd(self, inputs_list, outputs_list, index=None, verbose=False):
        rec_batches.append(([np64(x).reshape(-1) for x in inputs_list], [np64(y).reshape(-1) for y in outputs_list]))
        n0 = len(TAPE.rec)
        r = orig_fwd(self, inputs_list, outputs_list, index, verbose)
        rec_noise.append(TAPE.rec[n0:])
        return r
    R.NMGP.forward = fwd
    torch.manual_seed(0)
    TAPE.record()
    import io, contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        model, loss_list, time_list = R.inference(X_list, Y_list, z, 200, D, hyperpars=dict(TOY_HYPER), lr=0.005,
                                                  itnum=2, show_ELBO=False, seed=22)
    TAPE.off()
    R.NMGP.forward = orig_fwd
    d = {"z": z, "lr": 0.005, "x": np.concatenate(X_list).reshape(-1), "y": np.concatenate(Y_list).reshape(-1),
         "sizes": np.array([len(x) for x in X_list])}
    for it, ((xs, ys), nz) in enumerate(zip(rec_batches, rec_noise)):
        d[f"it{it}_x"] = np.concatenate(xs); d[f"it{it}_y"] = np.concatenate(ys)
        d[f"it{it}_sizes"] = np.array([len(x) for x in xs]); d[f"it{it}_noise"] = np.concatenate([a.reshape(-1) for a in nz])
    d["loss_list"] = np.array([float(l) for l in loss_list])
    for k in PARAM_NAMES:
        d["final_" + k] = np64(getattr(model, k))
    # initial params: the model's constructor state (seed 22) with the hyperpars the loop installs
    m0 = build_model(200, D, z, seed=22)
    for k in ["sigma2_tildeell_log", "sigma2_L0_log", "sigma2_err_log"]:
        getattr(m0, k).data.fill_(TOY_HYPER[k])
    getattr(m0, "sigma2_L0_log").data.fill_(TOY_HYPER["sigma2_L1_log"])   # reference quirk nmgp_dsvi.py:784-785
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        getattr(m0, k).data.fill_(TOY_HYPER[k])
    for k in PARAM_NAMES:
        d["init_" + k] = np64(getattr(m0, k))
    save("toy_inference", d)


def case_sample():
    """sample_Y / sample_FY (code/nmgp_dsvi.py:406-580) on the trained model.pt state with injected
    noise (reference call order per sample: z_v (M), z_t (N), Q x (N), G (D, N), z_F)."""
    X_list, _, _, _ = toy_data("low")
    ck = torch.load(os.path.join(REF, "code", "notebook", "model.pt"), weights_only=True)
    M, D, S = 20, 2, 3
    Q = D * (D + 1) // 2
    z = np.linspace(0, 1, M)
    m = build_model(200, D, z, seed=22)
    m.load_state_dict(ck["model_state_dict"])
    params = model_params(m)
    Xs = [X_list[0][:17], X_list[1][:13]]
    N = sum(x.shape[0] for x in Xs)
    rng = np.random.default_rng(5)
    noise_y = []
    for _ in range(S):
        noise_y += [rng.standard_normal(M).astype(np.float32), rng.standard_normal(N).astype(np.float32)]
        noise_y += [rng.standard_normal(N).astype(np.float32) for _ in range(Q)]
        noise_y += [rng.standard_normal((D, N)).astype(np.float32), rng.standard_normal(N).astype(np.float32)]
    TAPE.inject(noise_y)
    Ys, Ls, Gs, Ts = m.sample_Y([torch.from_numpy(x).type(DT) for x in Xs], n_sample=S)
    TAPE.off()
    xf = np.linspace(0.03, 0.97, 11)
    Nf = xf.shape[0]
    noise_f = []
    for _ in range(S):
        noise_f += [rng.standard_normal(M).astype(np.float32), rng.standard_normal(Nf).astype(np.float32)]
        noise_f += [rng.standard_normal(Nf).astype(np.float32) for _ in range(Q)]
        noise_f += [rng.standard_normal((D, Nf)).astype(np.float32), rng.standard_normal((Nf, D)).astype(np.float32)]
    TAPE.inject(noise_f)
    Tf, Yf, Cf = m.sample_FY(torch.from_numpy(xf).type(DT), n_sample=S)
    TAPE.off()
    flat = lambda arrs: np.concatenate([np.asarray(a, np.float64).reshape(-1) for a in arrs])
    d = {"z": z, "n_sample": S, "x0": Xs[0], "x1": Xs[1], "noise_y": flat(noise_y), "xf": xf,
         "noise_f": flat(noise_f), "Ys": np64(Ys), "Ls": np64(Ls), "Gs": np64(Gs), "tilde_ells": np64(Ts),
         "fy_tilde_ells": np64(Tf), "fy_Ys": np64(Yf), "fy_corrs": np64(Cf)}
    for k, v in params.items():
        d["p_" + k] = v
    save("sample_cases", d)


if __name__ == "__main__":
    torch.set_num_threads(8)
    if len(sys.argv) > 1:
        for name in sys.argv[1:]:
            globals()["case_" + name]()
        sys.exit(0)
    case_toy()
    case_modelpt()
    case_mid()
    case_pm25()
    case_elbo()
    case_utils()
    case_legacy()
    case_inference()
    case_sample()
    case_modelpt_file()
    case_hcp_like()
    case_driver_hyper()
    case_ecog_like()
