"""Drop-in for the reference module ``code/nmgp_dsvi.py`` on the MI355X.

Same names, signatures, argument meaning and return types as the reference:
``NMGP``, ``NMGP.forward``, ``NMGP.compute_ELBO``, ``NMGP.predict_Y``, ``inference``,
``vec2list``, ``trainData``, ``pre_intialization``, ``sample_Y``/``predict_Y`` (return numpy).
Parameters are float64 and live in ONE flat device vector (the 13 ``nn.Parameter`` objects are
views of it, registered in the reference order so ``state_dict`` / ``model.pt`` load unchanged);
the objective and all gradients come from the HIP engine (engine.py) in one fused call.

Noise: ``noise="torch"`` (default) draws the reference's own stream -- float32 ``torch.randn`` on
the CPU generator in the reference call order (code/utils.py:123,226,234) -- so a seeded run
reproduces the reference sample for sample; ``noise="device"`` draws Philox normals on the GPU
(fast path, statistically equivalent, used by the benchmark).
"""
import math
import time

import numpy as np
import torch
from torch.nn import Parameter
from torch.utils.data import DataLoader, Dataset

from . import distributed as DD
from . import hip_ops as H
from .engine import DsviEngine, HYPER_NAMES, PARAM_NAMES, param_layout
from .utils import TensorType, tridiagonal_jitter  # noqa: F401  (re-exported like the reference)

F64 = torch.float64


def _default_device():
    if not torch.cuda.is_available():
        raise RuntimeError("collaborative_nonstationary_multivariate_gaussian_process_amd needs a HIP device "
                           "(MI355X); there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def print_mem(itnum, bnum=1):
    """code/nmgp_dsvi.py:26-32 (host RSS) plus device memory."""
    import os
    import psutil
    mem = psutil.Process(os.getpid()).memory_info()[0] / 2. ** 20
    dev = torch.cuda.memory_allocated() / 2. ** 20 if torch.cuda.is_available() else 0.0
    return "iteration: {} batchnum {} memory use: {}MB (device {:.1f}MB)".format(itnum, bnum, mem, dev)


class Model(torch.nn.Module):
    """code/nmgp_dsvi.py:35-83 (kept for API parity)."""

    def forward(self):
        return None

    def _get_param_array(self):
        return np.concatenate([p.detach().cpu().numpy().reshape(-1) for p in self.parameters() if p.requires_grad])

    def _set_parameters(self, param_array):
        i = 0
        for p in self.parameters():
            if p.requires_grad:
                n = p.numel()
                p.data.copy_(torch.as_tensor(np.reshape(param_array[i:i + n], tuple(p.shape))))
                i += n


class trainData(Dataset):
    """code/nmgp_dsvi.py:86-96."""

    def __init__(self, X_data, Y_data, I):
        self.X_data, self.Y_data, self.I = X_data, Y_data, I

    def __getitem__(self, index):
        return self.X_data[index], self.Y_data[index], self.I[index]

    def __len__(self):
        return len(self.X_data)


class _DsviObjective(torch.autograd.Function):
    """-SELBO with its gradient computed in the same fused engine call (no autograd graph)."""

    @staticmethod
    def forward(ctx, model, *params):
        loss = model._engine_forward_backward()
        ctx.model = model
        ctx.grads = [g.clone() for g in model._grad_views]
        return loss.clone()

    @staticmethod
    def backward(ctx, gout):
        return (None,) + tuple(gout * g for g in ctx.grads)


class NMGP(Model):
    """code/nmgp_dsvi.py:99-155: variational parameters + 7 log hyper-parameters."""

    def __init__(self, number_observations, dim_outputs, Z, minibatch_size=None, mu_v=None, mu_W=None, mu_U=None,
                 sqrt_v=None, sqrt_W=None, sqrt_U=None, seed=22, device=None, noise="torch", dtype=F64):
        """Reference signature plus: ``device``; ``noise`` ("torch": the reference's CPU randn stream,
        "device": Philox on the GPU); ``dtype`` (float64 = the reference's arithmetic; float32 for
        the HCP / ECoG-shaped configurations, SURVEY §8d, parity gates loss 1e-3 / grad 2e-2)."""
        super().__init__()
        if dtype not in (torch.float64, torch.float32):
            raise ValueError("dtype must be torch.float64 or torch.float32")
        self.dtype_ = dtype
        self.device_ = torch.device(device) if device is not None else _default_device()
        Zt = torch.as_tensor(Z).detach().to(F64).reshape(-1, 1)
        self.Z = Zt.to(self.device_)
        self.M = int(Zt.shape[0])
        self.N = number_observations
        self.D = dim_outputs
        self.batch_size = minibatch_size
        self.noise = noise
        D, M = self.D, self.M
        # reference initialisation order on the CPU generator (code/nmgp_dsvi.py:115-155)
        torch.random.manual_seed(seed)
        init = {}
        init["mu_W"] = 0.1 * torch.randn(D, M).to(F64) if mu_W is None else torch.from_numpy(np.asarray(mu_W)).to(F64)
        init["sqrt_W"] = 0.1 * torch.randn(D, M, M).to(F64) if sqrt_W is None else torch.from_numpy(np.asarray(sqrt_W)).to(F64)
        init["mu_v"] = -4 * torch.ones(M, dtype=F64) if mu_v is None else torch.from_numpy(np.asarray(mu_v)).to(F64)
        init["sqrt_v"] = 0.1 * torch.randn(M, M).to(F64) if sqrt_v is None else torch.from_numpy(np.asarray(sqrt_v)).to(F64)
        init["mu_U"] = 0.1 * torch.randn(D, D, M).to(F64) if mu_U is None else torch.from_numpy(np.asarray(mu_U)).to(F64)
        init["sqrt_U"] = 0.1 * torch.randn(D, D, M, M).to(F64) if sqrt_U is None else torch.from_numpy(np.asarray(sqrt_U)).to(F64)
        self.sigma2_g = 1
        hyper0 = [0., -4., 0., -4., 0., -4., -2.]
        for k, v in zip(HYPER_NAMES, hyper0):
            init[k] = torch.tensor(v, dtype=F64)
        self._offs, n = param_layout(D, M)
        self._theta = torch.zeros(n, dtype=dtype, device=self.device_)
        self._grad = torch.zeros(n, dtype=dtype, device=self.device_)
        self._grad_views = []
        for k in PARAM_NAMES:
            o, shp = self._offs[k]
            cnt = int(np.prod(shp)) if shp else 1
            view = self._theta[o:o + cnt].view(shp)
            view.copy_(init[k].reshape(shp))
            setattr(self, k, Parameter(view))
            self._grad_views.append(self._grad[o:o + cnt].view(shp))
        self._engines = {}
        self._batch = None
        self._noise_seed = seed
        self._noise_counter = torch.zeros(1, dtype=torch.int64, device=self.device_)

    # ------------------------------------------------------------------------------ plumbing
    def _frozen_mask(self):
        m = 0
        for k, name in enumerate(HYPER_NAMES):
            if not getattr(self, name).requires_grad:
                m |= 1 << k
        return m

    def _assert_views(self):
        for k in PARAM_NAMES:
            p = getattr(self, k)
            o = self._offs[k][0]
            if p.data_ptr() != self._theta.data_ptr() + o * self._theta.element_size():
                raise RuntimeError(f"parameter {k} no longer aliases the flat device vector "
                                   "(re-assigning .data is not supported; use .data.copy_)")

    def engine(self, B, N=None):
        eng = self._engines.get(B)
        if eng is None:
            eng = DsviEngine(self.D, self.M, B, self.Z.cpu().numpy().reshape(-1), device=self.device_,
                             dtype=self.dtype_)
            self._engines[B] = eng
        eng.bind(self._theta, self._grad, frozen_mask=self._frozen_mask(), N=self.N if N is None else N)
        return eng

    def _torch_noise(self, B, n_pairs):
        """The reference's draws, in its call order: z_v (M), z_t (B), then one (B) per pair."""
        parts = [torch.randn(self.M), torch.randn(B)] + [torch.randn(B) for _ in range(n_pairs)]
        return torch.cat(parts).to(F64)

    def _prepare(self, inputs_list, outputs_list, index=None):
        xs = [torch.as_tensor(x).detach().reshape(-1).to(F64).cpu() for x in inputs_list]
        ys = [torch.as_tensor(y).detach().reshape(-1).to(F64).cpu() for y in outputs_list]
        sizes = [int(x.shape[0]) for x in xs]
        return torch.cat(xs).numpy(), torch.cat(ys).numpy(), sizes

    def _engine_forward_backward(self):
        eng, noise = self._batch
        if noise is None:
            eng.device_noise(self._noise_seed, self._noise_counter)
            H.counter_add_(self._noise_counter, 1)
        out = eng.forward_backward()
        return out[0]

    # ------------------------------------------------------------------------------ reference API
    def forward(self, inputs_list, outputs_list, index=None, verbose=False):
        """code/nmgp_dsvi.py:157-301: one-sample -SELBO; gradients to all 13 parameters."""
        t1 = time.time()
        self._assert_views()
        x, y, sizes = self._prepare(inputs_list, outputs_list, index)
        B = sum(sizes)
        eng = self.engine(B)
        noise = self._torch_noise(B, self.D * (self.D + 1) // 2) if self.noise == "torch" else None
        eng.load_batch(x, y, sizes, noise=noise, index=index)
        self._batch = (eng, noise)
        loss = _DsviObjective.apply(self, *[getattr(self, k) for k in PARAM_NAMES])
        if verbose:
            torch.cuda.synchronize()
            print("forward+backward (fused) costs {}s".format(time.time() - t1))
        return loss

    def compute_ELBO(self, inputs_list, outputs_list, index=None, n_sample=1000, verbose=False,
                     distributed=False, group=None):
        """code/nmgp_dsvi.py:303-404: MC mean of the column-gathered reconstruction term minus the
        KL terms of the LAST sample's K_G22 (reference quirks kept).

        distributed=True shards the samples over the ranks of `group` (every rank must call;
        every rank returns the same value): rank r evaluates samples r, r+W, ..., the noise
        stream is still consumed in sample order on every rank so results match one process.
        """
        self._assert_views()
        x, y, sizes = self._prepare(inputs_list, outputs_list, index)
        B = sum(sizes)
        eng = self.engine(B, N=self.N)
        acc = torch.zeros((), dtype=F64, device=self.device_)
        Q = self.D * (self.D + 1) // 2
        rank, world = DD.world_info(group) if distributed else (0, 1)
        out, kl = None, None
        for s in range(n_sample):
            if verbose:
                print("Monte Carlo index:", s)
            noise = self._torch_noise(B, Q) if self.noise == "torch" else None
            if s % world != rank:                       # another rank's sample: keep the stream in step
                if noise is None:
                    H.counter_add_(self._noise_counter, 1)
                continue
            eng.load_batch(x, y, sizes, noise=noise, index=index)
            if noise is None:
                eng.device_noise(self._noise_seed, self._noise_counter)
                H.counter_add_(self._noise_counter, 1)
            out = eng.elbo_sample(with_kl=(s == n_sample - 1))
            acc += out[1]
            if s == n_sample - 1:
                kl = out[2] + out[3] + out[4]
        if world == 1:
            return (acc / n_sample - out[2] - out[3] - out[4]).detach().clone()
        return DD.combine_elbo(acc, kl, n_sample, group=group, device=self.device_).detach().clone()

    def predict_Y(self, inputs_list, index=None):
        """code/nmgp_dsvi.py:666-722: posterior-mean prediction (returns a tensor)."""
        from . import predict
        return predict.predict_mean(self, inputs_list, index)


# ==================================================================================== module-level API
def plot_samples(grids, S, true_X, true_Y):
    raise NotImplementedError("plotting is out of scope (SURVEY §2 C14)")


def pre_intialization(M, D, factor=1e-2):
    """code/nmgp_dsvi.py:737-742."""
    mu_W = np.zeros([D, M])
    sqrt_v = np.eye(M) * factor
    sqrt_W = np.stack([np.eye(M) for _ in range(D)]) * factor
    sqrt_U = np.stack([np.stack([np.eye(M) for _ in range(D)]) for _ in range(D)]) * factor
    return mu_W, sqrt_v, sqrt_W, sqrt_U


def vec2list(X, Y, I, dim, device=None):
    """code/nmgp_dsvi.py:745-755: boolean-mask split per output (order preserved)."""
    X_list, Y_list = [], []
    for m in range(dim):
        mask = I == m
        xm, ym = X[mask], Y[mask]
        if device is not None:
            xm, ym = xm.to(device), ym.to(device)
        X_list.append(xm)
        Y_list.append(ym)
    return X_list, Y_list


def _apply_hyperpars(model, hyperpars, fix_hyperpars, continuous_training, PATH, optimizer_state):
    """code/nmgp_dsvi.py:779-814 including the sigma2_L1_log -> sigma2_L0_log quirk (:784-785)."""
    if hyperpars is not None:
        if "sigma2_tildeell_log" in hyperpars:
            model.sigma2_tildeell_log.data.fill_(hyperpars["sigma2_tildeell_log"])
        if "sigma2_L0_log" in hyperpars:
            model.sigma2_L0_log.data.fill_(hyperpars["sigma2_L0_log"])
        if "sigma2_L1_log" in hyperpars:
            model.sigma2_L0_log.data.fill_(hyperpars["sigma2_L1_log"])
        if "sigma2_err_log" in hyperpars:
            model.sigma2_err_log.data.fill_(hyperpars["sigma2_err_log"])
    if continuous_training:
        ck = torch.load(PATH, weights_only=True, map_location="cpu")
        with torch.no_grad():
            for k, v in ck["model_state_dict"].items():
                getattr(model, k).data.copy_(v.to(F64))
        optimizer_state.update(ck.get("optimizer_state_dict", {}) or {})
    if fix_hyperpars:
        for name in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
            getattr(model, name).requires_grad = False
            if name in hyperpars:   # TypeError when hyperpars is None, as the reference (:809)
                getattr(model, name).data.fill_(hyperpars[name])


class DsviTrainer:
    """The training-step core used by ``inference`` and the benchmark: fused HIP forward/backward,
    flat-vector HIP Adam (torch.optim.Adam semantics), optional HIP-graph capture of the step."""

    def __init__(self, model, lr, betas=(0.9, 0.999), eps=1e-8):
        self.model = model
        self.lr, self.betas, self.eps = lr, betas, eps
        dev = model.device_
        self.m = torch.zeros_like(model._theta)
        self.v = torch.zeros_like(model._theta)
        self.step_count = torch.zeros(1, dtype=torch.int64, device=dev)
        self.graphs = {}

    def load_optimizer_state(self, sd):
        """Adopt a torch.optim.Adam state_dict (model.pt) for the flat vector."""
        state = sd.get("state", {})
        if not state:
            return
        m = self.model
        steps = []
        for idx, name in enumerate(PARAM_NAMES):
            st = state.get(idx)
            if st is None:
                continue
            o, shp = m._offs[name]
            n = int(np.prod(shp)) if shp else 1
            self.m[o:o + n] = st["exp_avg"].reshape(-1).to(F64)
            self.v[o:o + n] = st["exp_avg_sq"].reshape(-1).to(F64)
            steps.append(int(st["step"]))
        if steps:
            self.step_count.fill_(max(steps))

    def grad_step(self, eng, noise=None, timer=None):
        """[Minibatch gather if a dataset is bound] + noise (device Philox unless host noise was
        loaded) + fused forward/backward."""
        mdl = self.model
        if getattr(eng, "_dataset", None) is not None and noise is None and timer is None:
            # one launch: gather + Philox noise + counter advance + gradient zeroing
            eng.begin_step(mdl._noise_seed, mdl._noise_counter)
            eng.forward_backward(zero_grad=False)
            return eng.out[0]
        if getattr(eng, "_dataset", None) is not None:
            eng.gather_batch()
        if noise is None:
            eng.device_noise(mdl._noise_seed, mdl._noise_counter)
            H.counter_add_(mdl._noise_counter, 1)
        eng.forward_backward(timer=timer)
        return eng.out[0]

    def update(self):
        """torch.optim.Adam update of the flat parameter vector (one HIP launch)."""
        mdl = self.model
        H.adam_(mdl._theta, mdl._grad, self.m, self.v, self.step_count, self.lr, self.betas, self.eps)

    def step(self, eng, noise=None):
        """One DSVI iteration on the batch already loaded in `eng`; returns the device loss scalar."""
        loss = self.grad_step(eng, noise)
        self.update()
        return loss

    def capture(self, eng, include_update=True):
        """Capture noise -> forward -> backward (-> Adam) of `eng` into one HIP graph."""
        mdl = self.model
        body = self.step if include_update else self.grad_step
        s = torch.cuda.Stream(device=mdl.device_)
        s.wait_stream(torch.cuda.current_stream(mdl.device_))
        with torch.cuda.stream(s):
            for _ in range(2):                       # warm-up (lazy attrs, plan upload) outside capture
                body(eng)
        torch.cuda.current_stream(mdl.device_).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body(eng)
        self.graphs[id(eng)] = g
        return g


def inference(X_train_list, Y_train_list, z, batch_size, dim_outputs, hyperpars=None, fix_hyperpars=True,
              mu_v=None, mu_W=None, mu_U=None, sqrt_v=None, sqrt_W=None, sqrt_U=None, lr=0.01, itnum=1000,
              do_stop_criterion=False, seed=22, verbose=False, PATH="model.pt", continuous_training=False,
              show_ELBO=True, save_model=False, X_test_list=None, Y_test_list=None, device=None, noise="torch",
              use_graph=False, n_elbo_sample=1000, distributed=False, group=None, dtype=F64):
    """code/nmgp_dsvi.py:758-909 on the MI355X.

    Returns (model, loss_list, time_list), or (model, loss_list, rmse_test_list, time_list) when
    X_test_list is given -- as the reference.  Extra keyword-only knobs (defaults keep reference
    behaviour): device, noise ("torch" = reference RNG stream | "device"), use_graph (replay the
    step as a HIP graph; needs noise="device"), n_elbo_sample (compute_ELBO samples),
    distributed (data-parallel over the ranks of `group`: every rank draws the same global
    minibatch of batch_size * world rows -- the seeded DataLoader permutation -- trains on its
    contiguous slice, and the gradients are averaged with one all-reduce before the replicated
    Adam step; the reported loss is the rank mean; compute_ELBO shards its samples).
    """
    rank, world = DD.world_info(group) if distributed else (0, 1)
    X_train_vec = np.concatenate(X_train_list)
    Y_train_vec = np.concatenate(Y_train_list)
    train_index = np.concatenate([np.ones_like(Y_train_list[i]) * i for i in range(dim_outputs)]).astype(int)
    X = torch.from_numpy(X_train_vec).type(torch.DoubleTensor)
    Y = torch.from_numpy(Y_train_vec).type(torch.DoubleTensor)
    I = torch.from_numpy(train_index).type(torch.DoubleTensor)
    X_list, Y_list = vec2list(X, Y, I, dim=dim_outputs)
    model = NMGP(number_observations=Y_train_vec.shape[0], dim_outputs=dim_outputs, Z=np.asarray(z, np.float64),
                 minibatch_size=batch_size, mu_v=mu_v, mu_W=mu_W, mu_U=mu_U, sqrt_v=sqrt_v, sqrt_W=sqrt_W,
                 sqrt_U=sqrt_U, seed=seed, device=device, noise=noise, dtype=dtype)
    opt_state = {}
    _apply_hyperpars(model, hyperpars, fix_hyperpars, continuous_training, PATH, opt_state)
    trainer = DsviTrainer(model, lr)
    trainer.load_optimizer_state(opt_state)
    train_loader = DataLoader(trainData(X, Y, I), batch_size=batch_size * world, shuffle=True)
    loss_list, time_list = [], []
    if X_test_list is not None:
        rmse_test_list = []
        Y_test_vec = np.concatenate(Y_test_list)
    if use_graph and noise != "device":
        raise ValueError("use_graph=True needs noise='device' (host RNG cannot be replayed)")
    Q = dim_outputs * (dim_outputs + 1) // 2
    ts = time.time()
    epoch = 0
    losses_dev = []
    for epoch in range(itnum):
        batch = 0
        for X_batch, Y_batch, I_batch in train_loader:
            batch += 1
            if world > 1:                               # this rank's slice of the global minibatch
                sl = DD.rank_slice(X_batch.shape[0], rank, world)
                X_batch, Y_batch, I_batch = X_batch[sl], Y_batch[sl], I_batch[sl]
            X_bl, Y_bl = vec2list(X_batch, Y_batch, I_batch, dim=dim_outputs)
            model._assert_views()
            x, y, sizes = model._prepare(X_bl, Y_bl)
            B = sum(sizes)
            eng = model.engine(B)
            nz = model._torch_noise(B, Q) if noise == "torch" else None
            eng.load_batch(x, y, sizes, noise=nz)
            if use_graph:
                g = trainer.graphs.get(id(eng)) or trainer.capture(eng, include_update=(world == 1))
                g.replay()
                loss = eng.out[0]
            elif world == 1:
                loss = trainer.step(eng, noise=nz)
            else:
                loss = trainer.grad_step(eng, noise=nz)
            if world > 1:
                DD.allreduce_mean_(model._grad, group)
                trainer.update()
                loss = DD.allreduce_mean_(loss.clone().reshape(1), group)[0]
            losses_dev.append(loss.clone())
            torch.cuda.synchronize(model.device_)
            time_list.append(time.time() - ts)
            if X_test_list is not None:
                est = predict_Y(model, X_test_list)
                rmse_test_list.append(np.sqrt(np.mean((est[:, None] - Y_test_vec) ** 2)))
            if verbose:
                print("epoch: {}/{}, batch: {}/{}, loss: {}".format(epoch, itnum, batch,
                                                                   X_train_vec.shape[0] / batch_size, float(loss)))
        if do_stop_criterion and epoch % 5 == 4 and epoch > 5:
            la = np.array([float(v) for v in losses_dev])
            if la[-batch:].sum() > la[-batch * 6:-batch * 5].sum():
                print("Stop criteria is satisfied.")
                break
        if epoch % 100 == 99 and show_ELBO:
            elbo = model.compute_ELBO(X_list, Y_list, n_sample=n_elbo_sample, distributed=distributed, group=group)
            print("epoch: {}, ELBO: {}".format(epoch + 1, float(elbo)))
            print(print_mem(epoch + 1))
    print("training takes {}s".format(time.time() - ts))
    loss_list = [np.array(float(v)) for v in losses_dev]
    if save_model:
        torch.save({"epoch": epoch, "model_state_dict": {k: v.detach().cpu() for k, v in model.state_dict().items()},
                    "optimizer_state_dict": _adam_state_dict(model, trainer, lr),
                    "loss": torch.tensor(float(losses_dev[-1]) if losses_dev else float("nan"))}, PATH)
    if show_ELBO:
        elbo = model.compute_ELBO(X_list, Y_list, n_sample=n_elbo_sample, distributed=distributed, group=group)
        print("epoch: {}, ELBO: {}".format(epoch + 1, float(elbo)))
        print(print_mem(epoch + 1))
    if X_test_list is not None:
        return model, loss_list, rmse_test_list, time_list
    return model, loss_list, time_list


def _adam_state_dict(model, trainer, lr):
    state = {}
    step = float(trainer.step_count.cpu())
    for idx, name in enumerate(PARAM_NAMES):
        if not getattr(model, name).requires_grad:
            continue
        o, shp = model._offs[name]
        n = int(np.prod(shp)) if shp else 1
        state[idx] = {"step": torch.tensor(step), "exp_avg": trainer.m[o:o + n].reshape(shp).cpu(),
                      "exp_avg_sq": trainer.v[o:o + n].reshape(shp).cpu()}
    return {"state": state, "param_groups": [{"lr": lr, "betas": (0.9, 0.999), "eps": 1e-8, "weight_decay": 0,
                                              "amsgrad": False, "params": list(range(len(PARAM_NAMES)))}]}


def sample_Y(model, X_list, n_sample=1000):
    """code/nmgp_dsvi.py:912-918 (numpy outputs)."""
    from . import predict
    out = predict.sample_Y(model, [torch.from_numpy(np.asarray(x)).to(F64) for x in X_list], n_sample=n_sample)
    return tuple(o.cpu().numpy() for o in out)


def sample_FY(model, x, n_sample=1000):
    """code/nmgp_dsvi.py:921-924 (numpy outputs)."""
    from . import predict
    out = predict.sample_FY(model, torch.from_numpy(np.asarray(x)).to(F64), n_sample=n_sample)
    return tuple(o.cpu().numpy() for o in out)


def predict_Y(model, X_list):
    """code/nmgp_dsvi.py:927-930 (numpy output)."""
    X_list = [torch.from_numpy(np.asarray(x)).to(F64) for x in X_list]
    return model.predict_Y(X_list).detach().cpu().numpy()
