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
import os
import time

import numpy as np
import torch
from torch.nn import Parameter
from torch.utils.data import DataLoader, Dataset

from . import _lib as Lb
from . import distributed as DD
from . import hip_ops as H
from .engine import DsviEngine, use_adam_lower, HYPER_NAMES, PARAM_NAMES, lower_block_ranges, param_layout
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
                 sqrt_v=None, sqrt_W=None, sqrt_U=None, seed=22, device=None, noise="torch", dtype=F64,
                 pair_layout="auto"):
        """Reference signature plus: ``device``; ``noise`` ("torch": the reference's CPU randn stream,
        "device": Philox on the GPU); ``dtype`` (float64 = the reference's arithmetic; float32 for
        the HCP / ECoG-shaped configurations, SURVEY §8d, parity gates loss 1e-3 / grad 2e-2);
        ``pair_layout`` ("dense": mu_U (D, D, M) and sqrt_U (D, D, M, M) as the reference; "packed":
        only the Q = D(D+1)/2 live pairs, (Q, M) and (Q, M, M); "auto": packed when the dense sqrt_U
        would exceed 2^31 elements, e.g. the ECoG shape D=128, M=1024).  state_dict() always exports
        the reference's dense shapes (dead upper pairs zero) and load_state_dict accepts them.

        Packed-layout initialisation without explicit mu_U / sqrt_U draws the live pairs' 0.1 N(0,1)
        values on the device (seeded by `seed`): the reference's CPU draw of all D^2 M^2 values is 69
        GB at the ECoG shape.  Pass mu_U / sqrt_U to reproduce a reference initialisation."""
        super().__init__()
        if dtype not in (torch.float64, torch.float32):
            raise ValueError("dtype must be torch.float64 or torch.float32")
        D = dim_outputs
        Zt = torch.as_tensor(Z).detach().to(F64).reshape(-1, 1)
        M = int(Zt.shape[0])
        if pair_layout not in ("dense", "packed", "auto"):
            raise ValueError("pair_layout must be 'dense', 'packed' or 'auto'")
        packed = pair_layout == "packed" or (pair_layout == "auto" and D * D * M * M > 2 ** 31)
        dev = torch.device(device) if device is not None else _default_device()
        # reference initialisation order on the CPU generator (code/nmgp_dsvi.py:115-155)
        torch.random.manual_seed(seed)
        init = {}
        arr = lambda a: torch.from_numpy(np.asarray(a)).to(F64)
        init["mu_W"] = 0.1 * torch.randn(D, M).to(F64) if mu_W is None else arr(mu_W)
        init["sqrt_W"] = 0.1 * torch.randn(D, M, M).to(F64) if sqrt_W is None else arr(sqrt_W)
        init["mu_v"] = -4 * torch.ones(M, dtype=F64) if mu_v is None else arr(mu_v)
        init["sqrt_v"] = 0.1 * torch.randn(M, M).to(F64) if sqrt_v is None else arr(sqrt_v)
        if not packed:
            init["mu_U"] = 0.1 * torch.randn(D, D, M).to(F64) if mu_U is None else arr(mu_U)
            init["sqrt_U"] = 0.1 * torch.randn(D, D, M, M).to(F64) if sqrt_U is None else arr(sqrt_U)
        else:
            init["mu_U"] = None if mu_U is None else _pack_pairs(arr(mu_U), D)
            init["sqrt_U"] = None if sqrt_U is None else _pack_pairs(arr(sqrt_U), D)
        hyper0 = [0., -4., 0., -4., 0., -4., -2.]
        for k, v in zip(HYPER_NAMES, hyper0):
            init[k] = torch.tensor(v, dtype=F64)
        self._setup(number_observations, D, Zt, minibatch_size, noise, dtype, dev, seed, init=init, packed=packed)

    def _setup(self, N, D, Zt, batch_size, noise, dtype, device, seed, init=None, theta=None, packed=False):
        """Allocate the flat parameter vector on `device` and register the 13 parameters as views of it
        (from per-parameter `init` tensors, or from an already flat host `theta`).  init[k] None: the
        packed pair parameters, drawn on the device (0.1 N(0,1), generator seeded by `seed`)."""
        self.dtype_ = dtype
        self.device_ = device
        self.packed = bool(packed)
        self.Z = Zt.to(self.device_)
        self.M = int(Zt.shape[0])
        self.N = N
        self.D = D
        self.batch_size = batch_size
        self.noise = noise
        self.sigma2_g = 1
        M = self.M
        self._offs, n = param_layout(D, M, packed=self.packed)
        if theta is not None:
            assert theta.numel() == n
            self._theta = theta.to(device=self.device_, dtype=dtype).contiguous()
        else:
            self._theta = torch.zeros(n, dtype=dtype, device=self.device_)
        self._grad = torch.zeros(n, dtype=dtype, device=self.device_)
        self._grad_views = []
        for k in PARAM_NAMES:
            o, shp = self._offs[k]
            cnt = int(np.prod(shp)) if shp else 1
            view = self._theta[o:o + cnt].view(shp)
            if init is not None:
                if init[k] is None:
                    gen = torch.Generator(device=self.device_)
                    gen.manual_seed(int(seed) * 1000003 + PARAM_NAMES.index(k))
                    view.copy_(0.1 * torch.randn(shp, generator=gen, device=self.device_, dtype=dtype))
                else:
                    view.copy_(init[k].reshape(shp))
            setattr(self, k, Parameter(view))
            self._grad_views.append(self._grad[o:o + cnt].view(shp))
        self._engines = {}
        self._pending_info = []
        self._batch = None
        self._noise_seed = seed
        self._noise_counter = torch.zeros(1, dtype=torch.int64, device=self.device_)

    def __reduce__(self):
        """Picklable like the reference's NMGP objects (the drivers pickle whole models,
        code/NMGP_PM25.py:101-106): the flat parameter vector travels through the host; engines
        (device workspaces) are rebuilt on first use after loading."""
        state = {"N": self.N, "D": self.D, "Z": self.Z.detach().cpu(), "batch_size": self.batch_size,
                 "noise": self.noise, "dtype": str(self.dtype_).replace("torch.", ""),
                 "device": str(self.device_), "seed": self._noise_seed,
                 "noise_counter": int(self._noise_counter.cpu()[0]), "theta": self._theta.detach().cpu(),
                 "requires_grad": {k: bool(getattr(self, k).requires_grad) for k in PARAM_NAMES},
                 "packed": self.packed}
        return (_rebuild_nmgp, (state,))

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

    def mu_U_dense(self):
        """mu_U in the reference's (D, D, M) layout (zero dead upper pairs in the packed layout)."""
        return _unpack_pairs(self.mu_U.detach(), self.D) if self.packed else self.mu_U.detach()

    def sqrt_U_pair(self, i, j):
        """The (M, M) block of coefficient pair (i, j <= i), in either layout."""
        return self.sqrt_U[i * (i + 1) // 2 + j] if self.packed else self.sqrt_U[i, j]

    def state_dict(self, *args, **kwargs):
        """The reference's 13 keys with its dense shapes (code/nmgp_dsvi.py:117-155, model.pt).

        Packed models export mu_U / sqrt_U as dense HOST tensors, unpacked output by output straight
        from the device vector: the dense sqrt_U is 69 GB in fp32 at the ECoG shape, which must not be
        materialised in HBM next to the model (the other keys stay device views as usual)."""
        sd = super().state_dict(*args, **kwargs)
        if self.packed:
            prefix = kwargs.get("prefix", args[1] if len(args) > 1 else "")
            for k in ("mu_U", "sqrt_U"):
                sd[prefix + k] = _unpack_pairs_host(sd[prefix + k].detach(), self.D)
        return sd

    def load_state_dict(self, state_dict, strict=True, assign=False):
        if self.packed:
            state_dict = dict(state_dict)
            for k in ("mu_U", "sqrt_U"):
                v = state_dict.get(k)
                if v is not None and tuple(v.shape[:2]) == (self.D, self.D):
                    state_dict[k] = _pack_pairs(v, self.D)
        if assign:
            raise ValueError("assign=True would detach the parameters from the flat device vector")
        return super().load_state_dict(state_dict, strict=strict)

    def check_numerics(self, engines=None):
        """Synchronise and raise like the reference would: torch.linalg.LinAlgError when a Cholesky
        factor was not positive-definite (the reference's torch.cholesky raises, code/utils.py:46,
        347-348), HipError when a bounded inter-workgroup spin gave up."""
        Lb.check_device_status()
        for eng in (engines if engines is not None else self._engines.values()):
            eng.check_info()
        pend, self._pending_info = getattr(self, "_pending_info", []), []
        if pend and int(torch.cat(pend).abs().max().cpu()) != 0:   # deferred predict_Y Cholesky checks
            raise torch.linalg.LinAlgError("cholesky: K22 + 1e-4 I is not positive-definite (predict_Y)")

    def engine(self, B, N=None):
        eng = self._engines.get(B)
        if eng is None:
            ws = next(iter(self._engines.values())).factor_workspace() if self._engines else None
            eng = DsviEngine(self.D, self.M, B, self.Z.cpu().numpy().reshape(-1), device=self.device_,
                             dtype=self.dtype_, packed=self.packed, factor_ws=ws)
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
        self.check_numerics([eng])          # a non-PD factor raises here, as torch.cholesky would
        if verbose:
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
        first = True
        # the KL terms: on one process with the last sample; sharded, every rank adds a factor range
        # with its own last sample (KL_W / KL_v on the owner of the global last sample, DD.kl_shares)
        my_last = max([s for s in range(n_sample) if s % world == rank], default=-1)
        kl_part = None
        if world > 1 and n_sample >= world:
            kl_part = DD.kl_shares(eng.nW, eng.Q, world, DD.last_sample_owner(n_sample, world))[rank]
        for s in range(n_sample):
            if verbose:
                print("Monte Carlo index:", s)
            noise = self._torch_noise(B, Q) if self.noise == "torch" else None
            if s % world != rank:                       # another rank's sample: keep the stream in step
                if noise is None:
                    H.counter_add_(self._noise_counter, 1)
                continue
            if first:
                eng.load_batch(x, y, sizes, noise=noise, index=index)
            elif noise is not None:
                eng.load_noise(noise)               # regrouped like the rows of the first load_batch
            if noise is None:
                eng.device_noise(self._noise_seed, self._noise_counter)
                H.counter_add_(self._noise_counter, 1)
            # the first sample of this rank computes everything; later ones reuse the sample-independent
            # RBF-prior factors and pair quadratic forms (engine.elbo_sample(cached=True))
            with_kl = (s == my_last) if kl_part is not None else (s == n_sample - 1)
            out = eng.elbo_sample(with_kl=with_kl, cached=not first, kl_part=kl_part if with_kl else None)
            first = False
            acc += out[1]
            if with_kl:
                kl = out[2] + out[3] + out[4]
        if out is not None:
            self.check_numerics([eng])
        if world == 1:
            return (acc / n_sample - out[2] - out[3] - out[4]).detach().clone()
        return DD.combine_elbo(acc, kl, n_sample, group=group, device=self.device_).detach().clone()

    def predict_Y(self, inputs_list, index=None):
        """code/nmgp_dsvi.py:666-722: posterior-mean prediction (returns a tensor)."""
        from . import predict
        return predict.predict_mean(self, inputs_list, index)


def _pack_pairs(dense, D):
    """(D, D, ...) -> (Q, ...): the live pairs (i, j <= i) in (i, j) order."""
    ii, jj = np.tril_indices(D)
    return dense[torch.from_numpy(ii), torch.from_numpy(jj)].contiguous()


def _unpack_pairs(packed, D):
    """(Q, ...) -> (D, D, ...) with zero dead (upper) pairs."""
    out = torch.zeros((D, D) + tuple(packed.shape[1:]), dtype=packed.dtype, device=packed.device)
    ii, jj = np.tril_indices(D)
    out[torch.from_numpy(ii).to(packed.device), torch.from_numpy(jj).to(packed.device)] = packed
    return out


def _unpack_pairs_host(packed, D):
    """(Q, ...) device tensor -> (D, D, ...) host tensor with zero dead (upper) pairs, copied one output
    row at a time (the pairs (i, 0..i) are contiguous in the packed layout), so no dense or temporary
    copy is ever allocated on the device."""
    out = torch.zeros((D, D) + tuple(packed.shape[1:]), dtype=packed.dtype)
    for i in range(D):
        q0 = i * (i + 1) // 2
        out[i, :i + 1].copy_(packed[q0:q0 + i + 1])
    return out


def _rebuild_nmgp(state):
    """Unpickle an NMGP (see NMGP.__reduce__) onto its saved device, or the current one."""
    dev = torch.device(state["device"])
    if dev.type != "cuda":
        dev = _default_device()
    elif not torch.cuda.is_available():
        raise RuntimeError("unpickling an NMGP needs a HIP device; there is no CPU fallback")
    m = NMGP.__new__(NMGP)
    torch.nn.Module.__init__(m)
    m._setup(state["N"], state["D"], state["Z"], state["batch_size"], state["noise"],
             getattr(torch, state["dtype"]), dev, state["seed"], theta=state["theta"],
             packed=state.get("packed", False))
    for k, rg in state["requires_grad"].items():
        getattr(m, k).requires_grad = rg
    m._noise_counter.fill_(int(state["noise_counter"]))
    return m


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
        model.load_state_dict(ck["model_state_dict"])
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
        """Adopt a torch.optim.Adam state_dict (model.pt, code/nmgp_dsvi.py:792) for the flat vector,
        as Optimizer.load_state_dict does: the checkpoint's lr / betas / eps replace the constructor's;
        per-parameter exp_avg / exp_avg_sq are restored.  The flat-vector Adam keeps ONE step counter,
        so states whose parameters were stepped a different number of times (or a mix of stepped and
        never-stepped trainable parameters) are rejected rather than bias-corrected wrongly.  Frozen
        parameters (requires_grad False) keep zero moments: torch skips them (grad None), and a
        nonzero exp_avg would otherwise keep moving them."""
        groups = sd.get("param_groups") or []
        if groups:
            g0 = groups[0]
            self.lr = float(g0.get("lr", self.lr))
            self.betas = tuple(float(b) for b in g0.get("betas", self.betas))
            self.eps = float(g0.get("eps", self.eps))
        state = sd.get("state", {})
        if not state:
            return
        m = self.model
        # saved parameter ids in registration order: 0..12 (current torch) or the object ids an older
        # torch wrote (code/notebook/model.pt); Optimizer.load_state_dict maps them by position
        ids = list(groups[0]["params"]) if groups and "params" in groups[0] else list(range(len(PARAM_NAMES)))
        if len(ids) != len(PARAM_NAMES):
            raise ValueError(f"optimizer state lists {len(ids)} parameters, NMGP has {len(PARAM_NAMES)}")
        steps, missing = set(), []
        for idx, name in enumerate(PARAM_NAMES):
            pid = ids[idx]
            st = state.get(pid, state.get(str(pid)))
            trainable = getattr(m, name).requires_grad
            o, shp = m._offs[name]
            n = int(np.prod(shp)) if shp else 1
            if st is None:
                if trainable:
                    missing.append(name)
                continue
            if not trainable:
                continue
            ea, eq = st["exp_avg"], st["exp_avg_sq"]
            if m.packed and name in ("mu_U", "sqrt_U") and tuple(ea.shape[:2]) == (m.D, m.D):
                ea, eq = _pack_pairs(ea, m.D), _pack_pairs(eq, m.D)
            self.m[o:o + n] = ea.reshape(-1).to(self.m.dtype)
            self.v[o:o + n] = eq.reshape(-1).to(self.v.dtype)
            steps.add(int(float(st["step"])))
        if len(steps) > 1 or (steps and missing):
            raise NotImplementedError(
                f"optimizer state with per-parameter step counts {sorted(steps)} (never stepped: {missing}); "
                "the flat-vector Adam keeps one shared step counter")
        if steps:
            self.step_count.fill_(steps.pop())

    def grad_step(self, eng, noise=None, timer=None):
        """[Minibatch gather if a dataset is bound] + noise (device Philox unless host noise was
        loaded) + fused forward/backward."""
        mdl = self.model
        if getattr(eng, "_dataset", None) is not None and noise is None and timer is None:
            # one launch: gather + Philox noise + counter advance + gradient zeroing
            eng.begin_forward_backward(mdl._noise_seed, mdl._noise_counter)
            return eng.out[0]
        if getattr(eng, "_dataset", None) is not None:
            eng.gather_batch()
        if noise is None:
            eng.device_noise(mdl._noise_seed, mdl._noise_counter)
            H.counter_add_(mdl._noise_counter, 1)
        eng.forward_backward(timer=timer)
        return eng.out[0]

    def dp_grad_step(self, eng, group=None, noise=None):
        """Data-parallel gradient of one step with the all-reduce bucketed and overlapped with the
        backward (eager launches; SURVEY §8e axis 2).  Bucket 1 -- the sqrt_U and sqrt_W gradient
        rows, >99% of the bytes at HCP / ECoG shapes -- is final once the side stream's L-bar products
        are done ("lbar_done"): its all-reduce starts then, on a communication stream, while the main
        stream runs the rest of the backward (R / prior adjoints / t chain / v chain / finalize).  The
        small remainder (mu rows, sqrt_v, hyper-parameters) is reduced after the step.  The element-wise
        sums are those of one all-reduce of the whole vector, so results are identical."""
        mdl = self.model
        rank, world = DD.world_info(group)
        g = mdl._grad
        big, small = DD.grad_buckets(mdl._offs, g)
        comm = self._comm_stream()
        works = []

        def start(ev):
            with torch.cuda.stream(comm):
                comm.wait_event(ev)
                works.extend(DD.bucketed_allreduce_sum_(big, group))
        eng.hooks = {"lbar_done": start}
        try:
            loss = self.grad_step(eng, noise=noise)
        finally:
            eng.hooks = {}
        works.extend(DD.bucketed_allreduce_sum_(small, group))
        for w in works:
            w.wait()
        g.div_(world)
        return loss

    def _comm_stream(self):
        if getattr(self, "_comm", None) is None:
            self._comm = torch.cuda.Stream(device=self.model.device_)
        return self._comm

    # "auto" on the graph path = flat (round 6): the bucketed, overlapped all-reduce has one measurement, gloo ranks
    # sharing one GPU (profiles/r05n_*: 296 ms/step bucketed vs 8.0 flat at N = 2), where gloo stages every bucket
    # through the host; RCCL over xGMI has not run with N > 1 on this project's hardware, so nothing justifies a size
    # threshold yet.  Set DP_BUCKET_MIN_BYTES (bytes of gradient) to make "auto" pick the bucketed form from that size
    # on once a multi-GPU run measures it; "bucketed" forces it.
    DP_BUCKET_MIN_BYTES = None

    def dp_bucketed(self, mode="auto"):
        if mode not in ("auto", "bucketed", "flat"):
            raise ValueError(f"dp all-reduce mode {mode!r}")
        g = self.model._grad
        thr = self.DP_BUCKET_MIN_BYTES
        return mode == "bucketed" or (mode == "auto" and thr is not None and g.numel() * g.element_size() >= thr)

    def capture_dp(self, eng, world, mode="auto"):
        """The data-parallel step as two graphs around the gradient all-reduce (dp_graph_step): the gradient graph
        of `eng` and the update graph (1/world + Adam).  Bucketed (mode "bucketed", or "auto" from 64 MB of
        gradient): the gradient graph carries an EXTERNAL event node at "lbar_done" (hip_ops.ExtEvent: the point
        after which the sqrt_W / sqrt_U gradient rows are final) for the overlapped all-reduce; "flat": one
        all-reduce of the whole vector after the graph."""
        bucketed = self.dp_bucketed(mode)
        if bucketed and "lbar_done" not in getattr(eng, "ext_events", {}):
            eng.ext_events = {"lbar_done": H.ExtEvent()}
        g = self.capture(eng, include_update=False)
        if not hasattr(self, "_dp_graphs"):
            self._dp_graphs = {}
        self._dp_graphs[self._dp_key(eng)] = (g, eng.ext_events["lbar_done"] if bucketed else None,
                                              self.capture_update(world))
        return self._dp_graphs[self._dp_key(eng)]

    @staticmethod
    def _dp_key(eng):
        # the captured graph holds the bound dataset's buffer pointers: a rebind (the device pipeline's slot
        # rebuilt after the number of minibatches changed) must recapture, not replay freed buffers
        ds = getattr(eng, "_dataset", None)
        return (id(eng),) + (tuple(t.data_ptr() for t in ds) if ds is not None else ())

    def dp_graph_step(self, eng, group=None, graphs=None):
        """One data-parallel step on the graph path (SURVEY §8e axis 2; the reference's loss.backward();
        optimizer.step(), code/nmgp_dsvi.py:847-854, with the gradient average between them).  Bucketed:
          main:  replay the gradient graph ........................ | wait comm | replay 1/world + Adam
          comm:  wait for the graph's lbar_done node -> all-reduce(sqrt_W, sqrt_U rows)
                 wait for the graph's end -> all-reduce(the small remainder)
        The sqrt rows' all-reduce runs while the graph's remaining backward (R, prior adjoints, t and v chains,
        finalize: none of them touches those rows) still runs.  Flat: replay, one all-reduce, replay.  Sums are
        element-wise those of one flat all-reduce (bit-identical at two ranks)."""
        mdl = self.model
        rank, world = DD.world_info(group)
        dpg = graphs if graphs is not None else getattr(self, "_dp_graphs", {}).get(self._dp_key(eng))
        g, ev, upd = dpg if dpg is not None else self.capture_dp(eng, world)
        if ev is None:
            g.replay()
            DD.allreduce_sum_(mdl._grad, group)
            upd.replay()
            return
        main = torch.cuda.current_stream(mdl.device_)
        comm = self._comm_stream()
        big, small = DD.grad_buckets(mdl._offs, mdl._grad)
        g.replay()
        ev.wait(comm)                     # the graph's external lbar_done node (recorded at its launch)
        with torch.cuda.stream(comm):
            works = DD.bucketed_allreduce_sum_(big, group)
            comm.wait_stream(main)        # the end of the gradient graph
            works += DD.bucketed_allreduce_sum_(small, group)
        for w in works:
            w.wait()                      # (nccl: the current stream waits for the collective)
        main.wait_stream(comm)
        upd.replay()

    def update(self):
        """torch.optim.Adam update of the flat parameter vector (one HIP launch; from M = 512 on the sqrt blocks'
        lower triangles only, nmgp_adam_lower: their upper triangles never move)."""
        mdl = self.model
        if use_adam_lower(mdl.M, mdl._theta.dtype, mdl._offs):
            H.adam_lower_(mdl._theta, mdl._grad, self.m, self.v, self.step_count, self.lr,
                          lower_block_ranges(mdl._offs), mdl.M, self.betas, self.eps)
        else:
            H.adam_(mdl._theta, mdl._grad, self.m, self.v, self.step_count, self.lr, self.betas, self.eps)

    # round 6: in the captured single-process step the finalize kernel advances the step counter and the update reads
    # it (nmgp_adam_lower_advanced_*): one launch fewer at the step's tail; NMGP_FOLD_STEP=0 keeps the counter launch
    FOLD_STEP = os.environ.get("NMGP_FOLD_STEP", "1") != "0"

    def step(self, eng, noise=None):
        """One DSVI iteration on the batch already loaded in `eng`; returns the device loss scalar."""
        loss = self.grad_step(eng, noise)
        self.update()
        return loss

    def capture(self, eng, include_update=True):
        """Capture [gather +] noise -> forward -> backward (-> Adam) of `eng` into one HIP graph.

        The warm-up runs (lazy attributes, descriptor uploads) happen outside the capture and
        without the Adam update; the noise counter and the bound dataset's batch counter they
        advance are restored afterwards, so capturing leaves parameters, optimizer state and the
        random stream exactly as they were (the first replay is the first real step)."""
        mdl = self.model
        body = self.step if include_update else self.grad_step
        cur = torch.cuda.current_stream(mdl.device_)
        saved = [(mdl._noise_counter, mdl._noise_counter.clone())]
        ds = getattr(eng, "_dataset", None)
        if ds is not None:
            saved.append((ds[4], ds[4].clone()))
        s = torch.cuda.Stream(device=mdl.device_)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            for _ in range(2):
                self.grad_step(eng)
        cur.wait_stream(s)
        for t, v in saved:
            t.copy_(v)
        g = H.HipGraph(mdl.device_)          # captured through the HIP runtime (nmgp_graph_*), not torch
        fold = (include_update and self.FOLD_STEP and getattr(eng, "_dataset", None) is not None
                and use_adam_lower(mdl.M, mdl._theta.dtype, mdl._offs) and len(lower_block_ranges(mdl._offs)) <= 4)
        with g.capture():
            if fold:
                eng.set_adam_step(self.step_count)
                try:
                    self.grad_step(eng)
                finally:
                    eng.set_adam_step(None)      # eager steps keep the counter launch of update()
                H.adam_lower_advanced_(mdl._theta, mdl._grad, self.m, self.v, self.step_count, self.lr,
                                       lower_block_ranges(mdl._offs), mdl.M, self.betas, self.eps)
            else:
                body(eng)
        self.graphs[id(eng)] = g
        return g

    def capture_update(self, world=1):
        """The Adam update alone as a HIP graph: the data-parallel step replays the gradient graph, runs ONE
        sum all-reduce of the flat gradient, then replays this -- the 1/world scaling of the summed gradient
        and Adam (code/nmgp_dsvi.py:847-854's backward -> optimizer.step with the collective between them) --
        so no optimizer launch is issued eagerly."""
        key = ("update", int(world))
        g = self.graphs.get(key)
        if g is None:
            g = H.HipGraph(self.model.device_)
            with g.capture():
                if world > 1:
                    self.model._grad.div_(world)
                self.update()
            self.graphs[key] = g
        return g


class _IndexData(Dataset):
    """Row indices 0..n-1.  A DataLoader over it with the same length, batch size, shuffle flag and
    generator draws exactly the permutation the reference's DataLoader(trainData(X, Y, I)) draws
    (code/nmgp_dsvi.py:816-817): the sampler only sees len(dataset).  __getitems__ hands the whole
    index list to collate in one call instead of collating B scalar rows."""

    def __init__(self, n):
        self.n = int(n)

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return i

    def __getitems__(self, idx):
        return idx


def _index_batch(idx):
    return torch.as_tensor(idx, dtype=torch.long)


def _index_loader(n, batch_size, generator=None):
    return DataLoader(_IndexData(n), batch_size=batch_size, shuffle=True, generator=generator,
                      collate_fn=_index_batch)


class _DevicePipeline:
    """the training loop's input pipeline on the device (noise="device").

    The training set stays in HBM.  Per epoch the host draws the DataLoader's index permutation
    (same draws as the reference's loader); the minibatches are gathered, grouped by output in
    vec2list order (a stable sort on the output id) and segment-tabled on the device, written into
    the buffers bound to the engine (`DsviEngine.bind_dataset`), and each step then starts with ONE
    `nmgp_step_begin` launch (gather + Philox noise + counter advance + gradient zeroing).  With a
    graph the whole step is one replay; there is no host synchronisation per step -- losses stay on
    the device and the per-step wall clock comes from HIP events.  A ragged last minibatch gets its
    own engine (its own B) and buffers."""

    def __init__(self, model, trainer, X, Y, I, batch_size, rank, world, use_graph, include_update):
        self.model, self.trainer = model, trainer
        dev = model.device_
        self.dt = model.dtype_
        self.D = model.D
        self.X = X.to(dev, self.dt)
        self.Y = Y.to(dev, self.dt)
        self.I = I.to(dev).long()
        self.bs, self.rank, self.world = batch_size, rank, world
        self.use_graph, self.include_update = use_graph, include_update
        self.slots = {}           # B -> dict(eng, bufs, counter, graph)
        self.ar = torch.arange(self.D + 1, device=dev)

    def _slot(self, B, nb):
        sl = self.slots.get(B)
        if sl is not None and sl["nb"] == nb:
            return sl
        dev = self.model.device_
        eng = self.model.engine(B)
        bufs = (torch.empty(nb, B, dtype=self.dt, device=dev), torch.empty(nb, B, dtype=self.dt, device=dev),
                torch.empty(nb, B, dtype=torch.int32, device=dev), torch.empty(nb, self.D + 1, dtype=torch.int32,
                                                                                device=dev))
        ctr = eng.bind_dataset(*bufs)
        sl = {"eng": eng, "bufs": bufs, "ctr": ctr, "graph": None, "dp": None, "nb": nb}
        self.slots[B] = sl
        return sl

    def _fill(self, sl, idx):
        """idx (nb, B) row indices on the device -> output-grouped batches in the bound buffers."""
        Ib = self.I[idx]
        order = torch.sort(Ib, dim=1, stable=True).indices
        idx = idx.gather(1, order)
        Ib = Ib.gather(1, order)
        Xb, Yb, Ibuf, Sb = sl["bufs"]
        Xb.copy_(self.X[idx])
        Yb.copy_(self.Y[idx])
        Ibuf.copy_(Ib)
        Sb.copy_(torch.searchsorted(Ib, self.ar.expand(Ib.shape[0], -1).contiguous()))
        sl["ctr"].zero_()

    def epoch(self, index_batches):
        """Upload one epoch; returns the ordered list of (slot) to step, one entry per minibatch."""
        dev = self.model.device_
        rows = []
        for b in index_batches:
            if self.world > 1:
                if b.numel() < self.world:       # every rank skips the same short global batch
                    continue
                b = b[DD.rank_slice(b.numel(), self.rank, self.world)]
            rows.append(b)
        plan, groups = [], {}
        for b in rows:
            groups.setdefault(b.numel(), []).append(b)
        for B, bl in groups.items():
            sl = self._slot(B, len(bl))
            # pinned, so the upload is a stream-ordered async copy: from pageable memory it waited for the
            # previous epoch's queued steps, which drained the GPU once per epoch while the host drew the next
            # permutation (inference(noise="device") ran 16% below the bench loop)
            self._fill(sl, torch.stack(bl).pin_memory().to(dev, non_blocking=True))
        for b in rows:
            plan.append(self.slots[b.numel()])
        return plan

    def step(self, sl, group=None):
        tr = self.trainer
        if self.use_graph and self.world > 1:
            # data parallel on the graph path: gradient graph, all-reduce (flat by default; bucketed and overlapped
            # with the graph's tail from its lbar_done node when DsviTrainer.dp_bucketed says so), update graph
            if sl.get("dp") is None:          # kept in the slot: a rebound slot starts without graphs
                sl["dp"] = tr.capture_dp(sl["eng"], self.world)
            tr.dp_graph_step(sl["eng"], group, graphs=sl["dp"])
        elif self.use_graph:
            if sl["graph"] is None:
                sl["graph"] = tr.capture(sl["eng"], include_update=self.include_update)
            sl["graph"].replay()
        elif self.include_update:
            tr.step(sl["eng"])
        else:
            tr.grad_step(sl["eng"])
        return sl["eng"]


def inference(X_train_list, Y_train_list, z, batch_size, dim_outputs, hyperpars=None, fix_hyperpars=True,
              mu_v=None, mu_W=None, mu_U=None, sqrt_v=None, sqrt_W=None, sqrt_U=None, lr=0.01, itnum=1000,
              do_stop_criterion=False, seed=22, verbose=False, PATH="model.pt", continuous_training=False,
              show_ELBO=True, save_model=False, X_test_list=None, Y_test_list=None, device=None, noise="torch",
              use_graph=None, n_elbo_sample=1000, distributed=False, group=None, dtype=F64, check_every=64):
    """code/nmgp_dsvi.py:758-909 on the MI355X.

    Returns (model, loss_list, time_list), or (model, loss_list, rmse_test_list, time_list) when
    X_test_list is given -- as the reference.  Extra keyword-only knobs (defaults keep reference
    behaviour): device, noise ("torch" = the reference RNG stream, replayable sample for sample |
    "device" = on-device Philox and the on-device input pipeline of SURVEY f4), use_graph (replay
    each step as one HIP graph; default: on for noise="device", impossible for "torch"),
    n_elbo_sample (compute_ELBO samples), distributed (data-parallel over the ranks of `group`:
    every rank draws the same global minibatch of batch_size * world rows from an identically
    seeded DataLoader generator, trains on its contiguous slice, and the gradients are averaged
    with one all-reduce before the replicated Adam step; global batches with fewer rows than
    ranks are skipped on every rank; the reported loss is the rank mean; compute_ELBO shards its
    samples), check_every (noise="device": steps between the host checks of the Cholesky info /
    device status -- the only synchronisations of the loop besides verbose / test / ELBO output).
    A non-positive-definite factor raises torch.linalg.LinAlgError, as the reference's
    torch.cholesky does.
    """
    rank, world = DD.world_info(group) if distributed else (0, 1)
    if use_graph is None:
        # device noise: one graph per step; data parallel on the graph path: gradient graph, one all-reduce,
        # 1/world + Adam graph (DsviTrainer.dp_graph_step; the bucketed form on request, DP_BUCKET_MIN_BYTES)
        use_graph = noise == "device"
    if use_graph and noise != "device":
        raise ValueError("use_graph=True needs noise='device' (host RNG cannot be replayed)")
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
    # data parallel: the loader's permutation must be identical on every rank and independent of
    # the per-rank torch.randn draws (noise="torch" draws B_r-sized vectors from the global stream)
    gen = None
    if world > 1:
        gen = torch.Generator()
        gen.manual_seed(int(seed) + 0x5eed)
    N_train = X_train_vec.shape[0]
    if X_test_list is not None:
        # per-iteration predict_Y (code/nmgp_dsvi.py:865-868) on the device: test inputs uploaded once, the
        # RMSE kept on the device (the reference's broadcast est[:, None] - Y_test_vec included) and read
        # back after the loop, the predictions' Cholesky checks deferred to the loop's check points
        from . import predict as _pred
        rmse_dev = []
        Y_test_vec = np.concatenate(Y_test_list)
        test_prep = _pred.prepare_inputs(model, [np.asarray(x, np.float64) for x in X_test_list])
        Y_test_dev = torch.as_tensor(np.asarray(Y_test_vec, np.float64)).to(model.device_)
        # one prediction plan for the whole run (buffers, descriptors; with the device pipeline a HIP graph
        # replayed after every iteration), its Cholesky info words checked at the loop's check points
        test_plan = _pred.PredictPlan(model, test_prep, graph=(noise == "device"))
        model._pending_info.append(test_plan.info_acc)

        def _test_rmse():
            est = test_plan()
            if not any(t is test_plan.info_acc for t in model._pending_info):
                model._pending_info.append(test_plan.info_acc)
            rmse_dev.append(torch.sqrt(torch.mean((est[:, None] - Y_test_dev) ** 2)))
    Q = dim_outputs * (dim_outputs + 1) // 2
    pipe = None
    if noise == "device":
        pipe = _DevicePipeline(model, trainer, X.reshape(-1), Y.reshape(-1), I.reshape(-1), batch_size, rank, world,
                               use_graph, include_update=(world == 1))
        loader = _index_loader(N_train, batch_size * world, gen)
    else:
        # the reference's DataLoader(trainData(X, Y, I)) draws: same sampler, same global-RNG consumption
        # (tests/test_host_logic.py), rows gathered by index instead of B per-row fetches + collate
        loader = _index_loader(N_train, batch_size * world, gen)
    loss_list, time_list = [], []
    losses_dev = []
    events = []
    ts = time.time()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev0.record()
    epoch = 0
    nstep = 0

    def _sync_check():
        torch.cuda.synchronize(model.device_)
        model.check_numerics()

    for epoch in range(itnum):
        batch = 0
        if pipe is not None:
            for sl in pipe.epoch(list(loader)):
                batch += 1
                if world > 1 and not use_graph:
                    eng = sl["eng"]
                    trainer.dp_grad_step(eng, group)        # bucketed all-reduce overlapped with the backward
                    trainer.update()
                else:
                    # (world > 1: DsviTrainer.dp_graph_step -- gradient graph, all-reduce, 1/world + Adam graph)
                    eng = pipe.step(sl, group)
                losses_dev.append(eng.out[0].clone())
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                events.append(ev)
                nstep += 1
                if check_every and nstep % check_every == 0:
                    _sync_check()
                if X_test_list is not None:
                    _test_rmse()
                if verbose:
                    print("epoch: {}/{}, batch: {}/{}, loss: {}".format(epoch, itnum, batch, N_train / batch_size,
                                                                       float(losses_dev[-1])))
        else:
            for idx in loader:
                X_batch, Y_batch, I_batch = X[idx], Y[idx], I[idx]
                if world > 1:                               # this rank's slice of the global minibatch
                    if X_batch.shape[0] < world:            # every rank skips the same short global batch
                        continue
                    sl = DD.rank_slice(X_batch.shape[0], rank, world)
                    X_batch, Y_batch, I_batch = X_batch[sl], Y_batch[sl], I_batch[sl]
                batch += 1
                X_bl, Y_bl = vec2list(X_batch, Y_batch, I_batch, dim=dim_outputs)
                model._assert_views()
                x, y, sizes = model._prepare(X_bl, Y_bl)
                B = sum(sizes)
                eng = model.engine(B)
                nz = model._torch_noise(B, Q)
                eng.load_batch(x, y, sizes, noise=nz)
                if world == 1:
                    loss = trainer.step(eng, noise=nz)
                else:
                    loss = trainer.dp_grad_step(eng, group, noise=nz)
                    trainer.update()
                losses_dev.append(loss.clone())
                torch.cuda.synchronize(model.device_)
                eng.check_info()
                time_list.append(time.time() - ts)
                nstep += 1
                if X_test_list is not None:
                    _test_rmse()
                if verbose:
                    print("epoch: {}/{}, batch: {}/{}, loss: {}".format(epoch, itnum, batch, N_train / batch_size,
                                                                       float(loss)))
        if do_stop_criterion and epoch % 5 == 4 and epoch > 5:
            # (data parallel: decided on the rank-mean losses, so every rank stops at the same epoch)
            recent = torch.stack([l.reshape(()) for l in losses_dev[-batch * 6:]]).to(torch.float64)
            if world > 1:
                DD.allreduce_mean_(recent, group)
            la = recent.cpu().numpy()
            if la[-batch:].sum() > la[-batch * 6:-batch * 5].sum():
                print("Stop criteria is satisfied.")
                break
        if epoch % 100 == 99 and show_ELBO:
            elbo = model.compute_ELBO(X_list, Y_list, n_sample=n_elbo_sample, distributed=distributed, group=group)
            print("epoch: {}, ELBO: {}".format(epoch + 1, float(elbo)))
            print(print_mem(epoch + 1))
    _sync_check()
    if events:
        time_list = [ev0.elapsed_time(e) / 1e3 for e in events]     # device completion of each step
    print("training takes {}s".format(time.time() - ts))
    if losses_dev:
        lv = torch.stack([l.reshape(()) for l in losses_dev]).to(torch.float64)
        if world > 1:
            DD.allreduce_mean_(lv, group)        # the rank mean of every step's loss, one collective
        loss_list = [np.array(v) for v in lv.cpu().numpy()]
    if save_model:
        torch.save({"epoch": epoch, "model_state_dict": {k: v.detach().cpu() for k, v in model.state_dict().items()},
                    "optimizer_state_dict": _adam_state_dict(model, trainer),
                    "loss": torch.tensor(float(loss_list[-1]) if loss_list else float("nan"))}, PATH)
    if show_ELBO:
        elbo = model.compute_ELBO(X_list, Y_list, n_sample=n_elbo_sample, distributed=distributed, group=group)
        print("epoch: {}, ELBO: {}".format(epoch + 1, float(elbo)))
        print(print_mem(epoch + 1))
    if X_test_list is not None:
        rmse_test_list = [np.float64(v) for v in torch.stack(rmse_dev).cpu().numpy()] if rmse_dev else []
        return model, loss_list, rmse_test_list, time_list
    return model, loss_list, time_list


def _adam_state_dict(model, trainer):
    """torch.optim.Adam.state_dict() layout for the flat-vector optimizer (code/nmgp_dsvi.py:897)."""
    state = {}
    step = float(trainer.step_count.cpu())
    for idx, name in enumerate(PARAM_NAMES):
        if not getattr(model, name).requires_grad:
            continue
        o, shp = model._offs[name]
        n = int(np.prod(shp)) if shp else 1
        ea, eq = trainer.m[o:o + n].reshape(shp), trainer.v[o:o + n].reshape(shp)
        if model.packed and name in ("mu_U", "sqrt_U"):      # the reference's dense shapes, built on the host
            ea, eq = _unpack_pairs_host(ea, model.D), _unpack_pairs_host(eq, model.D)
        state[idx] = {"step": torch.tensor(step), "exp_avg": ea.cpu(), "exp_avg_sq": eq.cpu()}
    return {"state": state, "param_groups": [{"lr": trainer.lr, "betas": tuple(trainer.betas), "eps": trainer.eps,
                                              "weight_decay": 0,
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
