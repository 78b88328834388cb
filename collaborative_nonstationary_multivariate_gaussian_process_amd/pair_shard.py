"""Pair sharding of the coefficient GPs across ranks (SURVEY.md §8e axis 3; HCP / ECoG shapes).

The reference keeps every coefficient pair (i, j <= i) of the D x D LMC matrix in one process:
mu_U (D, D, M), sqrt_U (D, D, M, M), the Q Cholesky factors of Sigma_U and their KL terms
(code/nmgp_dsvi.py:136-155, 227-237, 281-295).  At the ECoG shape (D = 128, M = 1024, Q = 8256)
those are 35 GB of parameters per copy (fp32, packed) and ~95% of a training step's flops.

Here rank r owns a contiguous range of OUTPUTS [i0, i1) and with it

* the pairs (i, j <= i) of those outputs (a contiguous window of the packed pair layout): their
  mu_U / sqrt_U rows, Adam moments, Sigma_U factorizations and KL_U terms -- never communicated;
* the observations of those outputs: row n of output i reads only the pairs (i, j), j <= i
  (code/nmgp_dsvi.py:238, the row gather of the training step), so a rank's rows need no pair it
  does not own.

Everything else -- mu_W / sqrt_W (every output's rows read all latent functions j <= i), mu_v /
sqrt_v (the shared length-scale process) and the 7 hyper-parameters -- is replicated; its gradient
is the SUM over ranks of the per-rank gradients (one all-reduce per step, two buffers), so every rank
applies the same Adam update.  KL_W and KL_v are added by rank 0 only (kl_owner), KL_U by the owner
of each pair, so the summed loss is the whole model's -SELBO.  z_v is drawn from a seed shared by all
ranks (every rank samples the same v, hence the same Gibbs prior); the row and pair noise from
rank-distinct streams.

Minibatches are stratified by output: rank r draws b_r = round(b * N_r / N) of its N_r rows and
scales its reconstruction term by N_r / b_r.  With the full batch (b = N) this is exactly the
reference's objective; with minibatches it is an unbiased estimator of the same ELBO whose
row sampling is stratified by output instead of uniform over all rows (documented deviation).

Not sharded this way: compute_ELBO (its column gather reads pairs (s, o) of every s >= o,
code/nmgp_dsvi.py:361) -- it shards over Monte-Carlo samples (distributed.py).
"""
import numpy as np
import torch

from . import distributed as DD
from . import hip_ops as H
from .engine import (DsviEngine, lower_block_ranges, use_adam_lower, param_layout, pair_window, PARAM_NAMES,
                     HYPER_NAMES)


def pair_shard_ranges(D, world):
    """Contiguous output ranges [(i0, i1)] for `world` ranks minimising the largest factor count: output i
    brings i + 1 pair factors, rank 0 additionally the D + 1 W / v factors whose KL it owns.  Binary search
    on the per-rank capacity with a greedy fill (every rank keeps at least one output).  At D = 128 over 8
    ranks the largest share is 1075 factors (the mean is 1048); the earlier split at the cumulative-target
    points left one rank 1156 and was measured 65 ms per step against ~52 ms for the lightest."""
    if world > D:
        raise ValueError(f"pair sharding needs at least one output per rank (D={D}, world={world})")
    cost = np.arange(1, D + 1, dtype=np.int64)
    pre = np.concatenate([[0], np.cumsum(cost)])

    def fill(cap):
        bounds, i = [0], 0
        for r in range(world):
            extra = D + 1 if r == 0 else 0
            j = i + 1                                   # at least one output
            last = D - (world - r - 1)                  # leave one for each later rank
            while j < last and pre[j + 1] - pre[i] + extra <= cap:
                j += 1
            if r == world - 1:
                j = D
            bounds.append(j)
            i = j
        loads = [pre[bounds[r + 1]] - pre[bounds[r]] + (D + 1 if r == 0 else 0) for r in range(world)]
        return bounds, max(loads)

    lo, hi = int(pre[-1] + D + 1) // world, int(pre[-1] + D + 1)
    while lo < hi:
        mid = (lo + hi) // 2
        if fill(mid)[1] <= mid:
            hi = mid
        else:
            lo = mid + 1
    bounds = fill(lo)[0]
    return [(int(bounds[r]), int(bounds[r + 1])) for r in range(world)]


def _pack(t, D):
    """(D, D, ...) dense pair blocks -> (Q, ...) packed in (i, j <= i) order."""
    idx = [i * D + j for i in range(D) for j in range(i + 1)]
    return t.reshape(D * D, *t.shape[2:])[idx]


class PairShard:
    """One rank's share of a pair-sharded DSVI model: local parameter vector (replicated W / v /
    hyper-parameters + the owned pairs), its engine, Adam state and the per-step all-reduce.

    params: the 13 parameters (dense reference shapes, or packed mu_U (Q, M) / sqrt_U (Q, M, M)); each
    rank takes its window.  B_r: this rank's minibatch rows.  N_r: its number of observations (the
    reconstruction scale is N_r / B_r)."""

    def __init__(self, params, z, B_r, N_r, rank=None, world=None, group=None, dtype=torch.float32,
                 device="cuda", lr=0.01, betas=(0.9, 0.999), eps=1e-8, frozen=(), seed=22, ranges=None,
                 pairs_local=False):
        """pairs_local: params' mu_U / sqrt_U already hold only this rank's pair window (Q_r, ...)."""
        r_, w_ = DD.world_info(group)
        self.rank = r_ if rank is None else int(rank)
        self.world = w_ if world is None else int(world)
        self.group = group
        D, M = params["mu_W"].shape
        self.D, self.M = int(D), int(M)
        self.ranges = ranges if ranges is not None else pair_shard_ranges(self.D, self.world)
        self.pair_range = tuple(self.ranges[self.rank])
        self.q0, self.Q = pair_window(self.D, self.pair_range)
        self.kl_owner = self.rank == 0
        self.dt, self.dev = dtype, torch.device(device)
        self.offs, n = param_layout(self.D, self.M, packed=True, pair_range=self.pair_range)
        self.theta = torch.zeros(n, dtype=dtype, device=self.dev)
        self.grad = torch.zeros_like(self.theta)
        for name in PARAM_NAMES:
            o, shp = self.offs[name]
            t = torch.as_tensor(params[name]).detach()
            if name in ("mu_U", "sqrt_U"):
                if pairs_local:
                    assert t.shape[0] == self.Q, (name, tuple(t.shape), self.Q)
                else:
                    if t.dim() == (3 if name == "mu_U" else 4) and t.shape[0] == self.D and t.shape[1] == self.D:
                        t = _pack(t, self.D)
                    t = t[self.q0:self.q0 + self.Q]
            cnt = int(np.prod(shp)) if shp else 1
            self.theta[o:o + cnt] = t.reshape(-1).to(device=self.dev, dtype=dtype)
        self.B, self.N = int(B_r), float(N_r)
        self.engine = DsviEngine(self.D, self.M, self.B, z, device=self.dev, dtype=dtype, packed=True,
                                 pair_range=self.pair_range, kl_owner=self.kl_owner)
        mask = 0
        for k, name in enumerate(HYPER_NAMES):
            if name in frozen:
                mask |= 1 << k
        self.engine.bind(self.theta, self.grad, frozen_mask=mask, N=self.N)
        # replicated slices (summed over ranks): mu_W, sqrt_W, mu_v, sqrt_v | the 7 hyper-parameters
        self._rep = [self.grad[:self.offs["mu_U"][0]], self.grad[self.offs[HYPER_NAMES[0]][0]:]]
        self.m = torch.zeros_like(self.theta)
        self.v = torch.zeros_like(self.theta)
        self.step_count = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.lr, self.betas, self.eps = lr, betas, eps
        self.seed = int(seed)
        self.noise_counter = torch.zeros(1, dtype=torch.int64, device=self.dev)

    # ------------------------------------------------------------------------------------ data
    def load(self, xs, ys, noise=None):
        """This rank's minibatch: xs / ys = lists of row arrays of its outputs i0 .. i1-1 (in order).
        noise: optional injected (M + B_r + Q_r * B_r) vector (z_v | z_t of these rows | the owned pairs'
        rows, reference call order); otherwise device Philox noise is drawn in grad_step."""
        i0, i1 = self.pair_range
        assert len(xs) == len(ys) == i1 - i0, "one row list per owned output"
        sizes = [len(np.asarray(x).reshape(-1)) for x in xs]
        x = np.concatenate([np.asarray(a, np.float64).reshape(-1) for a in xs])
        y = np.concatenate([np.asarray(a, np.float64).reshape(-1) for a in ys])
        self.engine.load_batch(x, y, sizes, noise=noise, index=list(range(i0, i1)))
        self._host_noise = noise is not None

    def bind_rows(self, xs, ys, b_r=None, seed=0):
        """SURVEY f4 for a pair-sharded rank: ALL of this rank's rows (xs / ys: one array per owned output, in
        order) stay resident in HBM, and every epoch is a device permutation cut into minibatches of b_r rows
        (default: the engine's B), each grouped by output as vec2list groups them and given its segment table
        -- bound to the engine (DsviEngine.bind_dataset), so a step starts with ONE on-device gather and the
        whole step replays from a HIP graph (capture()).  The minibatch stratification is the one `load`
        documents: rank r draws its b_r rows from its own N_r.  Returns the number of minibatches per epoch."""
        i0, i1 = self.pair_range
        assert len(xs) == len(ys) == i1 - i0, "one row list per owned output"
        B = self.B if b_r is None else int(b_r)
        assert B == self.B, "the engine's minibatch size is fixed at construction (B_r)"
        dev, dt = self.dev, self.dt
        sizes = [len(np.asarray(x).reshape(-1)) for x in xs]
        cat = lambda a: torch.as_tensor(np.concatenate([np.asarray(v, np.float64).reshape(-1) for v in a]))
        self._rows = (cat(xs).to(dev, dt), cat(ys).to(dev, dt),
                      torch.as_tensor(np.repeat(np.arange(i0, i1), sizes)).to(dev))
        n = int(sum(sizes))
        nb = n // B
        if nb < 1:
            raise ValueError(f"rank {self.rank} holds {n} rows, fewer than one minibatch of {B}")
        self._epoch_gen = torch.Generator(device=dev)
        self._epoch_gen.manual_seed(int(seed) + 7919 * (self.rank + 1))
        self._bufs = (torch.empty(nb, B, dtype=dt, device=dev), torch.empty(nb, B, dtype=dt, device=dev),
                      torch.empty(nb, B, dtype=torch.int32, device=dev),
                      torch.empty(nb, self.D + 1, dtype=torch.int32, device=dev))
        self._bctr = self.engine.bind_dataset(*self._bufs)
        self._ar = torch.arange(self.D + 1, device=dev)
        self._host_noise = False
        self.new_epoch()
        return nb

    def new_epoch(self):
        """Refill the bound minibatches from a fresh device permutation of this rank's rows (no host copy)."""
        X, Y, I = self._rows
        Xb, Yb, Ib, Sb = self._bufs
        nb, B = Xb.shape
        idx = torch.randperm(X.numel(), generator=self._epoch_gen, device=self.dev)[:nb * B].view(nb, B)
        ids = I[idx]
        order = torch.sort(ids, dim=1, stable=True).indices
        idx, ids = idx.gather(1, order), ids.gather(1, order)
        Xb.copy_(X[idx])
        Yb.copy_(Y[idx])
        Ib.copy_(ids)
        Sb.copy_(torch.searchsorted(ids, self._ar.expand(nb, -1).contiguous()))
        self._bctr.zero_()

    def draw_noise(self):
        """z_v from the seed every rank shares (one v sample for the whole model), the row / pair noise
        from a rank-distinct stream; then advance the shared counter."""
        nz, M = self.engine.noise, self.M
        H.normal_(nz[:M], self.seed, counter=self.noise_counter)
        H.normal_(nz[M:], self.seed + 1000003 * (self.rank + 1), counter=self.noise_counter)
        H.counter_add_(self.noise_counter, 1)

    # ------------------------------------------------------------------------------------ step
    def _grad_body(self):
        """The rank-local part of a step: [on-device minibatch gather] + noise + fused forward / backward."""
        if getattr(self.engine, "_dataset", None) is not None:
            self.engine.gather_batch()
        if not getattr(self, "_host_noise", False):
            self.draw_noise()
        self.engine.forward_backward()

    def _reduce(self, loss):
        if self.world > 1:
            import torch.distributed as dist
            for t in self._rep:
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            dist.all_reduce(loss, op=dist.ReduceOp.SUM, group=self.group)

    def grad_step(self, reduce=True):
        """-SELBO of the whole model (summed over ranks) and this rank's gradient: owned pairs exact,
        replicated parameters summed over ranks.  reduce=False: this share's own terms only (the
        caller sums them, e.g. several shares simulated in one process)."""
        self._grad_body()
        loss = self.engine.out[0:1].clone()
        if reduce:
            self._reduce(loss)
        return loss[0]

    def update(self):
        if use_adam_lower(self.engine.M, self.theta.dtype, self.engine.offs):   # lower triangles only (nmgp_adam_lower)
            H.adam_lower_(self.theta, self.grad, self.m, self.v, self.step_count, self.lr,
                          lower_block_ranges(self.engine.offs), self.engine.M, self.betas, self.eps)
        else:
            H.adam_(self.theta, self.grad, self.m, self.v, self.step_count, self.lr, self.betas, self.eps)

    def capture(self):
        """Capture the rank-local step (gather + noise + forward / backward) and the Adam update as two HIP
        graphs (hip_ops.HipGraph); step() then replays them around the replicated-gradient all-reduce.  Needs
        device noise; the warm-up runs outside the capture and restores the noise / batch counters, so the
        first replay is the next real step."""
        if getattr(self, "_host_noise", False):
            raise ValueError("graph capture needs device noise (no host noise loaded)")
        ds = getattr(self.engine, "_dataset", None)
        saved = [(self.noise_counter, self.noise_counter.clone())]
        if ds is not None:
            saved.append((ds[4], ds[4].clone()))
        cur = torch.cuda.current_stream(self.dev)
        st = torch.cuda.Stream(device=self.dev)
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            for _ in range(2):
                self._grad_body()
        cur.wait_stream(st)
        for t, v in saved:
            t.copy_(v)
        g = H.HipGraph(self.dev)
        with g.capture():
            self._grad_body()
        u = H.HipGraph(self.dev)
        with u.capture():
            self.update()
        self._graphs = (g, u)
        return self._graphs

    def step(self):
        """One training step: graph replays when captured (capture()), eager launches otherwise."""
        graphs = getattr(self, "_graphs", None)
        if graphs is None:
            loss = self.grad_step()
            self.update()
            return loss
        graphs[0].replay()
        loss = self.engine.out[0:1].clone()
        self._reduce(loss)
        graphs[1].replay()
        return loss[0]

    def check(self):
        self.engine.check_info()

    # ------------------------------------------------------------------------------------ state
    def local(self, name):
        o, shp = self.offs[name]
        cnt = int(np.prod(shp)) if shp else 1
        return self.theta[o:o + cnt].view(shp) if shp else self.theta[o]

    def local_grad(self, name):
        o, shp = self.offs[name]
        cnt = int(np.prod(shp)) if shp else 1
        return self.grad[o:o + cnt].view(shp) if shp else self.grad[o]

    def gather_state_dict(self, dst=0):
        """The reference's dense state_dict (code/nmgp_dsvi.py:117-155 shapes, dead upper pair blocks 0)
        assembled on rank `dst` from every rank's pair window (None on the other ranks)."""
        D, M = self.D, self.M
        is_dst = self.rank == dst
        if is_dst:
            muU = torch.zeros(D, D, M, dtype=self.dt)
            sU = torch.zeros(D, D, M, M, dtype=self.dt)
        for r in range(self.world):
            if not (is_dst or self.rank == r):
                continue
            i0, i1 = self.ranges[r]
            if r == self.rank:
                mu, su = self.local("mu_U").detach(), self.local("sqrt_U").detach()
            if self.world > 1 and r != dst:
                # point to point, only between rank r and dst, in bounded chunks (NCCL: device buffers)
                nq = i1 * (i1 + 1) // 2 - i0 * (i0 + 1) // 2
                if is_dst:
                    mu, su = torch.empty(nq, M, dtype=self.dt), torch.empty(nq, M, M, dtype=self.dt)
                for t in (mu, su):
                    self._p2p_chunks(t.reshape(-1), r, dst)
            if is_dst:
                q = 0
                for i in range(i0, i1):                  # pairs (i, 0..i) are contiguous in the window
                    muU[i, :i + 1].copy_(mu[q:q + i + 1])
                    sU[i, :i + 1].copy_(su[q:q + i + 1])
                    q += i + 1
        if not is_dst:
            return None
        sd = {name: self.local(name).detach().cpu().clone() for name in PARAM_NAMES if name not in ("mu_U", "sqrt_U")}
        sd["mu_U"], sd["sqrt_U"] = muU, sU
        return {k: sd[k] for k in PARAM_NAMES}

    def _p2p_chunks(self, flat, src, dst, chunk=1 << 26):
        """Send `flat` (on src: this rank's device window) to dst's host tensor `flat` in chunks of at most
        `chunk` elements (256 MB fp32): NCCL moves device buffers, gloo host ones."""
        import torch.distributed as dist
        dev_comm = dist.get_backend(self.group) == "nccl"
        # send / recv take ranks of the default group
        g_src, g_dst = (src, dst) if self.group is None else (dist.get_global_rank(self.group, src),
                                                               dist.get_global_rank(self.group, dst))
        stage = None
        for c0 in range(0, flat.numel(), chunk):
            c1 = min(flat.numel(), c0 + chunk)
            if self.rank == src:
                part = flat[c0:c1]
                dist.send(part.contiguous() if dev_comm else part.cpu(), g_dst, group=self.group)
            else:
                if not dev_comm:
                    dist.recv(flat[c0:c1], g_src, group=self.group)
                    continue
                if stage is None:
                    stage = torch.empty(min(chunk, flat.numel()), dtype=flat.dtype, device=self.dev)
                dist.recv(stage[:c1 - c0], g_src, group=self.group)
                flat[c0:c1].copy_(stage[:c1 - c0])
