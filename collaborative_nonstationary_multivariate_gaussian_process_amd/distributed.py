"""Multi-GPU decomposition of the DSVI path (one process per GPU, RCCL over xGMI).

Two independent axes:

* **observations** (training, `inference` / bench): the global minibatch of W*b rows is cut into
  W contiguous slices, rank r trains on slice r, every rank replicates the O(M^3) prior and
  variational factorizations, and the flat gradient is averaged with ONE all-reduce before the
  replicated Adam step.  Because the objective is -(N/b) R_r + KL on every rank, the average is
  -(N/(W b)) sum_r R_r + KL: the gradient of the global-batch objective (bit-for-bit up to the
  reduction order when the ranks share z_v and the row noise of the global batch).
* **Monte-Carlo samples** (`compute_ELBO`, code/nmgp_dsvi.py:330-380): rank r evaluates samples
  r, r+W, ...; the KL terms are split over the ranks too (kl_shares: the pairs' KL_U by factor range,
  KL_W and KL_v on the rank owning the LAST sample -- the reference evaluates KL with the last sample's
  K_G22, :385); one all-reduce of [sum_s R_s, KL share].

Backend-neutral (`nccl` = RCCL on the GPU box, `gloo` in the CPU tests); uses SUM + divide
rather than ReduceOp.AVG, which gloo does not implement.
"""
import torch

try:
    import torch.distributed as dist
except ImportError:  # pragma: no cover
    dist = None


def world_info(group=None):
    """(rank, world_size) of `group`, or (0, 1) when torch.distributed is not initialised."""
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def shard_bounds(n, rank, world):
    """[start, stop) of rank's contiguous share of n items; sizes differ by at most one."""
    base, extra = divmod(int(n), int(world))
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def rank_slice(n, rank, world):
    s, e = shard_bounds(n, rank, world)
    return slice(s, e)


def allreduce_mean_(t, group=None):
    """In-place mean over ranks (no-op on one rank)."""
    rank, world = world_info(group)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.div_(world)
    return t


def allreduce_sum_(t, group=None):
    rank, world = world_info(group)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def grad_buckets(offs, grad):
    """The two all-reduce buckets of the flat DSVI gradient (engine.param_layout offsets `offs`):
    big   -- the sqrt_W and sqrt_U rows: final once the side stream's L-bar products are done (the engine's
             "lbar_done" point), > 99% of the bytes at the HCP / ECoG shapes, 64% at PM2.5;
    small -- everything else (mu_W, mu_v, sqrt_v, mu_U, hyper-parameters): final at the end of the step.
    Views into `grad`; together they cover it exactly once."""
    import numpy as np
    n_sW = int(np.prod(offs["sqrt_W"][1]))
    n_sU = int(np.prod(offs["sqrt_U"][1]))
    big = [grad[offs["sqrt_W"][0]:offs["sqrt_W"][0] + n_sW], grad[offs["sqrt_U"][0]:offs["sqrt_U"][0] + n_sU]]
    small = [grad[0:offs["sqrt_W"][0]], grad[offs["mu_v"][0]:offs["sqrt_U"][0]],
             grad[offs["sigma2_tildeell_log"][0]:]]
    return big, small


def bucketed_allreduce_sum_(buckets, group=None):
    """SUM all-reduce of each view in `buckets` (in order, asynchronously); returns the works.  The element-wise
    sums are those of one all-reduce of the whole vector."""
    rank, world = world_info(group)
    if world <= 1:
        return []
    return [dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True) for t in buckets if t.numel()]


def sample_ids(n_sample, rank, world):
    """Monte-Carlo samples owned by `rank` (round-robin)."""
    return list(range(rank, int(n_sample), int(world)))


def last_sample_owner(n_sample, world):
    return (int(n_sample) - 1) % int(world)


def kl_shares(n_w, n_pairs, world, owner):
    """compute_ELBO's KL terms split over the ranks: the variational factors are W_0..W_{n_w-1} then the
    n_pairs coefficient pairs (the engine's factor list, Sigma_v separate).  Returns, per rank, the
    factor range [f0, f1) and whether it adds KL_v.  The W factors need the LAST sample's K_G22
    (the reference evaluates KL_W with it, code/nmgp_dsvi.py:385), so they -- and KL_v -- go to the
    rank that owns the last sample (`owner`); the pairs (KL_U: sample-independent, ~all the work at
    the ECoG shape) are split so that every rank carries about (n_w + n_pairs + 1) / world factors.
    The ranges tile [0, n_w + n_pairs) exactly once."""
    n = n_w + n_pairs
    shares = [None] * world
    # chunk c of a near-even split of the n + 1 factors (v counted as the owner's) goes to rank owner + c
    tot = n + 1
    bounds = [min(n, (c * tot) // world) for c in range(world + 1)]
    bounds[0], bounds[world] = 0, n
    # the owner's chunk must cover the W factors
    bounds[1] = max(bounds[1], min(n, n_w))
    for c in range(2, world + 1):
        bounds[c] = max(bounds[c], bounds[c - 1])
    for c in range(world):
        shares[(owner + c) % world] = (bounds[c], bounds[c + 1], c == 0)
    return shares


def combine_elbo(r_sum, kl, n_sample, group=None, device=None, dtype=torch.float64):
    """ELBO = (1/n) sum_s R_s - KL from per-rank partials.

    r_sum: this rank's sum of reconstruction terms over its samples (0-d tensor or float);
    kl:    this rank's share of KL_W + KL_v + KL_U (kl_shares; KL_W with the last sample's K_G22, on its
           owner), or None.  Returns a 0-d tensor on `device` (identical on every rank).
    """
    rank, world = world_info(group)
    dev = device if device is not None else (r_sum.device if torch.is_tensor(r_sum) else "cpu")
    buf = torch.zeros(2, dtype=dtype, device=dev)
    buf[0] = r_sum if torch.is_tensor(r_sum) else float(r_sum)
    if kl is not None:
        buf[1] = kl if torch.is_tensor(kl) else float(kl)
    allreduce_sum_(buf, group)
    return buf[0] / int(n_sample) - buf[1]
