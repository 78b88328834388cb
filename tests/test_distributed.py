"""Multi-process (gloo, world_size 2-4, CPU) tests of the DSVI decomposition over ranks.

The GPU path runs the same `distributed.py` code over RCCL; here the per-rank objective is the
closed-form mirror (tests/dsvi_mirror.py, the engine's algebra in torch) and the per-sample
ELBO is the oracle, so the tests check the sharding and reduction semantics:

* data parallel: mean over ranks of the rank-slice gradients == the gradient of the global
  minibatch (ranks share z_v and take their rows' noise) -- SURVEY §8e axis 2;
* sample sharding: sum of per-rank R_s + KL from the last sample's owner == compute_ELBO on one
  process -- SURVEY §8e axis 1.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from collaborative_nonstationary_multivariate_gaussian_process_amd import distributed as DD

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(fn, *args, world=WORLD):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_worker, args=(r, port, fn, args, q, world)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get() for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(res, key=lambda t: t[0])
    for r, out in res:
        if isinstance(out, str):
            raise AssertionError(f"rank {r} failed:\n{out}")
    return [out for _, out in res]


def _worker(rank, port, fn, args, q, world):
    import traceback
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        out = fn(rank, *args)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception:
        q.put((rank, traceback.format_exc()))


# ------------------------------------------------------------------------------------ host logic
@pytest.mark.parametrize("n,world", [(0, 2), (7, 2), (200, 2), (10, 3), (5, 8)])
def test_shard_bounds_cover_once(n, world):
    seen = []
    sizes = []
    for r in range(world):
        s, e = DD.shard_bounds(n, r, world)
        seen += list(range(s, e))
        sizes.append(e - s)
    assert seen == list(range(n))
    assert max(sizes) - min(sizes) <= 1


def test_sample_ids_and_owner():
    ids = [DD.sample_ids(9, r, 4) for r in range(4)]
    assert sorted(sum(ids, [])) == list(range(9))
    assert 8 in ids[DD.last_sample_owner(9, 4)]
    assert DD.world_info() == (0, 1)


# ------------------------------------------------------------------------------------ data parallel
def _toy_global():
    from tests import _golden as G
    g = G.load("toy_forward")
    D, M = 2, 20
    p = G.params(g, D=D, M=M)
    B = int(np.sum(g["sizes"]))
    I = np.repeat(np.arange(D), g["sizes"])
    noise = np.asarray(g["noise"], np.float64)
    Q = D * (D + 1) // 2
    z_v, z_t, z_p = noise[:M], noise[M:M + B], noise[M + B:].reshape(Q, B)
    perm = np.random.default_rng(3).permutation(B)      # the global minibatch, DataLoader order
    return g, p, I, z_v, z_t, z_p, perm


def _rows_problem(g, I, z_v, z_t, z_p, rows):
    """x, y, sizes, noise of `rows` (global ids) grouped by output like vec2list."""
    D = 2
    rows = rows[np.argsort(I[rows], kind="stable")]
    sizes = [int(np.sum(I[rows] == d)) for d in range(D)]
    noise = np.concatenate([z_v, z_t[rows], z_p[:, rows].reshape(-1)])
    return (torch.from_numpy(g["x"][rows].copy()), torch.from_numpy(g["y"][rows].copy()), sizes,
            torch.from_numpy(noise))


def _dp_rank(rank):
    from tests import dsvi_mirror as MR
    g, p, I, z_v, z_t, z_p, perm = _toy_global()
    rank_, world = DD.world_info()
    assert rank_ == rank
    rows = perm[DD.rank_slice(len(perm), rank, world)]
    x, y, sizes, noise = _rows_problem(g, I, z_v, z_t, z_p, rows)
    loss, grads, _ = MR.forward_backward(p, x, y, sizes, torch.from_numpy(g["z"]), float(g["N"]), noise)
    flat = torch.cat([grads[k].reshape(-1) for k in sorted(grads)])
    DD.allreduce_mean_(flat)
    lt = DD.allreduce_mean_(torch.tensor([float(loss)], dtype=torch.float64))
    return flat.numpy(), float(lt[0])


@pytest.mark.parametrize("world", [2, 4])
def test_data_parallel_gradient_equals_global_batch(world):
    from tests import dsvi_mirror as MR
    outs = _run(_dp_rank, world=world)
    g, p, I, z_v, z_t, z_p, perm = _toy_global()
    x, y, sizes, noise = _rows_problem(g, I, z_v, z_t, z_p, perm)
    loss, grads, _ = MR.forward_backward(p, x, y, sizes, torch.from_numpy(g["z"]), float(g["N"]), noise)
    ref = torch.cat([grads[k].reshape(-1) for k in sorted(grads)]).numpy()
    for flat, lmean in outs:
        assert np.array_equal(flat, outs[0][0])                     # identical on every rank
        assert np.linalg.norm(flat - ref) <= 1e-12 * np.linalg.norm(ref)
        assert lmean == pytest.approx(float(loss), rel=1e-12)


# ------------------------------------------------------------------------------------ sample sharding
N_SAMPLE = 5


def _elbo_tape():
    from tests import _golden as G
    g = G.load("toy_elbo")
    return g


def _elbo_rank(rank):
    from oracle import nmgp_oracle as O
    from tests import _golden as G
    g = _elbo_tape()
    xs, ys = G.split_lists(g)
    p = G.params(g, D=2, M=20)
    M, B, Q = 20, int(np.sum(g["sizes"])), 3
    per = M + B + Q * B
    tape = np.asarray(g["noise"], np.float64)
    rank_, world = DD.world_info()
    r_sum, kl = 0.0, None
    for s in DD.sample_ids(N_SAMPLE, rank_, world):
        elbo_s, lps = O.compute_ELBO(p, xs, ys, g["z"], float(g["N"]), O.TapeNoise(tape[s * per:(s + 1) * per]),
                                     n_sample=1)
        r_sum += float(lps[0])
        if s == N_SAMPLE - 1:
            kl = float(lps[0]) - float(elbo_s)       # elbo_1 = R_s - KL(last sample)
    return float(DD.combine_elbo(torch.tensor(r_sum, dtype=torch.float64), kl, N_SAMPLE))


@pytest.mark.parametrize("world", [2, 4])
def test_sample_sharded_elbo_equals_single_process(world):
    from oracle import nmgp_oracle as O
    from tests import _golden as G
    outs = _run(_elbo_rank, world=world)
    g = _elbo_tape()
    xs, ys = G.split_lists(g)
    p = G.params(g, D=2, M=20)
    M, B, Q = 20, int(np.sum(g["sizes"])), 3
    tape = np.asarray(g["noise"], np.float64)[:N_SAMPLE * (M + B + Q * B)]
    ref, _ = O.compute_ELBO(p, xs, ys, g["z"], float(g["N"]), O.TapeNoise(tape), n_sample=N_SAMPLE)
    assert all(o == outs[0] for o in outs)
    assert outs[0] == pytest.approx(float(ref), rel=1e-12)


@pytest.mark.parametrize("D,world,owner", [(2, 2, 1), (2, 3, 0), (4, 8, 3), (5, 2, 0), (128, 8, 7), (50, 4, 2)])
def test_kl_shares_tile_the_factors(D, world, owner):
    """DD.kl_shares: the W | pairs factor ranges of the ranks tile [0, D + Q) exactly once, the owner of the
    last sample holds every W factor and KL_v, and the loads (v counted) differ by at most D + 1."""
    Q = D * (D + 1) // 2
    sh = DD.kl_shares(D, Q, world, owner)
    cover = sorted(f for (f0, f1, _) in sh for f in range(f0, f1))
    assert cover == list(range(D + Q))
    assert sh[owner][0] == 0 and sh[owner][1] >= D and sh[owner][2]
    assert sum(1 for s in sh if s[2]) == 1
    loads = [f1 - f0 + (1 if v else 0) for (f0, f1, v) in sh]
    assert max(loads) - min(loads) <= D + 1


def _factor_kls(p, c, K_G22, D, M):
    """Per-factor KL terms in the engine's factor order (W_0..W_{D-1}, pairs (i, j <= i), then v), the
    oracle's KL_Gaussian against the priors of sample core `c` (KL_W with this sample's K_G22)."""
    from oracle import nmgp_oracle as O
    Sigma_W, Sigma_v, Sigma_U = O._covs(p)
    zero = torch.zeros(M, dtype=torch.float64)
    kls = [float(v) for v in O.KL_Gaussian(p["mu_W"], Sigma_W, zero, K_G22)]
    for i in range(D):
        for j in range(i + 1):
            K22 = c["K_L1_22"] if i == j else c["K_L0_22"]
            kls.append(float(O.KL_Gaussian(p["mu_U"][i, j][None], Sigma_U[i, j][None], zero, K22)[0]))
    kls.append(float(O.KL_Gaussian(p["mu_v"], Sigma_v, zero, c["K_t22"])))
    return kls


def _elbo_kl_sharded_rank(rank):
    """compute_ELBO with the samples AND the KL terms sharded (nmgp_dsvi.compute_ELBO(distributed=True)'s
    decomposition): each rank adds the KL of its kl_shares factor range, evaluated with its own last
    sample (the W factors -- on the owner of the global last sample -- with that sample's K_G22)."""
    from oracle import nmgp_oracle as O
    from tests import _golden as G
    g = _elbo_tape()
    xs, ys = G.split_lists(g)
    D, M = 2, 20
    p = G.params(g, D=D, M=M)
    B, Q = int(np.sum(g["sizes"])), 3
    per = M + B + Q * B
    tape = np.asarray(g["noise"], np.float64)
    rank_, world = DD.world_info()
    owner = DD.last_sample_owner(N_SAMPLE, world)
    f0, f1, with_v = DD.kl_shares(D, Q, world, owner)[rank_]
    mine = DD.sample_ids(N_SAMPLE, rank_, world)
    r_sum, kl = 0.0, None
    Z = torch.as_tensor(np.asarray(g["z"], np.float64)).reshape(-1, 1)
    inputs = torch.cat([torch.as_tensor(x) for x in xs]).reshape(-1, 1)
    for s in mine:
        nz = tape[s * per:(s + 1) * per]
        _, lps = O.compute_ELBO(p, xs, ys, g["z"], float(g["N"]), O.TapeNoise(nz), n_sample=1)
        r_sum += float(lps[0])
        if s == mine[-1]:
            Sigma_W, Sigma_v, Sigma_U = O._covs(p)
            c = O._sample_core(p, Sigma_v, Sigma_U, O._hyper(p), Z, inputs, D, O.TapeNoise(nz), float(g["N"]))
            K_G22 = O.create_Gibbs(Z, Z, c["ell_Z"], c["ell_Z"])
            kls = _factor_kls(p, c, K_G22, D, M)
            kl = sum(kls[f] for f in range(f0, f1)) + (kls[-1] if with_v else 0.0)
    return float(DD.combine_elbo(torch.tensor(r_sum, dtype=torch.float64), kl, N_SAMPLE))


@pytest.mark.parametrize("world", [2, 4])
def test_kl_sharded_elbo_equals_single_process(world):
    from oracle import nmgp_oracle as O
    from tests import _golden as G
    outs = _run(_elbo_kl_sharded_rank, world=world)
    g = _elbo_tape()
    xs, ys = G.split_lists(g)
    p = G.params(g, D=2, M=20)
    M, B, Q = 20, int(np.sum(g["sizes"])), 3
    tape = np.asarray(g["noise"], np.float64)[:N_SAMPLE * (M + B + Q * B)]
    ref, _ = O.compute_ELBO(p, xs, ys, g["z"], float(g["N"]), O.TapeNoise(tape), n_sample=N_SAMPLE)
    assert all(o == outs[0] for o in outs)
    assert outs[0] == pytest.approx(float(ref), rel=1e-12)


# ------------------------------------------------------------------------------------ pair sharding
REP = ["mu_W", "sqrt_W", "mu_v", "sqrt_v", "sigma2_tildeell_log", "length_scales_tildeell_log", "sigma2_L0_log",
       "length_scales_L0_log", "sigma2_L1_log", "length_scales_L1_log", "sigma2_err_log"]


def _pair_problem(name):
    from tests import _golden as G
    g = G.load(name)
    sizes = [int(s) for s in g["sizes"]]
    D, M = len(sizes), len(g["z"])
    p = G.params(g, D=D, M=M)
    B = sum(sizes)
    Q = D * (D + 1) // 2
    noise = np.asarray(g["noise"], np.float64)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(int)
    return g, p, sizes, D, M, B, noise[:M], noise[M:M + B], noise[M + B:].reshape(Q, B), off


def _pair_share(name, rank, world, pair_range):
    """Rank `rank`'s share (mirror): rows and pairs of outputs [i0, i1), KL_W / KL_v on rank 0."""
    from tests import dsvi_mirror as MR
    g, p, sizes, D, M, B, z_v, z_t, z_p, off = _pair_problem(name)
    i0, i1 = pair_range
    rows = np.arange(off[i0], off[i1])
    sz = [sizes[d] if i0 <= d < i1 else 0 for d in range(D)]
    q0, q1 = i0 * (i0 + 1) // 2, i1 * (i1 + 1) // 2
    noise = np.concatenate([z_v, z_t[rows], z_p[q0:q1][:, rows].reshape(-1)])
    N_r = float(g["N"]) * len(rows) / B                 # N_r / B_r = N / B: the full-batch objective
    loss, grads, _ = MR.forward_backward(p, torch.from_numpy(g["x"][rows].copy()), torch.from_numpy(g["y"][rows].copy()),
                                         sz, torch.from_numpy(g["z"]), N_r, torch.from_numpy(noise),
                                         pair_range=pair_range, kl_owner=rank == 0)
    rep = torch.cat([grads[k].reshape(-1) for k in REP])
    own = {(i, j): (grads["mu_U"][i, j].numpy(), grads["sqrt_U"][i, j].numpy())
           for i in range(i0, i1) for j in range(i + 1)}
    return float(loss), rep, own


def _pair_rank(rank, name):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.pair_shard import pair_shard_ranges
    rank_, world = DD.world_info()
    g = _pair_problem(name)
    loss, rep, own = _pair_share(name, rank_, world, pair_shard_ranges(g[3], world)[rank_])
    DD.allreduce_sum_(rep)
    lt = DD.allreduce_sum_(torch.tensor([loss], dtype=torch.float64))
    return rep.numpy(), float(lt[0]), own


@pytest.mark.parametrize("name,world", [("toy_forward", 2), ("mid_forward", 2), ("mid_forward", 3)])
def test_pair_sharded_objective_equals_whole_model(name, world):
    """SURVEY §8e axis 3: ranks owning contiguous output ranges (their rows, their pairs; KL_W / KL_v on
    rank 0) sum to the whole model's -SELBO and gradient; pair gradients never leave their rank."""
    from tests import dsvi_mirror as MR
    outs = _run(_pair_rank, name, world=world)
    g, p, sizes, D, M, B, z_v, z_t, z_p, off = _pair_problem(name)
    loss, grads, _ = MR.forward_backward(p, torch.from_numpy(g["x"]), torch.from_numpy(g["y"]), sizes,
                                         torch.from_numpy(g["z"]), float(g["N"]), torch.from_numpy(np.asarray(g["noise"])))
    ref = torch.cat([grads[k].reshape(-1) for k in REP]).numpy()
    seen = set()
    for rep, lsum, own in outs:
        assert np.array_equal(rep, outs[0][0])                       # identical on every rank
        # (row sums split over ranks: summation order only)
        assert np.linalg.norm(rep - ref) <= 1e-11 * np.linalg.norm(ref)
        assert lsum == pytest.approx(float(loss), rel=1e-12)
        for (i, j), (gm, gs) in own.items():
            assert (i, j) not in seen
            seen.add((i, j))
            np.testing.assert_allclose(gm, grads["mu_U"][i, j].numpy(), rtol=1e-10, atol=1e-12)
            np.testing.assert_allclose(gs, grads["sqrt_U"][i, j].numpy(), rtol=1e-10, atol=1e-12)
    assert seen == {(i, j) for i in range(D) for j in range(i + 1)}


@pytest.mark.parametrize("D,world", [(2, 2), (3, 2), (5, 4), (9, 4), (12, 3), (50, 8), (128, 8)])
def test_pair_shard_ranges_cover_outputs(D, world):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.pair_shard import pair_shard_ranges
    rs = pair_shard_ranges(D, world)
    assert rs[0][0] == 0 and rs[-1][1] == D
    assert all(a < b for a, b in rs) and all(rs[k][1] == rs[k + 1][0] for k in range(world - 1))
    loads = [(b * (b + 1) - a * (a + 1)) // 2 + (D + 1 if k == 0 else 0) for k, (a, b) in enumerate(rs)]
    if D >= 8 * world:
        assert max(loads) <= 1.25 * (sum(loads) / world)
    # the largest share is the minimum over all contiguous splits (dynamic programme over split points)
    cost = lambda a, b, k: (b * (b + 1) - a * (a + 1)) // 2 + (D + 1 if k == 0 else 0)
    best = {(0, 0): 0}
    for k in range(world):
        nxt = {}
        for (r, a), m in best.items():
            for b in range(a + 1, D - (world - k - 1) + 1):
                key = (r + 1, b)
                v = max(m, cost(a, b, k))
                if v < nxt.get(key, float("inf")):
                    nxt[key] = v
        best = nxt
    assert max(loads) == best[(world, D)]


def _bucketed_vs_flat(rank):
    """distributed.grad_buckets + bucketed_allreduce_sum_ (the data-parallel step's two buckets) against one
    all-reduce of the flat vector: the buckets tile the gradient exactly once; with integer-valued gradients
    (exact sums) the result is bit-identical for any world size, with random ones bit-identical at world 2
    (a + b commutes) and within rounding above it -- a ring reduction's summation order depends on where an
    element falls in the ring's chunks, so bucketing may reorder a 3+-term sum.  Every rank ends identical."""
    import numpy as np
    from collaborative_nonstationary_multivariate_gaussian_process_amd import distributed as DD
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import param_layout
    world = dist.get_world_size()
    offs, n = param_layout(4, 16)
    gen = torch.Generator().manual_seed(11 + rank)
    cases = [torch.randint(-2 ** 20, 2 ** 20, (n,), generator=gen).to(torch.float64),
             torch.randn(n, dtype=torch.float64, generator=gen) * (10.0 ** rank)]
    for exact, g0 in zip((True, world == 2), cases):
        flat = g0.clone()
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        g = g0.clone()
        big, small = DD.grad_buckets(offs, g)
        cover = np.zeros(n, np.int64)
        for t in big + small:
            o = (t.data_ptr() - g.data_ptr()) // g.element_size()
            cover[o:o + t.numel()] += 1
        assert (cover == 1).all()
        for w in DD.bucketed_allreduce_sum_(big) + DD.bucketed_allreduce_sum_(small):
            w.wait()
        if exact:
            assert torch.equal(g, flat)
        else:
            assert float((g - flat).abs().max() / flat.abs().max()) < 1e-15
        allg = [torch.empty_like(g) for _ in range(world)]
        dist.all_gather(allg, g)
        assert all(torch.equal(allg[0], t) for t in allg)
    return True


@pytest.mark.parametrize("world", [2, 4])
def test_bucketed_allreduce_equals_flat(world):
    assert all(_run(_bucketed_vs_flat, world=world))
