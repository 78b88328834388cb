"""Multi-process (gloo, world_size 2, CPU) tests of the DSVI decomposition over ranks.

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


def _run(fn, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_worker, args=(r, port, fn, args, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get() for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(res, key=lambda t: t[0])
    for r, out in res:
        if isinstance(out, str):
            raise AssertionError(f"rank {r} failed:\n{out}")
    return [out for _, out in res]


def _worker(rank, port, fn, args, q):
    import traceback
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
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
    assert rank_ == rank and world == WORLD
    rows = perm[DD.rank_slice(len(perm), rank, world)]
    x, y, sizes, noise = _rows_problem(g, I, z_v, z_t, z_p, rows)
    loss, grads, _ = MR.forward_backward(p, x, y, sizes, torch.from_numpy(g["z"]), float(g["N"]), noise)
    flat = torch.cat([grads[k].reshape(-1) for k in sorted(grads)])
    DD.allreduce_mean_(flat)
    lt = DD.allreduce_mean_(torch.tensor([float(loss)], dtype=torch.float64))
    return flat.numpy(), float(lt[0])


def test_data_parallel_gradient_equals_global_batch():
    from tests import dsvi_mirror as MR
    outs = _run(_dp_rank)
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


def test_sample_sharded_elbo_equals_single_process():
    from oracle import nmgp_oracle as O
    from tests import _golden as G
    outs = _run(_elbo_rank)
    g = _elbo_tape()
    xs, ys = G.split_lists(g)
    p = G.params(g, D=2, M=20)
    M, B, Q = 20, int(np.sum(g["sizes"])), 3
    tape = np.asarray(g["noise"], np.float64)[:N_SAMPLE * (M + B + Q * B)]
    ref, _ = O.compute_ELBO(p, xs, ys, g["z"], float(g["N"]), O.TapeNoise(tape), n_sample=N_SAMPLE)
    assert outs[0] == outs[1]
    assert outs[0] == pytest.approx(float(ref), rel=1e-12)
