"""Pair sharding on the HIP path (SURVEY §8e axis 3): each rank's engine holds only the pairs of a
contiguous output range (engine.DsviEngine(pair_range=..., kl_owner=...), pair_shard.PairShard).

* one process, shares of 2-3 ranks evaluated in turn on the golden fixtures: the summed loss and
  replicated gradients, and every share's pair gradients, against the oracle's autograd at the same
  gates as the whole-model engine (tests/test_gpu_engine.py CASES) and against the whole-model engine;
* two ranks on the box's GPU (gloo transport): Adam steps keep the replicated parameters identical on
  both ranks, the first loss equals the one-process sum of the shares, and the gathered dense
  state_dict holds each rank's pair blocks.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import nmgp_oracle as O
from tests import _golden as G
from tests.test_gpu_engine import CASES, SURVEY_FP64_GRAD, SURVEY_FP64_LOSS, _rel

pytestmark = pytest.mark.gpu

REP = ["mu_W", "sqrt_W", "mu_v", "sqrt_v"] + O.PARAM_NAMES[6:]


def _shares(case, world, dtype=torch.float64):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.pair_shard import PairShard, pair_shard_ranges
    D, M = CASES[case][:2]
    g = G.load(case)
    xs, ys = G.split_lists(g)
    p = G.params(g, D=D, M=M)
    sizes = [len(x) for x in xs]
    B = sum(sizes)
    Q = D * (D + 1) // 2
    noise = np.asarray(g["noise"], np.float64)
    z_v, z_t, z_p = noise[:M], noise[M:M + B], noise[M + B:].reshape(Q, B)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(int)
    out = []
    for r, (i0, i1) in enumerate(pair_shard_ranges(D, world)):
        rows = np.arange(off[i0], off[i1])
        q0, q1 = i0 * (i0 + 1) // 2, i1 * (i1 + 1) // 2
        nz = np.concatenate([z_v, z_t[rows], z_p[q0:q1][:, rows].reshape(-1)])
        sh = PairShard(p, g["z"], B_r=len(rows), N_r=float(g["N"]) * len(rows) / B, rank=r, world=world,
                       dtype=dtype, device="cuda")
        sh.load(xs[i0:i1], ys[i0:i1], noise=nz)
        loss = sh.grad_step(reduce=False)
        torch.cuda.synchronize()
        sh.check()
        out.append((sh, float(loss)))
    return g, xs, ys, p, out


@pytest.mark.parametrize("case,world", [("toy_forward", 2), ("mid_forward", 2), ("mid_forward", 3),
                                        ("pm25_forward", 2), ("pm25_forward", 3)])
def test_pair_shares_sum_to_oracle(case, world):
    g, xs, ys, p, shares = _shares(case, world)
    D, M, ltol, gtol = CASES[case]
    q = {k: v.clone().requires_grad_() for k, v in p.items()}
    loss, _ = O.forward(q, xs, ys, g["z"], float(g["N"]), O.TapeNoise(g["noise"]))
    loss.backward()
    tot = sum(l for _, l in shares)
    gd = {k: sum(sh.local_grad(k).detach().double().cpu() for sh, _ in shares) for k in REP}
    muU = torch.zeros(D, D, M, dtype=torch.float64)
    sU = torch.zeros(D, D, M, M, dtype=torch.float64)
    for sh, _ in shares:
        i0, i1 = sh.pair_range
        gm, gs = sh.local_grad("mu_U").double().cpu(), sh.local_grad("sqrt_U").double().cpu()
        for n, (i, j) in enumerate([(i, j) for i in range(i0, i1) for j in range(i + 1)]):
            muU[i, j], sU[i, j] = gm[n], gs[n]
    gd["mu_U"], gd["sqrt_U"] = muU, sU
    lerr = abs(tot - float(loss)) / abs(float(loss))
    errs = {k: _rel(gd[k], q[k].grad) for k in O.PARAM_NAMES if float(q[k].grad.norm()) > 0}
    whole = _rel(torch.cat([gd[k].reshape(-1) for k in O.PARAM_NAMES]),
                 torch.cat([q[k].grad.reshape(-1) for k in O.PARAM_NAMES]))
    print(f"PARITY pair-shard {case} x{world}: loss rel {lerr:.3e}  max grad rel-norm {max(errs.values()):.3e}  "
          f"whole {whole:.3e}")
    assert lerr <= min(ltol, SURVEY_FP64_LOSS) and whole <= SURVEY_FP64_GRAD, (lerr, whole)
    bad = {k: e for k, e in errs.items() if e > gtol}
    assert not bad, f"gradient mismatch {bad} (all: {errs})"


def test_pair_share_sizes_are_sharded():
    """Each share's parameter vector and factor workspace hold only its pairs (ECoG-style memory cut)."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import param_layout
    g, xs, ys, p, shares = _shares("mid_forward", 2)
    D, M = 3, 64
    full = param_layout(D, M, packed=True)[1]
    assert sum(sh.theta.numel() for sh, _ in shares) < 2 * full
    for sh, _ in shares:
        assert sh.engine.Afac.shape[0] == sh.engine.NF + 4 and sh.engine.NF == sh.engine.nW + sh.Q + 1
    assert shares[1][0].engine.nW == 0 and shares[0][0].engine.nW == D


# ------------------------------------------------------------------------------------ two ranks
WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, fn, q):
    import traceback
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        out = fn(rank)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception:
        q.put((rank, traceback.format_exc()))


def _run(fn):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_worker, args=(r, port, fn, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted([q.get() for _ in range(WORLD)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=300)
    for r, out in res:
        if isinstance(out, str):
            raise AssertionError(f"rank {r} failed:\n{out}")
    return [out for _, out in res]


def _train_problem():
    rng = np.random.default_rng(11)
    D, M, n = 4, 48, 60
    xs = [np.sort(rng.uniform(0, 1, n)) for _ in range(D)]
    ys = [np.sin(5 * x + d) + 0.1 * rng.standard_normal(n) for d, x in enumerate(xs)]
    p = O.new_params(D, M, seed=22)
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        p[k] = torch.tensor(-1.0, dtype=torch.float64)
    return D, M, xs, ys, p, np.linspace(0, 1, M)


def _share(rank, world):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.pair_shard import PairShard, pair_shard_ranges
    D, M, xs, ys, p, z = _train_problem()
    i0, i1 = pair_shard_ranges(D, world)[rank]
    nr = sum(len(x) for x in xs[i0:i1])
    sh = PairShard(p, z, B_r=nr, N_r=nr, rank=rank, world=world, dtype=torch.float64, device="cuda:0", lr=0.01,
                   frozen=("length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"))
    sh.load(xs[i0:i1], ys[i0:i1])
    return sh


def _train(rank):
    sh = _share(rank, WORLD)
    losses = [float(sh.step()) for _ in range(4)]
    torch.cuda.synchronize()
    sh.check()
    rep = torch.cat([sh.local(k).reshape(-1) for k in REP]).cpu().numpy()
    sd = sh.gather_state_dict()
    own = {name: sh.local(name).cpu().numpy() for name in ("mu_U", "sqrt_U")}
    return losses, rep, (None if sd is None else {k: v.numpy() for k, v in sd.items()}), own, sh.pair_range


def test_two_rank_pair_sharded_training():
    outs = _run(_train)
    (l0, rep0, sd, own0, pr0), (l1, rep1, _, own1, pr1) = outs
    assert l0 == l1 and all(np.isfinite(l0))
    assert np.array_equal(rep0, rep1)                       # replicated parameters stay identical
    # first loss = the one-process sum of both shares' terms (same seeds -> same noise)
    first = 0.0
    for r in range(WORLD):
        sh = _share(r, WORLD)
        first += float(sh.grad_step(reduce=False))
    assert l0[0] == pytest.approx(first, rel=1e-13)
    # the gathered dense state holds every rank's pairs
    for own, (i0, i1) in ((own0, pr0), (own1, pr1)):
        for n, (i, j) in enumerate([(i, j) for i in range(i0, i1) for j in range(i + 1)]):
            assert np.array_equal(sd["mu_U"][i, j], own["mu_U"][n])
            assert np.array_equal(sd["sqrt_U"][i, j], own["sqrt_U"][n])
    assert not np.any(sd["sqrt_U"][0, 1])                   # dead upper pair blocks stay zero


def _share_rows(rank, world, nb=2):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.pair_shard import PairShard, pair_shard_ranges
    D, M, xs, ys, p, z = _train_problem()
    i0, i1 = pair_shard_ranges(D, world)[rank]
    nr = sum(len(x) for x in xs[i0:i1])
    sh = PairShard(p, z, B_r=nr // nb, N_r=nr, rank=rank, world=world, dtype=torch.float64, device="cuda:0", lr=0.01,
                   frozen=("length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"))
    assert sh.bind_rows(xs[i0:i1], ys[i0:i1], seed=3) == nb
    return sh


def _train_pipeline(rank):
    """The rank's rows resident in HBM, minibatches gathered on the device: eager steps vs graph replays."""
    out = []
    for graph in (False, True):
        sh = _share_rows(rank, WORLD)
        if graph:
            sh.capture()
        losses = []
        for it in range(5):
            if it == 2:
                sh.new_epoch()                # a fresh device permutation between epochs
            losses.append(float(sh.step()))
        torch.cuda.synchronize()
        sh.check()
        out.append((losses, sh.theta.cpu().numpy()))
    return out


def test_two_rank_pair_sharded_training_device_pipeline_graph():
    """the pair-sharded step with its rows in HBM (bind_rows / new_epoch: one on-device
    gather per step) replays from HIP graphs around the replicated-gradient all-reduce; the replayed steps
    equal the eager ones bit for bit and the replicated parameters stay identical on both ranks."""
    outs = _run(_train_pipeline)
    for (eager, graph) in outs:
        assert eager[0] == graph[0] and all(np.isfinite(eager[0]))
        assert np.array_equal(eager[1], graph[1])
    assert outs[0][1][0] == outs[1][1][0]                  # the summed loss is the same on both ranks
