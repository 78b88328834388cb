"""Two ranks on one GPU (gloo transport; RCCL is exercised by bench.py under torchrun): the HIP
path's sample-sharded compute_ELBO equals the single-process value, and data-parallel
`inference` keeps the replicated parameters identical on every rank."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

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


def _toy_model():
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP
    from tests import _golden as G
    g = G.load("toy_elbo")
    xs, ys = G.split_lists(g)
    model = NMGP(number_observations=int(g["N"]), dim_outputs=2, Z=g["z"], seed=22, device="cuda:0")
    return model, xs, ys


def _elbo(rank, distributed=True):
    model, xs, ys = _toy_model()
    torch.manual_seed(5)
    xl = [torch.from_numpy(x) for x in xs]
    yl = [torch.from_numpy(y) for y in ys]
    return float(model.compute_ELBO(xl, yl, n_sample=5, distributed=distributed))


def test_sample_sharded_compute_elbo_matches_one_process():
    outs = _run(_elbo)
    ref = _elbo(0, distributed=False)
    assert outs[0] == outs[1]
    assert outs[0] == pytest.approx(ref, rel=1e-12)


def _dp_train(rank):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import inference
    from tests import _golden as G
    g = G.load("toy_elbo")
    xs, ys = G.split_lists(g)
    torch.manual_seed(0)
    model, losses, _ = inference(xs, ys, g["z"], 50, 2, hyperpars={}, fix_hyperpars=True, lr=0.005, itnum=1,
                                 show_ELBO=False, device="cuda:0", noise="device", distributed=True)
    return model._theta.detach().cpu().numpy(), [float(v) for v in losses]


def test_data_parallel_inference_keeps_ranks_in_sync():
    outs = _run(_dp_train)
    (t0, l0), (t1, l1) = outs
    assert np.array_equal(t0, t1)
    assert l0 == l1 and len(l0) == 2            # 200 rows / (50 x 2 ranks) = 2 global steps
    assert all(np.isfinite(l0))


def _dp_train_ragged(rank):
    """N % (batch * world) != 0 with the reference RNG (noise='torch'), several epochs: the ragged last
    global batch splits unevenly, one global batch is shorter than the world and must be skipped on
    every rank, and the per-rank torch.randn draws must not desynchronise the loader."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import inference
    from tests import _golden as G
    g = G.load("toy_elbo")
    xs, ys = G.split_lists(g)
    xs = [xs[0], xs[1][:-29]]                      # 171 rows: global batches of 2 x 50 -> 100, 71 (36 / 35)
    ys = [ys[0], ys[1][:-29]]
    torch.manual_seed(100 + rank)                  # different global streams per rank on purpose
    model, losses, _ = inference(xs, ys, g["z"], 50, 2, hyperpars={}, fix_hyperpars=True, lr=0.005, itnum=3,
                                 show_ELBO=False, device="cuda:0", noise="torch", distributed=True)
    return model._theta.detach().cpu().numpy(), [float(v) for v in losses]


def test_data_parallel_ragged_batches_torch_noise_keep_ranks_in_sync():
    outs = _run(_dp_train_ragged)
    (t0, l0), (t1, l1) = outs
    assert np.array_equal(t0, t1)
    assert l0 == l1 and len(l0) == 3 * 2           # 2 usable global batches per epoch
    assert all(np.isfinite(l0))


def _dp_train_device_ragged(rank):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import inference
    from tests import _golden as G
    g = G.load("toy_elbo")
    xs, ys = G.split_lists(g)
    xs = [xs[0], np.concatenate([xs[1], xs[1][:1] + 1e-3])]     # 201 rows: 100, 100, 1 (skipped on both ranks)
    ys = [ys[0], np.concatenate([ys[1], ys[1][:1]])]
    torch.manual_seed(7)
    model, losses, _ = inference(xs, ys, g["z"], 50, 2, hyperpars={}, fix_hyperpars=True, lr=0.005, itnum=2,
                                 show_ELBO=False, device="cuda:0", noise="device", distributed=True)
    return model._theta.detach().cpu().numpy(), [float(v) for v in losses]


def test_data_parallel_device_pipeline_ragged_keeps_ranks_in_sync():
    outs = _run(_dp_train_device_ragged)
    (t0, l0), (t1, l1) = outs
    assert np.array_equal(t0, t1)
    assert l0 == l1 and len(l0) == 2 * 2           # the 1-row global batch is skipped every epoch
    assert all(np.isfinite(l0))


def _dp_overlap_vs_single(rank):
    """The bucketed all-reduce overlapped with the backward (eager step) sums exactly what the single
    all-reduce after the graph-replayed step sums: identical parameters."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import inference
    from tests import _golden as G
    g = G.load("toy_elbo")
    xs, ys = G.split_lists(g)
    out = []
    for use_graph in (False, True):
        torch.manual_seed(3)
        model, losses, _ = inference(xs, ys, g["z"], 50, 2, hyperpars={}, fix_hyperpars=True, lr=0.005, itnum=2,
                                     show_ELBO=False, device="cuda:0", noise="device", distributed=True,
                                     use_graph=use_graph)
        out.append((model._theta.detach().cpu().numpy(), [float(v) for v in losses]))
    return out


def test_data_parallel_overlapped_allreduce_equals_single():
    outs = _run(_dp_overlap_vs_single)
    for (eager, graph) in outs:
        assert np.array_equal(eager[0], graph[0])
        assert eager[1] == graph[1]
    assert np.array_equal(outs[0][0][0], outs[1][0][0])


def _dp_graph_bucketed_vs_flat(rank):
    """The data-parallel step on the graph path (DsviTrainer.dp_graph_step: gradient graph with an external
    event node at lbar_done, the sqrt_W / sqrt_U bucket all-reduced from that node on while the backward's
    tail runs, then the remainder, then the 1/world + Adam graph) against the flat form (gradient graph, ONE
    all-reduce of the whole vector, update graph): identical parameters after 4 steps (two ranks: a + b
    commutes, so the sums are bit-identical)."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
    from tests import _golden as G
    g = G.load("toy_elbo")
    xs, ys = G.split_lists(g)
    half = [slice(0, len(x) // 2) if rank == 0 else slice(len(x) // 2, len(x)) for x in xs]
    xr = [x[h] for x, h in zip(xs, half)]
    yr = [y[h] for y, h in zip(ys, half)]
    thetas = []
    for bucketed in (False, True):
        model = NMGP(number_observations=int(g["N"]), dim_outputs=2, Z=g["z"], seed=22, device="cuda:0",
                     noise="device")
        model._noise_seed = 22 + 7919 * rank
        tr = DsviTrainer(model, lr=0.005)
        x, y, sizes = model._prepare(xr, yr)
        eng = model.engine(sum(sizes))
        eng.load_batch(x, y, sizes)
        if bucketed:
            tr.capture_dp(eng, WORLD, mode="bucketed")
        else:
            gg, upd = tr.capture(eng, include_update=False), tr.capture_update(WORLD)
        for _ in range(4):
            if bucketed:
                tr.dp_graph_step(eng)
            else:
                gg.replay()
                dist.all_reduce(model._grad, op=dist.ReduceOp.SUM)
                upd.replay()
        torch.cuda.synchronize()
        thetas.append(model._theta.detach().cpu().numpy())
    return thetas


def test_data_parallel_graph_bucketed_allreduce_equals_flat():
    outs = _run(_dp_graph_bucketed_vs_flat)
    for flat, bucketed in outs:
        assert np.all(np.isfinite(flat))
        assert np.array_equal(flat, bucketed)
    assert np.array_equal(outs[0][1], outs[1][1])
    assert not np.array_equal(outs[0][1], _toy_theta0())       # the steps moved the parameters


def _toy_theta0():
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP
    from tests import _golden as G
    g = G.load("toy_elbo")
    return NMGP(number_observations=int(g["N"]), dim_outputs=2, Z=g["z"], seed=22,
                device="cuda:0")._theta.detach().cpu().numpy()
