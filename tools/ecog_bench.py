"""ECoG-full-shaped configuration (BASELINE.json configs[3]) on one MI355X.

  D = 128 channels (Q = 8256 coefficient pairs), M = 1024 inducing points, N = 50,048 rows (391 per
  channel), fp32, packed Q-pair layout (pair_layout="packed": 35 GB per copy of the parameters instead
  of 69 GB dense), device Philox noise.

modes:
  train  one DSVI iteration (B = 512 rows, forward + backward + Adam) replayed as a HIP graph: it/s.
         Memory: parameters + gradient + Adam moments 141 GB, factor workspaces 106 GB.
  elbo   compute_ELBO on all N rows, S Monte-Carlo samples (default 8 = one GPU's share of 64 over 8
         GPUs): samples/s; the first sample of the call also builds the sample-independent factors
         (RBF priors, pair quadratic forms), the last one the KL terms (8385 Cholesky factors).
  shard  pair sharding (SURVEY §8e axis 3, pair_shard.PairShard): the training step split over W ranks by
         output ranges; each rank's share (its rows b_r = B N_r / N, its pairs, KL_W / KL_v on rank 0) is
         built and timed ALONE on this GPU, one after the other (eager launches; the per-step all-reduce of
         the replicated gradient is reported as bytes).  The W-GPU step is bounded by the slowest share.
usage: python tools/ecog_bench.py {train|elbo|shard} [--steps K] [--samples S] [--D 128] [--M 1024] [--rows 391]
       [--world W] [--ranks r0,r1,..]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def data(D, rows, seed=7):
    rng = np.random.default_rng(seed)
    xs = [np.sort(rng.uniform(0, 1, rows)) for _ in range(D)]
    ys = [np.sin(6 * x + 0.1 * d) + 0.3 * rng.standard_normal(rows) for d, x in enumerate(xs)]
    return xs, ys


def model(D, M, N, dev):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP
    t0 = time.time()
    m = NMGP(number_observations=N, dim_outputs=D, Z=np.linspace(0, 1, M), minibatch_size=512, seed=22, device=dev,
             noise="device", dtype=torch.float32, pair_layout="packed")
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        getattr(m, k).data.fill_(float(np.log(3.0 / M)))
        getattr(m, k).requires_grad = False
    return m, time.time() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["train", "elbo", "shard"])
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ranks", type=str, default="")
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--M", type=int, default=1024)
    ap.add_argument("--rows", type=int, default=391)
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--samples", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    D, M = a.D, a.M
    xs, ys = data(D, a.rows)
    N = D * a.rows
    if a.mode == "shard":
        return shard(a, xs, ys, N, dev)
    m, t_init = model(D, M, N, dev)
    rec = {"config": f"ECoG-shaped: D={D}, Q={D * (D + 1) // 2}, M={M}, N={N}, fp32, packed pairs",
           "init_s": round(t_init, 2), "param_GB": round(m._theta.numel() * 4 / 1e9, 2)}
    if a.mode == "train":
        from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import DsviTrainer
        tr = DsviTrainer(m, lr=0.01)
        eng = m.engine(a.B)
        X = np.concatenate(xs); Y = np.concatenate(ys)
        I = np.concatenate([np.full(a.rows, d) for d in range(D)])
        rng = np.random.default_rng(3)
        nb = 4
        bx, by, bi, bs = [], [], [], []
        for s in range(nb):
            idx = rng.choice(N, a.B, replace=False)
            idx = idx[np.argsort(I[idx], kind="stable")]
            bx.append(X[idx]); by.append(Y[idx]); bi.append(I[idx])
            bs.append(np.concatenate([[0], np.cumsum(np.bincount(I[idx], minlength=D))]))
        f = lambda v, t: torch.tensor(np.stack(v), dtype=t, device=dev)
        eng.bind_dataset(f(bx, torch.float32), f(by, torch.float32), f(bi, torch.int32), f(bs, torch.int32))
        t0 = time.time()
        g = tr.capture(eng)
        torch.cuda.synchronize()
        rec["capture_s"] = round(time.time() - t0, 2)
        g.replay()
        torch.cuda.synchronize()
        m.check_numerics()
        t0 = time.time()
        for _ in range(a.steps):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.time() - t0) / a.steps
        m.check_numerics()
        rec.update({"mode": "train", "B": a.B, "steps": a.steps, "s_per_step": round(dt, 4), "it_per_s": round(1 / dt, 3),
                    "loss": float(eng.out[0]), "peak_mem_GB": round(torch.cuda.max_memory_allocated() / 1e9, 1)})
    else:
        Xl = [torch.from_numpy(x) for x in xs]
        Yl = [torch.from_numpy(y) for y in ys]
        t0 = time.time()
        e1 = m.compute_ELBO(Xl, Yl, n_sample=1)                 # one sample incl. factors + KL (and warm-up)
        torch.cuda.synchronize()
        t_one = time.time() - t0
        t0 = time.time()
        e = m.compute_ELBO(Xl, Yl, n_sample=a.samples)
        torch.cuda.synchronize()
        t_s = time.time() - t0
        # per-part costs on the engine: first (uncached) sample, a cached sample, the KL of the last one
        eng = m._engines[N]
        parts = {}
        for name, kw in (("first_sample_s", dict(with_kl=False, cached=False)), ("cached_sample_s", dict(with_kl=False, cached=True)),
                         ("cached_sample_with_kl_s", dict(with_kl=True, cached=True))):
            eng.device_noise(1, m._noise_counter)
            torch.cuda.synchronize()
            t0 = time.time()
            eng.elbo_sample(**kw)
            torch.cuda.synchronize()
            parts[name] = round(time.time() - t0, 4)
        rec.update(parts)
        c, f, k = parts["cached_sample_s"], parts["first_sample_s"], parts["cached_sample_with_kl_s"] - parts["cached_sample_s"]
        rec["projected_64_samples_s"] = {str(W): round(f + (64 // W - 1) * c + k, 3) for W in (1, 2, 4, 8)}
        rec["projected_scaling_8"] = round(rec["projected_64_samples_s"]["1"] / rec["projected_64_samples_s"]["8"], 2)
        rec.update({"mode": "elbo", "samples": a.samples, "first_call_1_sample_s": round(t_one, 3),
                    "call_s": round(t_s, 3), "samples_per_s": round(a.samples / t_s, 3), "elbo": float(e),
                    "elbo_1": float(e1), "peak_mem_GB": round(torch.cuda.max_memory_allocated() / 1e9, 1)})
    print(json.dumps(rec), flush=True)


def shard(a, xs, ys, N, dev):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.pair_shard import PairShard, pair_shard_ranges
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import pair_window
    D, M, W = a.D, a.M, a.world
    ranges = pair_shard_ranges(D, W)
    ranks = [int(r) for r in a.ranks.split(",")] if a.ranks else list(range(W))
    out = {"config": f"ECoG-shaped: D={D}, Q={D * (D + 1) // 2}, M={M}, N={N}, fp32, B={a.B}, pair-sharded over {W} ranks",
           "ranges": ranges, "ranks": {}}
    rep_bytes = None
    for r in ranks:
        i0, i1 = ranges[r]
        q0, Q = pair_window(D, (i0, i1))
        g = torch.Generator(device=dev).manual_seed(100 + r)
        rn = lambda *s: torch.randn(*s, generator=g, device=dev, dtype=torch.float32)
        p = {"mu_W": 0.1 * rn(D, M), "sqrt_W": 0.1 * rn(D, M, M), "mu_v": -4 * torch.ones(M, device=dev),
             "sqrt_v": 0.1 * rn(M, M), "mu_U": 0.1 * rn(Q, M), "sqrt_U": 0.1 * rn(Q, M, M),
             "sigma2_tildeell_log": torch.tensor(0.), "length_scales_tildeell_log": torch.tensor(float(np.log(3.0 / M))),
             "sigma2_L0_log": torch.tensor(0.), "length_scales_L0_log": torch.tensor(float(np.log(3.0 / M))),
             "sigma2_L1_log": torch.tensor(0.), "length_scales_L1_log": torch.tensor(float(np.log(3.0 / M))),
             "sigma2_err_log": torch.tensor(-2.)}
        n_r = sum(len(x) for x in xs[i0:i1])
        b_r = max(1, int(round(a.B * n_r / N)))
        rng = np.random.default_rng(5 + r)
        torch.cuda.reset_peak_memory_stats()
        t0 = time.time()
        sh = PairShard(p, np.linspace(0, 1, M), B_r=b_r, N_r=n_r, rank=r, world=W, dtype=torch.float32, device=dev,
                       frozen=("length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"),
                       ranges=ranges, pairs_local=True)
        del p
        # stratified minibatch: b_r rows of this rank's outputs
        idx = np.sort(rng.choice(n_r, b_r, replace=False))
        cuts = np.concatenate([[0], np.cumsum([len(x) for x in xs[i0:i1]])])
        bx = [xs[i0 + k][idx[(idx >= cuts[k]) & (idx < cuts[k + 1])] - cuts[k]] for k in range(i1 - i0)]
        by = [ys[i0 + k][idx[(idx >= cuts[k]) & (idx < cuts[k + 1])] - cuts[k]] for k in range(i1 - i0)]
        sh.load(bx, by)
        t_init = time.time() - t0
        sh.grad_step(reduce=False)                  # warm-up (plans, first launches)
        sh.update()
        torch.cuda.synchronize()
        sh.check()
        t0 = time.time()
        for _ in range(a.steps):
            loss = sh.grad_step(reduce=False)
            sh.update()
        torch.cuda.synchronize()
        dt = (time.time() - t0) / a.steps
        sh.check()
        rep_bytes = sum(t.numel() for t in sh._rep) * 4
        out["ranks"][r] = {"outputs": [i0, i1], "pairs": Q, "factors": sh.engine.NF, "rows": b_r,
                           "s_per_step": round(dt, 4), "loss_share": float(loss), "init_s": round(t_init, 2),
                           "param_GB": round(sh.theta.numel() * 4 / 1e9, 2),
                           "peak_mem_GB": round(torch.cuda.max_memory_allocated() / 1e9, 1)}
        print(json.dumps({"rank": r, **out["ranks"][r]}), flush=True)
        del sh, loss
        import gc
        gc.collect()                                # the engine's schedule closures form cycles
        torch.cuda.empty_cache()
    ts = [v["s_per_step"] for v in out["ranks"].values()]
    out["slowest_share_s"] = max(ts)
    out["replicated_grad_bytes_per_step"] = rep_bytes
    # ring all-reduce: 2 (W-1)/W of the bytes over each GPU's busiest xGMI link (~150 GB/s spec)
    out["allreduce_s_at_150GBps"] = round(2 * (W - 1) / W * rep_bytes / 150e9, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
