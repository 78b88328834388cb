"""Measurement of the non-headline configurations of BASELINE.json / SURVEY §8d (GPU box).

bench.py measures the headline PM2.5-shaped step; this prints one JSON line per extra config:
  hcp     D=50 outputs x 10,000 timepoints (500k rows), M=512, B=5000, fp32 engine, ell = 3/M
          (cond(K_uu + 1e-4 I) <~ 1e5 as SURVEY §8d prescribes), device noise, HIP-graph step.
  pm25f32 the PM2.5 shape through the fp32 engine (for the fp32/fp64 ratio).
  toy     the shipped toy shape (D=2, M=20, B=200), fp64, graph step (latency floor).
usage: python tools/bench_configs.py [config ...]   (default: toy pm25f32 hcp)
Synthetic data (seeded); the ECoG shape (D=128, M=1024, packed pairs) is measured by
tools/ecog_bench.py and bench.py's compute_ELBO leg.
"""
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {  # name: (D, rows per output, M, B, dtype, length-scale log (None = bench default -1))
    "toy": (2, 100, 20, 200, torch.float64, None),
    "pm25f32": (5, 2000, 256, 2000, torch.float32, -1.0),
    "hcp": (50, 10000, 512, 5000, torch.float32, math.log(3.0 / 512)),
}


def run(name, steps=20, warmup=3):
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
    D, n, M, B, dt, ls = CONFIGS[name]
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(2024)
    xs = [np.sort(rng.uniform(0, 1, n)) if name != "hcp" else np.arange(n) / n for _ in range(D)]
    ys = [np.sin(6 * x + d) + 0.3 * rng.standard_normal(n) for d, x in enumerate(xs)]
    t_init = time.time()
    model = NMGP(number_observations=D * n, dim_outputs=D, Z=np.linspace(0, 1, M), minibatch_size=B, seed=22,
                 device=dev, noise="device", dtype=dt)
    t_init = time.time() - t_init
    if ls is not None:
        for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
            getattr(model, k).data.fill_(ls)
            getattr(model, k).requires_grad = False
    trainer = DsviTrainer(model, lr=0.01)
    eng = model.engine(B)
    # one epoch of output-grouped minibatches resident in HBM, gathered on device each step
    X = np.concatenate(xs); Y = np.concatenate(ys)
    I = np.concatenate([np.full(n, d) for d in range(D)])
    perm = rng.permutation(len(X))
    nb = min(len(X) // B, 16)
    bx, by, bi, bs = [], [], [], []
    for s in range(nb):
        idx = perm[s * B:(s + 1) * B]
        idx = idx[np.argsort(I[idx], kind="stable")]
        bx.append(X[idx]); by.append(Y[idx]); bi.append(I[idx])
        bs.append(np.concatenate([[0], np.cumsum(np.bincount(I[idx], minlength=D))]))
    f = lambda a, t: torch.tensor(np.stack(a), dtype=t, device=dev)
    eng.bind_dataset(f(bx, dt), f(by, dt), f(bi, torch.int32), f(bs, torch.int32))
    graph = trainer.capture(eng, include_update=True)
    for _ in range(warmup):
        graph.replay()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(steps):
        graph.replay()
    torch.cuda.synchronize()
    el = time.time() - t0
    loss = float(eng.out[0])
    eng.check_info()
    return {"config": name, "metric": "DSVI ELBO iterations/sec", "value": round(steps / el, 3), "unit": "it/s",
            "ms_per_step": round(1000 * el / steps, 3), "steps": steps, "warmup": warmup,
            "dtype": "f32" if dt == torch.float32 else "f64", "data": "synthetic",
            "shape": {"D_outputs": D, "rows_per_output": n, "M_inducing": M, "minibatch_rows": B,
                      "Q_pairs": D * (D + 1) // 2, "params": int(model._theta.numel())},
            "loss_finite": bool(np.isfinite(loss)), "host_init_s": round(t_init, 1)}


if __name__ == "__main__":
    names = sys.argv[1:] or ["toy", "pm25f32", "hcp"]
    for nm in names:
        print(json.dumps(run(nm)), flush=True)
