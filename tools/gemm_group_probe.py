"""Per-group GEMM timing of the PM2.5-shaped step: every grouped GEMM launch of the engine, alone, on
the 64x64 tile kernel and on the latency kernel (same descriptors), each replayed REPS times inside a
HIP graph so launch overhead is excluded; prints algorithmic GFLOP, us per launch and TF/s.

usage (GPU box): python tools/gemm_group_probe.py [group ...] [--reps 50] [--kt-caps 8,16,32] [--cfg hcp|ecog]
--cfg: the fp32 training configurations of bench.py (bench.train_setup) instead of the PM2.5-shaped step.
--kt-caps: also time the tile kernel with GemmGroup(kt_cap=c) for each c (split so that no workgroup runs
more than ~c k-tiles), as "tile_cap<c>" entries.
Outputs of the groups are scratch here (the probe runs the launches back to back on the same buffers).
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
    import collaborative_nonstationary_multivariate_gaussian_process_amd.hip_ops as H
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 50
    caps = ([int(c) for c in sys.argv[sys.argv.index("--kt-caps") + 1].split(",")]
            if "--kt-caps" in sys.argv else [])
    args = [a for a in args if not (a[0].isdigit() or a == ",")]
    D, M, B, n = 5, 256, 2000, 2000
    dev = torch.device("cuda", 0)
    cfg = sys.argv[sys.argv.index("--cfg") + 1] if "--cfg" in sys.argv else None
    args = [a for a in args if a not in ("hcp", "ecog")]
    rng = np.random.default_rng(0)
    xs = [torch.from_numpy(np.sort(rng.uniform(0, 1, n))) for _ in range(D)]
    ys = [torch.from_numpy(rng.standard_normal(n)) for _ in range(D)]
    if cfg:
        sys.path.insert(0, ROOT)
        import bench
        model, trainer, eng = bench.train_setup(dev, cfg)
        trainer.grad_step(eng)                          # buffers hold one step's values (bound epoch)
    else:
        model = NMGP(number_observations=D * n, dim_outputs=D, Z=np.linspace(0, 1, M), minibatch_size=B, seed=1,
                     device=dev, noise="device")
        eng = model.engine(B)
        idx = rng.permutation(D * n)[:B]
        X = torch.cat(xs)[idx]
        Y = torch.cat(ys)[idx]
        I = torch.from_numpy(np.repeat(np.arange(D), n))[idx]
        xl = [X[I == d] for d in range(D)]
        yl = [Y[I == d] for d in range(D)]
        x, y, sizes = model._prepare(xl, yl)
        eng.load_batch(x, y, sizes)
        DsviTrainer(model, 0.01).grad_step(eng)          # buffers hold one step's values
    torch.cuda.synchronize()
    seg_host = eng.seg.cpu().numpy()
    s = torch.cuda.Stream(device=dev)
    for name, grp in eng.gemm_groups():
        if args and name not in args:
            continue
        if not hasattr(grp, "descs"):                   # BigBatch / Seq launches (gemm_big): not grouped GEMMs
            continue
        row = {"group": name, "nprob": grp.n, "gflop": round(2.0 * grp.macs(seg_host) / 1e9, 4)}
        for kern in ["tile", "lat"] + [f"tile_cap{c}" for c in caps]:
            try:
                descs = [type(d).from_buffer_copy(d) for d in grp.descs]
                if kern.startswith("tile_cap"):
                    g2 = H.GemmGroup(descs, dev, eng.dt, seg=grp.seg, kernel="tile", kt_cap=int(kern[8:]))
                else:
                    g2 = H.GemmGroup(descs, dev, eng.dt, seg=grp.seg, kernel=kern)
            except ValueError:
                continue
            with torch.cuda.stream(s):
                for _ in range(3):
                    g2()
                torch.cuda.synchronize()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=s):
                    for _ in range(reps):
                        g2()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            graph.replay()
            torch.cuda.synchronize()
            e0.record(s)
            with torch.cuda.stream(s):
                graph.replay()
            e1.record(s)
            torch.cuda.synchronize()
            us = 1000.0 * e0.elapsed_time(e1) / reps
            row[kern] = {"us": round(us, 1), "tflops": round(row["gflop"] / us * 1e3, 2),
                         "tiles": g2.total, "ksplit_max": max(int(d.ksplit) for d in g2.descs)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
