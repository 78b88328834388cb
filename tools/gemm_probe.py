"""Per-group timing of the grouped f64 GEMM launches of one PM2.5-shaped DSVI step (GPU box).

Runs one real step (so every operand holds realistic data), then replays each GEMM group alone
`reps` times between HIP events on the engine's stream, and prints ms / GFLOP / TF/s per group
plus the tile and split-K counts.  Usage: python tools/gemm_probe.py [reps]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    verbose = "-v" in sys.argv
    import bench
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
    D, M, B = bench.D, bench.M, bench.B
    dev = torch.device("cuda", 0)
    xs, ys = bench.synth_data(0)
    model = NMGP(number_observations=D * bench.N_LOC, dim_outputs=D, Z=np.linspace(0, 1, M), minibatch_size=B,
                 seed=22, device=dev, noise="device")
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        getattr(model, k).data.fill_(-1.0)
        getattr(model, k).requires_grad = False
    trainer = DsviTrainer(model, lr=0.01)
    eng = model.engine(B)
    x, y, I, seg = bench.epoch_batches(xs, ys, np.random.default_rng(1))[0]
    sizes = np.diff(seg)
    eng.load_batch(x, y, sizes)
    trainer.grad_step(eng)
    torch.cuda.synchronize()
    total_ms, total_gf = 0.0, 0.0
    print(f"{'group':12s} {'probs':>5s} {'tiles':>6s} {'ms':>8s} {'GFLOP':>8s} {'TF/s':>7s}")
    for name, grp in eng.gemm_groups():
        # replay `reps` launches from a HIP graph: Python launch overhead (~10-20 us per ctypes call)
        # would otherwise hide every kernel shorter than that
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                grp()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                grp()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        gf = 2.0 * grp.macs(seg) / 1e9
        total_ms += ms
        total_gf += gf
        print(f"{name:12s} {len(grp.descs):5d} {grp.total:6d} {ms:8.4f} {gf:8.4f} {gf / ms:7.3f}")
        if verbose:
            shapes = {}
            for dd in grp.descs:
                segs = seg if dd.row_seg >= 0 or dd.k_seg >= 0 else None
                m = int(segs[dd.row_seg + max(dd.seg_span, 1)] - segs[dd.row_seg]) if dd.row_seg >= 0 else dd.m
                k = int(segs[dd.k_seg + max(dd.seg_span, 1)] - segs[dd.k_seg]) if dd.k_seg >= 0 else dd.k
                key = (m, dd.n, k, dd.kbA, dd.kbB, dd.flags, dd.ksplit, int(dd.sA_k == 1), int(dd.sB_j == 1))
                shapes[key] = shapes.get(key, 0) + 1
            for key, c in sorted(shapes.items(), key=lambda t: -t[0][0] * t[0][1] * t[0][2] * t[1]):
                print(f"    {c:3d} x m={key[0]} n={key[1]} k={key[2]} kbA={key[3]} kbB={key[4]} flags={key[5]} "
                      f"ksplit={key[6]} a_kc={key[7]} b_jc={key[8]}")
    print(f"{'TOTAL':12s} {'':5s} {'':6s} {total_ms:8.4f} {total_gf:8.4f} {total_gf / total_ms:7.3f}")


if __name__ == "__main__":
    main()
