"""Benchmark: DSVI iterations/s on the PM2.5-shaped config (BASELINE.json configs[1]).

One step = one DSVI iteration of the reference training loop (code/nmgp_dsvi.py:829-863):
device Philox noise -> fused closed-form forward/backward (all 13 gradients) -> Adam, on a
minibatch of B = 2000 rows drawn from N = 10,000 synthetic observations (2,000 locations x
D = 5 outputs, M = 256 inducing points, fp64).  The step is replayed as one HIP graph.
Multi-GPU (torchrun): each rank draws its own minibatch from its own shard, gradients are
averaged with one RCCL all-reduce, every rank applies the same Adam update (weak scaling:
value = minibatch iterations per second summed over ranks).

Prints ONE JSON line (rank 0).  Also reports the per-phase breakdown, the roofline of the
dominant kernel (the grouped MFMA GEMM) and the CPU baseline (the oracle, op for op the
reference's torch-CPU path, timed on this host's cores).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

D, M, N_LOC, B = 5, 256, 2000, 2000
FP64_MFMA_PEAK_TFLOPS = 78.6          # MI355X dense FP64 matrix peak (spec)
HBM_PEAK_GBS = 8000.0
sys.path.insert(0, os.path.join(ROOT, "tools"))
from provenance import code_hash  # noqa: E402

CODE_HASH = code_hash()


def matched_profile(pattern):
    """The committed profile (profiles/<pattern>) measured on THIS code: the newest file whose code_hash
    (tools/provenance.py, written by the summary tools on the GPU box) equals the running tree's.  Without one
    the newest file is returned with stale=True, and every figure taken from it is marked stale in the line."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    data = []
    for f in files:
        try:
            data.append((f, json.load(open(f))))
        except (OSError, ValueError):
            continue
    for f, d in reversed(data):
        if isinstance(d, dict) and d.get("code_hash") == CODE_HASH:
            return os.path.relpath(f, ROOT), d, False
    if data:
        return os.path.relpath(data[-1][0], ROOT), data[-1][1], True
    return None, None, True


def synth_data(rank):
    """PM2.5-shaped synthetic data: all 5 outputs observed at 2,000 locations."""
    rng = np.random.default_rng(1000 + rank)
    xs = [np.sort(rng.uniform(0, 1, N_LOC)) for _ in range(D)]
    ys = [rng.standard_normal(N_LOC) for _ in range(D)]
    return xs, ys


def epoch_batches(xs, ys, rng):
    """One epoch of DataLoader(shuffle=True) minibatches, each split per output like vec2list."""
    X = np.concatenate(xs)
    Y = np.concatenate(ys)
    I = np.concatenate([np.full(len(x), d) for d, x in enumerate(xs)])
    perm = rng.permutation(len(X))
    out = []
    for s in range(0, len(X) - B + 1, B):
        idx = perm[s:s + B]
        idx = idx[np.argsort(I[idx], kind="stable")]        # vec2list order: grouped by output
        seg = np.concatenate([[0], np.cumsum(np.bincount(I[idx], minlength=D))]).astype(np.int32)
        out.append((X[idx], Y[idx], I[idx].astype(np.int32), seg))
    return out


def stress_cholesky(dev, reps=5):
    """BASELINE.json configs[4] beside the headline: one SPD M=4096 fp32 matrix (A = G G^T / M + I,
    G ~ N(0,1), seed 0) factored by the blocked right-looking potrf (nmgp_potrf_blocked_f32), and its
    dominant kernel -- the trailing-update SYRK on the 128x128 f32 MFMA kernel -- timed alone at
    n = k = 4096.  GFLOP/s counts M^3/3 for the factorization and n(n+1)k for the SYRK (lower half).
    The CPU figure is torch.linalg.cholesky (LAPACK spotrf: what the reference calls through
    torch.cholesky, code/utils.py:40) on this host's cores."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    Mst = 4096
    g = torch.Generator(device=dev).manual_seed(0)
    G = torch.randn(Mst, Mst, generator=g, dtype=torch.float64, device=dev)
    A0 = (G @ G.t() / Mst + torch.eye(Mst, dtype=torch.float64, device=dev)).float().contiguous()
    W = A0.clone()
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        W.copy_(A0)
        H.potrf_blocked_(W, info=info)
    torch.cuda.current_stream().wait_stream(s)

    def graph_ms(body, n=reps):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(n):
                body()
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    def fac():
        W.copy_(A0)
        H.potrf_blocked_(W, info=info)

    t_fac = graph_ms(fac)
    assert int(info.item()) == 0, "stress potrf reported a non-positive pivot"
    idx = torch.arange(0, Mst, 16, device=dev)
    Ld = W.double()
    resid = float((Ld[idx] @ Ld.t() - A0.double()[idx]).norm() / A0.double()[idx].norm())
    del Ld
    t_fac -= graph_ms(lambda: W.copy_(A0))     # the per-rep restore copy is not factorization time
    # the trailing-update SYRK alone at n = k = 4096 (stream-K over the lower tiles)
    X = (torch.rand(Mst, Mst, generator=g, device=dev) * 2 - 1)
    C = torch.zeros(Mst, Mst, device=dev)
    ws = H.big_workspace(dev, L.lib().nmgp_gemm_big_workspace_size())
    t_syrk = graph_ms(lambda: H.gemm_big(X, X, C, flags=L.OUT_LOWER, alpha=-1.0, beta=1.0, ws=ws), n=20)
    syrk_tf = Mst * (Mst + 1.0) * Mst / (t_syrk * 1e-3) / 1e12
    del G, X, C
    # CPU: LAPACK spotrf through torch on the host cores, one call (about 0.1-1 s)
    Ac = A0.cpu()
    torch.linalg.cholesky(Ac[:512, :512])
    t0 = time.time()
    torch.linalg.cholesky(Ac)
    t_cpu = time.time() - t0
    f = Mst ** 3 / 3.0
    return {"workload": "stress: one SPD M=4096 fp32 matrix (BASELINE.json configs[4])",
            "kernel": "nmgp_potrf_blocked_f32 (128-wide fused leaves; 32-row panel + lookahead step kernel; "
                      "side stream: 32-row strip of block column j+2, then the trailing SYRK)",
            "potrf_ms": round(t_fac, 4), "gflops": round(f / (t_fac * 1e-3) / 1e9, 1),
            "residual": resid,
            "hbm": _stress_hbm(t_fac),
            "syrk_in_factorization": _stress_syrk_pmc(),
            "syrk_in_ecog_factorization": _ecog_syrk_pmc(),
            "syrk_isolated_proxy": {"kernel": "gemm_big_kernel (128x128 f32 MFMA, stream-K)", "n": Mst, "k": Mst,
                                    "ms": round(t_syrk, 4), "achieved_tflops": round(syrk_tf, 2), "peak_tflops": 157.3,
                                    "frac": round(syrk_tf / 157.3, 4),
                                    "note": "a fresh n = k = 4096 SYRK, NOT an update the factorization issues"},
            "cpu": {"potrf_ms": round(1e3 * t_cpu, 2), "gflops": round(f / t_cpu / 1e9, 1),
                    "cores": torch.get_num_threads(), "kind": "torch.linalg.cholesky (LAPACK spotrf)"},
            "speedup_vs_cpu": round(t_cpu * 1e3 / t_fac, 1)}


def kron_mv_leg(dev, P=5, N=8192, reps=20):
    """The Kronecker mat-vec of the legacy Kronecker likelihood (SIM_code/Utility/kronecker_operation.py:72-85,
    distributions.py:26-52): (B kron K) y with B (P x P), K (N x N), fp64, on the fused one-pass kernel
    (csrc/kron.hip kron_mv_kernel).  HBM-bound: algorithmic bytes per call = 8 (N^2 + P N + P^2 + P N) --
    K read once, y read, out written.  Timed with HIP events around a graph of `reps` launches on the
    stream they run on."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H
    g = torch.Generator(device=dev).manual_seed(3)
    Bm = torch.randn(P, P, generator=g, dtype=torch.float64, device=dev)
    K = torch.randn(N, N, generator=g, dtype=torch.float64, device=dev)
    y = torch.randn(P * N, generator=g, dtype=torch.float64, device=dev)
    out = torch.empty(P * N, dtype=torch.float64, device=dev)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        H.kron_mv(Bm, K, y, out=out)
    torch.cuda.current_stream(dev).wait_stream(s)
    gr = H.HipGraph(dev)
    with gr.capture():
        for _ in range(reps):
            H.kron_mv(Bm, K, y, out=out)
    with torch.cuda.stream(s):
        gr.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        gr.replay()
        e1.record(s)
    torch.cuda.synchronize(dev)
    us = 1000.0 * e0.elapsed_time(e1) / reps
    ref = torch.kron(Bm[:2, :2].cpu(), K[:64, :64].cpu()) @ torch.cat([y[:64], y[N:N + 64]]).cpu()
    chk = H.kron_mv(Bm[:2, :2].contiguous(), K[:64, :64].contiguous(), torch.cat([y[:64], y[N:N + 64]])).cpu()
    nbytes = 8.0 * (N * N + P * N + P * P + P * N)
    gbs = nbytes / (us * 1e-6) / 1e9
    del K
    return {"workload": f"kron_mv: (B kron K) y, B {P}x{P}, K {N}x{N}, fp64 (legacy Kronecker likelihood)",
            "kernel": "kron_mv_kernel<double, 2> (one pass over K, 16-byte rows, DPP wave reductions)",
            "us_per_call": round(us, 2), "algorithmic_bytes": int(nbytes), "achieved_GBs": round(gbs, 1),
            "peak_GBs": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4), "bound": "hbm",
            "check_rel_err": float((chk - ref).norm() / ref.norm())}


def _stress_syrk_pmc():
    """MFMA-busy of the trailing-update SYRK launches INSIDE the M=4096 factorization (k = 128), time-weighted,
    from the committed rocprofv3 PMC pass (tools/syrk_inside_pmc.sh: SQ_VALU_MFMA_BUSY_CYCLES /
    (GRBM_GUI_ACTIVE/8 * 4 * 256), one pass, no tracing domains) and the whole factorization's."""
    src, d, stale = matched_profile("r*_stress_potrf_mfma_util.json")
    if d is None:
        return None
    rows = d["rows"]
    nm = lambda r: r["kernel"]
    syrk = [r for r in rows if "gemm_big_kernel" in nm(r)]
    fac = [r for r in rows if any(k in nm(r) for k in ("gemm_big_kernel", "potrf_step", "potrf_strip", "chol_inv"))]
    tw = lambda rs: sum(r["mfma_util"] * r["avg_us"] * r["dispatches"] for r in rs) / max(
        1e-9, sum(r["avg_us"] * r["dispatches"] for r in rs))
    return {"kernel": "gemm_big_kernel (the factorization's own trailing SYRKs, k = 128)",
            "launches": sum(r["dispatches"] for r in syrk), "mfma_busy_time_weighted": round(tw(syrk), 4),
            "factorization_kernels_mfma_busy": round(tw(fac), 4), "source": src, "stale": stale}


def _stress_hbm(potrf_ms):
    """HBM traffic of one stress factorization from the committed FETCH_SIZE / WRITE_SIZE passes
    (tools/stress_hbm.sh; FETCH x2 per the gfx950 note + WRITE) over the factorization time measured here,
    beside the algorithmic bytes (A read once, L written once: 2 M^2 4 B)."""
    src, d, stale = matched_profile("r*_stress_potrf_hbm.json")
    alg = 2.0 * 4096 * 4096 * 4
    out = {"algorithmic_bytes": int(alg), "algorithmic_GBs": round(alg / (potrf_ms * 1e-3) / 1e9, 1),
           "peak_GBs": HBM_PEAK_GBS}
    if d is not None:
        t = d["traffic_bytes"]
        out.update({"traffic_bytes": t, "read_bytes_x2corrected": d["read_bytes_x2corrected"],
                    "write_bytes": d["write_bytes"], "achieved_GBs": round(t / (potrf_ms * 1e-3) / 1e9, 1),
                    "frac": round(t / (potrf_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "source": src, "stale": stale})
    return out


# ECoG batched recursive Cholesky of the 8384 M = 1024 variational factors (chol.hip chol_inv_rec_big): its trailing
# SYRKs A22 -= L21 L21^T per recursion level, identified by grid (threads = 256 x lower tiles x 8384 factors, or
# twice that for the 8-wave tiles)
ECOG_SYRK_LEVELS = [("top, n2 = 512, k = 512 (10 lower tiles)", 21463040, 1.0),
                    ("level 2, n2 = 256, k = 256 (3 lower tiles)", 6438912, 1.0),
                    # one-tile k = 128 products of this template share a grid: the L21 panel and the SYRK, equal
                    # shapes (the inverse product X21 = -X22 T reads T row-major since round 5: another template)
                    ("level 3, n2 = 128, k = 128 (1 tile; 1 of the 2 one-tile products of the grid)", 2146304, 1 / 2.)]


def _ecog_syrk_pmc():
    """MFMA-busy of the trailing-update SYRKs inside the batched recursive Cholesky of the ECoG-shaped step
    (BASELINE.json configs[3]: 8384 variational factors of M = 1024), from the committed PMC pass of one
    training step (tools/syrk_inside_pmc.sh -> profiles/r*_ecog_step_mfma_util.json): the top level and every
    level, time-weighted."""
    src, d, stale = matched_profile("r*_ecog_step_mfma_util.json")
    if d is None:
        return None
    lev = []
    for label, grid, share in ECOG_SYRK_LEVELS:
        # (4-wave launches: 256 threads per tile, 8-wave launches from round 5: 512)
        rs = [r for r in d["rows"] if r["kernel"].startswith("void nmgp::gemm_big_kernel<true, true, 0")
              and r["grid_threads"] in (grid, 2 * grid)]
        if rs:
            us = sum(r["avg_us"] * r["dispatches"] for r in rs)
            lev.append({"level": label, "us_total": round(us * share, 1),
                        "mfma_busy": round(sum(r["mfma_util"] * r["avg_us"] * r["dispatches"] for r in rs) / us, 4)})
    if not lev:
        # persistent batched launches (round 5) share one grid (2 workgroups per CU) whatever the level, so the
        # levels cannot be told apart by grid: report the time-weighted MFMA-busy over every launch of the
        # recursion's k-contiguous template -- the trailing SYRKs AND the L21 panel products of all levels
        rs = [r for r in d["rows"] if r["kernel"].startswith("void nmgp::gemm_big_kernel<true, true, 0")]
        if not rs:
            return None
        us = sum(r["avg_us"] * r["dispatches"] for r in rs)
        busy = round(sum(r["mfma_util"] * r["avg_us"] * r["dispatches"] for r in rs) / us, 4)
        return {"kernel": "gemm_big_kernel (batched trailing SYRKs A22 -= L21 L21^T and L21 panels of the recursive "
                          "Cholesky of 8384 M=1024 factors, persistent launches)",
                "mfma_busy_time_weighted": busy, "mfma_busy_all_levels_time_weighted": busy,
                "mfma_busy_top_level_k512": None,
                "levels": [{"level": "all levels, SYRK + L21 panel launches (one grid for every level)",
                            "us_total": round(us, 1), "mfma_busy": busy,
                            "dispatches": sum(r["dispatches"] for r in rs)}],
                "source": src, "stale": stale}
    w = sum(x["us_total"] for x in lev)
    return {"kernel": "gemm_big_kernel (batched trailing SYRK A22 -= L21 L21^T of 8384 M=1024 factors)",
            "mfma_busy_time_weighted": lev[0]["mfma_busy"], "mfma_busy_top_level_k512": lev[0]["mfma_busy"],
            "mfma_busy_all_levels_time_weighted": round(sum(x["mfma_busy"] * x["us_total"] for x in lev) / w, 4),
            "levels": lev, "source": src, "stale": stale}


def api_path(dev, xs, ys, z, epochs_device=100, epochs_torch=20):
    """The same PM2.5 workload through the reference's entry point, nmgp_dsvi.inference().

    noise="device": the on-device input pipeline (loader permutation -> HBM index gather -> one HIP
    graph per step, Cholesky info checked every 64 steps); noise="torch": the reference's RNG stream,
    host DataLoader + vec2list + a PCIe copy and a host sync per step.  Rate = steps between the end of
    the first epoch and the last step / their device-event time span (time_list).  Not `value`.
    """
    import contextlib
    import io
    from collaborative_nonstationary_multivariate_gaussian_process_amd import nmgp_dsvi
    out = {"workload": "nmgp_dsvi.inference() on the bench data (D=5, N=10,000, M=256, batch_size=2000, "
                       "length-scale logs frozen at -1 as in the timed loop)"}
    hyper = {k: -1.0 for k in ("length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log")}
    for noise, epochs in (("device", epochs_device), ("torch", epochs_torch)):
        with contextlib.redirect_stdout(io.StringIO()):
            _, losses, tl = nmgp_dsvi.inference(xs, ys, z, B, D, hyperpars=hyper, itnum=epochs, show_ELBO=False,
                                                noise=noise, device=dev, seed=22)
        per_epoch = len(tl) // epochs
        span = tl[-1] - tl[per_epoch - 1]
        out[noise] = {"epochs": epochs, "steps": len(tl), "it_per_s": round((len(tl) - per_epoch) / span, 2),
                      "final_loss": float(losses[-1])}
    # the reference's published PM2.5 workload (RMSE-vs-time charts): training with predict_Y on held-out
    # test inputs after EVERY iteration (code/nmgp_dsvi.py:865-868), 200 test points per output
    rng = np.random.default_rng(77)
    xt = [np.sort(rng.uniform(0, 1, 200)) for _ in range(D)]
    yt = [rng.standard_normal(200) for _ in range(D)]
    epochs = epochs_device // 2
    with contextlib.redirect_stdout(io.StringIO()):
        _, losses, rmse, tl = nmgp_dsvi.inference(xs, ys, z, B, D, hyperpars=hyper, itnum=epochs, show_ELBO=False,
                                                  noise="device", device=dev, seed=22,
                                                  X_test_list=[x[:, None] for x in xt], Y_test_list=[y[:, None] for y in yt])
    per_epoch = len(tl) // epochs
    span = tl[-1] - tl[per_epoch - 1]
    out["device_with_predict_Y"] = {"epochs": epochs, "steps": len(tl), "test_points": D * 200,
                                    "it_per_s": round((len(tl) - per_epoch) / span, 2),
                                    "final_loss": float(losses[-1]), "final_test_rmse": float(rmse[-1])}
    return out


def elbo_sharded(dev, world, rank, dist, D=128, M=1024, rows=391, samples=64):
    """North-star's sample-sharded ELBO (BASELINE.json configs[3], ECoG-full shape): compute_ELBO over all
    N = D * rows observations with `samples` Monte-Carlo samples split round-robin over the ranks
    (rank r runs samples r, r + W, ...; one scalar all-reduce; the owner of the last sample adds the KL
    terms).  fp32, packed Q-pair layout, device Philox noise.  Timed after one warm-up call, barrier +
    synchronize on both sides, max over ranks."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP
    rng = np.random.default_rng(7)
    xs = [torch.from_numpy(np.sort(rng.uniform(0, 1, rows))) for _ in range(D)]
    ys = [torch.sin(6 * x + 0.1 * d) + 0.3 * torch.from_numpy(rng.standard_normal(rows)) for d, x in enumerate(xs)]
    m = NMGP(number_observations=D * rows, dim_outputs=D, Z=np.linspace(0, 1, M), seed=22, device=dev,
             noise="device", dtype=torch.float32, pair_layout="packed")
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        getattr(m, k).data.fill_(float(np.log(3.0 / M)))
    m.compute_ELBO(xs, ys, n_sample=world, distributed=world > 1)          # warm-up: plans, first launches
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.time()
    e = m.compute_ELBO(xs, ys, n_sample=samples, distributed=world > 1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.time() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    out = {"workload": f"compute_ELBO, ECoG-full shape D={D} (Q={D * (D + 1) // 2} pairs), M={M}, N={D * rows}, fp32, "
                       f"{samples} MC samples sharded over {world} rank(s)",
           "samples": samples, "ranks": world, "seconds": round(el, 4), "samples_per_s": round(samples / el, 3),
           "elbo": float(e), "peak_mem_GB": round(torch.cuda.max_memory_allocated(dev) / 1e9, 1)}
    del m
    import gc
    gc.collect()                  # the engines' launch schedules hold reference cycles: free the 235 GB now
    torch.cuda.empty_cache()
    return out


FP32_MFMA_PEAK_TFLOPS = 157.3         # MI355X dense FP32 matrix peak (spec)


def train_setup(dev, cfg):
    """Model, trainer and engine of one fp32 training configuration (graph_train below; tools/gemm_group_probe.py
    --cfg): synthetic rows, the epoch's minibatches bound in HBM (device gather + Philox noise per step)."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
    Dc, n, Mc, Bc, fwd_gflop = TRAIN_CFGS[cfg]
    rng = np.random.default_rng(2024)
    xs = [np.arange(n) / n if cfg == "hcp" else np.sort(rng.uniform(0, 1, n)) for _ in range(Dc)]
    ys = [np.sin(6 * x + 0.1 * d) + 0.3 * rng.standard_normal(n) for d, x in enumerate(xs)]
    m = NMGP(number_observations=Dc * n, dim_outputs=Dc, Z=np.linspace(0, 1, Mc), minibatch_size=Bc, seed=22,
             device=dev, noise="device", dtype=torch.float32, pair_layout="packed")
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        getattr(m, k).data.fill_(float(np.log(3.0 / Mc)))
        getattr(m, k).requires_grad = False
    tr = DsviTrainer(m, lr=0.01)
    eng = m.engine(Bc)
    X, Y = np.concatenate(xs), np.concatenate(ys)
    I = np.repeat(np.arange(Dc), n)
    perm = rng.permutation(len(X))
    bx, by, bi, bs = [], [], [], []
    for s in range(min(len(X) // Bc, 8)):
        idx = perm[s * Bc:(s + 1) * Bc]
        idx = idx[np.argsort(I[idx], kind="stable")]
        bx.append(X[idx]); by.append(Y[idx]); bi.append(I[idx])
        bs.append(np.concatenate([[0], np.cumsum(np.bincount(I[idx], minlength=Dc))]))
    f = lambda a, t: torch.tensor(np.stack(a), dtype=t, device=dev)
    eng.bind_dataset(f(bx, torch.float32), f(by, torch.float32), f(bi, torch.int32), f(bs, torch.int32))
    return m, tr, eng


TRAIN_CFGS = {"hcp": (50, 10000, 512, 5000, 263.0), "ecog": (128, 391, 1024, 512, 6150.0)}


def train_roofline(eng, cfg):
    """Roofline of an fp32 training step (BASELINE configs[2] / [3]) for the kernel FAMILY with the most busy time
    in the committed rocprofv3 breakdown of the graphed step (profiles/r*_{cfg}_train_kernels.json from
    tools/train_trace.sh, code-hash matched): every template instance of one kernel counts as one family.
      gemm_big_kernel (128x128 f32): the batched factor products -- Sigma_f = tril(S) tril(S)^T (syrk_side),
        Xs = C^-1 L (xs_side), the KL L-bar -C^-T Xs (kl_lbar), the pair / latent L-bar P^T W-hat (bwd_lbar) and
        the GEMMs of the recursive factor + inverse of every variational factor (chol_side);
      gemm_kernel<float> (grouped 64x64 f32): the row-segmented quad-form / P-bar products.
    Algorithmic flops per step = 2 x multiply-adds over the launches of that family (triangular zeros, skipped
    output halves and padding not counted; row / k segments of this minibatch), over the family's busy time
    per step (sum of its launch durations: concurrent streams overlap, so this is conservative)."""
    seg_host = eng.seg.cpu().numpy()
    # family -> [GFLOP, group names, launches, algorithmic bytes] per step
    fams = {"gemm_big_kernel": [0.0, [], 0, 0], "gemm_kernel<float": [0.0, [], 0, 0]}
    for nm, grp in eng.gemm_groups():
        parts = grp.parts if hasattr(grp, "parts") else [grp]
        for p_ in parts:
            if isinstance(p_, H_BigBatch()):
                f = fams["gemm_big_kernel"]
            elif hasattr(p_, "macs") and not getattr(p_, "lat", False) and p_.dtype == torch.float32:
                f = fams["gemm_kernel<float"]
            else:
                continue
            f[0] += 2.0 * p_.macs(seg_host) / 1e9
            f[1].append(nm)
            f[2] += 1
            f[3] += p_.algo_bytes(seg_host)
    from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H
    kf0, kf1 = eng._plan(0)["kl_range"]
    if eng.M > 256:      # chol_side: recursive factor + inverse of the variational factors on gemm_big
        fams["gemm_big_kernel"][0] += (kf1 - kf0) * 2.0 * H.chol_inv_rec_macs(eng.M) / 1e9
        fams["gemm_big_kernel"][3] += (kf1 - kf0) * H.chol_inv_rec_bytes(eng.M)
        fams["gemm_big_kernel"][1].append("chol_side (recursive factor + inverse GEMMs)")
    src, d, stale = matched_profile(f"r*_{cfg}_train_kernels.json")
    tsrc, td, tstale = matched_profile(f"r*_{cfg}_train_traffic.json")
    busy = {}
    if d is not None:
        for r in d["kernels"]:
            for fam in fams:
                if r["kernel"].startswith(fam):
                    b_ = busy.setdefault(fam, [0.0, 0.0, 0.0])
                    b_[0] += r["ms_per_step"]
                    b_[1] += r["share_of_busy"]
                    b_[2] += r["launches_per_step"]
    lines = {}
    for fam, (gf, names, n, abytes) in fams.items():
        e = {"kernel": fam + ("> (grouped 64x64 MFMA f32 GEMM)" if fam.startswith("gemm_kernel")
                              else " (128x128 MFMA f32, batched factor products)"),
             "bound": "mfma", "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
             "algorithmic_gflop_per_step": round(gf, 3), "groups": sorted(set(names)), "traffic": None,
             # each product's operands read once and its output written once (structural zeros not counted):
             # hip_ops.desc_bytes / BigBatch.algo_bytes / chol_inv_rec_bytes
             "algorithmic_bytes": int(abytes), "algorithmic_bytes_unit": "bytes/step"}
        if fam in busy:
            ms, share, launches = busy[fam]
            ach = gf / ms                                   # GFLOP / ms = TFLOP/s
            e.update({"profile_launches_per_step": launches, "source": src, "stale": stale,
                      "in_graph_overlapped": {
                          "ms_per_step": round(ms, 4), "share_of_busy": round(share, 4), "achieved": round(ach, 3),
                          "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
                          "timing": "rocprofv3 --kernel-trace busy time of the family per graphed step (streams "
                                    "overlap: a launch's time includes waits for CUs other streams hold)"}})
            e["achieved"], e["frac"] = e["in_graph_overlapped"]["achieved"], e["in_graph_overlapped"]["frac"]
            e["timing"] = e["in_graph_overlapped"]["timing"]
        if tsrc is not None and fam in td.get("families", {}):
            # HBM traffic of the family per step from the FETCH / WRITE PMC passes (tools/train_pmc.sh)
            tf_ = td["families"][fam]
            tb = tf_["traffic_bytes_per_step"]
            e.update({"traffic": tb, "traffic_unit": "bytes/step (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                      "traffic_source": tsrc, "traffic_stale": tstale,
                      "traffic_ratio": round(tb / abytes, 3) if abytes else None})
            ser = tf_.get("serialised_ms_per_step")
            if ser:
                # the line's achieved / frac: the family's own kernel time, dispatches serialised by the PMC pass
                ach = gf / ser
                e.update({"serialised_ms_per_step": ser, "achieved": round(ach, 3),
                          "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
                          "timing": "rocprofv3 PMC (FETCH_SIZE) pass of the graphed step: the family's dispatch "
                                    "durations, serialised by counter collection"})
            if fam in busy:
                e["traffic_GBs_over_busy_time"] = round(tb / (busy[fam][0] * 1e-3) / 1e9, 1)
        lines[fam] = e
    top = max(lines, key=lambda f: busy.get(f, [0.0])[0]) if busy else "gemm_big_kernel"
    out = dict(lines[top])
    out["other_family"] = [lines[f] for f in lines if f != top][0]
    out["dominant_by"] = "busy time per step in " + (src or "(no profile)")
    return out


def H_BigBatch():
    from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H
    return H.BigBatch


def graph_train(dev, cfg, steps, warmup=2):
    """A training configuration of BASELINE.json beside the headline (one GPU, fp32, graph-replayed steps,
    the epoch's minibatches resident in HBM, device Philox noise, Adam inside the graph):
      hcp  configs[2]: D=50 outputs x 10,000 timepoints (500k rows), M=512, B=5000, length scales 3/M;
      ecog configs[3]: D=128 channels x 391 rows (N=50,048), M=1024, B=512, length scales 3/M.
    Packed pair layout (the pairs are initialised on the device; HCP's dense layout runs the same kernels
    at the same speed).  Step TFLOP/s uses SURVEY §8d's algorithmic forward FLOPs x 3 (backward ~ 2x
    forward): HCP 263 GFLOP, ECoG 6.15 TFLOP forward per step."""
    import gc
    Dc, n, Mc, Bc, fwd_gflop = TRAIN_CFGS[cfg]
    torch.cuda.reset_peak_memory_stats(dev)
    t0 = time.time()
    m, tr, eng = train_setup(dev, cfg)
    g = tr.capture(eng, include_update=True)
    t_setup = time.time() - t0
    for _ in range(warmup):
        g.replay()
    torch.cuda.synchronize()
    m.check_numerics()
    t0 = time.time()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    el = (time.time() - t0) / steps
    m.check_numerics()
    loss = float(eng.out[0])
    tf = 3.0 * fwd_gflop / 1e3 / el
    roof = train_roofline(eng, cfg)
    out = {"workload": f"{cfg.upper()}-shaped training step (BASELINE.json configs[{2 if cfg == 'hcp' else 3}]): D={Dc}, "
                       f"Q={Dc * (Dc + 1) // 2} pairs, M={Mc}, N={Dc * n}, B={Bc}, fp32, packed pairs, HIP graph",
           "steps": steps, "warmup": warmup, "s_per_step": round(el, 5), "it_per_s": round(1.0 / el, 3),
           "loss": loss, "loss_finite": bool(np.isfinite(loss)),
           "algorithmic_tflop_per_step": round(3.0 * fwd_gflop / 1e3, 4),
           "step_tflops": round(tf, 2), "peak_tflops": FP32_MFMA_PEAK_TFLOPS,
           "frac_of_fp32_peak": round(tf / FP32_MFMA_PEAK_TFLOPS, 4),
           "flop_convention": "SURVEY §8d: 3 x algorithmic forward FLOPs (backward ~ 2 x forward)",
           "setup_s": round(t_setup, 1), "params": int(m._theta.numel()),
           "peak_mem_GB": round(torch.cuda.max_memory_allocated(dev) / 1e9, 1), "roofline": roof}
    del g, tr, eng, m
    gc.collect()
    torch.cuda.empty_cache()
    return out


def pair_sharded_train(dev, world, rank, dist, D=128, M=1024, rows=391, B=512, steps=4):
    """SURVEY §8e axis 3 at the ECoG-full shape (BASELINE.json configs[3]): the training step with the
    coefficient pairs sharded over the ranks by output range (pair_shard.PairShard): each rank holds its
    pairs' parameters / Adam state / factors, draws b_r = B N_r / N rows of its outputs, and the
    replicated gradient (mu_W, sqrt_W, mu_v, sqrt_v, hyper-parameters) is summed with one RCCL
    all-reduce per step.  fp32; each rank's rows resident in HBM, one on-device minibatch gather per step,
    the rank-local step and Adam replayed as HIP graphs around the all-reduce (PairShard.bind_rows /
    capture); timed over `steps` steps after one warm-up step,
    barrier + synchronize on both sides, max over ranks.  A rank that fails to build its share makes
    every rank skip the leg (flag all-reduce) instead of leaving the others in a collective."""
    import gc
    from collaborative_nonstationary_multivariate_gaussian_process_amd.pair_shard import PairShard, pair_shard_ranges
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import pair_window
    ok = torch.ones(1, device=dev)
    sh, err = None, None
    try:
        ranges = pair_shard_ranges(D, world)
        i0, i1 = ranges[rank]
        q0, Q = pair_window(D, (i0, i1))
        g = torch.Generator(device=dev).manual_seed(100 + rank)
        rn = lambda *s: torch.randn(*s, generator=g, device=dev, dtype=torch.float32)
        # replicated parameters drawn from one seed on every rank; the pair window from the rank's own
        gr = torch.Generator(device=dev).manual_seed(99)
        rr = lambda *s: torch.randn(*s, generator=gr, device=dev, dtype=torch.float32)
        ls = float(np.log(3.0 / M))
        p = {"mu_W": 0.1 * rr(D, M), "sqrt_W": 0.1 * rr(D, M, M), "mu_v": -4 * torch.ones(M, device=dev),
             "sqrt_v": 0.1 * rr(M, M), "mu_U": 0.1 * rn(Q, M), "sqrt_U": 0.1 * rn(Q, M, M),
             "sigma2_tildeell_log": torch.tensor(0.), "length_scales_tildeell_log": torch.tensor(ls),
             "sigma2_L0_log": torch.tensor(0.), "length_scales_L0_log": torch.tensor(ls),
             "sigma2_L1_log": torch.tensor(0.), "length_scales_L1_log": torch.tensor(ls), "sigma2_err_log": torch.tensor(-2.)}
        rng = np.random.default_rng(7)
        xs = [np.sort(rng.uniform(0, 1, rows)) for _ in range(D)]
        ys = [np.sin(6 * x + 0.1 * d) + 0.3 * rng.standard_normal(rows) for d, x in enumerate(xs)]
        N = D * rows
        n_r = rows * (i1 - i0)
        b_r = max(1, int(round(B * n_r / N)))
        sh = PairShard(p, np.linspace(0, 1, M), B_r=b_r, N_r=n_r, rank=rank, world=world, dtype=torch.float32,
                       device=dev, frozen=("length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"),
                       ranges=ranges, pairs_local=True)
        del p
        # the rank's rows stay in HBM; each step gathers its minibatch on the device and replays as HIP graphs
        nb = sh.bind_rows(xs[i0:i1], ys[i0:i1], seed=5)
        sh.capture()
    except Exception as exc:                      # e.g. out of memory on a small world
        ok.zero_()
        err = f"{type(exc).__name__}: {exc}"[:300]
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if float(ok) == 0:
        sh = None
        gc.collect()
        torch.cuda.empty_cache()
        return {"error": err or "another rank could not build its share"}
    sh.step()                                     # warm-up: first replays
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.time()
    for it in range(steps):
        if (it + 1) % nb == 0:
            sh.new_epoch()
        loss = sh.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = (time.time() - t0) / steps
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    sh.check()
    out = {"workload": f"DSVI training step, ECoG-full shape D={D} (Q={D * (D + 1) // 2} pairs), M={M}, N={D * rows}, "
                       f"B={B}, fp32, pairs sharded over {world} rank(s) by output range",
           "ranges": pair_shard_ranges(D, world), "s_per_step": round(el, 4), "it_per_s": round(1.0 / el, 3),
           "loss": float(loss), "rank0_pairs": sh.Q, "rank0_param_GB": round(sh.theta.numel() * 4 / 1e9, 2),
           "replicated_allreduce_MB": round(sum(t.numel() for t in sh._rep) * 4 / 1e6, 1),
           "peak_mem_GB_rank0": round(torch.cuda.max_memory_allocated(dev) / 1e9, 1)}
    if D == 128 and M == 1024:
        # NOT measured in this run: the same step unsharded on one GPU (packed pairs, 247 GB peak), cited
        # from the committed profile (the N = 1 bench line measures it live, "ecog_train")
        out["ref_single_gpu_s_per_step_from_profile"] = {"value": 0.405, "source": "profiles/r02d_ecog_train.json"}
    del sh, loss
    gc.collect()
    torch.cuda.empty_cache()
    return out


class PhaseTimer:
    """HIP events around every launch of an eager step, recorded on the stream the kernel is launched on.
    concurrent=False: the step runs serially on one stream (isolated launch times); concurrent=True: on its
    four streams as in the graph (launch times under the same contention as the timed loop)."""

    def __init__(self, concurrent=False):
        self.rec = []
        self.cur = None
        self.concurrent = concurrent

    def start(self, name, kind, stream=None):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        self.cur = e

    def stop(self, name, kind, stream=None):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        self.rec.append((name, kind, self.cur, e))

    def summary(self, nsteps):
        torch.cuda.synchronize()
        per_name, per_kind = {}, {}
        for name, kind, a, b in self.rec:
            ms = a.elapsed_time(b)
            per_name[name] = per_name.get(name, 0.0) + ms / nsteps
            per_kind[kind] = per_kind.get(kind, 0.0) + ms / nsteps
        return per_name, per_kind


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds, xs, ys, z):
    """The oracle (reference op for op: per-pair LU solves, dense D x D Sigma_U, torch autograd,
    Adam) on the same PM2.5-shaped minibatch, on this host's cores; bounded to ~`seconds`."""
    from oracle import nmgp_oracle as O
    # the host cores this process may run on (on the GPU box: the job's CPU share; os.cpu_count()
    # reports the whole machine there), capped by OMP_NUM_THREADS when the launcher sets it
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    nthreads = max(1, min(avail, omp) if omp > 0 else avail)
    torch.set_num_threads(nthreads)
    p = O.new_params(D, M, seed=22)
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        p[k] = torch.tensor(-1.0, dtype=torch.float64)
    p = {k: v.clone().requires_grad_() for k, v in p.items()}
    frozen = {"length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"}
    rng = np.random.default_rng(7)
    batches = epoch_batches(xs, ys, rng)
    state = {}
    times = []
    t_start = time.time()
    it = 0
    while True:
        x, y, I, seg = batches[it % len(batches)]
        xl = [x[seg[d]:seg[d + 1]] for d in range(D)]
        yl = [y[seg[d]:seg[d + 1]] for d in range(D)]
        t0 = time.time()
        for v in p.values():
            v.grad = None
        loss, _ = O.forward(p, xl, yl, z, float(D * N_LOC), O.TorchNoise())
        loss.backward()
        O.adam_step(p, {k: v.grad for k, v in p.items() if k not in frozen}, state, 0.01)
        times.append(time.time() - t0)
        it += 1
        if it >= 2 and (time.time() - t_start > seconds or it >= 40):
            break
    steady = times[1:]
    # thread scaling of the same loop (short samples): where the oracle saturates below the job's share
    scan = {}
    for nt in sorted({t for t in (1, 4, 8) if t < nthreads}):
        torch.set_num_threads(nt)
        ts = []
        for k in range(4):
            x, y, I, seg = batches[k % len(batches)]
            xl = [x[seg[d]:seg[d + 1]] for d in range(D)]
            yl = [y[seg[d]:seg[d + 1]] for d in range(D)]
            t0 = time.time()
            for v in p.values():
                v.grad = None
            loss, _ = O.forward(p, xl, yl, z, float(D * N_LOC), O.TorchNoise())
            loss.backward()
            ts.append(time.time() - t0)
        scan[str(nt)] = round(1.0 / float(np.mean(ts[1:])), 3)
    scan[str(nthreads)] = round(1.0 / float(np.mean(steady)), 3)
    torch.set_num_threads(nthreads)
    return {"value": round(1.0 / float(np.mean(steady)), 4), "unit": "it/s", "cores": nthreads, "kind": "port",
            "thread_scan_it_per_s": scan,
            "cores_note": ("the GPU box gives one GPU's job a 16-core CPU share (OMP_NUM_THREADS=16 set by the "
                           "harness; os.cpu_count() reports the whole machine), so the baseline runs at that share; "
                           "thread_scan shows the oracle's scaling below it"),
            "cpu_model": _cpu_model(), "os_cpu_count": os.cpu_count(), "affinity_cpus": avail,
            "oracle_vs_reference": "oracle/reference CPU time 0.957 on the build container, interleaved medians "
                                   "(profiles/r02_cpu_oracle_vs_reference.json, tests/analysis/cpu_baseline_check.py)",
            "sample": f"{len(steady)} timed DSVI iterations (after 1 warm-up) of the oracle "
                      f"(torch-CPU fp64 restatement of code/nmgp_dsvi.py:157-301 + autograd + Adam) on the same "
                      f"D=5, M=256, B=2000 config; mean {1000 * float(np.mean(steady)):.1f} ms/it"}


def _relaunch_under_torchrun(n):
    """`python bench.py --gpus N` without a launcher: run the same command under torchrun with N ranks on
    127.0.0.1 as a child process (no exec: the parent has not touched the GPU, and never will)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-breakdown", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no HIP graph (launch every kernel from Python)")
    ap.add_argument("--no-stress", action="store_true", help="skip the M=4096 stress Cholesky line (configs[4])")
    ap.add_argument("--no-elbo", action="store_true", help="skip the sample-sharded ECoG compute_ELBO leg (configs[3])")
    ap.add_argument("--no-api", action="store_true", help="skip the inference() API-path leg")
    ap.add_argument("--no-hcp", action="store_true", help="skip the HCP-shaped training leg (configs[2])")
    ap.add_argument("--no-ecog", action="store_true", help="skip the ECoG-shaped training leg (configs[3])")
    ap.add_argument("--no-pair", action="store_true", help="skip the pair-sharded ECoG training leg (N > 1 only)")
    ap.add_argument("--no-kron", action="store_true", help="skip the Kronecker mat-vec leg")
    ap.add_argument("--pair-D", type=int, default=128, help="channels of the pair-sharded leg (default: ECoG-full 128)")
    ap.add_argument("--elbo-D", type=int, default=128, help="channels of the ELBO leg (default: ECoG-full 128)")
    ap.add_argument("--dp-allreduce", choices=["auto", "bucketed", "flat"], default="auto",
                    help="N > 1 gradient all-reduce: flat (auto: DsviTrainer.DP_BUCKET_MIN_BYTES unset) or bucketed + overlapped")
    args = ap.parse_args()

    # --gpus N is honoured before anything touches the GPU: without a launcher, N > 1 re-runs this
    # script under torchrun as a CHILD process (one rank per GPU) and exits with its status; under a
    # launcher whose WORLD_SIZE disagrees with N the run is refused instead of reporting the wrong N
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_relaunch_under_torchrun(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to report n_gpus={world}",
              file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one process per GPU (rank LOCAL_RANK on cuda:LOCAL_RANK, RCCL).  NMGP_DIST_BACKEND=gloo with more
    # ranks than devices is the rehearsal mode for a one-GPU box (ranks share cuda:0); never the
    # measured configuration.
    backend = os.environ.get("NMGP_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend != "nccl" and ndev > 0:
        local = local % ndev
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import param_layout

    xs, ys = synth_data(rank)
    z = np.linspace(0, 1, M)
    model = NMGP(number_observations=D * N_LOC, dim_outputs=D, Z=z, minibatch_size=B, seed=22, device=dev,
                 noise="device")
    model._noise_seed = 22 + 7919 * rank
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        getattr(model, k).data.fill_(-1.0)
        getattr(model, k).requires_grad = False
    trainer = DsviTrainer(model, lr=0.01)
    eng = model.engine(B)
    rng = np.random.default_rng(55 + rank)
    host_batches = epoch_batches(xs, ys, rng)
    nb = len(host_batches)
    Xb = torch.tensor(np.stack([b[0] for b in host_batches]), dtype=torch.float64, device=dev)
    Yb = torch.tensor(np.stack([b[1] for b in host_batches]), dtype=torch.float64, device=dev)
    Ib = torch.tensor(np.stack([b[2] for b in host_batches]), dtype=torch.int32, device=dev)
    Sb = torch.tensor(np.stack([b[3] for b in host_batches]), dtype=torch.int32, device=dev)

    # the epoch stays in HBM; every step starts with one on-device gather of the next minibatch
    batch_ctr = eng.bind_dataset(Xb, Yb, Ib, Sb)

    def load(bi):
        batch_ctr.fill_(bi)

    if world > 1:
        dist.broadcast(model._theta, 0)
    graph = None
    dp_bucketed = False
    if not args.eager:
        if world > 1:
            # gradient graph (with an external event node where the sqrt_W / sqrt_U rows are final) and the
            # 1/world + Adam graph; the bucketed RCCL all-reduce between them overlaps the backward's tail
            graph = trainer.capture_dp(eng, world, mode=args.dp_allreduce)[0]
            dp_bucketed = trainer.dp_bucketed(args.dp_allreduce)
        else:
            graph = trainer.capture(eng, include_update=True)

    def step(i):
        if graph is not None and world > 1:
            trainer.dp_graph_step(eng)                       # graph | overlapped bucketed all-reduce | update
        elif graph is not None:
            graph.replay()
        elif world > 1:
            trainer.dp_grad_step(eng)                        # eager: the same buckets, hooked on lbar_done
            trainer.update()
        else:
            trainer.grad_step(eng)
            trainer.update()

    for i in range(args.warmup):
        step(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.time()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.time() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    loss_val = float(eng.out[0])
    ms_per_step = 1000.0 * elapsed / args.steps
    value = world * args.steps / elapsed

    # ---------------------------------------------------------------- per-phase breakdown (eager)
    breakdown, roofline, chol = None, None, None
    if not args.no_breakdown:
        nrep = 10
        seg_host = host_batches[(nrep - 1) % nb][3]
        gemm_flops = 2.0 * sum(g.macs(seg_host) for _, g in eng.gemm_groups())

        def timed(concurrent):
            timer = PhaseTimer(concurrent=concurrent)
            for i in range(nrep):
                load(i % nb)
                trainer.grad_step(eng, timer=timer)
            per_name, per_kind = timer.summary(nrep)
            fam = {"lat": [0.0, 0.0, 0], "tile": [0.0, 0.0, 0]}     # flops, ms, launches per step
            by_launch = {}
            for nm, grp in eng.gemm_groups():
                if hasattr(grp, "macs") and nm in per_name:
                    gf = 2.0 * grp.macs(seg_host) / 1e9
                    by_launch[nm] = {"ms": round(per_name[nm], 4), "gflop": round(gf, 4),
                                     "kernel": "gemm_lat_kernel" if getattr(grp, "lat", False) else "gemm_kernel",
                                     "tflops": round(gf / per_name[nm], 2) if per_name[nm] > 0 else None}
                    f = fam["lat" if getattr(grp, "lat", False) else "tile"]
                    f[0] += gf * 1e9
                    f[1] += per_name[nm]
                    f[2] += 1
            return per_name, per_kind, fam, by_launch

        # the step's launches on its four streams as in the graph, each timed on its own stream: the
        # durations carry the same contention as the graphed timed loop (what rocprofv3 reports there)
        _, _, fam, _ = timed(True)
        # serially on one stream: the isolated per-launch breakdown
        per_name, per_kind, fam_iso, gemm_by_launch = timed(False)
        gemm_ms = per_kind.get("gemm", 0.0)
        n_gemm = sum(1 for it in eng._sched if len(it) > 1 and it[1] == "gemm")

        def fam_line(fm, key, label):
            fl, ms, n = fm[key]
            ach = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
            return {"kernel": label, "bound": "mfma", "achieved": round(ach, 4), "peak": FP64_MFMA_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(ach / FP64_MFMA_PEAK_TFLOPS, 5), "traffic": None,
                    "launches_per_step": n, "avg_launch_us": round(1000 * ms / max(n, 1), 2),
                    "algorithmic_gflop_per_step": round(fl / 1e9, 4),
                    "algorithmic_gflop_per_launch": round(fl / 1e9 / max(n, 1), 5)}

        def with_iso(key, label):
            line = fam_line(fam, key, label)
            iso = fam_line(fam_iso, key, label)
            line["timing"] = ("live HIP events on each launch's own stream, the step's four streams running "
                              "concurrently as in the graph (10 eager steps)")
            line["isolated"] = {"avg_launch_us": iso["avg_launch_us"], "achieved": iso["achieved"], "frac": iso["frac"],
                                "timing": "the same launches serialised on one stream"}
            return line
        # the dominant kernel by GPU time is the latency-oriented grouped GEMM (gemm_lat.hip) -- the
        # rocprofv3 kernel stats under profiles/ name it; the 64x64 tile kernel is reported beside it
        roofline = with_iso("lat", "gemm_lat_kernel<double> + gemm_lat_pipe_kernel<double> (latency-oriented grouped "
                                   "MFMA f64 GEMM, 32x32 tiles; the persistent two-tiles-in-flight form on groups of "
                                   "more than 512 tiles)")
        roofline["tile_kernel"] = with_iso("tile", "gemm_kernel<double> (grouped 64x64 MFMA f64 GEMM)")
        roofline["all_gemm"] = {"algorithmic_gflop_per_step": round(gemm_flops / 1e9, 4), "ms_per_step": round(gemm_ms, 4),
                                "achieved": round(gemm_flops / (gemm_ms * 1e-3) / 1e12, 4), "launches_per_step": n_gemm}
        nchol = eng.NF + 4
        chol_ms = per_kind.get("chol", 0.0)   # serial (timed) run: the three fused factor+inverse launches
        fuse_tp = bool(getattr(eng, "fuse_tp", False))
        # fused prior launches (round 6): besides factor + inverse of the 4 priors, their row workgroups form
        # T = K12 L^-T and P = T L^-1 (B M^2 flops each, triangular) for the 4 priors
        chol_gflop = nchol * 2.0 * M ** 3 / 3.0 + (4 * 2.0 * B * M ** 2 if fuse_tp else 0.0)
        chol = {"matrices_per_step": nchol, "n": M, "ms_per_step": round(chol_ms, 4),
                "kernel": ("chol_tp_kernel (2 launches: factor + update + inverse roles of the 4 GP priors with row "
                           "workgroups forming K12, T = K12 L^-T and P = T L^-1) + chol_inv7_kernel (variational "
                           "factors)" if fuse_tp else
                           "chol_inv7_kernel (factor + trailing-update + two inverse workgroups per matrix)"),
                "algorithmic_gflop_per_step": round(chol_gflop / 1e9, 4),
                "gflops": round(chol_gflop / (chol_ms * 1e-3) / 1e9, 2)}
        breakdown = {k: round(v, 4) for k, v in sorted(per_kind.items(), key=lambda kv: -kv[1])}
        breakdown_names = {k: round(v, 4) for k, v in sorted(per_name.items(), key=lambda kv: -kv[1])}

    if roofline is not None:
        # The line's achieved / frac: the SERIALISED per-launch time of the kernel, measured live in this run (HIP
        # events on the one stream the launches run on, `isolated` above) -- a kernel's own duration, so
        # launches x avg_launch_us <= ms_per_step must hold (checked below).  Beside it, from the committed
        # rocprofv3 runs of THIS code (code_hash match, tools/provenance.py; else "stale": true): the average
        # inside the graphed timed loop, where the four streams overlap and a launch's duration includes time
        # it waits for CUs held by other streams (tools/profile_bench.sh --kernel-trace --stats), the serialised
        # average of the PMC pass (dispatches serialised by counter collection) and the HBM traffic per launch
        # (FETCH_SIZE x2 per the gfx950 calibration note + WRITE_SIZE).
        ssrc, summ, sstale = matched_profile("r*_pm25_bench_summary.json")
        msrc, mfj, mstale = matched_profile("r*_pm25_mfma.json")

        def attach(entry, pred):
            iso = entry.pop("isolated")
            entry["live_concurrent"] = {"avg_launch_us": entry["avg_launch_us"], "achieved": entry["achieved"],
                                        "frac": entry["frac"], "timing": entry.pop("timing")}
            entry["avg_launch_us"], entry["achieved"], entry["frac"] = (iso["avg_launch_us"], iso["achieved"],
                                                                        iso["frac"])
            entry["timing"] = ("live HIP events around each launch on its stream, the step's launches serialised "
                               "on one stream (10 eager steps of this run)")
            entry["launches_x_avg_us"] = round(entry["launches_per_step"] * entry["avg_launch_us"], 1)
            entry["within_step"] = bool(entry["launches_x_avg_us"] <= 1000.0 * ms_per_step)
            per_launch = entry["algorithmic_gflop_per_launch"] * 1e9
            if summ is not None:
                gk = [k for k in summ["kernels"] if pred(k["name"])]
                calls = sum(k["calls"] for k in gk)
                if calls:
                    prof_us = 1000.0 * sum(k["total_ms"] for k in gk) / calls
                    prof_tf = per_launch / (prof_us * 1e-6) / 1e12
                    entry["in_graph_overlapped"] = {
                        "source": ssrc, "stale": sstale, "avg_launch_us": round(prof_us, 2),
                        "achieved": round(prof_tf, 4), "frac": round(prof_tf / FP64_MFMA_PEAK_TFLOPS, 5),
                        "launches_x_avg_us": round(entry["launches_per_step"] * prof_us, 1),
                        "timing": "rocprofv3 --kernel-trace average inside the graphed timed loop of this bench"}
                    if "hbm_write_bytes_per_launch" in gk[0]:
                        entry["traffic"] = int(sum((k["hbm_read_bytes_per_launch_x2corrected"] +
                                                    k["hbm_write_bytes_per_launch"]) * k["calls"] for k in gk) / calls)
                        entry["traffic_unit"] = "bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)"
                        entry["traffic_source"] = ssrc
                        entry["traffic_stale"] = sstale
            if mfj is not None:
                rs = [r for r in mfj["rows"] if pred(r["kernel"])]
                w = sum(r["avg_us"] * r["dispatches"] for r in rs)
                if w:
                    ser_us = w / sum(r["dispatches"] for r in rs)
                    entry["serialised_profile"] = {
                        "source": msrc, "stale": mstale, "avg_launch_us": round(ser_us, 2),
                        "achieved": round(per_launch / (ser_us * 1e-6) / 1e12, 4),
                        "timing": "rocprofv3 PMC pass, dispatches serialised by counter collection"}
                    entry["mfma_busy"] = round(sum(r["mfma_util"] * r["avg_us"] * r["dispatches"] for r in rs) / w, 4)
                    entry["mfma_busy_source"] = msrc

        attach(roofline, lambda n: "gemm_lat_kernel<double" in n or "gemm_lat_pipe_kernel<double" in n)
        attach(roofline["tile_kernel"], lambda n: n.startswith("void nmgp::gemm_kernel<double"))
        roofline["code_hash"] = CODE_HASH
        if chol is not None and mfj is not None:
            rs = [r for r in mfj["rows"] if any(k in r["kernel"] for k in ("chol_inv7_kernel", "chol_inv3_kernel",
                                                                          "chol_tp_kernel"))]
            w = sum(r["avg_us"] * r["dispatches"] for r in rs)
            if w:
                chol["mfma_busy"] = round(sum(r["mfma_util"] * r["avg_us"] * r["dispatches"] for r in rs) / w, 4)

    # free the headline workload before the large ELBO leg
    elbo = None
    used_graph = graph is not None
    if not args.no_elbo:
        used_graph = graph is not None
        del graph, trainer, eng, model, Xb, Yb, Ib, Sb
        torch.cuda.empty_cache()
        try:
            elbo = elbo_sharded(dev, world, rank, dist, D=args.elbo_D)
        except Exception as exc:                        # reported, never masks the headline line
            elbo = {"error": f"{type(exc).__name__}: {exc}"[:300]}

    # the HCP and ECoG training configurations (BASELINE.json configs[2], configs[3]) on one GPU
    hcp, ecog = None, None
    if world == 1 and not args.no_hcp:
        torch.cuda.empty_cache()
        try:
            hcp = graph_train(dev, "hcp", steps=20)
        except Exception as exc:
            hcp = {"error": f"{type(exc).__name__}: {exc}"[:300]}
    if world == 1 and not args.no_ecog:
        torch.cuda.empty_cache()
        try:
            ecog = graph_train(dev, "ecog", steps=2, warmup=1)
        except Exception as exc:
            ecog = {"error": f"{type(exc).__name__}: {exc}"[:300]}

    pair = None
    if world > 1 and not args.no_pair:
        torch.cuda.empty_cache()
        pair = pair_sharded_train(dev, world, rank, dist, D=args.pair_D)

    api = None
    if rank == 0 and world == 1 and not args.no_api:
        torch.cuda.empty_cache()
        try:
            api = api_path(dev, xs, ys, z)
        except Exception as exc:
            api = {"error": f"{type(exc).__name__}: {exc}"[:300]}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds, xs, ys, z)

    stress = None
    if rank == 0 and world == 1 and not args.no_stress:
        stress = stress_cholesky(dev)

    kron = None
    if rank == 0 and world == 1 and not args.no_kron:
        try:
            kron = kron_mv_leg(dev)
        except Exception as exc:
            kron = {"error": f"{type(exc).__name__}: {exc}"[:300]}

    if rank == 0:
        rec = {"metric": "DSVI ELBO iterations/sec (PM2.5-shaped, fp64, 1 iteration = fwd+bwd+Adam on B=2000)",
               "value": round(value, 3), "unit": "it/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
               "config": {"workload": "PM2.5-shaped synthetic DSVI step (BASELINE.json configs[1])",
                          "D_outputs": D, "M_inducing": M, "minibatch_rows": B, "N_observations": D * N_LOC,
                          "global_batch": B * world, "parallelism": f"dp{world}" if world > 1 else "single",
                          "hip_graph": used_graph,
                          "dp_allreduce": (("bucketed: the sqrt_W / sqrt_U rows on a communication stream from the step "
                                            "graph's external lbar_done node (overlapping the backward's tail), the "
                                            "remainder after it; then the 1/N + Adam graph" if dp_bucketed else
                                            "flat: one all-reduce of the whole gradient between the gradient graph and "
                                            "the 1/N + Adam graph") if used_graph else
                                           "eager: bucketed, hooked on lbar_done") if world > 1 else None},
               "roofline": roofline, "cpu_baseline": cpu, "cholesky": chol, "cholesky_stress": stress,
               "kron_mv": kron,
               "elbo_sample_sharded": elbo,
               "hcp_train": hcp, "ecog_train": ecog,
               "pair_sharded_train": pair,
               "api_path": api,
               "phase_ms": breakdown,
               "final_loss": loss_val, "code_hash": CODE_HASH}
        if cpu is not None:
            rec["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 1)
        if breakdown is not None:
            rec["phase_ms_by_launch"] = breakdown_names
            rec["gemm_by_launch"] = gemm_by_launch
        print(json.dumps(rec))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
