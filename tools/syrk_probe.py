"""Trailing-update SYRK / GEMM rate on the 128x128 f32 MFMA kernel (gemm_big.hip), GPU box.

Shapes: the trailing updates of the M=4096 stress Cholesky (recursive split: A22 -= L21 L21^T with
n2 = k = 2048 at the top level, 1024 below) and of a right-looking blocked factorization
(n2 = 4096 - j*256, k = 256), plus a 4096^3 square GEMM.  Algorithmic flops: n2 (n2 + 128) k for
the lower-tile SYRK as launched -- reported as n2^2 k (the useful half, 2 * n2(n2+1)/2 * k) --
and 2 m n k for GEMMs.  Peak: 157.3 TF/s (MI355X fp32 MFMA, dense).  Prints one JSON line per shape.
usage: python tools/syrk_probe.py [--reps R] [--legacy]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H  # noqa: E402
from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L  # noqa: E402

PEAK = 157.3


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--legacy", action="store_true", help="also time the 64x64 grouped kernel on the same shapes")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    ws = H.big_workspace(dev, L.lib().nmgp_gemm_big_workspace_size())
    cases = [("syrk", 2048, 2048, 2048), ("syrk", 1024, 1024, 1024), ("syrk", 3840, 3840, 256),
             ("syrk", 2048, 2048, 256), ("syrk", 4096, 4096, 4096), ("gemm", 4096, 4096, 4096),
             ("gemm", 2048, 2048, 2048)]
    for kind, m, n, k in cases:
        A = torch.rand(m, k, generator=g, device=dev) * 2 - 1
        B = A if kind == "syrk" else torch.rand(n, k, generator=g, device=dev) * 2 - 1
        C = torch.zeros(m, n, device=dev)
        flags = L.OUT_LOWER if kind == "syrk" else 0
        beta = 1.0 if kind == "syrk" else 0.0
        ms = timed(lambda: H.gemm_big(A, B, C, flags=flags, alpha=-1.0, beta=beta, ws=ws), args.reps)
        flops = (float(m) * (m + 1) * k) if kind == "syrk" else 2.0 * m * n * k
        rec = {"kernel": "gemm_big_kernel (128x128 f32 MFMA)", "kind": kind, "m": m, "n": n, "k": k,
               "ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 2), "frac_of_fp32_mfma_peak":
               round(flops / ms / 1e9 / PEAK, 4), "flop_count": "n(n+1)k (lower half)" if kind == "syrk" else "2mnk"}
        if args.legacy:
            ms2 = timed(lambda: H.matmul(A, B if kind == "gemm" else A, transB=True, out=C), args.reps)
            rec["legacy_64x64_full_ms"] = round(ms2, 4)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
