"""Isolated timings of the ECoG-shaped batched factor products on gemm_big_kernel (HIP events, one stream).

  python tools/big_probe.py [--nf 1024] [--M 1024] [--reps 5]

Variants: the three products of the training step (syrk_side, xs_side, kl_lbar as engine.py builds them) and
ablations of kl_lbar (no epilogue; k-contiguous A and/or B -- wrong values, same masks and tile ranges) that
separate the epilogue's cost from the transposed-operand staging.  Prints one JSON line per variant.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L  # noqa: E402
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nf", type=int, default=1024)
    ap.add_argument("--M", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    M, nf = a.M, a.nf
    MM = M * M
    g = torch.Generator(device=dev).manual_seed(0)
    mk = lambda: torch.randn(nf * MM, device=dev, generator=g) * 0.01
    th, Cinv, Xs, gr, Af = mk(), mk(), mk(), mk(), mk()
    rs = torch.rand(nf * M, device=dev, generator=g)
    offs = [f * MM for f in range(nf)]
    roffs = [f * M for f in range(nf)]
    BB = H.BigBatch
    base = dict(lda=M, ldb=M)
    lb = L.A_UPPER | L.B_LOWER | L.OUT_TRIL
    epi = (th, offs, (M, 1), rs, roffs, 1.0)
    v = {
        "syrk_side": BB(th, th, Af, offs, offs, offs, M, M, M, b_kcontig=True,
                        flags=L.A_LOWER | L.B_UPPER | L.OUT_LOWER, diag_add=1e-4, **base),
        "xs_side": BB(Cinv, th, Xs, offs, offs, offs, M, M, M, b_kcontig=False,
                      flags=L.A_LOWER | L.B_LOWER | L.OUT_TRIL, **base),
        "kl_lbar": BB(Cinv, Xs, gr, offs, offs, offs, M, M, M, a_kcontig=False, b_kcontig=False,
                      flags=lb | L.EPI_E_LOWER, alpha=-1.0, beta=1.0, epi=epi, **base),
        "kl_lbar_noepi_beta1": BB(Cinv, Xs, gr, offs, offs, offs, M, M, M, a_kcontig=False, b_kcontig=False,
                                  flags=lb, alpha=-1.0, beta=1.0, **base),
        "kl_lbar_noepi_beta0": BB(Cinv, Xs, gr, offs, offs, offs, M, M, M, a_kcontig=False, b_kcontig=False,
                                  flags=lb, alpha=-1.0, beta=0.0, **base),
        "kl_lbar_ak_beta0": BB(Cinv, Xs, gr, offs, offs, offs, M, M, M, a_kcontig=True, b_kcontig=False,
                               flags=lb, alpha=-1.0, beta=0.0, **base),
        "kl_lbar_ak_bk_beta0": BB(Cinv, Xs, gr, offs, offs, offs, M, M, M, a_kcontig=True, b_kcontig=True,
                                  flags=lb, alpha=-1.0, beta=0.0, **base),
    }
    st = torch.cuda.current_stream()
    for name, bb in v.items():
        macs = bb.macs()
        bb()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.reps):
            bb()
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        print(json.dumps({"variant": name, "nf": nf, "M": M, "ms": round(ms, 3), "tflop": round(2 * macs / 1e12, 4),
                          "tflops": round(2 * macs / ms / 1e9, 2), "ms_per_8384": round(ms * 8384 / nf, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
