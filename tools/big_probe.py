"""gemm_big_kernel (128x128 f32 MFMA, gemm_big.hip) on the shapes of the stress potrf's k = 512 updates, GPU box.

Every case reads L from the first 512 columns of a 4096 x 4096 row-major matrix (lda = 4096) and updates a
lower / tall-lower block of it, as potrf_two_level_f32 does: C -= L_a L_b^T.  Timed per launch as the mean of
a graph-replayed run of `reps` launches, with the split-K workspace (the library's automatic split / stream-K)
and without it (one workgroup per tile).  Algorithmic flops: 2 * (stored elements) * k.
usage: python tools/big_probe.py [--reps R]"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H  # noqa: E402
from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L  # noqa: E402

PEAK = 157.3
N = 4096


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(N, N, generator=g, device=dev) * 2 - 1) * 1e-3
    ws = H.big_workspace(dev, L.lib().nmgp_gemm_big_workspace_size())
    lib = L.lib()
    # (name, row0 of C, col0 of C, m, n, k): C = A[row0:row0+m, col0:col0+n], L rows = same rows, k columns 0..k
    cases = [("np_first", 512, 512, 3584, 128, 512), ("np_rest", 640, 640, 3456, 384, 512),
             ("far_full_p0", 1024, 1024, 3072, 3072, 512), ("far_piece_p0", 1024, 1024, 3072, 640, 512),
             ("far_full_p3", 2560, 2560, 1536, 1536, 512), ("tile1", 3968, 3968, 128, 128, 512),
             ("far_full_k1024", 2048, 2048, 2048, 2048, 1024), ("syrk_k128", 256, 256, 3840, 3840, 128)]
    for name, r0, c0, m, n, k in cases:
        for split in (True, False):
            Lp = A[r0:, :k]
            Lb = A[c0:, :k]
            C = A[r0:, c0:]

            def body():
                rc = lib.nmgp_gemm_big_f32(ctypes.c_void_p(Lp.data_ptr()), N, ctypes.c_void_p(Lb.data_ptr()), N, 1,
                                           ctypes.c_void_p(C.data_ptr()), N, 1, m, n, k, L.OUT_LOWER, -1.0, 1.0, 0, 0,
                                           0, 1, ctypes.c_void_p(ws.data_ptr()) if split else None,
                                           L.stream_handle())
                L.check(rc, "gemm_big")
            body()
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for _ in range(args.reps):
                    body()
            gr.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = 1e9
            for _ in range(3):
                e0.record()
                gr.replay()
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / args.reps)
            tri = min(m, n)
            elems = tri * (tri + 1) // 2 + (m - tri) * n
            tf = 2.0 * elems * k / (best * 1e-3) / 1e12
            print(json.dumps({"case": name, "m": m, "n": n, "k": k, "split": split, "us": round(best * 1e3, 2),
                              "tflops": round(tf, 2), "frac": round(tf / PEAK, 4)}), flush=True)


if __name__ == "__main__":
    main()
