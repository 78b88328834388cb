"""Peak check of gemm_kernel on large dense problems (GPU box): TF/s vs the 78.6 TF/s fp64 peak."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H  # noqa: E402

dev = torch.device("cuda", 0)
for (m, n, k) in [(4096, 4096, 4096), (2048, 2048, 2048), (2000, 256, 1280), (256, 256, 2000), (2000, 256, 256)]:
    for dt in (torch.float64, torch.float32):
        A = torch.randn(m, k, dtype=dt, device=dev)
        B = torch.randn(k, n, dtype=dt, device=dev)
        C = torch.empty(m, n, dtype=dt, device=dev)
        d = H.gemm_desc(C, A, B, m, n, k, (k, 1, 0), (n, 1, 0), (n, 1))
        grp = H.GemmGroup([d], dev, dt)
        grp()
        torch.cuda.synchronize()
        ref = (A.double() @ B.double())
        err = float((C.double() - ref).norm() / ref.norm())
        reps = 10
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
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
        print(f"{m}x{n}x{k} {str(dt)[6:]:8s} split {grp.descs[0].ksplit:2d} wgs {grp.total:5d} {ms * 1000:9.1f} us "
              f"{2 * m * n * k / ms / 1e9:8.2f} TF/s  relerr {err:.1e}", flush=True)
