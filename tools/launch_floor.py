"""Launch floor of the grouped f64 GEMM (GPU box): graph-replayed per-launch time of tiny problems
against a one-thread kernel, and of a 256^3 product with split-K 1 / 2 / 4.  Prints one line each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H  # noqa: E402
from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L  # noqa: E402

dev = torch.device("cuda", 0)
F64 = torch.float64


def graph_us(fn, reps=200):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
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
    return 1000.0 * e0.elapsed_time(e1) / reps





for (m, n, k, ks) in [(64, 64, 32, 1), (64, 64, 256, 1), (256, 256, 256, 1), (256, 256, 256, 2), (256, 256, 256, 4),
                      (2000, 256, 256, 1)]:
    A = torch.randn(m, k, dtype=F64, device=dev)
    B = torch.randn(k, n, dtype=F64, device=dev)
    C = torch.zeros(m, n, dtype=F64, device=dev)
    d = H.gemm_desc(C, A, B, m, n, k, (k, 1, 0), (n, 1, 0), (n, 1))
    d.ksplit = ks
    grp = H.GemmGroup([d], dev, F64)
    print(f"grouped f64 GEMM m={m} n={n} k={k} ksplit={grp.descs[0].ksplit} tiles={grp.total}: "
          f"{graph_us(grp):.2f} us/launch", flush=True)
x = torch.zeros(8, dtype=F64, device=dev)
print(f"torch fill of 8 doubles: {graph_us(lambda: x.fill_(1.0)):.2f} us/launch")
