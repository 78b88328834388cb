"""Round-4 bisection of the side <-> side2 ping-pong capture crash (hipStreamEndCapture segfaulted when the
ping-pong of tests/test_gpu_primitives.py::test_hip_graph_side_stream_ping_pong was captured through the
library's nmgp_graph_* calls, while tools/graph_edge_repro2.hip's identical raw-HIP sequence captures fine).
Each variant runs in its own process (a segfault ends only that variant):
  torch_ev       torch.cuda.Event record / wait, torch elementwise kernels   (the failing test)
  raw_ev         HIP events through ctypes (hipEventCreateWithFlags / hipEventRecord / hipStreamWaitEvent on
                 the torch streams' handles), torch elementwise kernels
  raw_ev_libk    HIP events through ctypes, the library's own kernels (nmgp_counter_add)
  torch_ev_libk  torch events, the library's kernels
usage: python tools/graph_edge_probe2.py            (driver: runs every variant, prints one line each)
       python tools/graph_edge_probe2.py <variant>  (one variant)"""
import os as _os
import sys as _sys

if _os.environ.get("NMGP_RUN_KNOWN_CRASH") != "1":
    # Its crashing variants segfault in hipStreamEndCapture of torch's bundled ROCm 7.0 runtime (result recorded
    # in DESIGN.md §4).  Not run by default: a known crash is not worth GPU time.
    print("graph edge probe: known-crash bisection, recorded in DESIGN.md §4; set NMGP_RUN_KNOWN_CRASH=1 to re-run")
    _sys.exit(0)
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = ["torch_ev", "raw_ev", "raw_ev_libk", "torch_ev_libk"]


def run(variant):
    import torch
    sys.path.insert(0, ROOT)
    from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    dev = torch.device("cuda", 0)
    hip = ctypes.CDLL("libamdhip64.so")
    raw = variant.startswith("raw_ev")
    libk = variant.endswith("libk")

    class Ev:
        def __init__(self):
            if raw:
                self.h = ctypes.c_void_p()
                assert hip.hipEventCreateWithFlags(ctypes.byref(self.h), 2) == 0     # hipEventDisableTiming
            else:
                self.t = torch.cuda.Event()

        def record(self, s):
            if raw:
                assert hip.hipEventRecord(self.h, ctypes.c_void_p(s.cuda_stream)) == 0
            else:
                self.t.record(s)

        def wait(self, s):
            if raw:
                assert hip.hipStreamWaitEvent(ctypes.c_void_p(s.cuda_stream), self.h, 0) == 0
            else:
                s.wait_event(self.t)

    if libk:
        x = torch.zeros(1, dtype=torch.int64, device=dev)
        y = torch.zeros(1, dtype=torch.int64, device=dev)
        kx1 = lambda: H.counter_add_(x, 1)
        ky = lambda: H.counter_add_(y, 3)
        kx2 = lambda: H.counter_add_(x, 5)
        expect = (18, 9)
    else:
        x = torch.zeros(4096, dtype=torch.float64, device=dev)
        y = torch.zeros(4096, dtype=torch.float64, device=dev)
        kx1 = lambda: x.add_(1.0)
        ky = lambda: y.add_(x)
        kx2 = lambda: x.mul_(2.0)
        expect = (14, 11)
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    g = H.HipGraph(dev)
    print("stage capture", flush=True)
    with g.capture():
        main = torch.cuda.current_stream(dev)
        e0, e1, e2, e3 = Ev(), Ev(), Ev(), Ev()
        e0.record(main)
        e0.wait(s1)
        e0.wait(s2)
        with torch.cuda.stream(s1):
            kx1()
            e1.record(s1)
        with torch.cuda.stream(s2):
            e1.wait(s2)
            ky()
            e2.record(s2)
        with torch.cuda.stream(s1):
            e2.wait(s1)
            kx2()
            e3.record(s1)
        e3.wait(main)
        e2.wait(main)
        print("stage end_capture", flush=True)
    print("stage replay", flush=True)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print("ok", variant, float(x.reshape(-1)[0]), float(y.reshape(-1)[0]), "expect", expect, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
        sys.exit(0)
    for v in VARIANTS:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), v], capture_output=True, text=True, timeout=120)
        print(v, "rc", r.returncode, " | ".join(l for l in r.stdout.splitlines() if l.strip()), flush=True)
