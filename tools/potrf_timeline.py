"""One M=4096 fp32 blocked potrf (the stress configuration) replayed from a graph, for rocprofv3
kernel tracing: python tools/potrf_timeline.py [n]  (then tools/potrf_timeline.py --show <csv>)."""
import csv
import sys

if len(sys.argv) > 2 and sys.argv[1] == "--show":
    r = list(csv.DictReader(open(sys.argv[2])))
    r.sort(key=lambda x: int(x["Start_Timestamp"]))
    # last factorization: from the last zero_upper_kernel back to the previous one
    zu = [i for i, x in enumerate(r) if "zero_upper" in x["Kernel_Name"]]
    lo, hi = zu[-2] + 1, zu[-1] + 1
    t0 = int(r[lo]["Start_Timestamp"])
    busy = {}
    for x in r[lo:hi]:
        s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
        nm = x["Kernel_Name"].split("(")[0].replace("void ", "").replace("nmgp::", "")[:34]
        busy[nm] = busy.get(nm, 0) + (e - s) / 1e3
        print(f"{nm:34s} q{x['Queue_Id']} grid {x['Grid_Size_X']:>8} t={(s - t0) / 1e3:8.1f} dur {(e - s) / 1e3:7.1f}")
    print("total", (int(r[hi - 1]["End_Timestamp"]) - t0) / 1e3, "us; busy per kernel:", {k: round(v, 1) for k, v in busy.items()})
    sys.exit(0)

import os  # noqa: E402
import torch  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
G = torch.randn(n, n, generator=g, dtype=torch.float64, device=dev)
A0 = (G @ G.t() / n + torch.eye(n, dtype=torch.float64, device=dev)).float().contiguous()
W = A0.clone()
info = torch.zeros(1, dtype=torch.int32, device=dev)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    H.potrf_blocked_(W, info=info)
torch.cuda.current_stream().wait_stream(s)
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    W.copy_(A0)
    H.potrf_blocked_(W, info=info)
for _ in range(3):
    gr.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
gr.replay()
e1.record()
torch.cuda.synchronize()
print("potrf ms (incl. restore copy)", e0.elapsed_time(e1), "info", int(info.item()))
