"""Per-term error of the engine's -SELBO on the M = 1024 ECoG-like fixture (GPU box; analysis only):
reconstruction term and the three KL terms, fp64 and fp32 engines, against the CPU oracle."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import nmgp_oracle as O  # noqa: E402
from tests import _golden as G  # noqa: E402
from tests.test_gpu_ecog import _theta  # noqa: E402
from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import DsviEngine  # noqa: E402

g = G.load("ecog_like_forward")
p = G.params(g, D=4, M=1024)
xs, ys = G.split_lists(g)
N = float(g["N"])
with torch.no_grad():
    loss, c = O.forward(p, xs, ys, g["z"], N, O.TapeNoise(g["noise"]))
ref = {"loss": float(loss), "SELBO_R": float(c["SELBO_R"]), "KL_W": float(c["KL_W"]), "KL_v": float(c["KL_v"]),
       "KL_U": float(c["KL_U"])}
print("oracle", ref, flush=True)
sizes = [int(s) for s in g["sizes"]]
for dt, packed in ((torch.float64, False), (torch.float32, True), (torch.float32, False)):
    eng = DsviEngine(4, 1024, sum(sizes), g["z"], dtype=dt, packed=packed)
    th = _theta(p, 4, 1024, dt, packed)
    eng.bind(th, torch.zeros_like(th), N=N)
    eng.load_batch(g["x"], g["y"], sizes, noise=g["noise"])
    eng.forward_backward()
    torch.cuda.synchronize()
    o = eng.out.double().cpu().numpy()
    got = dict(zip(["loss", "SELBO_R", "KL_W", "KL_v", "KL_U"], o[:5]))
    print(str(dt), "packed" if packed else "dense",
          {k: f"{got[k]:.10e} rel {abs(got[k] - ref[k]) / abs(ref[k]):.2e}" for k in ref}, flush=True)

# the error inherent in fp32 INPUTS: the fp64 engine on parameters / data / noise rounded to fp32
r32 = lambda a: np.asarray(a, np.float64).astype(np.float32).astype(np.float64)
p32 = {k: v.float().double() for k, v in p.items()}
eng = DsviEngine(4, 1024, sum(sizes), r32(g["z"]), dtype=torch.float64)
th = _theta(p32, 4, 1024, torch.float64, False)
eng.bind(th, torch.zeros_like(th), N=N)
eng.load_batch(r32(g["x"]), r32(g["y"]), sizes, noise=g["noise"])
eng.forward_backward()
torch.cuda.synchronize()
o = eng.out.double().cpu().numpy()
got = dict(zip(["loss", "SELBO_R", "KL_W", "KL_v", "KL_U"], o[:5]))
print("fp64 engine on fp32-rounded inputs", {k: f"rel {abs(got[k] - ref[k]) / abs(ref[k]):.2e}" for k in ref}, flush=True)
