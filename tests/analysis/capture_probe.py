"""Capture one DSVI step of the toy fixture into a HIP graph and replay it (schedule A/B probe)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests import _golden as G  # noqa: E402
from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer  # noqa: E402

g = G.load("mid_forward")
xs, ys = G.split_lists(g)
m = NMGP(4096, 3, g["z"], device="cuda:0", noise="device")
tr = DsviTrainer(m, lr=0.01)
eng = m.engine(sum(len(x) for x in xs))
eng.load_batch(g["x"], g["y"], [len(x) for x in xs])
gr = tr.capture(eng)
gr.replay()
torch.cuda.synchronize()
print("captured + replayed, loss", float(eng.out[0]), flush=True)
