"""One eager ECoG-shaped gradient evaluation (no Adam) for A/B runs of summation-order knobs (e.g.
NMGP_KSPLIT_FACTOR): prints the loss and the gradient norm.  usage: python tools/ksplit_check.py [D]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ecog_bench as E  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 128
dev = torch.device("cuda", 0)
xs, ys = E.data(D, 391)
m, _ = E.model(D, 1024, D * 391, dev)
from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import DsviTrainer  # noqa: E402
tr = DsviTrainer(m, lr=0.01)
eng = m.engine(512)
rng = np.random.default_rng(3)
X = np.concatenate(xs); Y = np.concatenate(ys); I = np.concatenate([np.full(391, d) for d in range(D)])
idx = np.sort(rng.choice(len(X), 512, replace=False))
idx = idx[np.argsort(I[idx], kind="stable")]
sizes = [int((I[idx] == d).sum()) for d in range(D)]
eng.load_batch(torch.tensor(X[idx]), torch.tensor(Y[idx]), sizes)
loss = float(tr.grad_step(eng))
torch.cuda.synchronize()
g = m._grad
print(json.dumps({"D": D, "loss": loss, "grad_norm": float(g.norm()), "env": os.environ.get("NMGP_KSPLIT_FACTOR")}))
