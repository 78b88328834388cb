"""Phase ticks (100 MHz) of the finalize kernel in one PM2.5-shaped step (library built with
-DNMGP_FIN_TRACE; loaded through NMGP_LIB_OVERRIDE)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
D, M, B = bench.D, bench.M, bench.B
dev = torch.device("cuda", 0)
xs, ys = bench.synth_data(0)
model = NMGP(number_observations=D * bench.N_LOC, dim_outputs=D, Z=np.linspace(0, 1, M), minibatch_size=B, seed=22,
             device=dev, noise="device")
trainer = DsviTrainer(model, lr=0.01)
eng = model.engine(B)
x, y, I, seg = bench.epoch_batches(xs, ys, np.random.default_rng(1))[0]
eng.load_batch(x, y, np.diff(seg))
for _ in range(3):
    trainer.grad_step(eng)
torch.cuda.synchronize()
print("finalize ticks (10 ns): loads/partials %.0f  block_sum %.0f  grads %.0f" % tuple(float(v) for v in eng.out[5:8]))
