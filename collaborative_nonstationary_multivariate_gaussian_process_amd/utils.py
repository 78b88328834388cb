"""Drop-in for the reference module ``code/utils.py`` (GP math helpers) on the MI355X.

Constants keep the reference's names and values (code/utils.py:6-13).  The helper functions are
provided by ``gp_ops`` (HIP-backed, autograd-capable) and re-exported here under the reference names.
"""
import torch

TensorType = torch.DoubleTensor          # code/utils.py:6 (dtype marker; data live on the device)
tridiagonal_jitter = 1e-4                # code/utils.py:7
dev = "cuda"
device = torch.device(dev)

from .gp_ops import (  # noqa: E402,F401
    reparameterize, mat2ltri, squared_distance, squared_dist, create_RBF, create_Gibbs, MGP_d, MGP_mu_sigma2,
    MGP_mu, MGP, JGP, JGP_S, CGP, Normal_logprob, log_determinant_halfpower, batch_trace_XXT, batch_mahalanobis,
    KL_Gaussian,
)
