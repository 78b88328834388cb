"""MI355X-native DSVI hot path of Collaborative Nonstationary Multivariate GP inference.

Drop-in modules mirroring the reference's entry points for that path:
  ``nmgp_dsvi`` (NMGP, inference, ...), ``utils`` (create_RBF, create_Gibbs, MGP_d, ...),
  ``Utility.kernels`` / ``Utility.kronecker_operation`` (legacy signatures), ``drivers`` (VTVLCM).
Compute runs in hand-written HIP kernels (libnmgp_hip.so, C ABI in include/nmgp_hip.h).
"""
__version__ = "0.1.0"
