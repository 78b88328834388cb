"""ctypes binding of libnmgp_hip.so (the C ABI declared in include/nmgp_hip.h).

The library is built in-tree (``make -C collaborative_nonstationary_multivariate_gaussian_process_amd/csrc``
or ``python -c "import __graft_entry__ as g; g.build()"``).  There is NO fallback: if the .so is missing
or a device call fails, the calls raise.  torch is imported first so that the process's HIP runtime
is torch's own libamdhip64 (same SONAME), which the .so then binds to.
"""
import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime the library binds to)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NMGP_LIB_OVERRIDE") or os.path.join(_HERE, "libnmgp_hip.so")  # override: A/B experiments

c_int, c_i64, c_dbl, c_vp, c_u64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p, ctypes.c_uint64


class HipError(RuntimeError):
    pass


class GemmDesc(ctypes.Structure):
    _fields_ = [("A", c_vp), ("B", c_vp), ("C", c_vp), ("kscale", c_vp), ("epi_E", c_vp), ("epi_rs", c_vp),
                ("sA_i", c_i64), ("sA_k", c_i64), ("sA_kb", c_i64),
                ("sB_k", c_i64), ("sB_j", c_i64), ("sB_kb", c_i64),
                ("sC_i", c_i64), ("sC_j", c_i64), ("sE_i", c_i64), ("sE_j", c_i64),
                ("m", c_int), ("n", c_int), ("k", c_int), ("kbA", c_int), ("kbB", c_int), ("flags", c_int),
                ("row_seg", c_int), ("k_seg", c_int),
                ("alpha", c_dbl), ("beta", c_dbl), ("gamma", c_dbl), ("diag_add", c_dbl),
                ("tiles_m", c_int), ("tiles_n", c_int), ("tile_start", c_int), ("seg_span", c_int),
                ("ksplit", c_int), ("pad2_", c_int), ("ws", c_vp), ("counters", c_vp),
                ("sA_b", c_i64), ("sB_b", c_i64), ("sC_b", c_i64), ("batch", c_int), ("pad3_", c_int)]


class PairwiseDesc(ctypes.Structure):
    _fields_ = [("X", c_vp), ("Z", c_vp), ("ellX", c_vp), ("ellZ", c_vp), ("sigX", c_vp), ("sigZ", c_vp),
                ("hyp", c_vp), ("K", c_vp), ("ldk", c_i64),
                ("n", c_int), ("m", c_int), ("p", c_int), ("mode", c_int), ("dist", c_int), ("flags", c_int),
                ("scale2", c_dbl), ("length_scale", c_dbl), ("diag_add", c_dbl),
                ("tiles", c_int), ("tile_start", c_int)]


class PairwiseBwdDesc(ctypes.Structure):
    _fields_ = [("X", c_vp), ("Z", c_vp), ("ellX", c_vp), ("ellZ", c_vp), ("hyp", c_vp),
                ("K", c_vp), ("Rbar", c_vp), ("Pm", c_vp), ("rowcoef", c_vp),
                ("row_part", c_vp), ("col_part", c_vp), ("scal_part", c_vp), ("ld", c_i64),
                ("n", c_int), ("m", c_int), ("p", c_int), ("mode", c_int), ("flags", c_int), ("tiles", c_int),
                ("tile_start", c_int), ("pad_", c_int), ("scale2", c_dbl), ("length_scale", c_dbl)]


class PairDesc(ctypes.Structure):
    _fields_ = [("a_off", c_i64), ("l_off", c_i64), ("c_off", c_i64), ("seg", c_int), ("pad", c_int)]


class DsviArgs(ctypes.Structure):
    _fields_ = [("D", c_int), ("M", c_int), ("B", c_int), ("Q", c_int), ("NF", c_int), ("elbo_mode", c_int),
                ("frozen_mask", c_int), ("pair_packed", c_int), ("N_over_B", c_dbl), ("jitter", c_dbl),
                ("theta", c_vp), ("grad", c_vp),
                ("off_muW", c_i64), ("off_sW", c_i64), ("off_muv", c_i64), ("off_sv", c_i64), ("off_muU", c_i64),
                ("off_sU", c_i64), ("off_hyp", c_i64),
                ("x", c_vp), ("y", c_vp), ("row_out", c_vp), ("seg", c_vp), ("Z", c_vp), ("noise", c_vp),
                ("Afac", c_vp), ("Cinv", c_vp), ("Ainv", c_vp), ("K12", c_vp), ("P", c_vp), ("Pbar", c_vp),
                ("R", c_vp), ("Abar", c_vp), ("WG", c_vp), ("WP", c_vp), ("Y", c_vp), ("Xs", c_vp),
                ("v", c_vp), ("vbar", c_vp), ("ellZ", c_vp), ("ellX", c_vp), ("var_t", c_vp),
                ("rowbuf", c_vp), ("facbuf", c_vp), ("red", c_vp), ("out", c_vp),
                ("gib_row", c_vp), ("gib_col", c_vp), ("scal_part", c_vp), ("phi", c_vp),
                ("info", c_vp), ("n_ct", c_int), ("n_rt", c_int), ("n_rt22", c_int), ("nblk_rows", c_int),
                ("scal_off", c_i64 * 8), ("T", c_vp),
                ("pair_q0", c_int), ("n_wfac", c_int), ("kl_v", c_int), ("pair_pad", c_int), ("T64", c_vp),
                ("kl_f0", c_int), ("kl_f1", c_int), ("v64", c_vp), ("ellZ64", c_vp), ("K12_64", c_vp),
                ("t64", c_vp), ("scal64", c_vp), ("adam_step", c_vp)]


class CholTpMat(ctypes.Structure):
    _fields_ = [("reserved", c_int), ("rows", c_int), ("hyp", c_vp), ("K12", c_vp), ("T", c_vp), ("P", c_vp)]


class CholTpArgs(ctypes.Structure):
    _fields_ = [("A", c_vp), ("n", c_i64), ("lda", c_i64), ("strideA", c_i64), ("X", c_vp), ("ldx", c_i64),
                ("strideX", c_i64), ("batch", c_i64), ("info", c_vp), ("jitter", c_dbl), ("Z", c_vp), ("ellZ", c_vp),
                ("x", c_vp), ("B", c_i64), ("Pt", c_vp), ("Tt", c_vp), ("v", c_vp), ("zt", c_vp), ("hyp_t", c_vp),
                ("ellX", c_vp), ("var_t", c_vp), ("mats", CholTpMat * 4), ("vg_muv", c_vp), ("vg_z", c_vp),
                ("vg_v", c_vp), ("vg_ellZ", c_vp), ("vg_K22", c_vp), ("vg_wgs", c_i64)]


# flags (include/nmgp_hip.h)
A_LOWER, A_UPPER, B_LOWER, B_UPPER = 1, 2, 4, 8
OUT_LOWER, OUT_TRIL, KSCALE, EPI, EPI_E_LOWER, DIAG_ADD, EPI_RS_NEG = 16, 32, 64, 128, 256, 512, 1024
LAT_COLPACK = 2048
RBF, GIBBS = 0, 1
DIST_DIFF, DIST_EXPAND = 0, 1
HYP_LOG = 1

_SIGS = {
    "nmgp_version": (c_int, []),
    "nmgp_graph_begin": (c_int, [c_vp]),
    "nmgp_graph_end": (c_int, [c_vp, ctypes.POINTER(c_vp)]),
    "nmgp_graph_launch": (c_int, [c_vp, c_vp]),
    "nmgp_graph_destroy": (c_int, [c_vp]),
    "nmgp_event_create": (c_int, [ctypes.POINTER(c_vp)]),
    "nmgp_event_destroy": (c_int, [c_vp]),
    "nmgp_event_record_external": (c_int, [c_vp, c_vp]),
    "nmgp_stream_wait_event": (c_int, [c_vp, c_vp]),
    "nmgp_device_status": (c_int, [ctypes.POINTER(ctypes.c_uint32), c_int]),
    "nmgp_sizeof_gemm_desc": (c_i64, []),
    "nmgp_sizeof_pair_desc": (c_i64, []),
    "nmgp_pair_quad_f64": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp]),
    "nmgp_pair_quad_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp]),
    "nmgp_pair_dot_f64": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp]),
    "nmgp_pair_dot_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp]),
    "nmgp_pair_rank_f64": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp]),
    "nmgp_pair_rank_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp]),
    "nmgp_pair_mv_f64": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp]),
    "nmgp_pair_mv_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp]),
    "nmgp_pair_pbar_reduce_f64": (c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_int, c_int, c_int, c_int, c_int,
                                          c_vp]),
    "nmgp_pair_pbar_reduce_f32": (c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_int, c_int, c_int, c_int, c_int,
                                          c_vp]),
    "nmgp_sizeof_pairwise_desc": (c_i64, []),
    "nmgp_sizeof_pairwise_bwd_desc": (c_i64, []),
    "nmgp_sizeof_dsvi_args": (c_i64, []),
    "nmgp_sizeof_chol_tp_args": (c_i64, []),
    "nmgp_chol_tp_f64": (c_int, [c_vp, c_vp]),
    "nmgp_chol_tp_trace": (c_int, [c_vp, c_i64]),
    "nmgp_gemm_grouped_f64": (c_int, [c_vp, c_int, c_int, c_vp, c_vp]),
    "nmgp_gemm_grouped_f32": (c_int, [c_vp, c_int, c_int, c_vp, c_vp]),
    "nmgp_gemm_grouped_dyn_f64": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp]),
    "nmgp_gemm_grouped_dyn_f32": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp]),
    "nmgp_gemm_grouped_lat_f64": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp]),
    "nmgp_gemm_grouped_lat_f32": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp]),
    "nmgp_gemm_plan": (c_int, [c_vp, c_int, c_vp, c_vp, c_vp]),
    "nmgp_gemm_plan_lat": (c_int, [c_vp, c_int, c_vp, c_vp, c_vp]),
    "nmgp_gemm_grouped_dyn_planned_f64": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp]),
    "nmgp_gemm_grouped_dyn_planned_f32": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp]),
    "nmgp_gemm_grouped_lat_planned_f64": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp]),
    "nmgp_gemm_grouped_lat_planned_f32": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp]),
    "nmgp_gemm_grouped_lat_pipe_f64": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp]),
    "nmgp_gemm_grouped_lat_pipe_f32": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp]),
    "nmgp_gemm_f64": (c_int, [ctypes.POINTER(GemmDesc), c_vp, c_vp]),
    "nmgp_gemm_f32": (c_int, [ctypes.POINTER(GemmDesc), c_vp, c_vp]),
    "nmgp_potrf_batched_f64": (c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "nmgp_potrf_batched_f32": (c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "nmgp_trtri_batched_f64": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "nmgp_trtri_batched_f32": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "nmgp_chol_inv_batched_f64": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "nmgp_chol_inv_batched_f32": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "nmgp_chol_inv_workspace_size_f32": (c_i64, [c_i64, c_i64]),
    "nmgp_potrf_blocked_workspace_size_f32": (c_i64, [c_i64]),
    "nmgp_potrf_blocked_workspace_size_f64": (c_i64, [c_i64]),
    "nmgp_potrf_blocked_f32": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "nmgp_potrf_blocked_f64": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "nmgp_chol_inv_batched_ws_f32": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64,
                                             c_vp]),
    "nmgp_chol_split_point": (c_i64, [c_i64]),
    "nmgp_chol_blockinv_batched_f32": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "nmgp_syevj_workspace_size_f64": (c_i64, [c_i64]),
    "nmgp_syevj_batched_f64": (c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64,
                                       c_vp]),
    "nmgp_gemm_big_workspace_size": (c_i64, []),
    "nmgp_gemm_big_f32": (c_int, [c_vp, c_i64, c_vp, c_i64, c_int, c_vp, c_i64, c_i64, c_int, c_int, c_int, c_int,
                                  c_dbl, c_dbl, c_i64, c_i64, c_i64, c_int, c_vp, c_vp]),
    "nmgp_gemm_big_offsets_f32": (c_int, [c_vp, c_i64, c_vp, c_i64, c_int, c_vp, c_i64, c_i64, c_int, c_int, c_int,
                                          c_int, c_dbl, c_dbl, c_dbl, c_vp, c_vp, c_vp, c_int, c_vp, c_vp]),
    "nmgp_gemm_big_offsets_epi_f32": (c_int, [c_vp, c_i64, c_int, c_vp, c_i64, c_int, c_vp, c_i64, c_i64, c_int, c_int,
                                              c_int, c_int, c_dbl, c_dbl, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64,
                                              c_i64, c_vp, c_vp, c_dbl, c_vp, c_vp, c_vp, c_int, c_vp, c_vp]),
    "nmgp_gemm_big_offsets_seg_f32": (c_int, [c_vp, c_i64, c_int, c_vp, c_i64, c_int, c_vp, c_i64, c_i64, c_int, c_int,
                                              c_int, c_int, c_dbl, c_dbl, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64,
                                              c_i64, c_vp, c_vp, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp,
                                              c_vp]),
    "nmgp_gemm_big_offsets_dual_f32": (c_int, [c_vp, c_i64, c_int, c_vp, c_i64, c_int, c_vp, c_i64, c_i64, c_int,
                                               c_int, c_int, c_int, c_dbl, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64,
                                               c_i64, c_vp, c_vp, c_dbl, c_vp, c_vp, c_i64, c_int, c_vp]),
    "nmgp_pairwise_f64": (c_int, [c_vp, c_int, c_int, c_vp]),
    "nmgp_pairwise_f32": (c_int, [c_vp, c_int, c_int, c_vp]),
    "nmgp_pairwise_single_f64": (c_int, [ctypes.POINTER(PairwiseDesc), c_vp]),
    "nmgp_pairwise_single_f32": (c_int, [ctypes.POINTER(PairwiseDesc), c_vp]),
    "nmgp_pairwise_bwd_f64": (c_int, [c_vp, c_int, c_int, c_vp]),
    "nmgp_pairwise_bwd_f32": (c_int, [c_vp, c_int, c_int, c_vp]),
    "nmgp_pairwise_bwd_single_f64": (c_int, [ctypes.POINTER(PairwiseBwdDesc), c_vp]),
    "nmgp_pairwise_bwd_single_f32": (c_int, [ctypes.POINTER(PairwiseBwdDesc), c_vp]),
    "nmgp_colsum_f64": (c_int, [c_vp, c_i64, c_i64, c_dbl, c_vp, c_vp]),
    "nmgp_colsum_f32": (c_int, [c_vp, c_i64, c_i64, c_dbl, c_vp, c_vp]),
    "nmgp_kron_product_f64": (c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "nmgp_kron_product_f32": (c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "nmgp_kron_product_diag_f64": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp]),
    "nmgp_kron_product_diag_f32": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp]),
    "nmgp_kron_mv_f64": (c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "nmgp_kron_mv_f32": (c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "nmgp_dsvi_hyper_f64": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_hyper_f32": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_vg22_f64": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_vg22_f32": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_trow_f64": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_trow_f32": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_recon_f64": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_recon_f32": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_kl_f64": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_kl_f32": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_delta_f64": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_delta_f32": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_tbwd_f64": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_tbwd_f32": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_vbwd_f64": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_vbwd_f32": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_finalize_f64": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_finalize_f32": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_mugrad_f64": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_mugrad_f32": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_prefinal_f64": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_dsvi_prefinal_f32": (c_int, [ctypes.POINTER(DsviArgs), c_vp]),
    "nmgp_adam_f64": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_dbl, c_dbl, c_dbl, c_dbl, c_vp]),
    "nmgp_adam_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_dbl, c_dbl, c_dbl, c_dbl, c_vp]),
    "nmgp_adam_lower_f64": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_int, c_int, c_vp, c_dbl, c_dbl, c_dbl,
                                    c_dbl, c_vp]),
    "nmgp_adam_lower_advanced_f64": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_int, c_int, c_vp, c_dbl, c_dbl,
                                             c_dbl, c_dbl, c_vp]),
    "nmgp_adam_lower_advanced_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_int, c_int, c_vp, c_dbl, c_dbl,
                                             c_dbl, c_dbl, c_vp]),
    "nmgp_adam_lower_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_int, c_int, c_vp, c_dbl, c_dbl, c_dbl,
                                    c_dbl, c_vp]),
    "nmgp_normal_f64": (c_int, [c_vp, c_i64, c_u64, c_vp, c_i64, c_vp]),
    "nmgp_normal_f32": (c_int, [c_vp, c_i64, c_u64, c_vp, c_i64, c_vp]),
    "nmgp_counter_add": (c_int, [c_vp, c_i64, c_vp]),
    "nmgp_pbar_reduce_f64": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_int, c_int, c_int, c_vp]),
    "nmgp_pbar_reduce_f32": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_int, c_int, c_int, c_vp]),
    "nmgp_lbar_reduce_f64": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_int, c_int, c_vp]),
    "nmgp_lbar_reduce_f32": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_int, c_int, c_vp]),
    "nmgp_convert_f32_to_f64": (c_int, [c_vp, c_vp, c_i64, c_vp]),
    "nmgp_convert_f64_to_f32": (c_int, [c_vp, c_vp, c_i64, c_vp]),
    "nmgp_step_begin_f64": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_u64, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "nmgp_step_begin_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_u64, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "nmgp_batch_gather_f64": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      c_vp]),
    "nmgp_batch_gather_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      c_vp]),
}

_lib = None


def lib():
    """Load (once) and return the ctypes library; raises if it is missing or mismatched."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C {os.path.join(_HERE, 'csrc')}` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    for cls, fn in [(GemmDesc, "nmgp_sizeof_gemm_desc"), (PairwiseDesc, "nmgp_sizeof_pairwise_desc"),
                    (PairwiseBwdDesc, "nmgp_sizeof_pairwise_bwd_desc"), (DsviArgs, "nmgp_sizeof_dsvi_args"),
                    (PairDesc, "nmgp_sizeof_pair_desc"), (CholTpArgs, "nmgp_sizeof_chol_tp_args")]:
        if ctypes.sizeof(cls) != getattr(L, fn)():
            raise ImportError(f"ABI mismatch: ctypes {cls.__name__} is {ctypes.sizeof(cls)} bytes, "
                              f"library says {getattr(L, fn)()}")
    _lib = L
    return L


def exported_symbols():
    return list(_SIGS.keys())


def check(rc, what):
    if rc != 0:
        raise HipError(f"{what} failed with status {rc}")


STATUS_BITS = {1: "two-role Cholesky: the inverse workgroup gave up waiting for its factor workgroup",
               2: "grouped GEMM: a cooperative split-K chunk gave up waiting for a peer",
               4: "blocked potrf: a step workgroup gave up waiting for the panel publisher"}


def device_status(clear=True):
    """OR of the device status words (include/nmgp_hip.h NMGP_STATUS_*); synchronises the device."""
    v = ctypes.c_uint32(0)
    check(lib().nmgp_device_status(ctypes.byref(v), 1 if clear else 0), "device_status")
    return int(v.value)


def check_device_status():
    """Raise if a bounded inter-workgroup spin gave up since the last check (results untrustworthy)."""
    st = device_status(clear=True)
    if st:
        what = "; ".join(msg for bit, msg in STATUS_BITS.items() if st & bit)
        raise HipError(f"device status 0x{st:x}: {what} -- the results since the last check are not valid")


def stream_handle(device=None):
    """The raw hipStream_t of torch's current stream on `device`."""
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t, offset_elems=0):
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr() + offset_elems * t.element_size())


def require_device(t, name="tensor"):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device (HIP) tensor; there is no CPU fallback")
