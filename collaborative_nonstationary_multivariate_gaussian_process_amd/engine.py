"""The DSVI step engine: closed-form -SELBO and all 13 gradients on the MI355X (fp64, or fp32 for
the HCP / ECoG-shaped configurations of SURVEY §8d).

One engine instance owns the device workspace for a fixed (D outputs, M inducing points,
B minibatch rows) and enqueues the ~30 HIP launches of one step on torch's
current stream.  Nothing in a step allocates, synchronises or touches the host, so a whole step
(noise -> forward -> backward -> Adam) can be captured once in a HIP graph and replayed.

Reference path replaced: NMGP.forward + loss.backward() (code/nmgp_dsvi.py:157-301, 839-847),
NMGP.compute_ELBO (code/nmgp_dsvi.py:303-404) and the Adam step (:777, :854).
"""
import ctypes
import os
import math

import numpy as np
import torch

from . import _lib as L
from . import hip_ops as H

F64 = torch.float64
F32 = torch.float32
JITTER = 1e-4   # code/utils.py:7
MUGRAD_IN_FINALIZE_MAX = 65536     # include/nmgp_hip.h NMGP_MUGRAD_IN_FINALIZE_MAX


def _sfx(dt):
    return "f64" if dt == F64 else "f32"

PARAM_NAMES = ["mu_W", "sqrt_W", "mu_v", "sqrt_v", "mu_U", "sqrt_U",
               "sigma2_tildeell_log", "length_scales_tildeell_log", "sigma2_L0_log",
               "length_scales_L0_log", "sigma2_L1_log", "length_scales_L1_log", "sigma2_err_log"]
HYPER_NAMES = PARAM_NAMES[6:]


def pair_window(D, pair_range=None):
    """(q0, Q) of the packed pairs held for outputs [i0, i1): the pairs (i, j <= i) of those outputs are
    the contiguous packed indices [i0(i0+1)/2, i1(i1+1)/2).  None = all D outputs."""
    i0, i1 = (0, D) if pair_range is None else (int(pair_range[0]), int(pair_range[1]))
    if not 0 <= i0 < i1 <= D:
        raise ValueError(f"pair_range {pair_range} must be a non-empty output range inside [0, {D})")
    q0 = i0 * (i0 + 1) // 2
    return q0, i1 * (i1 + 1) // 2 - q0


def param_layout(D, M, packed=False, pair_range=None):
    """Offsets (elements) of the 13 parameters inside the flat theta vector, registration order.

    packed=False: the reference's dense layout, mu_U (D, D, M) and sqrt_U (D, D, M, M) with all D^2
    coefficient blocks (code/nmgp_dsvi.py:136-143).  packed=True: only the Q = D(D+1)/2 live pairs
    (i, j <= i) in (i, j) order, mu_U (Q, M) and sqrt_U (Q, M, M) -- the dead upper blocks never
    receive a gradient, and at the ECoG shape (D=128, M=1024) the dense layout is
    69 GB per copy of sqrt_U in fp32 against 35 GB packed.  pair_range=(i0, i1) (packed only): a
    pair-sharded rank's vector -- mu_U / sqrt_U hold only the pairs of outputs [i0, i1)."""
    if pair_range is not None and not packed:
        raise ValueError("pair_range needs the packed pair layout")
    Q = pair_window(D, pair_range)[1]
    if packed:
        shapes = [(D, M), (D, M, M), (M,), (M, M), (Q, M), (Q, M, M)] + [()] * 7
    else:
        shapes = [(D, M), (D, M, M), (M,), (M, M), (D, D, M), (D, D, M, M)] + [()] * 7
    offs, o = {}, 0
    for name, shp in zip(PARAM_NAMES, shapes):
        n = int(np.prod(shp)) if shp else 1
        offs[name] = (o, shp)
        o += n
    return offs, o


def lower_block_ranges(offs):
    """(offset, blocks) of the parameters that are stacks of M x M blocks used only through their lower triangle
    (sqrt_W, sqrt_v, sqrt_U: mat2ltri, code/utils.py:68-72), ascending -- hip_ops.adam_lower_'s ranges."""
    out = []
    for name in ("sqrt_W", "sqrt_v", "sqrt_U"):
        o, shp = offs[name]
        out.append((o, int(np.prod(shp[:-2])) if len(shp) > 2 else 1))
    return sorted(out)


# the triangular-block Adam from this M on.  Round 6: nmgp_adam_lower is one launch over the whole flat vector
# (csrc/dsvi.hip adam_flat_kernel), so the PM2.5 shape (M = 256) takes it too -- its sqrt blocks' upper halves are no
# longer streamed (before: 512, below which the per-range launches cost more than the saved traffic).  Small toy
# shapes keep the dense update, which also moves upper-triangle entries a synthetic gradient may carry;
# NMGP_ADAM_LOWER_MIN_M overrides (A/B)
ADAM_LOWER_MIN_M = int(os.environ.get("NMGP_ADAM_LOWER_MIN_M", "256"))


def use_adam_lower(M, dtype, offs):
    """nmgp_adam_lower walks 16-byte vectors of each block row: it needs M and every block range's offset to be
    multiples of 16 / element size (the C side returns -8 otherwise, csrc/dsvi.hip adam_lower).  Shapes that are
    not (fp32 M % 4 != 0, fp64 odd M) keep the dense update."""
    V = 16 // torch.empty((), dtype=dtype).element_size()
    return M >= ADAM_LOWER_MIN_M and M % V == 0 and all(o % V == 0 for o, _ in lower_block_ranges(offs))


def pair_list(D, pair_range=None):
    i0, i1 = (0, D) if pair_range is None else pair_range
    return [(i, j) for i in range(i0, i1) for j in range(i + 1)]


class DsviEngine:
    """Workspace + launch schedule of one DSVI step for fixed (D, M, B)."""

    def __init__(self, D, M, B, z, device="cuda", jitter=JITTER, dtype=F64, packed=False, factor_ws=None,
                 pair_range=None, kl_owner=True):
        """packed: the parameter vector uses the packed pair layout of param_layout.  factor_ws: the
        (Afac, Cinv, Xs) factor workspaces of another engine of the same (D, M, dtype) to share (they
        hold no state between steps; a model's engines never run concurrently).

        Pair sharding (SURVEY §8e axis 3, training steps only): pair_range=(i0, i1) makes this the
        engine of a rank that owns outputs [i0, i1) -- its minibatch holds only rows of those outputs,
        its parameter vector only their pairs (param_layout(pair_range=...)), and it factors only their
        Sigma_U blocks; kl_owner=False drops KL_W and KL_v (and the W factors, which only the KL needs)
        so that exactly one rank adds them.  The loss and the replicated gradients (mu_W, sqrt_W, mu_v,
        sqrt_v, hyper-parameters) of the ranks then sum to the whole model's (distributed.PairShard)."""
        if not torch.cuda.is_available():
            raise RuntimeError("DsviEngine needs a HIP device; there is no CPU fallback")
        if dtype not in (F64, F32):
            raise ValueError("DsviEngine computes in float64 or float32")
        L.lib()
        self.dt = dtype
        self.sfx = _sfx(dtype)
        self.D, self.M, self.B = D, M, B
        if pair_range is not None and not packed:
            raise ValueError("pair sharding needs the packed pair layout")
        self.pair_range = None if pair_range is None else (int(pair_range[0]), int(pair_range[1]))
        self.q0, self.Q = pair_window(D, self.pair_range)
        self.pairs = pair_list(D, self.pair_range)
        self.kl_owner = bool(kl_owner)
        self.nW = D if self.kl_owner else 0      # W factors in the factor list (only their KL needs them)
        self.NF = self.nW + 1 + self.Q
        self.dev = torch.device(device)
        self.jitter = jitter
        self.packed = bool(packed)
        self.offs, self.nparam = param_layout(D, M, packed=self.packed, pair_range=self.pair_range)
        Q, NF = self.Q, self.NF
        self.NPC = Q if self.packed else D * D     # pair columns of mu_U / Y_0 / Y_1 / sel
        e = lambda *shape: torch.zeros(*shape, dtype=self.dt, device=self.dev)
        self.Z = torch.as_tensor(np.asarray(z, np.float64).reshape(-1, 1), device=self.dev).to(self.dt).contiguous()
        assert self.Z.shape[0] == M
        # minibatch (rows grouped by output) + noise
        self.x = e(B)
        self.y = e(B)
        self.row_out = torch.zeros(B, dtype=torch.int32, device=self.dev)
        self.seg = torch.zeros(D + 1, dtype=torch.int32, device=self.dev)
        self.noise = e(M + B + Q * B)
        # factors
        if factor_ws is not None:
            self.Afac, self.Cinv, self.Xs = factor_ws
            assert self.Afac.shape == (NF + 4, M, M) and self.Afac.dtype == self.dt
        else:
            self.Afac = e(NF + 4, M, M)
            self.Cinv = e(NF + 4, M, M)
            self.Xs = e(NF, M, M)
        self.Ainv = e(4, M, M)
        self.K12 = e(4, B, M)
        self.P = e(4, B, M)
        self.T = e(4, B, M)             # K12 C2^-T per prior: Nystrom variances ||T_row||^2, P = T C2^-1
        self.Pbar = e(4, B, M)
        self.R = e(4, B, M)
        self.Abar = e(4, M, M)
        self.WG = e(D, B, M)
        self.WP = e(D, B, M)
        self.Zg = e(D, B, M)            # per-factor P-bar_G products W-hat_d L_d^T (rows of outputs >= d)
        # round 5: where every output owns few minibatch rows (ECoG: B / D = 4) the per-pair products -- the
        # quadratic-form factors P L_ij, their P-bar W-hat L_ij^T and the pair L-bar P^T W-hat -- stream each
        # M x M block once on the pair kernels (csrc/pairs.hip) instead of 64-row MFMA tiles that are ~94 %
        # padding.  NMGP_PAIR_STREAM=0 keeps them on the grouped kernels (tests' equivalence switch).
        n_out = (self.pair_range[1] - self.pair_range[0]) if self.pair_range is not None else D
        self.pair_stream = (self.Q > 0 and B <= 32 * max(1, n_out) and M % 4 == 0 and M <= 1024
                            and os.environ.get("NMGP_PAIR_STREAM", "1") != "0")
        self.big_side = self.dt == torch.float32 and M >= 512 and os.environ.get("NMGP_BIG_SIDE", "1") != "0"
        # round 6: with big_side the row-segmented B x M x M products (W = P L, P-bar = W-hat L^T) run on the 128x128
        # kernel too; NMGP_BIG_ROWS=0 keeps them on the grouped kernel (A/B and equivalence switch)
        self.big_rows = self.big_side and os.environ.get("NMGP_BIG_ROWS", "1") != "0"
        # round 6: the KL L-bar of the variational factors in the solve form, Sigma^-1 L = C^-T (C^-1 L) applied
        # blockwise from the factor and the inverses of its two diagonal blocks (the recursion's top-level
        # off-diagonal inverse block, two products, is not formed: nmgp_chol_blockinv_batched_f32).  NMGP_KL_SOLVE=0
        # keeps the explicit-inverse form (A/B and equivalence switch)
        self.kl_solve = (self.big_side and M > 256 and M % 128 == 0 and os.environ.get("NMGP_KL_SOLVE", "1") != "0")
        self._ones = torch.ones(M, dtype=self.dt, device=self.dev) if self.kl_solve else None
        # per-pair P-bar products W-hat_ij L_ij^T, slot j (pair kernels, or the 128x128 kernel at M >= 512)
        self.Zp = e(D, B, M) if (self.pair_stream or (self.big_rows and self.Q > 0)) else None
        # HCP / ECoG shapes (fp32, M >= 512): the D+Q factor products run on the 128x128 f32 MFMA kernel at
        # per-factor offsets (BigBatch) instead of the grouped 64x64 tiles.  NMGP_BIG_SIDE=0 keeps them on the
        # grouped kernel: the only schedule switch left, for tests/test_gpu_engine.py's equivalence check (set above,
        # where the per-pair Z buffer is sized)
        # round 6: fp64 engines of 128 <= M <= 256 run the GP priors as two fused launches (nmgp_chol_tp_f64): the
        # RBF priors' K22 built, factored and inverted with K12 / T / P of their rows formed by the same launch, and
        # likewise the Gibbs prior with its t-row sample -- no builder, invG / projG or t-row launches on the chain.
        # NMGP_FUSE_TP=0 keeps the separate launches (the tests' equivalence switch)
        self.fuse_tp = (self.dt == torch.float64 and 128 <= M <= 256 and B <= 4096
                        and os.environ.get("NMGP_FUSE_TP", "1") != "0")
        # and the Gibbs prior's K22 from the first of them (NMGP_FUSE_VG=0: its own launch, dsvi_vg22)
        self.fuse_vg = self.fuse_tp and os.environ.get("NMGP_FUSE_VG", "1") != "0"
        # per-(output, factor) L-bar products of the grouped backward (bwd_lbar), summed by nmgp_lbar_reduce: D(D+1)/2
        # slots of M x M + M.  Only where the slots stay small (PM2.5: 15 slots, 7.9 MB); many outputs with few
        # rows each (HCP-like D = 50) keep one product per factor, whose k loop is then short anyway
        nsl = D * (D + 1) // 2
        self.Ylb = e(nsl * (M * M + M)) if (not self.big_side and nsl * (M * M + M) * self.dt.itemsize
                                                   <= (64 << 20)) else None
        self.Y = e(D + 1 + 2 * self.NPC, M)
        self.T2 = e(M, M)
        self.v, self.ellZ = e(M), e(M)
        self.vbar = e(2 * M)            # [0:M] P_t^T tbar (GEMM), [M:2M] completed by the v-backward kernel
        self.ellX, self.var_t = e(B), e(B)
        self.rowbuf = e(2 * D + 5, B)
        # KL per factor | delta/w vectors (8M) | selection weights (4D^2) | e_f rows (NF M) | KL slab partials
        self.facbuf = e(NF + 8 * M + 4 * self.NPC + NF * M + NF * ((M + 15) // 16) * 4)
        self.nblk = B                       # recon partials: one per row; then (B+3)//4 t-row partials
        self.red = e(4 * B + (B + 3) // 4)
        self.out = e(16)          # [0..4] loss / SELBO_R / KL_W / KL_v / KL_U, [8..14] training pre-sums
        self.n_ct = (M + 63) // 64
        self.n_rt = H.bwd_tiles(B, M)[2]        # row tiles of the pairwise backward's column partials
        self.n_rt22 = H.bwd_tiles(M, M)[2]
        self.gib_row = e(self.n_ct * B + self.n_ct * M)
        self.gib_col = e(self.n_rt * M + self.n_rt22 * M)
        tb = H.bwd_tiles(B, M)[0]
        tm = H.bwd_tiles(M, M)[0]
        scal_tiles = [tb, tm, tb, tm, tb, tm]          # L0_12, L0_22, L1_12, L1_22, t12, t22
        self.scal_off = [0] + list(np.cumsum(scal_tiles))
        self.scal_part = e(2 * int(self.scal_off[-1]))
        self.phi = e(M, M)
        self.info = torch.zeros(NF + 4, dtype=torch.int32, device=self.dev)
        # fp32 engines factor the four GP priors (t, L0, L1, G) in fp64 and round L, L^-1 back: the
        # explicit-inverse projections K12 (K22 + 1e-4 I)^-1 of smooth priors otherwise lose
        # ~cond(K22) * eps32 (HCP-like fixture: P_G off by 40% with an fp32 factorization, 5e-4 with
        # an fp64 one -- DESIGN.md §5).
        self.prior64 = self.p64 = dtype == F32
        if self.prior64:
            # with p64 a fifth fp64 slot in front holds Sigma_v + 1e-4 I: [v | t | L0 | L1 | G] is then
            # one contiguous batch whose first four slots factor in one launch, like the fp32 slots
            # FV .. FV + 3 (v, t, L0, L1) they are rounded back into
            nsl = 5 if self.p64 else 4
            rawA = torch.zeros(nsl, M, M, dtype=F64, device=self.dev)
            rawX = torch.zeros(nsl, M, M, dtype=F64, device=self.dev)
            self.pri_A64, self.pri_X64 = rawA[nsl - 4:], rawX[nsl - 4:]
            self.v_A64, self.v_X64 = (rawA[0], rawX[0]) if self.p64 else (None, None)
        # fp32 engines also form the prior kernel matrices K22 / K12, the Nystrom factors T = K12 C2^-T,
        # the projections P = T C2^-1 and the prior inverses in fp64 (rounded to fp32 only for the fp32
        # consumers), and take the Nystrom variances k11 - ||T_row||^2 from the fp64 T: built in fp32, the
        # entries' rounding is amplified by A^-1 (cond ~1e5-1e6 at length scales 3/M) -- the ECoG-like
        # fixture's loss was 1.6e-3 off with fp32 projections (tests/analysis/ecog_fp32_diag.py).  With it
        # the v sample (fp64 factor of Sigma_v) and the prior adjoint chains (R, A-bar, builder backward,
        # hyper-parameter partial sums) are fp64 as well (tests/analysis/ecog_hyper_sensitivity.py: the
        # hyper-parameter gradients cancel to ~1e-7 of their terms; fp32 adjoints left them 14-30% off).
        if self.p64:
            z64 = lambda *s: torch.zeros(*s, dtype=F64, device=self.dev)
            self.x64, self.hyp64, self.ellX64, self.ellZ64 = z64(B), z64(8), z64(B), z64(M)
            self.Z64 = torch.as_tensor(np.asarray(z, np.float64).reshape(-1, 1), device=self.dev).contiguous()
            self.K12_64, self.T64, self.P64 = z64(4, B, M), z64(4, B, M), z64(4, B, M)
            self.Ainv64 = z64(4, M, M)
            # the v sample in fp64: sqrt_v / mu_v widened, Sigma_v + 1e-4 I formed and factored in fp64
            self.sv64, self.muv64 = z64(M * M), z64(M)
            # the t-prior adjoints in fp64: P-bar_t | varbar | varbar partials (t-row
            # backward), R_t, A-bar_t, the KL_v parts' delta_t | Y_t, and the t12 / t22 builder partials
            self.t64 = z64(B * M + B + (B + 3) // 4)
            self.Rt64, self.Abt64, self.dY64 = z64(B, M), z64(M, M), z64(2 * M)
            # the L0 / L1 prior adjoints likewise: P-bar_0/1 and their KL A-bar parts widened, the
            # row coefficients c0 / c1, R and A-bar in fp64; all six builder partial sets in fp64
            # (same tile offsets as scal_part)
            self.PbL64, self.RL64, self.AbL64, self.rcL64 = z64(2, B, M), z64(2, B, M), z64(2, M, M), z64(2, B)
            self.scal64 = z64(2 * int(self.scal_off[6]))
        # selection weights for the -1/2 Y diag(sel) Y^T prior adjoint (static)
        sel = np.zeros((4, self.NPC))
        for (i, j) in self.pairs:
            sel[2 if i == j else 1, self.pidx(i, j)] = 1.0
        base = NF + 8 * M
        self.facbuf[base:base + 4 * self.NPC] = torch.from_numpy(sel.reshape(-1)).to(self.dev)
        self._theta = None
        self._plans = {}
        self._elbo_kl = None      # (f0, f1, with_v): compute_ELBO KL share (None: the whole model's)

    def pidx(self, i, j):
        """Block index of coefficient pair (i, j) in mu_U / sqrt_U (dense i*D + j, or packed)."""
        return i * (i + 1) // 2 + j - self.q0 if self.packed else i * self.D + j

    def factor_workspace(self):
        return (self.Afac, self.Cinv, self.Xs)

    # ------------------------------------------------------------------------------------ binding
    def bind(self, theta, grad, frozen_mask=0, N=None):
        """Attach the flat parameter / gradient vectors (device, engine dtype) and build the launch plans."""
        assert theta.dtype == self.dt and theta.is_cuda and theta.numel() == self.nparam
        assert grad.dtype == self.dt
        if self._theta is not None and theta.data_ptr() == self._theta.data_ptr() and \
                grad.data_ptr() == self._grad.data_ptr() and frozen_mask == self.frozen_mask:
            if N is not None:
                self.N = N
            return
        self._theta, self._grad = theta, grad
        self.frozen_mask = frozen_mask
        self.N = N if N is not None else self.B
        self._plans = {}

    def _args(self, elbo_mode=0):
        a = L.DsviArgs()
        D, M, B = self.D, self.M, self.B
        a.D, a.M, a.B, a.Q, a.NF = D, M, B, self.Q, self.NF
        a.elbo_mode, a.frozen_mask = elbo_mode, self.frozen_mask
        a.pair_packed = 1 if self.packed else 0
        a.N_over_B = float(self.N) / float(B)
        a.jitter = self.jitter
        a.theta, a.grad = self._theta.data_ptr(), self._grad.data_ptr()
        o = self.offs
        a.off_muW, a.off_sW, a.off_muv, a.off_sv = o["mu_W"][0], o["sqrt_W"][0], o["mu_v"][0], o["sqrt_v"][0]
        a.off_muU, a.off_sU, a.off_hyp = o["mu_U"][0], o["sqrt_U"][0], o["sigma2_tildeell_log"][0]
        for name in ["x", "y", "row_out", "seg", "Z", "noise", "Afac", "Cinv", "Ainv", "K12", "P", "Pbar", "R",
                     "Abar", "WG", "WP", "Y", "Xs", "v", "vbar", "ellZ", "ellX", "var_t", "rowbuf", "facbuf",
                     "red", "out", "gib_row", "gib_col", "scal_part", "phi", "info", "T"]:
            setattr(a, name, getattr(self, name).data_ptr())
        a.n_ct, a.n_rt, a.n_rt22, a.nblk_rows = self.n_ct, self.n_rt, self.n_rt22, self.nblk
        for i, v in enumerate(self.scal_off):
            a.scal_off[i] = int(v)
        a.pair_q0, a.n_wfac, a.kl_v = self.q0, self.nW, 1 if self.kl_owner else 0
        a.T64 = self.T64.data_ptr() if self.p64 else 0
        if self.p64:
            a.v64, a.ellZ64, a.K12_64 = self.v_A64.data_ptr(), self.ellZ64.data_ptr(), self.K12_64.data_ptr()
            a.t64, a.scal64 = self.t64.data_ptr(), self.scal64.data_ptr()
        a.kl_f0, a.kl_f1 = 0, self.NF - 1
        kp = self._elbo_kl if elbo_mode else None
        if kp is not None:                       # this rank's share of compute_ELBO's KL terms
            a.kl_f0, a.kl_f1 = kp[0], kp[1]
            a.kl_v = 1 if (kp[2] and self.kl_owner) else 0
        return a

    # ------------------------------------------------------------------------------------ plans
    def _plan(self, elbo_mode):
        key = (elbo_mode, self._elbo_kl if elbo_mode else None)
        if key in self._plans:
            return self._plans[key]
        D, M, B, NF, Q = self.D, self.M, self.B, self.NF, self.Q
        MM, BM = M * M, B * M
        th, gr = self._theta, self._grad
        o = self.offs
        sW, sv, sU = o["sqrt_W"][0], o["sqrt_v"][0], o["sqrt_U"][0]
        muW, muv, muU, hyp = o["mu_W"][0], o["mu_v"][0], o["mu_U"][0], o["sigma2_tildeell_log"][0]
        if elbo_mode and self.pair_range is not None:
            raise NotImplementedError("compute_ELBO gathers a column of L (code/nmgp_dsvi.py:361): rows of output o "
                                      "need the pairs (s, o) of every s >= o, so it is sharded over samples, not pairs")
        pairs = self.pairs
        nW = self.nW
        i0, i1 = self.pair_range if self.pair_range is not None else (0, D)
        # factor order: W (nW) | pairs (Q) | v  -> v and the 3 static priors are contiguous slots NF-1..NF+2
        pq = self.pidx
        NPC = self.NPC
        fac_off = [sW + d * MM for d in range(nW)] + [sU + pq(i, j) * MM for (i, j) in pairs] + [sv]
        prior_of = [3] * nW + [2 if i == j else 1 for (i, j) in pairs] + [0]
        NFK = NF if self.kl_owner else NF - 1    # factors whose KL this engine adds (v is last)
        FV = NF - 1
        dev, seg = self.dev, self.seg
        G = lambda descs: H.GemmGroup(descs, dev, self.dt, seg=seg)
        g = H.gemm_desc
        rows_all = dict(row_seg=0, seg_span=D)          # all rows of the minibatch via the segment table
        p = {}
        # F1: RBF builders (K_t12, K_t22 + lam I, K_L0_*, K_L1_*)
        bl = []
        for k, hoff in [(0, hyp + 0), (1, hyp + 2), (2, hyp + 4)]:
            K12v = self.K12[k]
            bl.append(H.pairwise_desc(K12v, self.x, self.Z, mode=L.RBF, hyp=th, hyp_off=hoff, hyp_log=True))
            if not self.p64:
                bl.append(H.pairwise_desc(self.Afac[NF + k], self.Z, self.Z, mode=L.RBF, hyp=th, hyp_off=hoff,
                                          hyp_log=True, diag_add=self.jitter))
        p["build_rbf"] = H.PairwiseGroup(bl, dev)
        p64 = self.p64
        if p64:
            # the fp64 path of fp32 engines: K12 / K22 + lam I of the RBF priors in fp64 (K22 straight into
            # the fp64 factor slots), from fp64 copies of x and the hyper-parameters (conv_in)
            bl64 = []
            for k, hoff in [(0, 0), (1, 2), (2, 4)]:
                bl64.append(H.pairwise_desc(self.K12_64[k], self.x64, self.Z64, mode=L.RBF, hyp=self.hyp64,
                                            hyp_off=hoff, hyp_log=True))
                bl64.append(H.pairwise_desc(self.pri_A64[k], self.Z64, self.Z64, mode=L.RBF, hyp=self.hyp64,
                                            hyp_off=hoff, hyp_log=True, diag_add=self.jitter))
            p["build_rbf64"] = H.PairwiseGroup(bl64, dev)
            G64 = lambda descs: H.GemmGroup(descs, dev, F64, seg=seg)
            X64 = self.pri_X64
            ainv64 = lambda k: g(self.Ainv64, X64, X64, M, M, M, (1, M, 0), (M, 1, 0), (M, 1),
                                 flags=L.A_UPPER | L.B_LOWER, offs=(k * MM, k * MM, k * MM))
            tproj64 = lambda k: g(self.T64, self.K12_64, X64, B, M, M, (M, 1, 0), (1, M, 0), (M, 1), flags=L.B_UPPER,
                                  offs=(k * BM, k * MM, k * BM), **rows_all)
            pproj64 = lambda k: g(self.P64, self.T64, X64, B, M, M, (M, 1, 0), (M, 1, 0), (M, 1), flags=L.B_LOWER,
                                  offs=(k * BM, k * MM, k * BM), **rows_all)
            p["inv3_64"] = G64([ainv64(k) for k in range(3)] + [tproj64(k) for k in range(3)])
            p["proj3_64"] = G64([pproj64(k) for k in range(3)])
            p["invG_64"] = G64([ainv64(3), tproj64(3)])
            p["projG_64"] = G64([pproj64(3)])
        # F2: A1_f = tril(S_f) tril(S_f)^T + lam I (lower part); v on the main path, the rest on the side stream
        syrk = lambda f: g(self.Afac, th, th, M, M, M, (M, 1, 0), (1, M, 0), (M, 1),
                           flags=L.A_LOWER | L.B_UPPER | L.OUT_LOWER, diag_add=self.jitter,
                           offs=(fac_off[f], fac_off[f], f * MM))
        xs = lambda f: g(self.Xs, self.Cinv, th, M, M, M, (M, 1, 0), (M, 1, 0), (M, 1),
                         flags=L.A_LOWER | L.B_LOWER | L.OUT_TRIL, offs=(f * MM, fac_off[f], f * MM))
        p["syrk"] = G([syrk(FV)])
        if self.p64:
            p["syrk"] = H.GemmGroup([g(self.v_A64, self.sv64, self.sv64, M, M, M, (M, 1, 0), (1, M, 0), (M, 1),
                                       flags=L.A_LOWER | L.B_UPPER | L.OUT_LOWER, diag_add=self.jitter,
                                       offs=(0, 0, 0))], dev, F64, seg=seg)
        # the side factors: all W / pair factors, or in compute_ELBO this rank's KL share of them
        kf0, kf1 = (self._elbo_kl[0], self._elbo_kl[1]) if (elbo_mode and self._elbo_kl is not None) else (0, FV)
        p["kl_range"] = (kf0, kf1)
        p["syrk_side"] = G([syrk(f) for f in range(kf0, kf1)]) if kf1 > kf0 else None
        p["syrk_all"] = G([syrk(f) for f in range(FV + 1)])   # training step: Sigma_v with the others
        # F5: prior inverses t,0,1 and Xs_f = Cinv_f L_f (KL gradient)
        d5 = [g(self.Ainv, self.Cinv, self.Cinv, M, M, M, (1, M, 0), (M, 1, 0), (M, 1), flags=L.A_UPPER | L.B_LOWER,
                offs=((NF + k) * MM, (NF + k) * MM, k * MM)) for k in range(3)]
        # T_k = K12_k C_k^-T (same launch: independent of the inverses); the projections below are
        # P_k = T_k C_k^-1, i.e. two triangular applications instead of K12 (C^-T C^-1)
        tproj = lambda k: g(self.T, self.K12, self.Cinv, B, M, M, (M, 1, 0), (1, M, 0), (M, 1), flags=L.B_UPPER,
                            offs=(k * BM, (NF + k) * MM, k * BM), **rows_all)
        pproj = lambda k: g(self.P, self.T, self.Cinv, B, M, M, (M, 1, 0), (M, 1, 0), (M, 1), flags=L.B_LOWER,
                            offs=(k * BM, (NF + k) * MM, k * BM), **rows_all)
        if not self.fuse_tp:
            d5 += [tproj(k) for k in range(3)]
        if p64:
            d5 = []                       # prior inverses and T in fp64 (inv3_64)
        if not elbo_mode:
            d5.append(xs(FV))
            p["xs_side"] = G([xs(f) for f in range(FV)])
        p["inv3"] = G(d5) if d5 else None
        if self.big_side:
            # HCP / ECoG shapes: the D+Q factor products are 1000s of M x M triangular products --
            # the 128x128 f32 MFMA kernel at per-factor parameter offsets instead of 64x64 grouped tiles
            offs_f, slots = fac_off[:FV], [f * MM for f in range(FV)]
            if kf1 > kf0:
                p["syrk_side"] = H.BigBatch(th, th, self.Afac, offs_f[kf0:kf1], offs_f[kf0:kf1], slots[kf0:kf1], M, M,
                                            M, lda=M, ldb=M, b_kcontig=True, flags=L.A_LOWER | L.B_UPPER | L.OUT_LOWER,
                                            diag_add=self.jitter)
            if not elbo_mode:
                p["xs_side"] = H.BigBatch(self.Cinv, th, self.Xs, slots, offs_f, slots, M, M, M, lda=M, ldb=M,
                                          b_kcontig=False, flags=L.A_LOWER | L.B_LOWER | L.OUT_TRIL)
                if self.kl_solve and FV > 0:
                    p["xs_side"] = self._kl_solve_xs(th, slots, offs_f)
        # F6: P_k = K12_k Ainv_k (k = t,0,1) ; Y_t, Y_0, Y_1
        d6 = [pproj(k) for k in range(3)] if not (p64 or self.fuse_tp) else []
        d6 += [g(self.Y, self.Ainv, th, M, 1, M, (M, 1, 0), (1, M, 0), (1, M), offs=(0, muv, D * M)),
               g(self.Y, self.Ainv, th, M, NPC, M, (M, 1, 0), (1, M, 0), (1, M), offs=(MM, muU, (D + 1) * M)),
               g(self.Y, self.Ainv, th, M, NPC, M, (M, 1, 0), (1, M, 0), (1, M),
                 offs=(2 * MM, muU, (D + 1 + NPC) * M))]
        p["proj3"] = G(d6)
        # F9: Gibbs builders (K_G22 + lam I into the G prior slot, K_G12)
        # K_G22 + lam I needs only ell_Z (the v sample) and feeds chol_G on the main chain; K_G12 also needs
        # ell_X (the t-row) and is built on the second side stream beside chol_G
        if not p64:
            p["build_g22"] = H.PairwiseGroup([
                H.pairwise_desc(self.Afac[NF + 3], self.Z, self.Z, mode=L.GIBBS, ellX=self.ellZ, ellZ=self.ellZ,
                                diag_add=self.jitter)], dev)
        else:
            # K_G22 + lam I in fp64 from ell_Z (fp32 sample, widened), straight into the fp64 factor slot
            p["build_g22"] = H.PairwiseGroup([
                H.pairwise_desc(self.pri_A64[3], self.Z64, self.Z64, mode=L.GIBBS, ellX=self.ellZ64,
                                ellZ=self.ellZ64, diag_add=self.jitter)], dev)
        bg12 = [H.pairwise_desc(self.K12[3], self.x, self.Z, mode=L.GIBBS, ellX=self.ellX, ellZ=self.ellZ)]
        p["build_g12"] = H.PairwiseGroup(bg12, dev)
        if p64:
            p["build_g12_64"] = H.PairwiseGroup([
                H.pairwise_desc(self.K12_64[3], self.x64, self.Z64, mode=L.GIBBS, ellX=self.ellX64,
                                ellZ=self.ellZ64)], dev)
        p["invG"] = G([g(self.Ainv, self.Cinv, self.Cinv, M, M, M, (1, M, 0), (M, 1, 0), (M, 1),
                         flags=L.A_UPPER | L.B_LOWER, offs=((NF + 3) * MM, (NF + 3) * MM, 3 * MM))] +
                      ([] if self.fuse_tp else [tproj(3)])) if not p64 else None
        p["projG"] = G(([pproj(3)] if not (p64 or self.fuse_tp) else []) +
                       [g(self.Y, self.Ainv, th, M, D, M, (M, 1, 0), (1, M, 0), (1, M), offs=(3 * MM, muW, 0))])
        if self.fuse_tp:
            # the two fused prior launches (hip_ops.CholTp): [v | t | L0 | L1] with the three RBF priors' K12 / T / P
            # rows formed in the launch, then the Gibbs prior with the t-row and K_G12 rows.  The RBF priors' K22 +
            # lam I (theta only) are built off the chain at the step's start (build_k22), K_G22 by the v launch
            hyp_addr = lambda k: th.data_ptr() + (hyp + k) * th.element_size()
            rbf = [dict(rows=1, hyp=hyp_addr(2 * k), K12=self.K12[k], T=self.T[k], P=self.P[k]) for k in range(3)]
            # training steps: K_G22 (and v, ell_Z) from extra workgroups of the same launch once L_v is factored
            # (round 6; compute_ELBO keeps the v launch, which its cached samples rerun alone)
            vg = None
            if not elbo_mode and self.fuse_vg:
                vg = dict(muv=th.data_ptr() + muv * th.element_size(), z=self.noise, v=self.v, ellZ=self.ellZ,
                          K22=self.Afac[NF + 3], wgs=int(os.environ.get("NMGP_VG_WGS", "8")))
            p["chol_tp_main"] = H.CholTp(self.Afac[FV], self.Cinv[FV], self.info[FV:], M, [dict()] + rbf,
                                         jitter=self.jitter, Z=self.Z, x=self.x, B=B, vg=vg)
            p["chol_tp_G"] = H.CholTp(self.Afac[NF + 3], self.Cinv[NF + 3], self.info[NF + 3:], M,
                                      [dict(rows=2, K12=self.K12[3], T=self.T[3], P=self.P[3])],
                                      jitter=self.jitter, Z=self.Z, ellZ=self.ellZ, x=self.x, B=B,
                                      trow=dict(Pt=self.P[0], Tt=self.T[0], v=self.v, zt=self.noise[M:M + B],
                                                hyp_t=hyp_addr(0), ellX=self.ellX, var_t=self.var_t))
            p["build_k22"] = H.PairwiseGroup([
                H.pairwise_desc(self.Afac[NF + k], self.Z, self.Z, mode=L.RBF, hyp=th, hyp_off=hoff, hyp_log=True,
                                diag_add=self.jitter) for k, hoff in [(0, hyp + 0), (1, hyp + 2), (2, hyp + 4)]], dev)
        # F14: quadratic-form factors W = P L on the rows that use them
        d14 = []
        for d in range(D):
            rs = dict(row_seg=d, seg_span=D - d) if not elbo_mode else dict(row_seg=0, seg_span=d + 1)
            d14.append(g(self.WG, self.P, th, B, M, M, (M, 1, 0), (M, 1, 0), (M, 1), flags=L.B_LOWER,
                         offs=(3 * BM, sW + d * MM, d * BM), **rs))
        for (i, j) in pairs:
            typ = 2 if i == j else 1
            slot, rseg = (j, i) if not elbo_mode else (i, j)
            d14.append(g(self.WP, self.P, th, B, M, M, (M, 1, 0), (M, 1, 0), (M, 1), flags=L.B_LOWER,
                         offs=(typ * BM, sU + pq(i, j) * MM, slot * BM), row_seg=rseg))
        p["quad"] = G(d14)
        if self.pair_stream:
            qp = []
            for (i, j) in pairs:
                slot, rseg = (j, i) if not elbo_mode else (i, j)
                qp.append(((2 if i == j else 1) * BM, sU + pq(i, j) * MM, slot * BM, rseg))
            pair_quad = H.PairStream("quad", self.P, th, self.WP, qp, seg, M)
            p["quad"] = H.Seq([G(d14[:D]), pair_quad])
        if not elbo_mode:
            # the pair factors W_P = P_{0,1} L_ij need only the L0 / L1 projections (proj3, side2): they run
            # on side2 beside the Gibbs prior chain; only the latent factors W_G = P_G L_d follow projG
            p["quad_W"] = G(d14[:D])
            p["quad_P"] = pair_quad if self.pair_stream else G(d14[D:])
        if elbo_mode:
            # later Monte-Carlo samples of compute_ELBO: the pair factors W_P = P_{0,1} L_ij do not depend
            # on the sample (the L priors and Sigma_U are fixed within a call) -- only the D latent ones
            p["quad_W"] = G(d14[:D])
        if self.big_rows:
            # fp32 M >= 512 (HCP): the quadratic-form factors W = P L on the 128x128 f32 kernel at per-factor offsets,
            # each problem's rows from the segment table (round 6: the grouped 64x64 kernel ran them at 21-28 TFLOP/s,
            # profiles/r04h_hcp_gemm_groups.jsonl).  Same products as d14.
            rsW = [(d, D - d) if not elbo_mode else (0, d + 1) for d in range(D)]
            bq_w = self._big_rows(self.P, self.WG, [3 * BM] * D, [sW + d * MM for d in range(D)],
                                  [d * BM for d in range(D)], rsW, L.B_LOWER, False)
            p["quad_W"] = bq_w
            bq_p = None
            if pairs and not self.pair_stream:
                sl = [((j, i) if not elbo_mode else (i, j)) for (i, j) in pairs]
                bq_p = self._big_rows(self.P, self.WP, [(2 if i == j else 1) * BM for (i, j) in pairs],
                                      [sU + pq(i, j) * MM for (i, j) in pairs], [s_ * BM for s_, _ in sl],
                                      [(r, 1) for _, r in sl], L.B_LOWER, False)
                if not elbo_mode:
                    p["quad_P"] = bq_p
            if elbo_mode:
                p["quad"] = H.Seq([bq_w] + ([pair_quad] if self.pair_stream else [bq_p] if bq_p is not None else []))
        if elbo_mode:
            self._plans[key] = p
            return p
        # B2: P-bar += W-hat L^T ; L-bar = P^T W-hat ; mu-bar = P^T adjoints
        # rows of output i: P-bar_G += sum_{d <= i} W-hat_d L_d^T.  Round 4: each latent factor's product is formed
        # once for every row that uses it, Z_d = W-hat_d[rows of outputs >= d] L_d^T (W-hat_d holds only those
        # rows; k = M per problem, short tiles), and nmgp_pbar_reduce adds Z_0 + ... + Z_i onto each row of output
        # i.  The round-3 form ran one k = (i + 1) M product per output: at PM2.5 a 40-k-tile loop per output tile
        # on the main chain (64 us, split-K capped), at ECoG (4 rows per output) up to 4096 k-tiles per tile.
        d17G = [g(self.Zg, self.WG, th, B, M, M, (M, 1, 0), (1, M, 0), (M, 1), flags=L.B_UPPER,
                  offs=(d * BM, sW + d * MM, d * BM), row_seg=d, seg_span=D - d) for d in range(D)]
        d17P = []
        for i in range(i0, i1):
            d17P.append(g(self.Pbar, self.WP, th, B, M, M, (M, 1, 0), (1, M, 0), (M, 1), flags=L.B_UPPER,
                          beta=1.0, offs=(i * BM, sU + pq(i, i) * MM, 2 * BM), row_seg=i))
            if i > 0:
                d17P.append(g(self.Pbar, self.WP, th, B, M, i * M, (M, 1, BM), (1, M, MM), (M, 1),
                              flags=L.B_UPPER, kb=(M, M), beta=1.0, offs=(0, sU + pq(i, 0) * MM, 1 * BM), row_seg=i))
        # the latent P-bar_G products feed R_G on the main chain; the pair P-bar_0/1 products feed only the
        # L0 / L1 prior adjoints and run on the third side stream.  In the per-factor Z_d form every P-bar_G
        # problem has k = M (a short loop of M/32 k-tiles), so no k-tile cap is needed.  (History: the round-3
        # per-output form ran k = (i + 1) M loops and capped them at 20 k-tiles per workgroup in fp64,
        # profiles/r03za_kt_cap_ab.txt.)
        p["bwd_wG"] = G(d17G)
        p["bwd_wP"] = G(d17P) if d17P else None
        if self.big_rows:
            # fp32 M >= 512: Z_d = W-hat_d L_d^T (rows of outputs >= d) on the 128x128 kernel; the pair P-bar in the
            # per-pair form Z_ij = W-hat_ij L_ij^T into slot j (rows of output i), summed onto P-bar_0 / P-bar_1 in
            # j order by nmgp_pair_pbar_reduce (the k-blocked d17P products sum the same terms in one k loop)
            p["bwd_wG"] = self._big_rows(self.WG, self.Zg, [d * BM for d in range(D)], [sW + d * MM for d in range(D)],
                                         [d * BM for d in range(D)], [(d, D - d) for d in range(D)], L.B_UPPER, True)
            if pairs and not self.pair_stream:
                dot = self._big_rows(self.WP, self.Zp, [j * BM for (i, j) in pairs],
                                     [sU + pq(i, j) * MM for (i, j) in pairs], [j * BM for (i, j) in pairs],
                                     [(i, 1) for (i, j) in pairs], L.B_UPPER, True)
                Zp_, Pb1_, Pb2_ = self.Zp, self.Pbar[1], self.Pbar[2]
                p["bwd_wP"] = H.Seq([dot, lambda s_: H.pair_pbar_reduce(Zp_, BM, Pb1_, Pb2_, M, seg, D, i0, i1, B, M,
                                                                        s_)])
        if self.pair_stream:
            # Z_ij = W-hat_ij L_ij^T into slot j (rows of output i), then P-bar_1 += Z_ii and P-bar_0 += Z_i0 + ...
            # + Z_i,i-1 in j order (csrc/pairs.hip pair_pbar_reduce)
            pair_dot = H.PairStream("dot", self.WP, th, self.Zp,
                                    [(j * BM, sU + pq(i, j) * MM, j * BM, i) for (i, j) in pairs], seg, M)
            Zp, Pb1, Pb2 = self.Zp, self.Pbar[1], self.Pbar[2]
            p["bwd_wP"] = H.Seq([pair_dot, lambda s_: H.pair_pbar_reduce(Zp, BM, Pb1, Pb2, M, seg, D, i0, i1, B, M,
                                                                         s_)])
        d17 = []
        if self.Ylb is not None:
            # round 4: one product per (output i, factor d <= i) over output i's rows into slot (i, d) of Ylb,
            # summed in i order onto factor d's gradient by nmgp_lbar_reduce -- every workgroup runs a k loop of
            # one output's rows, where one product per d ran the rows of outputs d..D-1 (at PM2.5 a 32-k-tile loop
            # per output tile of factor 0: the longest workgroup of the step).  The slots' upper triangles are
            # never written (OUT_LOWER: no zero tiles); the reduction sets the gradient's upper triangle to 0
            SY = MM + M
            for d in range(D):
                first = d * D - d * (d - 1) // 2
                for i in range(d, D):
                    s_ = (first + i - d) * SY
                    d17.append(g(self.Ylb, self.P, self.WG, M, M, B, (1, M, 0), (M, 1, 0), (M, 1), flags=L.OUT_LOWER,
                                 offs=(3 * BM, d * BM, s_), k_seg=i))
                    d17.append(g(self.Ylb, self.P, self.rowbuf, M, 1, B, (1, M, 0), (1, 1, 0), (1, 1),
                                 offs=(3 * BM, d * B, s_ + MM), k_seg=i))
        else:
            for d in range(D):
                d17.append(g(gr, self.P, self.WG, M, M, B, (1, M, 0), (M, 1, 0), (M, 1), flags=L.OUT_TRIL, beta=1.0,
                             offs=(3 * BM, d * BM, sW + d * MM), k_seg=d, seg_span=D - d))
                d17.append(g(gr, self.P, self.rowbuf, M, 1, B, (1, M, 0), (1, 1, 0), (1, 1), beta=1.0,
                             offs=(3 * BM, d * B, muW + d * M), k_seg=d, seg_span=D - d))
        for (i, j) in pairs:
            typ = 2 if i == j else 1
            if not self.pair_stream:
                d17.append(g(gr, self.P, self.WP, M, M, B, (1, M, 0), (M, 1, 0), (M, 1), flags=L.OUT_TRIL, beta=1.0,
                             offs=(typ * BM, j * BM, sU + pq(i, j) * MM), k_seg=i))
                d17.append(g(gr, self.P, self.rowbuf, M, 1, B, (1, M, 0), (1, 1, 0), (1, 1), beta=1.0,
                             offs=(typ * BM, (D + j) * B, muU + pq(i, j) * M), k_seg=i))
        # pair mu-bar on the pair kernel (round 6): mu-bar_ij += P_typ[rows of i]^T c_j, one block per pair instead of
        # M / 64 GEMM tiles with k ~ B / D
        pair_mv = H.PairStream("mv", self.P, self.rowbuf, gr,
                               [((2 if i == j else 1) * BM, (D + j) * B, muU + pq(i, j) * M, i) for (i, j) in pairs],
                               seg, M) if self.pair_stream else None
        # pair L-bar on the pair kernel: G_ij(lower) += P_typ[rows of i]^T W-hat_ij (the KL L-bar, this block's
        # first writer on the same stream, already zeroed the strictly upper part: OUT_TRIL)
        pair_rank = H.PairStream("rank", self.P, gr, self.WP,
                                 [((2 if i == j else 1) * BM, sU + pq(i, j) * MM, j * BM, i) for (i, j) in pairs],
                                 seg, M) if self.pair_stream else None
        if not self.big_side:
            p["bwd_lbar"] = G(d17) if pair_rank is None else H.Seq([G(d17), pair_rank, pair_mv])
        else:
            # the D + Q L-bar products P^T W (k over each factor's row segment) on the 128x128 kernel,
            # the M x 1 mu-bar products stay one grouped launch
            bw_w = H.BigBatch(self.P, self.WG, gr, [3 * BM] * D, [d * BM for d in range(D)],
                              [sW + d * MM for d in range(D)], M, M, B, lda=M, ldb=M, a_kcontig=False,
                              b_kcontig=False, flags=L.OUT_TRIL, beta=1.0,
                              kseg=(seg, list(range(D)), [D - d for d in range(D)]))
            bw_u = pair_rank if pair_rank is not None else H.BigBatch(
                self.P, self.WP, gr, [(2 if i == j else 1) * BM for (i, j) in pairs], [j * BM for (i, j) in pairs],
                [sU + pq(i, j) * MM for (i, j) in pairs], M, M, B, lda=M, ldb=M, a_kcontig=False, b_kcontig=False,
                flags=L.OUT_TRIL, beta=1.0, kseg=(seg, [i for (i, j) in pairs], [1] * len(pairs)))
            mu = G([dd for dd in d17 if dd.n == 1])
            p["bwd_lbar"] = H.Seq([bw_w, bw_u, mu] + ([pair_mv] if pair_mv is not None else []))
        # B3: R_k = Pbar_k Ainv_k (G,0,1) ; Abar_k = Cinv^T diag(delta) Cinv ; KL L-bar
        d18 = [g(self.R, self.Pbar, self.Ainv, B, M, M, (M, 1, 0), (M, 1, 0), (M, 1), offs=(k * BM, k * MM, k * BM),
                 **rows_all) for k in (3, 1, 2)]
        fb = self.facbuf
        for k in range(4):
            d18.append(g(self.Abar, self.Cinv, self.Cinv, M, M, M, (1, M, 0), (M, 1, 0), (M, 1),
                         flags=L.A_UPPER | L.B_LOWER, kscale=(fb, NF + k * M),
                         offs=((NF + k) * MM, (NF + k) * MM, k * MM)))
        for f in range(NFK):
            k = prior_of[f]
            d18.append(g(gr, self.Cinv, self.Xs, M, M, M, (1, M, 0), (M, 1, 0), (M, 1),
                         flags=L.A_UPPER | L.B_LOWER | L.OUT_TRIL | L.EPI_E_LOWER, alpha=-1.0, beta=1.0,
                         epi=(th, fac_off[f], (M, 1), (fb, NF + 4 * M + k * M), 1.0),
                         offs=(f * MM, f * MM, fac_off[f])))
        # R products on the main chain; the KL-only parts (prior adjoint init, L-bar of the variational
        # factors) depend on forward quantities only and run on the side stream, overlapped with
        # quad / recon (see _schedule)
        p["bwd_R"] = G(d18[:1])          # R_G: the main chain (Gibbs builder backward -> t chain)
        p["bwd_R_L"] = G(d18[1:3])       # R_0, R_1: only the L0/L1 hyper-parameter gradients need them
        p["kl_abar"] = G(d18[4:7] if p64 else d18[3:7])      # (p64: the t prior's below, in fp64)
        p["kl_lbar"] = G(d18[7:])
        if p64:
            X64 = self.pri_X64
            G64 = lambda descs: H.GemmGroup(descs, dev, F64, seg=seg)
            # A-bar_t = C_t^-T diag(delta_t) C_t^-1 and Y_t = A_t^-1 mu_v in fp64, then -1/2 Y_t Y_t^T
            p["kl_t64a"] = G64([g(self.Abt64, X64, X64, M, M, M, (1, M, 0), (M, 1, 0), (M, 1),
                                  flags=L.A_UPPER | L.B_LOWER, kscale=(self.dY64, 0), offs=(0, 0, 0)),
                                g(self.dY64, self.Ainv64, self.muv64, M, 1, M, (M, 1, 0), (1, M, 0), (1, M),
                                  offs=(0, 0, M))])
            p["kl_t64b"] = G64([g(self.Abt64, self.dY64, self.dY64, M, M, 1, (1, M, 0), (M, 1, 0), (M, 1),
                                  alpha=-0.5, beta=1.0, offs=(M, M, 0))]) if self.kl_owner else None
        if self.big_side:
            # KL L-bar of all NF factors: -C_f^-T Xs_f + diag(1/C_ii^2) L_f on the 128x128 kernel
            slots = [f * MM for f in range(NFK)]
            p["kl_lbar"] = H.BigBatch(self.Cinv, self.Xs, gr, slots, slots, fac_off[:NFK], M, M, M, lda=M, ldb=M,
                                      a_kcontig=False, b_kcontig=False,
                                      flags=L.A_UPPER | L.B_LOWER | L.OUT_TRIL | L.EPI_E_LOWER, alpha=-1.0, beta=1.0,
                                      epi=(th, fac_off[:NFK], (M, 1), fb,
                                           [NF + 4 * M + prior_of[f] * M for f in range(NFK)], 1.0))
            if self.kl_solve and FV > 0 and not elbo_mode:
                p["kl_lbar"] = self._kl_solve_lbar(th, gr, fb, fac_off, prior_of, NFK)
        # B4: Abar_k -= 1/2 Y_k diag(sel_k) Y_k^T
        ybase = [D * M, (D + 1) * M, (D + 1 + NPC) * M, 0]
        ncol = [1, NPC, NPC, D]
        sel_base = NF + 8 * M
        d19 = []
        for k in range(4):
            if (k == 0 and (not self.kl_owner or p64)) or (k == 3 and nW == 0):
                continue                          # KL_v / KL_W belong to another rank (p64: KL_v's in fp64)
            ks = (fb, sel_base + k * NPC) if k in (1, 2) else None
            d19.append(g(self.Abar, self.Y, self.Y, M, M, ncol[k], (1, M, 0), (M, 1, 0), (M, 1), alpha=-0.5,
                         beta=1.0, kscale=ks, offs=(ybase[k], ybase[k], k * MM)))
        p["bwd_kly"] = G(d19)
        # B5: Abar_k -= P_k^T R_k (G,0,1)
        pr = [g(self.Abar, self.P, self.R, M, M, B, (1, M, 0), (M, 1, 0), (M, 1), alpha=-1.0, beta=1.0,
                offs=(k * BM, k * BM, k * MM), k_seg=0, seg_span=D) for k in (3, 1, 2)]
        p["bwd_pr"] = G(pr[:1])
        p["bwd_pr_L"] = G(pr[1:])
        # B6: builder backward for G12, G22, L0_*, L1_*
        rbd = self.rowbuf
        so = self.scal_off
        bw = [H.pairwise_bwd_desc(self.x, self.Z, self.K12, self.R, mode=L.GIBBS, ld=M, Pm=self.P,
                                  rowcoef=(rbd, 2 * D * B), ellX=self.ellX, ellZ=self.ellZ, row_part=self.gib_row,
                                  col_part=self.gib_col, offs=(3 * BM, 3 * BM, 3 * BM, 0, 0, 0)),
              H.pairwise_bwd_desc(self.Z, self.Z, None, self.Abar, mode=L.GIBBS, ld=M, ellX=self.ellZ,
                                  ellZ=self.ellZ, row_part=self.gib_row, col_part=self.gib_col,
                                  offs=(0, 3 * MM, 0, self.n_ct * B, self.n_rt * M, 0))]
        for q, (k, hoff, rc) in enumerate([(1, hyp + 2, 2 * D + 1), (2, hyp + 4, 2 * D + 2)]):
            bw.append(H.pairwise_bwd_desc(self.x, self.Z, self.K12, self.R, mode=L.RBF, ld=M, Pm=self.P,
                                          rowcoef=(rbd, rc * B), hyp=th, hyp_off=hoff, hyp_log=True,
                                          scal_part=self.scal_part,
                                          offs=(k * BM, k * BM, k * BM, 0, 0, 2 * int(so[2 * q]))))
            bw.append(H.pairwise_bwd_desc(self.Z, self.Z, None, self.Abar, mode=L.RBF, ld=M, hyp=th, hyp_off=hoff,
                                          hyp_log=True, scal_part=self.scal_part,
                                          offs=(0, k * MM, 0, 0, 0, 2 * int(so[2 * q + 1]))))
        p["bwd_build12"] = H.PairwiseBwdGroup(bw[:1], dev)    # G12: ell_X adjoints (feeds the t chain)
        p["bwd_build22"] = H.PairwiseBwdGroup(bw[1:2], dev)   # G22: ell_Z adjoints (v chain only)
        p["bwd_build_L"] = H.PairwiseBwdGroup(bw[2:], dev)    # L0_*, L1_* (hyper-parameter partials only)
        # B7: t chain
        p["bwd_t1"] = G([g(self.R, self.Pbar, self.Ainv, B, M, M, (M, 1, 0), (M, 1, 0), (M, 1), offs=(0, 0, 0),
                           **rows_all)])
        # vbar[0:M] = P_t^T tbar: the v backward's only input from the t chain -- its own launch on the
        # side stream right after the t-row backward, so the v chain does not wait for R_t
        p["bwd_vt"] = G([g(self.vbar, self.P, self.rowbuf, M, 1, B, (1, M, 0), (1, 1, 0), (1, 1),
                           offs=(0, (2 * D + 3) * B, 0), k_seg=0, seg_span=D)])
        p["bwd_t2"] = G([g(self.Abar, self.P, self.R, M, M, B, (1, M, 0), (M, 1, 0), (M, 1), alpha=-1.0, beta=1.0,
                           offs=(0, 0, 0), k_seg=0, seg_span=D)])
        p["bwd_tbuild"] = H.PairwiseBwdGroup([
            H.pairwise_bwd_desc(self.x, self.Z, self.K12, self.R, mode=L.RBF, ld=M, Pm=self.P,
                                rowcoef=(rbd, (2 * D + 4) * B), hyp=th, hyp_off=hyp, hyp_log=True,
                                scal_part=self.scal_part, offs=(0, 0, 0, 0, 0, 2 * int(so[4]))),
            H.pairwise_bwd_desc(self.Z, self.Z, None, self.Abar, mode=L.RBF, ld=M, hyp=th, hyp_off=hyp,
                                hyp_log=True, scal_part=self.scal_part, offs=(0, 0, 0, 0, 0, 2 * int(so[5])))], dev)
        if p64:
            # the t-prior chain in fp64 from the t-row backward's fp64 P-bar_t / varbar: R_t = P-bar_t A_t^-1,
            # A-bar_t -= P_t^T R_t, builder backward (K_t12 - P_t K_t22 cancels to ~1e-4 P_t: the
            # sigma2 / length-scale partials of the t prior lost all digits in fp32 at ECoG length scales)
            G64 = lambda descs: H.GemmGroup(descs, dev, F64, seg=seg)
            p["bwd_t1"] = G64([g(self.Rt64, self.t64, self.Ainv64, B, M, M, (M, 1, 0), (M, 1, 0), (M, 1),
                                 offs=(0, 0, 0), **rows_all)])
            p["bwd_t2"] = G64([g(self.Abt64, self.P64, self.Rt64, M, M, B, (1, M, 0), (M, 1, 0), (M, 1), alpha=-1.0,
                                 beta=1.0, offs=(0, 0, 0), k_seg=0, seg_span=D)])
            p["bwd_tbuild"] = H.PairwiseBwdGroup([
                H.pairwise_bwd_desc(self.x64, self.Z64, self.K12_64, self.Rt64, mode=L.RBF, ld=M, Pm=self.P64,
                                    rowcoef=(self.t64, B * M), hyp=self.hyp64, hyp_off=0, hyp_log=True,
                                    scal_part=self.scal64, offs=(0, 0, 0, 0, 0, 2 * int(so[4]))),
                H.pairwise_bwd_desc(self.Z64, self.Z64, None, self.Abt64, mode=L.RBF, ld=M, hyp=self.hyp64,
                                    hyp_off=0, hyp_log=True, scal_part=self.scal64,
                                    offs=(0, 0, 0, 0, 0, 2 * int(so[5])))], dev)
            # L0 / L1: R_k = P-bar_k A_k^-1, A-bar_k -= P_k^T R_k, builder backward, all fp64 (k = 1, 2)
            p["bwd_R_L"] = G64([g(self.RL64, self.PbL64, self.Ainv64, B, M, M, (M, 1, 0), (M, 1, 0), (M, 1),
                                  offs=(q * BM, (q + 1) * MM, q * BM), **rows_all) for q in range(2)])
            p["bwd_pr_L"] = G64([g(self.AbL64, self.P64, self.RL64, M, M, B, (1, M, 0), (M, 1, 0), (M, 1),
                                   alpha=-1.0, beta=1.0, offs=((q + 1) * BM, q * BM, q * MM), k_seg=0, seg_span=D)
                                 for q in range(2)])
            bwL = []
            for q, hoff in ((0, 2), (1, 4)):
                bwL.append(H.pairwise_bwd_desc(self.x64, self.Z64, self.K12_64, self.RL64, mode=L.RBF, ld=M,
                                               Pm=self.P64, rowcoef=(self.rcL64, q * B), hyp=self.hyp64,
                                               hyp_off=hoff, hyp_log=True, scal_part=self.scal64,
                                               offs=((q + 1) * BM, q * BM, (q + 1) * BM, 0, 0, 2 * int(so[2 * q]))))
                bwL.append(H.pairwise_bwd_desc(self.Z64, self.Z64, None, self.AbL64, mode=L.RBF, ld=M,
                                               hyp=self.hyp64, hyp_off=hoff, hyp_log=True, scal_part=self.scal64,
                                               offs=(0, q * MM, 0, 0, 0, 2 * int(so[2 * q + 1]))))
            p["bwd_build_L"] = H.PairwiseBwdGroup(bwL, dev)
        # B9: v Cholesky backward: grad_sv += Cinv_v^T (Psi Xs_v)
        p["bwd_v1"] = G([g(self.T2, self.phi, self.Xs, M, M, M, (M, 1, 0), (M, 1, 0), (M, 1), flags=L.B_LOWER,
                           offs=(0, FV * MM, 0))])
        p["bwd_v2"] = G([g(gr, self.Cinv, self.T2, M, M, M, (1, M, 0), (M, 1, 0), (M, 1),
                           flags=L.A_UPPER | L.OUT_TRIL, beta=1.0, offs=(FV * MM, 0, sv))])
        self._plans[key] = p
        return p

    # ------------------------------------------------------------------------------------ data
    def load_batch(self, x, y, sizes, noise=None, index=None):
        """Copy one minibatch (rows grouped by output, `sizes` rows per list entry) to the device."""
        D, B = self.D, self.B
        sizes = [int(s) for s in sizes]
        assert sum(sizes) == B, (sum(sizes), B)
        ids = list(range(len(sizes))) if index is None else [int(i) for i in index]
        if len(ids) != len(sizes) or any(i < 0 or i >= D for i in ids):
            raise ValueError(f"index {ids} must give one output id in [0, {D}) per input list")
        # rows of output j in the reference's row order (code/nmgp_dsvi.py:163-169 with `index`): the
        # engine addresses outputs as contiguous segments, so rows (and their per-row noise) are put in
        # output order, stably -- the objective is a sum over rows, invariant to that permutation
        row_ids = np.repeat(np.asarray(ids, np.int64), sizes)
        order = np.argsort(row_ids, kind="stable")
        perm = not np.array_equal(order, np.arange(B))
        seg = np.concatenate([[0], np.cumsum(np.bincount(row_ids, minlength=D))]).astype(np.int32)
        row_out = row_ids[order].astype(np.int32)
        xv = np.asarray(x, np.float64).reshape(-1)
        yv = np.asarray(y, np.float64).reshape(-1)
        self.x.copy_(torch.as_tensor(xv[order] if perm else xv).to(self.dt))
        self.y.copy_(torch.as_tensor(yv[order] if perm else yv).to(self.dt))
        self.seg.copy_(torch.from_numpy(seg))
        self.row_out.copy_(torch.from_numpy(row_out))
        # kept for load_noise: later noise draws for the same batch (compute_ELBO's further samples)
        # must be regrouped exactly like the rows
        self._row_order = torch.from_numpy(order) if perm else None
        if noise is not None:
            self.load_noise(noise)

    def load_noise(self, noise):
        """Copy one step's host noise (z_v (M), z_t (B), then Q x (B) pair rows, the reference's draw
        order) into the engine, its per-row parts permuted like the rows of the batch last loaded by
        load_batch (rows regrouped by output when `index` was not in output order)."""
        M, B, Q = self.M, self.B, self.Q
        nz = torch.as_tensor(noise, dtype=F64).reshape(-1)
        if nz.numel() != M + B + Q * B:
            raise ValueError(f"noise has {nz.numel()} values, the step draws M + B + Q*B = {M + B + Q * B}")
        o = getattr(self, "_row_order", None)
        if o is not None:
            nz = torch.cat([nz[:M], nz[M:M + B][o], nz[M + B:].reshape(Q, B)[:, o].reshape(-1)])
        self.noise.copy_(nz.to(self.dt))

    def bind_dataset(self, Xb, Yb, Ib, Sb, counter=None):
        """Keep an epoch of pre-split minibatches resident in HBM (Xb, Yb (nb, B) engine dtype; Ib (nb, B) int32
        output ids; Sb (nb, D+1) int32 segment tables, rows grouped by output as vec2list makes them).
        Each step then starts with ONE gather launch (batch (*counter) % nb, counter advanced on the
        device), so a captured step graph walks the epoch by itself."""
        nb, B = Xb.shape
        assert B == self.B and Sb.shape == (nb, self.D + 1)
        for t, dt in ((Xb, self.dt), (Yb, self.dt), (Ib, torch.int32), (Sb, torch.int32)):
            assert t.is_cuda and t.dtype == dt and t.is_contiguous()
        if counter is None:
            counter = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self._dataset = (Xb, Yb, Ib, Sb, counter)
        self._sched_key = None
        return counter

    def gather_batch(self, stream=None):
        Xb, Yb, Ib, Sb, ctr = self._dataset
        s = L.stream_handle() if stream is None else stream
        L.check(getattr(L.lib(), "nmgp_batch_gather_" + self.sfx)(*(ctypes.c_void_p(t.data_ptr()) for t in (Xb, Yb, Ib, Sb)), self.B,
                                              self.D + 1, Xb.shape[0], ctypes.c_void_p(ctr.data_ptr()),
                                              *(ctypes.c_void_p(t.data_ptr()) for t in (self.x, self.y, self.row_out,
                                                                                        self.seg)), s),
                "batch_gather")

    def set_adam_step(self, step):
        """Round 6: the training schedule's finalize launch advances `step` (an int64 device counter) at its end
        (nmgp_dsvi_args.adam_step; None: off).  Set around a capture only (DsviTrainer.capture), after the warm-up
        built the schedule: launches copy the argument struct when they are issued."""
        ptr = None if step is None else ctypes.c_void_p(step.data_ptr())
        for (elbo_mode, _), a in getattr(self, "_keep_args", {}).items():
            if not elbo_mode:
                a.adam_step = ptr

    def begin_step(self, seed, counter, stream=None):
        """Gather + device noise + noise-counter advance + gradient zeroing in one launch
        (nmgp_step_begin_*); the forward_backward that follows must not zero the gradient again."""
        Xb, Yb, Ib, Sb, ctr = self._dataset
        if getattr(self, "_begin_done", None) is None:
            self._begin_done = torch.zeros(1, dtype=torch.int32, device=self.dev)
        s = L.stream_handle() if stream is None else stream
        vp = ctypes.c_void_p
        L.check(getattr(L.lib(), "nmgp_step_begin_" + self.sfx)(
            *(vp(t.data_ptr()) for t in (Xb, Yb, Ib, Sb)), self.B, self.D + 1, Xb.shape[0], vp(ctr.data_ptr()),
            *(vp(t.data_ptr()) for t in (self.x, self.y, self.row_out, self.seg)), vp(self.noise.data_ptr()),
            self.noise.numel(), ctypes.c_uint64(seed), vp(counter.data_ptr()), vp(self._begin_done.data_ptr()),
            vp(self._grad.data_ptr()), self._grad.numel(), s), "step_begin")

    def begin_forward_backward(self, seed, counter):
        """begin_step + forward_backward(zero_grad=False), back to back on the current stream.  (Round 3 measured
        the step-begin launch on its own stream beside the theta-only head of the forward chain: bit-identical,
        6% slower -- profiles/r03zh_early_begin_ab.txt.)"""
        self.begin_step(seed, counter)
        return self.forward_backward(zero_grad=False)

    def device_noise(self, seed, counter):
        H.normal_(self.noise, seed, counter=counter)   # dtype-dispatched Philox normals

    # ------------------------------------------------------------------------------------ step
    def _call(self, fn, a, s):
        L.check(fn(ctypes.byref(a), s), fn.__name__)

    def _schedule(self, elbo_mode, with_kl=True, cached=False):
        """The ordered launch list of one step.  Items are (name, kind, callable(stream), where) with where
        one of the four streams, plus ("sig", stream, tag) / ("wait", stream, tag) event edges: the D+Q
        variational factors that only the KL terms need are factored on a side stream, overlapping the
        forward chain; the backward's independent chains run on three side streams."""
        lib = L.lib()
        D, M, NF = self.D, self.M, self.NF
        MM = M * M
        FV = NF - 1
        fuse = self.fuse_tp
        p = self._plan(elbo_mode)
        a = self._args(elbo_mode)
        self._keep_args = getattr(self, "_keep_args", {})
        self._keep_args[(elbo_mode, with_kl)] = a
        Af, Ci, info = self.Afac.data_ptr(), self.Cinv.data_ptr(), self.info.data_ptr()
        vp = ctypes.c_void_p

        def row(fn):
            return lambda s: L.check(fn(ctypes.byref(a), s), fn.__name__)

        # segment-sized groups of the training step whose tile plans are computed ahead, on the side
        # stream right after the minibatch gather (off the main chain)
        pre_planned = set()
        if not elbo_mode:
            pre_planned = {nm for nm in ("quad", "quad_W", "bwd_wG", "bwd_wP")
                           if isinstance(p.get(nm), H.GemmGroup) and p[nm].plan is not None}

        def gemm(name):
            if name in pre_planned:
                return lambda s: p[name](s, planned=True)
            return lambda s: p[name](s)

        pbar_fn = getattr(lib, "nmgp_pbar_reduce_" + self.sfx)
        esz = self.Pbar.element_size()

        def pbar_reduce(s):
            # P-bar_G (slot 3) rows += Z_0 + ... + Z_i, i the row's output
            L.check(pbar_fn(vp(self.Zg.data_ptr()), self.B * M, vp(self.Pbar.data_ptr() + 3 * self.B * M * esz), M,
                            vp(self.seg.data_ptr()), D, self.B, M, s), "pbar_reduce")

        lbar_fn = getattr(lib, "nmgp_lbar_reduce_" + self.sfx)

        def lbar_reduce(s):
            # latent L-bar / mu-bar gradient rows += Y_{d,d} + ... + Y_{D-1,d} (bwd_lbar's per-output products)
            gp = self._grad.data_ptr()
            L.check(lbar_fn(vp(self.Ylb.data_ptr()), M * M + M, vp(gp + self.offs["sqrt_W"][0] * esz), M * M,
                            vp(gp + self.offs["mu_W"][0] * esz), M, D, M, s), "lbar_reduce")

        def plans(s):
            for nm in sorted(pre_planned):
                p[nm].plan_now(s)

        def pw(name):
            return lambda s: p[name](self.dt, s)

        def pw64(name):
            return lambda s: p[name](F64, s)

        conv_up32, conv_dn64 = lib.nmgp_convert_f32_to_f64, lib.nmgp_convert_f64_to_f32

        def widen(src, dst, n, src_off=0):
            # fp32 -> fp64 copy of n elements (the fp64 path's inputs)
            return lambda s: L.check(conv_up32(vp(src.data_ptr() + 4 * src_off), vp(dst.data_ptr()), n, s), "convert")

        def conv_in(s):
            widen(self.x, self.x64, self.B)(s)
            widen(self._theta, self.hyp64, 7, self.offs["sigma2_tildeell_log"][0])(s)
            widen(self._theta, self.sv64, MM, self.offs["sqrt_v"][0])(s)
            widen(self._theta, self.muv64, M, self.offs["mu_v"][0])(s)

        def round_back(k0, cnt):
            # fp64 P / prior inverses of priors k0 .. k0+cnt-1 -> the fp32 buffers the fp32 kernels read
            def run(s):
                BM_, MM_ = self.B * self.M, self.M * self.M
                L.check(conv_dn64(vp(self.P64.data_ptr() + 8 * k0 * BM_), vp(self.P.data_ptr() + 4 * k0 * BM_),
                                  cnt * BM_, s), "convert")
                L.check(conv_dn64(vp(self.Ainv64.data_ptr() + 8 * k0 * MM_), vp(self.Ainv.data_ptr() + 4 * k0 * MM_),
                                  cnt * MM_, s), "convert")
            return run

        chol_fn = getattr(lib, "nmgp_chol_inv_batched_" + self.sfx)

        def chol(first, count, blockinv=False):
            # fused factor + inverse: Afac <- L (in place), Cinv <- L^{-1} (blockinv: the inverses of the two
            # diagonal blocks of the top-level split only -- the KL L-bar solve form)
            es = self.Afac.element_size()
            fn = lib.nmgp_chol_blockinv_batched_f32 if blockinv else chol_fn
            return lambda s: L.check(fn(vp(Af + first * MM * es), M, M, MM, vp(Ci + first * MM * es), M, MM, count,
                                        vp(info + first * 4), s), "chol_inv")

        if self.prior64:
            conv_up, conv_dn = lib.nmgp_convert_f32_to_f64, lib.nmgp_convert_f64_to_f32
            chol64 = lib.nmgp_chol_inv_batched_f64
            A64, X64 = self.pri_A64.data_ptr(), self.pri_X64.data_ptr()
            es = self.Afac.element_size()

            def chol_prior(k0, cnt, v_too=False):
                # slots NF + k0 .. NF + k0 + cnt - 1: up-convert K22 + lam I (built in fp64 already with the
                # fp64 projections), fp64 factor + inverse, round L and L^-1 back into the fp32 slots (info as
                # the fp32 kernel reports it)
                if v_too and self.p64:
                    # Sigma_v + lam I (fp64 syrk) and the three RBF priors: one fp64 batch of 4 from slot FV
                    VA, VX, n4 = self.v_A64.data_ptr(), self.v_X64.data_ptr(), 4 * MM

                    def run4(s):
                        L.check(chol64(vp(VA), M, M, MM, vp(VX), M, MM, 4, vp(info + FV * 4), s),
                                "chol_inv f64 prior")
                        L.check(conv_dn(vp(VA), vp(Af + FV * MM * es), n4, s), "convert")
                        L.check(conv_dn(vp(VX), vp(Ci + FV * MM * es), n4, s), "convert")
                    return run4
                f32 = chol(FV, 1) if v_too else None
                n = cnt * MM

                def run(s):
                    if f32 is not None:
                        f32(s)
                    src = vp(Af + (NF + k0) * MM * es)
                    if not self.p64:
                        L.check(conv_up(src, vp(A64 + k0 * MM * 8), n, s), "convert")
                    L.check(chol64(vp(A64 + k0 * MM * 8), M, M, MM, vp(X64 + k0 * MM * 8), M, MM, cnt,
                                   vp(info + (NF + k0) * 4), s), "chol_inv f64 prior")
                    L.check(conv_dn(vp(A64 + k0 * MM * 8), src, n, s), "convert")
                    L.check(conv_dn(vp(X64 + k0 * MM * 8), vp(Ci + (NF + k0) * MM * es), n, s), "convert")
                return run
            chol_main, chol_g = chol_prior(0, 3, v_too=True), chol_prior(3, 1)
        else:
            chol_main, chol_g = chol(FV, 4), chol(NF + 3, 1)
        if fuse:
            chol_main, chol_g = p["chol_tp_main"], p["chol_tp_G"]

        kf0, kf1 = p["kl_range"]
        need_side = (not elbo_mode) or (with_kl and kf1 > kf0)
        steps = []
        # Streams: main (the forward / backward dependency chain), side (variational factors, KL, L-bar, v
        # chain), side2 (t-prior projections, t-row, K_G12, pair quad forms; in the backward the G-prior
        # adjoint), side3 (pair P-bar and the L0 / L1 prior adjoints).  side2 and side3 synchronise with the
        # main stream and one-way with side, never side <-> side2 both ways: hipStreamEndCapture of the HIP
        # runtime this process runs (torch's bundled ROCm 7.0 libamdhip64) segfaults on such a ping-pong, so
        # those edges are relayed through main (quad_P plans inline on side2).  In a replayed graph
        # a node's FIRST-created child keeps its hardware queue and every other child starts on another queue
        # behind a cross-queue barrier (10-20 us per hop in the r03 traces), so the critical-path child of each
        # fork is captured first (v after chol, quad_W after projG, bwd_R after bwd_wG, bwd_t1 after tbwd).
        # Sigma_v: fp64 engines without the fused priors form it first on the side stream (one small launch beside
        # the RBF builders on main); in fp32 its summation order shows through ell_Z = exp(v), so fp32 engines keep
        # the grouped main launch.  Fused priors: the RBF K22 and Sigma_v both on main, after the side stream's
        # first launch (side keeps the hardware queue; on the side stream the fused launch waited for a cross-queue
        # hand-off after them: 0.671 -> 0.667 ms A/B, profiles/r06q_head_main_after_fork_ab.txt)
        v_on_side = need_side and not elbo_mode and self.dt == torch.float64 and not fuse
        if need_side:
            steps += [("sig", "main", "fork"), ("wait", "side", "fork")]
            if v_on_side:
                steps += [("syrk", "gemm", gemm("syrk"), "side"), ("sig", "side", "syrk")]
            steps.append(("syrk_side", "gemm", gemm("syrk_side"), "side"))
            if pre_planned:
                steps += [("plans", "gemm_plan", plans, "side"), ("sig", "side", "plans")]
            side_fac = [("chol_side", "chol", chol(kf0, kf1 - kf0, self.kl_solve and not elbo_mode), "side")]
            if not elbo_mode:
                side_fac.append(("xs_side", "gemm", gemm("xs_side"), "side"))
            side_after = fuse
            if not side_after:
                steps += side_fac
                side_fac = []
        if self.p64:
            steps += [("conv_in", "convert", conv_in, "main"),
                      ("build_rbf64", "pairwise", pw64("build_rbf64"), "main")]
        if not fuse:
            steps.append(("build_rbf", "pairwise", pw("build_rbf"), "main"))
        else:
            steps.append(("build_k22", "pairwise", pw("build_k22"), "main"))
        steps.append(("wait", "main", "syrk") if v_on_side else ("syrk", "gemm", gemm("syrk"), "main"))
        # forward chain: chol -> v -> K_G22 -> chol_G -> invG -> projG.  The t-prior projections, the
        # t-row (ell_X) and K_G12 run on the second side stream beside v / K_G22 / chol_G: they are
        # needed only from invG on (T_G = K_G12 C_G^-T)
        side_fac = side_fac if need_side else []
        steps += [
            ("chol", "chol", chol_main, "main"),
            ("sig", "main", "chol"),
        ]
        vg_in_chol = fuse and self.fuse_vg and not elbo_mode
        if not vg_in_chol:
            steps += [
                # fused: v and K_G22 + lam I in one wide launch (dsvi_vg22_kernel)
                ("v", "row", row(getattr(lib, ("nmgp_dsvi_vg22_" if fuse else "nmgp_dsvi_hyper_") + self.sfx)), "main"),
            ]
        steps.append(("sig", "main", "v"))
        if vg_in_chol:
            # the Gibbs launch follows the first one directly: captured before the other streams' waits on it, so
            # that it is the first launch's first child and keeps its hardware queue
            steps += [("chol_G", "chol", chol_g, "main"), ("sig", "main", "cholG")]
        if side_fac:        # the variational factors' batched factorization after the fused prior launch
            steps += [("wait", "side", "chol")] + side_fac
        steps.append(("wait", "side2", "chol"))
        if self.p64:
            steps += [("inv3_64", "gemm", gemm("inv3_64"), "side2"),
                      ("proj3_64", "gemm", gemm("proj3_64"), "side2"),
                      ("conv3", "convert", round_back(0, 3), "side2")]
        if fuse:
            # fused priors: T / P of t, L0, L1 came with their factorization; side2 runs the pair factors W_P first
            # (recon waits for them), then the prior inverses and Y = A^-1 mu (KL and backward only); the Gibbs
            # prior's launch on the main stream forms the t-row, K_G12, T_G and P_G itself
            qp = [("quad_P", "gemm", gemm("quad_P"), "side2"), ("sig", "side2", "quadP")] if not elbo_mode else []
            i3 = [("inv3", "gemm", gemm("inv3"), "side2"), ("proj3", "gemm", gemm("proj3"), "side2")]
            steps += i3 + qp
            if not vg_in_chol:
                steps += [("chol_G", "chol", chol_g, "main"), ("sig", "main", "cholG")]
        else:
            if p["inv3"] is not None:
                steps.append(("inv3", "gemm", gemm("inv3"), "side2"))
            steps += [
                ("proj3", "gemm", gemm("proj3"), "side2"),
                ("build_g22", "pairwise", (pw64 if self.p64 else pw)("build_g22"), "main"),
                ("wait", "side2", "v"),
                ("trow", "row", row(getattr(lib, "nmgp_dsvi_trow_" + self.sfx)), "side2"),
            ]
            if self.p64:
                steps.append(("conv_ellX", "convert", widen(self.ellX, self.ellX64, self.B), "side2"))
            steps.append(("build_g12", "pairwise", pw("build_g12"), "side2"))
            if self.p64:
                steps.append(("build_g12_64", "pairwise", pw64("build_g12_64"), "side2"))
            steps.append(("sig", "side2", "g12"))
            if not elbo_mode:
                # the pair factors W_P = P_{0,1} L_ij need only the L0 / L1 projections: beside the Gibbs chain
                steps += [("quad_P", "gemm", gemm("quad_P"), "side2"), ("sig", "side2", "quadP")]
            steps += [
                ("chol_G", "chol", chol_g, "main"),
                ("wait", "main", "g12"),
            ]
            if self.p64:
                steps += [("invG_64", "gemm", gemm("invG_64"), "main"),
                          ("projG_64", "gemm", gemm("projG_64"), "main"),
                          ("convG", "convert", round_back(3, 1), "main")]
            else:
                steps.append(("invG", "gemm", gemm("invG"), "main"))
            steps.append(("projG", "gemm", gemm("projG"), "main"))
        # fused: A_G^-1 and Y_G = A_G^-1 mu_W (KL_W, R_G) on side2 after the Gibbs launch, captured after the main
        # stream's next launch so that the chain's child keeps the hardware queue
        invG_side = [("wait", "side2", "cholG"), ("invG", "gemm", gemm("invG"), "side2"),
                     ("projG", "gemm", gemm("projG"), "side2"), ("sig", "side2", "kl_in")] if fuse else []
        if elbo_mode:
            steps.append(("quad", "gemm", gemm("quad"), "main"))
            steps += invG_side
            if need_side:
                steps += [("sig", "side", "join"), ("wait", "main", "join")]
            if with_kl:
                if fuse:
                    steps.append(("wait", "main", "kl_in"))
                steps.append(("kl", "row", row(getattr(lib, "nmgp_dsvi_kl_" + self.sfx)), "main"))
            steps += [("recon", "row", row(getattr(lib, "nmgp_dsvi_recon_" + self.sfx)), "main"),
                      ("finalize", "row", row(getattr(lib, "nmgp_dsvi_finalize_" + self.sfx)), "main")]
            if cached:
                # sample-independent work of an earlier sample of the same compute_ELBO call is reused:
                # the RBF priors t, L0, L1 (builds, factors, inverses, projections P / T / Y), chol(Sigma_v)
                # and the pair quadratic-form factors W_P; per sample only v, ell_X, the Gibbs prior and
                # the latent-function factors W_G are recomputed (code/nmgp_dsvi.py:330-376)
                skip = {"build_rbf", "build_k22", "syrk", "chol", "inv3", "proj3",
                        "conv_in", "build_rbf64", "inv3_64", "proj3_64", "conv3"}
                steps = [it for it in steps if not (len(it) == 4 and it[0] in skip)]
                steps = [("quad_W",) + it[1:] if len(it) == 4 and it[0] == "quad" else it for it in steps]
                steps = [(it[0], it[1], gemm("quad_W"), it[3]) if it[0] == "quad_W" else it for it in steps]
            return steps
        # KL branch on the side stream once all prior factors and Y = A^-1 mu exist (after projG):
        # KL terms, prior-diagonal adjoints, the variational factors' KL L-bar (first writer of those
        # gradient rows -- bwd_lbar follows it on the same stream, so the accumulation order is fixed) and the
        # KL part of the prior adjoints Abar (the main stream waits for it before R_G is signalled)
        if not fuse:
            steps.append(("sig", "main", "kl_in"))
        if pre_planned:
            steps.append(("wait", "main", "plans"))
        steps.append(("quad_W", "gemm", gemm("quad_W"), "main"))
        steps += invG_side
        steps += [
            ("wait", "side", "kl_in"),
            ("kl", "row", row(getattr(lib, "nmgp_dsvi_kl_" + self.sfx)), "side"),
            ("delta", "row", row(getattr(lib, "nmgp_dsvi_delta_" + self.sfx)), "side"),
        ]
        if self.p64:
            steps += [("conv_d64", "convert", widen(self.facbuf, self.dY64, M, NF), "side"),
                      ("kl_t64a", "gemm", gemm("kl_t64a"), "side")]
            if p["kl_t64b"] is not None:
                steps.append(("kl_t64b", "gemm", gemm("kl_t64b"), "side"))
        steps += [
            ("kl_lbar", "gemm", gemm("kl_lbar"), "side"),
            ("sig", "side", "kl_lbar"),
            ("kl_abar", "gemm", gemm("kl_abar"), "side"),
            ("bwd_kly", "gemm", gemm("bwd_kly"), "side"),
            ("sig", "side", "kl_done"),
            ("wait", "main", "quadP"),
            ("recon", "row", row(getattr(lib, "nmgp_dsvi_recon_" + self.sfx)), "main"),
            ("sig", "main", "recon"),
        ]
        wp_first = fuse and p["bwd_wP"] is not None
        if wp_first:
            steps += [("wait", "side3", "recon"), ("bwd_wP", "gemm", gemm("bwd_wP"), "side3")]
        steps += [
            ("bwd_wG", "gemm", gemm("bwd_wG"), "main"),
            ("bwd_wGr", "row", pbar_reduce, "main"),
        ]
        if fuse:
            steps.append(("wait", "main", "kl_in"))      # R_G = P-bar_G A_G^-1 (side2's invG, long done)
        steps += [
            ("bwd_R", "gemm", gemm("bwd_R"), "main"),
            # L-bar / mu-bar gradient rows: after the KL L-bar (their first writer, same stream) and recon.
            ("wait", "side", "recon"),
            # the recon row partials and the KL slabs summed here, off the main chain (finalize adds them)
            ("prefinal", "row", row(getattr(lib, "nmgp_dsvi_prefinal_" + self.sfx)), "side"),
        ]
        lbar_steps = [("bwd_lbar", "gemm", gemm("bwd_lbar"), "side")]
        if self.Ylb is not None:
            lbar_steps.append(("bwd_lbr", "row", lbar_reduce, "side"))
        lbar_steps.append(("sig", "side", "lbar_done"))
        # (bwd_lbar after R_G instead, so that it does not compete with the P-bar_G -> R_G chain for CUs: 1380 ->
        # 1270 it/s, profiles/r04s_lbar_per_output_ab.txt.  Round 6, HCP / ECoG: bwd_lbar on the idle main stream
        # before the KL L-bar, beside the factor chain: ECoG 0.2764 -> 0.2747 s, HCP 58.7 -> 57.4 it/s, not kept --
        # profiles/r06zh_kl_solve_lbar_early_ab.txt)
        steps += lbar_steps
        BM = self.B * M
        # the pair P-bar_0/1 products start on the third side stream right after recon (beside bwd_wG), then --
        # with the KL parts of A-bar_0/1 (kl_done, a one-way side -> side3 edge) -- the L0 / L1 prior adjoints
        # R_0/1 -> P^T R -> builder backward (hyper-parameter partials only; p64: P-bar_0/1, the KL parts of
        # A-bar_0/1 and the row coefficients c0 / c1 widened first)
        if not wp_first:
            steps.append(("wait", "side3", "recon"))
            if p["bwd_wP"] is not None:
                steps.append(("bwd_wP", "gemm", gemm("bwd_wP"), "side3"))
        steps.append(("wait", "side3", "kl_done"))
        if self.p64:
            steps += [("wPbL", "convert", widen(self.Pbar, self.PbL64, 2 * BM, BM), "side3"),
                      ("wrcL", "convert", widen(self.rowbuf, self.rcL64, 2 * self.B, (2 * D + 1) * self.B), "side3")]
        steps.append(("bwd_R_L", "gemm", gemm("bwd_R_L"), "side3"))
        if self.p64:
            steps.append(("wAbL", "convert", widen(self.Abar, self.AbL64, 2 * MM, MM), "side3"))
        steps += [
            ("bwd_pr_L", "gemm", gemm("bwd_pr_L"), "side3"),
            ("bwd_build_L", "pairwise_bwd", (pw64 if self.p64 else pw)("bwd_build_L"), "side3"),
            ("sig", "side3", "L_done"),
            # (the KL part of Abar_G reaches side2 through main: the KL branch is long finished when bwd_R is)
            ("wait", "main", "kl_done"),
            ("sig", "main", "R_G"),
            # G prior: R_G -> the K_G12 builder backward (ell_X adjoints) stays on the main chain; the prior
            # adjoint Abar_G -= P_G^T R_G and the K_G22 builder backward (ell_Z adjoints: the v chain only) run
            # on the second side stream
            ("bwd_build12", "pairwise_bwd", pw("bwd_build12"), "main"),
            ("wait", "side2", "R_G"),
            ("bwd_pr", "gemm", gemm("bwd_pr"), "side2"),
            ("bwd_build22", "pairwise_bwd", pw("bwd_build22"), "side2"),
            ("sig", "side2", "g22"),
            # after the t-row backward the t-prior chain (bwd_t1 -> bwd_t2 -> builder backward) and the v-factor
            # Cholesky backward (P_t^T tbar -> vbwd -> bwd_v1 -> bwd_v2, reading vbar and the Gibbs partials)
            # share no buffer: the v chain runs on the side stream (after bwd_lbar there, which keeps the order
            # of the sqrt_v gradient accumulation fixed: kl_lbar, bwd_lbar, bwd_v2), waiting for the K_G22
            # builder backward itself (a one-way side2 -> side edge), followed by the KL mean gradients
            ("tbwd", "row", row(getattr(lib, "nmgp_dsvi_tbwd_" + self.sfx)), "main"),
            ("sig", "main", "tb"),
            ("bwd_t1", "gemm", gemm("bwd_t1"), "main"),
        ]
        vchain = [("bwd_vt", "gemm", gemm("bwd_vt"), None),      # (reads P_t and tbar only)
                  ("vbwd", "row", row(getattr(lib, "nmgp_dsvi_vbwd_" + self.sfx)), None),
                  ("bwd_v1", "gemm", gemm("bwd_v1"), None),
                  ("bwd_v2", "gemm", gemm("bwd_v2"), None)]
        # (the KL mean gradients -- after bwd_lbar's mu products and vbwd's vbar -- are added by finalize)
        if fuse:
            # the v chain on side2 behind the K_G22 builder backward (its Gibbs partials; the KL L-bar -- first writer
            # of the sqrt_v rows -- is done: side2 waited for R_G, which followed kl_done), not behind bwd_lbar on
            # the side stream
            steps += [("wait", "side2", "tb")] + [it[:3] + ("side2",) for it in vchain] + [("sig", "side2", "v_done")]
            steps += [("bwd_t2", "gemm", gemm("bwd_t2"), "main"),
                      ("bwd_tbuild", "pairwise_bwd", (pw64 if self.p64 else pw)("bwd_tbuild"), "main"),
                      ("wait", "main", "v_done"), ("wait", "main", "lbar_done")]
        else:
            steps += [("wait", "side", "tb"), vchain[0][:3] + ("side",), ("wait", "side", "g22")]
            steps += [it[:3] + ("side",) for it in vchain[1:]] + [("sig", "side", "v_done")]
            steps += [("bwd_t2", "gemm", gemm("bwd_t2"), "main"),
                      ("bwd_tbuild", "pairwise_bwd", (pw64 if self.p64 else pw)("bwd_tbuild"), "main"),
                      ("wait", "main", "v_done"), ("wait", "main", "lbar_done")]
        steps += [
            ("wait", "main", "L_done"),
            ("wait", "main", "g22"),          # (explicit join of side2; long done)
        ]
        # the KL mean gradients: inside finalize for small engines, else their own launch first (include/nmgp_hip.h
        # NMGP_MUGRAD_IN_FINALIZE_MAX; the same count as csrc/dsvi.hip mugrad_count)
        if D * M + M + self.NPC * M > MUGRAD_IN_FINALIZE_MAX:
            steps.append(("mugrad", "row", row(getattr(lib, "nmgp_dsvi_mugrad_" + self.sfx)), "main"))
        steps.append(("finalize", "row", row(getattr(lib, "nmgp_dsvi_finalize_" + self.sfx)), "main"))
        return steps

    def _run(self, steps, stream, timer):
        """Enqueue `steps`.  timer=None: on the four streams.  A timer with concurrent=False: serially on
        one stream, every launch bracketed by events (isolated launch times).  concurrent=True: on the four
        streams as in the graph, each launch bracketed by events on ITS stream (recorded after its
        cross-stream waits), so the durations include the contention with the other streams' kernels."""
        main = stream if stream is not None else torch.cuda.current_stream(self.dev)
        s_main = ctypes.c_void_p(main.cuda_stream)
        conc = timer is not None and getattr(timer, "concurrent", False)
        if timer is None or conc:
            if getattr(self, "_side", None) is None:
                self._side = torch.cuda.Stream(device=self.dev)
                self._side2 = torch.cuda.Stream(device=self.dev)
                self._side3 = torch.cuda.Stream(device=self.dev)
            streams = {"main": main, "side": self._side, "side2": self._side2, "side3": self._side3}
            handles = {k: ctypes.c_void_p(v.cuda_stream) for k, v in streams.items()}
        events = {}
        for item in steps:
            if item[0] in ("sig", "wait"):
                if timer is not None and not conc:
                    continue                       # timed runs are serial on one stream
                _, who, tag = item
                st = streams[who]
                if item[0] == "sig":
                    ev = torch.cuda.Event()
                    ev.record(st)
                    events[tag] = ev
                    hook = getattr(self, "hooks", {}).get(tag)
                    if hook is not None:           # e.g. start a gradient bucket's all-reduce
                        hook(ev)
                    ext = getattr(self, "ext_events", {}).get(tag)
                    if ext is not None:            # an external event node of a captured graph (dp_graph_step)
                        ext.record(st)
                else:
                    st.wait_event(events[tag])
                continue
            name, kind, fn, where = item
            if conc:
                timer.start(name, kind, streams[where])
                fn(handles[where])
                timer.stop(name, kind, streams[where])
            elif timer is not None:
                timer.start(name, kind)
                fn(s_main)
                timer.stop(name, kind)
            else:
                fn(handles[where])

    def forward_backward(self, stream=None, timer=None, zero_grad=True):
        """Enqueue -SELBO (self.out[0]) and all gradients (into the bound grad vector)."""
        key = ("fb", self._theta.data_ptr(), self._grad.data_ptr(), self.frozen_mask, self.N)
        if getattr(self, "_sched_key", None) != key:
            self._sched = self._schedule(0)
            self._sched_key = key
        if zero_grad:
            self._grad.zero_()
        self._run(self._sched, stream, timer)
        return self.out

    def elbo_sample(self, stream=None, with_kl=False, cached=False, kl_part=None):
        """Enqueue one Monte-Carlo sample of compute_ELBO's reconstruction term (self.out[1]);
        with_kl also evaluates the KL terms from THIS sample's K_G22 (out[2..4]).  cached: reuse the
        sample-independent factors of the previous (uncached) sample of the same call -- parameters,
        data and the factor workspace must be unchanged since then.  kl_part=(f0, f1, with_v): only
        the KL terms of the variational factors f0 .. f1-1 of the W | pairs list (and of Sigma_v when
        with_v) -- a rank's share of the KL when compute_ELBO is sharded (W factors need THIS sample's
        K_G22: only the owner of the last sample may include them)."""
        self._elbo_kl = None if kl_part is None else (int(kl_part[0]), int(kl_part[1]), bool(kl_part[2]))
        key = ("elbo", with_kl, cached, self._theta.data_ptr(), self.frozen_mask, self.N, self._elbo_kl)
        cache = getattr(self, "_elbo_sched", {})
        if key not in cache:
            cache[key] = self._schedule(1, with_kl, cached)
            self._elbo_sched = cache
        self._run(cache[key], stream, None)
        return self.out

    def _kl_solve_xs(self, th, slots, offs_f):
        """W_f = C_f^-1 L_f of the variational factors f < FV from the factor C and the inverses X11, X22 of its two
        diagonal blocks (nmgp_chol_blockinv_batched_f32: C21 in X21's place, A21 scratch): W11 = X11 L11,
        W22 = X22 L22, R = L21 - C21 W11 (staged in A21), W21 = X22 R -- the forward substitution of the KL gradient's
        Sigma_f^-1 L_f (code/utils.py:339-351 and its autograd) by blocks.  The triangular blocks are stored on
        their lower tiles only (OUT_LOWER: the elements above a diagonal are never read -- B_LOWER masks them)."""
        M = self.M
        n1 = int(L.lib().nmgp_chol_split_point(M))
        n2 = M - n1
        r1 = n1 * M
        Ci, Xs, Af = self.Cinv, self.Xs, self.Afac
        sh = lambda offs, d: [o + d for o in offs]
        fl_tri = L.A_LOWER | L.B_LOWER | L.OUT_LOWER
        if n1 == n2:
            diag = [H.BigBatch(Ci, th, Xs, slots + sh(slots, r1 + n1), list(offs_f) + sh(offs_f, r1 + n1),
                               slots + sh(slots, r1 + n1), n1, n1, n1, lda=M, ldb=M, b_kcontig=False, sC=(M, 1),
                               flags=fl_tri)]
        else:
            diag = [H.BigBatch(Ci, th, Xs, sh(slots, d), sh(offs_f, d), sh(slots, d), nn, nn, nn, lda=M, ldb=M,
                               b_kcontig=False, sC=(M, 1), flags=fl_tri) for d, nn in ((0, n1), (r1 + n1, n2))]
        r = H.BigBatch(Ci, Xs, Af, sh(slots, r1), slots, sh(slots, r1), n2, n1, n1, lda=M, ldb=M, b_kcontig=False,
                       sC=(M, 1), flags=L.B_LOWER, alpha=-1.0, beta=0.0,
                       epi=(th, sh(offs_f, r1), (M, 1), self._ones, [0] * len(slots), 1.0))
        w21 = H.BigBatch(Ci, Af, Xs, sh(slots, r1 + n1), sh(slots, r1), sh(slots, r1), n2, n1, n2, lda=M, ldb=M,
                         b_kcontig=False, sC=(M, 1), flags=L.A_LOWER)
        return H.Seq(diag + [r, w21])

    def _kl_solve_lbar(self, th, gr, fb, fac_off, prior_of, NFK):
        """KL L-bar -Sigma_f^-1 L_f + diag(1/C2_ii^2) L_f (lower part) of the variational factors f < FV from W_f
        (_kl_solve_xs): G21 = X22^T W21 (its raw value also kept in A21), G22 = X22^T W22, Y = W11 - C21^T G21 (in
        W11's place, lower part), G11 = X11^T Y -- the backward substitution by blocks; Sigma_v (f = FV, factored
        with its full inverse in the prior launch) keeps the explicit-inverse product.  The triangular blocks' upper
        parts are not stored (OUT_LOWER): those gradient elements stay as zeroed at the step's start (and bwd_lbar's
        OUT_TRIL products store zeros there)."""
        M, NF, FV = self.M, self.NF, self.NF - 1
        n1 = int(L.lib().nmgp_chol_split_point(M))
        n2 = M - n1
        r1 = n1 * M
        Ci, Xs, Af = self.Cinv, self.Xs, self.Afac
        MM = M * M
        slots = [f * MM for f in range(FV)]
        fo = list(fac_off[:FV])
        sh = lambda offs, d: [o + d for o in offs]
        rs = [NF + 4 * M + prior_of[f] * M for f in range(FV)]
        g21 = H.BigBatch(Ci, Xs, gr, sh(slots, r1 + n1), sh(slots, r1), sh(fo, r1), n2, n1, n2, lda=M, ldb=M,
                         a_kcontig=False, b_kcontig=False, sC=(M, 1), flags=L.A_UPPER, alpha=-1.0, beta=1.0,
                         epi=(th, sh(fo, r1), (M, 1), fb, sh(rs, n1), 1.0), dstore=(Af, sh(slots, r1), M))
        g22 = H.BigBatch(Ci, Xs, gr, sh(slots, r1 + n1), sh(slots, r1 + n1), sh(fo, r1 + n1), n2, n2, n2, lda=M,
                         ldb=M, a_kcontig=False, b_kcontig=False, sC=(M, 1),
                         flags=L.A_UPPER | L.B_LOWER | L.OUT_LOWER | L.EPI_E_LOWER, alpha=-1.0, beta=1.0,
                         epi=(th, sh(fo, r1 + n1), (M, 1), fb, sh(rs, n1), 1.0))
        y = H.BigBatch(Ci, Af, Xs, sh(slots, r1), sh(slots, r1), slots, n1, n1, n2, lda=M, ldb=M, a_kcontig=False,
                       b_kcontig=False, sC=(M, 1), flags=L.OUT_LOWER, alpha=-1.0, beta=1.0)
        g11 = H.BigBatch(Ci, Xs, gr, slots, slots, fo, n1, n1, n1, lda=M, ldb=M, a_kcontig=False, b_kcontig=False,
                         sC=(M, 1), flags=L.A_UPPER | L.B_LOWER | L.OUT_LOWER | L.EPI_E_LOWER, alpha=-1.0, beta=1.0,
                         epi=(th, fo, (M, 1), fb, rs, 1.0))
        parts = [g21, g22, y, g11]
        if NFK > FV:
            parts.append(H.BigBatch(Ci, Xs, gr, [FV * MM], [FV * MM], [fac_off[FV]], M, M, M, lda=M, ldb=M,
                                    a_kcontig=False, b_kcontig=False,
                                    flags=L.A_UPPER | L.B_LOWER | L.OUT_TRIL | L.EPI_E_LOWER, alpha=-1.0, beta=1.0,
                                    epi=(th, [fac_off[FV]], (M, 1), fb, [NF + 4 * M + prior_of[FV] * M], 1.0)))
        return H.Seq(parts)

    def _big_rows(self, A, C, offA, offB, offC, rows, flags, b_kcontig):
        """B x M x M products op(A) L on the 128x128 f32 kernel (BigBatch), L = theta at offB, problem b on the rows
        [seg[r], seg[r + span]) of A and C, rows[b] = (r, span)."""
        M = self.M
        return H.BigBatch(A, self._theta, C, offA, offB, offC, self.B, M, M, lda=M, ldb=M, b_kcontig=b_kcontig,
                          flags=flags, rseg=(self.seg, [r for r, _ in rows], [s_ for _, s_ in rows]))

    def gemm_groups(self):
        """(name, GemmGroup) of the training step, for FLOP accounting."""
        p = self._plan(0)
        return [(it[0], p[it[0]]) for it in self._schedule(0) if len(it) > 1 and it[1] == "gemm"]

    def check_info(self):
        info = self.info.cpu()
        if int(info.abs().sum()) != 0:
            bad = int(torch.nonzero(info)[0])
            raise torch.linalg.LinAlgError(f"cholesky: matrix {bad} is not positive-definite "
                                           f"(leading minor of order {int(info[bad])})")
