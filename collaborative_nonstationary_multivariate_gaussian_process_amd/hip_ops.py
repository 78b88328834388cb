"""Thin Python wrappers over the libnmgp_hip.so C ABI (device tensors in, device tensors out).

Everything here enqueues HIP kernels on torch's current stream; nothing falls back to CPU math.
"""
import ctypes
import os
import math

import torch

from . import _lib as L

_F64 = torch.float64
_F32 = torch.float32


def _sfx(dtype):
    if dtype == _F64:
        return "f64"
    if dtype == _F32:
        return "f32"
    raise TypeError(f"unsupported dtype {dtype}")


def _addr(t, off=0):
    return 0 if t is None else t.data_ptr() + off * t.element_size()


# ------------------------------------------------------------------------------------ GEMM
def gemm_desc(C, A, B, m, n, k, sA, sB, sC, *, flags=0, alpha=1.0, beta=0.0, kb=(0, 0), kscale=None,
              epi=None, diag_add=0.0, row_seg=-1, k_seg=-1, seg_span=1, offs=(0, 0, 0)):
    """Describe C(i,j) = alpha sum_k op(A)(i,k) s(k) op(B)(k,j) + beta C + gamma rs(i) E(i,j).

    sA = (sA_i, sA_k, sA_kb), sB = (sB_k, sB_j, sB_kb), sC = (sC_i, sC_j) element strides;
    offs = element offsets into A, B, C; epi = (E, E_off, (sE_i, sE_j), rs or None, gamma).
    """
    d = L.GemmDesc()
    d.A, d.B, d.C = _addr(A, offs[0]), _addr(B, offs[1]), _addr(C, offs[2])
    d.kscale = _addr(kscale[0], kscale[1]) if kscale is not None else 0
    d.sA_i, d.sA_k, d.sA_kb = sA
    d.sB_k, d.sB_j, d.sB_kb = sB
    d.sC_i, d.sC_j = sC
    d.m, d.n, d.k = int(m), int(n), int(k)
    d.kbA, d.kbB = kb
    d.flags = flags | (L.KSCALE if kscale is not None else 0)
    d.row_seg, d.k_seg, d.seg_span = row_seg, k_seg, seg_span
    d.alpha, d.beta, d.diag_add = alpha, beta, diag_add
    if epi is not None:
        E, eoff, (se_i, se_j), rs, gamma = epi
        d.epi_E = _addr(E, eoff)
        d.sE_i, d.sE_j = se_i, se_j
        d.epi_rs = _addr(rs[0], rs[1]) if rs is not None else 0
        d.gamma = gamma
        d.flags |= L.EPI
    if diag_add:
        d.flags |= L.DIAG_ADD
    d.tiles_m = (d.m + 63) // 64
    d.tiles_n = (d.n + 63) // 64
    return d




GEMM_BK = 32   # k-tile of gemm_kernel (csrc/gemm.hip GBK)
# split a problem's k loop beyond this many times the balanced per-workgroup share (tools/gemm_probe.py; PM2.5
# bench A/B in round 2: 2.0 -> 1283-1291 it/s, 4.0 -> 1300-1302, 8.0 -> 1298-1329, no large-k split 1315-1322)
_KSPLIT_FACTOR = 8.0


def _auto_ksplit(k_eff, group_tiles, work_per_wg):
    """Split-K factor of one problem.  A split costs a workspace round trip and an ordered
    reduction by the last arriver, so it is used only where it shortens the launch's critical
    path (measured with tools/gemm_probe.py): tiny groups (<= 64 tiles: latency-bound k loops, chunks
    down to 2 k-tiles), and problems whose k loop is more than twice the balanced per-workgroup
    share (chunks >= 4 k-tiles)."""
    kt = -(-max(k_eff, 1) // GEMM_BK)
    if group_tiles <= 64 and kt >= 4:
        return max(1, min(16, kt // 2, -(-256 // max(group_tiles, 1))))
    if kt > _KSPLIT_FACTOR * work_per_wg and kt >= 8:
        return max(1, min(16, kt // 4, -(-kt // work_per_wg)))
    return 1


def _cap_ksplit(ksplit, k_eff, kt_cap):
    """Split-K factor raised so that no chunk of a k range of k_eff runs more than ~kt_cap k-tiles of
    GEMM_BK (GemmGroup(kt_cap=)); at most 16 chunks, never lowered."""
    if kt_cap <= 0:
        return ksplit
    kt = -(-max(k_eff, 1) // GEMM_BK)
    return max(ksplit, min(16, -(-kt // kt_cap)))


# row-segmented groups get the device tile plan only from this many static tiles on (round 2 A/B: 128 / 256 /
# 512 / 1024 within noise on the PM2.5 bench)
_DYN_MIN_TILES = 1024

LAT_TILE = 32       # output tile of the latency kernel (csrc/gemm_lat.hip LTM / LTN)
LAT_PANEL = 64      # panel alignment the latency kernel needs of k-blocked operands
LAT_WAVES, LAT_KP = 8, 32   # waves per workgroup and k-panel width (gemm_lat.hip launch config 1)
_LAT_MODE = "auto"        # "0": never (the tests compare the two kernels), "force": wherever eligible
# a workgroup of the latency kernel loads each round of panels (LAT_WAVES x LAT_KP of k) in one go and
# waits for it; groups that leave more rounds than this per workgroup after split-K (many output tiles
# AND long k: the P-bar / L-bar products over several latent blocks or the minibatch) stay on the
# LDS-pipelined tile kernel (per-group A/B on the box: tools/gemm_group_probe.py)
_LAT_MAX_ROUNDS = 2
# persistent two-tiles-in-flight launches (gemm_lat_pipe_kernel) for latency-kernel groups with more tiles than one
# round of workgroups (two 8-wave workgroups per CU): "auto", "0" (never), "force" (every latency-kernel group).
# Off by default: measured on the PM2.5 step (round 6, gpurun_out r06l) it LOST -- one workgroup per CU (the second
# operand buffer needs ~210 VGPRs) leaves 8 waves per CU where the one-tile kernel keeps 16, and the reduction /
# epilogue phases then idle the matrix cores: bwd_wG 72 -> 135 us, bwd_lbar 100 -> 174 us, step 0.68 -> 0.83 ms
_LAT_PIPE = os.environ.get("NMGP_LAT_PIPE", "0")
LAT_ROUND_WGS = 512


def _lat_split(descs, seg, target_wgs):
    """Split-K factor per descriptor for the latency kernel and the rounds of k panels a workgroup
    then still runs: ([ksplit], max rounds)."""
    nseg = (seg.numel() - 1) if seg is not None else 1
    frac = lambda d, s_: (max(d.seg_span, 1) / nseg) if s_ >= 0 else 1.0
    tiles = [-(-max(d.m, 0) // LAT_TILE) * -(-max(d.n, 0) // LAT_TILE) for d in descs]
    group_tiles = max(1, sum(tiles))
    ks, worst = [], 0
    for d in descs:
        k_eff = max(1, round(max(d.k, 1) * frac(d, d.k_seg)))
        rounds = -(-(-(-k_eff // LAT_KP)) // LAT_WAVES)
        k = int(max(1, min(16, rounds, round(target_wgs / group_tiles))))
        ks.append(k)
        worst = max(worst, -(-rounds // k))
    return ks, worst


def _lat_colpack_groups(d):
    """Column-tile groups of a B-triangular latency-kernel problem (csrc/gemm_lat.hip, NMGP_LAT_COLPACK flag): with
    B_LOWER the column tile j of an n == k == 32 T problem has T - j k panels (B_UPPER: j + 1), so {0}, {g, T - g}
    and, for even T, {T / 2} each fill at most the 8 waves of a workgroup.  0 when the problem does not qualify."""
    f = d.flags
    bmask = f & (L.B_LOWER | L.B_UPPER)
    if bmask not in (L.B_LOWER, L.B_UPPER):
        return 0
    if f & (L.A_LOWER | L.A_UPPER | L.OUT_LOWER | L.OUT_TRIL) or d.k_seg >= 0 or d.ksplit > 1:
        return 0
    K = d.k
    if K <= 0 or K % LAT_TILE or d.n != K or (0 < d.kbB < K) or (0 < d.kbA < K):
        return 0
    T = K // LAT_TILE
    if T < 3 or T > LAT_WAVES:
        return 0
    return 1 + (T - 1) // 2 + (1 if T % 2 == 0 else 0)


def _lat_eligible(d, esz):
    """Can gemm_lat.hip run this descriptor?  Non-negative strides, k-blocks that panels never
    straddle, and operand extents (incl. the rows / k a tile may touch past the problem) addressable
    by a 32-bit buffer offset."""
    if d.batch > 1:
        return False
    st = (d.sA_i, d.sA_k, d.sA_kb, d.sB_k, d.sB_j, d.sB_kb)
    if min(st) < 0:
        return False
    K = max(d.k, 1)
    for kb in (d.kbA, d.kbB):
        if 0 < kb < K and kb % LAT_PANEL:
            return False
    kinA = d.kbA if 0 < d.kbA < K else K
    kinB = d.kbB if 0 < d.kbB < K else K
    nkbA = -(-K // kinA)
    nkbB = -(-K // kinB)
    extA = ((d.m + LAT_TILE) * d.sA_i + (kinA + LAT_PANEL) * d.sA_k + nkbA * d.sA_kb) * esz
    extB = ((kinB + LAT_PANEL) * d.sB_k + (d.n + LAT_TILE) * d.sB_j + nkbB * d.sB_kb) * esz
    return max(extA, extB) < 0x7fff0000


class GemmGroup:
    """A fixed list of GEMM problems launched as ONE grouped kernel (descriptors uploaded once).

    Two kernels share the descriptor format: the LDS-staged 64x64 kernel (gemm.hip: long k loops,
    split-K) and the latency kernel (gemm_lat.hip: 32x32 tiles, the k range split over the waves of
    a workgroup, operands loaded straight into registers) for groups whose k loops are short -- the
    B x M x M and M x M x M products of the DSVI step.  `kernel`: "auto" (latency kernel when every
    problem is eligible and k <= NMGP_GEMM_LAT_KMAX), "tile", "lat"."""

    def __init__(self, descs, device, dtype, seg=None, target_wgs=512, dyn_plan=True, kernel="auto", kt_cap=0,
                 max_grid=0):
        """Split-K is chosen per problem so that the launch has ~target_wgs workgroups when the
        outputs alone are too few tiles (the M x B x M products P^T R with K = B).  kt_cap > 0 (tile
        kernel only; forces it): split every problem so that no workgroup runs more than ~kt_cap k-tiles -- for groups
        on the step's critical path, where the longest tile's k loop, not the chip's fill, sets the
        launch time.  max_grid > 0 (tile kernel): at most that many workgroups, striding over the tiles
        (longest k loops first) -- for off-critical-path groups whose long-lived workgroups would otherwise
        hold every CU slot while the critical chain's launches wait for them."""
        self.dtype = dtype
        self.seg = seg
        self.lat = self.pipe = False
        self._static_plan = False
        # the group owns copies: split-K, tile counts, workspaces and flags are set per group, so a descriptor
        # list shared by two groups (or reused by the caller) never carries one group's choices into another
        descs = [L.GemmDesc.from_buffer_copy(d) for d in descs]
        if kt_cap or max_grid:
            # split caps and grid caps are tile-kernel features: never let "auto" drop them silently
            if kernel == "lat":
                raise ValueError("GemmGroup: kt_cap / max_grid apply to the tile kernel only")
            kernel = "tile"
        esz = 8 if dtype == _F64 else 4
        if kernel != "tile" and _LAT_MODE != "0" and descs:
            ok = all(_lat_eligible(d, esz) for d in descs)
            if kernel == "lat" and not ok:
                raise ValueError("GemmGroup(kernel='lat'): a descriptor is not addressable by the latency kernel")
            short = ok and _lat_split(descs, seg, target_wgs)[1] <= _LAT_MAX_ROUNDS
            # f32 too (round 2) where k <= 256: PM2.5-shaped fp32 step 1150 -> 1285 it/s A/B on the box.  At
            # M = 512 (HCP) it was no faster and its different summation order moved the HCP-like fp32 loss
            # from 6.1e-4 to 2.7e-3 of the fp64 reference (gate 1e-3): those groups stay on the tile kernel
            f32_ok = dtype == _F64 or all(d.k <= 256 for d in descs)
            self.lat = ok and (kernel == "lat" or _LAT_MODE == "force" or (short and f32_ok))
        if self.lat:
            self._init_lat(descs, device, dyn_plan, target_wgs)
            return
        arr = (L.GemmDesc * len(descs))()
        group_tiles = sum(d.tiles_m * d.tiles_n for d in descs)
        nseg = (seg.numel() - 1) if seg is not None else 1
        # expected k / rows of segment-addressed problems: their share of the (balanced) segments
        frac = lambda d, s_: (max(d.seg_span, 1) / nseg) if s_ >= 0 else 1.0
        eff = [(max(1, round(d.tiles_m * frac(d, d.row_seg))) * d.tiles_n,
                max(1, round(max(d.k, 1) * frac(d, d.k_seg)))) for d in descs]
        total_ktiles = sum(t_ * -(-k_ // GEMM_BK) for t_, k_ in eff)
        work_per_wg = max(2, total_ktiles // target_wgs)   # k-tiles per workgroup if the launch were balanced
        esz = 8 if dtype == _F64 else 4
        self._ws = []
        for i, d in enumerate(descs):
            if d.ksplit <= 1:
                d.ksplit = _auto_ksplit(eff[i][1], group_tiles, work_per_wg)
            d.ksplit = _cap_ksplit(d.ksplit, eff[i][1], kt_cap)
        # longest k-loop per workgroup first: those workgroups are dispatched first instead of
        # forming the launch's tail (problems of one group write disjoint outputs, so their order in
        # the launch is free)
        order = sorted(range(len(descs)), key=lambda i: -(-(-eff[i][1] // GEMM_BK) // max(descs[i].ksplit, 1)))
        descs = [descs[i] for i in order]
        t = 0
        for i, d in enumerate(descs):
            if d.ksplit <= 1:
                d.ksplit = 1
            if d.ksplit > 1:
                ntile = d.tiles_m * d.tiles_n
                ws = torch.empty(ntile * d.ksplit * 4096, dtype=dtype, device=device)
                ctr = torch.zeros(ntile, dtype=torch.int32, device=device)
                self._ws += [ws, ctr]
                d.ws, d.counters = ws.data_ptr(), ctr.data_ptr()
            else:
                d.ksplit = 1
            d.tile_start = t
            t += d.tiles_m * d.tiles_n * d.ksplit
            arr[i] = d
        self.total = t
        self.n = len(descs)
        self.descs = list(descs)
        raw = bytes(memoryview(arr).cast("B"))
        self.dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)
        # row-segmented problems (rows of one output) are sized on device per minibatch: a plan
        # kernel + a grid of about the expected tile count striding over the tiles that exist
        # (only where the static grid is mostly idle workgroups: the plan launch costs more than it
        # saves on small grids; PM2.5 quad / bwd_w: +2-3% it/s; HCP, D=50: ~95% of the quad-form workgroups removed)
        self.plan, self.grid = None, 0
        if max_grid > 0 and t > max_grid:
            if any(d.row_seg >= 0 for d in descs):
                self.plan = torch.zeros(len(descs) + 1, dtype=torch.int32, device=device)
            else:                                  # the plan is the static tile layout: uploaded once
                self.plan = torch.tensor([d.tile_start for d in descs] + [t], dtype=torch.int32, device=device)
                self._static_plan = True
            self.grid = int(max_grid)
        elif seg is not None and dyn_plan and any(d.row_seg >= 0 for d in descs):
            ksp = {id(d): max(d.ksplit, 1) for d in descs}
            expect = sum(eff[order[i]][0] * ksp[id(d)] for i, d in enumerate(descs))
            if dyn_plan == "force" or (t >= _DYN_MIN_TILES and expect < 0.5 * t):
                self.plan = torch.zeros(len(descs) + 1, dtype=torch.int32, device=device)
                self.grid = int(min(t, max(256, min(4096, round(1.15 * expect)))))

    def _init_lat(self, descs, device, dyn_plan, target_wgs):
        """Latency-kernel layout: 32x32 tiles; a problem whose k range needs more than one round of
        panels over the workgroup's waves is split over up to that many workgroups when the group's
        tiles alone leave the chip idle (workspace + counters as the tile kernel's split-K).
        Row-segmented groups whose static grid is mostly idle get the device tile plan (the grid stays
        a multiple of 8 for the XCD mapping)."""
        nseg = (self.seg.numel() - 1) if self.seg is not None else 1
        frac = lambda d, s_: (max(d.seg_span, 1) / nseg) if s_ >= 0 else 1.0
        arr = (L.GemmDesc * len(descs))()
        ksplits, _ = _lat_split(descs, self.seg, target_wgs)
        t, expect = 0, 0.0
        self._ws = []
        for i, d in enumerate(descs):
            d.tiles_m = -(-d.m // LAT_TILE) if d.m > 0 else 0
            d.tiles_n = -(-d.n // LAT_TILE) if d.n > 0 else 0
            d.ksplit = ksplits[i]
            d.flags &= ~L.LAT_COLPACK                # (set below only when this group packs the problem)
            groups = _lat_colpack_groups(d)
            if groups:
                d.flags |= L.LAT_COLPACK          # tiles_n = column-tile groups (5 instead of 8 at M = 256)
                d.tiles_n = groups
            nt = d.tiles_m * d.tiles_n
            if d.ksplit > 1:
                ws = torch.empty(nt * d.ksplit * LAT_TILE * LAT_TILE, dtype=self.dtype, device=device)
                ctr = torch.zeros(max(nt, 1), dtype=torch.int32, device=device)
                self._ws += [ws, ctr]
                d.ws, d.counters = ws.data_ptr(), ctr.data_ptr()
            d.tile_start = t
            t += nt * d.ksplit
            expect += nt * d.ksplit * frac(d, d.row_seg)
            arr[i] = d
        self.total = t
        self.n = len(descs)
        self.descs = list(descs)
        raw = bytes(memoryview(arr).cast("B"))
        self.dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)
        # more (expected) tiles than one round of workgroups: the persistent launch (bit-identical results)
        self.pipe = _LAT_PIPE == "force" or (_LAT_PIPE == "auto" and expect > LAT_ROUND_WGS)
        self.plan, self.grid = None, 0
        if self.seg is not None and dyn_plan and any(d.row_seg >= 0 for d in descs):
            if dyn_plan == "force" or (t >= _DYN_MIN_TILES and expect < 0.5 * t):
                self.plan = torch.zeros(len(descs) + 1, dtype=torch.int32, device=device)
                self.grid = int(min(-(-t // 8) * 8, max(256, min(8192, 8 * round(1.15 * expect / 8)))))

    def macs(self, seg=None):
        return sum(desc_macs(d, seg) for d in self.descs)

    def algo_bytes(self, seg=None):
        esz = 8 if self.dtype == _F64 else 4
        return sum(desc_bytes(d, seg, esz, beta=d.beta, epi=bool(d.flags & L.EPI)) for d in self.descs)

    def plan_now(self, stream=None):
        """Enqueue only the device tile plan of a segment-sized group (e.g. right after the minibatch
        gather, on another stream); later calls with planned=True reuse it.  No-op for static groups."""
        if self.plan is None or self.n == 0 or self.total == 0 or self._static_plan:
            return False
        s = stream if stream is not None else L.stream_handle()
        fn = L.lib().nmgp_gemm_plan_lat if self.lat else L.lib().nmgp_gemm_plan
        L.check(fn(ctypes.c_void_p(self.dev.data_ptr()), self.n, ctypes.c_void_p(self.seg.data_ptr()),
                   ctypes.c_void_p(self.plan.data_ptr()), s), "gemm_plan")
        return True

    def __call__(self, stream=None, planned=False):
        if self.n == 0 or self.total == 0:
            return
        s = stream if stream is not None else L.stream_handle()
        segp = ctypes.c_void_p(self.seg.data_ptr()) if self.seg is not None else None
        pre = "_planned_" if ((planned or self._static_plan) and self.plan is not None) else "_"
        if self.lat:
            plan = ctypes.c_void_p(self.plan.data_ptr()) if self.plan is not None else None
            if self.pipe:
                fn = getattr(L.lib(), "nmgp_gemm_grouped_lat_pipe_" + _sfx(self.dtype))
                L.check(fn(ctypes.c_void_p(self.dev.data_ptr()), self.n, self.total, segp, plan,
                           1 if pre == "_planned_" else 0, s), "gemm_grouped_lat_pipe")
                return
            fn = getattr(L.lib(), "nmgp_gemm_grouped_lat" + pre + _sfx(self.dtype))
            L.check(fn(ctypes.c_void_p(self.dev.data_ptr()), self.n, self.total, segp, plan, self.grid, s),
                    "gemm_grouped_lat")
            return
        if self.plan is not None:
            fn = getattr(L.lib(), "nmgp_gemm_grouped_dyn" + pre + _sfx(self.dtype))
            L.check(fn(ctypes.c_void_p(self.dev.data_ptr()), self.n, self.total, segp,
                       ctypes.c_void_p(self.plan.data_ptr()), self.grid, s), "gemm_grouped_dyn")
            return
        fn = getattr(L.lib(), "nmgp_gemm_grouped_" + _sfx(self.dtype))
        L.check(fn(ctypes.c_void_p(self.dev.data_ptr()), self.n, self.total, segp, s), "gemm_grouped")


def desc_macs(d, seg=None):
    """Algorithmic multiply-adds of one problem: structural zeros of triangular operands and the
    skipped upper half of OUT_LOWER / OUT_TRIL outputs are not counted; row / k ranges resolved
    from the host copy of the segment table."""
    import numpy as np
    span = d.seg_span if d.seg_span > 0 else 1
    m = d.m if d.row_seg < 0 else int(seg[d.row_seg + span] - seg[d.row_seg])
    K = d.k if d.k_seg < 0 else int(seg[d.k_seg + span] - seg[d.k_seg])
    n = d.n
    if m <= 0 or n <= 0 or K <= 0:
        return 0
    kb = d.kbA if 0 < d.kbA < K else K
    nblk = K // kb
    f = d.flags
    i = np.arange(m)[:, None]
    j = np.arange(n)[None, :]
    lo = np.zeros((m, n), np.int64)
    hi = np.full((m, n), kb - 1, np.int64)
    if f & L.A_UPPER:
        lo = np.maximum(lo, i)
    if f & L.B_LOWER:
        lo = np.maximum(lo, j)
    if f & L.A_LOWER:
        hi = np.minimum(hi, i)
    if f & L.B_UPPER:
        hi = np.minimum(hi, j)
    cnt = np.clip(hi - lo + 1, 0, None)
    if f & (L.OUT_LOWER | L.OUT_TRIL):
        cnt = np.where(j <= i, cnt, 0)
    return int(cnt.sum()) * nblk


def desc_bytes(d, seg=None, esz=4, beta=0.0, epi=False):
    """Algorithmic HBM bytes of one problem: its operands read once (structurally zero triangles of triangular
    operands not counted), C written once (the skipped upper half of OUT_LOWER / OUT_TRIL outputs not counted) and
    read as well when beta != 0, the epilogue operand E read once; row / k ranges from the host segment table."""
    span = d.seg_span if d.seg_span > 0 else 1
    m = d.m if d.row_seg < 0 else int(seg[d.row_seg + span] - seg[d.row_seg])
    K = d.k if d.k_seg < 0 else int(seg[d.k_seg + span] - seg[d.k_seg])
    n = d.n
    if m <= 0 or n <= 0:
        return 0
    f = d.flags
    tri = lambda r, c: r * c - (min(r, c) * (min(r, c) - 1)) // 2 if r == c else r * c
    a = tri(m, K) if f & (L.A_LOWER | L.A_UPPER) else m * K
    b = tri(K, n) if f & (L.B_LOWER | L.B_UPPER) else K * n
    c = (m * (m + 1)) // 2 if (f & (L.OUT_LOWER | L.OUT_TRIL)) and m == n else m * n
    e = ((m * (m + 1)) // 2 if f & L.EPI_E_LOWER else m * n) if epi else 0
    ab = (a + b) if K > 0 else 0
    return esz * (ab + c * (2 if beta != 0.0 else 1) + e)


def chol_inv_rec_bytes(n, esz=4):
    """Algorithmic HBM bytes of one factor + inverse of an n x n SPD matrix: its lower triangle read once, L and
    L^-1 (lower triangles) written once."""
    return esz * 3 * (n * (n + 1)) // 2


def chol_inv_rec_macs(n):
    """Multiply-adds of the GEMMs one recursive factor + inverse of an n x n matrix issues (csrc/chol.hip
    chol_inv_rec_big / chol_inv_rec: split at n1 = the multiple of 128 nearest above n/2; L21 = A21 X11^T,
    A22 -= L21 L21^T (lower), T = L21 X11, X21 = -X22 T; leaves n <= 128 run in the fused kernel, not counted)."""
    import types
    if n <= 128:
        return 0
    n1 = ((n // 2 + 127) // 128) * 128
    if n1 >= n:
        n1 = n - 128
    n2 = n - n1
    d = lambda m_, n_, k_, f: desc_macs(types.SimpleNamespace(m=m_, n=n_, k=k_, flags=f, row_seg=-1, k_seg=-1,
                                                              seg_span=0, kbA=0))
    return (chol_inv_rec_macs(n1) + chol_inv_rec_macs(n2) + d(n2, n1, n1, L.B_UPPER) + d(n2, n2, n1, L.OUT_LOWER)
            + d(n2, n1, n1, L.B_LOWER) + d(n2, n1, n2, L.A_LOWER))


def gemm_single(desc, dtype, seg=None):
    fn = getattr(L.lib(), "nmgp_gemm_" + _sfx(dtype))
    L.check(fn(ctypes.byref(desc), ctypes.c_void_p(seg.data_ptr()) if seg is not None else None,
               L.stream_handle()), "gemm")


def matmul(A, B, transA=False, transB=False, maskA=0, maskB=0, out=None, alpha=1.0):
    """C = alpha op(A) op(B) for 2-D device tensors (op = transpose when requested)."""
    L.require_device(A, "A")
    A = A.contiguous()
    B = B.contiguous()
    m, k = (A.shape[1], A.shape[0]) if transA else A.shape
    k2, n = (B.shape[1], B.shape[0]) if transB else B.shape
    assert k == k2, (A.shape, B.shape)
    if out is None:
        out = torch.empty(m, n, dtype=A.dtype, device=A.device)
    sA = (1, A.shape[1], 0) if transA else (A.shape[1], 1, 0)
    sB = (1, B.shape[1], 0) if transB else (B.shape[1], 1, 0)
    d = gemm_desc(out, A, B, m, n, k, sA, sB, (n, 1), flags=maskA | maskB, alpha=alpha)
    gemm_single(d, A.dtype)
    return out


def bmm(A, B, transA=False, transB=False, maskA=0, maskB=0, out=None, alpha=1.0):
    """Batched C[b] = alpha op(A[b]) op(B[b]) in ONE launch (grid.y = batch).  A or B may be 2-D and is
    then shared by every batch entry (batch stride 0)."""
    L.require_device(A, "A")
    A = A.contiguous()
    B = B.contiguous()
    nb = A.shape[0] if A.dim() == 3 else B.shape[0]
    a2, b2 = A.shape[-2:], B.shape[-2:]
    m, k = (a2[1], a2[0]) if transA else a2
    k2, n = (b2[1], b2[0]) if transB else b2
    assert k == k2 and (A.dim() == 2 or A.shape[0] == nb) and (B.dim() == 2 or B.shape[0] == nb), (A.shape, B.shape)
    if out is None:
        out = torch.empty(nb, m, n, dtype=A.dtype, device=A.device)
    sA = (1, a2[1], 0) if transA else (a2[1], 1, 0)
    sB = (1, b2[1], 0) if transB else (b2[1], 1, 0)
    d = gemm_desc(out, A, B, m, n, k, sA, sB, (n, 1), flags=maskA | maskB, alpha=alpha)
    d.batch = int(nb)
    d.sA_b = a2[0] * a2[1] if A.dim() == 3 else 0
    d.sB_b = b2[0] * b2[1] if B.dim() == 3 else 0
    d.sC_b = m * n
    gemm_single(d, A.dtype)
    return out


# ------------------------------------------------------------------------------------ Cholesky
def potrf_(A, info=None):
    """In-place lower Cholesky of a (batch, n, n) or (n, n) contiguous device tensor."""
    L.require_device(A, "A")
    assert A.is_contiguous()
    n = A.shape[-1]
    batch = A.numel() // (n * n) if n else 0
    if info is None:
        info = torch.zeros(max(batch, 1), dtype=torch.int32, device=A.device)
    fn = getattr(L.lib(), "nmgp_potrf_batched_" + _sfx(A.dtype))
    L.check(fn(ctypes.c_void_p(A.data_ptr()), n, n, n * n, batch, ctypes.c_void_p(info.data_ptr()),
               L.stream_handle()), "potrf")
    return info


def trtri(Lm, out=None):
    L.require_device(Lm, "L")
    Lm = Lm.contiguous()
    n = Lm.shape[-1]
    batch = Lm.numel() // (n * n) if n else 0
    if out is None:
        out = torch.empty_like(Lm)
    fn = getattr(L.lib(), "nmgp_trtri_batched_" + _sfx(Lm.dtype))
    L.check(fn(ctypes.c_void_p(Lm.data_ptr()), n, n, n * n, ctypes.c_void_p(out.data_ptr()), n, n * n, batch,
               L.stream_handle()), "trtri")
    return out


_WS = {}


def big_workspace(device, nbytes, tag="gemm"):
    """Zero-filled device workspace of the split-K GEMM paths, one per (device, layout tag), grown on
    demand (the kernels leave its counters zero again, so it is reused by every call in stream
    order).  Layouts differ per tag (the blocked potrf puts its own counters elsewhere), so callers
    with different layouts never share one."""
    key = (torch.device(device).index or 0, tag)
    ws = _WS.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.zeros(int(nbytes), dtype=torch.uint8, device=device)
        _WS[key] = ws
    return ws


def chol_inv_(A, out=None, info=None, ws=None):
    """Fused in-place lower Cholesky of A (batch, n, n) and X = L^{-1}; returns (X, info).
    f32 with n > 256 runs the recursive path with split-K workspace (`ws`, or a cached one)."""
    L.require_device(A, "A")
    assert A.is_contiguous()
    n = A.shape[-1]
    batch = A.numel() // (n * n) if n else 0
    if out is None:
        out = torch.empty_like(A)
    if info is None:
        info = torch.zeros(max(batch, 1), dtype=torch.int32, device=A.device)
    lib = L.lib()
    if A.dtype == torch.float32:
        need = lib.nmgp_chol_inv_workspace_size_f32(n, batch)
        if need > 0:
            if ws is None:
                ws = big_workspace(A.device, need)
            L.check(lib.nmgp_chol_inv_batched_ws_f32(ctypes.c_void_p(A.data_ptr()), n, n, n * n,
                                                     ctypes.c_void_p(out.data_ptr()), n, n * n, batch,
                                                     ctypes.c_void_p(info.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                                     ws.numel(), L.stream_handle()), "chol_inv")
            return out, info
    fn = getattr(lib, "nmgp_chol_inv_batched_" + _sfx(A.dtype))
    L.check(fn(ctypes.c_void_p(A.data_ptr()), n, n, n * n, ctypes.c_void_p(out.data_ptr()), n, n * n, batch,
               ctypes.c_void_p(info.data_ptr()), L.stream_handle()), "chol_inv")
    return out, info


def _ptr(t):
    """Device address of a tensor (its data_ptr), an int address, or 0 for None."""
    if t is None:
        return 0
    return int(t) if isinstance(t, int) else t.data_ptr()


class CholTp:
    """The fused GP-prior launch (nmgp_chol_tp_f64, fp64, 128 <= n <= 256): `batch` n x n slots of A (K22 + jitter I,
    stride n*n from A's first element) factored in place with X <- L^-1 and info as chol_inv_, where mats[b]["rows"]
    != 0 also forms the minibatch products in the same launch (1: RBF K12 rows from x with hyp = (log s2, log ls) at
    mats[b]["hyp"]; 2: the t-row sample -- ell_X, var_t from trow = dict(Pt, Tt, v, zt, hyp_t, ellX, var_t) -- then
    Gibbs K12 rows with ellZ): K12, T = K12 L^-T and P = T L^-1 written to the (B, n) tensors mats[b]["K12" / "T" /
    "P"].  The argument struct is built once; a call is one launch (graph-capturable)."""

    def __init__(self, A, X, info, n, mats, *, jitter=0.0, Z=None, ellZ=None, x=None, B=0, trow=None, vg=None):
        """vg = dict(muv, z, v, ellZ, K22, wgs): mats[0] is Sigma_v, and `wgs` extra workgroups form v = muv + L_v z,
        ellZ = exp(v) and the Gibbs prior's K22 + jitter I (n x n, lower 16 x 16 tiles) once L_v is factored."""
        for t_, nm in ((A, "A"), (X, "X"), (info, "info")):
            L.require_device(t_, nm)
        assert A.dtype == torch.float64 and X.dtype == torch.float64 and 1 <= len(mats) <= 4
        a = L.CholTpArgs()
        a.A, a.n, a.lda, a.strideA = A.data_ptr(), n, n, n * n
        a.X, a.ldx, a.strideX, a.batch = X.data_ptr(), n, n * n, len(mats)
        a.info, a.jitter = info.data_ptr(), float(jitter)
        a.Z, a.ellZ, a.x, a.B = _ptr(Z), _ptr(ellZ), _ptr(x), int(B)
        tr = trow or {}
        for k in ("Pt", "Tt", "v", "zt", "hyp_t", "ellX", "var_t"):
            setattr(a, k, _ptr(tr.get(k)))
        for b, m in enumerate(mats):
            mt = a.mats[b]
            mt.reserved, mt.rows = 0, int(m.get("rows", 0))
            mt.hyp, mt.K12, mt.T, mt.P = (_ptr(m.get(k)) for k in ("hyp", "K12", "T", "P"))
        if vg is not None:
            a.vg_muv, a.vg_z, a.vg_v, a.vg_ellZ, a.vg_K22 = (_ptr(vg[k]) for k in ("muv", "z", "v", "ellZ", "K22"))
            a.vg_wgs = int(vg.get("wgs", 16))
        self.a = a
        self._keep = (A, X, info, Z, ellZ, x, tr, mats, vg)     # the struct holds raw addresses of these

    def __call__(self, stream=None):
        s = stream if stream is not None else L.stream_handle()
        L.check(L.lib().nmgp_chol_tp_f64(ctypes.byref(self.a), s), "chol_tp")


class BigBatch:
    """`batch` same-shape f32 products at per-problem element offsets on the 128x128 MFMA kernel
    (nmgp_gemm_big_offsets_epi_f32): C_b = alpha op(A_b) op(B_b) + beta C_b (+ diag_add on the diagonal)
    (+ gamma rs_b(i) E_b(i, j) with `epi`).  op(A_b)(i, k) = A_b[i*lda + k] (a_kcontig) or
    A_b[k*lda + i]; op(B_b)(k, j) = B_b[j*ldb + k] (b_kcontig) or B_b[k*ldb + j]; X_b = X + offX[b].
    epi = (E, offE, (sEi, sEj), RS, offRS, gamma).  kseg / rseg = (seg, [segment index per problem], [segment span
    per problem]): per-problem k range / row range (rows of A, C, E, RS; m bounds them) from the device segment table.
    dstore = (D, offD, sDi) (with epi, full outputs): the raw product is also stored to D + offD[b] (row stride sDi).
    Offsets are uploaded once; a call is one launch (graph-capturable)."""

    def __init__(self, A, B, C, offA, offB, offC, m, n, k, *, lda, ldb, b_kcontig, a_kcontig=True, sC=None,
                 flags=0, alpha=1.0, beta=0.0, diag_add=0.0, epi=None, kseg=None, rseg=None, dstore=None):
        for t_, nm in ((A, "A"), (B, "B"), (C, "C")):
            L.require_device(t_, nm)
            assert t_.dtype == torch.float32
        dev = A.device
        self.A, self.B, self.C = A, B, C
        i64 = lambda o: torch.tensor(list(o), dtype=torch.int64, device=dev)
        self.off = [i64(o) for o in (offA, offB, offC)]
        self.batch = len(offA)
        assert len(offB) == self.batch and len(offC) == self.batch
        self.epi = None
        if epi is not None:
            E, offE, (sEi, sEj), RS, offRS, gamma = epi
            assert E.dtype == torch.float32 and RS.dtype == torch.float32
            assert len(offE) == self.batch and len(offRS) == self.batch
            self.epi = (E, i64(offE), sEi, sEj, RS, i64(offRS), gamma)
            flags |= L.EPI
        # kseg = (seg, [segment index per problem], [segment span per problem]): per-problem k range
        self.kseg = None
        if kseg is not None:
            seg, ks, sp = kseg
            assert seg.dtype == torch.int32 and len(ks) == self.batch and len(sp) == self.batch
            i32 = lambda o: torch.tensor(list(o), dtype=torch.int32, device=dev)
            self.kseg = (seg, i32(ks), i32(sp))
        self.rseg = None
        if rseg is not None:
            assert kseg is None, "BigBatch: row and k segments together are not supported"
            assert not (flags & L.OUT_LOWER)
            seg, rs_, sp = rseg
            assert seg.dtype == torch.int32 and len(rs_) == self.batch and len(sp) == self.batch
            i32 = lambda o: torch.tensor(list(o), dtype=torch.int32, device=dev)
            self.rseg = (seg, i32(rs_), i32(sp))
            self._rseg_host = (list(rs_), list(sp))
        self.dstore = None
        if dstore is not None:
            D, offD, sDi = dstore
            assert epi is not None and kseg is None and rseg is None and diag_add == 0.0
            assert not (flags & (L.OUT_LOWER | L.OUT_TRIL)) and D.dtype == torch.float32 and len(offD) == self.batch
            L.require_device(D, "D")
            self.dstore = (D, i64(offD), int(sDi))
        self.args = (m, n, k, lda, a_kcontig, ldb, b_kcontig, sC if sC is not None else (n, 1), flags, alpha, beta,
                     diag_add)

    def macs(self, seg=None):
        """Algorithmic multiply-adds of the batch (desc_macs per problem: triangular zeros and skipped output
        halves not counted; per-problem k from the host copy `seg` of the segment table with kseg)."""
        import types
        m, n, k, _, _, _, _, _, flags, _, _, _ = self.args
        if self.rseg is not None:
            return sum(desc_macs(types.SimpleNamespace(m=m, n=n, k=k, flags=flags, row_seg=a, k_seg=-1, seg_span=b,
                                                       kbA=0), seg) for a, b in zip(*self._rseg_host))
        if self.kseg is None:
            return self.batch * desc_macs(types.SimpleNamespace(m=m, n=n, k=k, flags=flags, row_seg=-1, k_seg=-1,
                                                                seg_span=0, kbA=0))
        ks, sp = self.kseg[1].tolist(), self.kseg[2].tolist()
        return sum(desc_macs(types.SimpleNamespace(m=m, n=n, k=k, flags=flags, row_seg=-1, k_seg=a, seg_span=b,
                                                   kbA=0), seg) for a, b in zip(ks, sp))

    def algo_bytes(self, seg=None):
        """Algorithmic HBM bytes of the batch (desc_bytes per problem, row / k ranges from the host `seg`)."""
        import types
        m, n, k, _, _, _, _, _, flags, _, beta, _ = self.args
        epi = self.epi is not None
        ns = lambda **kw: types.SimpleNamespace(m=m, n=n, k=k, flags=flags, kbA=0, **kw)
        if self.rseg is not None:
            return sum(desc_bytes(ns(row_seg=a, k_seg=-1, seg_span=b), seg, 4, beta, epi)
                       for a, b in zip(*self._rseg_host))
        if self.kseg is None:
            extra = self.batch * m * n * 4 if self.dstore is not None else 0
            return self.batch * desc_bytes(ns(row_seg=-1, k_seg=-1, seg_span=0), None, 4, beta, epi) + extra
        ks, sp = self.kseg[1].tolist(), self.kseg[2].tolist()
        return sum(desc_bytes(ns(row_seg=-1, k_seg=a, seg_span=b), seg, 4, beta, epi) for a, b in zip(ks, sp))

    def __call__(self, stream=None):
        if self.batch == 0:
            return
        m, n, k, lda, ak, ldb, bk, (sCi, sCj), flags, alpha, beta, dadd = self.args
        s = stream if stream is not None else L.stream_handle()
        vp = ctypes.c_void_p
        if self.epi is not None:
            E, oE, sEi, sEj, RS, oRS, gamma = self.epi
            ep = (vp(E.data_ptr()), vp(oE.data_ptr()), sEi, sEj, vp(RS.data_ptr()), vp(oRS.data_ptr()), gamma)
        else:
            ep = (None, None, 0, 0, None, None, 0.0)
        kp = tuple(vp(t_.data_ptr()) for t_ in self.kseg) if self.kseg is not None else (None, None, None)
        if self.dstore is not None:
            D, oD, sDi = self.dstore
            L.check(L.lib().nmgp_gemm_big_offsets_dual_f32(
                vp(self.A.data_ptr()), lda, 1 if ak else 0, vp(self.B.data_ptr()), ldb, 1 if bk else 0,
                vp(self.C.data_ptr()), sCi, sCj, m, n, k, flags, alpha, beta, vp(self.off[0].data_ptr()),
                vp(self.off[1].data_ptr()), vp(self.off[2].data_ptr()), *ep, vp(D.data_ptr()), vp(oD.data_ptr()), sDi,
                self.batch, s), "gemm_big_offsets_dual")
            return
        if self.rseg is not None:
            seg, rs_, sp = self.rseg
            L.check(L.lib().nmgp_gemm_big_offsets_seg_f32(
                vp(self.A.data_ptr()), lda, 1 if ak else 0, vp(self.B.data_ptr()), ldb, 1 if bk else 0,
                vp(self.C.data_ptr()), sCi, sCj, m, n, k, flags, alpha, beta, dadd, vp(self.off[0].data_ptr()),
                vp(self.off[1].data_ptr()), vp(self.off[2].data_ptr()), *ep, vp(seg.data_ptr()), None, None,
                vp(rs_.data_ptr()), vp(sp.data_ptr()), self.batch, None, s), "gemm_big_offsets_seg")
            return
        L.check(L.lib().nmgp_gemm_big_offsets_epi_f32(vp(self.A.data_ptr()), lda, 1 if ak else 0,
                                                      vp(self.B.data_ptr()), ldb, 1 if bk else 0,
                                                      vp(self.C.data_ptr()), sCi, sCj, m, n, k, flags, alpha, beta,
                                                      dadd, vp(self.off[0].data_ptr()), vp(self.off[1].data_ptr()),
                                                      vp(self.off[2].data_ptr()), *ep, *kp, self.batch, None, s),
                "gemm_big_offsets_epi")


class PairStream:
    """One launch of a pair-block streaming product (csrc/pairs.hip) over many problems, descriptors uploaded
    once: kind "quad" C[r] = A[r] L, "dot" Z[r] = W[r] L^T, "rank" G(lower) += P^T W, "mv" c += A^T x (A = a, x = l,
    c = c); problem p uses rows
    seg[s_p] .. seg[s_p + 1] - 1 and operands at the element offsets (a_off, l_off, c_off) of the bases
    (a, l, c).  Graph-capturable (no allocation per call)."""

    FNS = {"quad": "nmgp_pair_quad_", "dot": "nmgp_pair_dot_", "rank": "nmgp_pair_rank_", "mv": "nmgp_pair_mv_"}

    def __init__(self, kind, a, l, c, probs, seg, M):
        assert kind in self.FNS
        for t_, nm in ((a, "a"), (l, "l"), (c, "c"), (seg, "seg")):
            L.require_device(t_, nm)
        assert a.dtype == l.dtype == c.dtype and seg.dtype == torch.int32
        self.kind, self.a, self.l, self.c, self.seg, self.M = kind, a, l, c, seg, int(M)
        self.dtype = a.dtype
        arr = (L.PairDesc * max(1, len(probs)))()
        for i, (ao, lo, co, s_) in enumerate(probs):
            arr[i].a_off, arr[i].l_off, arr[i].c_off, arr[i].seg = int(ao), int(lo), int(co), int(s_)
        self.n = len(probs)
        self.dev = torch.frombuffer(bytearray(bytes(memoryview(arr).cast("B"))), dtype=torch.uint8).to(a.device)

    def __call__(self, stream=None):
        if self.n == 0:
            return
        s = stream if stream is not None else L.stream_handle()
        vp = ctypes.c_void_p
        fn = getattr(L.lib(), self.FNS[self.kind] + _sfx(self.dtype))
        L.check(fn(vp(self.a.data_ptr()), vp(self.l.data_ptr()), vp(self.c.data_ptr()), vp(self.dev.data_ptr()),
                   self.n, vp(self.seg.data_ptr()), self.M, s), "pair_" + self.kind)


def pair_pbar_reduce(Z, sZ, P0, P1, ldp, seg, D, i0, i1, B, M, stream=None):
    """P1[r] += Z_i[r], P0[r] += Z_0[r] + ... + Z_{i-1}[r] for every row r of output i, i0 <= i < i1."""
    s = stream if stream is not None else L.stream_handle()
    vp = ctypes.c_void_p
    fn = getattr(L.lib(), "nmgp_pair_pbar_reduce_" + _sfx(Z.dtype))
    L.check(fn(vp(Z.data_ptr()), int(sZ), vp(P0.data_ptr()), vp(P1.data_ptr()), int(ldp), vp(seg.data_ptr()), int(D),
               int(i0), int(i1), int(B), int(M), s), "pair_pbar_reduce")


class Seq:
    """Launch callables one after another on the same stream (a composite schedule item)."""

    def __init__(self, parts):
        self.parts = list(parts)

    def __call__(self, stream=None):
        for p_ in self.parts:
            p_(stream)

    def macs(self, seg=None):
        """Algorithmic multiply-adds of the parts that are products (reductions and other launches add none)."""
        return sum(p_.macs(seg) for p_ in self.parts if hasattr(p_, "macs"))

    def algo_bytes(self, seg=None):
        return sum(p_.algo_bytes(seg) for p_ in self.parts if hasattr(p_, "algo_bytes"))


def potrf_blocked_(A, info=None, ws=None):
    """In-place lower Cholesky of ONE large SPD matrix A (n, n) on the blocked right-looking path with
    lookahead (include/nmgp_hip.h nmgp_potrf_blocked_*); strictly upper part zeroed.  Returns info
    (int32 (1,), first non-positive pivot column, 1-based, as LAPACK potrf)."""
    L.require_device(A, "A")
    assert A.dim() == 2 and A.shape[0] == A.shape[1] and A.is_contiguous()
    n = A.shape[0]
    if info is None:
        info = torch.zeros(1, dtype=torch.int32, device=A.device)
    lib = L.lib()
    sfx = _sfx(A.dtype)
    need = getattr(lib, "nmgp_potrf_blocked_workspace_size_" + sfx)(n)
    if ws is None:
        ws = big_workspace(A.device, need, tag="potrf")
    L.check(getattr(lib, "nmgp_potrf_blocked_" + sfx)(ctypes.c_void_p(A.data_ptr()), n, n,
                                                      ctypes.c_void_p(info.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                                      ws.numel(), L.stream_handle()), "potrf_blocked")
    return info


def gemm_big(A, B, C, *, b_kcontig=True, flags=0, alpha=1.0, beta=0.0, ctrans=False, ws=None, split=True):
    """C = alpha * A op(B) + beta * C on the 128x128 f32 MFMA kernel (gemm_big.hip).
    A (m, k) row-major; B (n, k) if b_kcontig (op(B) = B^T) else (k, n); C (m, n), or (n, m)
    holding C^T when ctrans.  Leading batch dimension optional (contiguous)."""
    for t, nm in ((A, "A"), (B, "B"), (C, "C")):
        L.require_device(t, nm)
        assert t.dtype == torch.float32 and t.is_contiguous()
    batched = A.dim() == 3
    m, k = A.shape[-2:]
    n = B.shape[-2] if b_kcontig else B.shape[-1]
    assert (B.shape[-1] if b_kcontig else B.shape[-2]) == k
    assert tuple(C.shape[-2:]) == ((n, m) if ctrans else (m, n))
    batch = A.shape[0] if batched else 1
    if split and ws is None:
        ws = big_workspace(A.device, L.lib().nmgp_gemm_big_workspace_size())
    sCi, sCj = (1, m) if ctrans else (n, 1)
    L.check(L.lib().nmgp_gemm_big_f32(ctypes.c_void_p(A.data_ptr()), k, ctypes.c_void_p(B.data_ptr()),
                                      B.shape[-1], 1 if b_kcontig else 0, ctypes.c_void_p(C.data_ptr()), sCi, sCj,
                                      m, n, k, flags, alpha, beta, m * k if batched else 0,
                                      B.shape[-2] * B.shape[-1] if batched else 0, m * n if batched else 0, batch,
                                      ctypes.c_void_p(ws.data_ptr()) if ws is not None else None,
                                      L.stream_handle()), "gemm_big")
    return C


def syevj(A):
    """Symmetric eigendecomposition (parallel cyclic / block Jacobi, eig.hip) of (n, n) or (batch, n, n)
    f64 device matrices: returns (w ascending, V with eigenvectors as columns), like torch.linalg.eigh."""
    L.require_device(A, "A")
    assert A.dtype == torch.float64
    A = A.contiguous()
    n = A.shape[-1]
    batch = A.numel() // (n * n) if n else 0
    w = torch.empty(A.shape[:-1], dtype=A.dtype, device=A.device)
    V = torch.empty_like(A)
    lib = L.lib()
    need = lib.nmgp_syevj_workspace_size_f64(n)
    ws = big_workspace(A.device, need, tag="syevj") if need > 0 else None
    L.check(lib.nmgp_syevj_batched_f64(ctypes.c_void_p(A.data_ptr()), n, n, n * n, batch,
                                       ctypes.c_void_p(w.data_ptr()), n, ctypes.c_void_p(V.data_ptr()), n, n * n,
                                       ctypes.c_void_p(ws.data_ptr()) if ws is not None else None,
                                       ws.numel() if ws is not None else 0, L.stream_handle()), "syevj")
    return w, V


# ------------------------------------------------------------------------------------ pairwise
def pairwise_desc(K, X, Z, *, mode, dist=L.DIST_DIFF, scale2=1.0, length_scale=1.0, ellX=None, ellZ=None,
                  sigX=None, sigZ=None, hyp=None, hyp_off=0, hyp_log=False, diag_add=0.0):
    d = L.PairwiseDesc()
    d.X, d.Z = _addr(X), _addr(Z)
    d.ellX, d.ellZ = _addr(ellX), _addr(ellZ)
    d.sigX, d.sigZ = _addr(sigX), _addr(sigZ)
    d.hyp = _addr(hyp, hyp_off) if hyp is not None else 0
    d.K = _addr(K)
    n, p = X.shape[0], (X.shape[1] if X.dim() > 1 else 1)
    m = Z.shape[0]
    d.ldk = K.shape[-1]
    d.n, d.m, d.p, d.mode, d.dist = n, m, p, mode, dist
    d.flags = L.HYP_LOG if hyp_log else 0
    d.scale2, d.length_scale, d.diag_add = float(scale2), float(length_scale), float(diag_add)
    d.tiles = ((n + 7) // 8) * ((m + 63) // 64)   # csrc/pairwise.hip PRF x PC forward tiles
    return d


def pairwise(X, Z, *, mode, dist=L.DIST_DIFF, scale2=1.0, length_scale=1.0, ellX=None, ellZ=None, sigX=None,
             sigZ=None, diag_add=0.0, out=None):
    L.require_device(X, "X")
    X = X.contiguous()
    Z = Z.contiguous()
    if out is None:
        out = torch.empty(X.shape[0], Z.shape[0], dtype=X.dtype, device=X.device)
    d = pairwise_desc(out, X, Z, mode=mode, dist=dist, scale2=scale2, length_scale=length_scale, ellX=ellX,
                      ellZ=ellZ, sigX=sigX, sigZ=sigZ, diag_add=diag_add)
    fn = getattr(L.lib(), "nmgp_pairwise_single_" + _sfx(X.dtype))
    L.check(fn(ctypes.byref(d), L.stream_handle()), "pairwise")
    return out


class PairwiseGroup:
    def __init__(self, descs, device):
        arr = (L.PairwiseDesc * len(descs))()
        t = 0
        for i, d in enumerate(descs):
            d.tile_start = t
            t += d.tiles
            arr[i] = d
        self.total, self.n = t, len(descs)
        self.dev = torch.frombuffer(bytearray(bytes(memoryview(arr).cast("B"))), dtype=torch.uint8).to(device)

    def __call__(self, dtype, stream=None):
        fn = getattr(L.lib(), "nmgp_pairwise_" + _sfx(dtype))
        L.check(fn(ctypes.c_void_p(self.dev.data_ptr()), self.n, self.total,
                   stream if stream is not None else L.stream_handle()), "pairwise group")


def pairwise_bwd_desc(X, Z, K, Rbar, *, mode, ld, Pm=None, rowcoef=None, ellX=None, ellZ=None, hyp=None,
                      hyp_off=0, hyp_log=False, scale2=1.0, length_scale=1.0, row_part=None, col_part=None,
                      scal_part=None, offs=(0, 0, 0, 0, 0, 0)):
    """offs = element offsets into (K, Rbar, Pm, row_part, col_part, scal_part)."""
    d = L.PairwiseBwdDesc()
    d.X, d.Z = _addr(X), _addr(Z)
    d.ellX, d.ellZ = _addr(ellX), _addr(ellZ)
    d.hyp = _addr(hyp, hyp_off) if hyp is not None else 0
    d.K, d.Rbar, d.Pm = _addr(K, offs[0]), _addr(Rbar, offs[1]), _addr(Pm, offs[2])
    d.rowcoef = _addr(rowcoef[0], rowcoef[1]) if rowcoef is not None else 0
    d.row_part = _addr(row_part, offs[3]) if row_part is not None else 0
    d.col_part = _addr(col_part, offs[4]) if col_part is not None else 0
    d.scal_part = _addr(scal_part, offs[5]) if scal_part is not None else 0
    n = X.shape[0]
    m = Z.shape[0]
    d.ld = ld
    d.n, d.m, d.p, d.mode = n, m, (X.shape[1] if X.dim() > 1 else 1), mode
    d.flags = L.HYP_LOG if hyp_log else 0
    d.scale2, d.length_scale = float(scale2), float(length_scale)
    d.tiles = ((n + 7) // 8) * ((m + 63) // 64)   # csrc/pairwise.hip PR x PC backward tiles
    return d


class PairwiseBwdGroup:
    def __init__(self, descs, device):
        arr = (L.PairwiseBwdDesc * len(descs))()
        t = 0
        self.starts = []
        for i, d in enumerate(descs):
            d.tile_start = t
            self.starts.append(t)
            t += d.tiles
            arr[i] = d
        self.total, self.n = t, len(descs)
        self.dev = torch.frombuffer(bytearray(bytes(memoryview(arr).cast("B"))), dtype=torch.uint8).to(device)

    def __call__(self, dtype, stream=None):
        fn = getattr(L.lib(), "nmgp_pairwise_bwd_" + _sfx(dtype))
        L.check(fn(ctypes.c_void_p(self.dev.data_ptr()), self.n, self.total,
                   stream if stream is not None else L.stream_handle()), "pairwise bwd group")


def bwd_tiles(n, m):
    """(tiles, column tiles, row tiles) of a pairwise backward launch (csrc/pairwise.hip: 8 x 64 tiles)."""
    return ((n + 7) // 8) * ((m + 63) // 64), (m + 63) // 64, (n + 7) // 8


def colsum(a2d, out, beta=0.0):
    L.check(getattr(L.lib(), "nmgp_colsum_" + _sfx(a2d.dtype))(ctypes.c_void_p(a2d.data_ptr()), a2d.shape[0],
                                                               a2d.shape[1], beta,
                                    ctypes.c_void_p(out.data_ptr()), L.stream_handle()), "colsum")
    return out


# ------------------------------------------------------------------------------------ Kronecker
def kron_product(t1, t2):
    L.require_device(t1, "t1")
    t1, t2 = t1.contiguous(), t2.contiguous()
    r1, c1 = t1.shape
    r2, c2 = t2.shape
    out = torch.empty(r1 * r2, c1 * c2, dtype=t1.dtype, device=t1.device)
    fn = getattr(L.lib(), "nmgp_kron_product_" + _sfx(t1.dtype))
    L.check(fn(ctypes.c_void_p(t1.data_ptr()), r1, c1, ctypes.c_void_p(t2.data_ptr()), r2, c2,
               ctypes.c_void_p(out.data_ptr()), L.stream_handle()), "kron_product")
    return out


KRON_MV_FUSED_MAXP = 8      # csrc/kron.hip KMV_MAXP


def kron_mv(B, K, y, out=None):
    L.require_device(B, "B")
    B, K, y = B.contiguous(), K.contiguous(), y.contiguous()
    P1, P2 = B.shape
    N1, N2 = K.shape
    assert y.numel() == P2 * N2
    if out is None:
        out = torch.empty(P1 * N1, dtype=B.dtype, device=B.device)
    # P2 <= 8: one fused launch streaming K once (csrc/kron.hip kron_mv_kernel); wider B: two GEMMs via `work`
    work = torch.empty(N1 * P2, dtype=B.dtype, device=B.device) if P2 > KRON_MV_FUSED_MAXP else None
    fn = getattr(L.lib(), "nmgp_kron_mv_" + _sfx(B.dtype))
    L.check(fn(ctypes.c_void_p(B.data_ptr()), P1, P2, ctypes.c_void_p(K.data_ptr()), N1, N2,
               ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(out.data_ptr()),
               ctypes.c_void_p(work.data_ptr()) if work is not None else None, L.stream_handle()), "kron_mv")
    return out


# ------------------------------------------------------------------------------------ graphs
class HipGraph:
    """A captured launch sequence replayed as one HIP graph, captured through the library's own C ABI
    (nmgp_graph_begin / _end / _launch) instead of torch.cuda.CUDAGraph: torch's capture_end crashed on a
    side <-> side2 event ping-pong of the step schedule that the HIP runtime captures cleanly.

        g = HipGraph(device)
        with g.capture():          # the body runs on g.stream (torch's current stream inside the block)
            body()                 # launches, event records / waits across streams; no allocation, no sync
        g.replay()                 # on torch's current stream

    The body's side streams must join back into the capture stream before the block ends."""

    def __init__(self, device=None):
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.stream = torch.cuda.Stream(device=self.device)
        self.exec = None

    class _Capture:
        def __init__(self, g):
            self.g = g

        def __enter__(self):
            g = self.g
            if g.exec is not None:
                raise RuntimeError("HipGraph already holds a captured graph")
            cur = torch.cuda.current_stream(g.device)
            g.stream.wait_stream(cur)           # everything enqueued before the capture comes first
            torch.cuda.synchronize(g.device)    # (and is finished: a capture must not wait on pending work)
            # the body must not allocate through torch: torch does not know a capture is running, so a block
            # allocated (and freed) inside it would be handed out again while the graph still writes into it
            self.alloc0 = torch.cuda.memory_stats(g.device).get("allocation.all.allocated", 0)
            L.check(L.lib().nmgp_graph_begin(ctypes.c_void_p(g.stream.cuda_stream)), "graph_begin")
            self.ctx = torch.cuda.stream(g.stream)
            self.ctx.__enter__()
            return g

        def __exit__(self, et, ev, tb):
            g = self.g
            ex = ctypes.c_void_p()
            rc = L.lib().nmgp_graph_end(ctypes.c_void_p(g.stream.cuda_stream), ctypes.byref(ex))
            self.ctx.__exit__(et, ev, tb)
            if et is not None or rc != 0:
                if rc == 0 and ex.value:        # the body raised after a clean capture: drop the graph
                    L.lib().nmgp_graph_destroy(ex)
                if et is None:
                    L.check(rc, "graph_end")
                return False
            allocs = torch.cuda.memory_stats(g.device).get("allocation.all.allocated", 0) - self.alloc0
            if allocs:
                if ex.value:
                    L.lib().nmgp_graph_destroy(ex)
                raise RuntimeError(f"HipGraph capture body allocated {allocs} block(s) through torch; captured "
                                   "bodies must use preallocated buffers")
            g.exec = ex
            return False

    def capture(self):
        return HipGraph._Capture(self)

    def replay(self, stream=None):
        if self.exec is None:
            raise RuntimeError("HipGraph.replay before capture")
        s = stream if stream is not None else L.stream_handle(self.device)
        L.check(L.lib().nmgp_graph_launch(self.exec, s), "graph_launch")

    def __del__(self):
        ex = getattr(self, "exec", None)
        if ex is not None and L._lib is not None:
            try:
                L._lib.nmgp_graph_destroy(ex)
            except Exception:
                pass
            self.exec = None


class ExtEvent:
    """A HIP event that a captured graph records as an EXTERNAL event node (nmgp_event_record_external): after
    the graph is launched, `wait(stream)` makes a stream outside the graph wait for that point INSIDE the replay
    (outside a capture the record is an ordinary event record)."""

    def __init__(self):
        h = ctypes.c_void_p()
        L.check(L.lib().nmgp_event_create(ctypes.byref(h)), "event_create")
        self.h = h

    def record(self, stream):
        L.check(L.lib().nmgp_event_record_external(self.h, ctypes.c_void_p(stream.cuda_stream)), "event_record")

    def wait(self, stream):
        L.check(L.lib().nmgp_stream_wait_event(ctypes.c_void_p(stream.cuda_stream), self.h), "stream_wait_event")

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value and L._lib is not None:
            try:
                L._lib.nmgp_event_destroy(h)
            except Exception:
                pass
            self.h = None


# ------------------------------------------------------------------------------------ optimiser / rng
def adam_(theta, grad, m, v, step, lr, betas=(0.9, 0.999), eps=1e-8):
    fn = getattr(L.lib(), "nmgp_adam_" + _sfx(theta.dtype))
    L.check(fn(ctypes.c_void_p(theta.data_ptr()), ctypes.c_void_p(grad.data_ptr()), ctypes.c_void_p(m.data_ptr()),
               ctypes.c_void_p(v.data_ptr()), theta.numel(), ctypes.c_void_p(step.data_ptr()), float(lr),
               float(betas[0]), float(betas[1]), float(eps), L.stream_handle()), "adam")


def adam_lower_(theta, grad, m, v, step, lr, tri, M, betas=(0.9, 0.999), eps=1e-8):
    """adam_ with the ranges `tri` = [(offset, blocks), ...] of the flat vector treated as lower-triangular
    M x M blocks (only their lower-triangle vectors are read / written; bit-identical results)."""
    fn = getattr(L.lib(), "nmgp_adam_lower_" + _sfx(theta.dtype))
    arr = (ctypes.c_int64 * max(1, 2 * len(tri)))(*[int(x) for ab in tri for x in ab])
    L.check(fn(ctypes.c_void_p(theta.data_ptr()), ctypes.c_void_p(grad.data_ptr()), ctypes.c_void_p(m.data_ptr()),
               ctypes.c_void_p(v.data_ptr()), theta.numel(), arr, len(tri), int(M), ctypes.c_void_p(step.data_ptr()),
               float(lr), float(betas[0]), float(betas[1]), float(eps), L.stream_handle()), "adam_lower")


def adam_lower_advanced_(theta, grad, m, v, step, lr, tri, M, betas=(0.9, 0.999), eps=1e-8):
    """adam_lower_ for a step counter already advanced for this step (by the finalize kernel: the engine's
    adam_step); one launch, the counter untouched."""
    fn = getattr(L.lib(), "nmgp_adam_lower_advanced_" + _sfx(theta.dtype))
    arr = (ctypes.c_int64 * max(1, 2 * len(tri)))(*[int(x) for ab in tri for x in ab])
    L.check(fn(ctypes.c_void_p(theta.data_ptr()), ctypes.c_void_p(grad.data_ptr()), ctypes.c_void_p(m.data_ptr()),
               ctypes.c_void_p(v.data_ptr()), theta.numel(), arr, len(tri), int(M), ctypes.c_void_p(step.data_ptr()),
               float(lr), float(betas[0]), float(betas[1]), float(eps), L.stream_handle()), "adam_lower_advanced")


def normal_(out, seed, counter=None, offset=0):
    fn = getattr(L.lib(), "nmgp_normal_" + _sfx(out.dtype))
    L.check(fn(ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.c_uint64(seed),
               ctypes.c_void_p(counter.data_ptr()) if counter is not None else None,
               int(offset), L.stream_handle()), "normal")
    return out


def counter_add_(counter, inc):
    L.check(L.lib().nmgp_counter_add(ctypes.c_void_p(counter.data_ptr()), int(inc), L.stream_handle()), "counter")
