"""HIP primitives vs float64 CPU references (GEMM, potrf, trtri, builders, Kronecker, Adam, RNG)."""
import numpy as np
import pytest
import torch

from oracle import nmgp_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"
F64 = torch.float64


@pytest.fixture(scope="module")
def ops():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib
    _lib.lib()
    return hip_ops


def rel(a, b):
    a = a.detach().double().cpu().reshape(-1)
    b = b.detach().double().cpu().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


@pytest.mark.parametrize("m,n,k", [(64, 64, 16), (37, 23, 19), (200, 130, 257), (1, 5, 3)])
@pytest.mark.parametrize("tA,tB", [(False, False), (True, False), (False, True), (True, True)])
def test_gemm_transposes(ops, m, n, k, tA, tB):
    g = torch.Generator().manual_seed(m * 7 + n + k)
    A = torch.randn((k, m) if tA else (m, k), generator=g, dtype=F64)
    B = torch.randn((n, k) if tB else (k, n), generator=g, dtype=F64)
    ref = (A.t() if tA else A) @ (B.t() if tB else B)
    out = ops.matmul(A.to(DEV), B.to(DEV), transA=tA, transB=tB)
    assert rel(out, ref) < 1e-14


def test_gemm_f32(ops):
    g = torch.Generator().manual_seed(3)
    A = torch.randn(150, 70, generator=g, dtype=F64)
    B = torch.randn(70, 90, generator=g, dtype=F64)
    out = ops.matmul(A.float().to(DEV), B.float().to(DEV))
    assert rel(out, A @ B) < 1e-6


def test_gemm_masks_kscale_epilogue_diag(ops):
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    g = torch.Generator().manual_seed(5)
    n = 100
    S = torch.randn(n, n, generator=g, dtype=F64)
    s = torch.rand(n, generator=g, dtype=F64)
    E = torch.randn(n, n, generator=g, dtype=F64)
    rs = torch.randn(n, generator=g, dtype=F64)
    C0 = torch.randn(n, n, generator=g, dtype=F64)
    Ld = torch.tril(S)
    # C = 0.5 * tril(S) diag(s) tril(S)^T + 2*C0 - 1.5 * diag(rs) tril(E) + 0.25 I , lower-stored
    ref = 0.5 * Ld @ torch.diag(s) @ Ld.t() + 2 * C0 - 1.5 * rs[:, None] * torch.tril(E) + 0.25 * torch.eye(n, dtype=F64)
    Sd, sd, Ed, rsd = S.to(DEV), s.to(DEV), E.to(DEV), rs.to(DEV)
    C = C0.clone().to(DEV)
    d = ops.gemm_desc(C, Sd, Sd, n, n, n, (n, 1, 0), (1, n, 0), (n, 1),
                      flags=L.A_LOWER | L.B_UPPER | L.EPI_E_LOWER | L.EPI_RS_NEG, alpha=0.5, beta=2.0,
                      kscale=(sd, 0), epi=(Ed, 0, (n, 1), (rsd, 0), 1.5), diag_add=0.25)
    ops.gemm_single(d, F64)
    assert rel(C, ref) < 1e-14
    # OUT_TRIL: only the lower triangle, zeros above
    C2 = torch.full((n, n), 7.0, dtype=F64, device=DEV)
    d = ops.gemm_desc(C2, Sd, Sd, n, n, n, (n, 1, 0), (1, n, 0), (n, 1), flags=L.OUT_TRIL)
    ops.gemm_single(d, F64)
    assert rel(C2, torch.tril(S @ S.t())) < 1e-14


def test_gemm_kblocks_and_segments_grouped(ops):
    """k-concatenated blocks (sum_j W_j L_j^T) and run-time row / k segments in one grouped launch."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    g = torch.Generator().manual_seed(9)
    D, B, M = 3, 150, 40
    W = torch.randn(D, B, M, generator=g, dtype=F64)
    S = torch.randn(D, M, M, generator=g, dtype=F64)
    seg = torch.tensor([0, 40, 95, 150], dtype=torch.int32)
    Wd, Sd, segd = W.to(DEV), S.to(DEV), seg.to(DEV)
    out1 = torch.zeros(B, M, dtype=F64, device=DEV)
    out2 = torch.zeros(M, M, dtype=F64, device=DEV)
    out3 = torch.full((B, M), 3.0, dtype=F64, device=DEV)
    descs = [
        # out1 = sum_d W[d] tril(S[d])^T           (k = d*M + c, kb = M)
        ops.gemm_desc(out1, Wd, Sd, B, M, D * M, (M, 1, B * M), (1, M, M * M), (M, 1), flags=L.B_UPPER, kb=(M, M)),
        # out2 = W[1][rows seg 1..2]^T W[2][same rows]   (k over a 2-segment span)
        ops.gemm_desc(out2, Wd, Wd, M, M, B, (1, M, 0), (M, 1, 0), (M, 1), k_seg=1, seg_span=2, offs=(B * M, 2 * B * M, 0)),
        # out3[rows of seg 0] = W[0][seg 0] S[0]  (others untouched)
        ops.gemm_desc(out3, Wd, Sd, B, M, M, (M, 1, 0), (M, 1, 0), (M, 1), row_seg=0),
    ]
    grp = ops.GemmGroup(descs, DEV, F64, seg=segd)
    grp()
    ref1 = sum(W[d] @ torch.tril(S[d]).t() for d in range(D))
    assert rel(out1, ref1) < 1e-14
    ref2 = W[1][40:150].t() @ W[2][40:150]
    assert rel(out2, ref2) < 1e-14
    ref3 = torch.full((B, M), 3.0, dtype=F64)
    ref3[0:40] = W[0][0:40] @ S[0]
    assert rel(out3, ref3) < 1e-14


@pytest.mark.parametrize("dt", [F64, torch.float32])
def test_gemm_group_kt_cap_max_grid(ops, dt):
    """GemmGroup(kt_cap=) (split-K so no workgroup runs more than kt_cap k-tiles) and GemmGroup(max_grid=)
    (fewer workgroups striding over the tiles: device plan for row-segmented groups, a static plan
    otherwise) against torch references on k-blocked, row-segmented and k-segmented problems; the
    caller's descriptors are left untouched (the group works on copies)."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    g = torch.Generator().manual_seed(21)
    D, B, M = 4, 700, 128
    W = torch.randn(D, B, M, generator=g, dtype=F64)
    S = torch.randn(D, M, M, generator=g, dtype=F64)
    seg = torch.tensor([0, 100, 330, 520, 700], dtype=torch.int32)
    Wd, Sd, segd = W.to(dt).to(DEV), S.to(dt).to(DEV), seg.to(DEV)
    Wc, Sc = Wd.double().cpu(), Sd.double().cpu()
    tol = 1e-13 if dt == F64 else 3e-6
    for kw in (dict(), dict(kt_cap=2), dict(max_grid=7), dict(kt_cap=3, max_grid=5)):
        out1 = torch.zeros(B, M, dtype=dt, device=DEV)
        out2 = torch.zeros(D, M, M, dtype=dt, device=DEV)
        descs = []
        for i in range(D):   # rows of segment i: sum_{d <= i} W[d] tril(S[d])^T
            descs.append(ops.gemm_desc(out1, Wd, Sd, B, M, (i + 1) * M, (M, 1, B * M), (1, M, M * M), (M, 1),
                                       flags=L.B_UPPER, kb=(M, M), row_seg=i))
        # out2[d] = W[d][rows of segments d..]^T W[d][same rows]   (long k: split by kt_cap)
        descs += [ops.gemm_desc(out2, Wd, Wd, M, M, B, (1, M, 0), (M, 1, 0), (M, 1), k_seg=d, seg_span=D - d,
                                offs=(d * B * M, d * B * M, d * M * M), flags=L.OUT_TRIL) for d in range(D)]
        grp = ops.GemmGroup(descs, DEV, dt, seg=segd, **kw)     # (kt_cap / max_grid force the tile kernel)
        assert not grp.lat or not kw
        assert all(d.ksplit == 0 and d.tile_start == 0 for d in descs)
        if "kt_cap" in kw:
            assert max(x.ksplit for x in grp.descs) > 1
        if "max_grid" in kw:
            assert grp.plan is not None and grp.grid == kw["max_grid"]
        grp()
        sc = seg.tolist()
        ref1 = torch.zeros(B, M, dtype=F64)
        for i in range(D):
            r0, r1 = sc[i], sc[i + 1]
            ref1[r0:r1] = sum(Wc[d][r0:r1] @ torch.tril(Sc[d]).t() for d in range(i + 1))
        assert rel(out1, ref1) < tol, kw
        for d in range(D):
            r0 = sc[d]
            assert rel(out2[d], torch.tril(Wc[d][r0:].t() @ Wc[d][r0:])) < tol, (kw, d)


@pytest.mark.parametrize("dt", [F64, torch.float32])
def test_gemm_grouped_device_plan(ops, dt):
    """Row-segmented groups sized on device (plan kernel + grid-stride tiles) equal the static launch
    bit for bit, including an empty segment, a segment longer than the static estimate and split-K."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    g = torch.Generator().manual_seed(11)
    D, B, M = 6, 900, 96
    W = torch.randn(D, B, M, generator=g, dtype=F64).to(dt).to(DEV)
    S = torch.randn(D, M, M, generator=g, dtype=F64).to(dt).to(DEV)
    seg = torch.tensor([0, 0, 610, 700, 701, 840, 900], dtype=torch.int32, device=DEV)   # segment 0 empty
    outs = []
    for dyn in (False, True):
        out = torch.full((B, M), 2.0, dtype=dt, device=DEV)
        out2 = torch.zeros(D, M, M, dtype=dt, device=DEV)
        descs = [ops.gemm_desc(out, W, S, B, M, M, (M, 1, 0), (M, 1, 0), (M, 1), row_seg=d,
                               offs=(d * B * M, d * M * M, 0), alpha=0.5, beta=1.0) for d in range(D)]
        # out2[d] = W[d][rows of segment d]^T W[d][same rows]  (k over the segment: split-K)
        descs += [ops.gemm_desc(out2, W, W, M, M, B, (1, M, 0), (M, 1, 0), (M, 1), k_seg=d,
                                offs=(d * B * M, d * B * M, d * M * M)) for d in range(D)]
        grp = ops.GemmGroup(descs, DEV, dt, seg=seg, dyn_plan="force" if dyn else False)
        assert (grp.plan is not None) == dyn
        grp()
        grp()
        outs.append((out.clone(), out2.clone()))
    assert torch.equal(outs[0][1], outs[1][1])
    Wc, Sc, sc = W.double().cpu(), S.double().cpu(), seg.cpu().tolist()
    ref = torch.full((B, M), 2.0, dtype=F64)
    for d in range(D):
        r0, r1 = sc[d], sc[d + 1]
        for _ in range(2):
            ref[r0:r1] = 0.5 * (Wc[d][r0:r1] @ Sc[d]) + ref[r0:r1]
    tol = 1e-13 if dt == F64 else 2e-6
    assert rel(outs[1][0], ref) < tol and torch.equal(outs[0][0], outs[1][0])


@pytest.mark.parametrize("pipe", ["0", "force"])
@pytest.mark.parametrize("dt", [F64, torch.float32])
def test_gemm_latency_kernel(ops, dt, pipe, monkeypatch):
    """gemm_lat.hip (32x32 tiles, k split over the waves, register-direct operands) on the descriptor
    features the DSVI step uses: triangular operands whose zero triangles hold inf, k-scaling, the
    rs(i) E epilogue, diagonal add, beta, OUT_LOWER / OUT_TRIL, transposed operands, k-blocked
    operands (kb = 64), row / k segments, the device tile plan; repeat launches are bit-identical.
    pipe="force": the persistent two-tiles-in-flight launch (one workgroup per CU walking several tiles)."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    monkeypatch.setattr(ops, "_LAT_PIPE", pipe)
    g = torch.Generator().manual_seed(21)
    n, B, D, M = 100, 330, 3, 64
    S = torch.randn(n, n, generator=g, dtype=F64)
    Sinf = torch.tril(S) + torch.triu(torch.full((n, n), float("inf"), dtype=F64), 1)   # inf above the diagonal
    s = torch.rand(n, generator=g, dtype=F64)
    E = torch.randn(n, n, generator=g, dtype=F64)
    rs = torch.randn(n, generator=g, dtype=F64)
    C0 = torch.randn(n, n, generator=g, dtype=F64)
    W = torch.randn(D, B, M, generator=g, dtype=F64)
    U = torch.randn(D, M, M, generator=g, dtype=F64)
    seg = torch.tensor([0, 120, 121, 330], dtype=torch.int32)
    P = torch.randn(1500, M, generator=g, dtype=F64)
    C40 = torch.randn(M, M, generator=g, dtype=F64)
    dv = lambda x: x.to(dt).to(DEV)
    Pd = dv(P)
    Sd, sd, Ed, rsd, Wd, Ud, segd = dv(Sinf), dv(s), dv(E), dv(rs), dv(W), dv(U), seg.to(DEV)
    Wc, Uc, Sc = W.to(dt).double(), U.to(dt).double(), torch.tril(S.to(dt).double())
    results = []
    for rep in range(2):
        C1 = dv(C0)
        C2 = torch.full((n, n), 7.0, dtype=dt, device=DEV)
        C3 = torch.full((n, n), 7.0, dtype=dt, device=DEV)
        O1 = torch.zeros(B, M, dtype=dt, device=DEV)
        O2 = torch.zeros(M, M, dtype=dt, device=DEV)
        O3 = torch.full((B, M), 3.0, dtype=dt, device=DEV)
        O4 = dv(C40)
        descs = [
            # C1 = 0.5 L diag(s) L^T + 2 C0 - 1.5 diag(rs) tril(E) + 0.25 I   (L = tril(S): A_LOWER, B_UPPER)
            ops.gemm_desc(C1, Sd, Sd, n, n, n, (n, 1, 0), (1, n, 0), (n, 1),
                          flags=L.A_LOWER | L.B_UPPER | L.EPI_E_LOWER | L.EPI_RS_NEG, alpha=0.5, beta=2.0,
                          kscale=(sd, 0), epi=(Ed, 0, (n, 1), (rsd, 0), 1.5), diag_add=0.25),
            # C2 = tril(L^T L) with zeros above (A = L^T: A_UPPER, B = L: B_LOWER)
            ops.gemm_desc(C2, Sd, Sd, n, n, n, (1, n, 0), (n, 1, 0), (n, 1), flags=L.A_UPPER | L.B_LOWER | L.OUT_TRIL),
            # C3 lower part only of L L^T (upper untouched)
            ops.gemm_desc(C3, Sd, Sd, n, n, n, (n, 1, 0), (1, n, 0), (n, 1), flags=L.A_LOWER | L.B_UPPER | L.OUT_LOWER),
            # O1 = sum_d W[d] tril(U[d])^T   (k-blocked, kb = M = 64)
            ops.gemm_desc(O1, Wd, Ud, B, M, D * M, (M, 1, B * M), (1, M, M * M), (M, 1), flags=L.B_UPPER, kb=(M, M)),
            # O2 = W[1][rows of segments 1..2]^T W[2][same rows]
            ops.gemm_desc(O2, Wd, Wd, M, M, B, (1, M, 0), (M, 1, 0), (M, 1), k_seg=1, seg_span=2, offs=(B * M, 2 * B * M, 0)),
            # O3[rows of segment 2] = W[0][seg 2] U[0] + O3
            ops.gemm_desc(O3, Wd, Ud, B, M, M, (M, 1, 0), (M, 1, 0), (M, 1), row_seg=2, beta=1.0),
            # O4 = C40 - P^T P  (k = 1500: split over workgroups, last-arriver combine)
            ops.gemm_desc(O4, Pd, Pd, M, M, 1500, (1, M, 0), (M, 1, 0), (M, 1), alpha=-1.0, beta=1.0),
        ]
        grp = ops.GemmGroup(descs, DEV, dt, seg=segd, kernel="lat", dyn_plan="force" if rep else False)
        assert grp.lat and (grp.plan is not None) == bool(rep) and grp.pipe == (pipe == "force")
        assert max(d.ksplit for d in grp.descs) > 1
        grp()
        results.append([x.cpu() for x in (C1, C2, C3, O1, O2, O3, O4)])
    tol = 1e-13 if dt == F64 else 3e-6
    ref1 = 0.5 * Sc @ torch.diag(s.to(dt).double()) @ Sc.t() + 2 * C0.to(dt).double() \
        - 1.5 * rs.to(dt).double()[:, None] * torch.tril(E.to(dt).double()) + 0.25 * torch.eye(n, dtype=F64)
    ref2 = torch.tril(Sc.t() @ Sc)
    ref3 = torch.tril(Sc @ Sc.t()) + torch.triu(torch.full((n, n), 7.0, dtype=F64), 1)
    refO1 = sum(Wc[d] @ torch.tril(Uc[d]).t() for d in range(D))
    refO2 = Wc[1][120:330].t() @ Wc[2][120:330]
    refO3 = torch.full((B, M), 3.0, dtype=F64)
    refO3[121:330] += Wc[0][121:330] @ Uc[0]
    Pc = P.to(dt).double()
    refO4 = C40.to(dt).double() - Pc.t() @ Pc
    for got in results:
        for a, r in zip(got, (ref1, ref2, ref3, refO1, refO2, refO3, refO4)):
            assert torch.isfinite(a).all() and rel(a, r) < tol
    for a, b in zip(*results):          # static grid vs device plan: same tiles, same order of sums
        assert torch.equal(a, b)


@pytest.mark.parametrize("dt", [F64, torch.float32])
def test_gemm_lat_persistent_walks_many_tiles(ops, dt, monkeypatch):
    """The persistent latency launch (one workgroup per CU, the next tile's first panel loaded under the current
    tile's MFMAs and reduction) over groups of thousands of tiles -- row segments with the device plan, a
    B-triangular operand, a k range of several rounds (k = 600: 19 panels per 8 waves) and an odd tile count --
    equals the one-tile-per-workgroup launch bit for bit, and the float64 reference."""
    g = torch.Generator().manual_seed(5)
    Bn, M, D, K2 = 6007, 256, 3, 600
    W = torch.randn(D, Bn, M, generator=g, dtype=F64)
    U = torch.randn(D, M, M, generator=g, dtype=F64)
    A2 = torch.randn(1000, K2, generator=g, dtype=F64)
    B2 = torch.randn(K2, 160, generator=g, dtype=F64)
    seg = torch.tensor([0, 1800, 4100, Bn], dtype=torch.int32, device=DEV)
    dv = lambda x: x.to(dt).to(DEV)
    Wd, Ud, A2d, B2d = dv(W), dv(U), dv(A2), dv(B2)
    out = {}
    for pipe in ("0", "force"):
        monkeypatch.setattr(ops, "_LAT_PIPE", pipe)
        Z = torch.zeros(D, Bn, M, dtype=dt, device=DEV)
        C2 = torch.zeros(1000, 160, dtype=dt, device=DEV)
        descs = [ops.gemm_desc(Z, Wd, Ud, Bn, M, M, (M, 1, 0), (1, M, 0), (M, 1), flags=L_B_UPPER(),
                               offs=(d * Bn * M, d * M * M, d * Bn * M), row_seg=d, seg_span=D - d) for d in range(D)]
        grp = ops.GemmGroup(descs, DEV, dt, seg=seg, kernel="lat", dyn_plan="force")
        grp2 = ops.GemmGroup([ops.gemm_desc(C2, A2d, B2d, 1000, 160, K2, (K2, 1, 0), (160, 1, 0), (160, 1))], DEV, dt,
                             kernel="lat")
        assert grp.pipe == grp2.pipe == (pipe == "force") and grp.total > 1024
        grp()
        grp2()
        grp2()           # a second launch: split-K counters (if any) were re-armed
        out[pipe] = (Z.cpu(), C2.cpu())
    assert torch.equal(out["0"][0], out["force"][0]) and torch.equal(out["0"][1], out["force"][1])
    Wc, Uc = W.to(dt).double(), U.to(dt).double()
    ref = torch.zeros(D, Bn, M, dtype=F64)
    for d in range(D):
        r0 = int(seg[d])
        ref[d, r0:] = Wc[d, r0:] @ torch.tril(Uc[d]).t()     # (B_UPPER over B(k, j) = U[j, k])
    tol = 1e-13 if dt == F64 else 3e-6
    assert rel(out["force"][0], ref) < tol
    assert rel(out["force"][1], A2.to(dt).double() @ B2.to(dt).double()) < tol


def L_B_UPPER():
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    return L.B_UPPER


def test_gemm_latency_kernel_dsvi_step(ops, monkeypatch):
    """The PM2.5-shaped step (D=5, M=256, B=2000) with the latency kernel on its short-k groups equals
    the step with every group on the 64x64 tile kernel: loss and whole gradient to rounding."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
    import collaborative_nonstationary_multivariate_gaussian_process_amd.hip_ops as H
    D, M, B = 5, 256, 2000
    rng = np.random.default_rng(3)
    xs = [torch.from_numpy(np.sort(rng.uniform(0, 1, 400))) for _ in range(D)]
    ys = [torch.from_numpy(rng.standard_normal(400)) for _ in range(D)]
    res = {}
    for mode in ("0", "auto"):
        monkeypatch.setattr(H, "_LAT_MODE", mode)
        model = NMGP(number_observations=D * 400, dim_outputs=D, Z=np.linspace(0, 1, M), minibatch_size=B, seed=2,
                     device=DEV, noise="device")
        eng = model.engine(B)
        x, y, sizes = model._prepare(xs, ys)
        eng.load_batch(x, y, sizes)
        loss = DsviTrainer(model, 0.01).grad_step(eng)
        torch.cuda.synchronize()
        nlat = sum(1 for _, g_ in eng.gemm_groups() if getattr(g_, "lat", False))
        res[mode] = (float(loss), model._grad.detach().cpu().clone(), nlat)
    assert res["0"][2] == 0 and res["auto"][2] > 0
    assert abs(res["auto"][0] - res["0"][0]) <= 1e-12 * abs(res["0"][0])
    assert rel(res["auto"][1], res["0"][1]) < 1e-11


@pytest.mark.parametrize("K", [600, 2000, 4099])
def test_gemm_split_k_deterministic(ops, K):
    """Long-k products P^T R (few output tiles) take the split-K path; results are bit-identical
    across launches (fixed-order reduction of the chunk partials)."""
    g = torch.Generator().manual_seed(K)
    M = 100
    P = torch.randn(K, M, generator=g, dtype=F64)
    R = torch.randn(K, M, generator=g, dtype=F64)
    C0 = torch.randn(M, M, generator=g, dtype=F64)
    Pd, Rd = P.to(DEV), R.to(DEV)
    outs = []
    for rep in range(3):
        C = C0.clone().to(DEV)
        d = ops.gemm_desc(C, Pd, Rd, M, M, K, (1, M, 0), (M, 1, 0), (M, 1), alpha=-1.0, beta=1.0)
        grp = ops.GemmGroup([d], DEV, F64, kernel="tile")
        assert grp.descs[0].ksplit > 1
        grp()
        grp()          # counters were reset by the last arrivers: a second launch is valid too
        outs.append(C.cpu())
    ref = C0 - 2 * P.t() @ R
    assert rel(outs[0], ref) < 1e-13
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])


def _spd(n, batch, seed, cond_shift=0.1):
    g = torch.Generator().manual_seed(seed)
    G = torch.randn(batch, n, n + 3, generator=g, dtype=F64)
    return G @ G.transpose(-1, -2) / n + cond_shift * torch.eye(n, dtype=F64)


@pytest.mark.parametrize("n,batch", [(20, 3), (64, 2), (100, 5), (256, 4), (257, 1)])
def test_potrf_trtri(ops, n, batch):
    A = _spd(n, batch, n)
    Ld = A.clone().to(DEV)
    info = ops.potrf_(Ld)
    assert int(info.abs().sum()) == 0
    ref = torch.linalg.cholesky(A)
    assert rel(Ld, ref) < 1e-13
    X = ops.trtri(Ld)
    assert rel(X, torch.linalg.inv(ref)) < 1e-11
    assert float(torch.triu(X.cpu(), 1).abs().max()) == 0.0


@pytest.mark.parametrize("n,batch", [(16, 2), (20, 3), (48, 1), (64, 2), (100, 5), (176, 2), (256, 4), (257, 1)])
def test_chol_inv_fused(ops, n, batch):
    # n <= 256 runs the register-resident fused kernel (every tile-count bucket), 257 the fallback
    A = _spd(n, batch, 7 * n)
    Ad = A.clone().to(DEV)
    X, info = ops.chol_inv_(Ad)
    assert int(info.abs().sum()) == 0
    ref = torch.linalg.cholesky(A)
    assert rel(Ad, ref) < 1e-13
    assert rel(X, torch.linalg.inv(ref)) < 1e-11
    assert float(torch.triu(Ad.cpu(), 1).abs().max()) == 0.0
    assert float(torch.triu(X.cpu(), 1).abs().max()) == 0.0


@pytest.mark.parametrize("n,batch", [(128, 1), (176, 3), (192, 2), (250, 1), (256, 1), (256, 4), (256, 25)])
@pytest.mark.parametrize("dt", [F64, torch.float32])
def test_chol_inv_four_role_matches_three_role(ops, n, batch, dt, monkeypatch):
    """The four-role kernel (chol_inv7_kernel: the trailing update on its own workgroup, the factor applies
    only the last step to each block column) gives every tile the three-role kernel's MFMA updates in the
    same order: L and L^-1 bit-identical, the same info for a non-PD matrix, control words cleared."""
    A = _spd(n, batch, 13 * n + batch).to(dt)
    if batch > 2:
        A[1, n // 2, n // 2] = -5.0                    # not PD from column n // 2 on
    res = []
    for four in ("1", "0"):
        monkeypatch.setenv("NMGP_CHOL_4ROLE", four)
        Ad = A.clone().to(DEV)
        X = torch.full_like(Ad, float("nan"))          # stale control words must not pass for progress
        X, info = ops.chol_inv_(Ad, out=X)
        torch.cuda.synchronize()
        res.append((Ad.cpu(), X.cpu(), info.cpu()))
    (L1, X1, i1), (L0, X0, i0) = res
    assert torch.equal(i1, i0)
    if batch > 2:
        assert int(i1[1]) == n // 2 + 1 and int(i1[0]) == 0
    ok = [b for b in range(batch) if int(i1[b]) == 0]
    assert torch.equal(L1[ok], L0[ok]) and torch.equal(X1[ok], X0[ok])
    ref = torch.linalg.cholesky(A[ok].double())
    tl, tx = (1e-13, 1e-11) if dt == F64 else (1e-5, 1e-4)
    assert rel(L1[ok], ref) < tl and rel(X1[ok], torch.linalg.inv(ref)) < tx
    assert float(torch.triu(L1[ok], 1).abs().max()) == 0.0 and float(torch.triu(X1[ok], 1).abs().max()) == 0.0


@pytest.mark.parametrize("n,batch,dt", [(300, 2, F64), (512, 2, F64), (700, 1, F64), (520, 2, torch.float32),
                                        (1000, 1, torch.float32), (2048, 1, torch.float32)])
def test_chol_inv_blocked(ops, n, batch, dt):
    # n > 256: blocked path (128-wide diagonal blocks + batched GEMM panel / SYRK / inverse products)
    A = _spd(n, batch, n + 1)
    Ad = A.to(dt).to(DEV)
    X, info = ops.chol_inv_(Ad)
    assert int(info.abs().sum()) == 0
    ref = torch.linalg.cholesky(A)
    tl, tx = (1e-13, 1e-11) if dt == F64 else (1e-5, 1e-4)
    assert rel(Ad, ref) < tl
    assert rel(X, torch.linalg.inv(ref)) < tx
    assert float(torch.triu(Ad.cpu(), 1).abs().max()) == 0.0
    assert float(torch.triu(X.cpu(), 1).abs().max()) == 0.0


def _f32_ref(A, opB, flags, alpha=1.0, beta=0.0, C=None):
    A = A.double()
    opB = opB.double()
    if flags & 1:                       # A_LOWER
        A = torch.tril(A)
    if flags & 8:                       # B_UPPER: op(B)(k, j) = 0 for j < k
        opB = torch.triu(opB)
    if flags & 4:                       # B_LOWER: op(B)(k, j) = 0 for j > k
        opB = torch.tril(opB)
    out = alpha * A @ opB
    if C is not None:
        out = out + beta * C.double()
    return out


@pytest.mark.parametrize("m,n,k", [(128, 128, 32), (300, 200, 77), (1, 7, 5), (640, 384, 1000), (256, 256, 2048)])
@pytest.mark.parametrize("b_kcontig", [True, False])
def test_gemm_big_f32(ops, m, n, k, b_kcontig):
    # 128x128 f32 MFMA kernel (gemm_big.hip) vs fp64: tolerance of an exact-f32 fma chain over k
    g = torch.Generator().manual_seed(m + 3 * n + 7 * k)
    A = torch.randn(m, k, generator=g)
    B = torch.randn((n, k) if b_kcontig else (k, n), generator=g)
    C0 = torch.randn(m, n, generator=g)
    opB = B.t() if b_kcontig else B
    for alpha, beta in ((1.0, 0.0), (-1.0, 1.0)):
        C = C0.clone().to(DEV)
        ops.gemm_big(A.to(DEV), B.to(DEV), C, b_kcontig=b_kcontig, alpha=alpha, beta=beta)
        assert rel(C, _f32_ref(A, opB, 0, alpha, beta, C0)) < 2e-6
    # transposed store
    Ct = torch.zeros(n, m, device=DEV)
    ops.gemm_big(A.to(DEV), B.to(DEV), Ct, b_kcontig=b_kcontig, ctrans=True)
    assert rel(Ct.t(), _f32_ref(A, opB, 0)) < 2e-6


@pytest.mark.parametrize("flags,b_kcontig", [(1, True), (8, True), (4, False), (16, True)])
def test_gemm_big_masks_and_syrk(ops, flags, b_kcontig):
    # triangular operands: garbage outside the triangle must not leak (masked k-tiles); SYRK stores lower only
    n = 520
    g = torch.Generator().manual_seed(flags)
    A = torch.randn(n, n, generator=g)
    B = A.clone() if flags == 16 else torch.randn(n, n, generator=g)
    C0 = torch.randn(n, n, generator=g)
    C = C0.clone().to(DEV)
    ops.gemm_big(A.to(DEV), B.to(DEV), C, b_kcontig=b_kcontig, flags=flags, alpha=-1.0, beta=1.0)
    opB = B.t() if b_kcontig else B
    ref = _f32_ref(A, opB, flags, -1.0, 1.0, C0)
    if flags == 16:
        lo = torch.tril(torch.ones(n, n, dtype=torch.bool))
        assert rel(C.cpu()[lo], ref[lo]) < 2e-6
        assert torch.equal(C.cpu()[~lo], C0[~lo])          # upper part untouched
    else:
        assert rel(C, ref) < 2e-6


@pytest.mark.parametrize("m,n,k", [(700, 300, 200), (3584, 128, 512), (3456, 384, 512), (256, 256, 64)])
def test_gemm_big_out_lower_tall(ops, m, n, k):
    """OUT_LOWER on a tall output (m >= n: the blocked potrf's next-panel updates C -= L_p L_q^T): the
    lower triangle of the top n x n block and every row below it are updated, the strict upper part of
    the top block is untouched; stream-K / split-K tile counts cover the triangle plus the full rows."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    g = torch.Generator().manual_seed(m + n + k)
    A = torch.randn(m, k, generator=g)
    C0 = torch.randn(m, n, generator=g)
    Ad, C = A.to(DEV), C0.to(DEV)
    ops.gemm_big(Ad, Ad[:n].contiguous(), C, flags=L.OUT_LOWER, alpha=-1.0, beta=1.0)
    got = C.cpu().double()
    ref = C0.double() - A.double() @ A[:n].double().t()
    lo = torch.ones(m, n, dtype=torch.bool).tril()
    assert rel(got[lo], ref[lo]) < 2e-6
    assert torch.equal(got[~lo], C0.double()[~lo])


def test_gemm_big_split_k_deterministic_and_batched(ops):
    # few tiles, long k: split-K runs (workspace) and must be bit-reproducible and equal to no-split within f32 rounding
    g = torch.Generator().manual_seed(5)
    A = torch.randn(3, 256, 4096, generator=g).to(DEV)
    B = torch.randn(3, 256, 4096, generator=g).to(DEV)
    outs = []
    for _ in range(3):
        C = torch.zeros(3, 256, 256, device=DEV)
        ops.gemm_big(A, B, C)
        outs.append(C.clone())
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    C1 = torch.zeros(3, 256, 256, device=DEV)
    ops.gemm_big(A, B, C1, split=False)
    ref = torch.bmm(A.double().cpu(), B.double().cpu().transpose(1, 2))
    assert rel(outs[0], ref) < 2e-6 and rel(C1, ref) < 2e-6


@pytest.mark.parametrize("kind,n,k", [("syrk", 2048, 1024), ("gemm", 640, 8192), ("syrk", 1000, 4000)])
def test_gemm_big_stream_k(ops, kind, n, k):
    # batch-1 problems whose tile grid would leave most of the chip idle run stream-K (equal k-tile
    # ranges per workgroup, cut tiles combined in k order): bit-reproducible, fp64-accurate, and
    # the SYRK leaves the strict upper triangle untouched
    g = torch.Generator().manual_seed(n + k)
    A = (torch.rand(n, k, generator=g) * 2 - 1).to(DEV)
    B = A if kind == "syrk" else (torch.rand(n, k, generator=g) * 2 - 1).to(DEV)
    C0 = torch.randn(n, n, generator=g).to(DEV)
    flags = 16 if kind == "syrk" else 0
    outs = []
    for _ in range(3):
        C = C0.clone()
        ops.gemm_big(A, B, C, flags=flags, alpha=-1.0, beta=1.0)
        outs.append(C)
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    ref = C0.double() - A.double() @ B.double().t()
    C1 = C0.clone()
    ops.gemm_big(A, B, C1, flags=flags, alpha=-1.0, beta=1.0, split=False)
    if kind == "syrk":
        lo = torch.tril(torch.ones(n, n, dtype=torch.bool, device=DEV))
        assert rel(outs[0][lo], ref[lo]) < 2e-6 and rel(C1[lo], ref[lo]) < 2e-6
        assert torch.equal(outs[0][~lo], C0[~lo])
    else:
        assert rel(outs[0], ref) < 2e-6 and rel(C1, ref) < 2e-6


@pytest.mark.parametrize("n", [130, 300, 640, 1000, 2048, 4096, 4160])
@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_potrf_blocked(ops, n, dt):
    # large single-matrix blocked Cholesky with lookahead (stress path): fp64-accurate residual,
    # strictly upper part zero, graph replay bit-identical to the eager call
    A = _spd(n, 1, n + 1)[0]
    Ad = A.to(dt).to(DEV).contiguous()
    W = Ad.clone()
    info = ops.potrf_blocked_(W)
    torch.cuda.synchronize()
    assert int(info.item()) == 0
    Ld = W.double().cpu()
    assert torch.equal(torch.triu(Ld, 1), torch.zeros_like(Ld))
    tol = 1e-12 if dt == torch.float64 else 2e-6
    assert float((Ld @ Ld.t() - A).norm() / A.norm()) < tol
    assert rel(Ld, torch.linalg.cholesky(A)) < (1e-10 if dt == torch.float64 else 1e-4)
    G = Ad.clone()
    inf2 = torch.zeros(1, dtype=torch.int32, device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.potrf_blocked_(G, info=inf2)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        G.copy_(Ad)
        ops.potrf_blocked_(G, info=inf2)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(G, W)


@pytest.mark.parametrize("dt", [torch.float64, torch.float32])
def test_potrf_blocked_not_pd(ops, dt):
    # first failing pivot reported as a global 1-based column, inside a later block (f32: a fused block step)
    A = _spd(400, 1, 3)[0]
    A[333, 333] = -50.0
    W = A.to(dt).to(DEV).contiguous()
    info = ops.potrf_blocked_(W)
    ref = torch.linalg.cholesky_ex(A).info
    assert int(info.item()) == int(ref.item()) == 334


def test_gemm_big_offsets_batch(ops):
    # per-problem element offsets (non-uniform), OUT_TRIL zeroing, diag_add, OUT_LOWER + B_UPPER SYRK form
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    g = torch.Generator().manual_seed(21)
    M, nb = 300, 5
    pool = torch.randn(9 * M * M, generator=g)
    offs = [0, 3 * M * M + 17, M * M + 5, 7 * M * M, 5 * M * M + 1]
    P = pool.to(DEV)
    C = torch.full((nb, M, M), 7.0, device=DEV)
    cs = [b * M * M for b in range(nb)]
    syrk = ops.BigBatch(P, P, C, offs, offs, cs, M, M, M, lda=M, ldb=M, b_kcontig=True,
                        flags=L.A_LOWER | L.B_UPPER | L.OUT_LOWER, diag_add=0.25)
    syrk()
    lo = torch.tril(torch.ones(M, M, dtype=torch.bool))
    for b, o in enumerate(offs):
        S = torch.tril(pool[o:o + M * M].reshape(M, M).double())
        ref = S @ S.t() + 0.25 * torch.eye(M, dtype=F64)
        got = C[b].cpu()
        assert rel(got[lo], ref[lo]) < 2e-6 and torch.all(got[~lo] == 7.0)
    X = torch.full((nb, M, M), 3.0, device=DEV)
    xs = ops.BigBatch(C, P, X, cs, offs, cs, M, M, M, lda=M, ldb=M, b_kcontig=False,
                      flags=L.A_LOWER | L.B_LOWER | L.OUT_TRIL)
    xs()
    for b, o in enumerate(offs):
        A = torch.tril(C[b].cpu().double())
        Bm = torch.tril(pool[o:o + M * M].reshape(M, M).double())
        ref = A @ Bm
        got = X[b].cpu()
        assert rel(got, ref) < 2e-6 and torch.all(got[~lo] == 0)
    # KL L-bar form: G_b = -tril(C_b)^T tril(X_b) + G_b + diag-scaled E_b (lower), upper zeroed
    Gd = torch.randn(nb, M, M, generator=g).to(DEV)
    G0 = Gd.clone()
    RS = torch.randn(3 * M, generator=g).to(DEV)
    offr = [(b % 3) * M for b in range(nb)]
    kl = ops.BigBatch(C, X, Gd, cs, cs, cs, M, M, M, lda=M, ldb=M, a_kcontig=False, b_kcontig=False,
                      flags=L.A_UPPER | L.B_LOWER | L.OUT_TRIL | L.EPI_E_LOWER, alpha=-1.0, beta=1.0,
                      epi=(P, offs, (M, 1), RS, offr, 1.0))
    kl()
    for b, o in enumerate(offs):
        A = torch.tril(C[b].cpu().double())
        Xb = torch.tril(X[b].cpu().double())
        E = torch.tril(pool[o:o + M * M].reshape(M, M).double())
        rs = RS.cpu().double()[offr[b]:offr[b] + M]
        ref = torch.tril(-A.t() @ Xb + G0[b].cpu().double() + rs[:, None] * E)
        got = Gd[b].cpu()
        assert rel(got, ref) < 2e-6 and torch.all(got[~lo] == 0)


def test_gemm_big_row_epilogue_edges(ops):
    # the row-vector epilogue (row-contiguous, 16-byte aligned C and E): n = 130 leaves a partial 4-column chunk at
    # the right edge, OUT_LOWER chunks straddle the diagonal, beta = 1 and the E term read 16-byte chunks; the
    # row pitch 132 keeps the rows aligned.  Compared with fp64 torch element by element, masked parts untouched.
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    g = torch.Generator().manual_seed(41)
    M, LD, nb = 130, 132, 3
    pool = torch.randn(nb * M * M, generator=g)
    P = pool.to(DEV)
    offs = [b * M * M for b in range(nb)]
    C0 = torch.randn(nb, M, LD, generator=g)
    C = C0.clone().to(DEV)
    cs = [b * M * LD for b in range(nb)]
    syrk = ops.BigBatch(P, P, C, offs, offs, cs, M, M, M, lda=M, ldb=M, b_kcontig=True, sC=(LD, 1),
                        flags=L.A_LOWER | L.B_UPPER | L.OUT_LOWER, beta=1.0, diag_add=0.5)
    syrk()
    lo = torch.tril(torch.ones(M, M, dtype=torch.bool))
    for b, o in enumerate(offs):
        S = torch.tril(pool[o:o + M * M].reshape(M, M).double())
        ref = S @ S.t() + C0[b, :, :M].double() + 0.5 * torch.eye(M, dtype=F64)
        got = C[b].cpu()
        assert rel(got[:, :M][lo], ref[lo]) < 2e-6
        assert torch.equal(got[:, :M][~lo], C0[b, :, :M][~lo]) and torch.equal(got[:, M:], C0[b, :, M:])
    E = torch.randn(nb, M, LD, generator=g)
    Ed = E.to(DEV)
    RS = torch.randn(nb * M, generator=g).to(DEV)
    G0 = torch.randn(nb, M, LD, generator=g)
    G = G0.clone().to(DEV)
    kl = ops.BigBatch(P, P, G, offs, offs, cs, M, M, M, lda=M, ldb=M, a_kcontig=False, b_kcontig=False, sC=(LD, 1),
                      flags=L.A_UPPER | L.B_LOWER | L.OUT_TRIL | L.EPI_E_LOWER, alpha=-1.0, beta=1.0,
                      epi=(Ed, cs, (LD, 1), RS, [b * M for b in range(nb)], 2.0))
    kl()
    for b, o in enumerate(offs):
        A = torch.tril(pool[o:o + M * M].reshape(M, M).double())
        rs = RS.cpu().double()[b * M:(b + 1) * M]
        ref = torch.tril(-A.t() @ A + G0[b, :, :M].double() + 2.0 * rs[:, None] * torch.tril(E[b, :, :M].double()))
        got = G[b].cpu()
        assert rel(got[:, :M], ref) < 2e-6 and torch.all(got[:, :M][~lo] == 0)
        assert torch.equal(got[:, M:], G0[b, :, M:])


def test_gemm_big_kseg_batch(ops):
    # per-problem k ranges from a device segment table (L-bar products P^T W over each factor's rows),
    # transposed operands, OUT_TRIL + beta accumulate; an empty segment leaves C (lower) unchanged
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    g = torch.Generator().manual_seed(31)
    Bn, M, D = 700, 200, 4
    P = torch.randn(Bn, M, generator=g).to(DEV)
    W = torch.randn(3, Bn, M, generator=g).to(DEV)
    seg = torch.tensor([0, 250, 250, 600, 700], dtype=torch.int32, device=DEV)   # segment 1 empty
    probs = [(0, 1, 0), (1, 1, 1), (2, 2, 2), (3, 1, 0), (0, 4, 2)]            # (seg index, span, W slice)
    C0 = torch.randn(len(probs), M, M, generator=g).to(DEV)
    C = C0.clone()
    op = ops.BigBatch(P, W, C, [0] * len(probs), [w * Bn * M for (_, _, w) in probs],
                      [b * M * M for b in range(len(probs))], M, M, Bn, lda=M, ldb=M, a_kcontig=False,
                      b_kcontig=False, flags=L.OUT_TRIL, beta=1.0,
                      kseg=(seg, [s_ for (s_, _, _) in probs], [sp for (_, sp, _) in probs]))
    op()
    sc = seg.cpu().tolist()
    lo = torch.tril(torch.ones(M, M, dtype=torch.bool))
    for b, (s_, sp, w) in enumerate(probs):
        k0, k1 = sc[s_], sc[s_ + sp]
        ref = torch.tril(C0[b].cpu().double() + P[k0:k1].cpu().double().t() @ W[w, k0:k1].cpu().double())
        got = C[b].cpu()
        assert rel(got, ref) < 2e-6 and torch.all(got[~lo] == 0)


@pytest.mark.parametrize("bk", [False, True])
def test_gemm_big_rseg_batch(ops, bk):
    """Per-problem ROW ranges from a device segment table on the 128x128 kernel (the HCP-shaped quadratic-form
    factors W_d = P[rows of outputs >= d] L_d and the P-bar products W-hat_d L_d^T): B_LOWER (bk False: B = L
    k-strided) or B_UPPER over B(k, j) = L[j, k] (bk True), beta accumulate, an empty range and a range shorter
    than one tile; rows outside every problem's range stay untouched."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    g = torch.Generator().manual_seed(41)
    Bn, M = 1000, 512
    P = torch.randn(Bn, M, generator=g)
    Lm = torch.tril(torch.randn(4, M, M, generator=g)) + torch.triu(torch.full((M, M), float("inf")), 1)
    seg = torch.tensor([0, 300, 300, 350, 1000], dtype=torch.int32, device=DEV)   # segment 1 empty, 2 of 50 rows
    probs = [(0, 4), (1, 1), (2, 2), (3, 1), (0, 1)]                             # (first segment, span)
    C0 = torch.randn(len(probs), Bn, M, generator=g)
    C = C0.clone().to(DEV)
    flags = L.B_UPPER if bk else L.B_LOWER
    op = ops.BigBatch(P.to(DEV), Lm.to(DEV), C, [0] * len(probs), [(b % 4) * M * M for b in range(len(probs))],
                      [b * Bn * M for b in range(len(probs))], Bn, M, M, lda=M, ldb=M, b_kcontig=bk, flags=flags,
                      beta=1.0, rseg=(seg, [s_ for (s_, _) in probs], [sp for (_, sp) in probs]))
    op()
    sc = seg.cpu().tolist()
    Lc = torch.tril(torch.nan_to_num(Lm, posinf=0.0)).double()
    for b, (s_, sp) in enumerate(probs):
        r0, r1 = sc[s_], sc[s_ + sp]
        ref = C0[b].double().clone()
        Lb = Lc[b % 4]
        ref[r0:r1] += P[r0:r1].double() @ (Lb.t() if bk else Lb)
        got = C[b].cpu()
        assert rel(got, ref) < 2e-6
        assert torch.equal(got[:r0], C0[b][:r0]) and torch.equal(got[r1:], C0[b][r1:])
    assert op.macs(seg.cpu()) == sum((sc[s_ + sp] - sc[s_]) * M * (M + 1) // 2 for (s_, sp) in probs)


def test_gemm_big_persistent_multi_item_walk(ops):
    # a batched single-pass launch is a grid of 2 x CUs workgroups that walk the (tile, problem) items;
    # only with items > 2 x CUs does a workgroup run several.  M = 512 (16 tiles per problem) x 72 problems = 1152
    # items: per-problem kseg k ranges incl. empty ones (OUT_TRIL items with no k-tiles), beta accumulate, and a
    # rows-epilogue SYRK (OUT_LOWER + diag) handing LDS to the next item.  Bit-identical to the same problems
    # launched 8 at a time (128 items: one item per workgroup) and within f32 rounding of fp64 torch.
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    g = torch.Generator().manual_seed(51)
    Bn, M, nprob = 300, 512, 72
    P = torch.randn(Bn, M, generator=g).to(DEV)
    W = torch.randn(3, Bn, M, generator=g).to(DEV)
    seg = torch.tensor([0, 120, 120, 260, 300], dtype=torch.int32, device=DEV)   # segment 1 empty
    probs = [(b % 4, 1 + (b // 4) % 2 if b % 4 < 3 else 1, b % 3) for b in range(nprob)]
    probs[5] = (1, 1, 2)                                                          # empty k range
    C0 = torch.randn(nprob, M, M, generator=g).to(DEV)

    def run(chunk):
        C = C0.clone()
        for c0 in range(0, nprob, chunk):
            pr = probs[c0:c0 + chunk]
            op = ops.BigBatch(P, W, C, [0] * len(pr), [w * Bn * M for (_, _, w) in pr],
                              [(c0 + b) * M * M for b in range(len(pr))], M, M, Bn, lda=M, ldb=M, a_kcontig=False,
                              b_kcontig=False, flags=L.OUT_TRIL, beta=1.0,
                              kseg=(seg, [s_ for (s_, _, _) in pr], [sp for (_, sp, _) in pr]))
            op()
        return C
    got, ref8 = run(nprob), run(8)
    assert torch.equal(got, ref8)
    sc = seg.cpu().tolist()
    lo = torch.tril(torch.ones(M, M, dtype=torch.bool))
    for b in (0, 5, 6, 37, nprob - 1):
        s_, sp, w = probs[b]
        k0, k1 = sc[s_], sc[s_ + sp]
        ref = torch.tril(C0[b].cpu().double() + P[k0:k1].cpu().double().t() @ W[w, k0:k1].cpu().double())
        assert rel(got[b].cpu(), ref) < 2e-6 and torch.all(got[b].cpu()[~lo] == 0)
    assert torch.equal(got[5].cpu()[lo], C0[5].cpu()[lo])                           # k = 0: C kept
    # rows-epilogue SYRK items (OUT_LOWER + diag_add), 72 problems of M = 512 at per-problem offsets
    pool = torch.randn(4 * M * M, generator=g).to(DEV)
    offs = [(b % 4) * M * M for b in range(nprob)]

    def syrk(chunk):
        C = torch.full((nprob, M, M), 5.0, device=DEV)
        for c0 in range(0, nprob, chunk):
            o = offs[c0:c0 + chunk]
            ops.BigBatch(pool, pool, C, o, o, [(c0 + b) * M * M for b in range(len(o))], M, M, M, lda=M, ldb=M,
                         b_kcontig=True, flags=L.A_LOWER | L.B_UPPER | L.OUT_LOWER, diag_add=0.5)()
        return C
    s_all, s8 = syrk(nprob), syrk(8)
    assert torch.equal(s_all, s8)
    for b in (0, 41, nprob - 1):
        S = torch.tril(pool[offs[b]:offs[b] + M * M].reshape(M, M).double().cpu())
        ref = S @ S.t() + 0.5 * torch.eye(M, dtype=F64)
        assert rel(s_all[b].cpu()[lo], ref[lo]) < 2e-6 and torch.all(s_all[b].cpu()[~lo] == 5.0)


def _rbf(a, b, s2, ls):
    return s2 * torch.exp(-0.5 * (a[:, None] / ls - b[None, :] / ls) ** 2)


def _gibbs(a, b, la, lb):
    S = la[:, None] ** 2 + lb[None, :] ** 2
    return torch.sqrt(2 * la[:, None] * lb[None, :] / S) * torch.exp(-(a[:, None] - b[None, :]) ** 2 / S)


@pytest.mark.parametrize("n,B", [(256, 2000), (256, 1), (200, 130), (144, 64), (128, 63)])
def test_chol_tp_fused_priors_vs_torch(ops, n, B):
    """Round 6: nmgp_chol_tp_f64 -- [Sigma | three RBF priors] factored + inverted, the priors' K12 / T = K12 L^-T /
    P = T L^-1 formed by the launch's row workgroups; then a Gibbs prior whose row workgroups first draw the t-row
    ell_X.  Against fp64 torch on the same inputs: L, K12, ell_X tight; T / P at least as accurate as the unfused
    schedule's explicit-inverse products of the launch's own L^-1."""
    g = torch.Generator().manual_seed(n + B)
    jit = 1e-4
    Z = torch.linspace(0, 1, n, dtype=F64)
    x = torch.rand(B, generator=g, dtype=F64)
    hyp = torch.tensor([0.3, -1.2, -0.2, -0.9, 0.1, -1.5], dtype=F64)
    S = torch.tril(0.1 * torch.randn(n, n, generator=g, dtype=F64))
    A = torch.zeros(4, n, n, dtype=F64)
    A[0] = S @ S.t() + jit * torch.eye(n, dtype=F64)
    for k in range(3):
        A[k + 1] = _rbf(Z, Z, float(torch.exp(hyp[2 * k])), float(torch.exp(hyp[2 * k + 1]))) + jit * torch.eye(n, dtype=F64)
    Ad, Xd = A.to(DEV), torch.zeros(4, n, n, dtype=F64, device=DEV)
    info = torch.full((4,), 7, dtype=torch.int32, device=DEV)
    K12, T, P = (torch.zeros(3, B, n, dtype=F64, device=DEV) for _ in range(3))
    hd, Zd, xd = hyp.to(DEV), Z.to(DEV), x.to(DEV)
    mats = [dict()] + [dict(rows=1, hyp=hd[2 * k:], K12=K12[k], T=T[k], P=P[k]) for k in range(3)]
    ops.CholTp(Ad[0], Xd[0], info, n, mats, jitter=jit, Z=Zd, x=xd, B=B)()
    torch.cuda.synchronize()
    assert info.cpu().tolist() == [0, 0, 0, 0]
    up = torch.triu(torch.ones(n, n, dtype=torch.bool), 1)
    Lr = torch.linalg.cholesky(A[0])
    assert rel(Ad[0], Lr) < 1e-12 and rel(Xd[0], torch.linalg.inv(Lr)) < 1e-9
    for k in range(3):
        s2, ls = float(torch.exp(hyp[2 * k])), float(torch.exp(hyp[2 * k + 1]))
        K22 = _rbf(Z, Z, s2, ls) + jit * torch.eye(n, dtype=F64)
        Kx = _rbf(x, Z, s2, ls)
        Lk = torch.linalg.cholesky(K22)
        L_, X_ = Ad[k + 1].cpu(), Xd[k + 1].cpu()
        assert rel(L_, Lk) < 1e-11 and torch.all(L_[up] == 0) and torch.all(X_[up] == 0)
        assert rel(K12[k], Kx) < 1e-14
        _check_tp(T[k], P[k], Kx, Lk, X_, f"rbf{k}")
    # the Gibbs prior: t-row (ell_X) and K_G12 rows in the launch
    v = -1.5 + 0.3 * torch.randn(n, generator=g, dtype=F64)
    ellZ = torch.exp(v)
    Ptd = (0.02 * torch.randn(B, n, generator=g, dtype=F64)).to(DEV)
    Ttd = (0.02 * torch.randn(B, n, generator=g, dtype=F64)).to(DEV)
    zt = torch.randn(B, generator=g, dtype=F64)
    ht = torch.tensor([0.2], dtype=F64)
    K22 = _gibbs(Z, Z, ellZ, ellZ) + jit * torch.eye(n, dtype=F64)
    AG, XG = K22.to(DEV), torch.zeros(n, n, dtype=F64, device=DEV)
    infoG = torch.full((1,), 7, dtype=torch.int32, device=DEV)
    KG, TG, PG = (torch.zeros(B, n, dtype=F64, device=DEV) for _ in range(3))
    ellX, var_t = torch.zeros(B, dtype=F64, device=DEV), torch.zeros(B, dtype=F64, device=DEV)
    ops.CholTp(AG, XG, infoG, n, [dict(rows=2, K12=KG, T=TG, P=PG)], jitter=jit, Z=Zd, ellZ=ellZ.to(DEV),
               x=xd, B=B, trow=dict(Pt=Ptd, Tt=Ttd, v=v.to(DEV), zt=zt.to(DEV), hyp_t=ht.to(DEV), ellX=ellX,
                                    var_t=var_t))()
    torch.cuda.synchronize()
    assert int(infoG.item()) == 0
    var = float(torch.exp(ht)) - (Ttd.cpu() ** 2).sum(1)
    lx = torch.exp(Ptd.cpu() @ v + zt * torch.sqrt(var + jit))
    assert rel(var_t, var) < 1e-14 and rel(ellX, lx) < 1e-13
    Kx = _gibbs(x, Z, lx, ellZ)
    LG = torch.linalg.cholesky(K22)
    assert rel(AG, LG) < 1e-11 and rel(KG, Kx) < 1e-13
    _check_tp(TG, PG, Kx, LG, XG.cpu(), "gibbs")
    assert L_dev_status_clean()


def _check_tp(T, P, Kx, Lk, X_, tag):
    # T = Kx L^-T by substitution and P = T L^-1 against fp64 torch's triangular solves with torch's factor; the
    # unfused schedule's explicit-inverse products (Kx X^T, Kx X^T X with this launch's X = L^-1) beside them: the
    # fused launch must be at least about as accurate (both carry cond(K22) eps, ~1e6 eps here)
    Tr = torch.linalg.solve_triangular(Lk, Kx.t(), upper=False).t()
    Pr = torch.cholesky_solve(Kx.t(), Lk).t()
    eT, eP = rel(T, Tr), rel(P, Pr)
    xT, xP = rel(Kx @ X_.t(), Tr), rel(Kx @ X_.t() @ X_, Pr)
    print(f"CHOL_TP {tag}: T err {eT:.2e} (explicit inverse {xT:.2e})  P err {eP:.2e} (explicit {xP:.2e})")
    assert eT < max(3 * xT, 1e-13) and eP < max(3 * xP, 1e-12), (tag, eT, xT, eP, xP)
    assert eT < 1e-9 and eP < 1e-6


def L_dev_status_clean():
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    return L.device_status(clear=True) == 0


def test_chol_tp_not_pd_and_repeat(ops):
    """A non-PD matrix reports its column in info like chol_inv_ and leaves the other matrix of the launch exact; the
    progress words are re-armed, so the next launches on the same buffers (different B) agree bit for bit."""
    n, jit = 256, 1e-4
    Z = torch.linspace(0, 1, n, dtype=F64, device=DEV)
    hyp = torch.tensor([0.0, -1.0], dtype=F64, device=DEV)
    K22 = _rbf(Z.cpu(), Z.cpu(), 1.0, float(np.exp(-1.0))).to(DEV) + jit * torch.eye(n, dtype=F64, device=DEV)
    A = torch.zeros(2, n, n, dtype=F64, device=DEV)
    X = torch.zeros_like(A)
    info = torch.zeros(2, dtype=torch.int32, device=DEV)
    outs = []
    for B in (500, 77, 500):
        x = torch.linspace(0.01, 0.99, B, dtype=F64, device=DEV)
        K12, T, P = (torch.zeros(B, n, dtype=F64, device=DEV) for _ in range(3))
        A[0] = torch.eye(n, dtype=F64, device=DEV)
        A[0, 100, 100] = -1.0
        A[1] = K22
        ops.CholTp(A[0], X[0], info, n, [dict(), dict(rows=1, hyp=hyp, K12=K12, T=T, P=P)], jitter=jit,
                   Z=Z, x=x, B=B)()
        torch.cuda.synchronize()
        assert info.cpu().tolist() == [101, 0]
        outs.append((A[1].clone(), X[1].clone(), T.clone(), P.clone()))
    for a, b in zip(outs[0], outs[2]):
        assert torch.equal(a, b)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])   # the prior: B-independent
    assert L_dev_status_clean()


def test_chol_inv_blocked_not_pd_reports_global_column(ops):
    A = _spd(400, 2, 9)
    bad = A.clone()
    bad[1, 300, 300] = -50.0                       # third diagonal block: global column 301
    _, info = ops.chol_inv_(bad.to(DEV))
    info = info.cpu()
    assert int(info[0]) == 0 and int(info[1]) == 301


def test_chol_inv_f32_and_not_pd(ops):
    A = _spd(200, 3, 3)
    Ad = A.float().to(DEV)
    X, info = ops.chol_inv_(Ad)
    ref = torch.linalg.cholesky(A)
    assert rel(Ad, ref) < 1e-5 and rel(X, torch.linalg.inv(ref)) < 1e-4
    bad = A.clone()
    bad[2, 130, 130] = -5.0
    _, info = ops.chol_inv_(bad.to(DEV))
    info = info.cpu()
    assert int(info[0]) == 0 and int(info[1]) == 0 and int(info[2]) > 0


def test_potrf_f32_and_not_pd(ops):
    A = _spd(96, 2, 1)
    Ld = A.float().to(DEV)
    ops.potrf_(Ld)
    assert rel(Ld, torch.linalg.cholesky(A)) < 1e-5
    bad = A.clone()
    bad[1, 40, 40] = -5.0
    Bd = bad.to(DEV)
    info = ops.potrf_(Bd).cpu()
    assert int(info[0]) == 0 and int(info[1]) > 0


def test_pairwise_rbf_gibbs(ops):
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    g = np.random.default_rng(0)
    X = torch.from_numpy(g.uniform(0, 1, (300, 1)))
    Z = torch.from_numpy(np.linspace(0, 1, 70)[:, None])
    K = ops.pairwise(X.to(DEV), Z.to(DEV), mode=L.RBF, scale2=1.7, length_scale=0.13)
    assert rel(K, O.create_RBF(X, Z, 1.7, 0.13)) < 1e-14
    K22 = ops.pairwise(Z.to(DEV), Z.to(DEV), mode=L.RBF, scale2=1.7, length_scale=0.13, diag_add=1e-4)
    assert rel(K22, O.create_RBF(Z, None, 1.7, 0.13) + 1e-4 * torch.eye(70, dtype=F64)) < 1e-14
    eX = torch.from_numpy(np.exp(g.normal(-2, .3, 300)))
    eZ = torch.from_numpy(np.exp(g.normal(-2, .3, 70)))
    G = ops.pairwise(X.to(DEV), Z.to(DEV), mode=L.GIBBS, scale2=0.7, ellX=eX.to(DEV), ellZ=eZ.to(DEV))
    assert rel(G, O.create_Gibbs(X, Z, eX, eZ, 0.7)) < 1e-14


def test_pairwise_legacy_expand(ops):
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    g = np.random.default_rng(1)
    X1 = torch.from_numpy(g.standard_normal((31, 3)))
    X2 = torch.from_numpy(g.standard_normal((17, 3)))
    K = ops.pairwise(X1.to(DEV), X2.to(DEV), mode=L.RBF, dist=L.DIST_EXPAND, scale2=1.7 ** 2, length_scale=0.8)
    assert rel(K, O.RBF_cov(X1, X2, 1.7, 0.8)) < 1e-13
    s1, e1 = torch.from_numpy(np.exp(g.normal(0, .3, 31))), torch.from_numpy(np.exp(g.normal(0, .3, 31)))
    K11 = ops.pairwise(X1.to(DEV), X1.to(DEV), mode=L.GIBBS, dist=L.DIST_EXPAND, ellX=e1.to(DEV), ellZ=e1.to(DEV),
                       sigX=s1.to(DEV), sigZ=s1.to(DEV), diag_add=1e-6)
    assert rel(K11, O.Nonstationary_RBF_cov(X1, s1, e1)) < 1e-13


def test_pairwise_bwd(ops):
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    g = np.random.default_rng(2)
    n, m = 300, 70
    X = torch.from_numpy(g.uniform(0, 1, (n, 1)))
    Z = torch.from_numpy(np.linspace(0, 1, m)[:, None])
    Rb = torch.from_numpy(g.standard_normal((n, m)))
    Pm = torch.from_numpy(g.standard_normal((n, m)))
    rc = torch.from_numpy(g.standard_normal(n))
    Kbar = Rb - rc[:, None] * Pm
    # RBF: sums of Kbar*K and Kbar*K*r2 == d/dlog(s2), d/dlog(ls)
    ls2 = torch.tensor(np.log(1.3), requires_grad=True)
    lls = torch.tensor(np.log(0.2), requires_grad=True)
    Kc = O.create_RBF(X, Z, torch.exp(ls2), torch.exp(lls))
    (Kc * Kbar).sum().backward()
    # descriptors hold raw pointers: every device tensor they name must stay referenced
    Xd, Zd, Rbd, Pmd, rcd = X.to(DEV), Z.to(DEV), Rb.to(DEV), Pm.to(DEV), rc.to(DEV)
    Kd = ops.pairwise(Xd, Zd, mode=L.RBF, scale2=1.3, length_scale=0.2)
    tiles, nct, nrt = ops.bwd_tiles(n, m)
    sp = torch.zeros(tiles * 2, dtype=F64, device=DEV)
    d = ops.pairwise_bwd_desc(Xd, Zd, Kd, Rbd, mode=L.RBF, ld=m, Pm=Pmd,
                              rowcoef=(rcd, 0), scale2=1.3, length_scale=0.2, scal_part=sp)
    ops.PairwiseBwdGroup([d], DEV)(F64)
    s = sp.view(tiles, 2).sum(0).cpu()
    assert float(s[0]) == pytest.approx(float(ls2.grad), rel=1e-12)
    assert float(s[1]) == pytest.approx(float(lls.grad), rel=1e-12)
    # Gibbs: row / column partials == d/d ellX, d/d ellZ
    eX = torch.from_numpy(np.exp(g.normal(-2, .3, n))).requires_grad_()
    eZ = torch.from_numpy(np.exp(g.normal(-2, .3, m))).requires_grad_()
    Gc = O.create_Gibbs(X, Z, eX, eZ)
    (Gc * Kbar).sum().backward()
    eXd, eZd = eX.detach().to(DEV), eZ.detach().to(DEV)
    Gd = ops.pairwise(Xd, Zd, mode=L.GIBBS, ellX=eXd, ellZ=eZd)
    rp = torch.zeros(nct, n, dtype=F64, device=DEV)
    cp = torch.zeros(nrt, m, dtype=F64, device=DEV)
    d = ops.pairwise_bwd_desc(Xd, Zd, Gd, Rbd, mode=L.GIBBS, ld=m, Pm=Pmd,
                              rowcoef=(rcd, 0), ellX=eXd, ellZ=eZd, row_part=rp, col_part=cp)
    ops.PairwiseBwdGroup([d], DEV)(F64)
    gx = torch.zeros(n, dtype=F64, device=DEV)
    gz = torch.zeros(m, dtype=F64, device=DEV)
    ops.colsum(rp, gx)
    ops.colsum(cp, gz)
    assert rel(gx, eX.grad) < 1e-12
    assert rel(gz, eZ.grad) < 1e-12


def test_kron(ops):
    g = np.random.default_rng(4)
    A = torch.from_numpy(g.standard_normal((3, 4)))
    Bm = torch.from_numpy(g.standard_normal((5, 2)))
    out = ops.kron_product(A.to(DEV), Bm.to(DEV)).cpu()
    assert torch.equal(out, O.kronecker_product(A, Bm))       # bit-exact
    Bk = torch.from_numpy(g.standard_normal((4, 6)))
    Kk = torch.from_numpy(g.standard_normal((9, 5)))
    y = torch.from_numpy(g.standard_normal(30))
    mv = ops.kron_mv(Bk.to(DEV), Kk.to(DEV), y.to(DEV))
    assert rel(mv, O.kron_mv(Bk, Kk, y)) < 1e-14
    assert rel(mv, torch.kron(Bk, Kk) @ y) < 1e-13


@pytest.mark.parametrize("P1,P2,N1,N2", [(5, 5, 4096, 4096), (3, 8, 37, 61), (70, 2, 131, 64), (6, 9, 50, 40),
                                         (1, 1, 1, 1), (8, 3, 1000, 1001), (7, 5, 2049, 3000), (2, 4, 9, 514),
                                         (4, 0, 10, 10), (3, 2, 10, 0), (12, 0, 5, 6)])
@pytest.mark.parametrize("dt", [F64, torch.float32])
def test_kron_mv_fused_and_gemm_paths(ops, P1, P2, N1, N2, dt):
    """kron_mv (kronecker_operation.py:72-85): P2 <= 8 takes the fused one-pass kernel (16-byte rows when N2
    allows, scalar otherwise; row tails; P1 > 64 lanes strided), P2 > 8 the two-GEMM path; both in the
    reference's reshape order against the oracle restatement and the dense (B kron K) y."""
    g = torch.Generator().manual_seed(P1 * 1000 + P2 * 100 + N1 + N2)
    Bk = torch.randn(P1, P2, generator=g, dtype=F64)
    Kk = torch.randn(N1, N2, generator=g, dtype=F64)
    y = torch.randn(P2 * N2, generator=g, dtype=F64)
    mv = ops.kron_mv(Bk.to(dt).to(DEV), Kk.to(dt).to(DEV), y.to(dt).to(DEV)).double().cpu()
    Bc, Kc, yc = Bk.to(dt).double(), Kk.to(dt).double(), y.to(dt).double()
    tol = 1e-13 if dt == F64 else 2e-5          # (fp32: sums of up to 8 x 4096 products)
    if P2 == 0 or N2 == 0:                      # an empty contraction: exactly zero (no work buffer needed)
        assert mv.shape == (P1 * N1,) and torch.equal(mv, torch.zeros(P1 * N1, dtype=F64))
        return
    assert rel(mv, O.kron_mv(Bc, Kc, yc)) < tol
    if N1 * N2 <= 10 ** 6:
        assert rel(mv, torch.kron(Bc, Kc) @ yc) < tol


@pytest.mark.parametrize("sizes", [[400, 350, 500, 300, 450], [0, 7, 0, 129, 1], [3] * 40])
@pytest.mark.parametrize("dt", [F64, torch.float32])
def test_pbar_reduce_adds_each_rows_factor_products_in_order(ops, sizes, dt):
    """nmgp_pbar_reduce (the per-factor P-bar_G form of the backward): every row r of output i gets
    P[r] + Z_0[r] + ... + Z_i[r], summed left to right -- empty outputs and ragged segments included."""
    import ctypes
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    D, M = len(sizes), 300
    B = sum(sizes)
    seg = torch.tensor(np.concatenate([[0], np.cumsum(sizes)]), dtype=torch.int32)
    g = torch.Generator().manual_seed(D * 31 + B)
    Z = torch.randn(D, B, M, generator=g, dtype=dt)
    P = torch.randn(B, M, generator=g, dtype=dt)
    ref = P.clone()
    for i in range(D):
        for d in range(i + 1):
            ref[seg[i]:seg[i + 1]] += Z[d, seg[i]:seg[i + 1]]
    Zd, Pd, sd = Z.to(DEV), P.to(DEV), seg.to(DEV)
    fn = L.lib().nmgp_pbar_reduce_f64 if dt == F64 else L.lib().nmgp_pbar_reduce_f32
    vp = ctypes.c_void_p
    L.check(fn(vp(Zd.data_ptr()), B * M, vp(Pd.data_ptr()), M, vp(sd.data_ptr()), D, B, M, L.stream_handle()),
            "pbar_reduce")
    assert torch.equal(Pd.cpu(), ref)
    assert fn(vp(Zd.data_ptr()), B * M - 1, vp(Pd.data_ptr()), M, vp(sd.data_ptr()), D, B, M,
              L.stream_handle()) == -2


@pytest.mark.parametrize("D,M", [(5, 256), (1, 300), (7, 33)])
@pytest.mark.parametrize("dt", [F64, torch.float32])
def test_lbar_reduce_adds_each_factors_output_products_in_order(ops, D, M, dt):
    """nmgp_lbar_reduce (the per-(output, factor) L-bar form of the backward): factor d's M x M gradient block gets
    its lower triangle + Y_{d,d} + ... + Y_{D-1,d} (left to right) and its upper triangle set to 0, as the OUT_TRIL
    product it replaces; its M-vector gets the slots' vectors the same way.  Padding between blocks untouched."""
    import ctypes
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    MM, SY = M * M, M * M + M
    nsl = D * (D + 1) // 2
    g = torch.Generator().manual_seed(D * 7 + M)
    Y = torch.randn(nsl * SY, generator=g, dtype=dt)
    sA, sB = MM + 5, M + 3                       # gradient blocks with gaps between them
    gA = torch.randn(D * sA, generator=g, dtype=dt)
    gB = torch.randn(D * sB, generator=g, dtype=dt)
    refA, refB = gA.clone(), gB.clone()
    low = torch.tril(torch.ones(M, M, dtype=torch.bool)).reshape(-1)
    for d in range(D):
        first = d * D - d * (d - 1) // 2
        a = refA[d * sA:d * sA + MM]
        b = refB[d * sB:d * sB + M]
        for i in range(d, D):
            s = (first + i - d) * SY
            a += Y[s:s + MM]
            b += Y[s + MM:s + SY]
        a[~low] = 0
    Yd, gAd, gBd = Y.to(DEV), gA.to(DEV), gB.to(DEV)
    fn = L.lib().nmgp_lbar_reduce_f64 if dt == F64 else L.lib().nmgp_lbar_reduce_f32
    vp = ctypes.c_void_p
    L.check(fn(vp(Yd.data_ptr()), SY, vp(gAd.data_ptr()), sA, vp(gBd.data_ptr()), sB, D, M, L.stream_handle()),
            "lbar_reduce")
    assert torch.equal(gAd.cpu(), refA)
    assert torch.equal(gBd.cpu(), refB)
    assert fn(vp(Yd.data_ptr()), SY - 1, vp(gAd.data_ptr()), sA, vp(gBd.data_ptr()), sB, D, M,
              L.stream_handle()) == -2


def test_adam_matches_torch(ops):
    g = torch.Generator().manual_seed(8)
    p0 = torch.randn(1000, generator=g, dtype=F64)
    grads = [torch.randn(1000, generator=g, dtype=F64) for _ in range(3)]
    ref = p0.clone().requires_grad_()
    opt = torch.optim.Adam([ref], lr=0.01)
    th = p0.clone().to(DEV)
    m = torch.zeros_like(th)
    v = torch.zeros_like(th)
    step = torch.zeros(1, dtype=torch.int64, device=DEV)
    for gr in grads:
        ref.grad = gr.clone()
        opt.step()
        ops.adam_(th, gr.to(DEV), m, v, step, 0.01)
    assert rel(th, ref) < 1e-14
    assert int(step.cpu()) == 3


def test_normal_rng(ops):
    out = torch.empty(1 << 20, dtype=F64, device=DEV)
    cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
    ops.normal_(out, seed=1234, counter=cnt)
    x = out.cpu()
    assert abs(float(x.mean())) < 5e-3 and abs(float(x.std()) - 1) < 5e-3
    again = torch.empty_like(out)
    ops.normal_(again, seed=1234, counter=cnt)
    assert torch.equal(out, again)
    ops.counter_add_(cnt, 1)
    ops.normal_(again, seed=1234, counter=cnt)
    assert not torch.equal(out, again)


@pytest.mark.parametrize("n,batch", [(1, 1), (2, 3), (5, 2), (33, 2), (64, 1), (65, 1), (200, 1), (300, 2)])
def test_syevj(ops, n, batch):
    # Jacobi eigensolver (eig.hip) vs LAPACK eigh: eigenvalues ascending, V orthonormal, V diag(w) V^T = A
    g = torch.Generator().manual_seed(n * 31 + batch)
    G = torch.randn(batch, n, n, generator=g, dtype=F64)
    A = (G + G.transpose(1, 2)) / 2
    A[0] += torch.diag(torch.linspace(0, 3, n, dtype=F64))
    w, V = ops.syevj(A.to(DEV))
    w, V = w.cpu(), V.cpu()
    wr = torch.linalg.eigvalsh(A)
    scale = float(A.norm())
    assert float((w - wr).abs().max()) <= 1e-13 * scale
    eye = torch.eye(n, dtype=F64).expand(batch, n, n)
    assert float((V.transpose(1, 2) @ V - eye).abs().max()) < 1e-12
    assert float((V @ torch.diag_embed(w) @ V.transpose(1, 2) - A).abs().max()) < 1e-12 * scale


def test_syevj_degenerate_and_kernel_matrix(ops):
    # repeated eigenvalues (identity block) and an ill-conditioned Gibbs kernel matrix of the legacy simulation size
    A = torch.zeros(100, 100, dtype=F64)
    A[:50, :50] = torch.eye(50, dtype=F64)
    A[50:, 50:] = 2 * torch.eye(50, dtype=F64)
    w, V = ops.syevj(A.to(DEV))
    assert torch.equal(w.cpu(), torch.cat([torch.ones(50, dtype=F64), 2 * torch.ones(50, dtype=F64)]))
    x = torch.linspace(0, 1, 200, dtype=F64).view(-1, 1)
    ell = 0.05 + 0.1 * x.view(-1)
    K = O.Nonstationary_RBF_cov(x, ell1=ell)
    w, V = ops.syevj(K.to(DEV))
    wr = torch.linalg.eigvalsh(K)
    assert float((w.cpu() - wr).abs().max()) <= 1e-13 * float(K.norm())
    assert float((V.cpu() @ torch.diag(w.cpu()) @ V.cpu().t() - K).abs().max()) < 1e-12 * float(K.norm())


@pytest.mark.parametrize("P,N", [(2, 200), (3, 70)])
def test_kronecker_gaussian_legacy_sizes(ops, P, N):
    # kron_inv / kron_logdet / multivariate_normal_logpdf0 and the dense logpdf2 on the HIP path vs the oracle
    from collaborative_nonstationary_multivariate_gaussian_process_amd.Utility import kronecker_operation as KO
    from collaborative_nonstationary_multivariate_gaussian_process_amd.Utility import distributions as DI
    g = torch.Generator().manual_seed(P * N)
    Lb = torch.randn(P, P, generator=g, dtype=F64)
    Bm = Lb @ Lb.t() + 0.5 * torch.eye(P, dtype=F64)
    x = torch.linspace(0, 1, N, dtype=F64).view(-1, 1)
    K = torch.exp(-(x - x.t()) ** 2 / 0.05) + 1e-6 * torch.eye(N, dtype=F64)
    y = torch.randn(P * N, generator=g, dtype=F64)
    mu = torch.zeros(P * N, dtype=F64)
    s2 = torch.tensor(0.3, dtype=F64)
    assert float(KO.kron_logdet(s2, Bm, K)) == pytest.approx(float(O.kron_logdet(s2, Bm, K)), rel=1e-11)
    assert rel(KO.kron_inv(s2, Bm, K), O.kron_inv(s2, Bm, K)) < 1e-10
    lp = float(DI.multivariate_normal_logpdf0(y, mu, Bm, K, s2))
    assert lp == pytest.approx(float(O.multivariate_normal_logpdf0(y, mu, Bm, K, s2)), rel=1e-10)
    assert float(DI.multivariate_normal_logpdf2(y, mu, Bm, K, s2)) == pytest.approx(lp, rel=1e-9)


def test_hip_graph_relayed_side_stream_edges(ops):
    """hip_ops.HipGraph (capture through the library's nmgp_graph_* C ABI) with the engine's edge shape: two
    side streams that synchronise with each other only through the capture stream (side -> main -> side2 ->
    main -> side); the replays keep the stream order.  (A direct side <-> side2 ping-pong segfaults inside
    hipStreamEndCapture of the torch-bundled ROCm 7.0 runtime -- tools/graph_edge_probe2.py; the same calls
    on ROCm 7.2's runtime capture cleanly, tools/graph_edge_repro2.hip.)"""
    x = torch.zeros(4096, dtype=F64, device=DEV)
    y = torch.zeros(4096, dtype=F64, device=DEV)
    s1, s2 = torch.cuda.Stream(device=DEV), torch.cuda.Stream(device=DEV)
    g = ops.HipGraph(DEV)
    with g.capture():
        main = torch.cuda.current_stream(DEV)
        ev = lambda: torch.cuda.Event()
        e0 = ev()
        e0.record(main)
        s1.wait_event(e0)
        s2.wait_event(e0)
        with torch.cuda.stream(s1):
            x.add_(1.0)
            e1 = ev()
            e1.record(s1)
        main.wait_event(e1)                    # side -> main
        r1 = ev()
        r1.record(main)
        with torch.cuda.stream(s2):
            s2.wait_event(r1)                  # main -> side2
            y.add_(x)
            e2 = ev()
            e2.record(s2)
        main.wait_event(e2)                    # side2 -> main
        r2 = ev()
        r2.record(main)
        with torch.cuda.stream(s1):
            s1.wait_event(r2)                  # main -> side
            x.mul_(2.0)
            e3 = ev()
            e3.record(s1)
        main.wait_event(e3)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    # per replay: x += 1; y += x; x *= 2  ->  (x, y) = (2, 1), (6, 4), (14, 11)
    assert torch.all(x == 14.0) and torch.all(y == 11.0)


def test_training_step_graph_is_captured_through_hip(ops):
    """DsviTrainer.capture builds the step graph with hip_ops.HipGraph (not torch.cuda.CUDAGraph); side2 never
    waits on side directly while side waits on side2 (the ping-pong the runtime's capture crashes on); the
    replay equals the eager step bit for bit (D=3, M=64)."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
    rng = np.random.default_rng(8)
    D, n, M, B = 3, 120, 64, 360
    xs = [torch.from_numpy(np.sort(rng.uniform(0, 1, n))) for _ in range(D)]
    ys = [torch.from_numpy(np.cos(4 * x.numpy() + d) + 0.2 * rng.standard_normal(n)) for d, x in enumerate(xs)]
    res = []
    for graph in (True, False):
        model = NMGP(number_observations=D * n, dim_outputs=D, Z=np.linspace(0, 1, M), minibatch_size=B, seed=6,
                     device=DEV, noise="device")
        tr = DsviTrainer(model, 0.01)
        eng = model.engine(B)
        x, y, sizes = model._prepare(xs, ys)
        eng.load_batch(x, y, sizes)
        if graph:
            g = tr.capture(eng, include_update=False)
            assert isinstance(g, ops.HipGraph)
            sched = eng._schedule(0)
            sig = {it[2]: it[1] for it in sched if it[0] == "sig"}
            waits = [(it[1], sig[it[2]]) for it in sched if it[0] == "wait"]
            assert ("side", "side2") in waits and ("side2", "side") not in waits
            g.replay()
        else:
            tr.grad_step(eng)
        torch.cuda.synchronize()
        res.append((float(eng.out[0]), model._grad.detach().cpu().clone()))
    assert res[0][0] == res[1][0] and torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("dt,M", [(F64, 256), (torch.float32, 512)])
def test_captured_step_folded_counter_matches_counter_launch(ops, monkeypatch, dt, M):
    """The captured training step with the optimizer step counter advanced by the finalize kernel
    (nmgp_dsvi_args.adam_step) and the update reading it (nmgp_adam_lower_advanced_*) equals the step with the
    counter's own launch (DsviTrainer.FOLD_STEP = False) bit for bit after three replays: theta, m, v, and the
    counter = 3 (M = 256 fp64: the fused prior schedule; fp32 M = 512).  Eager steps afterwards are unaffected
    (the counter is advanced once per update, by update())."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd.nmgp_dsvi import NMGP, DsviTrainer
    rng = np.random.default_rng(21)
    D, B, nb = 3, 240, 2
    res = []
    for fold in (True, False):
        monkeypatch.setattr(DsviTrainer, "FOLD_STEP", fold)
        model = NMGP(number_observations=D * 400, dim_outputs=D, Z=np.linspace(0, 1, M), minibatch_size=B, seed=9,
                     device=DEV, noise="device", dtype=dt)
        tr = DsviTrainer(model, 0.01)
        eng = model.engine(B)
        g = np.random.default_rng(4)
        Xb = torch.tensor(g.uniform(0, 1, (nb, B)), dtype=dt, device=DEV)
        Yb = torch.tensor(g.standard_normal((nb, B)), dtype=dt, device=DEV)
        ids = np.sort(g.integers(0, D, (nb, B)), axis=1)
        Ib = torch.tensor(ids, dtype=torch.int32, device=DEV)
        Sb = torch.tensor(np.stack([np.concatenate([[0], np.cumsum(np.bincount(r, minlength=D))]) for r in ids]),
                          dtype=torch.int32, device=DEV)
        eng.bind_dataset(Xb, Yb, Ib, Sb)
        graph = tr.capture(eng, include_update=True)
        for _ in range(3):
            graph.replay()
        torch.cuda.synchronize()
        assert all(getattr(a, "adam_step", None) in (None, 0) for a in eng._keep_args.values())
        res.append((model._theta.detach().cpu().clone(), tr.m.cpu().clone(), tr.v.cpu().clone(),
                    int(tr.step_count.item())))
    for a, b in zip(res[0][:3], res[1][:3]):
        assert torch.equal(a, b)
    assert res[0][3] == res[1][3] == 3


def test_hip_graph_external_event_node_fires_mid_replay(ops):
    """nmgp_event_record_external inside a capture becomes an external event node: after the graph is
    launched, a stream OUTSIDE the graph that waits on the event runs as soon as that point of the replay is
    reached -- not at the graph's end.  Graph: x = 1 -> [event] -> ~10 ms of GEMMs -> y = 1; the outside
    stream copies (x, y) after its wait: x must be 1 (ordering) and y still 0 (it ran mid-replay).  This is
    what DsviTrainer.dp_graph_step builds the overlapped all-reduce on."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L
    x = torch.zeros(1, dtype=F64, device=DEV)
    y = torch.zeros(1, dtype=F64, device=DEV)
    out = torch.full((2, 3), -1.0, dtype=F64, device=DEV)
    Ab = torch.rand(4096, 4096, device=DEV)
    Cb = torch.zeros(4096, 4096, device=DEV)
    ws = ops.big_workspace(DEV, L.lib().nmgp_gemm_big_workspace_size())
    ops.gemm_big(Ab, Ab, Cb, ws=ws)                    # warm-up (attributes, workspace)
    ev = ops.ExtEvent()
    g = ops.HipGraph(DEV)
    with g.capture():
        main = torch.cuda.current_stream(DEV)
        x.zero_()
        y.zero_()
        x.fill_(1.0)
        ev.record(main)
        for _ in range(8):
            ops.gemm_big(Ab, Ab, Cb, ws=ws)
        y.fill_(1.0)
    comm = torch.cuda.Stream(device=DEV)
    torch.cuda.synchronize()
    # HIP maps streams onto GPU_MAX_HW_QUEUES (4) hardware queues round-robin: once a process has created many
    # streams (the whole suite), `comm` can share the graph stream's queue, and then nothing it holds can run before
    # the replay ends.  Probe that first: a marker on `comm` must finish while a long GEMM on the replay stream is
    # still running.
    cur = torch.cuda.current_stream(DEV)          # the stream the graph is replayed on
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record(cur)
    for _ in range(4):
        ops.gemm_big(Ab, Ab, Cb, ws=ws)
    e1.record(cur)
    comm.wait_event(e0)
    with torch.cuda.stream(comm):
        e2.record(comm)
    torch.cuda.synchronize()
    if e0.elapsed_time(e2) > 0.5 * e0.elapsed_time(e1):
        pytest.skip("the comm stream shares a hardware queue with another stream in this process")
    for rep in range(3):
        g.replay()
        ev.wait(comm)
        with torch.cuda.stream(comm):
            out[0, rep].copy_(x[0])
            out[1, rep].copy_(y[0])
        torch.cuda.current_stream(DEV).wait_stream(comm)
    torch.cuda.synchronize()
    o = out.cpu()
    assert torch.equal(o[0], torch.ones(3, dtype=F64)), o
    assert torch.equal(o[1], torch.zeros(3, dtype=F64)), o


@pytest.mark.parametrize("dt", [F64, torch.float32])
@pytest.mark.parametrize("M", [1024, 256, 68])
def test_pair_streaming_products_vs_torch(ops, dt, M):
    """csrc/pairs.hip (the per-pair products when every output owns few minibatch rows, ECoG shape): quad
    C[r] = A[r] tril(L), dot Z[r] = W[r] tril(L)^T, rank G += tril(P^T W) (strictly upper part of G untouched),
    and the P-bar reduction, against torch on ragged segments -- empty, one row, RB, RB + 1 and 3 RB + 2 rows (the
    chunked path) -- with the upper triangles of L holding junk (mat2ltri ignores them, code/utils.py:68-72)."""
    import torch as T
    g = T.Generator().manual_seed(M)
    sizes = [3, 0, 1, 8, 9, 4, 26, 2]
    D, B = len(sizes), sum(sizes)
    seg = T.tensor(np.concatenate([[0], np.cumsum(sizes)]), dtype=T.int32)
    pairs = [(i, j) for i in range(D) for j in range(i + 1)]
    Q = len(pairs)
    Lb = T.randn(Q, M, M, generator=g, dtype=F64)                    # upper parts junk on purpose
    A = T.randn(3, B, M, generator=g, dtype=F64)                     # P_typ rows
    Wp = T.randn(D, B, M, generator=g, dtype=F64)                    # W-hat slots
    G0 = T.randn(Q, M, M, generator=g, dtype=F64)
    tol = 1e-12 if dt == F64 else 3e-5
    dev = lambda t: t.to(dt).to(DEV).contiguous()
    Ld, Ad, Wd, Gd, segd = dev(Lb), dev(A), dev(Wp), dev(G0), seg.to(DEV)
    C = T.zeros(D, B, M, dtype=dt, device=DEV)
    Z = T.zeros(D, B, M, dtype=dt, device=DEV)
    BM, MM = B * M, M * M
    typ = lambda i, j: 2 if i == j else 1
    q = [(typ(i, j) * BM, p * MM, j * BM, i) for p, (i, j) in enumerate(pairs)]
    ops.PairStream("quad", Ad, Ld, C, q, segd, M)()
    ops.PairStream("dot", Wd, Ld, Z, [(j * BM, p * MM, j * BM, i) for p, (i, j) in enumerate(pairs)], segd, M)()
    ops.PairStream("rank", Ad, Gd, Wd, [(typ(i, j) * BM, p * MM, j * BM, i) for p, (i, j) in enumerate(pairs)],
                   segd, M)()
    torch.cuda.synchronize()
    C, Z, Gd = C.double().cpu(), Z.double().cpu(), Gd.double().cpu()
    Lr, Ar, Wr, G0r = Lb.to(dt).double(), A.to(dt).double(), Wp.to(dt).double(), G0.to(dt).double()
    Gref = G0r.clone()
    for p, (i, j) in enumerate(pairs):
        r = slice(int(seg[i]), int(seg[i + 1]))
        Lt = T.tril(Lr[p])
        Cref = Ar[typ(i, j), r] @ Lt
        Zref = Wr[j, r] @ Lt.t()
        Gref[p] += T.tril(Ar[typ(i, j), r].t() @ Wr[j, r])
        if sizes[i]:
            assert rel(C[j, r], Cref) < tol, (p, i, j)
            assert rel(Z[j, r], Zref) < tol, (p, i, j)
    assert rel(Gd, Gref) < tol
    up = T.triu(T.ones(M, M, dtype=T.bool), 1)
    assert T.equal(Gd[:, up], G0r[:, up])                            # strictly upper part untouched
    # P-bar reduction: P1[r] += Z_i[r], P0[r] += sum_{j < i} Z_j[r] (outputs 2..6 only)
    P = T.randn(4, B, M, generator=g, dtype=F64).to(dt).to(DEV)
    P0 = P.double().cpu()
    Zd = Z.to(dt).to(DEV).contiguous()
    ops.pair_pbar_reduce(Zd, BM, P[1], P[2], M, segd, D, 2, 7, B, M)
    torch.cuda.synchronize()
    ref = P0.clone()
    Zr = Zd.double().cpu()
    for i in range(2, 7):
        r = slice(int(seg[i]), int(seg[i + 1]))
        ref[2, r] += Zr[i, r]
        for j in range(i):
            ref[1, r] += Zr[j, r]
    assert rel(P.double().cpu(), ref) < tol
    assert T.equal(P.double().cpu()[:, :int(seg[2])], P0[:, :int(seg[2])])    # outputs outside [2, 7) untouched


@pytest.mark.parametrize("dt", [F64, torch.float32])
def test_adam_lower_matches_dense_adam(ops, dt):
    """nmgp_adam_lower (only the lower-triangle vectors of the sqrt blocks, code/utils.py:68-72's mat2ltri) equals
    the dense nmgp_adam bit for bit over several steps, with gradients that are zero above each block's diagonal
    (as the model's are) and dense ranges before, between and after the blocks; the step counter advances once."""
    g = torch.Generator().manual_seed(9)
    M = 24
    ranges = [(8, 2), (8 + 2 * M * M + 4, 1), (8 + 3 * M * M + 4 + 12, 3)]     # (offset, blocks), 16-byte aligned
    n = ranges[-1][0] + 3 * M * M + 20
    th0 = torch.randn(n, generator=g, dtype=F64)
    up = torch.triu(torch.ones(M, M, dtype=torch.bool), 1)
    outs = []
    for lower in (False, True):
        th, m, v = th0.to(dt).to(DEV), torch.zeros(n, dtype=dt, device=DEV), torch.zeros(n, dtype=dt, device=DEV)
        step = torch.zeros(1, dtype=torch.int64, device=DEV)
        gg = torch.Generator().manual_seed(10)
        for _ in range(3):
            gr = torch.randn(n, generator=gg, dtype=F64)
            for o, nb in ranges:
                blk = gr[o:o + nb * M * M].view(nb, M, M)
                blk[:, up] = 0.0
            gr = gr.to(dt).to(DEV)
            if lower:
                ops.adam_lower_(th, gr, m, v, step, 0.01, ranges, M)
            else:
                ops.adam_(th, gr, m, v, step, 0.01)
        torch.cuda.synchronize()
        outs.append((th.cpu(), m.cpu(), v.cpu(), int(step.item())))
    for a, b in zip(outs[0][:3], outs[1][:3]):
        assert torch.equal(a, b)
    assert outs[0][3] == outs[1][3] == 3
