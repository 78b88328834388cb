/*
 * nmgp_hip.h -- C ABI of libnmgp_hip.so, the MI355X (gfx950) kernels of the DSVI hot path of
 * Collaborative Nonstationary Multivariate GP inference (reference: code/nmgp_dsvi.py).
 *
 * Conventions:
 *   - plain pointers + sizes, no torch types; every buffer is caller-owned device memory;
 *   - every call only ENQUEUES work on the given hipStream_t (no implicit device sync, no
 *     allocation), so a caller may capture any sequence of calls into a hipGraph;
 *   - return 0 on success, <0 = index of the offending argument (argument error),
 *     NMGP_ERR_LAUNCH on a launch failure.  Numerical failures (non-PD matrix) are reported
 *     LAPACK-style through a device `info` array: info[b] = first failing column (1-based).
 *   - matrices are row-major; T = double (_f64) or float (_f32).
 *
 * Each entry point cites the reference interface it replaces.
 */
#ifndef NMGP_HIP_H
#define NMGP_HIP_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NMGP_OK 0
#define NMGP_ERR_LAUNCH (-1000)

/* ------------------------------------------------------------------ library info */
int nmgp_version(void);

/* Device status word.  Kernels that hand data between workgroups of one launch wait on peers with
 * BOUNDED spins (a lost peer must not hang the GPU); a spin that gives up sets one of these bits
 * instead of failing silently.  nmgp_device_status() ORs the words of every kernel file into *out
 * (host memory) and clears them when `clear` != 0.  It synchronises with the device: call it at a
 * point where the caller syncs anyway (the Python layer does so with the Cholesky `info` check).
 * Any nonzero bit means the results of the launches since the last check are not trustworthy.     */
#define NMGP_STATUS_CHOL_SPIN  1u   /* two-role Cholesky: the inverse role lost its factor role    */
#define NMGP_STATUS_GEMM_SPIN  2u   /* grouped GEMM: a cooperative split-K chunk lost a peer       */
#define NMGP_STATUS_POTRF_SPIN 4u   /* blocked potrf step: the panel publisher never arrived       */
int nmgp_device_status(uint32_t* out, int clear);
/* sizeof of the descriptor structs below (host code checks its own layout against these) */
int64_t nmgp_sizeof_gemm_desc(void);
int64_t nmgp_sizeof_pairwise_desc(void);
int64_t nmgp_sizeof_pairwise_bwd_desc(void);
int64_t nmgp_sizeof_dsvi_args(void);
int64_t nmgp_sizeof_pair_desc(void);
int64_t nmgp_sizeof_chol_tp_args(void);

/* ------------------------------------------------------------------ grouped GEMM (MFMA)
 * C(i,j) = alpha * sum_k op(A)(i,k) * s(k) * op(B)(k,j) + beta*C(i,j) + gamma*rs(i)*E(i,j)
 *          (+ diag_add on i==j)
 * Operands are addressed through strides, which covers transposes, k-concatenated blocks
 * (A(i,k) = A[i*sA_i + (k%kbA)*sA_k + (k/kbA)*sA_kb]) and row / k ranges taken at run time from
 * a device segment table (row_seg / k_seg >= 0: rows or k in [seg[s], seg[s+1])).
 * Replaces every torch.matmul / torch.solve(...)-product in code/utils.py:117-157 and
 * code/nmgp_dsvi.py:172-177 (Sigma = tril(S) tril(S)^T).                                  */
enum {
  NMGP_A_LOWER = 1,      /* op(A)(i,k) = 0 for k > i     */
  NMGP_A_UPPER = 2,      /* op(A)(i,k) = 0 for k < i     */
  NMGP_B_LOWER = 4,      /* op(B)(k,j) = 0 for j > k     */
  NMGP_B_UPPER = 8,      /* op(B)(k,j) = 0 for j < k     */
  NMGP_OUT_LOWER = 16,   /* store only j <= i            */
  NMGP_OUT_TRIL = 32,    /* store j <= i, zero for j > i */
  NMGP_KSCALE = 64,      /* multiply by s(k) = kscale[k] */
  NMGP_EPI = 128,        /* + gamma * rs(i) * E(i,j)     */
  NMGP_EPI_E_LOWER = 256,/* E(i,j) = 0 for j > i         */
  NMGP_DIAG_ADD = 512,   /* + diag_add on i == j         */
  NMGP_EPI_RS_NEG = 1024,/* rs(i) taken with a minus sign */
  NMGP_LAT_COLPACK = 2048,/* latency kernel only (set by the host): a B_LOWER / B_UPPER problem with n == k ==
                          * 32 T, T <= 8, no other mask: tiles_n counts column-tile GROUPS -- {0}, {g, T-g}
                          * for g = 1..(T-1)/2 and {T/2} for even T (B_UPPER mirrored) -- whose k panels add up
                          * to <= 8, one group per workgroup                                                  */
};

typedef struct nmgp_gemm_desc {
  const void* A; const void* B; void* C;
  const void* kscale; const void* epi_E; const void* epi_rs;
  int64_t sA_i, sA_k, sA_kb;
  int64_t sB_k, sB_j, sB_kb;
  int64_t sC_i, sC_j;
  int64_t sE_i, sE_j;
  int32_t m, n, k, kbA, kbB, flags, row_seg, k_seg;
  double alpha, beta, gamma, diag_add;
  int32_t tiles_m, tiles_n, tile_start;
  int32_t seg_span;      /* row_seg / k_seg cover seg[s] .. seg[s + max(seg_span,1)] */
  /* split-K: ksplit > 1 cuts the k range into ksplit chunks; each chunk's 64x64 partial goes to
   * ws (tiles_m*tiles_n*ksplit*4096 elements) and the last-arriving chunk of a tile (counter in
   * `counters`, tiles_m*tiles_n zero-initialised int32, reset by the kernel) sums them in chunk
   * order -- deterministic -- and applies the epilogue.  tiles = tiles_m*tiles_n*ksplit.        */
  int32_t ksplit, pad2_;
  void* ws;
  int32_t* counters;
  /* batch (single-problem launches only): problem b uses A + b*sA_b, B + b*sB_b, C + b*sC_b;
   * batch <= 1 means one problem.  Split-K and batch are exclusive.                           */
  int64_t sA_b, sB_b, sC_b;
  int32_t batch, pad3_;
} nmgp_gemm_desc;

/* d_desc: device array of nprob descriptors (tiles_m/tiles_n/tile_start filled by the host,
 * tiles = ceil(m/64)*ceil(n/64)); total_tiles = sum of tiles; d_seg may be NULL if unused.  */
int nmgp_gemm_grouped_f64(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles,
                          const int32_t* d_seg, hipStream_t stream);
int nmgp_gemm_grouped_f32(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles,
                          const int32_t* d_seg, hipStream_t stream);
/* The same sized on device for this minibatch: a one-workgroup plan kernel turns the segment table
 * into per-problem first tiles (row-segmented problems get ceil(segment rows / 64) row tiles instead
 * of the static tiles_m), written to plan[0..nprob] (caller buffer of nprob + 1 int32), then `grid`
 * workgroups (<= total_tiles; <= 0: total_tiles) stride over the planned tiles.  Same results as the
 * static launch; no workgroups are dispatched for rows other outputs own (HCP: D=50 segments).   */
int nmgp_gemm_grouped_dyn_f64(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles, const int32_t* d_seg,
                              int32_t* plan, int grid, hipStream_t stream);
int nmgp_gemm_grouped_dyn_f32(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles, const int32_t* d_seg,
                              int32_t* plan, int grid, hipStream_t stream);
/* The same descriptors through the latency-oriented kernel (gemm_lat.hip) for groups of short-k
 * problems: 32x32 output tiles (tiles_m = ceil(m/32), tiles_n = ceil(n/32), tile_start in those
 * units, ksplit ignored), the k range of a tile split over the waves of its workgroup, operands
 * loaded straight into MFMA registers.  Requirements: non-negative strides, kbA / kbB either >= k
 * or a multiple of 64, operand extents below 2 GiB.  plan != NULL: sized on device as
 * nmgp_gemm_grouped_dyn_* (32-row tiles), `grid` workgroups (rounded up to a multiple of 8).
 * Same role in the step as nmgp_gemm_grouped_*: code/utils.py:117-146, code/nmgp_dsvi.py:172-258. */
int nmgp_gemm_grouped_lat_f64(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles, const int32_t* d_seg,
                              int32_t* plan, int grid, hipStream_t stream);
int nmgp_gemm_grouped_lat_f32(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles, const int32_t* d_seg,
                              int32_t* plan, int grid, hipStream_t stream);
/* Tile plans computed ahead (e.g. right after the minibatch gather, on another stream): the plan
 * kernels alone (64-row tiles for the tile kernel, 32-row for the latency kernel), and the grouped
 * launches that use such a plan as is.                                                         */
int nmgp_gemm_plan(const nmgp_gemm_desc* d_desc, int nprob, const int32_t* d_seg, int32_t* plan, hipStream_t stream);
int nmgp_gemm_plan_lat(const nmgp_gemm_desc* d_desc, int nprob, const int32_t* d_seg, int32_t* plan,
                       hipStream_t stream);
int nmgp_gemm_grouped_dyn_planned_f64(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles,
                                      const int32_t* d_seg, int32_t* plan, int grid, hipStream_t stream);
int nmgp_gemm_grouped_dyn_planned_f32(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles,
                                      const int32_t* d_seg, int32_t* plan, int grid, hipStream_t stream);
int nmgp_gemm_grouped_lat_planned_f64(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles,
                                      const int32_t* d_seg, int32_t* plan, int grid, hipStream_t stream);
int nmgp_gemm_grouped_lat_planned_f32(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles,
                                      const int32_t* d_seg, int32_t* plan, int grid, hipStream_t stream);
/* Persistent latency-kernel launch for groups with more tiles than one round of workgroups: one
 * workgroup per CU walks its tiles with the next tile's first operand panel loaded under the
 * current tile's MFMAs and reduction; results bit-identical to nmgp_gemm_grouped_lat_*.
 * plan != NULL: device tile plan (planned != 0: already computed by nmgp_gemm_plan_lat).       */
int nmgp_gemm_grouped_lat_pipe_f64(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles,
                                   const int32_t* d_seg, int32_t* plan, int planned, hipStream_t stream);
int nmgp_gemm_grouped_lat_pipe_f32(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles,
                                   const int32_t* d_seg, int32_t* plan, int planned, hipStream_t stream);
/* one problem passed by value (host descriptor; tiles fields are filled internally)          */
int nmgp_gemm_f64(const nmgp_gemm_desc* h_desc, const int32_t* d_seg, hipStream_t stream);
int nmgp_gemm_f32(const nmgp_gemm_desc* h_desc, const int32_t* d_seg, hipStream_t stream);

/* ------------------------------------------------------------------ batched Cholesky
 * In place lower Cholesky of `batch` n x n SPD matrices (A + b*strideA), upper triangle zeroed.
 * Replaces torch.cholesky in code/utils.py:46,54,276,347-348.  info[b] = 0 or the first
 * non-positive pivot column (1-based), as LAPACK potrf.                                     */
int nmgp_potrf_batched_f64(double* A, int64_t n, int64_t lda, int64_t strideA, int64_t batch,
                           int32_t* info, hipStream_t stream);
int nmgp_potrf_batched_f32(float* A, int64_t n, int64_t lda, int64_t strideA, int64_t batch,
                           int32_t* info, hipStream_t stream);
/* Out-of-place inverse of lower-triangular L: X = L^{-1} (upper triangle of X zeroed).
 * Used for K22^{-1} = L^{-T} L^{-1} (replaces torch.solve, code/utils.py:119) and the
 * Cholesky / log-det backward of KL_Gaussian (code/utils.py:332-351).                        */
int nmgp_trtri_batched_f64(const double* L, int64_t n, int64_t ldl, int64_t strideL,
                           double* X, int64_t ldx, int64_t strideX, int64_t batch, hipStream_t stream);
int nmgp_trtri_batched_f32(const float* L, int64_t n, int64_t ldl, int64_t strideL,
                           float* X, int64_t ldx, int64_t strideX, int64_t batch, hipStream_t stream);
/* Fused factor + inverse: A <- L = chol(A) in place (upper zeroed), X <- L^{-1}, info as potrf.
 * n <= 256 runs one register-resident kernel per matrix (the DSVI shapes: code/nmgp_dsvi.py:172-177
 * priors and variational covariances, whose inverses feed K12 K22^{-1} and the KL); larger n (HCP
 * M=512, ECoG M=1024, the M=4096 stress case) recurses on halves: leaves (up to 256 wide in f32, 128 in f64) use that kernel,
 * the panel / SYRK / inverse products are batched MFMA GEMMs of size ~n/2, n/4, ...  X's strictly
 * upper part is used as scratch and left zero.  batch <= 65535.                                */
int nmgp_chol_inv_batched_f64(double* A, int64_t n, int64_t lda, int64_t strideA, double* X, int64_t ldx,
                              int64_t strideX, int64_t batch, int32_t* info, hipStream_t stream);
int nmgp_chol_inv_batched_f32(float* A, int64_t n, int64_t lda, int64_t strideA, float* X, int64_t ldx,
                              int64_t strideX, int64_t batch, int32_t* info, hipStream_t stream);
/* The same with caller workspace for n > 256 (f32): the recursion's products then run split-K where
 * their 128x128 tile grid would not fill the chip (M=4096 stress case).  ws: at least
 * nmgp_chol_inv_workspace_size_f32(n, batch) bytes, zero-filled once before first use (the kernels
 * leave their counters zero again); ws == NULL runs without split-K.                           */
int64_t nmgp_chol_inv_workspace_size_f32(int64_t n, int64_t batch);
int nmgp_chol_inv_batched_ws_f32(float* A, int64_t n, int64_t lda, int64_t strideA, float* X, int64_t ldx,
                                 int64_t strideX, int64_t batch, int32_t* info, void* ws, int64_t ws_bytes,
                                 hipStream_t stream);
/* Round 6, the KL L-bar solve form (f32, n > 256): A <- L as above, but X holds only the inverses X11, X22 of the
 * top-level split's two diagonal blocks (n1 = nmgp_chol_split_point(n) rows / columns, then n - n1): the off-diagonal
 * block X21 = -X22 L21 X11 (two products of the recursion's top level) is not formed, and the factor's off-diagonal
 * block L21 is returned in X21's place (X rows n1.., columns 0..n1-1) -- A21 is left as scratch, A12 and X12 are not
 * written (no staging copy, no zeroing).  The caller applies L^-1 / L^-T blockwise (engine.py, kl_solve):
 * Sigma^-1 L_f = L^-T (L^-1 L_f) for the KL gradient of code/utils.py:339-351 without forming L^-1.           */
int64_t nmgp_chol_split_point(int64_t n);
int nmgp_chol_blockinv_batched_f32(float* A, int64_t n, int64_t lda, int64_t strideA, float* X, int64_t ldx,
                                   int64_t strideX, int64_t batch, int32_t* info, hipStream_t stream);

/* Fused GP-prior launch (round 6): up to 4 prior matrices of one DSVI step (A: K22 + jitter I, read) factored and
 * inverted as nmgp_chol_inv_batched_f64 does (A <- L, X <- L^-1, info), where a matrix with rows != 0 also gets its
 * minibatch products formed by extra workgroups of the same launch while the factorization runs (rows 1: K12 =
 * RBF(x, Z) rows, s2 exp(-(x_i/ls - z_j/ls)^2 / 2) with hyp = (log s2, log ls), code/utils.py:91-94; rows 2: first
 * the t-row sample of JGP_S -- ell_X = exp(P_t v + z_t sqrt(s2_t - ||T_t row||^2 + jitter)), code/utils.py:216-237
 * -- then K12 = Gibbs(x, Z, ell_X, ellZ) rows, code/utils.py:97-103): K12 (written out), T = K12 L^-T (right-looking,
 * from the published block columns of L) and P = T L^-1 = K12 (K22 + jitter I)^-1 (from the published rows of
 * X) -- the projections torch.solve forms in code/utils.py:117-120, 140-146, 228-232.
 * 128 <= n <= 256, 1 <= batch <= 4, B <= 4096; every output of row stride n.  The mats with rows != 0 need K12 /
 * T / P, x and Z; rows 2 needs Pt, Tt (B x n, the t prior's P and T), v, zt, hyp_t (log s2_t), ellX, var_t (B
 * outputs) and ellZ.                                                                                           */
typedef struct nmgp_chol_tp_mat {
  int32_t reserved;   /* 0 */
  int32_t rows;       /* 0: no minibatch products; 1: RBF K12 rows; 2: t-row + Gibbs K12 rows */
  const double* hyp;  /* rows 1: (log sigma2, log lengthscale) */
  double* K12;        /* B x n */
  double* T;          /* B x n */
  double* P;          /* B x n */
} nmgp_chol_tp_mat;
typedef struct nmgp_chol_tp_args {
  double* A;
  int64_t n, lda, strideA;
  double* X;
  int64_t ldx, strideX, batch;
  int32_t* info;
  double jitter;
  const double* Z;     /* n inducing inputs */
  const double* ellZ;  /* n Gibbs length scales (rows 2) */
  const double* x;     /* B minibatch inputs */
  int64_t B;
  const double* Pt;    /* rows 2: the t prior's P and T (B x n), the v sample (n), z_t (B), log s2_t */
  const double* Tt;
  const double* v;
  const double* zt;
  const double* hyp_t;
  double* ellX;        /* rows 2 outputs (B) */
  double* var_t;
  nmgp_chol_tp_mat mats[4];
  /* vg_wgs > 0 (round 6): mats[0] is Sigma_v (rows 0) and vg_wgs extra workgroups form, once L_v is factored,
   * v = vg_muv + L_v vg_z -> vg_v, exp(v) -> vg_ellZ and the Gibbs prior's K22 + jitter I (lower 16 x 16 tiles,
   * leading dimension n) -> vg_K22: nmgp_dsvi_vg22_*'s outputs from the same launch (code/utils.py:97-103,
   * code/nmgp_dsvi.py:198-215).  0: off.                                                                 */
  const double* vg_muv;
  const double* vg_z;
  double* vg_v;
  double* vg_ellZ;
  double* vg_K22;
  int64_t vg_wgs;
} nmgp_chol_tp_args;
int nmgp_chol_tp_f64(const nmgp_chol_tp_args* args, hipStream_t stream);
/* diagnostics (synchronous): the launch's per-workgroup phase stamps, recorded when NMGP_TP_DBG has bit 16 set
 * (8 x 64-bit wall-clock words per workgroup, tools/chol_tp_probe.py)                                  */
int nmgp_chol_tp_trace(uint64_t* out, int64_t n);

/* Single large SPD matrix (the M=4096 stress configuration, BASELINE.json configs[4]): blocked
 * right-looking Cholesky, A <- L in place (strictly upper part zeroed), info as potrf (first
 * non-positive pivot column, 1-based).  Replaces torch.cholesky / LAPACK potrf on one K_uu + jitter
 * (code/utils.py:32-40, 343-344; SIM_code/Utility/kernels.py:64 for the legacy kernels).
 * 128-wide fused leaves, panel GEMM against the leaf's inverse, one block column of lookahead, and the
 * trailing SYRK on a library-owned side stream joined back to `stream` through events (capturable
 * into a graph).  ws: nmgp_potrf_blocked_workspace_size_*(n) bytes, zero-filled once before first use
 * (the split-K counters are left zero again).                                                   */
int64_t nmgp_potrf_blocked_workspace_size_f32(int64_t n);
int64_t nmgp_potrf_blocked_workspace_size_f64(int64_t n);
int nmgp_potrf_blocked_f32(float* A, int64_t n, int64_t lda, int32_t* info, void* ws, int64_t ws_bytes,
                           hipStream_t stream);
int nmgp_potrf_blocked_f64(double* A, int64_t n, int64_t lda, int32_t* info, void* ws, int64_t ws_bytes,
                           hipStream_t stream);

/* ------------------------------------------------------------------ symmetric eigensolver
 * W[b] = eigenvalues of the symmetric A[b] (ascending, as torch.linalg.eigh / torch.symeig), V[b] =
 * eigenvectors as columns (V[i*ldv + j] = component i of vector j).  Replaces torch.symeig(B) /
 * torch.symeig(K) in kron_inv / kron_logdet (code/SIM_code/Utility/kronecker_operation.py:45,47,66,
 * 67) and multivariate_normal_logpdf0/1 (code/SIM_code/Utility/distributions.py:37,40,67,70).
 * Parallel cyclic Jacobi: n <= 64 one workgroup per matrix in LDS; larger n block Jacobi on 64x64
 * pair sub-problems with a device convergence flag (asynchronous, graph-capturable).  A is not
 * modified.  ws: nmgp_syevj_workspace_size_f64(n) bytes (no zero-fill needed).                  */
int64_t nmgp_syevj_workspace_size_f64(int64_t n);
int nmgp_syevj_batched_f64(const double* A, int64_t n, int64_t lda, int64_t strideA, int64_t batch, double* W,
                           int64_t strideW, double* V, int64_t ldv, int64_t strideV, void* ws, int64_t ws_bytes,
                           hipStream_t stream);

/* ------------------------------------------------------------------ large-tile f32 GEMM / SYRK
 * C(i,j) = alpha * sum_k A[i*lda + k] * op(B)(k,j) + beta * C[i*sCi + j*sCj], batched with strides
 * sAb/sBb/sCb; op(B)(k,j) = B[j*ldb + k] (b_kcontig = 1) or B[k*ldb + j] (0).  flags: NMGP_A_LOWER,
 * NMGP_B_UPPER, NMGP_B_LOWER (structural zeros: k ranges trimmed, diagonal k-tiles masked) and
 * NMGP_OUT_LOWER (m == n: only the lower triangle is computed and stored -- SYRK).  128x128 tiles on
 * v_mfma_f32_32x32x2_f32.  The trailing update / panel / inverse products of the recursive
 * Cholesky (the torch.cholesky of code/utils.py:46,276,347 at M >= 512).  ws as above
 * (nmgp_gemm_big_workspace_size bytes) or NULL.                                                */
int64_t nmgp_gemm_big_workspace_size(void);
int nmgp_gemm_big_f32(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kcontig, float* C,
                      int64_t sCi, int64_t sCj, int m, int n, int k, int flags, double alpha, double beta,
                      int64_t sAb, int64_t sBb, int64_t sCb, int batch, void* ws, hipStream_t stream);
/* The same for `batch` problems at arbitrary element offsets (device int64 arrays offA/offB/offC:
 * problem b uses A + offA[b], B + offB[b], C + offC[b]) -- the D + Q variational factors of the
 * engine, which sit at non-uniform offsets of the parameter vector (the live i >= j blocks of the dense
 * D x D Sigma_U layout).  NMGP_OUT_TRIL stores zeros above the diagonal; diag_add is added to C(i,i)
 * (Sigma_f = tril(S_f) tril(S_f)^T + jitter I, code/nmgp_dsvi.py:172-177, code/utils.py:343-344).  */
int nmgp_gemm_big_offsets_f32(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kcontig, float* C,
                              int64_t sCi, int64_t sCj, int m, int n, int k, int flags, double alpha, double beta,
                              double diag_add, const int64_t* offA, const int64_t* offB, const int64_t* offC,
                              int batch, void* ws, hipStream_t stream);
/* General form: op(A)(i,k) = A[i*lda + k] (a_kcontig = 1) or A[k*lda + i] (0), NMGP_A_UPPER allowed,
 * and with NMGP_EPI (+ NMGP_EPI_E_LOWER) the epilogue adds gamma * RS_b[i] * E_b(i, j), E_b = E + offE[b]
 * with strides (sEi, sEj), RS_b = RS + offRS[b]: the KL L-bar of every variational factor,
 * -C^-T (C^-1 L) + diag(1/C_ii^2) L (code/utils.py:339-351 and its autograd), for all D + Q + 1
 * factors in one launch.  kseg != NULL: problem b sums k over [seg[kseg[b]], seg[kseg[b] + kspan[b]])
 * of the device segment table (A and B advanced to that k), the rows of the outputs it covers -- the
 * L-bar products P^T W of the quadratic forms (code/nmgp_dsvi.py:227-258 and their autograd).
 * All nmgp_gemm_big_* forms: every problem's A, B, C and E span must stay below 2 GiB (32-bit buffer
 * offsets; -40 otherwise), output strides are non-negative, and E must not alias C (a tile's C and E
 * values are read before its stores).                                                               */
int nmgp_gemm_big_offsets_epi_f32(const float* A, int64_t lda, int a_kcontig, const float* B, int64_t ldb,
                                  int b_kcontig, float* C, int64_t sCi, int64_t sCj, int m, int n, int k, int flags,
                                  double alpha, double beta, double diag_add, const int64_t* offA,
                                  const int64_t* offB, const int64_t* offC, const float* E, const int64_t* offE,
                                  int64_t sEi, int64_t sEj, const float* RS, const int64_t* offRS, double gamma,
                                  const int32_t* seg, const int32_t* kseg, const int32_t* kspan, int batch,
                                  void* ws, hipStream_t stream);
/* ... and with per-problem ROW ranges (rseg != NULL): problem b's rows are [seg[rseg[b]], seg[rseg[b] +
 * rspan[b]]) of A, C (and E, RS), at most m -- the quadratic-form factors W = P L and the P-bar products
 * W-hat L^T on the rows of the outputs each latent / pair factor serves (code/nmgp_dsvi.py:227-258), on the
 * 128x128 kernel for the fp32 M >= 512 shapes.  Not with NMGP_OUT_LOWER.                                  */
int nmgp_gemm_big_offsets_seg_f32(const float* A, int64_t lda, int a_kcontig, const float* B, int64_t ldb,
                                  int b_kcontig, float* C, int64_t sCi, int64_t sCj, int m, int n, int k, int flags,
                                  double alpha, double beta, double diag_add, const int64_t* offA,
                                  const int64_t* offB, const int64_t* offC, const float* E, const int64_t* offE,
                                  int64_t sEi, int64_t sEj, const float* RS, const int64_t* offRS, double gamma,
                                  const int32_t* seg, const int32_t* kseg, const int32_t* kspan, const int32_t* rseg,
                                  const int32_t* rspan, int batch, void* ws, hipStream_t stream);
/* NMGP_EPI product (offsets, no OUT_LOWER / OUT_TRIL, no split-K) that also stores the raw product
 * acc(i, j) = sum_k op(A)(i,k) op(B)(k,j) to D_b(i, j) = D[offD[b] + i*sDi + j] (sDi >= n) besides
 * C = alpha acc + beta C + gamma RS E: the KL L-bar solve form's G21 = X22^T W21, added to the gradient rows and
 * needed again for G11 = X11^T (W11 - L21^T G21).  a_kcontig 0 or 1, b_kcontig 0.                       */
int nmgp_gemm_big_offsets_dual_f32(const float* A, int64_t lda, int a_kcontig, const float* B, int64_t ldb,
                                   int b_kcontig, float* C, int64_t sCi, int64_t sCj, int m, int n, int k, int flags,
                                   double alpha, double beta, const int64_t* offA, const int64_t* offB,
                                   const int64_t* offC, const float* E, const int64_t* offE, int64_t sEi, int64_t sEj,
                                   const float* RS, const int64_t* offRS, double gamma, float* D, const int64_t* offD,
                                   int64_t sDi, int batch, hipStream_t stream);

/* ------------------------------------------------------------------ pairwise kernel builder
 * mode RBF:   K = scale2 * exp(-0.5 * ||x/ls - z/ls||^2)          (code/utils.py:91-94)
 *             EXPAND distance: ||x||^2+||z||^2-2x.z on x/ls, z/ls (SIM_code/Utility/kernels.py:24-43)
 * mode GIBBS: K = scale2 * [sigX sigZ] * sqrt(2 lx lz / (lx^2+lz^2)) * exp(-r2/(lx^2+lz^2))
 *             (code/utils.py:97-103; SIM_code/Utility/kernels.py:46-73 with sigma, EXPAND)
 * + diag_add on i == j (the 1e-4 / 1e-6 jitters).                                            */
enum { NMGP_RBF = 0, NMGP_GIBBS = 1 };
enum { NMGP_DIST_DIFF = 0, NMGP_DIST_EXPAND = 1 };
enum { NMGP_HYP_LOG = 1 };     /* hyp[] holds log(scale2), log(ls): exponentiate on device */

typedef struct nmgp_pairwise_desc {
  const void* X; const void* Z;          /* (n x p), (m x p) row-major                  */
  const void* ellX; const void* ellZ;    /* GIBBS per-point length scales               */
  const void* sigX; const void* sigZ;    /* optional per-point sigma (legacy), or NULL  */
  const void* hyp;                       /* device [scale2, ls] (RBF) / [scale2] (GIBBS), or NULL */
  void* K;
  int64_t ldk;
  int32_t n, m, p, mode, dist, flags;
  double scale2, length_scale, diag_add;
  int32_t tiles, tile_start;   /* tiles = ceil(n/8) * ceil(m/64) (8-row x 64-column output tiles)           */
} nmgp_pairwise_desc;

int nmgp_pairwise_f64(const nmgp_pairwise_desc* d_desc, int ndesc, int total_tiles, hipStream_t stream);
int nmgp_pairwise_f32(const nmgp_pairwise_desc* d_desc, int ndesc, int total_tiles, hipStream_t stream);
int nmgp_pairwise_single_f64(const nmgp_pairwise_desc* h_desc, hipStream_t stream);
int nmgp_pairwise_single_f32(const nmgp_pairwise_desc* h_desc, hipStream_t stream);

/* Backward of the builder for Kbar = Rbar - rowcoef(i) * Pm (Pm / rowcoef optional):
 *   RBF:   scal_part[t*2+0] += sum Kbar*K, scal_part[t*2+1] += sum Kbar*K*r2   (per tile t)
 *   GIBBS: row_part[ct*n + i] = sum_j Kbar*K*dlogK/dlx_i over column tile ct,
 *          col_part[rt*m + j] = sum_i Kbar*K*dlogK/dlz_j over row tile rt,
 *          scal_part[t*2+0]  = sum Kbar*K
 * Tiles are 8 rows x 64 columns (tiles = ceil(n/8) * ceil(m/64)); partial sums are deterministic.   */
typedef struct nmgp_pairwise_bwd_desc {
  const void* X; const void* Z; const void* ellX; const void* ellZ; const void* hyp;
  const void* K; const void* Rbar; const void* Pm; const void* rowcoef;
  void* row_part; void* col_part; void* scal_part;
  int64_t ld;
  int32_t n, m, p, mode, flags, tiles, tile_start, pad_;
  double scale2, length_scale;
} nmgp_pairwise_bwd_desc;

int nmgp_pairwise_bwd_f64(const nmgp_pairwise_bwd_desc* d_desc, int ndesc, int total_tiles, hipStream_t stream);
int nmgp_pairwise_bwd_f32(const nmgp_pairwise_bwd_desc* d_desc, int ndesc, int total_tiles, hipStream_t stream);
int nmgp_pairwise_bwd_single_f64(const nmgp_pairwise_bwd_desc* h_desc, hipStream_t stream);
int nmgp_pairwise_bwd_single_f32(const nmgp_pairwise_bwd_desc* h_desc, hipStream_t stream);

/* Deterministic column sums of a (rows x cols) row-major array: out[j] = beta*out[j] + sum_i a[i*cols+j] */
int nmgp_colsum_f64(const double* a, int64_t rows, int64_t cols, double beta, double* out, hipStream_t stream);
int nmgp_colsum_f32(const float* a, int64_t rows, int64_t cols, double beta, float* out, hipStream_t stream);

/* ------------------------------------------------------------------ Kronecker kernels
 * kronecker_product (SIM_code/Utility/kronecker_operation.py:5-22): out[(i*r2+k)*(c1*c2)+j*c2+l] =
 *   t1[i,j]*t2[k,l]  (one multiply per element: bit-exact)
 * kronecker_product_diag (:25-33): out[i*n2+k] = d1[i]*d2[k]
 * kron_mv (:72-85): out = (B kron K) y, B (P1 x P2), K (N1 x N2), y (P2*N2) -> (P1*N1).  P2 <= 8: one
 *   fused launch streaming K once (work unused, may be NULL); otherwise two GEMMs through work (N1*P2). */
int nmgp_kron_product_f64(const double* t1, int64_t r1, int64_t c1, const double* t2, int64_t r2, int64_t c2,
                          double* out, hipStream_t stream);
int nmgp_kron_product_diag_f64(const double* d1, int64_t n1, const double* d2, int64_t n2, double* out,
                               hipStream_t stream);
int nmgp_kron_mv_f64(const double* B, int64_t P1, int64_t P2, const double* K, int64_t N1, int64_t N2,
                     const double* y, double* out, double* work, hipStream_t stream);
int nmgp_kron_product_f32(const float* t1, int64_t r1, int64_t c1, const float* t2, int64_t r2, int64_t c2,
                          float* out, hipStream_t stream);
int nmgp_kron_product_diag_f32(const float* d1, int64_t n1, const float* d2, int64_t n2, float* out,
                               hipStream_t stream);
int nmgp_kron_mv_f32(const float* B, int64_t P1, int64_t P2, const float* K, int64_t N1, int64_t N2,
                     const float* y, float* out, float* work, hipStream_t stream);

/* ------------------------------------------------------------------ DSVI step kernels
 * The fused, closed-form DSVI objective and gradients (NMGP.forward + autograd backward,
 * code/nmgp_dsvi.py:157-301) are assembled by the host from the primitives above plus the
 * row / reduction kernels below, all reading one argument block.  See DESIGN.md §4.       */
typedef struct nmgp_dsvi_args {
  /* sizes */
  int32_t D, M, B, Q, NF, elbo_mode, frozen_mask;
  int32_t pair_packed;         /* 0: mu_U (D,D,M), sqrt_U (D,D,M,M) as the reference; 1: (Q,M), (Q,M,M) */
  double N_over_B, jitter;
  /* parameters: flat theta in the registration order of code/nmgp_dsvi.py:117-155 */
  const void* theta; void* grad;
  int64_t off_muW, off_sW, off_muv, off_sv, off_muU, off_sU, off_hyp;
  /* minibatch: rows grouped by output; seg[o]..seg[o+1] = rows of output o */
  const void* x; const void* y; const int32_t* row_out; const int32_t* seg; const void* Z;
  const void* noise;          /* z_v (M) | z_t (B) | z_pairs (Q x B), reference call order */
  /* factor storage (see DESIGN.md §3 for the layout) */
  void* Afac;                 /* (NF+4, M, M): A1 -> C1 (variational), then priors t,0,1,G -> C2 */
  void* Cinv;                 /* (NF+4, M, M) inverses of the factors                          */
  void* Ainv;                 /* (4, M, M) prior inverses t,0,1,G                              */
  void* K12; void* P; void* Pbar; void* R;   /* (4, B, M) each, order t,0,1,G           */
  void* Abar;                 /* (4, M, M) prior adjoints                                      */
  void* WG; void* WP;         /* (D, B, M) quadratic-form factors                              */
  void* Y;                    /* Ainv * mu : G (D x M) | t (1 x M) | 0 (D*D x M) | 1 (D*D x M)   */
  void* Xs;                   /* (NF, M, M) scratch: Cinv_f * L_f                              */
  void* v; void* vbar; void* ellZ; void* ellX; void* var_t;   /* (M),(M),(M),(B),(B)          */
  void* rowbuf;               /* (2D+5, B) per-row adjoints                                     */
  void* facbuf;               /* KL (NF) | delta (4,M) | wvec (4,M) | sel (4,D*D) | e (NF,M)   */
  void* red;                  /* per-block partial sums                                        */
  void* out;                  /* [0] loss [1] SELBO_R [2] KL_W [3] KL_v [4] KL_U  (16 entries;  */
                              /* [8..14] training-step pre-sums of nmgp_dsvi_prefinal_*)      */
  void* gib_row; void* gib_col; void* scal_part; void* phi;
  int32_t* info;
  int32_t n_ct, n_rt, n_rt22, nblk_rows;
  int64_t scal_off[8];        /* tile offsets of the RBF backward problems L0_12,L0_22,L1_12,L1_22,t12,t22 */
  void* T;                    /* (4, B, M) K12 C2^-T per prior (t,0,1,G): the Nystrom variance
                                 rowsum(P o K12) is formed as ||T_row||^2 (no cancellation-prone
                                 explicit-inverse product) and P = T C2^-1                       */
  /* pair sharding (SURVEY §8e axis 3; 0 / D / 1 = the whole model): the packed pairs this rank holds
     are [pair_q0, pair_q0 + Q) -- the pairs (i, j <= i) of a contiguous range of outputs, blocks of
     mu_U / sqrt_U / Y / noise numbered from pair_q0; n_wfac = number of W factors in the factor list
     (D on the rank that owns KL_W, else 0); kl_v = 1 on the rank that owns KL_v                   */
  int32_t pair_q0, n_wfac, kl_v, pair_pad;
  /* fp32 engines (round 3): (4, B, M) fp64 K12 C2^-T per prior, formed from fp64 kernel matrices and fp64
     prior factors; when set, the Nystrom variances k11 - ||T_row||^2 are taken from it in fp64 (the fp32
     T is not read).  NULL: use T */
  const void* T64;
  /* KL factor range (round 3, compute_ELBO with the KL sharded over ranks): only the variational factors
     f in [kl_f0, kl_f1) of the W | pairs list (and the v factor when kl_v) are given a KL term; the whole
     model is [0, NF - 1) */
  int32_t kl_f0, kl_f1;
  /* fp64 sample / hyper-gradient path of fp32 engines (round 3; all NULL otherwise):
     v64     (M, M) fp64 lower Cholesky factor of Sigma_v + 1e-4 I: the v sample mu_v + C z is formed in
             fp64 (ell_Z = exp(v) amplifies its absolute error), written to v / ellZ (fp32) and ellZ64;
     ellZ64  (M) fp64 ell_Z;
     K12_64  (4, B, M) fp64 K12 of the priors (slot 0 = t);
     t64     fp64 t-prior adjoint workspace: [P-bar_t (B x M) | varbar (B) | per-4-row varbar partials]
             written by the t-row backward (the t-prior builder backward and hyper-parameter partials then
             run in fp64 from it: K12 - P K22 cancels to ~1e-4 P, cond ~1e7 at the ECoG length scales);
     scal64  fp64 hyper-parameter partials of the t-prior builders (t12 tiles, then t22 tiles), summed
             by the finalize kernel in fp64 (sigma2_tildeell_log / length_scales_tildeell_log)          */
  const void* v64;
  void* ellZ64;
  const void* K12_64;
  void* t64;
  void* scal64;
  /* round 6: when non-NULL, the training step's finalize kernel advances this optimizer step counter by one at its
     end (the captured step then runs nmgp_adam_lower_advanced_*, which reads the advanced counter: one launch fewer
     at the step's tail).  NULL: untouched.                                                                      */
  int64_t* adam_step;
} nmgp_dsvi_args;

int nmgp_dsvi_hyper_f64(const nmgp_dsvi_args* a, hipStream_t s);      /* hyper values + v sample   */
int nmgp_dsvi_vg22_f64(const nmgp_dsvi_args* a, hipStream_t s);       /* v sample + K_G22 + jitter I (fused priors) */
int nmgp_dsvi_trow_f64(const nmgp_dsvi_args* a, hipStream_t s);       /* t-row forward             */
int nmgp_dsvi_recon_f64(const nmgp_dsvi_args* a, hipStream_t s);      /* recon + per-row adjoints  */
int nmgp_dsvi_kl_f64(const nmgp_dsvi_args* a, hipStream_t s);         /* KL per factor + e-vectors */
int nmgp_dsvi_delta_f64(const nmgp_dsvi_args* a, hipStream_t s);      /* prior diag adjoints delta, w */
int nmgp_dsvi_tbwd_f64(const nmgp_dsvi_args* a, hipStream_t s);       /* t-row backward            */
int nmgp_dsvi_vbwd_f64(const nmgp_dsvi_args* a, hipStream_t s);       /* v backward -> Phi         */
int nmgp_dsvi_finalize_f64(const nmgp_dsvi_args* a, hipStream_t s);   /* loss + scalar gradients   */
int nmgp_dsvi_mugrad_f64(const nmgp_dsvi_args* a, hipStream_t s);     /* KL mean gradients of mu_W / mu_v / mu_U */
/* Training steps: nmgp_dsvi_finalize_* adds the KL mean gradients itself when D M + M + (pair columns) M is at most
 * NMGP_MUGRAD_IN_FINALIZE_MAX; larger engines launch nmgp_dsvi_mugrad_* (after the L-bar and v backward, before
 * finalize).                                                                                                   */
#define NMGP_MUGRAD_IN_FINALIZE_MAX 65536
int nmgp_dsvi_prefinal_f64(const nmgp_dsvi_args* a, hipStream_t s);   /* training step: recon + KL sums -> out[8..14] */
/* fp32 twins (HCP / ECoG-shaped configurations): same arguments, every buffer float */
int nmgp_dsvi_hyper_f32(const nmgp_dsvi_args* a, hipStream_t s);
int nmgp_dsvi_vg22_f32(const nmgp_dsvi_args* a, hipStream_t s);
int nmgp_dsvi_trow_f32(const nmgp_dsvi_args* a, hipStream_t s);
int nmgp_dsvi_recon_f32(const nmgp_dsvi_args* a, hipStream_t s);
int nmgp_dsvi_kl_f32(const nmgp_dsvi_args* a, hipStream_t s);
int nmgp_dsvi_delta_f32(const nmgp_dsvi_args* a, hipStream_t s);
int nmgp_dsvi_tbwd_f32(const nmgp_dsvi_args* a, hipStream_t s);
int nmgp_dsvi_vbwd_f32(const nmgp_dsvi_args* a, hipStream_t s);
int nmgp_dsvi_finalize_f32(const nmgp_dsvi_args* a, hipStream_t s);
int nmgp_dsvi_mugrad_f32(const nmgp_dsvi_args* a, hipStream_t s);
int nmgp_dsvi_prefinal_f32(const nmgp_dsvi_args* a, hipStream_t s);

/* ------------------------------------------------------------------ optimiser / RNG
 * torch.optim.Adam update (code/nmgp_dsvi.py:777,854) on a flat parameter vector; step is a
 * device counter (incremented by the kernel's last block) so the call can be graph-replayed.  */
int nmgp_adam_f64(double* theta, const double* grad, double* m, double* v, int64_t n,
                  int64_t* step, double lr, double beta1, double beta2, double eps, hipStream_t stream);
int nmgp_adam_f32(float* theta, const float* grad, float* m, float* v, int64_t n,
                  int64_t* step, double lr, double beta1, double beta2, double eps, hipStream_t stream);
/* The same update where the ranges tri[2k] .. tri[2k] + tri[2k+1] M^2 of the vector are lower-triangular M x M
 * blocks (sqrt_W, sqrt_v, sqrt_U: their strictly upper triangles never receive a gradient, code/utils.py:68-72 --
 * torch's Adam leaves them unchanged): only the 16-byte vectors holding lower-triangle elements are read and
 * written there (bit-identical to nmgp_adam_*); ranges ascending and disjoint, 16-byte aligned, M % (16 / size) == 0.
 * tri is a HOST array of ntri (offset, blocks) pairs.  One step-counter increment.                          */
int nmgp_adam_lower_f64(double* theta, const double* grad, double* m, double* v, int64_t n, const int64_t* tri,
                        int ntri, int M, int64_t* step, double lr, double beta1, double beta2, double eps,
                        hipStream_t stream);
int nmgp_adam_lower_f32(float* theta, const float* grad, float* m, float* v, int64_t n, const int64_t* tri, int ntri,
                        int M, int64_t* step, double lr, double beta1, double beta2, double eps, hipStream_t stream);
/* The same update for a step counter that was ALREADY advanced for this step (by the finalize kernel, adam_step
 * above): the bias corrections use step[0] itself and the counter is not advanced again.  One launch; needs the
 * aligned single-launch form (16-byte pointers, M and every range offset multiples of 16 / size, ntri <= 4), else
 * -12.                                                                                                          */
int nmgp_adam_lower_advanced_f64(double* theta, const double* grad, double* m, double* v, int64_t n,
                                 const int64_t* tri, int ntri, int M, const int64_t* step, double lr, double beta1,
                                 double beta2, double eps, hipStream_t stream);
int nmgp_adam_lower_advanced_f32(float* theta, const float* grad, float* m, float* v, int64_t n, const int64_t* tri,
                                 int ntri, int M, const int64_t* step, double lr, double beta1, double beta2,
                                 double eps, hipStream_t stream);
/* Counter-based Philox4x32-10 standard normals: out[i] = N(0,1) for stream (seed, *counter + i) */
int nmgp_normal_f64(double* out, int64_t n, uint64_t seed, const int64_t* counter, int64_t offset,
                    hipStream_t stream);
int nmgp_normal_f32(float* out, int64_t n, uint64_t seed, const int64_t* counter, int64_t offset,
                    hipStream_t stream);
int nmgp_counter_add(int64_t* counter, int64_t inc, hipStream_t stream);
/* Element-wise precision conversion dst[i] = (dst type) src[i] (round to nearest for f64 -> f32).
 * fp32 engines (HCP / ECoG shapes) factor the four GP priors K22 + 1e-4 I in fp64: the fp32
 * explicit-inverse projections K12 (K22 + 1e-4 I)^-1 of code/utils.py:117-119 otherwise lose
 * ~cond(K22) * eps.                                                            */
/* P-bar_G of the DSVI backward (autograd of code/nmgp_dsvi.py:227-238 through utils.MGP_mu_sigma2,
 * code/utils.py:128-146): for every row r of output i (rows grouped by output, seg[0..D]),
 * P[r, :] += Z[0][r, :] + Z[1][r, :] + ... + Z[i][r, :] in that order, where Z[d] = W-hat_d L_d^T (stride sZ
 * elements between factors, row stride M) was formed for the rows of outputs >= d.  0 or -(argument). */
int nmgp_pbar_reduce_f64(const double* Z, int64_t sZ, double* P, int64_t ldp, const int32_t* seg, int D, int B, int M,
                         hipStream_t stream);
int nmgp_pbar_reduce_f32(const float* Z, int64_t sZ, float* P, int64_t ldp, const int32_t* seg, int D, int B, int M,
                         hipStream_t stream);
/* ------------------------------------------------------------------ pair-block streaming products (round 5)
 * The per-pair products of the DSVI step when each output owns few minibatch rows (ECoG: ~4 of B = 512 per
 * output, Q = 8256 pairs of M = 1024): one problem per coefficient pair (i, j), rows r in [seg[s], seg[s+1]).
 * Each streams its M x M lower-triangular block once (HBM-bound) with the rows' operands on chip; row r of an
 * operand at base + offset + r * M (row stride M), blocks row-major with leading dimension M.
 *   quad : C[r] = A[r] L              (A at a_off, L at l_off, C at c_off)  -- code/utils.py:115-120 (MGP_d),
 *                                      the quadratic-form factors W = P L_ij of code/nmgp_dsvi.py:227-237
 *   dot  : Z[r] = W[r] L^T            (W at a_off, L at l_off, Z at c_off)  -- their P-bar (autograd)
 *   rank : G[k][c] += sum_r P[r][k] W[r][c] for c <= k  (P at a_off, G at l_off, W at c_off; the strictly
 *          upper part of G is not touched)                                -- the pair's L-bar (autograd)
 *   mv   : C[c] += sum_r A[r][c] x[r] over the problem's rows (A at a_off, x at l_off, C at c_off; any M)
 *          -- the pair's mu-bar (autograd of mu_ij in W = mu + L eps), round 6
 *   pair_pbar_reduce: row r of output i (i0 <= i < i1): P1[r] += Z_i[r], P0[r] += Z_0[r] + ... + Z_{i-1}[r]
 *          in j order (Z_j at Z + j sZ) -- the L1 / L0 prior P-bars of code/nmgp_dsvi.py:227-237
 * M must be a multiple of 4 (f32) / 2 (f64); quad needs M <= 2048 (f32) / 3072 (f64), dot and rank M <= 1024.
 * Deterministic (fixed summation order).  0 or -(argument index).                                       */
typedef struct nmgp_pair_desc {
  int64_t a_off, l_off, c_off;   /* element offsets of the three operands */
  int32_t seg;                   /* segment index s: the problem's rows are seg[s] .. seg[s+1]-1 */
  int32_t pad;
} nmgp_pair_desc;
int nmgp_pair_quad_f64(const double* A, const double* L, double* C, const nmgp_pair_desc* descs, int nprob,
                       const int32_t* seg, int M, hipStream_t stream);
int nmgp_pair_quad_f32(const float* A, const float* L, float* C, const nmgp_pair_desc* descs, int nprob,
                       const int32_t* seg, int M, hipStream_t stream);
int nmgp_pair_dot_f64(const double* W, const double* L, double* Z, const nmgp_pair_desc* descs, int nprob,
                      const int32_t* seg, int M, hipStream_t stream);
int nmgp_pair_dot_f32(const float* W, const float* L, float* Z, const nmgp_pair_desc* descs, int nprob,
                      const int32_t* seg, int M, hipStream_t stream);
int nmgp_pair_rank_f64(const double* P, double* G, const double* W, const nmgp_pair_desc* descs, int nprob,
                       const int32_t* seg, int M, hipStream_t stream);
int nmgp_pair_rank_f32(const float* P, float* G, const float* W, const nmgp_pair_desc* descs, int nprob,
                       const int32_t* seg, int M, hipStream_t stream);
int nmgp_pair_mv_f64(const double* A, const double* x, double* C, const nmgp_pair_desc* descs, int nprob,
                     const int32_t* seg, int M, hipStream_t stream);
int nmgp_pair_mv_f32(const float* A, const float* x, float* C, const nmgp_pair_desc* descs, int nprob,
                     const int32_t* seg, int M, hipStream_t stream);
int nmgp_pair_pbar_reduce_f64(const double* Z, int64_t sZ, double* P0, double* P1, int64_t ldp, const int32_t* seg,
                              int D, int i0, int i1, int B, int M, hipStream_t stream);
int nmgp_pair_pbar_reduce_f32(const float* Z, int64_t sZ, float* P0, float* P1, int64_t ldp, const int32_t* seg,
                              int D, int i0, int i1, int B, int M, hipStream_t stream);
/* L-bar / mu-bar of the latent factors in the DSVI backward (autograd of code/nmgp_dsvi.py:198-215, W = mu + L eps
 * and MGP_d's L-products): factor d's gradient collects Y_{i,d} = P_G[rows of i]^T W-hat_d[rows of i] over outputs
 * i = d .. D-1.  Slot (i, d) is Y + (first(d) + i - d) * sY, first(d) = sum_{d' < d} (D - d'): an M x M matrix, then an
 * M-vector at offset M * M.  Adds, in i order, the matrices' lower triangles onto gA + d * sA (upper triangle set to
 * 0) and the vectors onto gB + d * sB.  0 or -(argument).                                                          */
int nmgp_lbar_reduce_f64(const double* Y, int64_t sY, double* gA, int64_t sA, double* gB, int64_t sB, int D, int M,
                         hipStream_t stream);
int nmgp_lbar_reduce_f32(const float* Y, int64_t sY, float* gA, int64_t sA, float* gB, int64_t sB, int D, int M,
                         hipStream_t stream);
int nmgp_convert_f32_to_f64(const float* src, double* dst, int64_t n, hipStream_t stream);
int nmgp_convert_f64_to_f32(const double* src, float* dst, int64_t n, hipStream_t stream);
/* On-device minibatch pipeline (replaces the host DataLoader + vec2list split of
 * code/nmgp_dsvi.py:816-837 for a dataset resident in HBM): copies minibatch
 * b = (*batch_counter) % nbatch of pre-split, output-grouped batches (Xb/Yb (nbatch,B) f64, Ib
 * (nbatch,B) int32 row->output, Sb (nbatch,nseg) int32 segment table) into the engine's inputs
 * and then advances *batch_counter -- one launch, graph-capturable, no host work per step.      */
/* Start of one training step in a single launch: the minibatch gather of nmgp_batch_gather_* (batch
 * (*bctr) % nbatch, bctr advanced), nnoise Philox normals exactly as nmgp_normal_*(noise, nnoise, seed,
 * nctr, 0) with *nctr advanced by one afterwards, and grad[0:ngrad] = 0 -- the DataLoader draw
 * (code/nmgp_dsvi.py:829-837), optimizer.zero_grad() (:830) and the step's torch.randn draws
 * (code/utils.py:123, 226, 234).  done: one int32, zero before first use (left zero).            */
int nmgp_step_begin_f64(const double* Xb, const double* Yb, const int32_t* Ib, const int32_t* Sb, int64_t B,
                        int64_t nseg, int64_t nbatch, int64_t* bctr, double* x, double* y, int32_t* row_out,
                        int32_t* seg, double* noise, int64_t nnoise, uint64_t seed, int64_t* nctr, int32_t* done,
                        double* grad, int64_t ngrad, hipStream_t stream);
int nmgp_step_begin_f32(const float* Xb, const float* Yb, const int32_t* Ib, const int32_t* Sb, int64_t B,
                        int64_t nseg, int64_t nbatch, int64_t* bctr, float* x, float* y, int32_t* row_out,
                        int32_t* seg, float* noise, int64_t nnoise, uint64_t seed, int64_t* nctr, int32_t* done,
                        float* grad, int64_t ngrad, hipStream_t stream);
int nmgp_batch_gather_f64(const double* Xb, const double* Yb, const int32_t* Ib, const int32_t* Sb, int64_t B,
                          int64_t nseg, int64_t nbatch, int64_t* batch_counter, double* x, double* y,
                          int32_t* row_out, int32_t* seg, hipStream_t stream);
int nmgp_batch_gather_f32(const float* Xb, const float* Yb, const int32_t* Ib, const int32_t* Sb, int64_t B,
                          int64_t nseg, int64_t nbatch, int64_t* batch_counter, float* x, float* y,
                          int32_t* row_out, int32_t* seg, hipStream_t stream);

/* Whole-step HIP graphs (the reference runs its step eagerly, code/nmgp_dsvi.py:829-854; the build captures
 * noise -> forward -> backward -> Adam once and replays it).  Capture goes straight through the HIP runtime:
 * begin on `stream` (thread-local mode; other streams join through event waits and must join back before
 * the end), end + instantiate into an executable graph handle, launch it on a stream, destroy it.  The body
 * must not allocate or synchronise.  Returns NMGP_ERR_LAUNCH on a runtime failure; a failed end of capture
 * leaves nothing behind.                                                                                  */
int nmgp_graph_begin(hipStream_t stream);
int nmgp_graph_end(hipStream_t stream, void** exec_out);
int nmgp_graph_launch(void* exec, hipStream_t stream);
int nmgp_graph_destroy(void* exec);

/* Events a captured step graph records as EXTERNAL event nodes (hipEventRecordWithFlags(...,
 * hipEventRecordExternal)): a stream outside the graph can wait on a point INSIDE a replayed step -- the
 * data-parallel step starts the all-reduce of the gradient rows that are final at that point (the sqrt_W /
 * sqrt_U rows after the L-bar products) while the rest of the backward still runs (SURVEY §8e axis 2; the
 * reference's loss.backward(); optimizer.step(), code/nmgp_dsvi.py:847-854, has no such overlap).  Outside a
 * capture the record is a plain event record.  Handles are opaque (hipEvent_t, timing disabled).         */
int nmgp_event_create(void** event_out);
int nmgp_event_destroy(void* event);
int nmgp_event_record_external(void* event, hipStream_t stream);
int nmgp_stream_wait_event(hipStream_t stream, void* event);

#ifdef __cplusplus
}
#endif
#endif /* NMGP_HIP_H */
