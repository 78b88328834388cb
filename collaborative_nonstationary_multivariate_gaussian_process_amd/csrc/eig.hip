// Symmetric eigensolver (parallel cyclic Jacobi) for the Kronecker-structured Gaussian algebra of the
// legacy path: torch.symeig(B) / torch.symeig(K) in kron_inv / kron_logdet
// (code/SIM_code/Utility/kronecker_operation.py:45,47,66,67) and multivariate_normal_logpdf0/1
// (code/SIM_code/Utility/distributions.py:37,40,67,70).  f64 (settings.torchType = DoubleTensor).
//
//   n <= 64 : one workgroup per matrix, A and V resident in LDS.  Each sweep runs the n-1 rounds of
//             the circle (round-robin) ordering; a round rotates n/2 disjoint (p, q) pairs at once:
//             parameters (one lane per pair), row update, column update (+ V), barriers between.
//             Sweeps stop when a whole sweep rotates nothing (|a_pq| below the relative threshold).
//   n > 64  : block Jacobi on 32-wide column blocks padded to a multiple of 64.  A round pairs the
//             blocks (circle ordering); every pair's 64x64 sub-problem [[A_II A_IJ][A_JI A_JJ]] is
//             diagonalised in LDS by the kernel above (its rotations accumulated into Q_IJ), then
//             A <- Q^T A Q on the paired row blocks and column blocks and V <- V Q, as 64x64 panel
//             products staged through LDS.  Convergence: the sweep's sum of ||A_IJ||_F^2 taken
//             before each pair is annihilated, against tol^2 ||A||_F^2 (a device flag; later
//             launches of a finished solve return at entry, so the whole solve is asynchronous and
//             graph-capturable).  Padding: extra diagonal entries of value ||A||_F + 1 with zero
//             coupling are never rotated and sort last.
//   Output: eigenvalues ascending (as torch.linalg.eigh / symeig) and eigenvectors as columns of V.
#include "common.hpp"

namespace nmgp {

constexpr int EJ_N = 64, EJ_P = 65, EJ_BLK = 32;

__device__ inline void circle_pair(int np, int r, int k, int& a, int& b) {
  const int m = np - 1;
  if (k == 0) {
    a = r % m;
    b = m;
  } else {
    a = (r + k) % m;
    b = (r - k + m) % m;
  }
  if (a > b) {
    const int t = a;
    a = b;
    b = t;
  }
}

// Jacobi sweeps on the np x np (np even, <= 64) matrix in As, rotations accumulated into Vs.
__device__ void jacobi_lds(double* As, double* Vs, int np, int max_sweeps, double abs_tol, double* rot, int* flag) {
  const int t = threadIdx.x, half = np >> 1;
  for (int sw = 0; sw < max_sweeps; ++sw) {
    if (t == 0) *flag = 0;
    __syncthreads();
    for (int r = 0; r < np - 1; ++r) {
      if (t < half) {
        int p, q;
        circle_pair(np, r, t, p, q);
        const double app = As[p * EJ_P + p], aqq = As[q * EJ_P + q], apq = As[p * EJ_P + q];
        double c = 1.0, s = 0.0;
        const double thr = fmax(2.2e-16 * sqrt(fabs(app * aqq)), abs_tol);
        if (fabs(apq) > thr) {
          const double tau = (aqq - app) / (2.0 * apq);
          const double tt = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
          c = 1.0 / sqrt(1.0 + tt * tt);
          s = tt * c;
          *flag = 1;
        }
        rot[2 * t] = c;
        rot[2 * t + 1] = s;
      }
      __syncthreads();
      for (int idx = t; idx < half * np; idx += blockDim.x) {   // rows p, q  <-  J^T A
        const int k = idx / np, j = idx - k * np;
        const double s = rot[2 * k + 1];
        if (s != 0.0) {
          int p, q;
          circle_pair(np, r, k, p, q);
          const double c = rot[2 * k];
          const double ap = As[p * EJ_P + j], aq = As[q * EJ_P + j];
          As[p * EJ_P + j] = c * ap - s * aq;
          As[q * EJ_P + j] = s * ap + c * aq;
        }
      }
      __syncthreads();
      for (int idx = t; idx < half * np; idx += blockDim.x) {   // columns p, q  <-  A J, V J
        const int i = idx / half, k = idx - i * half;
        const double s = rot[2 * k + 1];
        if (s != 0.0) {
          int p, q;
          circle_pair(np, r, k, p, q);
          const double c = rot[2 * k];
          const double ap = As[i * EJ_P + p], aq = As[i * EJ_P + q];
          As[i * EJ_P + p] = c * ap - s * aq;
          As[i * EJ_P + q] = s * ap + c * aq;
          const double vp = Vs[i * EJ_P + p], vq = Vs[i * EJ_P + q];
          Vs[i * EJ_P + p] = c * vp - s * vq;
          Vs[i * EJ_P + q] = s * vp + c * vq;
        }
      }
      __syncthreads();
    }
    if (*flag == 0) break;
    __syncthreads();
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------- direct path (n <= 64)
__global__ __launch_bounds__(256) void syevj_small_kernel(const double* A, int n, int64_t lda, int64_t sA, double* W,
                                                          int64_t sW, double* V, int64_t ldv, int64_t sV,
                                                          int max_sweeps) {
  extern __shared__ double ej_smem[];   // As, Vs (64 x 65 each), rot, red, wv: > 64 KB, dynamic
  double *As = ej_smem, *Vs = As + EJ_N * EJ_P, *rot = Vs + EJ_N * EJ_P, *red = rot + EJ_N, *wv = red + 16;
  __shared__ int flag;
  const int t = threadIdx.x;
  const int np = n + (n & 1);
  const double* Am = A + blockIdx.x * sA;
  double fro = 0.0;
  for (int idx = t; idx < np * np; idx += blockDim.x) {
    const int i = idx / np, j = idx - i * np;
    const double a = (i < n && j < n) ? Am[(int64_t)i * lda + j] : 0.0;
    As[i * EJ_P + j] = a;
    Vs[i * EJ_P + j] = (i == j) ? 1.0 : 0.0;
    fro += a * a;
  }
  fro = sqrt(block_sum(fro, red));
  if (np != n && t == 0) As[n * EJ_P + n] = fro + 1.0;   // padding row: decoupled, sorts last
  __syncthreads();
  jacobi_lds(As, Vs, np, max_sweeps, 1e-300, rot, &flag);
  if (t < np) wv[t] = As[t * EJ_P + t];
  __syncthreads();
  // ascending order by rank (ties by index); the padding sorts last and is dropped
  double* Wm = W + blockIdx.x * sW;
  double* Vm = V + blockIdx.x * sV;
  for (int i = t; i < n; i += blockDim.x) {
    const double w = wv[i];
    int rank = 0;
    for (int j = 0; j < np; ++j) rank += (wv[j] < w) || (wv[j] == w && j < i);
    Wm[rank] = w;
    for (int r = 0; r < n; ++r) Vm[(int64_t)r * ldv + rank] = Vs[r * EJ_P + i];
  }
}

// ---------------------------------------------------------------------------- block path (n > 64)
struct EigWs {
  double* Ap;     // np x np working matrix
  double* Vp;     // np x np eigenvectors
  double* Q;      // (nb/2) x 64 x 64 rotations of the current round
  double* off;    // per sweep: (nb-1) x nb/2 slots of ||A_IJ||_F^2
  double* scal;   // [0] = ||A||_F^2, [1] = last sweep's off
  int* conv;      // [0] = converged flag, [1] = sweeps run
  int* rank;      // np
};

__global__ __launch_bounds__(256) void eig_init_kernel(const double* A, int n, int64_t lda, EigWs w, int np) {
  __shared__ double red[16];
  const int t = threadIdx.x;
  double fro = 0.0;
  for (int64_t idx = t; idx < (int64_t)n * n; idx += blockDim.x) {
    const int64_t i = idx / n, j = idx - i * n;
    const double a = A[i * lda + j];
    fro += a * a;
  }
  fro = block_sum(fro, red);
  if (t == 0) {
    w.scal[0] = fro;
    w.scal[1] = 0.0;
    w.conv[0] = 0;
    w.conv[1] = 0;
  }
  const double pad = sqrt(fro) + 1.0;
  for (int64_t idx = t; idx < (int64_t)np * np; idx += blockDim.x) {
    const int64_t i = idx / np, j = idx - i * np;
    w.Ap[idx] = (i < n && j < n) ? A[i * lda + j] : (i == j ? pad : 0.0);
    w.Vp[idx] = (i == j) ? 1.0 : 0.0;
  }
}

// one workgroup per block pair of round r: load the 64x64 sub-problem, record ||A_IJ||^2, diagonalise
__global__ __launch_bounds__(256) void eig_sub_kernel(EigWs w, int np, int r, int sweep_slot, int inner) {
  if (w.conv[0]) return;
  extern __shared__ double ej_smem[];
  double *As = ej_smem, *Vs = As + EJ_N * EJ_P, *rot = Vs + EJ_N * EJ_P, *red = rot + EJ_N;
  __shared__ int flag;
  const int t = threadIdx.x, k = blockIdx.x, nb = np / EJ_BLK;
  int I, J;
  circle_pair(nb, r, k, I, J);
  double offn = 0.0;
  for (int idx = t; idx < EJ_N * EJ_N; idx += blockDim.x) {
    const int i = idx >> 6, j = idx & 63;
    const int gi = i < EJ_BLK ? I * EJ_BLK + i : J * EJ_BLK + i - EJ_BLK;
    const int gj = j < EJ_BLK ? I * EJ_BLK + j : J * EJ_BLK + j - EJ_BLK;
    const double a = w.Ap[(int64_t)gi * np + gj];
    As[i * EJ_P + j] = a;
    Vs[i * EJ_P + j] = (i == j) ? 1.0 : 0.0;
    if ((i < EJ_BLK) != (j < EJ_BLK)) offn += a * a;
  }
  offn = block_sum(offn, red);
  if (t == 0) w.off[(int64_t)sweep_slot * (nb / 2) + k] = 0.5 * offn;
  const double abs_tol = 1e-17 * sqrt(w.scal[0]) / np;
  jacobi_lds(As, Vs, EJ_N, inner, abs_tol, rot, &flag);
  double* Qk = w.Q + (int64_t)k * EJ_N * EJ_N;
  for (int idx = t; idx < EJ_N * EJ_N; idx += blockDim.x) Qk[idx] = Vs[(idx >> 6) * EJ_P + (idx & 63)];
}

// rows:    A[R_k, c0:c0+64] <- Q_k^T A[R_k, c0:c0+64]         (grid: np/64 chunks x nb/2 pairs)
// columns: M[r0:r0+64, C_k] <- M[r0:r0+64, C_k] Q_k, M = A, V  (grid: np/64 chunks x nb/2 pairs x 2)
template <bool ROWS>
__global__ __launch_bounds__(256) void eig_apply_kernel(EigWs w, int np, int r) {
  if (w.conv[0]) return;
  extern __shared__ double ej_smem[];
  double *Qs = ej_smem, *Ps = Qs + EJ_N * EJ_P;
  const int t = threadIdx.x, c0 = blockIdx.x * EJ_N, k = blockIdx.y, nb = np / EJ_BLK;
  int I, J;
  circle_pair(nb, r, k, I, J);
  double* M = (ROWS || blockIdx.z == 0) ? w.Ap : w.Vp;
  const double* Qk = w.Q + (int64_t)k * EJ_N * EJ_N;
  for (int idx = t; idx < EJ_N * EJ_N; idx += blockDim.x) {
    const int i = idx >> 6, j = idx & 63;
    Qs[i * EJ_P + j] = Qk[idx];
    if (ROWS) {
      const int gi = i < EJ_BLK ? I * EJ_BLK + i : J * EJ_BLK + i - EJ_BLK;
      Ps[i * EJ_P + j] = M[(int64_t)gi * np + c0 + j];
    } else {
      const int gj = j < EJ_BLK ? I * EJ_BLK + j : J * EJ_BLK + j - EJ_BLK;
      Ps[i * EJ_P + j] = M[(int64_t)(c0 + i) * np + gj];
    }
  }
  __syncthreads();
  const int ty = t >> 4, tx = t & 15;
  double acc[4][4] = {};
  for (int kk = 0; kk < EJ_N; ++kk) {
    double a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = ROWS ? Qs[kk * EJ_P + ty * 4 + u] : Ps[(ty * 4 + u) * EJ_P + kk];
      b[u] = ROWS ? Ps[kk * EJ_P + tx * 4 + u] : Qs[kk * EJ_P + tx * 4 + u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[u][v] = fma(a[u], b[v], acc[u][v]);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = ty * 4 + u, j = tx * 4 + v;
      if (ROWS) {
        const int gi = i < EJ_BLK ? I * EJ_BLK + i : J * EJ_BLK + i - EJ_BLK;
        M[(int64_t)gi * np + c0 + j] = acc[u][v];
      } else {
        const int gj = j < EJ_BLK ? I * EJ_BLK + j : J * EJ_BLK + j - EJ_BLK;
        M[(int64_t)(c0 + i) * np + gj] = acc[u][v];
      }
    }
}

// end of a sweep: deterministic sum of the sweep's off-block norms -> converged flag
__global__ __launch_bounds__(256) void eig_check_kernel(EigWs w, int nslots, double tol2) {
  if (w.conv[0]) return;
  __shared__ double red[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < nslots; i += blockDim.x) s += w.off[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    w.scal[1] = s;
    w.conv[1] += 1;
    if (s <= tol2 * w.scal[0]) w.conv[0] = 1;
  }
}

__global__ __launch_bounds__(256) void eig_rank_kernel(EigWs w, int np, double* W, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  const double x = w.Ap[(int64_t)i * np + i];
  int rank = 0;
  for (int j = 0; j < np; ++j) {
    const double y = w.Ap[(int64_t)j * np + j];
    rank += (y < x) || (y == x && j < i);
  }
  w.rank[i] = rank;
  if (rank < n) W[rank] = x;
}

__global__ __launch_bounds__(256) void eig_permute_kernel(EigWs w, int np, int n, double* V, int64_t ldv) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)n * np) return;
  const int r = (int)(idx / np), i = (int)(idx - (int64_t)r * np);
  const int rk = w.rank[i];
  if (rk < n) V[(int64_t)r * ldv + rk] = w.Vp[(int64_t)r * np + i];
}

constexpr size_t kEjSmem = (2 * EJ_N * EJ_P + EJ_N + 16 + EJ_N) * sizeof(double);

static void eig_set_smem() {
  static bool done = false;
  if (done) return;
  (void)hipFuncSetAttribute((const void*)syevj_small_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kEjSmem);
  (void)hipFuncSetAttribute((const void*)eig_sub_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kEjSmem);
  (void)hipFuncSetAttribute((const void*)eig_apply_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)kEjSmem);
  (void)hipFuncSetAttribute((const void*)eig_apply_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)kEjSmem);
  done = true;
}

static int eig_np(int64_t n) { return (int)(((n + 63) / 64) * 64); }

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

static EigWs eig_carve(void* ws, int np) {
  const int nb = np / EJ_BLK;
  char* p = (char*)ws;
  EigWs w;
  w.Ap = (double*)p; p += align256((size_t)np * np * 8);
  w.Vp = (double*)p; p += align256((size_t)np * np * 8);
  w.Q = (double*)p; p += align256((size_t)(nb / 2) * EJ_N * EJ_N * 8);
  w.off = (double*)p; p += align256((size_t)(nb - 1) * (nb / 2) * 8);
  w.scal = (double*)p; p += 256;
  w.conv = (int*)p; p += 256;
  w.rank = (int*)p; p += align256((size_t)np * 4);
  return w;
}

size_t syevj_ws_bytes(int64_t n) {
  if (n <= EJ_N) return 0;
  const int np = eig_np(n), nb = np / EJ_BLK;
  return align256((size_t)np * np * 8) * 2 + align256((size_t)(nb / 2) * EJ_N * EJ_N * 8) +
         align256((size_t)(nb - 1) * (nb / 2) * 8) + 512 + align256((size_t)np * 4);
}

constexpr int kEigMaxSweeps = 20, kEigInner = 10;

static int syevj_block(const double* A, int n, int64_t lda, double* W, double* V, int64_t ldv, void* ws,
                       hipStream_t s) {
  const int np = eig_np(n), nb = np / EJ_BLK;
  EigWs w = eig_carve(ws, np);
  hipLaunchKernelGGL(eig_init_kernel, dim3(1), dim3(256), 0, s, A, n, lda, w, np);
  NMGP_CHECK_LAUNCH();
  const double tol2 = 1e-30;   // (1e-15)^2: ||off||_F <= 1e-15 ||A||_F
  for (int sw = 0; sw < kEigMaxSweeps; ++sw) {
    for (int r = 0; r < nb - 1; ++r) {
      hipLaunchKernelGGL(eig_sub_kernel, dim3(nb / 2), dim3(256), kEjSmem, s, w, np, r, r, kEigInner);
      hipLaunchKernelGGL(eig_apply_kernel<true>, dim3(np / EJ_N, nb / 2), dim3(256), kEjSmem, s, w, np, r);
      hipLaunchKernelGGL(eig_apply_kernel<false>, dim3(np / EJ_N, nb / 2, 2), dim3(256), kEjSmem, s, w, np, r);
      NMGP_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(eig_check_kernel, dim3(1), dim3(256), 0, s, w, (nb - 1) * (nb / 2), tol2);
    NMGP_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(eig_rank_kernel, dim3((np + 255) / 256), dim3(256), 0, s, w, np, W, n);
  hipLaunchKernelGGL(eig_permute_kernel, dim3((unsigned)(((int64_t)n * np + 255) / 256)), dim3(256), 0, s, w, np, n, V,
                     ldv);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

static int syevj_launch(const double* A, int64_t n, int64_t lda, int64_t sA, int64_t batch, double* W, int64_t sW,
                        double* V, int64_t ldv, int64_t sV, void* ws, int64_t ws_bytes, hipStream_t s) {
  if (A == nullptr) return -1;
  if (n < 0) return -2;
  if (lda < n) return -3;
  if (batch < 0 || batch > 65535) return -5;
  if (W == nullptr) return -6;
  if (V == nullptr) return -8;
  if (ldv < n) return -9;
  if (n == 0 || batch == 0) return NMGP_OK;
  eig_set_smem();
  if (n <= EJ_N) {
    hipLaunchKernelGGL(syevj_small_kernel, dim3((unsigned)batch), dim3(256), kEjSmem, s, A, (int)n, lda, sA, W, sW, V, ldv, sV,
                       30);
    NMGP_CHECK_LAUNCH();
    return NMGP_OK;
  }
  if (ws == nullptr || ws_bytes < (int64_t)syevj_ws_bytes(n)) return -11;
  for (int64_t b = 0; b < batch; ++b) {
    const int rc = syevj_block(A + b * sA, (int)n, lda, W + b * sW, V + b * sV, ldv, ws, s);
    if (rc != NMGP_OK) return rc;
  }
  return NMGP_OK;
}

}  // namespace nmgp

extern "C" {
int64_t nmgp_syevj_workspace_size_f64(int64_t n) { return (int64_t)nmgp::syevj_ws_bytes(n); }
int nmgp_syevj_batched_f64(const double* A, int64_t n, int64_t lda, int64_t sA, int64_t batch, double* W, int64_t sW,
                           double* V, int64_t ldv, int64_t sV, void* ws, int64_t ws_bytes, hipStream_t s) {
  return nmgp::syevj_launch(A, n, lda, sA, batch, W, sW, V, ldv, sV, ws, ws_bytes, s);
}
}
