// Kronecker-structured covariance kernels (SIM_code/Utility/kronecker_operation.py:5-85).
//   kronecker_product       out[(i*r2+k), (j*c2+l)] = t1[i,j] * t2[k,l]   -- one multiply per
//                           element in the reference's operand order, so results are bit-exact;
//                           each thread writes 4 consecutive elements of one output row.
//   kronecker_product_diag  out[i*n2+k] = d1[i] * d2[k]
//   kron_mv                 (B kron K) y without forming B kron K: Y = y.view(P2,N2)^T, A = (K Y) B^T,
//                           out = vec(A^T) in the reference's reshape order (bit-exact index mapping).
//                           P2 <= 8 (the legacy likelihood's few outputs): ONE pass over K (round 4,
//                           kron_mv_kernel below) -- the HBM-bound case; wider B: two MFMA GEMMs.
#include "common.hpp"

namespace nmgp {

template <typename T>
__global__ void kron_product_kernel(const T* t1, int64_t r1, int64_t c1, const T* t2, int64_t r2, int64_t c2, T* out) {
  const int64_t cols = c1 * c2, rows = r1 * r2;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per_row = (cols + 3) / 4;
  const int64_t row = q / per_row;
  if (row >= rows) return;
  const int64_t c0 = (q - row * per_row) * 4;
  const int64_t i = row / r2, k = row - i * r2;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t col = c0 + e;
    if (col >= cols) break;
    const int64_t j = col / c2, l = col - j * c2;
    out[row * cols + col] = t1[i * c1 + j] * t2[k * c2 + l];
  }
}

template <typename T>
static int kron_product(const T* t1, int64_t r1, int64_t c1, const T* t2, int64_t r2, int64_t c2, T* out,
                        hipStream_t s) {
  if (!t1) return -1;
  if (!t2) return -4;
  if (!out) return -7;
  if (r1 < 0 || c1 < 0 || r2 < 0 || c2 < 0) return -2;
  const int64_t rows = r1 * r2, cols = c1 * c2;
  if (rows == 0 || cols == 0) return NMGP_OK;
  const int64_t nq = rows * ((cols + 3) / 4);
  hipLaunchKernelGGL(kron_product_kernel<T>, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, t1, r1, c1, t2, r2,
                     c2, out);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

// Fused Kronecker mat-vec for small P2 (the legacy likelihood: B is P x P over a few outputs, K is N x N).
// Each wave owns KR consecutive rows n of K and streams them once from HBM in 16-byte loads (lanes over k);
// y's P2 rows are re-read from L2 for every KR rows (KR-fold reuse).  Per lane: KR x P2 partial sums of
// work[n, m] = sum_k K[n,k] y[m N2 + k]; a DPP wave reduction (common.hpp wave_sum) completes them in every
// lane, and lane p < P1 writes out[p N1 + n] = sum_m B[p,m] work[n,m] -- the second GEMM in registers.
// Bound: HBM, N1 N2 s bytes of K (+ y, B, out: P2 N2 + P1 P2 + P1 N1 elements).
constexpr int KMV_MAXP = 8;   // P2 limit of the fused path
constexpr int KMV_ROWS = 4;   // rows of K per wave

template <typename T, int V>
__global__ __launch_bounds__(256) void kron_mv_kernel(const T* __restrict__ B, int P1, int P2, const T* __restrict__ K,
                                                      int N1, int N2, const T* __restrict__ y, T* __restrict__ out) {
  struct alignas(sizeof(T) * V) Vec { T e[V]; };
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int n0 = wave * KMV_ROWS;
  if (n0 >= N1) return;
  T acc[KMV_ROWS][KMV_MAXP];
#pragma unroll
  for (int r = 0; r < KMV_ROWS; ++r)
#pragma unroll
    for (int m = 0; m < KMV_MAXP; ++m) acc[r][m] = (T)0;
  const int nv = N2 / V;
  for (int kv = lane; kv < nv; kv += 64) {
    Vec kr[KMV_ROWS];
#pragma unroll
    for (int r = 0; r < KMV_ROWS; ++r) {
      const int n = min(n0 + r, N1 - 1);                      // (rows past N1 duplicate the last row; unused)
      kr[r] = *(const Vec*)(K + (int64_t)n * N2 + (int64_t)kv * V);
    }
#pragma unroll
    for (int m = 0; m < KMV_MAXP; ++m) {
      if (m < P2) {
        const Vec yv = *(const Vec*)(y + (int64_t)m * N2 + (int64_t)kv * V);
#pragma unroll
        for (int r = 0; r < KMV_ROWS; ++r)
#pragma unroll
          for (int e = 0; e < V; ++e) acc[r][m] = fma(kr[r].e[e], yv.e[e], acc[r][m]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < KMV_ROWS; ++r)
#pragma unroll
    for (int m = 0; m < KMV_MAXP; ++m)
      if (m < P2) acc[r][m] = wave_sum(acc[r][m]);
  // the second stage: lanes p < P1 (strided over P1 > 64) form out[p N1 + n]
  for (int p = lane; p < P1; p += 64) {
#pragma unroll
    for (int r = 0; r < KMV_ROWS; ++r) {
      const int n = n0 + r;
      if (n >= N1) break;
      T o = (T)0;
#pragma unroll
      for (int m = 0; m < KMV_MAXP; ++m)
        if (m < P2) o = fma(B[(int64_t)p * P2 + m], acc[r][m], o);
      out[(int64_t)p * N1 + n] = o;
    }
  }
}

template <typename T>
static int kron_mv(const T* B, int64_t P1, int64_t P2, const T* K, int64_t N1, int64_t N2, const T* y, T* out, T* work,
                   hipStream_t s, int (*gemm)(const nmgp_gemm_desc*, const int32_t*, hipStream_t)) {
  if (!B) return -1;
  if (!K) return -4;
  if (!y) return -7;
  if (!out) return -8;
  if (P1 == 0 || N1 == 0) return NMGP_OK;
  if (P2 >= 1 && P2 <= KMV_MAXP && N2 >= 1 && N1 < (1LL << 30) && N2 < (1LL << 30)) {
    const unsigned grid = (unsigned)((N1 + 4 * KMV_ROWS - 1) / (4 * KMV_ROWS));
    constexpr int V = 16 / (int)sizeof(T);
    const bool vec = N2 % V == 0 && ((uintptr_t)K & 15) == 0 && ((uintptr_t)y & 15) == 0;
    if (vec)
      hipLaunchKernelGGL((kron_mv_kernel<T, V>), dim3(grid), dim3(256), 0, s, B, (int)P1, (int)P2, K, (int)N1, (int)N2,
                         y, out);
    else
      hipLaunchKernelGGL((kron_mv_kernel<T, 1>), dim3(grid), dim3(256), 0, s, B, (int)P1, (int)P2, K, (int)N1, (int)N2,
                         y, out);
    NMGP_CHECK_LAUNCH();
    return NMGP_OK;
  }
  if (!work) return -9;
  // work(n, m) = sum_k K[n,k] * y[m*N2 + k]        (N1 x P2)
  nmgp_gemm_desc d{};
  d.A = K; d.B = y; d.C = work;
  d.sA_i = N2; d.sA_k = 1; d.sB_k = 1; d.sB_j = N2; d.sC_i = P2; d.sC_j = 1;
  d.m = (int)N1; d.n = (int)P2; d.k = (int)N2; d.row_seg = -1; d.k_seg = -1;
  d.alpha = 1.0;
  int rc = gemm(&d, nullptr, s);
  if (rc) return rc;
  // out[p*N1 + n] = sum_m B[p,m] * work[n,m]        (P1 x N1)
  nmgp_gemm_desc e{};
  e.A = B; e.B = work; e.C = out;
  e.sA_i = P2; e.sA_k = 1; e.sB_k = 1; e.sB_j = P2; e.sC_i = N1; e.sC_j = 1;
  e.m = (int)P1; e.n = (int)N1; e.k = (int)P2; e.row_seg = -1; e.k_seg = -1;
  e.alpha = 1.0;
  return gemm(&e, nullptr, s);
}

}  // namespace nmgp

extern "C" {
int nmgp_kron_product_f64(const double* t1, int64_t r1, int64_t c1, const double* t2, int64_t r2, int64_t c2,
                          double* out, hipStream_t s) {
  return nmgp::kron_product<double>(t1, r1, c1, t2, r2, c2, out, s);
}
int nmgp_kron_product_f32(const float* t1, int64_t r1, int64_t c1, const float* t2, int64_t r2, int64_t c2,
                          float* out, hipStream_t s) {
  return nmgp::kron_product<float>(t1, r1, c1, t2, r2, c2, out, s);
}
int nmgp_kron_product_diag_f64(const double* d1, int64_t n1, const double* d2, int64_t n2, double* out,
                               hipStream_t s) {
  return nmgp::kron_product<double>(d1, n1, 1, d2, n2, 1, out, s);
}
int nmgp_kron_product_diag_f32(const float* d1, int64_t n1, const float* d2, int64_t n2, float* out,
                               hipStream_t s) {
  return nmgp::kron_product<float>(d1, n1, 1, d2, n2, 1, out, s);
}
int nmgp_kron_mv_f64(const double* B, int64_t P1, int64_t P2, const double* K, int64_t N1, int64_t N2,
                     const double* y, double* out, double* work, hipStream_t s) {
  return nmgp::kron_mv<double>(B, P1, P2, K, N1, N2, y, out, work, s, nmgp_gemm_f64);
}
int nmgp_kron_mv_f32(const float* B, int64_t P1, int64_t P2, const float* K, int64_t N1, int64_t N2, const float* y,
                     float* out, float* work, hipStream_t s) {
  return nmgp::kron_mv<float>(B, P1, P2, K, N1, N2, y, out, work, s, nmgp_gemm_f32);
}
}
