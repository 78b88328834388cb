// Kronecker-structured covariance kernels (SIM_code/Utility/kronecker_operation.py:5-85).
//   kronecker_product       out[(i*r2+k), (j*c2+l)] = t1[i,j] * t2[k,l]   -- one multiply per
//                           element in the reference's operand order, so results are bit-exact;
//                           each thread writes 4 consecutive elements of one output row.
//   kronecker_product_diag  out[i*n2+k] = d1[i] * d2[k]
//   kron_mv                 (B kron K) y without forming B kron K: Y = y.view(P2,N2)^T,
//                           A = (K Y) B^T on the matrix cores (two GEMMs), out = vec(A^T) in the
//                           reference's reshape order (bit-exact index mapping).
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

template <typename T>
static int kron_mv(const T* B, int64_t P1, int64_t P2, const T* K, int64_t N1, int64_t N2, const T* y, T* out, T* work,
                   hipStream_t s, int (*gemm)(const nmgp_gemm_desc*, const int32_t*, hipStream_t)) {
  if (!B) return -1;
  if (!K) return -4;
  if (!y) return -7;
  if (!out) return -8;
  if (!work) return -9;
  if (P1 == 0 || N1 == 0) return NMGP_OK;
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
