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
// One workgroup owns KMV_ROWS (4) consecutive rows n of K and its 256 threads walk those rows together in
// 16-byte loads (thread t takes vectors t, t + 256, ... of every row), two iterations in flight: per thread
// 2 x KMV_ROWS nontemporal K loads (K is streamed exactly once and must not evict y from L2) against P2 y
// loads shared by the KMV_ROWS rows.  Per thread KMV_ROWS x P2 partial sums of
// work[n, m] = sum_k K[n,k] y[m N2 + k]; DPP wave reductions (common.hpp wave_sum), then the four wave partials
// are added in wave order through LDS (deterministic), and the second GEMM out[p N1 + n] = sum_m B[p,m]
// work[n,m] runs on the threads of the block.  P2 is a template parameter so the accumulators are exactly
// KMV_ROWS x P2 registers.  Bound: HBM, N1 N2 s bytes of K (+ y, B, out: P2 N2 + P1 P2 + P1 N1 elements).
// 4 rows per workgroup: 2048 workgroups of <= 128 VGPRs fill the 1024 slots (occupancy 4) in two even rounds
// (8 rows: 1024 workgroups at occupancy 3, 1.33 rounds, 94-98 us against 92-96 us).  Round 5: the round-4 form (one wave per 4 rows, P2 up to 8 in a fixed-size accumulator, one iteration in
// flight, 512 workgroups) streamed K at 2.6 TB/s.
constexpr int KMV_MAXP = 8;   // P2 limit of the fused path
constexpr int KMV_ROWS = 4;   // rows of K per workgroup

template <typename T, int V, int P2>
__global__ __launch_bounds__(256) void kron_mv_kernel(const T* __restrict__ B, int P1, const T* __restrict__ K, int N1,
                                                      int N2, const T* __restrict__ y, T* __restrict__ out) {
  typedef T Vec __attribute__((ext_vector_type(V)));
  __shared__ T red[4][KMV_ROWS][P2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n0 = blockIdx.x * KMV_ROWS;
  const Vec* Kr[KMV_ROWS];
#pragma unroll
  for (int r = 0; r < KMV_ROWS; ++r)          // rows past N1 re-read the last row (results unused)
    Kr[r] = (const Vec*)(K + (int64_t)min(n0 + r, N1 - 1) * N2);
  const Vec* yv = (const Vec*)y;
  const int nv = N2 / V;                      // vectors per row (V divides N2 on the vector path)
  const int ys = nv;                          // y row m starts at vector m * nv
  T acc[KMV_ROWS][P2];
#pragma unroll
  for (int r = 0; r < KMV_ROWS; ++r)
#pragma unroll
    for (int m = 0; m < P2; ++m) acc[r][m] = (T)0;
  int kv = tid;
  for (; kv + 256 < nv; kv += 512) {          // two vectors per thread per iteration, all loads issued first
    Vec ka[KMV_ROWS], kb[KMV_ROWS], ya[P2], yb[P2];
#pragma unroll
    for (int r = 0; r < KMV_ROWS; ++r) {
      ka[r] = __builtin_nontemporal_load(Kr[r] + kv);
      kb[r] = __builtin_nontemporal_load(Kr[r] + kv + 256);
    }
#pragma unroll
    for (int m = 0; m < P2; ++m) {
      ya[m] = yv[(int64_t)m * ys + kv];
      yb[m] = yv[(int64_t)m * ys + kv + 256];
    }
#pragma unroll
    for (int r = 0; r < KMV_ROWS; ++r)
#pragma unroll
      for (int m = 0; m < P2; ++m) {
#pragma unroll
        for (int e = 0; e < V; ++e) acc[r][m] = fma(ka[r][e], ya[m][e], acc[r][m]);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[r][m] = fma(kb[r][e], yb[m][e], acc[r][m]);
      }
  }
  if (kv < nv) {                              // the odd last vector of this thread
    Vec ka[KMV_ROWS], ya[P2];
#pragma unroll
    for (int r = 0; r < KMV_ROWS; ++r) ka[r] = __builtin_nontemporal_load(Kr[r] + kv);
#pragma unroll
    for (int m = 0; m < P2; ++m) ya[m] = yv[(int64_t)m * ys + kv];
#pragma unroll
    for (int r = 0; r < KMV_ROWS; ++r)
#pragma unroll
      for (int m = 0; m < P2; ++m)
#pragma unroll
        for (int e = 0; e < V; ++e) acc[r][m] = fma(ka[r][e], ya[m][e], acc[r][m]);
  }
#pragma unroll
  for (int r = 0; r < KMV_ROWS; ++r)
#pragma unroll
    for (int m = 0; m < P2; ++m) {
      const T s = wave_sum(acc[r][m]);
      if (lane == 0) red[w][r][m] = s;
    }
  __syncthreads();
  // the second stage: thread (p, r) forms out[p N1 + n0 + r]; the wave partials are added in wave order
  for (int q = tid; q < P1 * KMV_ROWS; q += 256) {
    const int p = q / KMV_ROWS, r = q - p * KMV_ROWS;
    if (n0 + r >= N1) continue;
    T o = (T)0;
#pragma unroll
    for (int m = 0; m < P2; ++m) {
      const T wk = ((red[0][r][m] + red[1][r][m]) + red[2][r][m]) + red[3][r][m];
      o = fma(B[(int64_t)p * P2 + m], wk, o);
    }
    out[(int64_t)p * N1 + n0 + r] = o;
  }
}

template <typename T, int V>
static void kron_mv_fused(const T* B, int P1, int P2, const T* K, int N1, int N2, const T* y, T* out, hipStream_t s) {
  const dim3 grid((unsigned)((N1 + KMV_ROWS - 1) / KMV_ROWS)), blk(256);
  switch (P2) {
#define NMGP_KMV_CASE(P)                                                                              \
  case P:                                                                                             \
    hipLaunchKernelGGL((kron_mv_kernel<T, V, P>), grid, blk, 0, s, B, P1, K, N1, N2, y, out);         \
    break;
    NMGP_KMV_CASE(1) NMGP_KMV_CASE(2) NMGP_KMV_CASE(3) NMGP_KMV_CASE(4)
    NMGP_KMV_CASE(5) NMGP_KMV_CASE(6) NMGP_KMV_CASE(7) NMGP_KMV_CASE(8)
#undef NMGP_KMV_CASE
  }
}

template <typename T>
static int kron_mv(const T* B, int64_t P1, int64_t P2, const T* K, int64_t N1, int64_t N2, const T* y, T* out, T* work,
                   hipStream_t s, int (*gemm)(const nmgp_gemm_desc*, const int32_t*, hipStream_t)) {
  if (P1 < 0 || P2 < 0) return -2;
  if (N1 < 0 || N2 < 0) return -5;
  if (P1 == 0 || N1 == 0) return NMGP_OK;    // empty output
  if (!out) return -8;
  if (P2 == 0 || N2 == 0)                    // an empty contraction (B, K or y may be NULL): out = 0
    return hipMemsetAsync(out, 0, (size_t)(P1 * N1) * sizeof(T), s) == hipSuccess ? NMGP_OK : NMGP_ERR_LAUNCH;
  if (!B) return -1;
  if (!K) return -4;
  if (!y) return -7;
  if (P2 >= 1 && P2 <= KMV_MAXP && N1 < (1LL << 30) && N2 < (1LL << 30)) {
    constexpr int V = 16 / (int)sizeof(T);
    const bool vec = N2 % V == 0 && ((uintptr_t)K & 15) == 0 && ((uintptr_t)y & 15) == 0;
    if (vec)
      kron_mv_fused<T, V>(B, (int)P1, (int)P2, K, (int)N1, (int)N2, y, out, s);
    else
      kron_mv_fused<T, 1>(B, (int)P1, (int)P2, K, (int)N1, (int)N2, y, out, s);
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
