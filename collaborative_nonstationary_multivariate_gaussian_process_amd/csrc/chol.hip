// Batched blocked Cholesky (potrf) and triangular inverse (trtri), one workgroup per matrix.
//
// Replaces torch.cholesky / torch.solve on the M x M SPD matrices of the DSVI step
// (code/utils.py:46,119,276,347-348): the 4 priors K22 + 1e-4 I and the D+1+Q variational
// covariances tril(S) tril(S)^T + 1e-4 I (code/nmgp_dsvi.py:172-177, KL at :266-295).
//
// Right-looking, 16-wide blocks:
//   phase 1  (wave 0)   the 16x16 diagonal block is factored (and inverted) in registers with
//                       wave shuffles: lane l holds row l&15, columns (l>>4)+4r  -- no LDS,
//                       no barriers inside the block;
//   phase 2  (4 waves)  panel  L[ib,kb] = A[ib,kb] * Lkk^-T  on the matrix cores, staged in LDS;
//   phase 3  (4 waves)  trailing SYRK A[ib,jb] -= L[ib,kb] L[jb,kb]^T, one 16x16 MFMA tile per
//                       wave step, operands from the LDS panel.
// trtri runs the same three phases on L X = I (X = L^-1), block row by block row.
#include "common.hpp"

namespace nmgp {

constexpr int CP = 17;  // LDS pitch (elements) of the 16-wide panel: conflict-free ds_read_b64

// Factor the 16x16 diagonal block held in a[4] (lane l: row l&15, col (l>>4)+4r) in place and
// return its inverse in x[4] (same layout). fail gets the 1-based first bad pivot, or 0.
template <typename T>
__device__ inline void chol16(T (&a)[4], T (&x)[4], int lane, int col0, int n, int& fail) {
  const int i = lane & 15;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int grp = j & 3, q = j >> 2;
    const T ajj = shfl(a[q], j + 16 * grp);
    if (!(ajj > (T)0) && fail == 0 && col0 + j < n) fail = col0 + j + 1;
    const T ljj = dsqrt(ajj);
    const T inv = (T)1 / ljj;
    if ((lane >> 4) == grp) a[q] = (i == j) ? ljj : (i > j ? a[q] * inv : (T)0);
    const T lij = shfl(a[q], i + 16 * grp);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = (lane >> 4) + 4 * r;
      const T lcj = shfl(a[q], c + 16 * grp);
      if (c > j && c <= i) a[r] -= lij * lcj;
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = (lane >> 4) + 4 * r;
    if (c > i) a[r] = 0;
  }
}

// x = inverse of the lower-triangular 16x16 block in a (same layout).
template <typename T>
__device__ inline void trinv16(const T (&a)[4], T (&x)[4], int lane) {
  const int i = lane & 15;
#pragma unroll
  for (int r = 0; r < 4; ++r) x[r] = (i == (lane >> 4) + 4 * r) ? (T)1 : (T)0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int grp = j & 3, q = j >> 2;
    const T ljj = shfl(a[q], j + 16 * grp);
    const T inv = (T)1 / ljj;
    if (i == j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) x[r] *= inv;
    }
    const T lij = shfl(a[q], i + 16 * grp);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const T xjc = shfl(x[r], j + (lane & 0x30));
      if (i > j) x[r] -= lij * xjc;
    }
  }
}

__device__ inline void tri_decode(int tt, int& a, int& b) {
  int r = (int)((sqrtf(8.0f * (float)tt + 1.0f) - 1.0f) * 0.5f);
  while ((r + 1) * (r + 2) / 2 <= tt) ++r;
  while (r * (r + 1) / 2 > tt) --r;
  a = r;
  b = tt - r * (r + 1) / 2;
}

template <typename T>
__global__ __launch_bounds__(256) void potrf_kernel(T* A, int n, int64_t lda, int64_t strideA, int32_t* info) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int nt = (n + 15) >> 4;
  T* Linv = (T*)smem_raw;          // 16 x CP
  T* Ps = Linv + 16 * CP;          // (nt*16) x CP  panel
  int* s_fail = (int*)(Ps + nt * 16 * CP);
  T* Am = A + (int64_t)blockIdx.x * strideA;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) *s_fail = 0;
  __syncthreads();
  for (int kb = 0; kb < nt; ++kb) {
    if (w == 0) {
      const int i = lane & 15;
      const int gi = kb * 16 + i;
      T a[4], x[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gc = kb * 16 + (lane >> 4) + 4 * r;
        a[r] = (gi < n && gc < n) ? Am[(int64_t)gi * lda + gc] : (gi == gc ? (T)1 : (T)0);
      }
      int fail = 0;
      chol16(a, x, lane, kb * 16, n, fail);
      trinv16(a, x, lane);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = (lane >> 4) + 4 * r;
        const int gc = kb * 16 + c;
        if (gi < n && gc < n) Am[(int64_t)gi * lda + gc] = a[r];
        Linv[i * CP + c] = x[r];
      }
      if (lane == 0 && fail && *s_fail == 0) *s_fail = fail;
    }
    __syncthreads();
    // phase 2: panel below the diagonal block
    for (int ib = kb + 1 + w; ib < nt; ib += 4) {
      typename Mfma<T>::acc_t acc = {0, 0, 0, 0};
      const int gi = ib * 16 + (lane & 15);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int kr = 4 * s + (lane >> 4);
        const int gk = kb * 16 + kr;
        const T av = (gi < n && gk < n) ? Am[(int64_t)gi * lda + gk] : (T)0;
        const T bv = Linv[(lane & 15) * CP + kr];
        acc = Mfma<T>::mma(av, bv, acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = Mfma<T>::row(lane, r), col = lane & 15;
        const int gr = ib * 16 + row, gc = kb * 16 + col;
        if (gr < n && gc < n) Am[(int64_t)gr * lda + gc] = acc[r];
        Ps[(ib * 16 + row) * CP + col] = acc[r];
      }
    }
    __syncthreads();
    // phase 3: trailing lower-triangular update
    const int S = nt - kb - 1;
    const int ntile = S * (S + 1) / 2;
    for (int tt = w; tt < ntile; tt += 4) {
      int ibo, jbo;
      tri_decode(tt, ibo, jbo);
      const int ib = kb + 1 + ibo, jb = kb + 1 + jbo;
      typename Mfma<T>::acc_t acc;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = ib * 16 + Mfma<T>::row(lane, r), gc = jb * 16 + (lane & 15);
        acc[r] = (gr < n && gc < n) ? Am[(int64_t)gr * lda + gc] : (T)0;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int kr = 4 * s + (lane >> 4);
        const T av = Ps[(ib * 16 + (lane & 15)) * CP + kr];
        const T bv = Ps[(jb * 16 + (lane & 15)) * CP + kr];
        acc = Mfma<T>::mma(-av, bv, acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = ib * 16 + Mfma<T>::row(lane, r), gc = jb * 16 + (lane & 15);
        if (gr < n && gc < n) Am[(int64_t)gr * lda + gc] = acc[r];
      }
    }
    __syncthreads();
  }
  for (int64_t idx = t; idx < (int64_t)n * n; idx += blockDim.x) {
    const int i = (int)(idx / n), j = (int)(idx - (int64_t)i * n);
    if (j > i) Am[(int64_t)i * lda + j] = 0;
  }
  if (t == 0 && info) info[blockIdx.x] = *s_fail;
}

template <typename T>
__global__ __launch_bounds__(256) void trtri_kernel(const T* L, int n, int64_t ldl, int64_t strideL, T* X, int64_t ldx,
                                                    int64_t strideX) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int nt = (n + 15) >> 4;
  T* Li = (T*)smem_raw;       // 16 x CP
  T* Xrow = Li + 16 * CP;     // nt tiles of 16x16 (row-major, pitch 16)
  const T* Lm = L + (int64_t)blockIdx.x * strideL;
  T* Xm = X + (int64_t)blockIdx.x * strideX;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int64_t idx = t; idx < (int64_t)n * n; idx += blockDim.x) {
    const int i = (int)(idx / n), j = (int)(idx - (int64_t)i * n);
    Xm[(int64_t)i * ldx + j] = 0;
  }
  __syncthreads();
  for (int kb = 0; kb < nt; ++kb) {
    if (w == 0) {
      const int i = lane & 15, gi = kb * 16 + i;
      T a[4], x[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gc = kb * 16 + (lane >> 4) + 4 * r;
        a[r] = (gi < n && gc < n && gc <= gi) ? Lm[(int64_t)gi * ldl + gc] : (gi == gc ? (T)1 : (T)0);
      }
      trinv16(a, x, lane);
#pragma unroll
      for (int r = 0; r < 4; ++r) Li[i * CP + (lane >> 4) + 4 * r] = x[r];
    }
    __syncthreads();
    for (int jb = w; jb <= kb; jb += 4) {
      typename Mfma<T>::acc_t acc = {0, 0, 0, 0};
      if (jb == kb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = Li[Mfma<T>::row(lane, r) * CP + (lane & 15)];
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int kr = 4 * s + (lane >> 4);
          const int gk = kb * 16 + kr, gj = jb * 16 + (lane & 15);
          const T av = Li[(lane & 15) * CP + kr];
          const T bv = (gk < n && gj < n) ? Xm[(int64_t)gk * ldx + gj] : (T)0;
          acc = Mfma<T>::mma(av, bv, acc);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = Mfma<T>::row(lane, r), col = lane & 15;
        const int gr = kb * 16 + row, gc = jb * 16 + col;
        if (gr < n && gc < n) Xm[(int64_t)gr * ldx + gc] = acc[r];
        Xrow[(jb * 16 + row) * 16 + col] = acc[r];
      }
    }
    __syncthreads();
    const int nr = nt - kb - 1, nc = kb + 1;
    for (int tt = w; tt < nr * nc; tt += 4) {
      const int ib = kb + 1 + tt / nc, jb = tt % nc;
      typename Mfma<T>::acc_t acc;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = ib * 16 + Mfma<T>::row(lane, r), gc = jb * 16 + (lane & 15);
        acc[r] = (gr < n && gc < n) ? Xm[(int64_t)gr * ldx + gc] : (T)0;
      }
      const int gi = ib * 16 + (lane & 15);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int kr = 4 * s + (lane >> 4);
        const int gk = kb * 16 + kr;
        const T av = (gi < n && gk < n) ? Lm[(int64_t)gi * ldl + gk] : (T)0;
        const T bv = Xrow[(jb * 16 + kr) * 16 + (lane & 15)];
        acc = Mfma<T>::mma(-av, bv, acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = ib * 16 + Mfma<T>::row(lane, r), gc = jb * 16 + (lane & 15);
        if (gr < n && gc < n) Xm[(int64_t)gr * ldx + gc] = acc[r];
      }
    }
    __syncthreads();
  }
}

template <typename T> static size_t potrf_smem(int n) {
  const int nt = (n + 15) >> 4;
  return (size_t)(16 * CP + nt * 16 * CP) * sizeof(T) + 16;
}
template <typename T> static size_t trtri_smem(int n) {
  const int nt = (n + 15) >> 4;
  return (size_t)(16 * CP + nt * 256) * sizeof(T);
}

template <typename T>
static int potrf_launch(T* A, int64_t n, int64_t lda, int64_t strideA, int64_t batch, int32_t* info, hipStream_t s) {
  if (A == nullptr) return -1;
  if (n < 0) return -2;
  if (lda < n) return -3;
  if (batch < 0) return -5;
  if (n == 0 || batch == 0) return NMGP_OK;
  const size_t sm = potrf_smem<T>((int)n);
  if (sm > 160 * 1024) return -2;
  static bool attr_done = false;
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)potrf_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_done = true;
  }
  hipLaunchKernelGGL(potrf_kernel<T>, dim3((unsigned)batch), dim3(256), sm, s, A, (int)n, lda, strideA, info);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

template <typename T>
static int trtri_launch(const T* L, int64_t n, int64_t ldl, int64_t strideL, T* X, int64_t ldx, int64_t strideX,
                        int64_t batch, hipStream_t s) {
  if (L == nullptr) return -1;
  if (n < 0) return -2;
  if (ldl < n) return -3;
  if (X == nullptr) return -5;
  if (ldx < n) return -6;
  if (batch < 0) return -8;
  if (n == 0 || batch == 0) return NMGP_OK;
  const size_t sm = trtri_smem<T>((int)n);
  if (sm > 160 * 1024) return -2;
  static bool attr_done = false;
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)trtri_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_done = true;
  }
  hipLaunchKernelGGL(trtri_kernel<T>, dim3((unsigned)batch), dim3(256), sm, s, L, (int)n, ldl, strideL, X, ldx,
                     strideX);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

}  // namespace nmgp

extern "C" {
int nmgp_potrf_batched_f64(double* A, int64_t n, int64_t lda, int64_t sA, int64_t b, int32_t* info, hipStream_t s) {
  return nmgp::potrf_launch<double>(A, n, lda, sA, b, info, s);
}
int nmgp_potrf_batched_f32(float* A, int64_t n, int64_t lda, int64_t sA, int64_t b, int32_t* info, hipStream_t s) {
  return nmgp::potrf_launch<float>(A, n, lda, sA, b, info, s);
}
int nmgp_trtri_batched_f64(const double* L, int64_t n, int64_t ldl, int64_t sL, double* X, int64_t ldx, int64_t sX,
                           int64_t b, hipStream_t s) {
  return nmgp::trtri_launch<double>(L, n, ldl, sL, X, ldx, sX, b, s);
}
int nmgp_trtri_batched_f32(const float* L, int64_t n, int64_t ldl, int64_t sL, float* X, int64_t ldx, int64_t sX,
                           int64_t b, hipStream_t s) {
  return nmgp::trtri_launch<float>(L, n, ldl, sL, X, ldx, sX, b, s);
}
}
