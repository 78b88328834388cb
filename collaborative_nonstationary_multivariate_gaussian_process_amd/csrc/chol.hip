// Batched blocked Cholesky (potrf) and triangular inverse (trtri), one workgroup per matrix.
//
// Replaces torch.cholesky / torch.solve on the M x M SPD matrices of the DSVI step
// (code/utils.py:46,119,276,347-348): the 4 priors K22 + 1e-4 I and the D+1+Q variational
// covariances tril(S) tril(S)^T + 1e-4 I (code/nmgp_dsvi.py:172-177, KL at :266-295).
//
// Right-looking, 16-wide blocks, 16 waves (1024 threads) per matrix:
//   phase 1  (wave 0)   the 16x16 diagonal block is factored in registers with wave shuffles:
//                       lane l holds row l&15, columns (l>>4)+4r -- no LDS, no barriers inside;
//   phase 2  (1 thread  panel  L[i,kb] = A[i,kb] L_kk^-T  by forward substitution, one thread per
//             per row)  row with L_kk broadcast from LDS, result staged in LDS;
//   phase 3  (16 waves) trailing SYRK A[ib,jb] -= L[ib,kb] L[jb,kb]^T on the matrix cores, four
//                       16x16 tiles in flight per wave so their global round trips overlap.
// trtri inverts all diagonal blocks first (one wave each, in parallel), then sweeps block rows:
// X[kb,:] = L_kk^-1 R[kb,:] and R[ib,:] -= L[ib,kb] X[kb,:] for ib > kb, again 4 tiles per wave.
#include "common.hpp"

#include <cstdlib>
#include <mutex>
#include <type_traits>

namespace nmgp {

constexpr int CP = 17;

#ifdef NMGP_CHOL_TRACE  // phase timestamps for tools/chol_probe.hip (never set in the library build)
__device__ unsigned long long* g_chol_trace;
#define CHOL_STAMP(kb, p) \
  if (threadIdx.x == 0 && blockIdx.x == 0) g_chol_trace[(kb) * 4 + (p)] = wall_clock64()
#define CHOL_STAMPW(kb, p) \
  if (threadIdx.x == 0 && blockIdx.x == 0) g_chol_trace[512 + (kb) * 4 + (p)] = wall_clock64()
#define CHOL_STAMP1(kb, p) \
  if (threadIdx.x == 0 && blockIdx.x == 1) g_chol_trace[256 + (kb) * 4 + (p)] = wall_clock64()
#define CHOL_STAMPX(i) \
  if (threadIdx.x == 0) g_chol_trace[1000 + 4 * blockIdx.x + (i)] = wall_clock64()
#define CHOL4_STAMP(role, k, ph) \
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 3) g_chol_trace[2048 + (role) * 512 + (k) * 8 + (ph)] = wall_clock64()
#else
#define CHOL4_STAMP(role, k, ph)
#define CHOL_STAMPX(i)
#define CHOL_STAMP1(kb, p)
#define CHOL_STAMP(kb, p)
#define CHOL_STAMPW(kb, p)
#endif  // LDS pitch (elements) of the 16-wide panel: conflict-free ds_read_b64

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

// 1024 threads (16 waves) per matrix.  Phase 3 work is issued in batches of 4 tiles per wave so
// four global round trips overlap; the panel is a row-wise forward substitution (one thread per
// row, L_kk broadcast from LDS) instead of a diagonal-block inverse + MFMA.
constexpr int CW = 16;         // waves per workgroup
constexpr int CT = CW * 64;     // threads

template <typename T>
__global__ __launch_bounds__(CT) void potrf_kernel(T* A, int n, int64_t lda, int64_t strideA, int32_t* info) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int nt = (n + 15) >> 4;
  T* Lkk = (T*)smem_raw;           // 16 x CP  factored diagonal block
  T* idg = Lkk + 16 * CP;          // 16       1 / L_jj
  T* Ps = idg + 16;                // (nt*16) x CP  panel (rows of the current block column)
  int* s_fail = (int*)(Ps + nt * 16 * CP);
  T* Am = A + (int64_t)blockIdx.x * strideA;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) *s_fail = 0;
  __syncthreads();
  for (int kb = 0; kb < nt; ++kb) {
    CHOL_STAMP(kb, 0);
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
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = (lane >> 4) + 4 * r;
        const int gc = kb * 16 + c;
        if (gi < n && gc < n) Am[(int64_t)gi * lda + gc] = a[r];
        Lkk[i * CP + c] = a[r];
        if (c == i) idg[i] = (T)1 / a[r];
      }
      if (lane == 0 && fail && *s_fail == 0) *s_fail = fail;
    }
    __syncthreads();
    CHOL_STAMP(kb, 1);
    // phase 2: panel rows below the diagonal block solve x L_kk^T = a, one thread per row.  Loads
    // are clamped in-bounds and masked (per-element branches here cost ~100 VGPRs of spills);
    // the panel goes to global memory from LDS, coalesced, at the start of phase 3.
    {
      const int gi = (kb + 1) * 16 + t;
      if (gi < nt * 16) {
        T x[16];
        const int64_t ro = (int64_t)min(gi, n - 1) * lda;
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const int gc = kb * 16 + c;
          const T v = Am[ro + min(gc, n - 1)];
          x[c] = (gi < n && gc < n) ? v : (T)0;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          T acc = x[j];
#pragma unroll
          for (int c = 0; c < 15; ++c)
            if (c < j) acc -= x[c] * Lkk[j * CP + c];
          x[j] = acc * idg[j];
        }
#pragma unroll
        for (int c = 0; c < 16; ++c) Ps[gi * CP + c] = x[c];
      }
    }
    __syncthreads();
    CHOL_STAMP(kb, 2);
    // phase 3: trailing lower-triangular SYRK, 4 tiles in flight per wave
    const int S = nt - kb - 1;
    const int ntile = S * (S + 1) / 2;
    for (int idx = t; idx < S * 256; idx += CT) {
      const int gi = (kb + 1) * 16 + (idx >> 4), gc = kb * 16 + (idx & 15);
      if (gi < n && gc < n) Am[(int64_t)gi * lda + gc] = Ps[gi * CP + (idx & 15)];
    }
    for (int base = w; base < ntile; base += CW * 4) {
      typename Mfma<T>::acc_t acc[4];
      int ibs[4], jbs[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int tt = base + u * CW;
        ibs[u] = -1;
        if (tt < ntile) {
          int ibo, jbo;
          tri_decode(tt, ibo, jbo);
          ibs[u] = kb + 1 + ibo;
          jbs[u] = kb + 1 + jbo;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int gr = ibs[u] * 16 + Mfma<T>::row(lane, r), gc = jbs[u] * 16 + (lane & 15);
            acc[u][r] = (gr < n && gc < n) ? Am[(int64_t)gr * lda + gc] : (T)0;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (ibs[u] < 0) continue;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int kr = 4 * s + (lane >> 4);
          const T av = Ps[(ibs[u] * 16 + (lane & 15)) * CP + kr];
          const T bv = Ps[(jbs[u] * 16 + (lane & 15)) * CP + kr];
          acc[u] = Mfma<T>::mma(-av, bv, acc[u]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gr = ibs[u] * 16 + Mfma<T>::row(lane, r), gc = jbs[u] * 16 + (lane & 15);
          if (gr < n && gc < n) Am[(int64_t)gr * lda + gc] = acc[u][r];
        }
      }
    }
    __syncthreads();
    CHOL_STAMP(kb, 3);
  }
  for (int64_t idx = t; idx < (int64_t)n * n; idx += blockDim.x) {
    const int i = (int)(idx / n), j = (int)(idx - (int64_t)i * n);
    if (j > i) Am[(int64_t)i * lda + j] = 0;
  }
  if (t == 0 && info) info[blockIdx.x] = *s_fail;
}

// X = L^{-1}: all diagonal-block inverses first (one wave each, in parallel), then block rows
// kb = 0..nt-1:  X[kb, jb] = Li_kk R[kb, jb]  (R accumulated in X),  R[ib, jb] -= L[ib, kb] X[kb, jb].
template <typename T>
__global__ __launch_bounds__(CT) void trtri_kernel(const T* L, int n, int64_t ldl, int64_t strideL, T* X, int64_t ldx,
                                                   int64_t strideX) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int nt = (n + 15) >> 4;
  T* Li = (T*)smem_raw;            // nt x (16 x CP) diagonal-block inverses
  T* Xrow = Li + nt * 16 * CP;     // nt tiles of 16x16 (row-major, pitch 16): block row kb of X
  const T* Lm = L + (int64_t)blockIdx.x * strideL;
  T* Xm = X + (int64_t)blockIdx.x * strideX;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int64_t idx = t; idx < (int64_t)n * n; idx += blockDim.x) {
    const int i = (int)(idx / n), j = (int)(idx - (int64_t)i * n);
    Xm[(int64_t)i * ldx + j] = 0;
  }
  for (int kb = w; kb < nt; kb += CW) {
    const int i = lane & 15, gi = kb * 16 + i;
    T a[4], x[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gc = kb * 16 + (lane >> 4) + 4 * r;
      a[r] = (gi < n && gc < n && gc <= gi) ? Lm[(int64_t)gi * ldl + gc] : (gi == gc ? (T)1 : (T)0);
    }
    trinv16(a, x, lane);
#pragma unroll
    for (int r = 0; r < 4; ++r) Li[(kb * 16 + i) * CP + (lane >> 4) + 4 * r] = x[r];
  }
  __syncthreads();
  for (int kb = 0; kb < nt; ++kb) {
    const T* Lik = Li + kb * 16 * CP;
    for (int jb = w; jb <= kb; jb += CW) {
      typename Mfma<T>::acc_t acc = {0, 0, 0, 0};
      if (jb == kb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = Lik[Mfma<T>::row(lane, r) * CP + (lane & 15)];
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int kr = 4 * s + (lane >> 4);
          const int gk = kb * 16 + kr, gj = jb * 16 + (lane & 15);
          const T av = Lik[(lane & 15) * CP + kr];
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
    const int nr = nt - kb - 1, nc = kb + 1, ntile = nr * nc;
    for (int base = w; base < ntile; base += CW * 4) {
      typename Mfma<T>::acc_t acc[4];
      int ibs[4], jbs[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int tt = base + u * CW;
        ibs[u] = -1;
        if (tt < ntile) {
          ibs[u] = kb + 1 + tt / nc;
          jbs[u] = tt % nc;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int gr = ibs[u] * 16 + Mfma<T>::row(lane, r), gc = jbs[u] * 16 + (lane & 15);
            acc[u][r] = (gr < n && gc < n) ? Xm[(int64_t)gr * ldx + gc] : (T)0;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (ibs[u] < 0) continue;
        const int gi = ibs[u] * 16 + (lane & 15);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int kr = 4 * s + (lane >> 4);
          const int gk = kb * 16 + kr;
          const T av = (gi < n && gk < n) ? Lm[(int64_t)gi * ldl + gk] : (T)0;
          const T bv = Xrow[(jbs[u] * 16 + kr) * 16 + (lane & 15)];
          acc[u] = Mfma<T>::mma(-av, bv, acc[u]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gr = ibs[u] * 16 + Mfma<T>::row(lane, r), gc = jbs[u] * 16 + (lane & 15);
          if (gr < n && gc < n) Xm[(int64_t)gr * ldx + gc] = acc[u][r];
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Fused register-resident factor + inverse for n <= 256:  A -> L (in place),  X = L^{-1}.
//
// Every 16x16 lower tile (ib >= jb) lives in the accumulator registers of one wave for the whole
// kernel (tile tt = w + 8u of the row-major lower-triangle order), so the trailing updates never
// touch global memory.  A tile serves potrf until its block column jb is factored, then the same
// registers hold the trtri remainder R[ib,jb] (initialised to I or 0), which is exactly the set of
// tiles the right-looking trtri sweep touches at step kb >= jb.  Step kb:
//   1. owners of block column kb spill it to LDS (colbuf) and reset the registers to R = 0;
//   2. every wave factors the 16x16 diagonal block redundantly, one row per lane (lanes 0..15),
//      broadcasting L_cj with v_readlane (no LDS, no barriers) while lanes 16..63 forward-solve
//      their panel rows against it; 16 identity rows on the last wave give L_kk^-T;
//   3. X[kb,:] = L_kk^-1 R[kb,:]  (the accumulator IS the MFMA B operand), then the potrf SYRK
//      A[ib,jb] -= L[ib,kb] L[jb,kb]^T and the trtri update R[ib,jb] -= L[ib,kb] X[kb,jb], operands
//      from LDS.  L and X leave through coalesced row copies of the LDS staging buffers.
// The MFMA k-index of lane l in slice s is row(l, s), which makes the accumulator layout equal to
// the B-operand layout for both f64 and f32.
constexpr int RW = 8;  // waves per workgroup of the register-resident kernel

template <typename T> __device__ inline T readlane(T v, int l);
template <> __device__ inline double readlane<double>(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <> __device__ inline float readlane<float>(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// s = sqrt(d) and inv = 1/s, both rounded to nearest as IEEE sqrt and division give them (the
// LAPACK dpotf2 pivot: sqrt, then scale by ONE/AJJ), in 9 dependent FMA-pipe operations instead of
// the ~25 of the library expansions: rsqrt estimate + one Newton step (rel. err ~2^-46), a Markstein
// residual correction for the square root and one for the reciprocal from the same estimate.  d is a
// positive normal pivot; non-positive / NaN pivots propagate NaN (flagged by the caller).  A plain
// refined rsqrt (s = d*y, inv = y) is 1-2 ulp off and measurably moved the trained model.pt loss
// through a cancelling pivot (4.9e-9 relative), so both results are corrected.
template <typename T> __device__ inline void sqrt_recip(T d, T& s, T& inv);
template <> __device__ inline void sqrt_recip<double>(double d, double& s, double& inv) {
  const double y0 = __builtin_amdgcn_rsq(d);
  const double h = d * y0;
  const double r = fma(-h, y0, 1.0);
  const double y1 = fma(0.5 * y0, r, y0);
  const double s0 = d * y1;
  const double rr = fma(-s0, s0, d);
  s = fma(rr, 0.5 * y1, s0);
  const double e = fma(-s, y1, 1.0);
  inv = fma(y1, e, y1);
}
// f32 pivots: the same corrected rsq sequence as f64 (8 FMA-pipe ops after v_rsq) instead of IEEE
// sqrtf + division.  A bare rsq (1 ulp, s = d * rsq) moved the fp32 engine's gradient by 4.5% on the
// ill-conditioned mid fixture (cond(K22 + 1e-4 I) ~ 1e5): the pivots must round like sqrt.
template <> __device__ inline void sqrt_recip<float>(float d, float& s, float& inv) {
  const float y0 = __builtin_amdgcn_rsqf(d);
  const float h = d * y0;
  const float r = fmaf(-h, y0, 1.0f);
  const float y1 = fmaf(0.5f * y0, r, y0);
  const float s0 = d * y1;
  const float rr = fmaf(-s0, s0, d);
  s = fmaf(rr, 0.5f * y1, s0);
  const float e = fmaf(-s, y1, 1.0f);
  inv = fmaf(y1, e, y1);
}

template <typename T, int NTPW>
__global__ __launch_bounds__(RW * 64) void chol_inv_kernel(T* A, int n, int64_t lda, int64_t strideA, T* X,
                                                           int64_t ldx, int64_t strideX, int32_t* info,
                                                           int col_off, int info_first) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  using acc_t = typename Mfma<T>::acc_t;
  const int nt = (n + 15) >> 4, NR = nt * 16;
  T* colbuf = (T*)smem_raw;   // NR x CP : block column kb before the panel step (local rows)
  T* Ps = colbuf + NR * CP;   // NR x CP : L[:, kb] (local rows, diagonal block first)
  T* Xrow = Ps + NR * CP;     // nt tiles x 16 rows x CP : X[kb, jb]
  T* LiT = Xrow + NR * CP;    // 16 x CP : (L_kk^-1)^T
  T* Am = A + (int64_t)blockIdx.x * strideA;
  T* Xm = X + (int64_t)blockIdx.x * strideX;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int ntiles = nt * (nt + 1) / 2;
  int ib[NTPW], jb[NTPW];
  acc_t acc[NTPW];
  int first_fail = 0;
#pragma unroll
  for (int u = 0; u < NTPW; ++u) {
    const int tt = w + RW * u;
    ib[u] = -1;
    jb[u] = -1;
    if (tt < ntiles) {
      tri_decode(tt, ib[u], jb[u]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = ib[u] * 16 + Mfma<T>::row(lane, r), gc = jb[u] * 16 + (lane & 15);
        const T v = Am[(int64_t)min(gr, n - 1) * lda + min(gc, n - 1)];
        acc[u][r] = (gr < n && gc < n) ? v : (gr == gc ? (T)1 : (T)0);
      }
    }
  }
  // strictly-upper block tiles of both outputs are zero (issued first; the stores drain while the
  // factorization runs -- the barriers below do not wait for global stores)
  for (int i = w; i < n; i += RW) {
    for (int j = ((i >> 4) + 1) * 16 + lane; j < n; j += 64) {
      Am[(int64_t)i * lda + j] = 0;
      Xm[(int64_t)i * ldx + j] = 0;
    }
  }
  for (int kb = 0; kb < nt; ++kb) {
    CHOL_STAMP(kb, 0);
    const int nrow = NR - kb * 16;  // local rows of block column kb
    // 1. block column kb -> colbuf, registers -> trtri remainder R
#pragma unroll
    for (int u = 0; u < NTPW; ++u) {
      if (jb[u] == kb) {
        const int dib = __builtin_amdgcn_readfirstlane(ib[u] - kb);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = Mfma<T>::row(lane, r);
          colbuf[(dib * 16 + row) * CP + (lane & 15)] = acc[u][r];
          acc[u][r] = 0;  // R[ib, kb] starts at 0; R[kb, kb] = I is applied in 3a
        }
      }
    }
    lds_barrier();
    CHOL_STAMP(kb, 1);
    // 2. diagonal factor (lanes 0..15 of every participating wave) + the nrow-16 panel rows and 16
    //    identity rows on lanes 16..63.  Only ceil(nrow/48) waves take part: the diagonal work is
    //    redundant per wave, so idle waves stay off the SIMDs.
    if (w < (nrow + 47) / 48) {
      int lr;
      bool ident = false;
      if (lane < 16) {
        lr = lane;
      } else {
        const int slot = w * 48 + lane - 16;
        ident = slot >= nrow - 16 && slot < nrow;
        lr = ident ? slot - (nrow - 16) : 16 + slot;
      }
      const bool active = ident || lr < nrow;
      T a[16];
      {
        // branch-free: a select on a loaded value lets the compiler sink each load into its own
        // exec-masked branch with a full LDS wait (16 serialized round trips)
        const T keep = (active && !ident) ? (T)1 : (T)0;
        const T* src = colbuf + min(lr, NR - 1) * CP;
#pragma unroll
        for (int c = 0; c < 16; ++c) a[c] = fma(src[c], keep, (ident && c == lr) ? (T)1 : (T)0);
      }
      // Critical path per column: readlane(d) -> sqrt_recip -> scale -> readlane -> fma.
      CHOL_STAMPW(kb, 0);
      unsigned int bad = 0;  // non-positive (or NaN) pivots of this block; NaN propagates onwards
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const T d = readlane(a[j], j);
        bad |= (d > (T)0) ? 0u : (1u << j);
        T sj, inv;
        sqrt_recip(d, sj, inv);
        a[j] = (lane == j) ? sj : a[j] * inv;
#pragma unroll
        for (int c = j + 1; c < 16; ++c) a[c] = fma(-a[j], readlane(a[j], c), a[c]);
      }
      CHOL_STAMPW(kb, 1);
      if (bad && first_fail == 0) {
        const int j0 = __builtin_ctz(bad);
        if (kb * 16 + j0 < n) first_fail = kb * 16 + j0 + 1;
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) a[c] = (lane < 16 && c > lane) ? (T)0 : a[c];
      // identity lanes hold rows of L_kk^-T: stored as LiT = (L_kk^-1)^T
      if (ident || (active && (lane >= 16 || w == 0))) {
        T* dst = (ident ? LiT : Ps) + lr * CP;
#pragma unroll
        for (int c = 0; c < 16; ++c) dst[c] = a[c];
      }
      CHOL_STAMPW(kb, 2);
    }
    lds_barrier();
    CHOL_STAMP(kb, 2);
    // 3a. X[kb, jb] = L_kk^-1 R[kb, jb]
#pragma unroll
    for (int u = 0; u < NTPW; ++u) {
      if (ib[u] == kb) {
        const int xj = __builtin_amdgcn_readfirstlane(jb[u] - kb) + kb;
        acc_t x = {0, 0, 0, 0};
        if (xj == kb) {
#pragma unroll
          for (int r = 0; r < 4; ++r) x[r] = LiT[(lane & 15) * CP + Mfma<T>::row(lane, r)];
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) x = Mfma<T>::mma(LiT[Mfma<T>::row(lane, s) * CP + (lane & 15)], acc[u][s], x);
        }
        acc[u] = x;
#pragma unroll
        for (int r = 0; r < 4; ++r) Xrow[(xj * 16 + Mfma<T>::row(lane, r)) * CP + (lane & 15)] = x[r];
      }
    }
    // 3b. potrf trailing update
#pragma unroll
    for (int u = 0; u < NTPW; ++u) {
      if (jb[u] > kb) {
        // readfirstlane of a loop-variant value: keeps per-tile LDS addresses from being hoisted
        // out of the kb loop into (spilled) per-tile VGPRs
        const int ra = __builtin_amdgcn_readfirstlane(ib[u] - kb) * 16 + (lane & 15);
        const int rb = __builtin_amdgcn_readfirstlane(jb[u] - kb) * 16 + (lane & 15);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int kr = Mfma<T>::row(lane, s);
          acc[u] = Mfma<T>::mma(-Ps[ra * CP + kr], Ps[rb * CP + kr], acc[u]);
        }
      }
    }
    for (int idx = t; idx < nrow * 16; idx += RW * 64) {
      const int lr = idx >> 4, c = idx & 15;
      const int gr = kb * 16 + lr, gc = kb * 16 + c;
      if (gr < n && gc < n) Am[(int64_t)gr * lda + gc] = Ps[lr * CP + c];
    }
    lds_barrier();
    CHOL_STAMP(kb, 3);
    // 3c. trtri update of the rows below kb
#pragma unroll
    for (int u = 0; u < NTPW; ++u) {
      if (ib[u] > kb && jb[u] >= 0 && jb[u] <= kb) {
        const int ra = __builtin_amdgcn_readfirstlane(ib[u] - kb) * 16 + (lane & 15);
        const int xj = __builtin_amdgcn_readfirstlane(jb[u] - kb) + kb;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int kr = Mfma<T>::row(lane, s);
          acc[u] = Mfma<T>::mma(-Ps[ra * CP + kr], Xrow[(xj * 16 + kr) * CP + (lane & 15)], acc[u]);
        }
      }
    }
    for (int idx = t; idx < (kb + 1) * 256; idx += RW * 64) {
      const int j = idx >> 8, k = (idx >> 4) & 15, c = idx & 15;
      const int gr = kb * 16 + k, gc = j * 16 + c;
      if (gr < n && gc < n) Xm[(int64_t)gr * ldx + gc] = Xrow[(j * 16 + k) * CP + c];
    }
  }
  CHOL_STAMP(nt, 0);
  // wave 0 tracked the pivots; in a blocked factorization (col_off > 0) an earlier block's failure
  // stays the reported one
  if (t == 0 && info) {
    if (info_first) info[blockIdx.x] = first_fail ? first_fail + col_off : 0;
    else if (first_fail && info[blockIdx.x] == 0) info[blockIdx.x] = first_fail + col_off;
  }
}

// Two workgroups per matrix (f64, 32 <= n <= 256): the fused kernel's MFMA work is split by role and
// the roles run concurrently, pipelined one block step apart.
//   role 0 (potrf): spill block column kb, panel factor (L_kk, L_kk^-1, L[:, kb]), trailing SYRK on
//     its register tiles; publishes L[:, kb] (final output A) and L_kk^-1 (the final diagonal block
//     of X) write-through, then a progress flag.
//   role 1 (trtri): register tiles of R (starts as I); per step waits for the flag, reads L[:, kb] and
//     L_kk^-1 (sc1 loads), forms X[kb, :] = L_kk^-1 R[kb, :] and updates the rows below.
// Visibility: payload stored sc1 and drained (vmcnt(0)) in every storing wave before a barrier and the
// flag store; the consumer polls the flag with an agent-scope load and reads the payload with sc1
// loads only (MI355X guide, inter-workgroup hand-off, row 1).  The flag lives in X(0, n-1), inside a
// strictly upper block tile (n >= 32) that role 1 zeroes at the end; its values carry a 48-bit tag
// so stale bits in an uninitialised X cannot pass for progress.  Role 1 waits only on its own
// role 0 (block 2b before 2b+1) and every spin is bounded: a lost peer gives wrong output, not a hang.
constexpr unsigned long long kFlagTag = 0x7ff8d5a1c0de0000ull;
// The 64-bit control words live at the end of X's row 0 (strictly upper, zeroed at the end): the
// progress flag in the last 8 bytes, the three-role consumer count in the 8 bytes before.  f32 needs
// n even and X 8-byte aligned (checked by the host, chol_ctl_ok).
template <typename T> constexpr int kCtl = 8 / (int)sizeof(T);     // elements per control word
template <typename T> __device__ inline unsigned long long* ctl_flag(T* Xm, int n) {
  return (unsigned long long*)(Xm + (n - kCtl<T>));
}
template <typename T> __device__ inline unsigned long long* ctl_done(T* Xm, int n) {
  return (unsigned long long*)(Xm + (n - 2 * kCtl<T>));
}
// fused prior launch (chol_tp_kernel): the inverse workgroup of block-column parity `par` publishes its finished X
// rows through X(0, n - (4 + par) words) (the four-role kernel's hflag is the third word)
template <typename T> __device__ inline unsigned long long* ctl_xflag(T* Xm, int n, int par) {
  return (unsigned long long*)(Xm + (n - (4 + par) * kCtl<T>));
}
// the fused launch's extra words, cleared by the last of a matrix's readers
template <typename T> __device__ inline void tp_clear_words(T* Xm, int n) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    __hip_atomic_store(ctl_xflag(Xm, n, q), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// K22 + jitter I element of a prior that the fused launch builds in the factor / update workgroups instead of
// reading it: the arithmetic of pairwise_kernel (csrc/pairwise.hip) for the same matrix -- RBF
// s2 exp(-(z_i/ls - z_j/ls)^2 / 2) (code/utils.py:91-94), Gibbs sqrt(2 l_i l_j / S) exp(-(z_i - z_j)^2 / S),
// S = l_i^2 + l_j^2 (code/utils.py:97-103)
// phase stamps of the fused launch (tools/chol_tp_probe.py, NMGP_TP_DBG bit 16): 8 words per workgroup, read back
// with nmgp_chol_tp_trace
__device__ unsigned long long g_tp_trace[8 * 512];
#define TP_STAMP(on, k) \
  if ((on) && threadIdx.x == 0 && blockIdx.x < 512) g_tp_trace[8 * blockIdx.x + (k)] = wall_clock64()
// Gibbs element from the squared distance and the two length scales: one division (1 / S) where pairwise_kernel
// divides twice (<= 1 ulp apart); the exp / sqrt chains are long, so callers evaluate batches of independent
// elements in straight-line code (no per-element branches) for the scheduler to interleave
__device__ inline double tp_gibbs(double r2, double lx, double lz) {
  const double iS = 1.0 / (lx * lx + lz * lz);
  return dsqrt(2.0 * (lx * lz) * iS) * dexp(-r2 * iS);
}
// the per-index inputs of the row workgroups' K12 elements, staged in LDS (one division per index, not per element)
__device__ inline void tp_stage(double* uz, double* ul, int mode, const double* Z, const double* ellZ, double ls,
                                int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    uz[i] = mode == 1 ? Z[i] / ls : Z[i] / 1.0;
    if (mode == 2) ul[i] = ellZ[i];
  }
  __syncthreads();
}

template <typename T, int NTPW>
__device__ __attribute__((always_inline)) inline void chol2_potrf_role(T* Am, T* Xm, int n, int64_t lda, int64_t ldx, int32_t* info, int col_off,
                                  int info_first, int mat, unsigned char* smem_raw) {
  using acc_t = typename Mfma<T>::acc_t;
  const int nt = (n + 15) >> 4, NR = nt * 16;
  T* colbuf = (T*)smem_raw;   // role 0: NR x CP block column kb before the panel step
  T* Ps = colbuf + NR * CP;   // NR x CP : L[:, kb] (local rows, diagonal block first)
  T* Xrow = Ps + NR * CP;     // role 1: nt tiles x 16 rows x CP : X[kb, jb]
  T* LiT = Xrow + NR * CP;    // 16 x CP : (L_kk^-1)^T
  unsigned long long* flag = ctl_flag(Xm, n);
  const __amdgpu_buffer_rsrc_t rAm = make_rsrc(Am, ((int64_t)(n - 1) * lda + n) * (int64_t)sizeof(T));
  const __amdgpu_buffer_rsrc_t rXm = make_rsrc(Xm, ((int64_t)(n - 1) * ldx + n) * (int64_t)sizeof(T));
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int ntiles = nt * (nt + 1) / 2;
  CHOL_STAMPX(0);
  int ib[NTPW], jb[NTPW];
  acc_t acc[NTPW];
  // decode every owned tile first, then issue all NTPW x 4 loads unconditionally (out-of-range ones
  // read 0 through the resource) so they share one memory round trip: loads behind the per-tile
  // branches went out one tile at a time (13 us of prologue at n = 256)
#pragma unroll
  for (int u = 0; u < NTPW; ++u) {
    const int tt = w + RW * u;
    ib[u] = -1;
    jb[u] = -1;
    if (tt < ntiles) tri_decode(tt, ib[u], jb[u]);
  }
#pragma unroll
  for (int u = 0; u < NTPW; ++u) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gr = ib[u] * 16 + Mfma<T>::row(lane, r), gc = jb[u] * 16 + (lane & 15);
      const bool in = ib[u] >= 0 && gr < n && gc < n;
      acc[u][r] = bload<T>(rAm, in ? (uint32_t)(((int64_t)gr * lda + gc) * sizeof(T)) : 0x80000000u);
    }
  }
#pragma unroll
  for (int u = 0; u < NTPW; ++u) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gr = ib[u] * 16 + Mfma<T>::row(lane, r), gc = jb[u] * 16 + (lane & 15);
      if (ib[u] >= 0 && !(gr < n && gc < n)) acc[u][r] = gr == gc ? (T)1 : (T)0;   // padding past n
    }
  }
  int first_fail = 0;
  // (the strictly-upper block tiles of L are zeroed by the inverse workgroups while they wait for the
  // first block column: here the ~n^2/2 stores sat in front of the first vmcnt wait, 10 us of prologue)
  CHOL_STAMPX(1);
  for (int kb = 0; kb < nt; ++kb) {
    CHOL_STAMP(kb, 0);
    const int nrow = NR - kb * 16;
#pragma unroll
    for (int u = 0; u < NTPW; ++u) {
      if (jb[u] == kb) {
        const int dib = __builtin_amdgcn_readfirstlane(ib[u] - kb);
#pragma unroll
        for (int r = 0; r < 4; ++r) colbuf[(dib * 16 + Mfma<T>::row(lane, r)) * CP + (lane & 15)] = acc[u][r];
      }
    }
    lds_barrier();
    CHOL_STAMP(kb, 1);
    if (w < (nrow + 47) / 48) {
      int lr;
      bool ident = false;
      if (lane < 16) {
        lr = lane;
      } else {
        const int slot = w * 48 + lane - 16;
        ident = slot >= nrow - 16 && slot < nrow;
        lr = ident ? slot - (nrow - 16) : 16 + slot;
      }
      const bool active = ident || lr < nrow;
      T a[16];
      {
        const T keep = (active && !ident) ? (T)1 : (T)0;
        const T* src = colbuf + min(lr, NR - 1) * CP;
#pragma unroll
        for (int c = 0; c < 16; ++c) a[c] = fma(src[c], keep, (ident && c == lr) ? (T)1 : (T)0);
      }
      CHOL_STAMPW(kb, 0);
      unsigned int bad = 0;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const T d = readlane(a[j], j);
        bad |= (d > (T)0) ? 0u : (1u << j);
        T sj, inv;
        sqrt_recip(d, sj, inv);
        a[j] = (lane == j) ? sj : a[j] * inv;
#pragma unroll
        for (int c = j + 1; c < 16; ++c) a[c] = fma(-a[j], readlane(a[j], c), a[c]);
      }
      CHOL_STAMPW(kb, 1);
      if (bad && first_fail == 0) {
        const int j0 = __builtin_ctz(bad);
        if (kb * 16 + j0 < n) first_fail = kb * 16 + j0 + 1;
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) a[c] = (lane < 16 && c > lane) ? (T)0 : a[c];
      if (ident || (active && (lane >= 16 || w == 0))) {
        T* dst = (ident ? LiT : Ps) + lr * CP;
#pragma unroll
        for (int c = 0; c < 16; ++c) dst[c] = a[c];
      }
      CHOL_STAMPW(kb, 2);
    }
    // the previous step's published stores had this step's spill and panel to drain: the wait is
    // (nearly) free here, where right after the SYRK it stalled every step for a full write round trip
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (t == 0 && kb > 0)
      __hip_atomic_store(flag, kFlagTag + (unsigned long long)kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    CHOL_STAMP(kb, 2);
    // publish L[:, kb] (final output) and L_kk^-1 (= the final X[kb, kb]) write-through
    for (int idx = t; idx < nrow * 16; idx += RW * 64) {
      const int lr = idx >> 4, c = idx & 15;
      const int gr = kb * 16 + lr, gc = kb * 16 + c;
      if (gr < n && gc < n) bstore_sc1<T>(rAm, (uint32_t)(((int64_t)gr * lda + gc) * sizeof(T)), Ps[lr * CP + c]);
    }
    if (t < 256) {
      const int r = t >> 4, c = t & 15;
      const int gr = kb * 16 + r, gc = kb * 16 + c;
      if (gr < n && gc < n) bstore_sc1<T>(rXm, (uint32_t)(((int64_t)gr * ldx + gc) * sizeof(T)), LiT[c * CP + r]);
    }
    // trailing SYRK while the stores drain
#pragma unroll
    for (int u = 0; u < NTPW; ++u) {
      if (jb[u] > kb) {
        const int ra = __builtin_amdgcn_readfirstlane(ib[u] - kb) * 16 + (lane & 15);
        const int rb = __builtin_amdgcn_readfirstlane(jb[u] - kb) * 16 + (lane & 15);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int kr = Mfma<T>::row(lane, s);
          acc[u] = Mfma<T>::mma(-Ps[ra * CP + kr], Ps[rb * CP + kr], acc[u]);
        }
      }
    }
    CHOL_STAMP(kb, 3);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  if (t == 0) __hip_atomic_store(flag, kFlagTag + (unsigned long long)nt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  CHOL_STAMP(nt, 0);
  CHOL_STAMPX(2);
  if (t == 0 && info) {
    if (info_first) info[mat] = first_fail ? first_fail + col_off : 0;
    else if (first_fail && info[mat] == 0) info[mat] = first_fail + col_off;
  }
}

template <typename T, int NTPW>
__device__ __attribute__((always_inline)) inline void chol2_trtri_role(T* Am, T* Xm, int n, int64_t lda, int64_t ldx, int32_t* info, int col_off,
                                  int info_first, int mat, unsigned char* smem_raw) {
  using acc_t = typename Mfma<T>::acc_t;
  const int nt = (n + 15) >> 4, NR = nt * 16;
  T* colbuf = (T*)smem_raw;   // role 0: NR x CP block column kb before the panel step
  T* Ps = colbuf + NR * CP;   // NR x CP : L[:, kb] (local rows, diagonal block first)
  T* Xrow = Ps + NR * CP;     // role 1: nt tiles x 16 rows x CP : X[kb, jb]
  T* LiT = Xrow + NR * CP;    // 16 x CP : (L_kk^-1)^T
  unsigned long long* flag = ctl_flag(Xm, n);
  const __amdgpu_buffer_rsrc_t rAm = make_rsrc(Am, ((int64_t)(n - 1) * lda + n) * (int64_t)sizeof(T));
  const __amdgpu_buffer_rsrc_t rXm = make_rsrc(Xm, ((int64_t)(n - 1) * ldx + n) * (int64_t)sizeof(T));
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int ntiles = nt * (nt + 1) / 2;
  int ib[NTPW], jb[NTPW];
  acc_t acc[NTPW];
#pragma unroll
  for (int u = 0; u < NTPW; ++u) {
    const int tt = w + RW * u;
    ib[u] = -1;
    jb[u] = -1;
    if (tt < ntiles) {
      tri_decode(tt, ib[u], jb[u]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = ib[u] * 16 + Mfma<T>::row(lane, r), gc = jb[u] * 16 + (lane & 15);
        acc[u][r] = gr == gc ? (T)1 : (T)0;  // R starts as the identity
      }
    }
  }
  for (int i = w; i < n; i += RW)
    for (int j = ((i >> 4) + 1) * 16 + lane; j < n; j += 64) {
      if (i != 0 || j < n - kCtl<T>) Xm[(int64_t)i * ldx + j] = 0;
      Am[(int64_t)i * lda + j] = 0;                // strictly-upper block tiles of L (factor role reads none)
    }
  for (int kb = 0; kb < nt; ++kb) {
    const int nrow = NR - kb * 16;
    if (t == 0) {
      bool seen = false;
      for (int spin = 0; spin < (1 << 26); ++spin) {
        const unsigned long long f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (f >= kFlagTag + (unsigned long long)(kb + 1) && f <= kFlagTag + (unsigned long long)nt) {
          seen = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (!seen) spin_gave_up(NMGP_STATUS_CHOL_SPIN);   // surfaced by nmgp_device_status()
    }
    CHOL_STAMP1(kb, 0);
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the poll
    {
      // all loads in flight before any LDS store: one memory round trip per step, not one per element
      constexpr int PER = 256 * 16 / (RW * 64);  // elements per thread at n = 256
      T v[PER];
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int idx = t + q * RW * 64, lr = idx >> 4, c = idx & 15;
        const int gr = kb * 16 + lr, gc = kb * 16 + c;
        // rows past n (and past this column's rows) load as 0: offset past the resource's range
        const uint32_t off =
            (idx < nrow * 16 && gr < n && gc < n) ? (uint32_t)(((int64_t)gr * lda + gc) * sizeof(T)) : 0x80000000u;
        v[q] = bload_sc1<T>(rAm, off);
      }
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int idx = t + q * RW * 64;
        if (idx < nrow * 16) Ps[(idx >> 4) * CP + (idx & 15)] = v[q];
      }
    }
    if (t < 256) {
      const int r = t >> 4, c = t & 15;
      const int gr = kb * 16 + r, gc = kb * 16 + c;
      const uint32_t off = (gr < n && gc < n) ? (uint32_t)(((int64_t)gr * ldx + gc) * sizeof(T)) : 0x80000000u;
      T v = bload_sc1<T>(rXm, off);
      if (gr >= n || gc >= n) v = (gr == gc) ? (T)1 : (T)0;  // padded identity past n
      LiT[c * CP + r] = v;
    }
    lds_barrier();
    CHOL_STAMP1(kb, 1);
    // X[kb, jb] = L_kk^-1 R[kb, jb]
#pragma unroll
    for (int u = 0; u < NTPW; ++u) {
      if (ib[u] == kb) {
        const int xj = __builtin_amdgcn_readfirstlane(jb[u] - kb) + kb;
        acc_t x = {0, 0, 0, 0};
        if (xj == kb) {
#pragma unroll
          for (int r = 0; r < 4; ++r) x[r] = LiT[(lane & 15) * CP + Mfma<T>::row(lane, r)];
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) x = Mfma<T>::mma(LiT[Mfma<T>::row(lane, s) * CP + (lane & 15)], acc[u][s], x);
        }
        acc[u] = x;
#pragma unroll
        for (int r = 0; r < 4; ++r) Xrow[(xj * 16 + Mfma<T>::row(lane, r)) * CP + (lane & 15)] = x[r];
      }
    }
    lds_barrier();
    CHOL_STAMP1(kb, 2);
    // rows below kb: R[ib, jb] -= L[ib, kb] X[kb, jb]
#pragma unroll
    for (int u = 0; u < NTPW; ++u) {
      if (ib[u] > kb && jb[u] >= 0 && jb[u] <= kb) {
        const int ra = __builtin_amdgcn_readfirstlane(ib[u] - kb) * 16 + (lane & 15);
        const int xj = __builtin_amdgcn_readfirstlane(jb[u] - kb) + kb;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int kr = Mfma<T>::row(lane, s);
          acc[u] = Mfma<T>::mma(-Ps[ra * CP + kr], Xrow[(xj * 16 + kr) * CP + (lane & 15)], acc[u]);
        }
      }
    }
    for (int idx = t; idx < (kb + 1) * 256; idx += RW * 64) {
      const int j = idx >> 8, k = (idx >> 4) & 15, c = idx & 15;
      const int gr = kb * 16 + k, gc = j * 16 + c;
      if (gr < n && gc < n) Xm[(int64_t)gr * ldx + gc] = Xrow[(j * 16 + k) * CP + c];
    }
    // the next step's loads overwrite Ps / LiT / Xrow: everyone must be done reading them
    lds_barrier();
    CHOL_STAMP1(kb, 3);
  }
  if (t == 0) __hip_atomic_store(flag, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Three workgroups per matrix (f64, 32 <= n <= 256): the factor role as above, and the inverse role
// split over two workgroups by block-column parity (X[:, jb] and R[:, jb] for jb % 2 == par): the
// trtri work of a late block step (rows below kb x columns up to kb) grows past the factor's step
// time on one CU, so a single inverse workgroup fell behind by up to 15 us per step.  Both read the
// factor role's published L[:, kb] / L_kk^-1; the last of them to finish re-arms the progress word
// (a second word, X(0, n-2), counts finished consumers; the factor role initialises it).
constexpr unsigned long long kDoneTag = 0x7ff8d5a1d0e00000ull;

__device__ inline void tri_decode_par(int tp, int par, int& ib, int& jb) {
  ib = -1;
  jb = -1;
  for (int r = par; r < 64; ++r) {           // row r holds (r - par) / 2 + 1 tiles of this parity
    const int c = (r - par) / 2 + 1;
    if (tp < c) {
      ib = r;
      jb = par + 2 * tp;
      return;
    }
    tp -= c;
  }
}

template <typename T, int NTPW, int NCTL = 2, bool XPUB = false>
__device__ __attribute__((always_inline)) inline void chol3_trtri_role(T* Am, T* Xm, int n, int64_t lda,
                                                                       int64_t ldx, int par, unsigned char* smem_raw,
                                                                       int nfin = 2) {
  using acc_t = typename Mfma<T>::acc_t;
  const int nt = (n + 15) >> 4, NR = nt * 16;
  T* Ps = (T*)smem_raw + NR * CP;
  T* Xrow = Ps + NR * CP;
  T* LiT = Xrow + NR * CP;
  unsigned long long* flag = ctl_flag(Xm, n);
  unsigned long long* done = ctl_done(Xm, n);
  const __amdgpu_buffer_rsrc_t rAm = make_rsrc(Am, ((int64_t)(n - 1) * lda + n) * (int64_t)sizeof(T));
  const __amdgpu_buffer_rsrc_t rXm = make_rsrc(Xm, ((int64_t)(n - 1) * ldx + n) * (int64_t)sizeof(T));
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  int ntp = 0;                                                          // lower tiles of this parity
  for (int j = par; j < nt; j += 2) ntp += nt - j;
  int ib[NTPW], jb[NTPW];
  acc_t acc[NTPW];
#pragma unroll
  for (int u = 0; u < NTPW; ++u) {
    const int tp = w + RW * u;
    ib[u] = -1;
    jb[u] = -1;
    if (tp < ntp) {
      tri_decode_par(tp, par, ib[u], jb[u]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = ib[u] * 16 + Mfma<T>::row(lane, r), gc = jb[u] * 16 + (lane & 15);
        acc[u][r] = gr == gc ? (T)1 : (T)0;  // R starts as the identity
      }
    }
  }
  // XPUB (the fused prior launch): X rows are stored write-through and, once drained, announced in xflag, so the
  // launch's row workgroups can read them while the factorization runs
  unsigned long long* xflag = ctl_xflag(Xm, n, par);
  // strictly upper part of X is zero (rows of this parity; the two control words stay)
  for (int i = 2 * w + par; i < n; i += 2 * RW)
    for (int j = ((i >> 4) + 1) * 16 + lane; j < n; j += 64) {
      if (i != 0 || j < n - NCTL * kCtl<T>) Xm[(int64_t)i * ldx + j] = 0;
      Am[(int64_t)i * lda + j] = 0;                // strictly-upper block tiles of L (factor role reads none)
    }
  for (int kb = 0; kb < nt; ++kb) {
    const int nrow = NR - kb * 16;
    if (t == 0) {
      bool seen = false;
      for (int spin = 0; spin < (1 << 26); ++spin) {
        const unsigned long long f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (f >= kFlagTag + (unsigned long long)(kb + 1) && f <= kFlagTag + (unsigned long long)nt) {
          seen = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (!seen) spin_gave_up(NMGP_STATUS_CHOL_SPIN);
    }
    CHOL_STAMP1(kb, 0);
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    {
      constexpr int PER = 256 * 16 / (RW * 64);
      T v[PER];
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int idx = t + q * RW * 64, lr = idx >> 4, c = idx & 15;
        const int gr = kb * 16 + lr, gc = kb * 16 + c;
        const uint32_t off =
            (idx < nrow * 16 && gr < n && gc < n) ? (uint32_t)(((int64_t)gr * lda + gc) * sizeof(T)) : 0x80000000u;
        v[q] = bload_sc1<T>(rAm, off);
      }
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int idx = t + q * RW * 64;
        if (idx < nrow * 16) Ps[(idx >> 4) * CP + (idx & 15)] = v[q];
      }
    }
    if (t < 256) {
      const int r = t >> 4, c = t & 15;
      const int gr = kb * 16 + r, gc = kb * 16 + c;
      const uint32_t off = (gr < n && gc < n) ? (uint32_t)(((int64_t)gr * ldx + gc) * sizeof(T)) : 0x80000000u;
      T v = bload_sc1<T>(rXm, off);
      if (gr >= n || gc >= n) v = (gr == gc) ? (T)1 : (T)0;
      LiT[c * CP + r] = v;
    }
    // (XPUB: the previous step's X rows had this step's poll and loads to drain)
    if constexpr (XPUB) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if constexpr (XPUB) {
      if (t == 0 && kb > 0)
        __hip_atomic_store(xflag, kFlagTag + (unsigned long long)kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    CHOL_STAMP1(kb, 1);
    // X[kb, jb] = L_kk^-1 R[kb, jb]   (jb <= kb of this parity)
#pragma unroll
    for (int u = 0; u < NTPW; ++u) {
      if (ib[u] == kb) {
        const int xj = __builtin_amdgcn_readfirstlane(jb[u] - kb) + kb;
        acc_t x = {0, 0, 0, 0};
        if (xj == kb) {
#pragma unroll
          for (int r = 0; r < 4; ++r) x[r] = LiT[(lane & 15) * CP + Mfma<T>::row(lane, r)];
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) x = Mfma<T>::mma(LiT[Mfma<T>::row(lane, s) * CP + (lane & 15)], acc[u][s], x);
        }
        acc[u] = x;
#pragma unroll
        for (int r = 0; r < 4; ++r) Xrow[(xj * 16 + Mfma<T>::row(lane, r)) * CP + (lane & 15)] = x[r];
      }
    }
    lds_barrier();
    CHOL_STAMP1(kb, 2);
    // rows below kb: R[ib, jb] -= L[ib, kb] X[kb, jb]
#pragma unroll
    for (int u = 0; u < NTPW; ++u) {
      if (ib[u] > kb && jb[u] >= 0 && jb[u] <= kb) {
        const int ra = __builtin_amdgcn_readfirstlane(ib[u] - kb) * 16 + (lane & 15);
        const int xj = __builtin_amdgcn_readfirstlane(jb[u] - kb) + kb;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int kr = Mfma<T>::row(lane, s);
          acc[u] = Mfma<T>::mma(-Ps[ra * CP + kr], Xrow[(xj * 16 + kr) * CP + (lane & 15)], acc[u]);
        }
      }
    }
    const int ncol = kb >= par ? (kb - par) / 2 + 1 : 0;   // own block columns <= kb
    for (int idx = t; idx < ncol * 256; idx += RW * 64) {
      const int j = par + 2 * (idx >> 8), k = (idx >> 4) & 15, c = idx & 15;
      const int gr = kb * 16 + k, gc = j * 16 + c;
      if (gr < n && gc < n) {
        if constexpr (XPUB)
          bstore_sc1<T>(rXm, (uint32_t)(((int64_t)gr * ldx + gc) * sizeof(T)), Xrow[(j * 16 + k) * CP + c]);
        else
          Xm[(int64_t)gr * ldx + gc] = Xrow[(j * 16 + k) * CP + c];
      }
    }
    lds_barrier();
    CHOL_STAMP1(kb, 3);
  }
  CHOL_STAMPX(2);
  if constexpr (XPUB) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (t == 0) __hip_atomic_store(xflag, kFlagTag + (unsigned long long)nt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (t == 0) {
    // the last of the launch's `nfin` readers of this matrix's words re-arms the progress word for the next launch
    // and clears the others
    const unsigned long long old = __hip_atomic_fetch_add(done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == kDoneTag + (unsigned long long)(nfin - 1)) {
      __hip_atomic_store(flag, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if constexpr (XPUB) tp_clear_words(Xm, n);
      __hip_atomic_store(done, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <typename T, int NTPW, int NTPW1>
__global__ __launch_bounds__(RW * 64) void chol_inv3_kernel(T* A, int n, int64_t lda, int64_t strideA, T* X,
                                                            int64_t ldx, int64_t strideX, int32_t* info, int col_off,
                                                            int info_first) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int mat = blockIdx.x / 3, role = blockIdx.x - 3 * mat;
  T* Am = A + (int64_t)mat * strideA;
  T* Xm = X + (int64_t)mat * strideX;
  if (role == 0) {
    if (threadIdx.x == 0) __hip_atomic_store(ctl_done(Xm, n), kDoneTag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    chol2_potrf_role<T, NTPW>(Am, Xm, n, lda, ldx, info, col_off, info_first, mat, smem_raw);
  } else {
    chol3_trtri_role<T, NTPW1>(Am, Xm, n, lda, ldx, role - 1, smem_raw);
  }
}

// ------------------------------------------------------------------------------------------------
// Four workgroups per matrix (chol_inv7_kernel, round 3): the three-role kernel's factor workgroup spent
// ~1.9 of its ~5.5 us per block step on the trailing SYRK of its register-resident tiles.  Here that
// update runs on a fourth workgroup on another CU:
//   role 0 (factor): per block step k takes block column k (the update workgroup has applied steps
//     <= k-4 to it), applies steps k-3 .. k-1 itself from the L[:, k-3 .. k-1] it still holds in LDS
//     (three buffers), then the panel exactly as chol2_potrf_role (lanes 0..15 the diagonal
//     rows of every panel wave, identity rows for L_kk^-T), publishes L[:, k] and L_kk^-1 write-through.
//     Column k+1's loads are issued right after column k's spill, so they are in flight during the panel.
//   role 1 (update): owns the tiles of block columns >= 4 in MFMA accumulators.  Per step j it reads the
//     published L[:, j], applies it to block column j+4 first and publishes that column (progress word
//     hflag = j+1), then to the columns beyond.  The three-step lookahead gives its memory round trips
//     (read L[:, j], publish column j+4) about two factor steps of slack, so the factor drains its own
//     stores where that is free (after the next panel) and never waits on a round trip.
//   roles 2, 3 (inverse): chol3_trtri_role, unchanged.
// Every tile receives the same MFMA updates in the same order as in chol2_potrf_role (steps <= k-3 on the
// update workgroup, steps k-3 .. k-1 on the factor; the accumulators round-trip through memory exactly), so L and
// L^-1 are bit-identical to the three-role kernel's.
template <typename T> __device__ inline unsigned long long* ctl_hflag(T* Xm, int n) {
  return (unsigned long long*)(Xm + (n - 3 * kCtl<T>));
}

template <typename T>
__device__ __attribute__((always_inline)) inline bool poll_word(unsigned long long* word, int need, int nt,
                                                                int max_spin = 1 << 26) {
  for (int spin = 0; spin < max_spin; ++spin) {
    const unsigned long long f = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (f >= kFlagTag + (unsigned long long)need && f <= kFlagTag + (unsigned long long)nt) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}

template <typename T>
__device__ __attribute__((always_inline)) inline void chol7_factor_role(T* Am, T* Xm, int n, int64_t lda,
                                                                        int64_t ldx, int32_t* info, int col_off,
                                                                        int info_first, int mat,
                                                                        unsigned char* smem_raw) {
  using acc_t = typename Mfma<T>::acc_t;
  const int nt = (n + 15) >> 4, NR = nt * 16;
  T* colbuf = (T*)smem_raw;            // NR x CP: block column k before its panel (local rows)
  T* Ps0 = colbuf + NR * CP;           // 3 x NR x CP: L[:, k] in buffer k % 3 (local rows, diagonal block first)
  T* LiT = Ps0 + 3 * NR * CP;          // 16 x CP: (L_kk^-1)^T
  unsigned long long* flag = ctl_flag(Xm, n);
  unsigned long long* hflag = ctl_hflag(Xm, n);
  const __amdgpu_buffer_rsrc_t rAm = make_rsrc(Am, ((int64_t)(n - 1) * lda + n) * (int64_t)sizeof(T));
  const __amdgpu_buffer_rsrc_t rXm = make_rsrc(Xm, ((int64_t)(n - 1) * ldx + n) * (int64_t)sizeof(T));
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  if (t == 0) __hip_atomic_store(hflag, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bool ok = true;
  acc_t acc[2];
  // block column k's tiles (kb + w + RW u, kb): issue their loads (out-of-range ones read 0)
  auto load_col = [&](int kb) {
    const int ntc = nt - kb;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int tl = w + RW * u;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = (kb + tl) * 16 + Mfma<T>::row(lane, r), gc = kb * 16 + (lane & 15);
        const bool in = tl < ntc && gr < n && gc < n;
        acc[u][r] = bload_sc1<T>(rAm, in ? (uint32_t)(((int64_t)gr * lda + gc) * sizeof(T)) : 0x80000000u);
      }
    }
  };
  lds_barrier();
  load_col(0);
  int first_fail = 0;
  for (int kb = 0; kb < nt; ++kb) {
    const int nrow = NR - kb * 16, ntc = nt - kb;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int tl = w + RW * u;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = (kb + tl) * 16 + Mfma<T>::row(lane, r), gc = kb * 16 + (lane & 15);
        if (tl < ntc && !(gr < n && gc < n)) acc[u][r] = gr == gc ? (T)1 : (T)0;   // padding past n
      }
    }
    // steps kb-3 .. kb-1 on this column, from L[:, kb-3 .. kb-1] in LDS (chol2_potrf_role's MFMA order)
#pragma unroll
    for (int back = 3; back >= 1; --back) {
      if (kb >= back) {
        const T* Pb = Ps0 + ((kb - back) % 3) * NR * CP;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int tl = w + RW * u;
          if (tl < ntc) {
            const int ra = (tl + back) * 16 + (lane & 15), rb = back * 16 + (lane & 15);
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
              const int kr = Mfma<T>::row(lane, s2);
              acc[u] = Mfma<T>::mma(-Pb[ra * CP + kr], Pb[rb * CP + kr], acc[u]);
            }
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int tl = w + RW * u;
      if (tl < ntc) {
#pragma unroll
        for (int r = 0; r < 4; ++r) colbuf[(tl * 16 + Mfma<T>::row(lane, r)) * CP + (lane & 15)] = acc[u][r];
      }
    }
    CHOL_STAMP(kb, 0);
    // block column kb+1 (from column 4 on: the update workgroup's steps <= kb-3 applied): its loads go out
    // now and land during the panel
    if (kb + 1 < nt) {
      if (kb + 1 >= 4) {
        bool seen = true;
        if (lane == 0) seen = poll_word<T>(hflag, kb - 2, nt);
        ok &= seen;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      load_col(kb + 1);
    }
    lds_barrier();
    CHOL_STAMP(kb, 1);
    T* Ps = Ps0 + (kb % 3) * NR * CP;
    if (w < (nrow + 47) / 48) {
      int lr;
      bool ident = false;
      if (lane < 16) {
        lr = lane;
      } else {
        const int slot = w * 48 + lane - 16;
        ident = slot >= nrow - 16 && slot < nrow;
        lr = ident ? slot - (nrow - 16) : 16 + slot;
      }
      const bool active = ident || lr < nrow;
      T a[16];
      {
        const T keep = (active && !ident) ? (T)1 : (T)0;
        const T* src = colbuf + min(lr, NR - 1) * CP;
#pragma unroll
        for (int c = 0; c < 16; ++c) a[c] = fma(src[c], keep, (ident && c == lr) ? (T)1 : (T)0);
      }
      unsigned int bad = 0;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const T d = readlane(a[j], j);
        bad |= (d > (T)0) ? 0u : (1u << j);
        T sj, inv;
        sqrt_recip(d, sj, inv);
        a[j] = (lane == j) ? sj : a[j] * inv;
#pragma unroll
        for (int c = j + 1; c < 16; ++c) a[c] = fma(-a[j], readlane(a[j], c), a[c]);
      }
      if (bad && first_fail == 0) {
        const int j0 = __builtin_ctz(bad);
        if (kb * 16 + j0 < n) first_fail = kb * 16 + j0 + 1;
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) a[c] = (lane < 16 && c > lane) ? (T)0 : a[c];
      if (ident || (active && (lane >= 16 || w == 0))) {
        T* dst = (ident ? LiT : Ps) + lr * CP;
#pragma unroll
        for (int c = 0; c < 16; ++c) dst[c] = a[c];
      }
    }
    // the stores of L[:, kb-1] had the whole panel to drain (and column kb+1's loads have landed): wait
    // for them here, where it is free, and raise the progress word
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (t == 0 && kb > 0)
      __hip_atomic_store(flag, kFlagTag + (unsigned long long)kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    CHOL_STAMP(kb, 2);
    // publish L[:, kb] (final output) and L_kk^-1 (= the final X[kb, kb]) write-through
    for (int idx = t; idx < nrow * 16; idx += RW * 64) {
      const int lr = idx >> 4, c = idx & 15;
      const int gr = kb * 16 + lr, gc = kb * 16 + c;
      if (gr < n && gc < n) bstore_sc1<T>(rAm, (uint32_t)(((int64_t)gr * lda + gc) * sizeof(T)), Ps[lr * CP + c]);
    }
    if (t < 256) {
      const int r = t >> 4, c = t & 15;
      const int gr = kb * 16 + r, gc = kb * 16 + c;
      if (gr < n && gc < n) bstore_sc1<T>(rXm, (uint32_t)(((int64_t)gr * ldx + gc) * sizeof(T)), LiT[c * CP + r]);
    }
    CHOL_STAMP(kb, 3);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  if (t == 0) {
    __hip_atomic_store(flag, kFlagTag + (unsigned long long)nt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(hflag, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // no reader left
    if (info) {
      if (info_first) info[mat] = first_fail ? first_fail + col_off : 0;
      else if (first_fail && info[mat] == 0) info[mat] = first_fail + col_off;
    }
  }
  if (lane == 0 && !ok) spin_gave_up(NMGP_STATUS_CHOL_SPIN);
}

template <typename T, int NTPW>
__device__ __attribute__((always_inline)) inline void chol7_update_role(T* Am, T* Xm, int n, int64_t lda,
                                                                        unsigned char* smem_raw) {
  using acc_t = typename Mfma<T>::acc_t;
  const int nt = (n + 15) >> 4, NR = nt * 16;
  T* Ps = (T*)smem_raw;                // NR x CP: L[:, j] (local rows)
  unsigned long long* flag = ctl_flag(Xm, n);
  unsigned long long* hflag = ctl_hflag(Xm, n);
  const __amdgpu_buffer_rsrc_t rAm = make_rsrc(Am, ((int64_t)(n - 1) * lda + n) * (int64_t)sizeof(T));
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  // the lower tiles of block columns >= 4 (ib >= jb >= 4), distributed over the waves
  const int nt4 = nt - 4, ntiles = nt4 > 0 ? nt4 * (nt4 + 1) / 2 : 0;
  int tij[NTPW];
  acc_t acc[NTPW];
#pragma unroll
  for (int u = 0; u < NTPW; ++u) {
    const int tt = w + RW * u;
    int i_ = -1, j_ = -1;
    if (tt < ntiles) {
      tri_decode(tt, i_, j_);
      i_ += 4;
      j_ += 4;
    }
    tij[u] = tt < ntiles ? (i_ << 8) | j_ : -1;
  }
#define IB7(u) (tij[u] < 0 ? -1 : (tij[u] >> 8))
#define JB7(u) (tij[u] < 0 ? -1 : (tij[u] & 255))
#pragma unroll
  for (int u = 0; u < NTPW; ++u) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gr = IB7(u) * 16 + Mfma<T>::row(lane, r), gc = JB7(u) * 16 + (lane & 15);
      const bool in = IB7(u) >= 0 && gr < n && gc < n;
      acc[u][r] = bload<T>(rAm, in ? (uint32_t)(((int64_t)gr * lda + gc) * sizeof(T)) : 0x80000000u);
    }
  }
#pragma unroll
  for (int u = 0; u < NTPW; ++u) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gr = IB7(u) * 16 + Mfma<T>::row(lane, r), gc = JB7(u) * 16 + (lane & 15);
      if (IB7(u) >= 0 && !(gr < n && gc < n)) acc[u][r] = gr == gc ? (T)1 : (T)0;   // padding past n
    }
  }
  bool ok = true;
  constexpr int PER = 256 * 16 / (RW * 64);
  for (int j = 0; j + 4 < nt; ++j) {
    const int nrow = NR - j * 16;
    if (t == 0) ok &= poll_word<T>(flag, j + 1, nt);              // L[:, j] published and drained
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    {
      T v[PER];
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int idx = t + q * RW * 64, lr = idx >> 4, c = idx & 15;
        const int gr = j * 16 + lr, gc = j * 16 + c;
        const uint32_t off =
            (idx < nrow * 16 && gr < n && gc < n) ? (uint32_t)(((int64_t)gr * lda + gc) * sizeof(T)) : 0x80000000u;
        v[q] = bload_sc1<T>(rAm, off);
      }
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int idx = t + q * RW * 64;
        if (idx < nrow * 16) Ps[(idx >> 4) * CP + (idx & 15)] = v[q];
      }
    }
    lds_barrier();
    // 1. block column j+4 first, then out to the factor workgroup
#pragma unroll
    for (int u = 0; u < NTPW; ++u) {
      if (JB7(u) == j + 4) {
        const int ra = __builtin_amdgcn_readfirstlane(IB7(u) - j) * 16 + (lane & 15);
        const int rb = 64 + (lane & 15);
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int kr = Mfma<T>::row(lane, s2);
          acc[u] = Mfma<T>::mma(-Ps[ra * CP + kr], Ps[rb * CP + kr], acc[u]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gr = IB7(u) * 16 + Mfma<T>::row(lane, r), gc = JB7(u) * 16 + (lane & 15);
          if (gr < n && gc < n) bstore_sc1<T>(rAm, (uint32_t)(((int64_t)gr * lda + gc) * sizeof(T)), acc[u][r]);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) __hip_atomic_store(hflag, kFlagTag + (unsigned long long)(j + 1), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    // 2. the columns beyond
#pragma unroll
    for (int u = 0; u < NTPW; ++u) {
      if (JB7(u) > j + 4) {
        const int ra = __builtin_amdgcn_readfirstlane(IB7(u) - j) * 16 + (lane & 15);
        const int rb = __builtin_amdgcn_readfirstlane(JB7(u) - j) * 16 + (lane & 15);
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int kr = Mfma<T>::row(lane, s2);
          acc[u] = Mfma<T>::mma(-Ps[ra * CP + kr], Ps[rb * CP + kr], acc[u]);
        }
      }
    }
    lds_barrier();                     // Ps is rewritten by the next step
  }
  if (!ok && t == 0) spin_gave_up(NMGP_STATUS_CHOL_SPIN);
#undef IB7
#undef JB7
}

template <typename T, int NTPW, int NTPW1, int NTPWU>
__global__ __launch_bounds__(RW * 64) void chol_inv7_kernel(T* A, int n, int64_t lda, int64_t strideA, T* X,
                                                            int64_t ldx, int64_t strideX, int32_t* info, int col_off,
                                                            int info_first) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int mat = blockIdx.x / 4, role = blockIdx.x - 4 * mat;
  T* Am = A + (int64_t)mat * strideA;
  T* Xm = X + (int64_t)mat * strideX;
  if (role == 0) {
    if (threadIdx.x == 0) __hip_atomic_store(ctl_done(Xm, n), kDoneTag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    chol7_factor_role<T>(Am, Xm, n, lda, ldx, info, col_off, info_first, mat, smem_raw);
  } else if (role == 1) {
    chol7_update_role<T, NTPWU>(Am, Xm, n, lda, smem_raw);
  } else {
    chol3_trtri_role<T, NTPW1, 3>(Am, Xm, n, lda, ldx, role - 2, smem_raw);
  }
}

// ------------------------------------------------------------------------------------------------
// Fused prior launch (nmgp_chol_tp_f64, round 6).  The DSVI step's critical path ran
//   RBF builders -> chol(v, t, L0, L1) -> v -> K_G22 builder -> chol(G) -> invG (T_G = K_G12 C_G^-T) ->
//   projG (P_G = T_G C_G^-1) -> quad_W
// with the t / L0 / L1 projections, the t-row and K_G12 on a side stream.  Here each chol launch carries, besides
// the four-role factorization of each matrix (chol_inv7_kernel's roles), TPR-row workgroups per prior with
// minibatch products ("rows" workgroups, tp_rows_role), fed by the factorization's own published data: block
// column kb of L and L_kk^-1 (the factor role's progress word) and block row kb of X = L^-1 (the inverse roles'
// xflag words, XPUB).  Each keeps R = its rows of K12 (built in registers, written out once) in MFMA accumulators
// and runs the right-looking triangular solve T = K12 L^-T one block column behind the factor:
// T(:, kb) = R(:, kb) L_kk^-T, then R(:, cb) -= T(:, kb) L(cb, kb)^T for cb > kb; and accumulates P = T X two
// block rows behind the inverse workgroups: P(:, cb) += T(:, kb) X(kb, cb), cb <= kb.  rows 2 first forms the
// rows' t-row sample ell_X (dsvi_trow_kernel's arithmetic) and builds Gibbs K12 rows from it.  (K22 is built
// outside: fp64 exp / sqrt / division chains on the few role workgroups cost 9-20 us per launch, measured.)
// The step loses the invG / projG products, the t-row and K12 builders and their graph hand-offs; T and P come out
// more accurate than the explicit-inverse products (substitution).  Role workgroups come first in the grid
// (in-order dispatch per XCD); rows workgroups only wait on them, never the reverse; the last of a matrix's
// readers re-arms its progress words.
constexpr int TPR = 32;             // minibatch rows per rows workgroup
constexpr int RB = TPR / 16;        // its row blocks
constexpr int CG = RW / RB;         // column groups of its waves (wave w: row block w % RB, columns w / RB + CG u)
constexpr int NU = 16 / CG;         // R / P tiles per wave (n <= 256)
// LDS below the staged per-index inputs: the roles' layout (chol_inv7_kernel's, with the third L buffer) or the row
// workgroups' (NR CP + 16 CP + 4 TPR CP + 16 * 257 + TPR doubles), whichever is larger
__host__ __device__ constexpr size_t chol_tp_roles_bytes(int n) {
  return (size_t)((4 * (((n + 15) >> 4) * 16) * CP + 16 * CP) > ((((n + 15) >> 4) * 16) * CP + 16 * CP + 4 * TPR * CP +
                                                                   16 * 257 + TPR)
                      ? (4 * (((n + 15) >> 4) * 16) * CP + 16 * CP)
                      : ((((n + 15) >> 4) * 16) * CP + 16 * CP + 4 * TPR * CP + 16 * 257 + TPR)) *
         sizeof(double);
}

struct TpDev {
  double* A;
  double* X;
  int32_t* info;
  int64_t lda, strideA, ldx, strideX;
  int n, batch, B, nct, ntp;
  double jitter;
  const double* Z;
  const double* ellZ;
  const double* x;
  const double* Pt;
  const double* Tt;
  const double* v;
  const double* zt;
  const double* hyp_t;
  double* ellX;
  double* var_t;
  int rows[4], tpm[4];
  int dbg;   // NMGP_TP_DBG bit 16: phase stamps (tools/chol_tp_probe.py)
  const double* hyp[4];
  double* K12[4];
  double* Tm[4];
  double* Pm[4];
  // fused K_G22 workgroups (nvg > 0; matrix 0 is Sigma_v): v = mu_v + L_v z_v, ell_Z = exp(v), K_G22 + jitter I
  int nvg;
  const double* vg_muv;
  const double* vg_z;
  double* vg_v;
  double* vg_ellZ;
  double* vg_K22;
};

// The Gibbs prior's K22 inside the launch that factors Sigma_v (round 6), pipelined behind the factorization: row
// block kb of v = mu_v + L_v z_v needs L_v's rows kb*16.., i.e. block columns 0..kb, so after matrix 0's factor role
// has published block column kb, every one of the nvg workgroups forms v[kb*16 .. kb*16+15] (two entries per wave,
// lanes over k: dsvi_vg22_kernel's sums) and then its share of the tiles (kb, J <= kb) of K_G22's lower 16 x 16 tiles
// (two tiles per pass, one per 256 threads; dsvi_vg22_kernel's element arithmetic).  What is left after the last
// column is one row block of tiles.  Workgroup 0 also writes v and ell_Z.  These workgroups are readers of matrix
// 0's progress word: the last of them and of its two inverse workgroups re-arms it.
__device__ __attribute__((always_inline)) inline void tp_vg_role(const TpDev& a, int g, unsigned char* smem_raw) {
  const int n = a.n, nt = (n + 15) >> 4;
  double* Xm = a.X;
  unsigned long long* flag = ctl_flag(Xm, n);
  unsigned long long* done = ctl_done(Xm, n);
  const __amdgpu_buffer_rsrc_t rAm = make_rsrc(a.A, ((int64_t)(n - 1) * a.lda + n) * (int64_t)sizeof(double));
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  double* vl = (double*)smem_raw;                 // v (n)
  int* s_ok = (int*)(vl + 256);
  const int half = t >> 8, r = (t & 255) >> 4, cc = t & 15;
  bool ok = true;
  for (int kb = 0; kb < nt; ++kb) {
    if (t == 0) {
      int good = 0;
      if (ok) {
        for (int spin = 0; spin < (1 << 22); ++spin) {
          const unsigned long long f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (f >= kFlagTag + (unsigned long long)(kb + 1) && f <= kFlagTag + (unsigned long long)nt) {
            good = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      *s_ok = good;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    ok = *s_ok != 0;
    // v[kb*16 + e], e = w, w + RW (RW = 8 waves: two entries each)
    for (int e = w; e < 16; e += RW) {
      const int c = kb * 16 + e;
      if (c < n) {
        double s = 0;
        for (int k = lane; k <= c; k += 64)
          s += bload_sc1<double>(rAm, (uint32_t)(((int64_t)c * a.lda + k) * (int64_t)sizeof(double))) * a.vg_z[k];
        s = wave_sum(s);
        if (lane == 0) {
          const double v = a.vg_muv[c] + s;
          vl[c] = v;
          if (g == 0) {
            a.vg_v[c] = v;
            a.vg_ellZ[c] = dexp(v);
          }
        }
      }
    }
    __syncthreads();
    // tiles (kb, J), J = 2 (g + nvg p) + half <= kb
    for (int J = 2 * g + half; J <= kb; J += 2 * a.nvg) {
      const int i = kb * 16 + r, j = J * 16 + cc;
      if (i < n && j < n) {
        const double lx = dexp(vl[i]), lz = dexp(vl[j]);
        double r2 = 0;
        const double dd = a.Z[i] / 1.0 - a.Z[j] / 1.0;
        r2 += dd * dd;
        const double S = lx * lx + lz * lz;
        const double C = dsqrt(2.0 * (lx * lz) / S);
        double k = 1.0 * C * dexp(-r2 / S);
        if (i == j) k += a.jitter;
        a.vg_K22[(int64_t)i * n + j] = k;
      }
    }
  }
  if (!ok && lane == 0) spin_gave_up(NMGP_STATUS_CHOL_SPIN);
  __syncthreads();
  if (t == 0) {
    const unsigned long long old = __hip_atomic_fetch_add(done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == kDoneTag + (unsigned long long)(2 + a.nvg - 1)) {
      __hip_atomic_store(flag, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ __attribute__((always_inline)) inline void tp_rows_role(const TpDev& a, int m, int rt,
                                                                   unsigned char* smem_raw) {
  using acc_t = f64x4;
  using MF = Mfma<double>;
  const int n = a.n, nt = (n + 15) >> 4, NR = nt * 16, B = a.B;
  constexpr int KP = 257;                // X-row pitch (n <= 256): compile-time, so LDS operand reads are one base
                                         // register + immediate offsets
  double* Ls = (double*)smem_raw;        // NR x CP: L[kb*16 + lr, kb*16 + c] (local rows)
  double* Li = Ls + NR * CP;             // 16 x CP: L_kk^-1
  double* Rs = Li + 16 * CP;             // TPR x CP: R(:, kb) (block column kb of the residual)
  double* Tc = Rs + TPR * CP;            // 3 x TPR x CP: T(:, kb), triple-buffered (P uses step kb - 2's)
  double* Xs = Tc + 3 * TPR * CP;        // 16 x KP: X[pk*16 + j, c], c <= pk*16 + j
  double* rowv = Xs + 16 * KP;           // TPR: ell_X of the rows (rows 2)
  double* Am = a.A + (int64_t)m * a.strideA;
  double* Xm = a.X + (int64_t)m * a.strideX;
  unsigned long long* flag = ctl_flag(Xm, n);
  unsigned long long* done = ctl_done(Xm, n);
  unsigned long long* xf0 = ctl_xflag(Xm, n, 0);
  unsigned long long* xf1 = ctl_xflag(Xm, n, 1);
  (void)xf0;
  const __amdgpu_buffer_rsrc_t rAm = make_rsrc(Am, ((int64_t)(n - 1) * a.lda + n) * (int64_t)sizeof(double));
  const __amdgpu_buffer_rsrc_t rXm = make_rsrc(Xm, ((int64_t)(n - 1) * a.ldx + n) * (int64_t)sizeof(double));
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int r0 = rt * TPR;
  const int mode = a.rows[m];
  double* K12 = a.K12[m];
  double* Tg = a.Tm[m];
  double* Pg = a.Pm[m];

  // 1. rows 2: the t-row sample of each row (JGP_S, code/utils.py:226-235), dsvi_trow_kernel's arithmetic; wave w
  //    takes rows w, w + 8, ... with all of their loads in flight together
  if (mode == 2) {
    const double s2t = dexp(a.hyp_t[0]);
    constexpr int RPW = TPR / RW;          // rows per wave
    constexpr int CPL = 256 / 64;          // columns per lane (n <= 256)
    double pv[RPW][CPL], tv[RPW][CPL], vv[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) vv[c] = (lane + 64 * c < n) ? a.v[lane + 64 * c] : 0.0;
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int r = min(r0 + w + RW * q, B - 1);
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int col = min(lane + 64 * c, n - 1);
        pv[q][c] = a.Pt[(int64_t)r * n + col];
        tv[q][c] = a.Tt[(int64_t)r * n + col];
      }
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      double mean = 0, qq = 0;
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        if (lane + 64 * c < n) {
          mean += pv[q][c] * vv[c];
          const double tt = tv[q][c];
          qq += (double)(tt * tt);
        }
      }
      mean = wave_sum(mean);
      qq = wave_sum(qq);
      const int i = w + RW * q, r = r0 + i;
      const double var = s2t - qq;
      const double lx = r < B ? dexp(mean + a.zt[r] * dsqrt(var + a.jitter)) : 1.0;
      if (lane == 0) {
        rowv[i] = lx;
        if (r < B) {
          a.ellX[r] = lx;
          a.var_t[r] = var;
        }
      }
    }
    __syncthreads();
  }

  // 2. R = this workgroup's rows of K12, built in the accumulator layout (pairwise_kernel's arithmetic; Gibbs with
  //    one division, tp_gibbs) and written out; straight-line, clamped indices, masked at the end.  Wave w owns the
  //    tiles (rb = w % RB, cb = w / RB + CG u), u < NU, of R and of P.
  const int rbw = w % RB, cgw = w / RB;
  acc_t R[NU], P[NU];
  double s2 = 1.0, ls = 1.0;
  if (mode == 1) {
    s2 = dexp(a.hyp[m][0]);
    ls = dexp(a.hyp[m][1]);
  }
  double* uz = (double*)(smem_raw + chol_tp_roles_bytes(n));
  double* ul = uz + 256;
  tp_stage(uz, ul, mode, a.Z, a.ellZ, ls, n);
  double xu[4], lxr[4];                 // x_i / ls (RBF) or x_i / 1 (Gibbs), ell_X of this lane's four rows
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = rbw * 16 + MF::row(lane, r);
    xu[r] = a.x[min(r0 + i, B - 1)] / ls;
    lxr[r] = mode == 2 ? rowv[i] : 1.0;
  }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int cb = cgw + CG * u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int col = min(cb * 16 + (lane & 15), n - 1);
      const double dd = xu[r] - uz[col];
      double r2 = 0;
      r2 += dd * dd;
      R[u][r] = mode == 1 ? dexp(-0.5 * r2) * s2 : tp_gibbs(r2, lxr[r], ul[col]);
      P[u][r] = 0;
    }
  }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int cb = cgw + CG * u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + rbw * 16 + MF::row(lane, r), col = cb * 16 + (lane & 15);
      const bool in = row < B && col < n;
      R[u][r] = in ? R[u][r] : 0.0;
      if (in) K12[(int64_t)row * n + col] = R[u][r];
    }
  }

  TP_STAMP((a.dbg & 16) != 0, 2);
  // 3. one step per block column of the factorization.  Step kb: wait for L[:, kb] / L_kk^-1 (factor) and X row
  //    block kb - 1 (both inverse workgroups: one poll loop reading all three words), issue their loads, and while
  //    they are in flight add step kb - 2's P product (X row kb - 2 and T(:, kb - 2) are in LDS); then T(:, kb) and
  //    the R update.  T is triple-buffered for that lag.
  bool ok = true;
  constexpr int PER = 256 * 16 / (RW * 64);   // elements per thread of a 256 x 16 block column / 16 x 256 block row
  auto poll3 = [&](int nf, int nx) -> bool {  // flag >= nf and both X-row words >= nx (nx == 0: not needed)
    for (int spin = 0; spin < (1 << 22); ++spin) {
      const unsigned long long f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long x0 = nx ? __hip_atomic_load(xf0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
      const unsigned long long x1 = nx ? __hip_atomic_load(xf1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
      const unsigned long long lo = kFlagTag, hi = kFlagTag + (unsigned long long)nt;
      const bool fok = nf == 0 || (f >= lo + (unsigned long long)nf && f <= hi);
      const bool xok = nx == 0 || (x0 >= lo + (unsigned long long)nx && x0 <= hi && x1 >= lo + (unsigned long long)nx &&
                                   x1 <= hi);
      if (fok && xok) return true;
      __builtin_amdgcn_s_sleep(1);
    }
    return false;
  };
  auto load_x_row = [&](int pk, double (&xv)[PER]) {   // X[pk*16 + j, c] for c <= pk*16 + j (lower)
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int idx = t + q * RW * 64, j = idx >> 8, c = idx & 255;
      const int gr = pk * 16 + j;
      const bool in = c < NR && gr < n && c < n && c <= gr;
      xv[q] = bload_sc1<double>(rXm, in ? (uint32_t)(((int64_t)gr * a.ldx + c) * sizeof(double)) : 0x80000000u);
    }
  };
  auto store_x_row = [&](const double (&xv)[PER], int pk) {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int idx = t + q * RW * 64, j = idx >> 8, c = idx & 255;
      if (c < (pk + 1) * 16) Xs[j * KP + c] = xv[q];
    }
  };
  auto p_update = [&](int pk) {    // P(:, cb) += T(:, pk) X(pk, cb), cb <= pk
    const double* Tp = Tc + (pk % 3) * TPR * CP;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int cb = cgw + CG * u;
      if (cb <= pk) {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int kk = s2 * 4 + (lane >> 4);
          P[u] = MF::mma(Tp[(rbw * 16 + (lane & 15)) * CP + kk], Xs[kk * KP + cb * 16 + (lane & 15)], P[u]);
        }
      }
      // (one tile's operands in flight at a time: hoisting all tiles' LDS reads spilled the accumulators)
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  for (int kb = 0; kb < nt; ++kb) {
    const int nrow = NR - kb * 16;
    // (bounded waits, and none after one gave up: a lost role costs wrong output and a status bit, not minutes)
    if (t == 0 && ok) ok = poll3(kb + 1, kb);
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double lv[PER], xv[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int idx = t + q * RW * 64, lr = idx >> 4, c = idx & 15;
      const int gr = kb * 16 + lr, gc = kb * 16 + c;
      const uint32_t off =
          (idx < nrow * 16 && gr < n && gc < n) ? (uint32_t)(((int64_t)gr * a.lda + gc) * sizeof(double)) : 0x80000000u;
      lv[q] = bload_sc1<double>(rAm, off);
    }
    double li = 0;
    if (t < 256) {
      const int r = t >> 4, c = t & 15;
      const int gr = kb * 16 + r, gc = kb * 16 + c;
      const uint32_t off = (gr < n && gc < n) ? (uint32_t)(((int64_t)gr * a.ldx + gc) * sizeof(double)) : 0x80000000u;
      li = bload_sc1<double>(rXm, off);
    }
    if (kb > 0) load_x_row(kb - 1, xv);
    if (kb >= 2) p_update(kb - 2);      // under the loads
    lds_barrier();                      // every wave is done reading the previous step's Rs / Ls / Li / Xs
    if (t < 256) {
      const int r = t >> 4, c = t & 15, gr = kb * 16 + r, gc = kb * 16 + c;
      if (gr >= n || gc >= n) li = (gr == gc) ? 1.0 : 0.0;      // padded identity past n
      Li[r * CP + c] = li;
    }
    // R(:, kb) to LDS (its owner waves)
    if (cgw == kb % CG) {
#pragma unroll
      for (int u = 0; u < NU; ++u)
        if (u == kb / CG) {
#pragma unroll
          for (int r = 0; r < 4; ++r) Rs[(rbw * 16 + MF::row(lane, r)) * CP + (lane & 15)] = R[u][r];
        }
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int idx = t + q * RW * 64;
      if (idx < nrow * 16) Ls[(idx >> 4) * CP + (idx & 15)] = lv[q];
    }
    if (kb > 0) store_x_row(xv, kb - 1);
    lds_barrier();
    // T(:, kb) = R(:, kb) L_kk^-T (waves 0 .. RB-1, one row block each) -> LDS and out
    double* Tk = Tc + (kb % 3) * TPR * CP;
    if (w < RB) {
      acc_t tacc = {0, 0, 0, 0};
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const int kk = s2 * 4 + (lane >> 4);
        tacc = MF::mma(Rs[(w * 16 + (lane & 15)) * CP + kk], Li[(lane & 15) * CP + kk], tacc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = w * 16 + MF::row(lane, r), row = r0 + i, col = kb * 16 + (lane & 15);
        Tk[i * CP + (lane & 15)] = tacc[r];
        if (row < B && col < n) Tg[(int64_t)row * n + col] = tacc[r];
      }
    }
    lds_barrier();
    // R(:, cb) -= T(:, kb) L(cb, kb)^T, cb > kb
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int cb = cgw + CG * u;
      if (cb > kb && cb < nt) {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int kk = s2 * 4 + (lane >> 4);
          R[u] = MF::mma(-Tk[(rbw * 16 + (lane & 15)) * CP + kk], Ls[((cb - kb) * 16 + (lane & 15)) * CP + kk], R[u]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  TP_STAMP((a.dbg & 16) != 0, 3);
  // the last two P products: X row nt - 2 is in LDS; X row nt - 1 once both inverse workgroups are done
  if (nt >= 2) p_update(nt - 2);
  if (t == 0 && ok) ok = poll3(0, nt);
  TP_STAMP((a.dbg & 16) != 0, 4);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  {
    double xv[PER];
    load_x_row(nt - 1, xv);
    lds_barrier();
    store_x_row(xv, nt - 1);
  }
  lds_barrier();
  p_update(nt - 1);
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int cb = cgw + CG * u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + rbw * 16 + MF::row(lane, r), col = cb * 16 + (lane & 15);
      if (row < B && col < n) Pg[(int64_t)row * n + col] = P[u][r];
    }
  }
  if (!ok && lane == 0) spin_gave_up(NMGP_STATUS_CHOL_SPIN);
  __syncthreads();
  if (t == 0) {
    const int nfin = 2 + a.nct;
    const unsigned long long old = __hip_atomic_fetch_add(done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == kDoneTag + (unsigned long long)(nfin - 1)) {
      __hip_atomic_store(flag, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      tp_clear_words(Xm, n);
      __hip_atomic_store(done, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int NTPW1, int NTPWU>
__global__ __launch_bounds__(RW * 64) void chol_tp_kernel(TpDev a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int nroles = 4 * a.batch;
  const bool tr = (a.dbg & 16) != 0;
  TP_STAMP(tr, 0);
  if ((int)blockIdx.x < nroles) {
    const int mat = blockIdx.x / 4, role = blockIdx.x - 4 * mat;
    double* Am = a.A + (int64_t)mat * a.strideA;
    double* Xm = a.X + (int64_t)mat * a.strideX;
    // a matrix without row workgroups runs chol_inv7_kernel's roles; with them, its inverse workgroups publish the
    // X rows (XPUB) and count the row workgroups among the readers of its progress words
    if (role == 0) {
      if (threadIdx.x == 0) __hip_atomic_store(ctl_done(Xm, a.n), kDoneTag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      chol7_factor_role<double>(Am, Xm, a.n, a.lda, a.ldx, a.info, 0, 1, mat, smem_raw);
    } else if (role == 1) {
      chol7_update_role<double, NTPWU>(Am, Xm, a.n, a.lda, smem_raw);
    } else if (a.rows[mat]) {
      chol3_trtri_role<double, NTPW1, 5, true>(Am, Xm, a.n, a.lda, a.ldx, role - 2, smem_raw, 2 + a.nct);
    } else {
      // (matrix 0 with the fused K_G22 workgroups: they are readers of its progress word too)
      chol3_trtri_role<double, NTPW1, 5>(Am, Xm, a.n, a.lda, a.ldx, role - 2, smem_raw, mat == 0 ? 2 + a.nvg : 2);
    }
  } else if ((int)blockIdx.x < nroles + a.ntp * a.nct) {
    const int c = blockIdx.x - nroles, k = c / a.nct;
    tp_rows_role(a, a.tpm[k], c - k * a.nct, smem_raw);
  } else {
    // (after the row workgroups: dispatched last, they never take a CU a row workgroup is waiting for)
    tp_vg_role(a, blockIdx.x - nroles - a.ntp * a.nct, smem_raw);
  }
  TP_STAMP(tr, 1);
}

static size_t chol_tp_smem(int n) {
  // the roles' layout (chol_inv7_kernel's, >= the row workgroups' NR CP + 16 CP + 4 TPR CP + 16 * 257 + TPR doubles),
  // then the staged per-index inputs uz / ul (2 x 256 doubles)
  return chol_tp_roles_bytes(n) + 2 * 256 * sizeof(double);
}

template <int NTPW1, int NTPWU>
static void chol_tp_go(const TpDev& a, unsigned grid, size_t sm, hipStream_t s) {
  static std::once_flag once;
  std::call_once(once, [] {
    (void)hipFuncSetAttribute((const void*)chol_tp_kernel<NTPW1, NTPWU>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
  });
  hipLaunchKernelGGL((chol_tp_kernel<NTPW1, NTPWU>), dim3(grid), dim3(RW * 64), sm, s, a);
}

static int chol_tp_launch(const nmgp_chol_tp_args* h, hipStream_t s) {
  if (h == nullptr) return -1;
  const nmgp_chol_tp_args& g = *h;
  if (!g.A || !g.X || g.n < 128 || g.n > 256 || g.lda < g.n || g.ldx < g.n || g.batch < 1 || g.batch > 4 ||
      g.B < 0 || g.B > 4096 || g.strideA < 0 || g.strideX < 0 || !g.info)
    return -1;
  TpDev a{};
  a.A = g.A;
  a.X = g.X;
  a.info = g.info;
  a.lda = g.lda;
  a.strideA = g.strideA;
  a.ldx = g.ldx;
  a.strideX = g.strideX;
  a.n = (int)g.n;
  a.batch = (int)g.batch;
  a.B = (int)g.B;
  a.jitter = g.jitter;
  a.Z = g.Z;
  a.ellZ = g.ellZ;
  a.x = g.x;
  a.Pt = g.Pt;
  a.Tt = g.Tt;
  a.v = g.v;
  a.zt = g.zt;
  a.hyp_t = g.hyp_t;
  a.ellX = g.ellX;
  a.var_t = g.var_t;
  for (int m = 0; m < a.batch; ++m) {
    const nmgp_chol_tp_mat& mt = g.mats[m];
    if (mt.reserved != 0 || mt.rows < 0 || mt.rows > 2) return -1;
    if (mt.rows && (!mt.K12 || !mt.T || !mt.P || !g.x || !g.Z)) return -1;
    if (mt.rows == 1 && !mt.hyp) return -1;
    if (mt.rows == 2 && (!g.Pt || !g.Tt || !g.v || !g.zt || !g.hyp_t || !g.ellX || !g.var_t || !g.ellZ)) return -1;
    a.rows[m] = g.B > 0 ? mt.rows : 0;
    a.hyp[m] = mt.hyp;
    a.K12[m] = mt.K12;
    a.Tm[m] = mt.T;
    a.Pm[m] = mt.P;
    if (a.rows[m]) a.tpm[a.ntp++] = m;
  }
  a.nct = g.B > 0 ? (int)((g.B + TPR - 1) / TPR) : 0;
  a.dbg = getenv("NMGP_TP_DBG") ? atoi(getenv("NMGP_TP_DBG")) : 0;
  if (g.vg_wgs < 0 || g.vg_wgs > 64) return -1;
  if (g.vg_wgs > 0) {
    if (!g.vg_muv || !g.vg_z || !g.vg_v || !g.vg_ellZ || !g.vg_K22 || !g.Z || a.rows[0] != 0) return -1;
    a.nvg = (int)g.vg_wgs;
    a.vg_muv = g.vg_muv;
    a.vg_z = g.vg_z;
    a.vg_v = g.vg_v;
    a.vg_ellZ = g.vg_ellZ;
    a.vg_K22 = g.vg_K22;
  }
  const unsigned grid = (unsigned)(4 * a.batch + a.nvg + a.ntp * a.nct);
  const size_t sm = chol_tp_smem(a.n);
  const int nt = (a.n + 15) >> 4, ntiles = nt * (nt + 1) / 2;
  if (ntiles <= RW * 9)
    chol_tp_go<5, 4>(a, grid, sm, s);
  else
    chol_tp_go<9, 10>(a, grid, sm, s);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

template <typename T, int NTPW>
__global__ __launch_bounds__(RW * 64) void chol_inv2_kernel(T* A, int n, int64_t lda, int64_t strideA, T* X,
                                                            int64_t ldx, int64_t strideX, int32_t* info, int col_off,
                                                            int info_first) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int mat = blockIdx.x >> 1;
  T* Am = A + (int64_t)mat * strideA;
  T* Xm = X + (int64_t)mat * strideX;
  // separate functions: with one shared tile set the two roles' live ranges merged past the
  // register file
  if ((blockIdx.x & 1) == 0)
    chol2_potrf_role<T, NTPW>(Am, Xm, n, lda, ldx, info, col_off, info_first, mat, smem_raw);
  else
    chol2_trtri_role<T, NTPW>(Am, Xm, n, lda, ldx, info, col_off, info_first, mat, smem_raw);
}

template <typename T> static size_t chol_inv_smem(int n) {
  const int nt = (n + 15) >> 4;
  return (size_t)(3 * nt * 16 * CP + 16 * CP) * sizeof(T);
}

template <typename T> static size_t potrf_smem(int n) {
  const int nt = (n + 15) >> 4;
  return (size_t)(16 * CP + 16 + nt * 16 * CP) * sizeof(T) + 16;
}
template <typename T> static size_t trtri_smem(int n) {
  const int nt = (n + 15) >> 4;
  return (size_t)(nt * 16 * CP + nt * 256) * sizeof(T);
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
  hipLaunchKernelGGL(potrf_kernel<T>, dim3((unsigned)batch), dim3(CT), sm, s, A, (int)n, lda, strideA, info);
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
  hipLaunchKernelGGL(trtri_kernel<T>, dim3((unsigned)batch), dim3(CT), sm, s, L, (int)n, ldl, strideL, X, ldx,
                     strideX);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

template <typename T, int NTPW>
static void chol_inv_go(T* A, int n, int64_t lda, int64_t sA, T* X, int64_t ldx, int64_t sX, int64_t batch,
                        int32_t* info, size_t sm, hipStream_t s, int col_off, int info_first) {
  static bool attr_done = false;
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)chol_inv_kernel<T, NTPW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr_done = true;
  }
  hipLaunchKernelGGL((chol_inv_kernel<T, NTPW>), dim3((unsigned)batch), dim3(RW * 64), sm, s, A, n, lda, sA, X, ldx,
                     sX, info, col_off, info_first);
}

// one diagonal block (n <= 256) with the fused register-resident kernel
template <typename T, int NTPW>
static void chol_inv2_go(T* A, int n, int64_t lda, int64_t sA, T* X, int64_t ldx, int64_t sX, int64_t batch,
                         int32_t* info, size_t sm, hipStream_t s, int col_off, int info_first) {
  static bool attr_done = false;
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)chol_inv2_kernel<T, NTPW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr_done = true;
  }
  hipLaunchKernelGGL((chol_inv2_kernel<T, NTPW>), dim3((unsigned)(2 * batch)), dim3(RW * 64), sm, s, A, n, lda, sA, X,
                     ldx, sX, info, col_off, info_first);
}

// Two-role split pays from n = 32 up; its workgroup pairs must be co-resident, so a launch holds at
// most 128 matrices (256 workgroups, one per CU).  The three-role split (inverse over two
// workgroups) for up to 85 matrices.
static bool use_two_role(int n, int64_t batch) { return n >= 32 && n <= 256 && batch <= 128; }
static bool use_three_role(int n, int64_t batch) {
  static int off = -1;
  if (off < 0) off = getenv("NMGP_CHOL_TWO_ROLE") ? 1 : 0;
  return !off && n >= 128 && n <= 256 && batch <= 85;
}

template <typename T, int NTPW, int NTPW1>
static void chol_inv3_go(T* A, int n, int64_t lda, int64_t sA, T* X, int64_t ldx, int64_t sX, int64_t batch,
                         int32_t* info, size_t sm, hipStream_t s, int col_off, int info_first) {
  static bool attr_done = false;
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)chol_inv3_kernel<T, NTPW, NTPW1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr_done = true;
  }
  hipLaunchKernelGGL((chol_inv3_kernel<T, NTPW, NTPW1>), dim3((unsigned)(3 * batch)), dim3(RW * 64), sm, s, A, n, lda,
                     sA, X, ldx, sX, info, col_off, info_first);
}

template <typename T, int NTPW1, int NTPWU>
static void chol_inv7_go(T* A, int n, int64_t lda, int64_t sA, T* X, int64_t ldx, int64_t sX, int64_t batch,
                         int32_t* info, size_t sm, hipStream_t s, int col_off, int info_first) {
  static bool attr_done = false;
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)chol_inv7_kernel<T, 1, NTPW1, NTPWU>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_done = true;
  }
  hipLaunchKernelGGL((chol_inv7_kernel<T, 1, NTPW1, NTPWU>), dim3((unsigned)(4 * batch)), dim3(RW * 64), sm, s, A, n,
                     lda, sA, X, ldx, sX, info, col_off, info_first);
}

// Four-role kernel (separate update workgroup): the default from n = 192 (at n = 256 f64: 85-88 us against
// the three-role kernel's 95-97 us per launch, PM2.5 step 1317-1320 -> 1339-1381 it/s in an A/B on the box;
// at n = 128 f32 it is slower, 31 against 27 us: the update workgroup has too few columns to run ahead).
// NMGP_CHOL_4ROLE=0 / 1 forces it off / on for 128 <= n <= 256 (read per launch: tests switch it
// in-process).  Its four workgroups per matrix must be co-resident: at most 64 matrices per launch.
static bool use_four_role(int n, int64_t batch) {
  if (n < 128 || n > 256 || batch > 64) return false;
  const char* e = getenv("NMGP_CHOL_4ROLE");
  if (e) return atoi(e) != 0;
  return n >= 192;
}

// the multi-role kernels keep 64-bit control words in X's row 0: f32 needs them 8-byte aligned
template <typename T> static bool chol_ctl_ok(int n, const T* X, int64_t sX) {
  if (sizeof(T) == 8) return true;
  static int off = -1;
  if (off < 0) off = getenv("NMGP_CHOL_F32_ROLES") && atoi(getenv("NMGP_CHOL_F32_ROLES")) == 0 ? 1 : 0;
  return !off && n % 2 == 0 && ((uintptr_t)X % 8) == 0 && sX % 2 == 0;
}

template <typename T>
static int chol_inv_small(T* A, int n, int64_t lda, int64_t sA, T* X, int64_t ldx, int64_t sX, int64_t batch,
                          int32_t* info, hipStream_t s, int col_off, int info_first, bool two_role = true,
                          size_t sm_min = 0) {
  const int nt = (n + 15) >> 4, ntiles = nt * (nt + 1) / 2;
  const size_t sm = chol_inv_smem<T>(n) > sm_min ? chol_inv_smem<T>(n) : sm_min;
  // multi-role kernels (f64 always; f32 when the control words can be 8-byte aligned, round 2)
  if (chol_ctl_ok<T>(n, X, sX)) {
    if (two_role && use_four_role(n, batch) && !getenv("NMGP_CHOL_FUSED1")) {
      const size_t sm7 = sm + (size_t)(((n + 15) >> 4) * 16 * CP) * sizeof(T);   // + the third L buffer
      // inverse-role tiles as the three-role kernel's thresholds; update-role tiles: (nt-4)(nt-3)/2 <= RW*10
      if (ntiles <= RW * 5)
        chol_inv7_go<T, 3, 2>(A, n, lda, sA, X, ldx, sX, batch, info, sm7, s, col_off, info_first);
      else if (ntiles <= RW * 9)
        chol_inv7_go<T, 5, 4>(A, n, lda, sA, X, ldx, sX, batch, info, sm7, s, col_off, info_first);
      else
        chol_inv7_go<T, 9, 10>(A, n, lda, sA, X, ldx, sX, batch, info, sm7, s, col_off, info_first);
      NMGP_CHECK_LAUNCH();
      return NMGP_OK;
    }
    if (two_role && use_three_role(n, batch) && !getenv("NMGP_CHOL_FUSED1")) {
      if (ntiles <= RW * 5)
        chol_inv3_go<T, 5, 3>(A, n, lda, sA, X, ldx, sX, batch, info, sm, s, col_off, info_first);
      else if (ntiles <= RW * 9)
        chol_inv3_go<T, 9, 5>(A, n, lda, sA, X, ldx, sX, batch, info, sm, s, col_off, info_first);
      else
        chol_inv3_go<T, 17, 9>(A, n, lda, sA, X, ldx, sX, batch, info, sm, s, col_off, info_first);
      NMGP_CHECK_LAUNCH();
      return NMGP_OK;
    }
    if (two_role && use_two_role(n, batch) && !getenv("NMGP_CHOL_FUSED1")) {
      if (ntiles <= RW * 3)
        chol_inv2_go<T, 3>(A, n, lda, sA, X, ldx, sX, batch, info, sm, s, col_off, info_first);
      else if (ntiles <= RW * 5)
        chol_inv2_go<T, 5>(A, n, lda, sA, X, ldx, sX, batch, info, sm, s, col_off, info_first);
      else if (ntiles <= RW * 9)
        chol_inv2_go<T, 9>(A, n, lda, sA, X, ldx, sX, batch, info, sm, s, col_off, info_first);
      else
        chol_inv2_go<T, 17>(A, n, lda, sA, X, ldx, sX, batch, info, sm, s, col_off, info_first);
      NMGP_CHECK_LAUNCH();
      return NMGP_OK;
    }
  }
  if (ntiles <= RW * 1)
    chol_inv_go<T, 1>(A, n, lda, sA, X, ldx, sX, batch, info, sm, s, col_off, info_first);
  else if (ntiles <= RW * 3)
    chol_inv_go<T, 3>(A, n, lda, sA, X, ldx, sX, batch, info, sm, s, col_off, info_first);
  else if (ntiles <= RW * 5)
    chol_inv_go<T, 5>(A, n, lda, sA, X, ldx, sX, batch, info, sm, s, col_off, info_first);
  else if (ntiles <= RW * 9)
    chol_inv_go<T, 9>(A, n, lda, sA, X, ldx, sX, batch, info, sm, s, col_off, info_first);
  else
    chol_inv_go<T, 17>(A, n, lda, sA, X, ldx, sX, batch, info, sm, s, col_off, info_first);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

// rows x cols block copy / zero, batched over blockIdx.y (the blocked path's scratch moves)
template <typename T>
__global__ __launch_bounds__(256) void block_copy_kernel(const T* src, int64_t lds, int64_t sS, T* dst, int64_t ldd,
                                                         int64_t sD, int rows, int cols) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)rows * cols) return;
  const int r = (int)(idx / cols), c = (int)(idx - (int64_t)r * cols);
  const int64_t b = blockIdx.y;
  dst[b * sD + (int64_t)r * ldd + c] = src ? src[b * sS + (int64_t)r * lds + c] : (T)0;
}
// 16-byte form (cols, strides and pointers multiples of 16 bytes): four f32 / two f64 per thread.  The
// recursion's block zeroing / staging moves 10-20 GB per ECoG step, which the scalar form streamed at ~1.6 TB/s.
template <typename T>
__global__ __launch_bounds__(256) void block_copy_v_kernel(const T* src, int64_t lds, int64_t sS, T* dst, int64_t ldd,
                                                           int64_t sD, int rows, int cols) {
  constexpr int V = 16 / (int)sizeof(T);
  struct alignas(16) Vec { T e[V]; };
  const int cv = cols / V;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * cv) return;
  const int r = idx / cv, c = (idx - r * cv) * V;
  const int64_t b = blockIdx.y;
  Vec v;
  if (src) {
    v = *(const Vec*)(src + b * sS + (int64_t)r * lds + c);
  } else {
#pragma unroll
    for (int e = 0; e < V; ++e) v.e[e] = (T)0;
  }
  *(Vec*)(dst + b * sD + (int64_t)r * ldd + c) = v;
}

template <typename T>
static int block_copy(const T* src, int64_t lds, int64_t sS, T* dst, int64_t ldd, int64_t sD, int rows, int cols,
                      int64_t batch, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return NMGP_OK;
  constexpr int V = 16 / (int)sizeof(T);
  const bool vec = cols % V == 0 && ldd % V == 0 && sD % V == 0 && ((uintptr_t)dst & 15) == 0 &&
                   (src == nullptr || (lds % V == 0 && sS % V == 0 && ((uintptr_t)src & 15) == 0)) &&
                   (int64_t)rows * (cols / V) < (1LL << 31) - 256;
  if (vec) {
    const int64_t nv = ((int64_t)rows * (cols / V) + 255) / 256;
    hipLaunchKernelGGL(block_copy_v_kernel<T>, dim3((unsigned)nv, (unsigned)batch), dim3(256), 0, s, src, lds, sS, dst,
                       ldd, sD, rows, cols);
    NMGP_CHECK_LAUNCH();
    return NMGP_OK;
  }
  const int64_t nb = ((int64_t)rows * cols + 255) / 256;
  hipLaunchKernelGGL(block_copy_kernel<T>, dim3((unsigned)nb, (unsigned)batch), dim3(256), 0, s, src, lds, sS, dst, ldd,
                     sD, rows, cols);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

static nmgp_gemm_desc gdesc(const void* A, int64_t sAi, int64_t sAk, const void* B, int64_t sBk, int64_t sBj, void* C,
                            int64_t sCi, int64_t sCj, int m, int n, int k, int flags, double alpha, double beta,
                            int64_t sAb, int64_t sBb, int64_t sCb, int64_t batch) {
  nmgp_gemm_desc d{};
  d.A = A; d.B = B; d.C = C;
  d.sA_i = sAi; d.sA_k = sAk; d.sB_k = sBk; d.sB_j = sBj; d.sC_i = sCi; d.sC_j = sCj;
  d.m = m; d.n = n; d.k = k; d.flags = flags; d.row_seg = -1; d.k_seg = -1;
  d.alpha = alpha; d.beta = beta;
  d.sA_b = sAb; d.sB_b = sBb; d.sC_b = sCb; d.batch = (int)batch;
  return d;
}

int gemm_big_f32(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kcontig, float* C, int64_t sCi,
                 int64_t sCj, int m, int n, int k, int flags, float alpha, float beta, int64_t sAb, int64_t sBb,
                 int64_t sCb, int batch, void* ws, hipStream_t s);
size_t gemm_big_ws_bytes();
int potrf_step_f32(float* P, float* C, const float* X, int64_t lda, int n2, int nb, int c1, int32_t* flag,
                   hipStream_t s);
int potrf_strip_f32(const float* L, float* C, int64_t lda, int m, int c1, hipStream_t s);

// f32 recursion (same algebra as chol_inv_rec below) with the products on the 128x128 MFMA kernel
// of gemm_big.hip, split-K into `ws` where the tile grid would not fill the chip.
static int chol_split_point(int n) {
  int n1 = ((n / 2 + 127) / 128) * 128;
  return n1 >= n ? n - 128 : n1;
}
// full = 0 (the top level of the KL L-bar solve form, nmgp_chol_blockinv_batched_f32): the factor and the inverses
// X11, X22 of the split's two diagonal blocks only -- X21 = -X22 L21 X11 (two products) is not formed.  The factor's
// off-diagonal block L21 is then written to X21 (its place in X is free) instead of A21: no staging copy of A21 and
// no zeroing of A12 (the solve form reads neither; A21 keeps the input block as scratch)
static int chol_inv_rec_big(float* A, int n, int64_t lda, int64_t sA, float* X, int64_t ldx, int64_t sX,
                            int64_t batch, int32_t* info, hipStream_t s, int col_off, void* ws, int full = 1) {
  // leaves up to 256 wide on the fused register-resident kernels (round 6: ECoG 0.2734 -> 0.2707 s, HCP 59.5 -> 60.1
  // it/s against 128-wide leaves, profiles/r06zj_rec_leaf_ab.txt); NMGP_REC_LEAF=128 keeps the deeper recursion
  static const int leaf = [] { const char* e = getenv("NMGP_REC_LEAF"); return e && atoi(e) == 128 ? 128 : 256; }();
  if (n <= leaf) return chol_inv_small<float>(A, n, lda, sA, X, ldx, sX, batch, info, s, col_off, col_off == 0);
  const int n1 = chol_split_point(n);
  const int n2 = n - n1, nb = (int)batch;
  int rc;
  float* A21 = A + (int64_t)n1 * lda;
  float* A22 = A21 + n1;
  float* X21 = X + (int64_t)n1 * ldx;
  float* X22 = X21 + n1;
  float* X12 = X + n1;
  if ((rc = chol_inv_rec_big(A, n1, lda, sA, X, ldx, sX, batch, info, s, col_off, ws)) != NMGP_OK) return rc;
  if (!full) {
    // L21 = A21 X11^T into X21, A22 -= L21 L21^T from there, then the second diagonal block
    if ((rc = gemm_big_f32(A21, lda, X, ldx, 1, X21, ldx, 1, n2, n1, n1, NMGP_B_UPPER, 1.f, 0.f, sA, sX, sX, nb, ws,
                           s)) != NMGP_OK)
      return rc;
    if ((rc = gemm_big_f32(X21, ldx, X21, ldx, 1, A22, lda, 1, n2, n2, n1, NMGP_OUT_LOWER, -1.f, 1.f, sX, sX, sA, nb,
                           ws, s)) != NMGP_OK)
      return rc;
    return chol_inv_rec_big(A22, n2, lda, sA, X22, ldx, sX, batch, info, s, col_off + n1, ws);
  }
  if ((rc = block_copy<float>(A21, lda, sA, X21, ldx, sX, n2, n1, batch, s)) != NMGP_OK) return rc;
  // L21 = A21 X11^T      (op(B)(k,j) = X11[j][k], upper)
  if ((rc = gemm_big_f32(X21, ldx, X, ldx, 1, A21, lda, 1, n2, n1, n1, NMGP_B_UPPER, 1.f, 0.f, sX, sX, sA, nb, ws,
                         s)) != NMGP_OK)
    return rc;
  // A22 -= L21 L21^T     (lower tiles only: the trailing SYRK)
  if ((rc = gemm_big_f32(A21, lda, A21, lda, 1, A22, lda, 1, n2, n2, n1, NMGP_OUT_LOWER, -1.f, 1.f, sA, sA, sA, nb,
                         ws, s)) != NMGP_OK)
    return rc;
  if ((rc = block_copy<float>(nullptr, 0, 0, A + n1, lda, sA, n1, n2, batch, s)) != NMGP_OK) return rc;   // L12 = 0
  if ((rc = chol_inv_rec_big(A22, n2, lda, sA, X22, ldx, sX, batch, info, s, col_off + n1, ws)) != NMGP_OK) return rc;
  // T = L21 X11 (op(B)(k,j) = X11[k][j], lower) staged in X12;  X21 = -X22 T.  With n1 == n2 (every level of the
  // power-of-two shapes) T fits X12 row-major: coalesced stores, and the second product reads it k-row-wise (the
  // non-k-contiguous operand path stages as fast as the k-contiguous one).  Otherwise T is stored transposed.
  const bool t_rows = n1 == n2;
  if ((rc = gemm_big_f32(A21, lda, X, ldx, 0, X12, t_rows ? ldx : 1, t_rows ? 1 : ldx, n2, n1, n1, NMGP_B_LOWER, 1.f,
                         0.f, sA, sX, sX, nb, ws, s)) != NMGP_OK)
    return rc;
  if ((rc = gemm_big_f32(X22, ldx, X12, ldx, t_rows ? 0 : 1, X21, ldx, 1, n2, n1, n2, NMGP_A_LOWER, -1.f, 0.f, sX, sX,
                         sX, nb, ws, s)) != NMGP_OK)
    return rc;
  return block_copy<float>(nullptr, 0, 0, X12, ldx, sX, n1, n2, batch, s);   // X12 = 0
}

// Recursive factor + inverse for n > 256 (the HCP / ECoG / stress shapes).  With A split at n1
// (a multiple of 128 near n/2):
//   [L11, X11] = chol_inv(A11)                         (recursion; leaves <= 128: fused kernel)
//   L21 = A21 X11^T                                    (GEMM, A21 staged in X21's place)
//   A22 -= L21 L21^T                                   (GEMM, lower output only -- the SYRK)
//   [L22, X22] = chol_inv(A22)                         (recursion)
//   X21 = -X22 (L21 X11)                               (two GEMMs, product staged transposed in X12)
// so the 2 n^3 / 3 flops run in GEMMs of size ~n/2, n/4, ... on the matrix cores, and only the
// 128-wide leaves are serial.  X's strictly upper part is scratch and is left zero; the factor's
// strictly upper part is zeroed block by block.
template <typename T>
static int chol_inv_rec(T* A, int n, int64_t lda, int64_t sA, T* X, int64_t ldx, int64_t sX, int64_t batch,
                        int32_t* info, hipStream_t s, int col_off, void* ws) {
  if (n <= 128) return chol_inv_small<T>(A, n, lda, sA, X, ldx, sX, batch, info, s, col_off, col_off == 0);
  if constexpr (std::is_same<T, float>::value) return chol_inv_rec_big(A, n, lda, sA, X, ldx, sX, batch, info, s,
                                                                       col_off, ws);
  int n1 = ((n / 2 + 127) / 128) * 128;
  if (n1 >= n) n1 = n - 128;
  const int n2 = n - n1;
  int rc;
  T* A21 = A + (int64_t)n1 * lda;
  T* A22 = A21 + n1;
  T* X21 = X + (int64_t)n1 * ldx;
  T* X22 = X21 + n1;
  T* X12 = X + n1;
  if ((rc = chol_inv_rec<T>(A, n1, lda, sA, X, ldx, sX, batch, info, s, col_off, ws)) != NMGP_OK) return rc;
  if ((rc = block_copy<T>(A21, lda, sA, X21, ldx, sX, n2, n1, batch, s)) != NMGP_OK) return rc;
  // L21 = A21 X11^T   (B(k,j) = X11[j][k]: upper triangular)
  nmgp_gemm_desc d1 = gdesc(X21, ldx, 1, X, 1, ldx, A21, lda, 1, n2, n1, n1, NMGP_B_UPPER, 1.0, 0.0, sX, sX, sA, batch);
  if ((rc = gemm_single<T>(d1, s)) != NMGP_OK) return rc;
  // A22 -= L21 L21^T (lower)
  nmgp_gemm_desc d2 = gdesc(A21, lda, 1, A21, 1, lda, A22, lda, 1, n2, n2, n1, NMGP_OUT_LOWER, -1.0, 1.0, sA, sA, sA,
                            batch);
  if ((rc = gemm_single<T>(d2, s)) != NMGP_OK) return rc;
  if ((rc = block_copy<T>(nullptr, 0, 0, A + n1, lda, sA, n1, n2, batch, s)) != NMGP_OK) return rc;   // L12 = 0
  if ((rc = chol_inv_rec<T>(A22, n2, lda, sA, X22, ldx, sX, batch, info, s, col_off + n1, ws)) != NMGP_OK)
    return rc;
  // T = L21 X11 (X11 lower) stored transposed in X12;  X21 = -X22 T
  nmgp_gemm_desc d3 = gdesc(A21, lda, 1, X, ldx, 1, X12, 1, ldx, n2, n1, n1, NMGP_B_LOWER, 1.0, 0.0, sA, sX, sX, batch);
  if ((rc = gemm_single<T>(d3, s)) != NMGP_OK) return rc;
  nmgp_gemm_desc d4 = gdesc(X22, ldx, 1, X12, 1, ldx, X21, ldx, 1, n2, n1, n2, NMGP_A_LOWER, -1.0, 0.0, sX, sX, sX,
                            batch);
  if ((rc = gemm_single<T>(d4, s)) != NMGP_OK) return rc;
  return block_copy<T>(nullptr, 0, 0, X12, ldx, sX, n1, n2, batch, s);   // X12 = 0
}

// L = chol(A) in place and X = L^{-1}: fused register-resident kernel for n <= 256, the recursive
// GEMM-based path above otherwise.
template <typename T>
static int chol_inv_launch(T* A, int64_t n, int64_t lda, int64_t sA, T* X, int64_t ldx, int64_t sX, int64_t batch,
                           int32_t* info, hipStream_t s, void* ws = nullptr) {
  if (A == nullptr) return -1;
  if (n < 0) return -2;
  if (lda < n) return -3;
  if (X == nullptr) return -5;
  if (ldx < n) return -6;
  if (batch < 0) return -8;
  if (n == 0 || batch == 0) return NMGP_OK;
  if (batch > 65535) return -8;
  if (n > 256) return chol_inv_rec<T>(A, (int)n, lda, sA, X, ldx, sX, batch, info, s, 0, ws);
  return chol_inv_small<T>(A, (int)n, lda, sA, X, ldx, sX, batch, info, s, 0, 1);
}

// ---------------------------------------------------------------------------------------------
// Large single-matrix Cholesky (the M=4096 stress configuration; LAPACK potrf semantics, upper
// triangle zeroed).  128-wide block columns; the diagonal blocks are the fused register-resident
// factor + inverse kernel ("leaf"), the panel below a block is L_j = A_j X_jj^T.
//
// f32 (the stress configuration): right-looking, lookahead depth 1.  Per block step j:
//   main:  leaf(j) -> step(j) = L_j = A_j X_jj^T for every row below + A(rows, block column j+1) -= L_j L_{j+1,j}^T
//          (potrf_step32_kernel, one launch; the next leaf needs only the updated block column j+1)
//   side:  after leaf(j+1): the strip of block column j+2 (k = 128, potrf_strip32_kernel; the next step kernel
//          waits for it) and the rest of the trailing SYRK (columns >= j+3, gemm_big), two block steps of slack.
// Measured and not kept (round 4, profiles/r04a_stress_potrf_two_level_*, profiles/r04d_stress_*):
//   * two levels -- 512-column outer panels, the panel's updates of the rest of the matrix deferred into k = 512
//     products: 2.31 ms against 1.51.  A 128 x 128 tile of a k = 512 product takes >= 36 us on one CU
//     (tools/big_trace.hip), so the next panel's first block column put 38-48 us per panel on the serial chain,
//     and the deferred products held CUs the step kernels needed;
//   * the step kernel split into the rows of block j+1 (4 workgroups, on the chain) and the rest (a side
//     stream): 1.69 ms.  The step kernel is bound by its memory round trips (load, write-through store,
//     hand-off, read-back, store: 14 us alone), not by its width, so the 4-workgroup launch took as long as the
//     full one, and 21-24 us beside the side stream's SYRK.
// f64: one level (round 1): panel and lookahead as two GEMMs on the 64x64 f64 kernel, panel staged
// through P, the trailing SYRK of step j on the side stream while block j+1 is factored.
constexpr int PNB = 128;

struct PotrfSide {
  hipStream_t side = nullptr;
  hipEvent_t ev_main = nullptr, ev_side = nullptr, ev_tail = nullptr;
};

static int potrf_side_ctx(PotrfSide*& out) {
  static PotrfSide ctx[64];
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return NMGP_ERR_LAUNCH;
  std::lock_guard<std::mutex> lk(mu);
  PotrfSide& c = ctx[dev];
  if (c.side == nullptr) {
    if (hipStreamCreateWithFlags(&c.side, hipStreamNonBlocking) != hipSuccess) return NMGP_ERR_LAUNCH;
    for (hipEvent_t* e : {&c.ev_main, &c.ev_side, &c.ev_tail})
      if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return NMGP_ERR_LAUNCH;
  }
  out = &c;
  return NMGP_OK;
}

static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

// Workspace: [f32: three split-K / stream-K workspaces of the 128x128 kernel (their counters must be zero on
// entry and are left zero) + the step kernel's flag] [the leaves' inverses X_jj] [f64: the panel staging P].
// The fixed-size part comes first so that a workspace reused for another n (hip_ops.big_workspace keeps one
// per device) finds its counters where the previous call left them zero.
static size_t potrf_fixed_ws(bool f32) { return f32 ? 3 * al256(gemm_big_ws_bytes()) + 256 : 0; }

template <typename T>
static size_t potrf_blocked_ws(int64_t n) {
  const int64_t nblk = (n + PNB - 1) / PNB;
  return potrf_fixed_ws(std::is_same<T, float>::value) + al256((size_t)nblk * PNB * PNB * sizeof(T)) +
         al256((size_t)n * PNB * sizeof(T));
}

// C(m x nn) = alpha * A(m x k, row stride lda) op(B) + beta * C, op(B)(k, c) = B[c * ldb + k]
template <typename T>
static int pgemm(const T* A, int64_t lda, const T* B, int64_t ldb, T* C, int64_t ldc, int m, int nn, int k, int flags,
                 double alpha, double beta, void* bigws, hipStream_t s) {
  if constexpr (std::is_same<T, float>::value) {
    return gemm_big_f32(A, lda, B, ldb, 1, C, ldc, 1, m, nn, k, flags, (float)alpha, (float)beta, 0, 0, 0, 1, bigws,
                        s);
  } else {
    nmgp_gemm_desc d = gdesc(A, lda, 1, B, 1, ldb, C, ldc, 1, m, nn, k, flags, alpha, beta, 0, 0, 0, 1);
    return gemm_single<T>(d, s);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void zero_upper_kernel(T* A, int n, int64_t lda) {
  const int i = blockIdx.x;
  for (int j = i + 1 + (int)threadIdx.x; j < n; j += 256) A[(int64_t)i * lda + j] = (T)0;
}

// f32 leaves reserve enough LDS that no trailing-update workgroup (2 x 36 KB stages) shares their CUs: the
// side streams' products run beside the leaf on the other CUs (round 2 A/B: 1.64 -> 1.51 ms)
constexpr size_t kLeafLds = 88 * 1024;

#define NMGP_HIP_TRY(x) \
  do {                  \
    if ((x) != hipSuccess) return NMGP_ERR_LAUNCH; \
  } while (0)
#define NMGP_TRY(x)                    \
  do {                                 \
    const int rc_ = (x);               \
    if (rc_ != NMGP_OK) return rc_;    \
  } while (0)

static int potrf_one_level_f32(float* A, int n, int64_t lda, int32_t* info, void* ws, hipStream_t s) {
  PotrfSide* ctx = nullptr;
  NMGP_TRY(potrf_side_ctx(ctx));
  char* w = (char*)ws;
  void* ws_side = w + al256(gemm_big_ws_bytes());
  int32_t* step_flag = (int32_t*)(w + 3 * al256(gemm_big_ws_bytes()));
  float* Xd = (float*)(w + potrf_fixed_ws(true));
  const int nblk = (n + PNB - 1) / PNB;
  bool side_used = false;
  // the trailing update of step j, issued after the leaf of step j+1 (see below)
  struct { const float* Lb; float* C; int n3; bool on; } pend{nullptr, nullptr, 0, false};
  auto issue_update = [&]() -> int {
    if (!pend.on) return NMGP_OK;
    pend.on = false;
    NMGP_HIP_TRY(hipStreamWaitEvent(ctx->side, ctx->ev_main, 0));
    // block column j+2 first (the next step kernel's lookahead writes it and waits for this strip only), then
    // the rest of the trailing SYRK (columns >= j+3), which the step after next waits for
    const int cs = min(PNB, pend.n3), n4 = pend.n3 - cs;
    NMGP_TRY(potrf_strip_f32(pend.Lb, pend.C, lda, pend.n3, cs, ctx->side));
    NMGP_HIP_TRY(hipEventRecord(ctx->ev_side, ctx->side));
    if (n4 > 0) {
      const float* Lb2 = pend.Lb + (int64_t)cs * lda;
      NMGP_TRY(pgemm<float>(Lb2, lda, Lb2, lda, pend.C + (int64_t)cs * lda + cs, lda, n4, n4, PNB, NMGP_OUT_LOWER,
                            -1.0, 1.0, ws_side, ctx->side));
    }
    NMGP_HIP_TRY(hipEventRecord(ctx->ev_tail, ctx->side));
    side_used = true;
    return NMGP_OK;
  };
  for (int jb = 0; jb < nblk; ++jb) {
    const int j0 = jb * PNB, nbj = min(PNB, n - j0), r0 = j0 + nbj, n2 = n - r0;
    float* Xj = Xd + (int64_t)jb * PNB * PNB;
    // the diagonal leaf on the multi-role kernel (factor + two inverse workgroups)
    NMGP_TRY(chol_inv_small<float>(A + (int64_t)j0 * lda + j0, nbj, lda, 0, Xj, PNB, 0, 1, info, s, j0, jb == 0, true,
                                   kLeafLds));
    // the previous step's trailing update follows the previous step kernel like this leaf does; issued after the
    // leaf, because in a replayed graph the first-issued child of a node keeps the node's hardware queue, so the
    // leaf -> step hand-off of the serial chain stays on one queue (the cross-queue wait moves to the update)
    NMGP_TRY(issue_update());
    if (n2 == 0) break;
    float* Lj = A + (int64_t)r0 * lda + j0;   // block column j below the diagonal block
    const int c1 = min(PNB, n2), n3 = n2 - c1;
    // panel + lookahead of block column j+1 in one launch; the strip of step j-1 wrote that column
    if (side_used) NMGP_HIP_TRY(hipStreamWaitEvent(s, ctx->ev_side, 0));
    NMGP_TRY(potrf_step_f32(Lj, A + (int64_t)r0 * lda + r0, Xj, lda, n2, nbj, c1, step_flag, s));
    if (n3 > 0) {
      NMGP_HIP_TRY(hipEventRecord(ctx->ev_main, s));
      pend = {Lj + (int64_t)c1 * lda, A + (int64_t)(r0 + c1) * lda + (r0 + c1), n3, true};
    }
  }
  NMGP_TRY(issue_update());
  if (side_used) NMGP_HIP_TRY(hipStreamWaitEvent(s, ctx->ev_tail, 0));
  hipLaunchKernelGGL(zero_upper_kernel<float>, dim3((unsigned)n), dim3(256), 0, s, A, n, lda);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

template <typename T>
static int potrf_blocked(T* A, int n, int64_t lda, int32_t* info, void* ws, hipStream_t s) {
  if constexpr (std::is_same<T, float>::value) return potrf_one_level_f32(A, n, lda, info, ws, s);
  PotrfSide* ctx = nullptr;
  NMGP_TRY(potrf_side_ctx(ctx));
  const int nblk = (n + PNB - 1) / PNB;
  char* w = (char*)ws + potrf_fixed_ws(false);
  T* Xd = (T*)w;
  w += al256((size_t)nblk * PNB * PNB * sizeof(T));
  T* P = (T*)w;
  bool side_used = false;
  for (int jb = 0; jb < nblk; ++jb) {
    const int j0 = jb * PNB, nbj = min(PNB, n - j0), r0 = j0 + nbj, n2 = n - r0;
    T* Xj = Xd + (int64_t)jb * PNB * PNB;
    NMGP_TRY(chol_inv_small<T>(A + (int64_t)j0 * lda + j0, nbj, lda, 0, Xj, PNB, 0, 1, info, s, j0, jb == 0));
    if (n2 == 0) break;
    T* Lj = A + (int64_t)r0 * lda + j0;   // block column j below the diagonal block
    const int c1 = min(PNB, n2), n3 = n2 - c1;
    // the f64 kernel's 64-wide tiles would let one workgroup overwrite rows another is still reading: the
    // panel is staged through P
    NMGP_TRY(block_copy<T>(Lj, lda, 0, P, PNB, 0, n2, nbj, 1, s));
    NMGP_TRY(pgemm<T>(P, PNB, Xj, PNB, Lj, lda, n2, nbj, nbj, NMGP_B_UPPER, 1.0, 0.0, nullptr, s));
    // the trailing SYRK of step j-1 wrote block column j+1: the lookahead update must follow it
    if (side_used) NMGP_HIP_TRY(hipStreamWaitEvent(s, ctx->ev_side, 0));
    NMGP_TRY(pgemm<T>(Lj, lda, Lj, lda, A + (int64_t)r0 * lda + r0, lda, n2, c1, nbj, 0, -1.0, 1.0, nullptr, s));
    if (n3 > 0) {
      NMGP_HIP_TRY(hipEventRecord(ctx->ev_main, s));
      NMGP_HIP_TRY(hipStreamWaitEvent(ctx->side, ctx->ev_main, 0));
      const T* Lb = Lj + (int64_t)c1 * lda;
      NMGP_TRY(pgemm<T>(Lb, lda, Lb, lda, A + (int64_t)(r0 + c1) * lda + (r0 + c1), lda, n3, n3, nbj, NMGP_OUT_LOWER,
                        -1.0, 1.0, nullptr, ctx->side));
      NMGP_HIP_TRY(hipEventRecord(ctx->ev_side, ctx->side));
      side_used = true;
    }
  }
  if (side_used) NMGP_HIP_TRY(hipStreamWaitEvent(s, ctx->ev_side, 0));
  hipLaunchKernelGGL(zero_upper_kernel<T>, dim3((unsigned)n), dim3(256), 0, s, A, n, lda);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

template <typename T>
static int potrf_blocked_launch(T* A, int64_t n, int64_t lda, int32_t* info, void* ws, int64_t ws_bytes,
                                hipStream_t s) {
  if (A == nullptr) return -1;
  if (n < 0 || n > (1 << 20)) return -2;
  if (lda < n) return -3;
  if (info == nullptr) return -4;
  if (n == 0) return NMGP_OK;
  if (ws == nullptr || ws_bytes < (int64_t)potrf_blocked_ws<T>(n)) return -5;
  return potrf_blocked<T>(A, (int)n, lda, info, ws, s);
}

NMGP_TU_STATUS_ACCESSOR(chol)

}  // namespace nmgp

extern "C" {
int64_t nmgp_sizeof_chol_tp_args(void) { return (int64_t)sizeof(nmgp_chol_tp_args); }
int nmgp_chol_tp_trace(uint64_t* out, int64_t n) {
  if (!out || n < 0 || n > 8 * 512) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(nmgp::g_tp_trace), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? NMGP_OK
             : NMGP_ERR_LAUNCH;
}
int nmgp_chol_tp_f64(const nmgp_chol_tp_args* args, hipStream_t s) { return nmgp::chol_tp_launch(args, s); }
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
int nmgp_chol_inv_batched_f64(double* A, int64_t n, int64_t lda, int64_t sA, double* X, int64_t ldx, int64_t sX,
                              int64_t b, int32_t* info, hipStream_t s) {
  return nmgp::chol_inv_launch<double>(A, n, lda, sA, X, ldx, sX, b, info, s);
}
int nmgp_chol_inv_batched_f32(float* A, int64_t n, int64_t lda, int64_t sA, float* X, int64_t ldx, int64_t sX,
                              int64_t b, int32_t* info, hipStream_t s) {
  return nmgp::chol_inv_launch<float>(A, n, lda, sA, X, ldx, sX, b, info, s);
}
int64_t nmgp_chol_split_point(int64_t n) { return n > 256 ? (int64_t)nmgp::chol_split_point((int)n) : 0; }
int nmgp_chol_blockinv_batched_f32(float* A, int64_t n, int64_t lda, int64_t sA, float* X, int64_t ldx, int64_t sX,
                                   int64_t b, int32_t* info, hipStream_t s) {
  if (A == nullptr) return -1;
  if (n <= 256) return -2;
  if (lda < n) return -3;
  if (X == nullptr) return -5;
  if (ldx < n) return -6;
  if (b < 0 || b > 65535) return -8;
  if (b == 0) return NMGP_OK;
  return nmgp::chol_inv_rec_big(A, (int)n, lda, sA, X, ldx, sX, b, info, s, 0, nullptr, 0);
}
int64_t nmgp_chol_inv_workspace_size_f32(int64_t n, int64_t batch) {
  return (n > 256 && batch > 0) ? (int64_t)nmgp::gemm_big_ws_bytes() : 0;
}
int nmgp_chol_inv_batched_ws_f32(float* A, int64_t n, int64_t lda, int64_t sA, float* X, int64_t ldx, int64_t sX,
                                 int64_t b, int32_t* info, void* ws, int64_t ws_bytes, hipStream_t s) {
  if (ws != nullptr && ws_bytes < nmgp_chol_inv_workspace_size_f32(n, b)) return -11;
  return nmgp::chol_inv_launch<float>(A, n, lda, sA, X, ldx, sX, b, info, s, ws);
}
int64_t nmgp_potrf_blocked_workspace_size_f32(int64_t n) { return n > 0 ? (int64_t)nmgp::potrf_blocked_ws<float>(n) : 0; }
int64_t nmgp_potrf_blocked_workspace_size_f64(int64_t n) { return n > 0 ? (int64_t)nmgp::potrf_blocked_ws<double>(n) : 0; }
int nmgp_potrf_blocked_f32(float* A, int64_t n, int64_t lda, int32_t* info, void* ws, int64_t ws_bytes, hipStream_t s) {
  return nmgp::potrf_blocked_launch<float>(A, n, lda, info, ws, ws_bytes, s);
}
int nmgp_potrf_blocked_f64(double* A, int64_t n, int64_t lda, int32_t* info, void* ws, int64_t ws_bytes, hipStream_t s) {
  return nmgp::potrf_blocked_launch<double>(A, n, lda, info, ws, ws_bytes, s);
}
}
