// Pairwise kernel-matrix builders (RBF and nonstationary Gibbs) and their backward reductions.
//
// Forward replaces code/utils.py:75-103 (create_RBF / create_Gibbs, difference distance) and
// SIM_code/Utility/kernels.py:5-73 (RBF_cov / Nonstationary_RBF_cov, expanded distance,
// per-point sigma, +1e-6 I).  Several matrices are built by ONE launch from a descriptor list
// (K_t12, K_t22, K_L0_*, K_L1_* of a DSVI step).  HBM-bound: each output element is written
// once, the per-point inputs (x, z, ell) are read coalesced and stay in L1/L2.
//
// Backward: Kbar = Rbar - rowcoef(i) * Pm (the closed-form DSVI adjoint of K12 is R - c * P, see
// DESIGN.md §4), reduced over 8-row x 64-column tiles into deterministic partial sums.
#include "common.hpp"

namespace nmgp {

// 8-row x 64-column tiles, two rows per wave (round 6: 32-row tiles left the M x M priors' K22 (256 x 256) at 96
// workgroups and the K_G12 backward (2000 x 256) at 252, each wave working through 8 rows in turn; include/nmgp_hip.h
// pairwise descriptors' `tiles`, the backward's partial sums are per 8-row tile)
constexpr int PR = 8, PC = 64;
constexpr int PRF = PR;

struct PwArgs {
  const nmgp_pairwise_desc* descs;
  int nd;
  nmgp_pairwise_desc inl;
};
struct PwBwdArgs {
  const nmgp_pairwise_bwd_desc* descs;
  int nd;
  nmgp_pairwise_bwd_desc inl;
};

template <typename D>
__device__ inline const D* find_desc(const D* descs, int nd, const D* inl, int tile) {
  if (descs == nullptr) return inl;
  int lo = 0, hi = nd - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].tile_start <= tile) lo = mid; else hi = mid - 1;
  }
  return &descs[lo];
}

template <typename T>
__device__ inline T sqdist(const T* X, const T* Z, int i, int j, int p, int dist, T inv_ls) {
  if (dist == NMGP_DIST_DIFF) {
    T r2 = 0;
    for (int f = 0; f < p; ++f) {
      const T dd = X[(int64_t)i * p + f] * inv_ls - Z[(int64_t)j * p + f] * inv_ls;
      r2 += dd * dd;
    }
    return r2;
  }
  T xn = 0, zn = 0, xz = 0;
  for (int f = 0; f < p; ++f) {
    const T a = X[(int64_t)i * p + f] * inv_ls, b = Z[(int64_t)j * p + f] * inv_ls;
    xn += a * a;
    zn += b * b;
    xz += a * b;
  }
  return xn + zn - (T)2 * xz;
}

// Division (not multiply-by-reciprocal) keeps the forward bit-closer to the reference's x / ls.
template <typename T>
__device__ inline T sqdist_div(const T* X, const T* Z, int i, int j, int p, int dist, T ls) {
  if (dist == NMGP_DIST_DIFF) {
    T r2 = 0;
    for (int f = 0; f < p; ++f) {
      const T dd = X[(int64_t)i * p + f] / ls - Z[(int64_t)j * p + f] / ls;
      r2 += dd * dd;
    }
    return r2;
  }
  T xn = 0, zn = 0, xz = 0;
  for (int f = 0; f < p; ++f) {
    const T a = X[(int64_t)i * p + f] / ls, b = Z[(int64_t)j * p + f] / ls;
    xn += a * a;
    zn += b * b;
    xz += a * b;
  }
  return xn + zn - (T)2 * xz;
}

template <typename T>
__device__ inline void hyper_of(const T* hyp, int mode, int flags, T& s2, T& ls) {
  if (hyp == nullptr) return;
  s2 = hyp[0];
  if (flags & NMGP_HYP_LOG) s2 = dexp(s2);
  if (mode == NMGP_RBF) {
    ls = hyp[1];
    if (flags & NMGP_HYP_LOG) ls = dexp(ls);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void pairwise_kernel(PwArgs args) {
  int tile = blockIdx.x;
  const nmgp_pairwise_desc& d = *find_desc(args.descs, args.nd, &args.inl, tile);
  tile -= d.tile_start;
  const int n = d.n, m = d.m, p = d.p;
  const int ctn = (m + PC - 1) / PC;
  const int rt = tile / ctn, ct = tile - rt * ctn;
  const int j = ct * PC + (threadIdx.x & 63);
  if (j >= m) return;
  constexpr int PR = PRF;
  T s2 = (T)d.scale2, ls = (T)d.length_scale;
  hyper_of((const T*)d.hyp, d.mode, d.flags, s2, ls);
  const T* X = (const T*)d.X;
  const T* Z = (const T*)d.Z;
  const T* ellX = (const T*)d.ellX;
  const T* ellZ = (const T*)d.ellZ;
  const T* sigX = (const T*)d.sigX;
  const T* sigZ = (const T*)d.sigZ;
  T* K = (T*)d.K;
  const T dadd = (T)d.diag_add;
  const T lz = d.mode == NMGP_GIBBS ? ellZ[j] : (T)0;
  const T sz = sigZ ? sigZ[j] : (T)1;
#pragma unroll 2
  for (int e = 0; e < PR / 4; ++e) {
    const int i = rt * PR + (threadIdx.x >> 6) + 4 * e;
    if (i >= n) break;
    T k;
    if (d.mode == NMGP_RBF) {
      const T r2 = sqdist_div(X, Z, i, j, p, d.dist, ls);
      k = dexp((T)-0.5 * r2) * s2;
    } else {
      const T r2 = sqdist_div(X, Z, i, j, p, d.dist, (T)1);
      const T lx = ellX[i];
      const T S = lx * lx + lz * lz;
      const T C = dsqrt((T)2 * (lx * lz) / S);
      k = sigX ? ((sigX[i] * sz) * C) * dexp(-r2 / S) : s2 * C * dexp(-r2 / S);
    }
    if (i == j) k += dadd;
    K[(int64_t)i * d.ldk + j] = k;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void pairwise_bwd_kernel(PwBwdArgs args) {
  __shared__ T colp[4][PC];
  __shared__ T red[16];
  int tile = blockIdx.x;
  const nmgp_pairwise_bwd_desc& d = *find_desc(args.descs, args.nd, &args.inl, tile);
  tile -= d.tile_start;
  const int n = d.n, m = d.m, p = d.p;
  const int ctn = (m + PC - 1) / PC;
  const int rt = tile / ctn, ct = tile - rt * ctn;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = ct * PC + lane;
  const bool jok = j < m;
  T s2 = (T)d.scale2, ls = (T)d.length_scale;
  hyper_of((const T*)d.hyp, d.mode, d.flags, s2, ls);
  const T* X = (const T*)d.X;
  const T* Z = (const T*)d.Z;
  const T* K = (const T*)d.K;
  const T* Rb = (const T*)d.Rbar;
  const T* Pm = (const T*)d.Pm;
  const T* rc = (const T*)d.rowcoef;
  const T* ellX = (const T*)d.ellX;
  const T* ellZ = (const T*)d.ellZ;
  T* row_part = (T*)d.row_part;
  const bool gibbs = d.mode == NMGP_GIBBS;
  const T lz = (gibbs && jok) ? ellZ[j] : (T)0;
  T s0 = 0, s1 = 0, gzacc = 0;
  // the wave's PR/4 rows: every row's loads and arithmetic first (no store in between, so the loads of all rows
  // are in flight together), then the per-row reductions of the Gibbs x-adjoints and their stores (round 6: the
  // row loop with a store after each row's reduction ran one row's memory round trip at a time -- 29 us for the
  // PM2.5 K_G12 backward, on the step's critical chain)
  T gxs[PR / 4];
#pragma unroll
  for (int e = 0; e < PR / 4; ++e) {
    const int i = rt * PR + w * (PR / 4) + e;
    T gx = 0;
    if (jok && i < n) {
      const int64_t idx = (int64_t)i * d.ld + j;
      T kb = Rb[idx];
      if (rc) kb -= rc[i] * Pm[idx];
      if (!gibbs) {
        const T r2 = sqdist_div(X, Z, i, j, p, NMGP_DIST_DIFF, ls);
        const T kv = K ? K[idx] : dexp((T)-0.5 * r2) * s2;   // K == NULL: recompute (K22 was factored in place)
        const T wv = kb * kv;
        s0 += wv;
        s1 += wv * r2;
      } else {
        const T r2 = sqdist_div(X, Z, i, j, p, NMGP_DIST_DIFF, (T)1);
        const T lx = ellX[i];
        const T S = lx * lx + lz * lz;
        const T kv = K ? K[idx] : s2 * dsqrt((T)2 * (lx * lz) / S) * dexp(-r2 / S);
        const T wv = kb * kv;
        s0 += wv;
        const T r2s = (T)2 * r2 / (S * S);
        gx = wv * ((T)0.5 / lx - lx / S + lx * r2s);
        gzacc += wv * ((T)0.5 / lz - lz / S + lz * r2s);
      }
    }
    gxs[e] = gx;
  }
  if (gibbs) {
#pragma unroll
    for (int e = 0; e < PR / 4; ++e) {
      const int i = rt * PR + w * (PR / 4) + e;
      const T gx = wave_sum(gxs[e]);
      if (lane == 0 && i < n) row_part[(int64_t)ct * n + i] = gx;
    }
  }
  if (gibbs) {
    colp[w][lane] = gzacc;
    __syncthreads();
    if (w == 0 && jok) {
      T* col_part = (T*)d.col_part;
      col_part[(int64_t)rt * m + j] = colp[0][lane] + colp[1][lane] + colp[2][lane] + colp[3][lane];
    }
  }
  if (d.scal_part) {
    s0 = block_sum(s0, red);
    s1 = block_sum(s1, red);
    if (threadIdx.x == 0) {
      T* sp = (T*)d.scal_part;
      sp[(int64_t)tile * 2 + 0] = s0;
      sp[(int64_t)tile * 2 + 1] = s1;
    }
  }
}

template <typename T>
__global__ void colsum_kernel(const T* a, int64_t rows, int64_t cols, T beta, T* out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= cols) return;
  T s = 0;
  for (int64_t i = 0; i < rows; ++i) s += a[i * cols + j];
  out[j] = (beta != (T)0 ? beta * out[j] : (T)0) + s;
}

static inline int pw_tiles(int n, int m) { return ((n + PR - 1) / PR) * ((m + PC - 1) / PC); }
static inline int pw_tiles_fwd(int n, int m) { return ((n + PRF - 1) / PRF) * ((m + PC - 1) / PC); }

template <typename T>
static int pw_launch(const nmgp_pairwise_desc* dd, int nd, int tt, const nmgp_pairwise_desc* inl, hipStream_t s) {
  if (tt <= 0) return NMGP_OK;
  PwArgs a;
  a.descs = dd;
  a.nd = nd;
  a.inl = inl ? *inl : nmgp_pairwise_desc{};
  hipLaunchKernelGGL(pairwise_kernel<T>, dim3(tt), dim3(256), 0, s, a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

template <typename T>
static int pwb_launch(const nmgp_pairwise_bwd_desc* dd, int nd, int tt, const nmgp_pairwise_bwd_desc* inl,
                      hipStream_t s) {
  if (tt <= 0) return NMGP_OK;
  PwBwdArgs a;
  a.descs = dd;
  a.nd = nd;
  a.inl = inl ? *inl : nmgp_pairwise_bwd_desc{};
  hipLaunchKernelGGL(pairwise_bwd_kernel<T>, dim3(tt), dim3(256), 0, s, a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

}  // namespace nmgp

extern "C" {
int nmgp_pairwise_f64(const nmgp_pairwise_desc* d, int nd, int tt, hipStream_t s) {
  if (!d) return -1;
  return nmgp::pw_launch<double>(d, nd, tt, nullptr, s);
}
int nmgp_pairwise_f32(const nmgp_pairwise_desc* d, int nd, int tt, hipStream_t s) {
  if (!d) return -1;
  return nmgp::pw_launch<float>(d, nd, tt, nullptr, s);
}
int nmgp_pairwise_single_f64(const nmgp_pairwise_desc* h, hipStream_t s) {
  if (!h) return -1;
  nmgp_pairwise_desc d = *h;
  d.tile_start = 0;
  d.tiles = nmgp::pw_tiles_fwd(d.n, d.m);
  return nmgp::pw_launch<double>(nullptr, 1, d.tiles, &d, s);
}
int nmgp_pairwise_single_f32(const nmgp_pairwise_desc* h, hipStream_t s) {
  if (!h) return -1;
  nmgp_pairwise_desc d = *h;
  d.tile_start = 0;
  d.tiles = nmgp::pw_tiles_fwd(d.n, d.m);
  return nmgp::pw_launch<float>(nullptr, 1, d.tiles, &d, s);
}
int nmgp_pairwise_bwd_f64(const nmgp_pairwise_bwd_desc* d, int nd, int tt, hipStream_t s) {
  if (!d) return -1;
  return nmgp::pwb_launch<double>(d, nd, tt, nullptr, s);
}
int nmgp_pairwise_bwd_f32(const nmgp_pairwise_bwd_desc* d, int nd, int tt, hipStream_t s) {
  if (!d) return -1;
  return nmgp::pwb_launch<float>(d, nd, tt, nullptr, s);
}
int nmgp_pairwise_bwd_single_f64(const nmgp_pairwise_bwd_desc* h, hipStream_t s) {
  if (!h) return -1;
  nmgp_pairwise_bwd_desc d = *h;
  d.tile_start = 0;
  d.tiles = nmgp::pw_tiles(d.n, d.m);
  return nmgp::pwb_launch<double>(nullptr, 1, d.tiles, &d, s);
}
int nmgp_pairwise_bwd_single_f32(const nmgp_pairwise_bwd_desc* h, hipStream_t s) {
  if (!h) return -1;
  nmgp_pairwise_bwd_desc d = *h;
  d.tile_start = 0;
  d.tiles = nmgp::pw_tiles(d.n, d.m);
  return nmgp::pwb_launch<float>(nullptr, 1, d.tiles, &d, s);
}
int nmgp_colsum_f32(const float* a, int64_t rows, int64_t cols, double beta, float* out, hipStream_t s) {
  if (!a) return -1;
  if (!out) return -5;
  if (cols <= 0) return NMGP_OK;
  hipLaunchKernelGGL(nmgp::colsum_kernel<float>, dim3((unsigned)((cols + 255) / 256)), dim3(256), 0, s, a, rows, cols,
                     (float)beta, out);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
int nmgp_colsum_f64(const double* a, int64_t rows, int64_t cols, double beta, double* out, hipStream_t s) {
  if (!a) return -1;
  if (!out) return -5;
  if (cols <= 0) return NMGP_OK;
  hipLaunchKernelGGL(nmgp::colsum_kernel<double>, dim3((unsigned)((cols + 255) / 256)), dim3(256), 0, s, a, rows, cols,
                     beta, out);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
}
