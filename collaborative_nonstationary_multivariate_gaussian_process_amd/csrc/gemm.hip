// Grouped, strided, masked GEMM on the MI355X matrix cores (v_mfma_f64_16x16x4f64 /
// v_mfma_f32_16x16x4f32).  One launch runs a whole list of problems (the Q coefficient pairs,
// the D latent functions, the 4 priors ...) so a DSVI step is a handful of launches instead of
// the reference's per-pair torch.solve / matmul calls (code/utils.py:117-146,
// code/nmgp_dsvi.py:172-177, 227-237).
//
// Tile 64x64x16 per 256-thread workgroup: 4 waves in a 2x2 grid, each wave 32x32 = 2x2 MFMA
// blocks of 16x16.  Operands are staged k-major in LDS (row pitch 80 elements so that the two
// 16-lane k rows of one ds_read_b64 land on disjoint bank halves).  Triangular operand masks
// trim the k range, so tril(S) tril(S)^T and L^-T L^-1 products skip the zero half.
#include "common.hpp"

namespace nmgp {

constexpr int GBM = 64, GBN = 64, GBK = 16, GPAD = 16;

struct GemmArgs {
  const nmgp_gemm_desc* descs;
  int nprob;
  const int32_t* seg;
  nmgp_gemm_desc inl;
};

template <typename T>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs args) {
  __shared__ T As[GBK][GBM + GPAD];
  __shared__ T Bs[GBK][GBN + GPAD];
  int tile = blockIdx.x;
  const nmgp_gemm_desc* dp = &args.inl;
  if (args.descs != nullptr) {
    int lo = 0, hi = args.nprob - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (args.descs[mid].tile_start <= tile) lo = mid; else hi = mid - 1;
    }
    dp = &args.descs[lo];
  }
  const nmgp_gemm_desc& d = *dp;
  __shared__ int s_last;
  tile -= d.tile_start;
  const int ksplit = d.ksplit > 1 ? d.ksplit : 1;
  const int ks = tile % ksplit;
  tile /= ksplit;
  const int tn = tile % d.tiles_n, tm = tile / d.tiles_n;
  int64_t r0 = 0;
  int m = d.m;
  const int span = d.seg_span > 0 ? d.seg_span : 1;
  if (d.row_seg >= 0) {
    r0 = args.seg[d.row_seg];
    m = args.seg[d.row_seg + span] - (int)r0;
  }
  int64_t k0 = 0;
  int K = d.k;
  if (d.k_seg >= 0) {
    k0 = args.seg[d.k_seg];
    K = args.seg[d.k_seg + span] - (int)k0;
  }
  const int n = d.n;
  const int i0 = tm * GBM, j0 = tn * GBN;
  if (i0 >= m) return;
  const int flags = d.flags;
  const bool above = j0 > i0 + GBM - 1;
  if (above && (flags & NMGP_OUT_LOWER)) return;
  const bool zero_tile = above && (flags & NMGP_OUT_TRIL);
  const int kbA = d.kbA > 0 ? d.kbA : 0x7fffffff;
  const int kbB = d.kbB > 0 ? d.kbB : 0x7fffffff;

  int kbeg = 0, kend = K;
  if (d.k_seg < 0) {
    if ((flags & NMGP_A_LOWER) && kbA >= K) kend = min(kend, i0 + GBM);
    if ((flags & NMGP_A_UPPER) && kbA >= K) kbeg = max(kbeg, i0);
    if ((flags & NMGP_B_LOWER) && kbB >= K) kbeg = max(kbeg, j0);
    if ((flags & NMGP_B_UPPER) && kbB >= K) kend = min(kend, j0 + GBN);
  }
  kbeg = (kbeg / GBK) * GBK;
  if (zero_tile) {
    if (ks != 0) return;          // one chunk writes the zero tile directly
    kend = kbeg;
  } else if (ksplit > 1) {        // this workgroup's k chunk (multiple of GBK)
    int chunk = (kend - kbeg + ksplit - 1) / ksplit;
    chunk = ((chunk + GBK - 1) / GBK) * GBK;
    const int cb = kbeg + ks * chunk;
    kend = max(cb, min(kend, cb + chunk));
    kbeg = cb;
  }

  const T* __restrict__ A = (const T*)d.A;
  const T* __restrict__ Bm = (const T*)d.B;
  const T* __restrict__ ksc = (const T*)d.kscale;
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  const bool a_kc = (d.sA_k == 1);
  const bool b_jc = (d.sB_j == 1);

  using acc_t = typename Mfma<T>::acc_t;
  acc_t acc00 = {0, 0, 0, 0}, acc01 = {0, 0, 0, 0}, acc10 = {0, 0, 0, 0}, acc11 = {0, 0, 0, 0};

  for (int kt = kbeg; kt < kend; kt += GBK) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int il, kl;
      if (a_kc) { il = t >> 2; kl = ((t & 3) << 2) + e; }
      else { kl = t >> 4; il = ((t & 15) << 2) + e; }
      const int gi = i0 + il, gk = kt + kl;
      T val = 0;
      if (gi < m && gk < K) {
        int kk = gk, kb = 0;
        if (d.k_seg < 0 && kbA < K) { kb = gk / kbA; kk = gk - kb * kbA; }
        const bool z = ((flags & NMGP_A_LOWER) && kk > gi) || ((flags & NMGP_A_UPPER) && kk < gi);
        if (!z) val = A[(r0 + gi) * d.sA_i + (k0 + kk) * d.sA_k + (int64_t)kb * d.sA_kb];
      }
      As[kl][il] = val;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int kl, jl;
      if (b_jc) { kl = t >> 4; jl = ((t & 15) << 2) + e; }
      else { jl = t >> 2; kl = ((t & 3) << 2) + e; }
      const int gk = kt + kl, gj = j0 + jl;
      T val = 0;
      if (gk < K && gj < n) {
        int kk = gk, kb = 0;
        if (d.k_seg < 0 && kbB < K) { kb = gk / kbB; kk = gk - kb * kbB; }
        const bool z = ((flags & NMGP_B_LOWER) && gj > kk) || ((flags & NMGP_B_UPPER) && gj < kk);
        if (!z) {
          val = Bm[(k0 + kk) * d.sB_k + (int64_t)gj * d.sB_j + (int64_t)kb * d.sB_kb];
          if (flags & NMGP_KSCALE) val *= ksc[k0 + gk];
        }
      }
      Bs[kl][jl] = val;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int kr = s * 4 + (lane >> 4);
      const T a0 = As[kr][wr * 32 + (lane & 15)];
      const T a1 = As[kr][wr * 32 + 16 + (lane & 15)];
      const T b0 = Bs[kr][wc * 32 + (lane & 15)];
      const T b1 = Bs[kr][wc * 32 + 16 + (lane & 15)];
      acc00 = Mfma<T>::mma(a0, b0, acc00);
      acc01 = Mfma<T>::mma(a0, b1, acc01);
      acc10 = Mfma<T>::mma(a1, b0, acc10);
      acc11 = Mfma<T>::mma(a1, b1, acc11);
    }
    __syncthreads();
  }

  if (ksplit > 1 && !zero_tile) {
    // deterministic split-K: publish this chunk's partial, the last arriver sums all chunks in order
    T* ws = (T*)d.ws + (int64_t)(tm * d.tiles_n + tn) * ksplit * 4096;
    T* mine = ws + (int64_t)ks * 4096 + t * 16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mine[r] = acc00[r];
      mine[4 + r] = acc01[r];
      mine[8 + r] = acc10[r];
      mine[12 + r] = acc11[r];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      int32_t* ctr = d.counters + tm * d.tiles_n + tn;
      const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = (old == ksplit - 1);
      if (last) {
        __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    acc00 = acc01 = acc10 = acc11 = acc_t{0, 0, 0, 0};
    for (int c = 0; c < ksplit; ++c) {
      const T* src = ws + (int64_t)c * 4096 + t * 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc00[r] += src[r];
        acc01[r] += src[4 + r];
        acc10[r] += src[8 + r];
        acc11[r] += src[12 + r];
      }
    }
  }

  T* __restrict__ C = (T*)d.C;
  const T* __restrict__ E = (const T*)d.epi_E;
  const T* __restrict__ rsp = (const T*)d.epi_rs;
  const T alpha = (T)d.alpha, beta = (T)d.beta, gamma = (T)d.gamma, dadd = (T)d.diag_add;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const acc_t& acc = q == 0 ? acc00 : q == 1 ? acc01 : q == 2 ? acc10 : acc11;
    const int mi = q >> 1, ni = q & 1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gi = i0 + wr * 32 + mi * 16 + Mfma<T>::row(lane, r);
      const int gj = j0 + wc * 32 + ni * 16 + (lane & 15);
      if (gi >= m || gj >= n) continue;
      const bool upper = gj > gi;
      if (upper && (flags & NMGP_OUT_LOWER)) continue;
      const int64_t ci = (r0 + gi) * d.sC_i + (int64_t)gj * d.sC_j;
      T val;
      if (upper && (flags & NMGP_OUT_TRIL)) {
        val = 0;
      } else {
        val = alpha * acc[r];
        if (beta != (T)0) val += beta * C[ci];
        if (flags & NMGP_EPI) {
          T e = 0;
          if (!((flags & NMGP_EPI_E_LOWER) && upper)) e = E[(r0 + gi) * d.sE_i + (int64_t)gj * d.sE_j];
          T rs = rsp ? rsp[r0 + gi] : (T)1;
          if (flags & NMGP_EPI_RS_NEG) rs = -rs;
          val += gamma * rs * e;
        }
        if ((flags & NMGP_DIAG_ADD) && gi == gj) val += dadd;
      }
      C[ci] = val;
    }
  }
}

template <typename T>
static int launch_grouped(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles, const int32_t* d_seg,
                          hipStream_t s) {
  if (d_desc == nullptr) return -1;
  if (nprob <= 0) return -2;
  if (total_tiles < 0) return -3;
  if (total_tiles == 0) return NMGP_OK;
  GemmArgs a;
  a.descs = d_desc;
  a.nprob = nprob;
  a.seg = d_seg;
  a.inl = nmgp_gemm_desc{};
  hipLaunchKernelGGL(gemm_kernel<T>, dim3(total_tiles), dim3(256), 0, s, a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

template <typename T>
static int launch_single(const nmgp_gemm_desc* h, const int32_t* d_seg, hipStream_t s) {
  if (h == nullptr) return -1;
  nmgp_gemm_desc d = *h;
  if (d.m < 0 || d.n < 0 || d.k < 0) return -1;
  if (d.m == 0 || d.n == 0) return NMGP_OK;
  d.tiles_m = (d.m + GBM - 1) / GBM;
  d.tiles_n = (d.n + GBN - 1) / GBN;
  d.tile_start = 0;
  d.ksplit = 1;
  GemmArgs a;
  a.descs = nullptr;
  a.nprob = 1;
  a.seg = d_seg;
  a.inl = d;
  hipLaunchKernelGGL(gemm_kernel<T>, dim3(d.tiles_m * d.tiles_n), dim3(256), 0, s, a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

}  // namespace nmgp

extern "C" {
int nmgp_version(void) { return 1; }
int64_t nmgp_sizeof_gemm_desc(void) { return (int64_t)sizeof(nmgp_gemm_desc); }
int64_t nmgp_sizeof_pairwise_desc(void) { return (int64_t)sizeof(nmgp_pairwise_desc); }
int64_t nmgp_sizeof_pairwise_bwd_desc(void) { return (int64_t)sizeof(nmgp_pairwise_bwd_desc); }
int64_t nmgp_sizeof_dsvi_args(void) { return (int64_t)sizeof(nmgp_dsvi_args); }

int nmgp_gemm_grouped_f64(const nmgp_gemm_desc* d, int np, int tt, const int32_t* seg, hipStream_t s) {
  return nmgp::launch_grouped<double>(d, np, tt, seg, s);
}
int nmgp_gemm_grouped_f32(const nmgp_gemm_desc* d, int np, int tt, const int32_t* seg, hipStream_t s) {
  return nmgp::launch_grouped<float>(d, np, tt, seg, s);
}
int nmgp_gemm_f64(const nmgp_gemm_desc* h, const int32_t* seg, hipStream_t s) {
  return nmgp::launch_single<double>(h, seg, s);
}
int nmgp_gemm_f32(const nmgp_gemm_desc* h, const int32_t* seg, hipStream_t s) {
  return nmgp::launch_single<float>(h, seg, s);
}
}
