// Grouped, strided, masked GEMM on the MI355X matrix cores (v_mfma_f64_16x16x4f64 /
// v_mfma_f32_16x16x4f32).  One launch runs a whole list of problems (the Q coefficient pairs,
// the D latent functions, the 4 priors ...) so a DSVI step is a handful of launches instead of
// the reference's per-pair torch.solve / matmul calls (code/utils.py:117-146,
// code/nmgp_dsvi.py:172-177, 227-237).
//
// Tile 64x64x32 per 256-thread workgroup: 4 waves in a 2x2 grid, each wave 32x32 = 2x2 MFMA
// blocks of 16x16.  Operands are staged k-major in ONE LDS array (pitch 65: the k-major stores of a
// k-contiguous operand are conflict-free).  Main loop = register prefetch pipeline: the global
// loads of k-tile t+1 are in flight while the MFMAs of tile t run; masks (bounds, triangular
// operands, k-scale) are applied when the registers are written to LDS, so nothing consumes a
// prefetched value early.  Fast path: buffer loads whose per-element byte offsets are fixed for the
// whole loop -- the k advance is a uniform change of the resource base, out-of-range reads give 0.
// Triangular operand masks trim the k range, so tril(S) tril(S)^T and L^-T L^-1 skip the zero half.
#include "common.hpp"

namespace nmgp {

#ifdef NMGP_GEMM_TRACE  // per-phase timestamps of workgroup 0 (tools/gemm_trace.hip only)
__device__ unsigned long long* g_gemm_trace;
#define GEMM_STAMP(i) \
  if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) g_gemm_trace[i] = __builtin_readcyclecounter()
#else
#define GEMM_STAMP(i)
#endif

constexpr int GBM = 64, GBN = 64, GBK = 32, LP = 65;
constexpr int LDS_T = 2 * GBK * LP;  // A image + B image (elements)

struct GemmArgs {
  const nmgp_gemm_desc* descs;
  int nprob;
  const int32_t* seg;
  nmgp_gemm_desc inl;
};

__device__ inline __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int64_t nbytes) {
  const int32_t nr = (int32_t)(nbytes <= 0 ? 0 : (nbytes > 0x7fffffffLL ? 0x7fffffffLL : nbytes));
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nr, 0x00020000);
}
template <typename T> __device__ inline T bload(__amdgpu_buffer_rsrc_t r, uint32_t off_bytes);
template <> __device__ inline double bload<double>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
template <> __device__ inline float bload<float>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

// Problem geometry resolved for one workgroup (all wave-uniform).
struct Tile {
  int64_t r0, k0;
  int m, n, K, i0, j0, kbeg, kend, kbA, kbB, flags;
};

// Per-thread element map of a GBM x GBK (A) / GBK x GBN (B) tile, 8 elements each, chosen so that
// each load instruction reads consecutive addresses across the wave for either layout.
struct EltMap {
  int a_il[8], a_kl[8], b_kl[8], b_jl[8];
};

template <typename T>
__device__ inline void stage_lds(T* As, T* Bs, const EltMap& em, const T (&ra)[8], const T (&rb)[8],
                                 const T (&rs)[8], unsigned okm, bool kscale) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    As[em.a_kl[e] * LP + em.a_il[e]] = (okm >> e) & 1u ? ra[e] : (T)0;
    T bv = (okm >> (8 + e)) & 1u ? rb[e] : (T)0;
    if (kscale) bv *= rs[e];
    Bs[em.b_kl[e] * LP + em.b_jl[e]] = bv;
  }
}

template <typename T, typename Acc>
__device__ inline void mma_tile(const T* As, const T* Bs, int lane, int wr, int wc, Acc& c00, Acc& c01, Acc& c10,
                                Acc& c11) {
#pragma unroll
  for (int s = 0; s < GBK / 4; ++s) {
    const int kr = s * 4 + (lane >> 4);
    const T a0 = As[kr * LP + wr * 32 + (lane & 15)];
    const T a1 = As[kr * LP + wr * 32 + 16 + (lane & 15)];
    const T b0 = Bs[kr * LP + wc * 32 + (lane & 15)];
    const T b1 = Bs[kr * LP + wc * 32 + 16 + (lane & 15)];
    c00 = Mfma<T>::mma(a0, b0, c00);
    c01 = Mfma<T>::mma(a0, b1, c01);
    c10 = Mfma<T>::mma(a1, b0, c10);
    c11 = Mfma<T>::mma(a1, b1, c11);
  }
}

// Triangular-operand and bounds validity of element (gi, kk) of A / (kk, gj) of B.
__device__ inline bool a_ok(int flags, int gi, int kk, int m, bool kin) {
  return gi < m && kin && !(((flags & NMGP_A_LOWER) && kk > gi) || ((flags & NMGP_A_UPPER) && kk < gi));
}
__device__ inline bool b_ok(int flags, int gj, int kk, int n, bool kin) {
  return gj < n && kin && !(((flags & NMGP_B_LOWER) && gj > kk) || ((flags & NMGP_B_UPPER) && gj < kk));
}

// Fast main loop: every k-tile lies inside one k-block of each operand (block length a multiple
// of GBK, or no blocking), so an element's byte offset from the tile's k origin never changes.
// Masks are computed only for k-tiles that need them (the k tail, tiles straddling a triangular
// operand's diagonal): rows past m / columns past n only feed outputs that are never stored, and
// reads past the operand's extent return 0 (buffer range check).  KS: k-scaled B (compile time).
template <typename T, bool KS, typename Acc>
__device__ inline void mainloop_fast(const nmgp_gemm_desc& d, const Tile& tl, const EltMap& em, T* As, T* Bs, int lane,
                                     int wr, int wc, Acc& c00, Acc& c01, Acc& c10, Acc& c11) {
  const char* Ab = (const char*)d.A;
  const char* Bb = (const char*)d.B;
  const GPtr<const T> ksc = (GPtr<const T>)(d.kscale ? d.kscale : d.B);
  const bool kbA_on = tl.kbA < tl.K, kbB_on = tl.kbB < tl.K;
  const int nkbA = kbA_on ? (tl.K + tl.kbA - 1) / tl.kbA : 1;
  const int nkbB = kbB_on ? (tl.K + tl.kbB - 1) / tl.kbB : 1;
  const int kinA = kbA_on ? tl.kbA : tl.K;  // k extent inside one block
  const int kinB = kbB_on ? tl.kbB : tl.K;
  const bool aLo = (tl.flags & NMGP_A_LOWER) != 0, aUp = (tl.flags & NMGP_A_UPPER) != 0;
  const bool bLo = (tl.flags & NMGP_B_LOWER) != 0, bUp = (tl.flags & NMGP_B_UPPER) != 0;
  // end of each operand's addressed extent (elements past the base pointer): the OOB bound
  const int64_t endA = tl.r0 * d.sA_i + (int64_t)(tl.m - 1) * d.sA_i + (tl.k0 + kinA - 1) * d.sA_k +
                       (int64_t)(nkbA - 1) * d.sA_kb + 1;
  const int64_t endB = (tl.k0 + kinB - 1) * d.sB_k + (int64_t)(tl.n - 1) * d.sB_j + (int64_t)(nkbB - 1) * d.sB_kb + 1;
  uint32_t offA[8], offB[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    offA[e] = (uint32_t)(((int64_t)(tl.i0 + em.a_il[e]) * d.sA_i + (int64_t)em.a_kl[e] * d.sA_k) * (int64_t)sizeof(T));
    offB[e] = (uint32_t)(((int64_t)em.b_kl[e] * d.sB_k + (int64_t)(tl.j0 + em.b_jl[e]) * d.sB_j) * (int64_t)sizeof(T));
  }
  auto load = [&](int kt, T (&ra)[8], T (&rb)[8], T (&rs)[8], unsigned& okm) {
    const int kbA_u = kbA_on ? kt / tl.kbA : 0, kbB_u = kbB_on ? kt / tl.kbB : 0;
    const int kkA = kt - kbA_u * (kbA_on ? tl.kbA : 0);
    const int kkB = kt - kbB_u * (kbB_on ? tl.kbB : 0);
    const int64_t baseA = tl.r0 * d.sA_i + (tl.k0 + kkA) * d.sA_k + (int64_t)kbA_u * d.sA_kb;
    const int64_t baseB = (tl.k0 + kkB) * d.sB_k + (int64_t)kbB_u * d.sB_kb;
    const __amdgpu_buffer_rsrc_t rA = make_rsrc(Ab + baseA * (int64_t)sizeof(T), (endA - baseA) * (int64_t)sizeof(T));
    const __amdgpu_buffer_rsrc_t rB = make_rsrc(Bb + baseB * (int64_t)sizeof(T), (endB - baseB) * (int64_t)sizeof(T));
#pragma unroll
    for (int e = 0; e < 8; ++e) ra[e] = bload<T>(rA, offA[e]);
#pragma unroll
    for (int e = 0; e < 8; ++e) rb[e] = bload<T>(rB, offB[e]);
    if (KS) {
#pragma unroll
      for (int e = 0; e < 8; ++e) rs[e] = ksc[tl.k0 + min(kt + em.b_kl[e], tl.K - 1)];
    }
    // wave-uniform: does this k-tile need element masks at all?
    // (a triangle applies inside each k-block, so wholly-masked tiles are possible when blocked)
    const bool need = (kt + GBK > tl.kend) || (aLo && kkA + GBK - 1 > tl.i0) || (aUp && kkA < tl.i0 + GBM - 1) ||
                      (bLo && tl.j0 + GBN - 1 > kkB) || (bUp && tl.j0 < kkB + GBK - 1);
    okm = 0xffffu;
    if (need) {
      okm = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        okm |= a_ok(tl.flags, tl.i0 + em.a_il[e], kkA + em.a_kl[e], 0x7fffffff, kt + em.a_kl[e] < tl.kend) ? (1u << e)
                                                                                                          : 0u;
        okm |= b_ok(tl.flags, tl.j0 + em.b_jl[e], kkB + em.b_kl[e], 0x7fffffff, kt + em.b_kl[e] < tl.kend)
                   ? (1u << (8 + e))
                   : 0u;
      }
    }
  };
  T ra[8], rb[8], rs[8];
  unsigned okm = 0;
  load(tl.kbeg, ra, rb, rs, okm);
  GEMM_STAMP(2);
  [[maybe_unused]] int it = 0;
  for (int kt = tl.kbeg; kt < tl.kend; kt += GBK) {
    stage_lds(As, Bs, em, ra, rb, rs, okm, KS);
    lds_barrier();
    GEMM_STAMP(3 + 2 * min(it, 30));
    if (kt + GBK < tl.kend) load(kt + GBK, ra, rb, rs, okm);
    mma_tile(As, Bs, lane, wr, wc, c00, c01, c10, c11);
    lds_barrier();
    GEMM_STAMP(4 + 2 * min(it, 30));
    ++it;
  }
}

// General main loop (k-blocks not aligned to GBK, small shapes): per-element block index.
template <typename T, typename Acc>
__device__ inline void mainloop_general(const nmgp_gemm_desc& d, const Tile& tl, const EltMap& em, T* As, T* Bs,
                                        int lane, int wr, int wc, Acc& c00, Acc& c01, Acc& c10, Acc& c11) {
  const GPtr<const T> A = (GPtr<const T>)d.A;
  const GPtr<const T> Bm = (GPtr<const T>)d.B;
  const GPtr<const T> ksc = (GPtr<const T>)(d.kscale ? d.kscale : d.B);
  const bool ksf = (tl.flags & NMGP_KSCALE) != 0;
  const bool kbA_on = tl.kbA < tl.K, kbB_on = tl.kbB < tl.K;
  auto load = [&](int kt, T (&ra)[8], T (&rb)[8], T (&rs)[8], unsigned& okm) {
    okm = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int gi = tl.i0 + em.a_il[e], gk = kt + em.a_kl[e];
      const int gkc = min(gk, tl.K - 1);
      const int kb = kbA_on ? gkc / tl.kbA : 0, kk = gkc - kb * (kbA_on ? tl.kbA : 0);
      ra[e] = A[(tl.r0 + min(gi, tl.m - 1)) * d.sA_i + (tl.k0 + kk) * d.sA_k + (int64_t)kb * d.sA_kb];
      okm |= a_ok(tl.flags, gi, kk, tl.m, gk < tl.kend) ? (1u << e) : 0u;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int gk = kt + em.b_kl[e], gj = tl.j0 + em.b_jl[e];
      const int gkc = min(gk, tl.K - 1);
      const int kb = kbB_on ? gkc / tl.kbB : 0, kk = gkc - kb * (kbB_on ? tl.kbB : 0);
      rb[e] = Bm[(tl.k0 + kk) * d.sB_k + (int64_t)min(gj, tl.n - 1) * d.sB_j + (int64_t)kb * d.sB_kb];
      rs[e] = ksc[tl.k0 + gkc];
      okm |= b_ok(tl.flags, gj, kk, tl.n, gk < tl.kend) ? (1u << (8 + e)) : 0u;
    }
  };
  T ra[8], rb[8], rs[8];
  unsigned okm = 0;
  load(tl.kbeg, ra, rb, rs, okm);
  for (int kt = tl.kbeg; kt < tl.kend; kt += GBK) {
    stage_lds(As, Bs, em, ra, rb, rs, okm, ksf);
    lds_barrier();
    if (kt + GBK < tl.kend) load(kt + GBK, ra, rb, rs, okm);
    mma_tile(As, Bs, lane, wr, wc, c00, c01, c10, c11);
    lds_barrier();
  }
}

template <typename T, bool GROUPED>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs args, const nmgp_gemm_desc* __restrict__ descs) {
  // ONE shared array (a second __shared__ object can make hipcc wait vmcnt(0) in the k-loop)
  __shared__ T smem[LDS_T + 2];
  T* As = smem;
  T* Bs = smem + GBK * LP;
  int* s_last = (int*)(smem + LDS_T);
  GEMM_STAMP(0);
  int tile = blockIdx.x;
  int idx = 0;
  if (GROUPED) {
    int lo = 0, hi = args.nprob - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (descs[mid].tile_start <= tile) lo = mid; else hi = mid - 1;
    }
    idx = lo;
  }
  // by value from a read-only uniform address: scalar loads once (a reference would be re-read after
  // every barrier, whose asm clobbers memory)
  nmgp_gemm_desc d = GROUPED ? descs[idx] : args.inl;
  if (!GROUPED && d.batch > 1) {            // batched single problem: blockIdx.y = problem
    const int64_t b = blockIdx.y;
    d.A = (const char*)d.A + b * d.sA_b * (int64_t)sizeof(T);
    d.B = (const char*)d.B + b * d.sB_b * (int64_t)sizeof(T);
    d.C = (char*)d.C + b * d.sC_b * (int64_t)sizeof(T);
  }
  tile -= d.tile_start;
  const int ksplit = d.ksplit > 1 ? d.ksplit : 1;
  const int ks = tile % ksplit;
  tile /= ksplit;
  const int tn = tile % d.tiles_n, tm = tile / d.tiles_n;
  Tile tl;
  tl.r0 = 0;
  tl.m = d.m;
  const int span = d.seg_span > 0 ? d.seg_span : 1;
  if (d.row_seg >= 0) {
    tl.r0 = args.seg[d.row_seg];
    tl.m = args.seg[d.row_seg + span] - (int)tl.r0;
  }
  tl.k0 = 0;
  tl.K = d.k;
  if (d.k_seg >= 0) {
    tl.k0 = args.seg[d.k_seg];
    tl.K = args.seg[d.k_seg + span] - (int)tl.k0;
  }
  tl.n = d.n;
  tl.i0 = tm * GBM;
  tl.j0 = tn * GBN;
  if (tl.i0 >= tl.m) return;
  tl.flags = d.flags;
  const int flags = tl.flags;
  const bool above = tl.j0 > tl.i0 + GBM - 1;
  if (above && (flags & NMGP_OUT_LOWER)) return;
  const bool zero_tile = above && (flags & NMGP_OUT_TRIL);
  tl.kbA = d.kbA > 0 ? d.kbA : 0x7fffffff;
  tl.kbB = d.kbB > 0 ? d.kbB : 0x7fffffff;
  int kbeg = 0, kend = tl.K;
  if (d.k_seg < 0) {
    if ((flags & NMGP_A_LOWER) && tl.kbA >= tl.K) kend = min(kend, tl.i0 + GBM);
    if ((flags & NMGP_A_UPPER) && tl.kbA >= tl.K) kbeg = max(kbeg, tl.i0);
    if ((flags & NMGP_B_LOWER) && tl.kbB >= tl.K) kbeg = max(kbeg, tl.j0);
    if ((flags & NMGP_B_UPPER) && tl.kbB >= tl.K) kend = min(kend, tl.j0 + GBN);
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
  tl.kbeg = kbeg;
  tl.kend = kend;
  GEMM_STAMP(1);

  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  EltMap em;
  const bool a_kc = (d.sA_k == 1), b_jc = (d.sB_j == 1);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if (a_kc) { em.a_kl[e] = t & 31; em.a_il[e] = (t >> 5) + 8 * e; }
    else { em.a_il[e] = t & 63; em.a_kl[e] = (t >> 6) + 4 * e; }
    if (b_jc) { em.b_jl[e] = t & 63; em.b_kl[e] = (t >> 6) + 4 * e; }
    else { em.b_kl[e] = t & 31; em.b_jl[e] = (t >> 5) + 8 * e; }
  }

  using acc_t = typename Mfma<T>::acc_t;
  acc_t acc00 = {0, 0, 0, 0}, acc01 = {0, 0, 0, 0}, acc10 = {0, 0, 0, 0}, acc11 = {0, 0, 0, 0};
  if (kbeg < kend) {
    const bool kb_fast = (tl.kbA >= tl.K || tl.kbA % GBK == 0) && (tl.kbB >= tl.K || tl.kbB % GBK == 0);
    if (kb_fast && (flags & NMGP_KSCALE))
      mainloop_fast<T, true>(d, tl, em, As, Bs, lane, wr, wc, acc00, acc01, acc10, acc11);
    else if (kb_fast)
      mainloop_fast<T, false>(d, tl, em, As, Bs, lane, wr, wc, acc00, acc01, acc10, acc11);
    else
      mainloop_general<T>(d, tl, em, As, Bs, lane, wr, wc, acc00, acc01, acc10, acc11);
  }

  GEMM_STAMP(70);
  const int64_t r0 = tl.r0;
  const int m = tl.m, n = tl.n, i0 = tl.i0, j0 = tl.j0;
  if (ksplit > 1 && !zero_tile) {
    // deterministic split-K (agent-scope release/acquire hand-off): publish this chunk's partial,
    // the last arriver sums all chunks in chunk order
    GPtr<T> ws = (GPtr<T>)d.ws + (int64_t)(tm * d.tiles_n + tn) * ksplit * 4096;
    GPtr<T> mine = ws + (int64_t)ks * 4096 + t * 16;
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
      *s_last = last;
    }
    __syncthreads();
    if (!*s_last) return;
    acc00 = acc01 = acc10 = acc11 = acc_t{0, 0, 0, 0};
    for (int c = 0; c < ksplit; ++c) {
      GPtr<const T> src = ws + (int64_t)c * 4096 + t * 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc00[r] += src[r];
        acc01[r] += src[4 + r];
        acc10[r] += src[8 + r];
        acc11[r] += src[12 + r];
      }
    }
  }

  const GPtr<T> C = (GPtr<T>)d.C;
  const GPtr<const T> E = (GPtr<const T>)d.epi_E;
  const GPtr<const T> rsp = (GPtr<const T>)d.epi_rs;
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
  GEMM_STAMP(71);
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
  hipLaunchKernelGGL((gemm_kernel<T, true>), dim3(total_tiles), dim3(256), 0, s, a, d_desc);
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
  hipLaunchKernelGGL((gemm_kernel<T, false>), dim3(d.tiles_m * d.tiles_n, d.batch > 1 ? d.batch : 1), dim3(256), 0, s,
                     a, (const nmgp_gemm_desc*)nullptr);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

// internal entry for other translation units (blocked Cholesky)
template <typename T> int gemm_single(const nmgp_gemm_desc& d, hipStream_t s) { return launch_single<T>(&d, nullptr, s); }
template int gemm_single<double>(const nmgp_gemm_desc&, hipStream_t);
template int gemm_single<float>(const nmgp_gemm_desc&, hipStream_t);

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
