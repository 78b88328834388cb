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
#define GEMM_STAMPB(i) \
  if (threadIdx.x == 0 && blockIdx.y == 0) g_gemm_trace[1024 + blockIdx.x * 4 + (i)] = wall_clock64()
#else
#define GEMM_STAMP(i)
#define GEMM_STAMPB(i)
#endif

constexpr int GBM = 64, GBN = 64, GBK = 32, LP = 65;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int LDS_T = 2 * GBK * LP;  // one stage: A image + B image (elements); two stages in flight

struct GemmArgs {
  const nmgp_gemm_desc* descs;
  int nprob;
  int coop;  // whole grid co-resident: split-K chunks combine cooperatively
  const int32_t* seg;
  const int32_t* dyn_start;   // device tile plan (nprob + 1) or nullptr: static tile_start
  nmgp_gemm_desc inl;
};

// Problem geometry resolved for one workgroup (all wave-uniform).
struct Tile {
  int64_t r0, k0;
  int m, n, K, i0, j0, kbeg, kend, kbA, kbB, flags;
};

// Per-thread element map of a GBM x GBK (A) / GBK x GBN (B) tile, 8 elements each, chosen so that
// each load instruction reads consecutive addresses across the wave for either layout.  Element e
// sits at a wave-uniform stride from element 0, so the map costs 4 registers, not 32.
struct EltMap {
  int a_il0, a_kl0, a_ie, a_ke;  // A element e: row a_il0 + e*a_ie, k a_kl0 + e*a_ke
  int b_kl0, b_jl0, b_ke, b_je;  // B element e: k b_kl0 + e*b_ke, column b_jl0 + e*b_je
  __device__ int a_il(int e) const { return a_il0 + e * a_ie; }
  __device__ int a_kl(int e) const { return a_kl0 + e * a_ke; }
  __device__ int b_kl(int e) const { return b_kl0 + e * b_ke; }
  __device__ int b_jl(int e) const { return b_jl0 + e * b_je; }
};

template <typename T, typename Acc>
__device__ inline void mma_step(T a0, T a1, T b0, T b1, Acc& c00, Acc& c01, Acc& c10, Acc& c11) {
  c00 = Mfma<T>::mma(a0, b0, c00);
  c01 = Mfma<T>::mma(a0, b1, c01);
  c10 = Mfma<T>::mma(a1, b0, c10);
  c11 = Mfma<T>::mma(a1, b1, c11);
}

// MFMAs of one LDS stage (As/Bs).  stage(s) runs between the MFMAs of k-step s: the fast main loop
// writes one element per operand of the next k-tile to the other LDS stage there and refetches a
// register unit from global memory, so LDS writes, address arithmetic, vector-memory issue and the
// fragment reads of step s+2 all issue while the matrix pipe is busy.
struct NoStage {
  __device__ void operator()(int) const {}
};

template <typename T, typename Acc, typename Stage = NoStage>
__device__ inline void mma_tile(const T* As, const T* Bs, int lane, int wr, int wc, Acc& c00, Acc& c01, Acc& c10,
                                Acc& c11, const Stage& stage = Stage()) {
  const T* pa = As + (lane >> 4) * LP + wr * 32 + (lane & 15);
  const T* pb = Bs + (lane >> 4) * LP + wc * 32 + (lane & 15);
  // fragments of k-steps s .. s+PF-1 in registers; step s+PF is read while step s multiplies (round 4: PF 2 -> 3,
  // the LDS latency of a fragment read outlasted one 4-MFMA step behind the staging writes)
  constexpr int PF = 3;
  T f[PF][4];
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    const int o = u * 4 * LP;
    f[u][0] = pa[o];
    f[u][1] = pa[o + 16];
    f[u][2] = pb[o];
    f[u][3] = pb[o + 16];
  }
#pragma unroll
  for (int s = 0; s < GBK / 4; ++s) {
    const int u = s % PF;
    const T a0 = f[u][0], a1 = f[u][1], b0 = f[u][2], b1 = f[u][3];
    if (s + PF < GBK / 4) {
      const int o = (s + PF) * 4 * LP;
      f[u][0] = pa[o];
      f[u][1] = pa[o + 16];
      f[u][2] = pb[o];
      f[u][3] = pb[o + 16];
    }
    mma_step(a0, a1, b0, b1, c00, c01, c10, c11);
    stage(s);
  }
}


// Fast-path register tile: 16-byte units (V = 16/sizeof(T) consecutive elements along the operand's
// contiguous dimension), 8/V units per thread and operand, so one buffer_load_dwordx4 fetches V
// elements (vector-memory issue, not bandwidth, bounds the staging beside the MFMAs).  Unit e of A
// starts at (row a_mn0 + e*a_mne, k a_k0 + e*a_ke); its elements run along k if a_pk else along rows.
struct UnitMap {
  int a_mn0, a_k0, a_mne, a_ke, a_pk;
  int b_mn0, b_k0, b_mne, b_ke, b_pk;
};

template <typename T> __device__ inline T unit_elem(u32x4 u, int v);
template <> __device__ inline double unit_elem<double>(u32x4 u, int v) {
  const unsigned lo = v ? u[2] : u[0], hi = v ? u[3] : u[1];
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
template <> __device__ inline float unit_elem<float>(u32x4 u, int v) {
  return __builtin_bit_cast(float, v == 0 ? u[0] : v == 1 ? u[1] : v == 2 ? u[2] : u[3]);
}

// Triangular-operand and bounds validity of element (gi, kk) of A / (kk, gj) of B.
__device__ inline bool a_ok(int flags, int gi, int kk, int m, bool kin) {
  return gi < m && kin && !(((flags & NMGP_A_LOWER) && kk > gi) || ((flags & NMGP_A_UPPER) && kk < gi));
}
__device__ inline bool b_ok(int flags, int gj, int kk, int n, bool kin) {
  return gj < n && kin && !(((flags & NMGP_B_LOWER) && gj > kk) || ((flags & NMGP_B_UPPER) && gj < kk));
}

// Whether the fast main loop can address this tile: k-blocks aligned to GBK, and each operand's
// extent from the tile's first k-tile within the 2 GiB a buffer resource range check covers.
template <typename T>
__device__ inline bool fast_ok(const nmgp_gemm_desc& d, const Tile& tl) {
  const bool kbA_on = tl.kbA < tl.K, kbB_on = tl.kbB < tl.K;
  if ((kbA_on && tl.kbA % GBK) || (kbB_on && tl.kbB % GBK)) return false;
  const int nkbA = kbA_on ? (tl.K + tl.kbA - 1) / tl.kbA : 1, nkbB = kbB_on ? (tl.K + tl.kbB - 1) / tl.kbB : 1;
  const int kinA = kbA_on ? tl.kbA : tl.K, kinB = kbB_on ? tl.kbB : tl.K;
  const int64_t spanA = ((int64_t)(tl.m - 1) * d.sA_i + (int64_t)(kinA - 1) * d.sA_k + (int64_t)(nkbA - 1) * d.sA_kb);
  const int64_t spanB = ((int64_t)(kinB - 1) * d.sB_k + (int64_t)(tl.n - 1) * d.sB_j + (int64_t)(nkbB - 1) * d.sB_kb);
  const int64_t lim = 0x7fffffffLL / (int64_t)sizeof(T) - 64;
  return d.sA_i >= 0 && d.sA_k >= 0 && d.sA_kb >= 0 && d.sB_k >= 0 && d.sB_j >= 0 && d.sB_kb >= 0 && spanA < lim &&
         spanB < lim;
}

// Fast main loop: k-blocks aligned to GBK, so each operand is addressed by one buffer resource over
// its whole extent and per-unit byte offsets that advance by a uniform step per k-tile (a jump at a
// k-block boundary).  Reads past the extent return 0 (the range check is per dword).  Element masks
// are applied, when staging, only to k-tiles that need them (the k tail, tiles straddling a
// triangular operand's diagonal); rows past m / columns past n need none: they only feed outputs
// that are never stored.  Two LDS stages: the MFMAs of k-tile t run while tile t+1 is written from
// registers to the other stage and tile t+2 is fetched into them; one barrier per k-tile.  KS:
// k-scaled B.
template <typename T, bool KS, typename Acc>
__device__ inline void mainloop_fast(const nmgp_gemm_desc& d, const Tile& tl, const UnitMap& um, T* S, int lane,
                                     int wr, int wc, Acc& c00, Acc& c01, Acc& c10, Acc& c11) {
  constexpr int V = 16 / (int)sizeof(T);  // elements per unit
  constexpr int NU = 8 / V;               // units per thread and operand
  constexpr int64_t sz = sizeof(T);
  const GPtr<const T> ksc = (GPtr<const T>)(d.kscale ? d.kscale : d.B);
  const bool kbA_on = tl.kbA < tl.K, kbB_on = tl.kbB < tl.K;
  const int nkbA = kbA_on ? (tl.K + tl.kbA - 1) / tl.kbA : 1;
  const int nkbB = kbB_on ? (tl.K + tl.kbB - 1) / tl.kbB : 1;
  const int kinA = kbA_on ? tl.kbA : tl.K;  // k extent inside one block
  const int kinB = kbB_on ? tl.kbB : tl.K;
  const bool aLo = (tl.flags & NMGP_A_LOWER) != 0, aUp = (tl.flags & NMGP_A_UPPER) != 0;
  const bool bLo = (tl.flags & NMGP_B_LOWER) != 0, bUp = (tl.flags & NMGP_B_UPPER) != 0;
  // position of the first k-tile inside its k-block
  int kbuA = kbA_on ? tl.kbeg / tl.kbA : 0, kbuB = kbB_on ? tl.kbeg / tl.kbB : 0;
  int kkA = tl.kbeg - kbuA * (kbA_on ? tl.kbA : 0), kkB = tl.kbeg - kbuB * (kbB_on ? tl.kbB : 0);
  const int64_t baseA = tl.r0 * d.sA_i + (tl.k0 + kkA) * d.sA_k + (int64_t)kbuA * d.sA_kb;
  const int64_t baseB = (tl.k0 + kkB) * d.sB_k + (int64_t)kbuB * d.sB_kb;
  const int64_t endA = tl.r0 * d.sA_i + (int64_t)(tl.m - 1) * d.sA_i + (tl.k0 + kinA - 1) * d.sA_k +
                       (int64_t)(nkbA - 1) * d.sA_kb + 1;
  const int64_t endB = (tl.k0 + kinB - 1) * d.sB_k + (int64_t)(tl.n - 1) * d.sB_j + (int64_t)(nkbB - 1) * d.sB_kb + 1;
  const __amdgpu_buffer_rsrc_t rA = make_rsrc((const char*)d.A + baseA * sz, (endA - baseA) * sz);
  const __amdgpu_buffer_rsrc_t rB = make_rsrc((const char*)d.B + baseB * sz, (endB - baseB) * sz);
  // unit e's byte offset = o + e * os; per k-tile the offsets advance by step (jump at a block end)
  uint32_t oA = (uint32_t)(((int64_t)(tl.i0 + um.a_mn0) * d.sA_i + (int64_t)um.a_k0 * d.sA_k) * sz);
  uint32_t oB = (uint32_t)(((int64_t)um.b_k0 * d.sB_k + (int64_t)(tl.j0 + um.b_mn0) * d.sB_j) * sz);
  const uint32_t osA = (uint32_t)(((int64_t)um.a_mne * d.sA_i + (int64_t)um.a_ke * d.sA_k) * sz);
  const uint32_t osB = (uint32_t)(((int64_t)um.b_ke * d.sB_k + (int64_t)um.b_mne * d.sB_j) * sz);
  const uint32_t stepA = (uint32_t)(GBK * d.sA_k * sz), stepB = (uint32_t)(GBK * d.sB_k * sz);
  const uint32_t jumpA = (uint32_t)((d.sA_kb - (int64_t)(kinA - GBK) * d.sA_k) * sz);
  const uint32_t jumpB = (uint32_t)((d.sB_kb - (int64_t)(kinB - GBK) * d.sB_k) * sz);
  // element s = e*V + v of this thread: LDS offsets of its A and B slots
  const int wa = um.a_k0 * LP + um.a_mn0, wsa = um.a_ke * LP + um.a_mne, wva = um.a_pk ? LP : 1;
  const int wb = um.b_k0 * LP + um.b_mn0, wsb = um.b_ke * LP + um.b_mne, wvb = um.b_pk ? LP : 1;
  auto a_mn = [&](int s) { return um.a_mn0 + (s / V) * um.a_mne + (um.a_pk ? 0 : s % V); };
  auto a_k = [&](int s) { return um.a_k0 + (s / V) * um.a_ke + (um.a_pk ? s % V : 0); };
  auto b_mn = [&](int s) { return um.b_mn0 + (s / V) * um.b_mne + (um.b_pk ? 0 : s % V); };
  auto b_k = [&](int s) { return um.b_k0 + (s / V) * um.b_ke + (um.b_pk ? s % V : 0); };

  unsigned okm = 0xffffu;  // element masks of the k-tile being fetched (bit s: A, bit 8+s: B)
  bool need = false;
  // wave-uniform: does k-tile kt need element masks at all?  (a triangle applies inside each
  // k-block, so wholly-masked tiles are possible when blocked)
  auto prep = [&](int kt) {
    need = (kt + GBK > tl.kend) || (aLo && kkA + GBK - 1 > tl.i0) || (aUp && kkA < tl.i0 + GBM - 1) ||
           (bLo && tl.j0 + GBN - 1 > kkB) || (bUp && tl.j0 < kkB + GBK - 1);
    okm = 0xffffu;
    if (need) {
      okm = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        okm |= a_ok(tl.flags, tl.i0 + a_mn(q), kkA + a_k(q), 0x7fffffff, kt + a_k(q) < tl.kend) ? (1u << q) : 0u;
        okm |= b_ok(tl.flags, tl.j0 + b_mn(q), kkB + b_k(q), 0x7fffffff, kt + b_k(q) < tl.kend) ? (1u << (8 + q))
                                                                                                 : 0u;
      }
    }
  };
  u32x4 ra[NU], rb[NU];
  T rs[8];
  int kload = tl.kbeg;  // k-tile the issue() calls fetch
  auto issue = [&](int e) {
    ra[e] = __builtin_amdgcn_raw_buffer_load_b128(rA, oA + e * osA, 0, 0);
    rb[e] = __builtin_amdgcn_raw_buffer_load_b128(rB, oB + e * osB, 0, 0);
    if (KS) {
#pragma unroll
      for (int v = 0; v < V; ++v) rs[e * V + v] = ksc[tl.k0 + min(kload + b_k(e * V + v), tl.K - 1)];
    }
  };
  auto step1 = [&]() {
    kload += GBK;
    kkA += GBK;
    if (kbA_on && kkA >= kinA) { kkA = 0; oA += jumpA; } else { oA += stepA; }
    kkB += GBK;
    if (kbB_on && kkB >= kinB) { kkB = 0; oB += jumpB; } else { oB += stepB; }
  };
  // k-tiles wholly inside a triangular operand's zero triangle are never fetched (inside k-blocks
  // the range trimming of the caller cannot remove them; uniform scalar test)
  auto tile_empty = [&]() {
    return (aLo && kkA > tl.i0 + GBM - 1) || (aUp && kkA + GBK - 1 < tl.i0) || (bLo && tl.j0 > kkB + GBK - 1) ||
           (bUp && tl.j0 + GBN - 1 < kkB);
  };
  auto advance = [&]() {
    step1();
    while (kload < tl.kend && tile_empty()) step1();
  };
  unsigned okm_st = 0xffffu;  // masks of the k-tile held in registers
  // element s of the register tile into LDS stage N (masked if the tile needs it); the last
  // element of a unit frees its registers for the refetch
  auto put = [&](T* N, int s, bool masked) {
    const int e = s / V, v = s % V;
    T a = unit_elem<T>(ra[e], v), b = unit_elem<T>(rb[e], v);
    if (masked) {
      a = keep_if(a, (okm_st >> s) & 1u);
      b = keep_if(b, (okm_st >> (8 + s)) & 1u);
    }
    if (KS) b *= rs[s];
    N[wa + e * wsa + v * wva] = a;
    N[GBK * LP + wb + e * wsb + v * wvb] = b;
  };
  while (kload < tl.kend && tile_empty()) step1();
  if (kload >= tl.kend) return;  // every k-tile of the range is structurally zero
  prep(kload);
#pragma unroll
  for (int e = 0; e < NU; ++e) issue(e);
  advance();
  okm_st = okm;
  GEMM_STAMP(2);
  if (need) {
#pragma unroll
    for (int q = 0; q < 8; ++q) put(S, q, true);
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) put(S, q, false);
  }
  // tiles past kend read garbage or zeros and are masked when staged, so the fetch needs no guard
  int kreg = kload;  // k-tile now being fetched into the registers
  prep(kload);
#pragma unroll
  for (int e = 0; e < NU; ++e) issue(e);
  advance();
  okm_st = okm;
  bool need_st = need;
  prep(kload);
  lds_barrier();
  int cur = 0;
  [[maybe_unused]] int it = 0;
  while (kreg < tl.kend) {  // LDS stage cur holds a tile, the registers hold tile kreg
    T* As = S + cur * LDS_T;
    T* Ns = S + (cur ^ 1) * LDS_T;
    GEMM_STAMP(3 + 2 * min(it, 30));
    if (need_st) {
      mma_tile(As, As + GBK * LP, lane, wr, wc, c00, c01, c10, c11, [&](int q) {
        put(Ns, q, true);
        if (q % V == V - 1) issue(q / V);
      });
    } else {
      mma_tile(As, As + GBK * LP, lane, wr, wc, c00, c01, c10, c11, [&](int q) {
        put(Ns, q, false);
        if (q % V == V - 1) issue(q / V);
      });
    }
    okm_st = okm;
    need_st = need;
    kreg = kload;
    GEMM_STAMP(100 + 4 * min(it, 30));
    advance();
    prep(kload);
    GEMM_STAMP(101 + 4 * min(it, 30));
    lds_barrier();
    GEMM_STAMP(4 + 2 * min(it, 30));
    cur ^= 1;
    ++it;
  }
  T* As = S + cur * LDS_T;
  mma_tile(As, As + GBK * LP, lane, wr, wc, c00, c01, c10, c11);
}

// General main loop (k-blocks not aligned to GBK, small shapes): per-element block index and
// clamped unconditional loads (masked when staged), one LDS stage, next k-tile fetched during the
// MFMAs.
template <typename T, typename Acc>
__device__ inline void mainloop_general(const nmgp_gemm_desc& d, const Tile& tl, const EltMap& em, T* S, int lane,
                                        int wr, int wc, Acc& c00, Acc& c01, Acc& c10, Acc& c11) {
  const GPtr<const T> A = (GPtr<const T>)d.A;
  const GPtr<const T> Bm = (GPtr<const T>)d.B;
  const GPtr<const T> ksc = (GPtr<const T>)(d.kscale ? d.kscale : d.B);
  const bool ksf = (tl.flags & NMGP_KSCALE) != 0;
  const bool kbA_on = tl.kbA < tl.K, kbB_on = tl.kbB < tl.K;
  auto load = [&](int kt, T (&ra)[8], T (&rb)[8], T (&rs)[8], unsigned& okm) {
    okm = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int gi = tl.i0 + em.a_il(e), gk = kt + em.a_kl(e);
      const int gkc = min(gk, tl.K - 1);
      const int kb = kbA_on ? gkc / tl.kbA : 0, kk = gkc - kb * (kbA_on ? tl.kbA : 0);
      ra[e] = A[(tl.r0 + min(gi, tl.m - 1)) * d.sA_i + (tl.k0 + kk) * d.sA_k + (int64_t)kb * d.sA_kb];
      okm |= a_ok(tl.flags, gi, kk, tl.m, gk < tl.kend) ? (1u << e) : 0u;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int gk = kt + em.b_kl(e), gj = tl.j0 + em.b_jl(e);
      const int gkc = min(gk, tl.K - 1);
      const int kb = kbB_on ? gkc / tl.kbB : 0, kk = gkc - kb * (kbB_on ? tl.kbB : 0);
      rb[e] = Bm[(tl.k0 + kk) * d.sB_k + (int64_t)min(gj, tl.n - 1) * d.sB_j + (int64_t)kb * d.sB_kb];
      rs[e] = ksf ? ksc[tl.k0 + gkc] : (T)1;
      okm |= b_ok(tl.flags, gj, kk, tl.n, gk < tl.kend) ? (1u << (8 + e)) : 0u;
    }
  };
  T* As = S;
  T* Bs = S + GBK * LP;
  T ra[8], rb[8], rs[8];
  unsigned okm = 0;
  load(tl.kbeg, ra, rb, rs, okm);
  for (int kt = tl.kbeg; kt < tl.kend; kt += GBK) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      As[em.a_kl(e) * LP + em.a_il(e)] = keep_if(ra[e], (okm >> e) & 1u);
      const T bv = keep_if(rb[e], (okm >> (8 + e)) & 1u);
      Bs[em.b_kl(e) * LP + em.b_jl(e)] = ksf ? bv * rs[e] : bv;
    }
    lds_barrier();
    if (kt + GBK < tl.kend) load(kt + GBK, ra, rb, rs, okm);
    mma_tile(As, Bs, lane, wr, wc, c00, c01, c10, c11);
    lds_barrier();
  }
}

// One output tile (or split-K chunk) `tile` of the launch: problem lookup, k-loop, epilogue.
template <typename T, bool GROUPED>
__device__ __forceinline__ void gemm_body(const GemmArgs& args, const nmgp_gemm_desc* __restrict__ descs, T* smem,
                                          int tile) {
  int* s_last = (int*)(smem + 2 * LDS_T);
  GEMM_STAMP(0);
  GEMM_STAMPB(0);
  int idx = 0;
  const int32_t* dyn = args.dyn_start;
  if (GROUPED) {
    // problem = last one whose first tile <= tile (problems with no tiles share the next start)
    int lo = 0, hi = args.nprob - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      const int st = dyn ? dyn[mid] : descs[mid].tile_start;
      if (st <= tile) lo = mid; else hi = mid - 1;
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
  tile -= (GROUPED && dyn) ? dyn[idx] : d.tile_start;
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
  if (d.sA_k == 1) { em.a_kl0 = t & 31; em.a_il0 = t >> 5; em.a_ie = 8; em.a_ke = 0; }
  else { em.a_il0 = t & 63; em.a_kl0 = t >> 6; em.a_ie = 0; em.a_ke = 4; }
  if (d.sB_j == 1) { em.b_jl0 = t & 63; em.b_kl0 = t >> 6; em.b_je = 0; em.b_ke = 4; }
  else { em.b_kl0 = t & 31; em.b_jl0 = t >> 5; em.b_je = 8; em.b_ke = 0; }
  UnitMap um;
  {
    constexpr int V = 16 / (int)sizeof(T);
    constexpr int KU = GBK / V, MU = GBM / V, NUU = GBN / V;
    if (d.sA_k == 1) { um.a_k0 = (t % KU) * V; um.a_mn0 = t / KU; um.a_mne = 256 / KU; um.a_ke = 0; um.a_pk = 1; }
    else { um.a_mn0 = (t % MU) * V; um.a_k0 = t / MU; um.a_ke = 256 / MU; um.a_mne = 0; um.a_pk = 0; }
    if (d.sB_j == 1) { um.b_mn0 = (t % NUU) * V; um.b_k0 = t / NUU; um.b_ke = 256 / NUU; um.b_mne = 0; um.b_pk = 0; }
    else { um.b_k0 = (t % KU) * V; um.b_mn0 = t / KU; um.b_mne = 256 / KU; um.b_ke = 0; um.b_pk = 1; }
  }

  using acc_t = typename Mfma<T>::acc_t;
  acc_t acc00 = {0, 0, 0, 0}, acc01 = {0, 0, 0, 0}, acc10 = {0, 0, 0, 0}, acc11 = {0, 0, 0, 0};
  if (kbeg < kend) {
    const bool kb_fast = fast_ok<T>(d, tl);
    if (kb_fast && (flags & NMGP_KSCALE))
      mainloop_fast<T, true>(d, tl, um, smem, lane, wr, wc, acc00, acc01, acc10, acc11);
    else if (kb_fast)
      mainloop_fast<T, false>(d, tl, um, smem, lane, wr, wc, acc00, acc01, acc10, acc11);
    else
      mainloop_general<T>(d, tl, em, smem, lane, wr, wc, acc00, acc01, acc10, acc11);
  }

  GEMM_STAMP(70);
  GEMM_STAMPB(1);
  const int64_t r0 = tl.r0;
  const int m = tl.m, n = tl.n, i0 = tl.i0, j0 = tl.j0;
  const GPtr<T> C = (GPtr<T>)d.C;
  const GPtr<const T> E = (GPtr<const T>)d.epi_E;
  const GPtr<const T> rsp = (GPtr<const T>)d.epi_rs;
  const T alpha = (T)d.alpha, beta = (T)d.beta, gamma = (T)d.gamma, dadd = (T)d.diag_add;
  // C(gi, gj) <- alpha * acc [+ beta C] [+ gamma rs(i) E] [+ diag], honouring the output masks
  auto emit = [&](int gi, int gj, T a) {
    if (gi >= m || gj >= n) return;
    const bool upper = gj > gi;
    if (upper && (flags & NMGP_OUT_LOWER)) return;
    const int64_t ci = (r0 + gi) * d.sC_i + (int64_t)gj * d.sC_j;
    T val;
    if (upper && (flags & NMGP_OUT_TRIL)) {
      val = 0;
    } else {
      val = alpha * a;
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
  };

  if (ksplit > 1 && !zero_tile) {
    // Deterministic split-K.  Every chunk publishes its partial tile write-through (sc1 stores: no
    // L2 write-back fence) and, after the workgroup's stores drained, one lane adds to the tile's
    // counter.  Partials are read back only with sc1 loads, which bypass the possibly stale L1, so
    // no acquire fence either.  Thread t owns values [16t, 16t+16) of a chunk (128 B, whole lines).
    constexpr int V = 16 / (int)sizeof(T);  // elements per 16-B access
    const char* wsb = (const char*)d.ws + (int64_t)(tm * d.tiles_n + tn) * ksplit * 4096 * (int64_t)sizeof(T);
    const __amdgpu_buffer_rsrc_t rws = make_rsrc(wsb, (int64_t)ksplit * 4096 * (int64_t)sizeof(T));
    {
      T vals[16];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        vals[r] = acc00[r];
        vals[4 + r] = acc01[r];
        vals[8 + r] = acc10[r];
        vals[12 + r] = acc11[r];
      }
      const uint32_t off = (uint32_t)(((int64_t)ks * 4096 + t * 16) * (int64_t)sizeof(T));
#pragma unroll
      for (int q = 0; q < 16 / V; ++q) {
        T w[V];
#pragma unroll
        for (int v = 0; v < V; ++v) w[v] = vals[q * V + v];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, w), rws, off + q * 16, 0, 16 /* sc1 */);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    GEMM_STAMPB(2);
    int32_t* ctr = d.counters + tm * d.tiles_n + tn;
    if (args.coop) {
      // Cooperative combine (the host enables it only when the whole grid is co-resident): all
      // chunks of the tile wait for each other, then chunk ks sums 256-value blocks b = ks, ks+S, ...
      // of the tile over all S chunks in chunk order and stores them -- S workgroups share the
      // combine instead of one summing S x 32 KB alone.
      if (t == 0) {
        __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // bounded spin: a lost peer must not hang the GPU (the result is then wrong, not stuck)
        bool seen = false;
        for (int spin = 0; spin < (1 << 24); ++spin) {
          if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= ksplit) {
            seen = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (!seen) spin_gave_up(NMGP_STATUS_GEMM_SPIN);   // surfaced by nmgp_device_status()
      }
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the poll
      constexpr int CB = 8;  // chunks in flight per thread
      for (int blk = ks; blk < 16; blk += ksplit) {
        const int idx = blk * 256 + t;
        T sum = 0;
        for (int c0 = 0; c0 < ksplit; c0 += CB) {
          T v[CB];
#pragma unroll
          for (int cc = 0; cc < CB; ++cc) {
            const int c = min(c0 + cc, ksplit - 1);
            v[cc] = bload_sc1<T>(rws, (uint32_t)(((int64_t)c * 4096 + idx) * (int64_t)sizeof(T)));
          }
#pragma unroll
          for (int cc = 0; cc < CB; ++cc) sum += keep_if(v[cc], c0 + cc < ksplit);
        }
        // value idx of the tile = element (idx & 15) of owner thread idx >> 4's accumulators
        const int tau = idx >> 4, q = (idx >> 2) & 3, r = idx & 3;
        const int ol = tau & 63, ow = tau >> 6;
        emit(i0 + (ow >> 1) * 32 + (q >> 1) * 16 + Mfma<T>::row(ol, r), j0 + (ow & 1) * 32 + (q & 1) * 16 + (ol & 15),
             sum);
      }
      if (t == 0) {
        // the last workgroup to leave resets the counter for the next launch
        const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == 2 * ksplit - 1) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      GEMM_STAMPB(3);
      return;
    }
    // Last arriver combines the whole tile.
    if (t == 0) {
      const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = (old == ksplit - 1);
      if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_last = last;
    }
    __syncthreads();
    if (!*s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the poll
    acc00 = acc01 = acc10 = acc11 = acc_t{0, 0, 0, 0};
    constexpr int CU = 4;  // chunks in flight
    for (int c0 = 0; c0 < ksplit; c0 += CU) {
      u32x4 raw[CU][16 / V];
#pragma unroll
      for (int cc = 0; cc < CU; ++cc) {
        const int c = min(c0 + cc, ksplit - 1);
        const uint32_t off = (uint32_t)(((int64_t)c * 4096 + t * 16) * (int64_t)sizeof(T));
#pragma unroll
        for (int q = 0; q < 16 / V; ++q) raw[cc][q] = __builtin_amdgcn_raw_buffer_load_b128(rws, off + q * 16, 0, 16);
      }
#pragma unroll
      for (int cc = 0; cc < CU; ++cc) {
        // chunks past the last were loaded clamped: add them as zeros (branch-free, so the loads of
        // all CU chunks stay in flight together)
        const bool live = c0 + cc < ksplit;
        T vals[16];
#pragma unroll
        for (int q = 0; q < 16 / V; ++q) {
          struct W { T v[V]; } w = __builtin_bit_cast(W, raw[cc][q]);
#pragma unroll
          for (int v = 0; v < V; ++v) vals[q * V + v] = keep_if(w.v[v], live);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          acc00[r] += vals[r];
          acc01[r] += vals[4 + r];
          acc10[r] += vals[8 + r];
          acc11[r] += vals[12 + r];
        }
      }
    }
  }

  // The thread's 16 outputs.  C (beta != 0) and the epilogue operand rs(i) E(i, j) are read for all 16 before the
  // first store, as branch-free buffer loads (an element that is not read takes an out-of-range offset and reads
  // 0): emit() per element waited on each C / E load before its store and the next load (16-32 dependent round
  // trips per tile).  Spans of 2 GiB or more keep the per-element form.
  const int64_t sz = (int64_t)sizeof(T);
  const int64_t extC = ((r0 + m - 1) * d.sC_i + (int64_t)(n - 1) * d.sC_j + 1) * sz;
  const int64_t extE = (flags & NMGP_EPI) ? ((r0 + m - 1) * d.sE_i + (int64_t)(n - 1) * d.sE_j + 1) * sz : 0;
  // (negative strides take emit(): a negative extent would build a 0-record resource that reads every element as 0)
  if (extC < 0x7fffffffLL && extE < 0x7fffffffLL && d.sC_i >= 0 && d.sC_j >= 0 &&
      (!(flags & NMGP_EPI) || (d.sE_i >= 0 && d.sE_j >= 0))) {
    const bool ldc = beta != (T)0, epi = (flags & NMGP_EPI) != 0;
    const __amdgpu_buffer_rsrc_t rC = make_rsrc(d.C, extC);
    const __amdgpu_buffer_rsrc_t rE = make_rsrc(epi ? d.epi_E : d.C, extE);
    const __amdgpu_buffer_rsrc_t rR = make_rsrc(epi && rsp ? (const void*)d.epi_rs : d.C, epi && rsp ? (r0 + m) * sz : 0);
    // raw values only in the load loop (arithmetic and flag tests there made the compiler wait on each load)
    T cv[16], ev[16], rv[8];
    const uint32_t oob = 0x80000000u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = i0 + wr * 32 + (q >> 1) * 16 + Mfma<T>::row(lane, r), gj = j0 + wc * 32 + (q & 1) * 16 + (lane & 15);
        const bool upper = gj > gi;
        const bool rd = gi < m && gj < n && !(upper && (flags & (NMGP_OUT_LOWER | NMGP_OUT_TRIL)));
        const bool rde = epi && rd && !((flags & NMGP_EPI_E_LOWER) && upper);
        cv[4 * q + r] = bload<T>(rC, ldc && rd ? (uint32_t)(((r0 + gi) * d.sC_i + (int64_t)gj * d.sC_j) * sz) : oob);
        ev[4 * q + r] = bload<T>(rE, rde ? (uint32_t)(((r0 + gi) * d.sE_i + (int64_t)gj * d.sE_j) * sz) : oob);
        if ((q & 1) == 0) rv[4 * (q >> 1) + r] = bload<T>(rR, gi < m ? (uint32_t)((r0 + gi) * sz) : oob);
      }
    }
    const T rsgn = (flags & NMGP_EPI_RS_NEG) ? (T)-1 : (T)1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const acc_t& acc = q == 0 ? acc00 : q == 1 ? acc01 : q == 2 ? acc10 : acc11;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = i0 + wr * 32 + (q >> 1) * 16 + Mfma<T>::row(lane, r), gj = j0 + wc * 32 + (q & 1) * 16 + (lane & 15);
        if (gi >= m || gj >= n) continue;
        const bool upper = gj > gi;
        if (upper && (flags & NMGP_OUT_LOWER)) continue;
        T val;
        if (upper && (flags & NMGP_OUT_TRIL)) {
          val = 0;
        } else {
          val = alpha * acc[r];
          if (ldc) val += beta * cv[4 * q + r];
          if (epi) {
            const T rs = (rsp ? rv[4 * (q >> 1) + r] : (T)1) * rsgn;
            val += gamma * rs * ev[4 * q + r];
          }
          if ((flags & NMGP_DIAG_ADD) && gi == gj) val += dadd;
        }
        C[(r0 + gi) * d.sC_i + (int64_t)gj * d.sC_j] = val;
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const acc_t& acc = q == 0 ? acc00 : q == 1 ? acc01 : q == 2 ? acc10 : acc11;
      const int mi = q >> 1, ni = q & 1;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        emit(i0 + wr * 32 + mi * 16 + Mfma<T>::row(lane, r), j0 + wc * 32 + ni * 16 + (lane & 15), acc[r]);
    }
  }
  GEMM_STAMP(71);
  GEMM_STAMPB(3);
}

// Static grids run one tile per workgroup.  With a device tile plan (args.dyn_start, written by
// gemm_plan_kernel from the segment table just before) the grid is a fixed number of workgroups
// striding over the tiles that exist for this minibatch: row-segmented problems (rows of one
// output) launch no workgroups for the rows other outputs own.
template <typename T, bool GROUPED>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmArgs args, const nmgp_gemm_desc* __restrict__ descs) {
  // ONE shared array (a second __shared__ object can make hipcc wait vmcnt(0) in the k-loop)
  __shared__ T smem[2 * LDS_T + 2];
  if constexpr (!GROUPED) {
    gemm_body<T, false>(args, descs, smem, blockIdx.x);
    return;
  }
  const int total = args.dyn_start ? args.dyn_start[args.nprob] : (int)gridDim.x;
  for (int tile = blockIdx.x; tile < total; tile += gridDim.x) {
    gemm_body<T, GROUPED>(args, descs, smem, tile);
    __syncthreads();
  }
}

// Tile plan of a grouped launch for this minibatch: dyn_start[p] = first tile of problem p with
// row-segmented problems sized by their actual segment (<= the static tiles_m), dyn_start[nprob] =
// total.  One workgroup, block-wide exclusive scan in chunks of 256 problems.
__global__ __launch_bounds__(256) void gemm_plan_kernel(const nmgp_gemm_desc* __restrict__ descs, int nprob,
                                                        const int32_t* __restrict__ seg, int32_t* dyn_start) {
  __shared__ int buf[256];
  __shared__ int carry;
  const int t = threadIdx.x;
  if (t == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < nprob; base += 256) {
    const int p = base + t;
    int v = 0;
    if (p < nprob) {
      const nmgp_gemm_desc& d = descs[p];
      int tm = d.tiles_m;
      if (d.row_seg >= 0 && seg != nullptr) {
        const int span = d.seg_span > 0 ? d.seg_span : 1;
        const int m = seg[d.row_seg + span] - seg[d.row_seg];
        tm = min(tm, max(0, (m + GBM - 1) / GBM));
      }
      v = tm * d.tiles_n * (d.ksplit > 1 ? d.ksplit : 1);
    }
    buf[t] = v;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {   // Hillis-Steele inclusive scan
      const int add = t >= off ? buf[t - off] : 0;
      __syncthreads();
      buf[t] += add;
      __syncthreads();
    }
    if (p < nprob) dyn_start[p] = carry + buf[t] - v;
    __syncthreads();
    if (t == 255) carry += buf[255];
    __syncthreads();
  }
  if (t == 0) dyn_start[nprob] = carry;
}

// Workgroups of the grouped kernel that are certainly resident at once: CUs x min(occupancy API, 2)
// (LDS and VGPRs allow two 256-thread workgroups per CU; the API can report one block too many).
template <typename T>
static int coresident_wgs() {
  static int cap = -1;
  if (cap < 0) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, gemm_kernel<T, true>, 256, 0) != hipSuccess) {
      cap = 0;
    } else {
      cap = cus * (per < 2 ? per : 2);
    }
  }
  return cap;
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
  a.coop = total_tiles <= coresident_wgs<T>() ? 1 : 0;
  a.seg = d_seg;
  a.dyn_start = nullptr;
  a.inl = nmgp_gemm_desc{};
  hipLaunchKernelGGL((gemm_kernel<T, true>), dim3(total_tiles), dim3(256), 0, s, a, d_desc);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

// Grouped launch sized on device: plan kernel (tiles of this minibatch's segments) + a grid of
// `grid` workgroups striding over them.  Split-K combines by last arriver (no co-residency waits).
template <typename T>
static int launch_grouped_dyn(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles, const int32_t* d_seg,
                              int32_t* d_plan, int grid, hipStream_t s, bool planned = false) {
  if (d_desc == nullptr) return -1;
  if (nprob <= 0) return -2;
  if (total_tiles < 0) return -3;
  if (d_plan == nullptr) return -5;
  if (total_tiles == 0) return NMGP_OK;
  if (grid <= 0 || grid > total_tiles) grid = total_tiles;
  if (!planned) {
    hipLaunchKernelGGL(gemm_plan_kernel, dim3(1), dim3(256), 0, s, d_desc, nprob, d_seg, d_plan);
    NMGP_CHECK_LAUNCH();
  }
  GemmArgs a;
  a.descs = d_desc;
  a.nprob = nprob;
  a.coop = 0;
  a.seg = d_seg;
  a.dyn_start = d_plan;
  a.inl = nmgp_gemm_desc{};
  hipLaunchKernelGGL((gemm_kernel<T, true>), dim3(grid), dim3(256), 0, s, a, d_desc);
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
  a.coop = 0;
  a.seg = d_seg;
  a.dyn_start = nullptr;
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

NMGP_TU_STATUS_ACCESSOR(gemm)

}  // namespace nmgp

extern "C" {
int nmgp_version(void) { return 1; }
int64_t nmgp_sizeof_gemm_desc(void) { return (int64_t)sizeof(nmgp_gemm_desc); }
int64_t nmgp_sizeof_pairwise_desc(void) { return (int64_t)sizeof(nmgp_pairwise_desc); }
int64_t nmgp_sizeof_pairwise_bwd_desc(void) { return (int64_t)sizeof(nmgp_pairwise_bwd_desc); }
int64_t nmgp_sizeof_dsvi_args(void) { return (int64_t)sizeof(nmgp_dsvi_args); }
int64_t nmgp_sizeof_pair_desc(void) { return (int64_t)sizeof(nmgp_pair_desc); }

int nmgp_gemm_grouped_f64(const nmgp_gemm_desc* d, int np, int tt, const int32_t* seg, hipStream_t s) {
  return nmgp::launch_grouped<double>(d, np, tt, seg, s);
}
int nmgp_gemm_grouped_dyn_f64(const nmgp_gemm_desc* d, int np, int tt, const int32_t* seg, int32_t* plan, int grid,
                              hipStream_t s) {
  return nmgp::launch_grouped_dyn<double>(d, np, tt, seg, plan, grid, s);
}
int nmgp_gemm_grouped_dyn_f32(const nmgp_gemm_desc* d, int np, int tt, const int32_t* seg, int32_t* plan, int grid,
                              hipStream_t s) {
  return nmgp::launch_grouped_dyn<float>(d, np, tt, seg, plan, grid, s);
}
int nmgp_gemm_plan(const nmgp_gemm_desc* d, int np, const int32_t* seg, int32_t* plan, hipStream_t s) {
  if (!d || !plan) return -1;
  if (np <= 0) return -2;
  hipLaunchKernelGGL(nmgp::gemm_plan_kernel, dim3(1), dim3(256), 0, s, d, np, seg, plan);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
int nmgp_gemm_grouped_dyn_planned_f64(const nmgp_gemm_desc* d, int np, int tt, const int32_t* seg, int32_t* plan,
                                      int grid, hipStream_t s) {
  return nmgp::launch_grouped_dyn<double>(d, np, tt, seg, plan, grid, s, true);
}
int nmgp_gemm_grouped_dyn_planned_f32(const nmgp_gemm_desc* d, int np, int tt, const int32_t* seg, int32_t* plan,
                                      int grid, hipStream_t s) {
  return nmgp::launch_grouped_dyn<float>(d, np, tt, seg, plan, grid, s, true);
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
