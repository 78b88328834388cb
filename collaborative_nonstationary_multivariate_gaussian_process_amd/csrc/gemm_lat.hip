// Latency-oriented grouped GEMM for the short-k products of the DSVI step (same descriptors and
// semantics as gemm.hip's grouped kernel; the host picks this kernel per group, hip_ops.GemmGroup).
//
// The step's GEMMs are B x M x M and M x M x M products with k = M = 256 (projections T = K12 C^-T,
// P = T C^-1, the quadratic-form factors W = P L, the P-bar / R adjoints, C^-T C^-1): 0.1-1 GFLOP
// each, a few hundred 64x64 tiles, 4-8 k-tiles per tile.  There the LDS-staged kernel waits on one
// global round trip per k-tile and on split-K hand-offs, and reaches 5-18% MFMA-busy.  This kernel
// is shaped for latency instead:
//   * 32x32 output tile per workgroup, the k range split over its waves in 32- or 64-wide panels (wave w
//     takes panels w, w+LW, ...), partial tiles summed through LDS in wave order (deterministic);
//   * no LDS staging of operands: each lane loads exactly the MFMA operands it feeds, straight into
//     registers, all of a panel's loads in flight at once.  The k index is permuted inside a panel
//     (MFMA step s, k-slot g = lane >> 4 takes k = kp + NV g + s, NV = panel / 4), so a lane's NV
//     values of one row of A (or column of B) are consecutive in k: 16-byte loads for a k-contiguous
//     operand, or a 128-byte segment across 16 lanes per load (k step in the scalar offset) for an
//     m/n-contiguous one;
//   * XCD-aware tile order: workgroup b runs on XCD b % 8 and gets tile (b % 8) * per + b / 8, so all
//     column tiles of a row block (which share its A rows) run on one XCD and hit its L2.
// Masks (bounds, triangular operands, k tail), k-blocked operands (kb % 64 == 0), segment-table row
// and k ranges, k-scaling, output masks and the beta / rs(i) E / diagonal epilogue follow
// nmgp_gemm_desc exactly.  Long k ranges (the M x M x B reductions over the minibatch) are also split
// over workgroups (desc.ksplit), partials combined by the last arriving chunk in chunk order.
#include "common.hpp"


namespace nmgp {
#ifdef NMGP_LAT_TRACE
// tools/lat_trace.hip only: shader-cycle stamps of wave 0 of every workgroup's first tile (8 per workgroup)
__device__ unsigned long long* g_lat_trace;
#define LAT_STAMP(i)                                                                          \
  if (threadIdx.x == 0 && first_tile) {                                                       \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                               \
    g_lat_trace[blockIdx.x * 8 + (i)] = __builtin_readcyclecounter();                         \
  }
#else
#define LAT_STAMP(i)
#endif
namespace {

constexpr int LTM = 32, LTN = 32;
typedef unsigned int lu32x4 __attribute__((ext_vector_type(4)));

struct LatArgs {
  const nmgp_gemm_desc* descs;
  int nprob;
  int total;                  // static tile count (a device plan overrides it)
  const int32_t* seg;
  const int32_t* dyn_start;   // device tile plan (nprob + 1) or nullptr
};

// NV values of one lane's operand row (A) / column (B), consecutive in k
template <typename T, int NV>
__device__ inline void loadv(T (&v)[NV], __amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t step, bool contig) {
  if (contig) {
    constexpr int V = 16 / (int)sizeof(T);
#pragma unroll
    for (int q = 0; q < NV / V; ++q) {
      const lu32x4 u = __builtin_amdgcn_raw_buffer_load_b128(r, off, 16 * q, 0);
      struct W { T x[V]; } w = __builtin_bit_cast(W, u);
#pragma unroll
      for (int e = 0; e < V; ++e) v[q * V + e] = w.x[e];
    }
  } else {
    // the k step is wave-uniform: it goes into the scalar offset, so the NV loads share one address VGPR
#pragma unroll
    for (int s = 0; s < NV; ++s) {
      if constexpr (sizeof(T) == 8)
        v[s] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, off, s * step, 0));
      else
        v[s] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, off, s * step, 0));
    }
  }
}

// One output tile (or COLPACK tile group) of a launch decoded from its descriptor: wave-uniform scalars plus this
// wave's panel range.  (The operands' buffer resources are rebuilt from it where they are used: a resource carried
// across the persistent kernel's loop becomes a loop phi the compiler places in VGPRs, and every load a waterfall.)
struct LatJob {
  int prob, tid, ks, ksplit, i0, m, K, flags;
  int64_t r0, k0;
  int jt[2], tnp[2];
  bool pack, blkA, blkB, first_tile;
  int kbA, kbB;
  int pfirst, pstep, npan, j0, kbeg, kend;
};

// decode tile `tile` of the launch; false when it has no output (rows past the segment, masked-out tiles)
template <typename T, int LW, int LKP>
__device__ __forceinline__ bool lat_decode(const LatArgs& args, const nmgp_gemm_desc* __restrict__ descs,
                                           const int32_t* __restrict__ dyn, int tile, bool first_tile, LatJob& J) {
  LAT_STAMP(0);
  int lo = 0, hi = args.nprob - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    const int st = dyn ? dyn[mid] : descs[mid].tile_start;
    if (st <= tile) lo = mid; else hi = mid - 1;
  }
  // wave-uniform problem index: the descriptor then comes in through scalar loads and the buffer
  // resources stay in SGPRs (a VGPR resource would turn every load into a readfirstlane loop)
  lo = __builtin_amdgcn_readfirstlane(lo);
  const nmgp_gemm_desc& d = descs[lo];
  tile -= dyn ? dyn[lo] : d.tile_start;
  LAT_STAMP(1);
  const int ksplit = d.ksplit > 1 ? d.ksplit : 1;
  const int ks = tile % ksplit;
  tile /= ksplit;
  const int tn = tile % d.tiles_n, tm = tile / d.tiles_n;
  const int span = d.seg_span > 0 ? d.seg_span : 1;
  int64_t r0 = 0, k0 = 0;
  int m = d.m, K = d.k;
  if (d.row_seg >= 0) {
    r0 = args.seg[d.row_seg];
    m = args.seg[d.row_seg + span] - (int)r0;
  }
  if (d.k_seg >= 0) {
    k0 = args.seg[d.k_seg];
    K = args.seg[d.k_seg + span] - (int)k0;
  }
  const int n = d.n, i0 = tm * LTM;
  if (i0 >= m) return false;
  const int flags = d.flags;
  // The output tiles of this workgroup: one, or with NMGP_LAT_COLPACK (a B-triangular problem whose column
  // tiles have k ranges of 1..T panels) a group of up to two column tiles whose panels add up to <= LW:
  // group 0 = {0}, g = 1..h = {g, T-g}, and for even T the middle tile alone (B_UPPER mirrored).  Wave w takes
  // panel w of the group's concatenated panel list, so no wave idles on a short-k tile.
  int jt[2] = {tn, -1};
  const bool pack = (flags & NMGP_LAT_COLPACK) != 0;
  if (pack) {
    const int Tn = (n + LTN - 1) / LTN, h = (Tn - 1) / 2;
    int a, b = -1;
    if (tn == 0) a = 0;
    else if (tn <= h) { a = tn; b = Tn - tn; }
    else a = Tn / 2;
    if (flags & NMGP_B_UPPER) {
      a = Tn - 1 - a;
      if (b >= 0) b = Tn - 1 - b;
    }
    jt[0] = a;
    jt[1] = b;
  }
  const bool blkA = d.kbA > 0 && d.kbA < K, blkB = d.kbB > 0 && d.kbB < K;
  const int kbA = blkA ? d.kbA : 0x40000000, kbB = blkB ? d.kbB : 0x40000000;
  int tkbeg[2], tkend[2], tnp[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    tkbeg[q] = 0;
    tkend[q] = 0;
    tnp[q] = 0;
    if (jt[q] < 0) continue;
    const int j0 = jt[q] * LTN;
    const bool above = j0 > i0 + LTM - 1;
    if (above && (flags & NMGP_OUT_LOWER)) {
      jt[q] = -1;                        // (never with COLPACK: the host packs only unmasked outputs)
      continue;
    }
    const bool zero_tile = above && (flags & NMGP_OUT_TRIL);
    int kbeg = 0, kend = K;
    if (d.k_seg < 0) {
      if ((flags & NMGP_A_LOWER) && !blkA) kend = min(kend, i0 + LTM);
      if ((flags & NMGP_A_UPPER) && !blkA) kbeg = max(kbeg, i0);
      if ((flags & NMGP_B_LOWER) && !blkB) kbeg = max(kbeg, j0);
      if ((flags & NMGP_B_UPPER) && !blkB) kend = min(kend, j0 + LTN);
    }
    kbeg = (kbeg / LKP) * LKP;
    if (zero_tile || K <= 0) kend = kbeg;
    if (ksplit > 1) {               // this workgroup's k chunk (whole panels)
      const int npan_all = kend > kbeg ? (kend - kbeg + LKP - 1) / LKP : 0;
      const int per = (npan_all + ksplit - 1) / ksplit;
      const int cb = kbeg + ks * per * LKP;
      kend = max(cb, min(kend, cb + per * LKP));
      kbeg = cb;
    }
    tkbeg[q] = kbeg;
    tkend[q] = kend;
    tnp[q] = kend > kbeg ? (kend - kbeg + LKP - 1) / LKP : 0;
  }
  if (jt[0] < 0 && jt[1] < 0) return false;
  J.prob = lo;
  J.tid = tm * d.tiles_n + tn;
  J.ks = ks;
  J.ksplit = ksplit;
  J.i0 = i0;
  J.m = m;
  J.K = K;
  J.flags = flags;
  J.r0 = r0;
  J.k0 = k0;
  J.pack = pack;
  J.blkA = blkA;
  J.blkB = blkB;
  J.first_tile = first_tile;
  J.kbA = kbA;
  J.kbB = kbB;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    J.jt[q] = jt[q];
    J.tnp[q] = tnp[q];
  }
  // this wave's tile (packed: the tile whose panel range holds panel w; otherwise tile 0, panels w, w+LW, ..)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int myq = (pack && w >= tnp[0]) ? 1 : 0;
  J.pfirst = pack ? (myq ? w - tnp[0] : w) : w;
  J.pstep = pack ? 0x40000000 : LW;
  J.npan = (pack && myq == 1 && jt[1] < 0) ? 0 : tnp[myq];
  J.j0 = jt[myq] < 0 ? 0 : jt[myq] * LTN;
  J.kbeg = tkbeg[myq];
  J.kend = tkend[myq];
  return true;
}

// the operands' buffer resources of a decoded tile (every value readfirstlane'd: provably uniform, so they stay in
// SGPRs)
template <typename T>
__device__ __forceinline__ void lat_rsrc(const LatJob& J, const nmgp_gemm_desc& d, __amdgpu_buffer_rsrc_t& rA,
                                         __amdgpu_buffer_rsrc_t& rB) {
  constexpr int64_t sz = sizeof(T);
  const int m = uniform32(J.m), K = uniform32(J.K);
  const int64_t r0 = uniform64(J.r0), k0 = uniform64(J.k0);
  const bool blkA = uniform32(J.blkA), blkB = uniform32(J.blkB);
  const int kbA = uniform32(J.kbA), kbB = uniform32(J.kbB);
  const int nkbA = blkA ? (K + kbA - 1) / kbA : 1, kinA = blkA ? kbA : K;
  const int nkbB = blkB ? (K + kbB - 1) / kbB : 1, kinB = blkB ? kbB : K;
  const char* baseA = (const char*)d.A + (r0 * d.sA_i + k0 * d.sA_k) * sz;
  const char* baseB = (const char*)d.B + (k0 * d.sB_k) * sz;
  const int64_t extA = ((int64_t)(m - 1) * d.sA_i + (int64_t)(kinA - 1) * d.sA_k + (int64_t)(nkbA - 1) * d.sA_kb + 1) * sz;
  const int64_t extB = ((int64_t)(kinB - 1) * d.sB_k + (int64_t)(d.n - 1) * d.sB_j + (int64_t)(nkbB - 1) * d.sB_kb + 1) * sz;
  rA = make_rsrc(baseA, extA);
  rB = make_rsrc(baseB, extB);
}

// this lane's operands of panel p (NV k values of two A rows and two B columns)
template <typename T, int LW, int LKP>
__device__ __forceinline__ void lat_load(const LatJob& J, const nmgp_gemm_desc& d, int p, __amdgpu_buffer_rsrc_t rA,
                                         __amdgpu_buffer_rsrc_t rB, T (&a)[2][LKP / 4], T (&b)[2][LKP / 4]) {
  constexpr int NV = LKP / 4;
  constexpr int64_t sz = sizeof(T);
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int kp = J.kbeg + p * LKP;
  const int ba = kp / J.kbA, bb = kp / J.kbB;        // k-block of the panel (panels never straddle one)
  const int kkA0 = kp - ba * (J.blkA ? J.kbA : 0), kkB0 = kp - bb * (J.blkB ? J.kbB : 0);   // block-local k
  const int ka = kkA0 + NV * g, kbl = kkB0 + NV * g;   // this lane's first k (block-local)
  const uint32_t stA = (uint32_t)(d.sA_k * sz), stB = (uint32_t)(d.sB_k * sz);
#pragma unroll
  for (int bi = 0; bi < 2; ++bi) {
    const int64_t row = J.i0 + 16 * bi + li;
    loadv<T, NV>(a[bi], rA, (uint32_t)((row * d.sA_i + (int64_t)ka * d.sA_k + (int64_t)ba * d.sA_kb) * sz), stA,
                 d.sA_k == 1);
  }
#pragma unroll
  for (int bj = 0; bj < 2; ++bj) {
    const int64_t col = J.j0 + 16 * bj + li;
    loadv<T, NV>(b[bj], rB, (uint32_t)(((int64_t)kbl * d.sB_k + col * d.sB_j + (int64_t)bb * d.sB_kb) * sz), stB,
                 d.sB_k == 1);
  }
}

// the first panel of a decoded tile (the one a persistent workgroup loads ahead)
template <typename T, int LW, int LKP>
__device__ __forceinline__ void lat_load_first(const LatJob& J, const nmgp_gemm_desc* __restrict__ descs,
                                               T (&a)[2][LKP / 4], T (&b)[2][LKP / 4]) {
  if (J.pfirst >= J.npan) return;
  const nmgp_gemm_desc& d = descs[uniform32(J.prob)];
  __amdgpu_buffer_rsrc_t rA, rB;
  lat_rsrc<T>(J, d, rA, rB);
  lat_load<T, LW, LKP>(J, d, J.pfirst, rA, rB, a, b);
}

// k scaling, element masks and the MFMAs of panel p
template <typename T, int LW, int LKP>
__device__ __forceinline__ void lat_mma(const LatJob& J, const nmgp_gemm_desc& d, int p, T (&a)[2][LKP / 4],
                                        T (&b)[2][LKP / 4], typename Mfma<T>::acc_t (&acc)[2][2]) {
  constexpr int NV = LKP / 4;
  const bool first_tile = J.first_tile;
  LAT_STAMP(2);
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int flags = J.flags;
  const int kp = J.kbeg + p * LKP;
  const int ba = kp / J.kbA, bb = kp / J.kbB;
  const int kkA0 = kp - ba * (J.blkA ? J.kbA : 0), kkB0 = kp - bb * (J.blkB ? J.kbB : 0);
  const int ka = kkA0 + NV * g, kbl = kkB0 + NV * g;
  if (flags & NMGP_KSCALE) {
    const GPtr<const T> ksc = (GPtr<const T>)d.kscale;
    const int kg = kp + NV * g;
#pragma unroll
    for (int s = 0; s < NV; ++s) {
      const T sc = ksc[J.k0 + min(kg + s, J.K - 1)];
      b[0][s] *= sc;
      b[1][s] *= sc;
    }
  }
  const bool aLo = flags & NMGP_A_LOWER, aUp = flags & NMGP_A_UPPER;
  const bool bLo = flags & NMGP_B_LOWER, bUp = flags & NMGP_B_UPPER;
  const int i0 = J.i0, j0 = J.j0, kend = J.kend;
  // element masks only on panels that need them (wave-uniform tests)
  const bool tail = kp + LKP > kend;
  const bool mA = tail || (aLo && kkA0 + LKP - 1 > i0) || (aUp && kkA0 < i0 + LTM - 1);
  // (the k tail is masked in both operands: memory past kend inside an operand's extent may hold
  // non-finite values, and 0 * inf would reach the sum)
  const bool mB = tail || (bLo && j0 + LTN - 1 > kkB0) || (bUp && kkB0 + LKP - 1 > j0);
  if (mA) {
#pragma unroll
    for (int bi = 0; bi < 2; ++bi) {
      const int gi = i0 + 16 * bi + li;
#pragma unroll
      for (int s = 0; s < NV; ++s) {
        const int kk = ka + s;
        const bool ok = (kp + NV * g + s < kend) && !(aLo && kk > gi) && !(aUp && kk < gi);
        a[bi][s] = keep_if(a[bi][s], ok);
      }
    }
  }
  if (mB) {
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) {
      const int gj = j0 + 16 * bj + li;
#pragma unroll
      for (int s = 0; s < NV; ++s) {
        const int kk = kbl + s;
        const bool ok = (kp + NV * g + s < kend) && !(bLo && gj > kk) && !(bUp && gj < kk);
        b[bj][s] = keep_if(b[bj][s], ok);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < NV; ++s) {
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q >> 1][q & 1] = Mfma<T>::mma(a[q >> 1][s], b[q & 1][s], acc[q >> 1][q & 1]);
  }
}

// the waves' partial tiles summed through LDS in wave order, split-K hand-off, epilogue and store
template <typename T, int LW, int LKP>
__device__ __forceinline__ void lat_finish(const LatArgs& args, const LatJob& J, const nmgp_gemm_desc& d,
                                           typename Mfma<T>::acc_t (&acc)[2][2], T* red) {
  const bool first_tile = J.first_tile;
  LAT_STAMP(3);
  const int t = threadIdx.x, lane = t & 63, li = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      red[w * (LTM * LTN) + (16 * (q >> 1) + Mfma<T>::row(lane, r)) * LTN + 16 * (q & 1) + li] = acc[q >> 1][q & 1][r];
  }
  lds_barrier();
  LAT_STAMP(4);
  constexpr int NE = (LTM * LTN) / (64 * LW);   // output values per thread and tile
  const bool pack = J.pack;
  const int ksplit = J.ksplit, i0 = J.i0, m = J.m, flags = J.flags;
  const int64_t r0 = J.r0;
  const int ntl = (J.jt[1] >= 0) ? 2 : 1;
  for (int qt = 0; qt < ntl; ++qt) {
    const int jtq = qt ? J.jt[1] : J.jt[0];      // (selects, not an indexed member: J stays in registers)
    if (jtq < 0) continue;
    // waves holding this tile's partials: all (unpacked) or the tile's panel range (packed)
    const int wb = pack ? (qt ? J.tnp[0] : 0) : 0;
    const int we = pack ? (qt ? J.tnp[0] + J.tnp[1] : J.tnp[0]) : LW;
    const int tj0 = jtq * LTN;
    T vals[NE];
#pragma unroll
    for (int q = 0; q < NE; ++q) {
      const int e = t + 64 * LW * q;
      T sum = we > wb ? red[wb * LTM * LTN + e] : (T)0;
      for (int v = wb + 1; v < we; ++v) sum += red[v * LTM * LTN + e];
      vals[q] = sum;
    }
    if (ksplit > 1) {
      // Deterministic split-K: every chunk publishes its partial tile write-through (sc1) and, once its
      // stores drained, bumps the tile's counter; the last arriver sums all partials in chunk order from
      // memory (sc1 loads bypass the stale L1) and runs the epilogue.  No waiting, so no co-residency
      // assumption; the last arriver re-arms the counter for the next launch.  (Never packed.)
      T* wsb = (T*)d.ws + (int64_t)J.tid * ksplit * (LTM * LTN);
      const __amdgpu_buffer_rsrc_t rws = make_rsrc(wsb, (int64_t)ksplit * (LTM * LTN) * (int64_t)sizeof(T));
#pragma unroll
      for (int q = 0; q < NE; ++q)
        bstore_sc1<T>(rws, (uint32_t)(((int64_t)J.ks * (LTM * LTN) + t + 64 * LW * q) * (int64_t)sizeof(T)), vals[q]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* s_last = (int*)red;          // the partial tiles in LDS are consumed (vals) -- reuse a word
      if (t == 0) {
        int32_t* ctr = d.counters + J.tid;
        const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == ksplit - 1;
        if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *s_last = last;
      }
      __syncthreads();
      const bool last = *s_last != 0;
      if (!last) return;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keeps the loads below the counter
#pragma unroll
      for (int q = 0; q < NE; ++q) {
        const int e = t + 64 * LW * q;
        T sum = 0;
        for (int c = 0; c < ksplit; ++c)
          sum += bload_sc1<T>(rws, (uint32_t)(((int64_t)c * (LTM * LTN) + e) * (int64_t)sizeof(T)));
        vals[q] = sum;
      }
    }
    LAT_STAMP(5);
    const GPtr<T> C = (GPtr<T>)d.C;
    const GPtr<const T> E = (GPtr<const T>)d.epi_E;
    const GPtr<const T> rsp = (GPtr<const T>)d.epi_rs;
    const T alpha = (T)d.alpha, beta = (T)d.beta, gamma = (T)d.gamma, dadd = (T)d.diag_add;
#pragma unroll
    for (int q = 0; q < NE; ++q) {
      const int e = t + 64 * LW * q;
      const int gi = i0 + (e / LTN), gj = tj0 + (e % LTN);
      const T sum = vals[q];
      if (gi >= m || gj >= d.n) continue;
      const bool upper = gj > gi;
      if (upper && (flags & NMGP_OUT_LOWER)) continue;
      const int64_t ci = (r0 + gi) * d.sC_i + (int64_t)gj * d.sC_j;
      T val;
      if (upper && (flags & NMGP_OUT_TRIL)) {
        val = 0;
      } else {
        val = alpha * sum;
        if (beta != (T)0) val += beta * C[ci];
        if (flags & NMGP_EPI) {
          T ev = 0;
          if (!((flags & NMGP_EPI_E_LOWER) && upper)) ev = E[(r0 + gi) * d.sE_i + (int64_t)gj * d.sE_j];
          T rs = rsp ? rsp[r0 + gi] : (T)1;
          if (flags & NMGP_EPI_RS_NEG) rs = -rs;
          val += gamma * rs * ev;
        }
        if ((flags & NMGP_DIAG_ADD) && gi == gj) val += dadd;
      }
      C[ci] = val;
    }
  }
  LAT_STAMP(6);
}

// a decoded tile whose first panel (p = J.pfirst) is in a / b: its MFMAs, the wave's further panels, the finish
template <typename T, int LW, int LKP>
__device__ __forceinline__ void lat_run(const LatArgs& args, const nmgp_gemm_desc* __restrict__ descs,
                                        const LatJob& J, T (&a)[2][LKP / 4], T (&b)[2][LKP / 4], T* red) {
  const nmgp_gemm_desc& d = descs[uniform32(J.prob)];
  using acc_t = typename Mfma<T>::acc_t;
  acc_t acc[2][2];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q >> 1][q & 1] = acc_t{0, 0, 0, 0};
  if (J.pfirst < J.npan) {
    lat_mma<T, LW, LKP>(J, d, J.pfirst, a, b, acc);
    if (J.pfirst + J.pstep < J.npan) {      // further rounds (loaded in place)
      __amdgpu_buffer_rsrc_t rA, rB;
      lat_rsrc<T>(J, d, rA, rB);
      for (int p = J.pfirst + J.pstep; p < J.npan; p += J.pstep) {
        lat_load<T, LW, LKP>(J, d, p, rA, rB, a, b);
        lat_mma<T, LW, LKP>(J, d, p, a, b, acc);
      }
    }
  }
  lat_finish<T, LW, LKP>(args, J, d, acc, red);
}

template <typename T, int LW, int LKP, int OCC>
__global__ __launch_bounds__(64 * LW, OCC) void gemm_lat_kernel(LatArgs args,
                                                                             const nmgp_gemm_desc* __restrict__ descs,
                                                                             const int32_t* __restrict__ dyn) {
  __shared__ T red[LW * LTM * LTN];
  const int total = __builtin_amdgcn_readfirstlane(dyn ? dyn[args.nprob] : args.total);
  const int per = (total + 7) >> 3;   // tiles per XCD chunk
  for (int b = blockIdx.x; b < 8 * per; b += gridDim.x) {
    const int tile = (b & 7) * per + (b >> 3);
    LatJob J;
    if (tile < total && lat_decode<T, LW, LKP>(args, descs, dyn, tile, b == (int)blockIdx.x, J)) {
      T a[2][LKP / 4], bv[2][LKP / 4];
      lat_load_first<T, LW, LKP>(J, descs, a, bv);
      lat_run<T, LW, LKP>(args, descs, J, a, bv, red);
    }
    __syncthreads();
  }
}

// the next tile with output in this workgroup's sequence b, b + gridDim.x, ... (b advanced past it)
template <typename T, int LW, int LKP>
__device__ __forceinline__ bool lat_next(const LatArgs& args, const nmgp_gemm_desc* __restrict__ descs,
                                         const int32_t* __restrict__ dyn, int total, int per, int lim, int& b,
                                         LatJob& J) {
  for (; b < lim; b += gridDim.x) {
    const int tile = (b & 7) * per + (b >> 3);
    if (tile < total && lat_decode<T, LW, LKP>(args, descs, dyn, tile, b == (int)blockIdx.x, J)) {
      b += gridDim.x;
      return true;
    }
  }
  return false;
}

// Persistent form for launches with more tiles than one round of workgroups (round 6): one
// workgroup per CU walks its tiles (the same XCD-chunked order as gemm_lat_kernel) with two tiles in flight -- the
// first panel of the next tile is loaded before the current tile's MFMAs and LDS reduction, so its global round
// trip hides under them.  Each tile is computed exactly as gemm_lat_kernel computes it (same panels per wave, same
// reduction order): results are bit-identical to the non-persistent launch.
template <typename T, int LW, int LKP>
__global__ __launch_bounds__(64 * LW, 1) void gemm_lat_pipe_kernel(LatArgs args,
                                                                   const nmgp_gemm_desc* __restrict__ descs,
                                                                   const int32_t* __restrict__ dyn) {
  __shared__ T red[LW * LTM * LTN];
  constexpr int NV = LKP / 4;
  const int total = __builtin_amdgcn_readfirstlane(dyn ? dyn[args.nprob] : args.total);
  const int per = (total + 7) >> 3;
  const int lim = 8 * per;
  int b = blockIdx.x;
  LatJob J0, J1;
  T a0[2][NV], b0[2][NV], a1[2][NV], b1[2][NV];
  bool h0 = lat_next<T, LW, LKP>(args, descs, dyn, total, per, lim, b, J0);
  if (h0) lat_load_first<T, LW, LKP>(J0, descs, a0, b0);
  while (h0) {
    const bool h1 = lat_next<T, LW, LKP>(args, descs, dyn, total, per, lim, b, J1);
    if (h1) lat_load_first<T, LW, LKP>(J1, descs, a1, b1);
    lat_run<T, LW, LKP>(args, descs, J0, a0, b0, red);
    __syncthreads();
    if (!h1) break;
    h0 = lat_next<T, LW, LKP>(args, descs, dyn, total, per, lim, b, J0);
    if (h0) lat_load_first<T, LW, LKP>(J0, descs, a0, b0);
    lat_run<T, LW, LKP>(args, descs, J1, a1, b1, red);
    __syncthreads();
  }
}

// Tile plan of a grouped launch for this minibatch (as gemm.hip's plan kernel, 32-row tiles).
__global__ __launch_bounds__(256) void lat_plan_kernel(const nmgp_gemm_desc* __restrict__ descs, int nprob,
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
        tm = min(tm, max(0, (m + LTM - 1) / LTM));
      }
      v = tm * d.tiles_n * (d.ksplit > 1 ? d.ksplit : 1);
    }
    buf[t] = v;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
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

template <typename T>
int launch_lat(const nmgp_gemm_desc* d_desc, int nprob, int total_tiles, const int32_t* d_seg, int32_t* d_plan,
               int grid, hipStream_t s, bool planned = false, bool pipe = false) {
  if (d_desc == nullptr) return -1;
  if (nprob <= 0) return -2;
  if (total_tiles < 0) return -3;
  if (total_tiles == 0) return NMGP_OK;
  LatArgs a;
  a.descs = d_desc;
  a.nprob = nprob;
  a.total = total_tiles;
  a.seg = d_seg;
  a.dyn_start = nullptr;
  int wgs = ((total_tiles + 7) / 8) * 8;
  if (d_plan != nullptr) {
    if (!planned) {
      hipLaunchKernelGGL(lat_plan_kernel, dim3(1), dim3(256), 0, s, d_desc, nprob, d_seg, d_plan);
      NMGP_CHECK_LAUNCH();
    }
    a.dyn_start = d_plan;
    if (grid > 0) wgs = min(wgs, ((grid + 7) / 8) * 8);   // a multiple of 8 keeps each workgroup on one XCD chunk
  }
  if (pipe) {
    // persistent: one workgroup per CU (the XCD chunking needs a multiple of 8), never more than the tiles
    static int n_cu = 0;
    if (n_cu == 0) {
      int dev = 0, v = 0;
      if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                  hipSuccess && v > 0)
        n_cu = v;
      else
        n_cu = 256;
    }
    wgs = min(wgs, max(8, (n_cu / 8) * 8));
    hipLaunchKernelGGL((gemm_lat_pipe_kernel<T, 8, 32>), dim3(wgs), dim3(512), 0, s, a, d_desc, a.dyn_start);
    NMGP_CHECK_LAUNCH();
    return NMGP_OK;
  }
  // 8 waves x 32-wide panels with registers capped at 128 so two workgroups share a CU (round 2: PM2.5 step +1%
  // over one workgroup per CU).  hip_ops.GemmGroup sizes split-K for 8 waves x 32.
  hipLaunchKernelGGL((gemm_lat_kernel<T, 8, 32, 4>), dim3(wgs), dim3(512), 0, s, a, d_desc, a.dyn_start);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

}  // namespace
}  // namespace nmgp

extern "C" {
int nmgp_gemm_grouped_lat_f64(const nmgp_gemm_desc* d, int np, int tt, const int32_t* seg, int32_t* plan, int grid,
                              hipStream_t s) {
  return nmgp::launch_lat<double>(d, np, tt, seg, plan, grid, s);
}
int nmgp_gemm_grouped_lat_f32(const nmgp_gemm_desc* d, int np, int tt, const int32_t* seg, int32_t* plan, int grid,
                              hipStream_t s) {
  return nmgp::launch_lat<float>(d, np, tt, seg, plan, grid, s);
}
int nmgp_gemm_plan_lat(const nmgp_gemm_desc* d, int np, const int32_t* seg, int32_t* plan, hipStream_t s) {
  if (!d || !plan) return -1;
  if (np <= 0) return -2;
  hipLaunchKernelGGL(nmgp::lat_plan_kernel, dim3(1), dim3(256), 0, s, d, np, seg, plan);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
int nmgp_gemm_grouped_lat_planned_f64(const nmgp_gemm_desc* d, int np, int tt, const int32_t* seg, int32_t* plan,
                                      int grid, hipStream_t s) {
  if (!plan) return -5;
  return nmgp::launch_lat<double>(d, np, tt, seg, plan, grid, s, true);
}
int nmgp_gemm_grouped_lat_planned_f32(const nmgp_gemm_desc* d, int np, int tt, const int32_t* seg, int32_t* plan,
                                      int grid, hipStream_t s) {
  if (!plan) return -5;
  return nmgp::launch_lat<float>(d, np, tt, seg, plan, grid, s, true);
}
// persistent two-tiles-in-flight launches (same arguments; planned != 0: the device tile plan is already computed)
int nmgp_gemm_grouped_lat_pipe_f64(const nmgp_gemm_desc* d, int np, int tt, const int32_t* seg, int32_t* plan,
                                   int planned, hipStream_t s) {
  if (planned && !plan) return -5;
  return nmgp::launch_lat<double>(d, np, tt, seg, plan, 0, s, planned != 0, true);
}
int nmgp_gemm_grouped_lat_pipe_f32(const nmgp_gemm_desc* d, int np, int tt, const int32_t* seg, int32_t* plan,
                                   int planned, hipStream_t s) {
  if (planned && !plan) return -5;
  return nmgp::launch_lat<float>(d, np, tt, seg, plan, 0, s, planned != 0, true);
}
}
