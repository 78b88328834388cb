// Large-tile f32 GEMM / SYRK for the recursive Cholesky of big matrices (HCP M=512, ECoG M=1024,
// the M=4096 stress case): the trailing update A22 -= L21 L21^T and the three inverse / panel
// products of chol_inv_rec (chol.hip).  The step GEMMs of the DSVI engine stay on the grouped
// 64x64 kernel (gemm.hip); this one is for few, large, dense problems.
//
//   * 128x128x32 block tile, 256 threads = 4 waves in 2x2, each wave 64x64 as 2x2
//     v_mfma_f32_32x32x2_f32 accumulators (exact f32 products, 64 FLOP/clk/SIMD: the fp32 peak).
//   * k is permuted inside a k-tile: at k-step s lane l feeds k = 16*(l>>5) + s instead of the
//     instruction's 2s + (l>>5), for both operands -- a sum over k does not care -- so each lane's
//     16 operand values of a k-tile are contiguous in LDS and arrive with four ds_read_b128.
//   * LDS images [row][k] with a 36-float pitch (conflict-free b128 reads), two stages; the next
//     k-tile's 16-byte global (buffer) loads are in flight while the current one's 64 MFMAs issue.
//   * Triangular operands restrict each tile's k range (A_LOWER / B_UPPER / B_LOWER) and only the
//     k-tiles that straddle the diagonal, and a k tail, pay for element masks.  OUT_LOWER launches
//     only the lower tiles (SYRK).
//   * Deterministic split-K when the grid would not fill the chip: partials are published
//     write-through (sc1) into caller workspace, the last-arriving chunk of a tile sums them in
//     chunk order (its own from registers) and applies the epilogue.
//   * blockIdx -> tile mapping is XCD-aware: single problems give each of the 8 XCDs a contiguous run of
//     tiles (shared A rows stay in one L2); batched problems rotate the tile index per problem so no XCD
//     gets the same (for triangular operands: the longest-k) tile row of every problem.
#include "common.hpp"
#include "potrf_parts.hpp"   // ps_* row-panel helpers (shared with chol.hip's fused leaf + step kernel)

namespace nmgp {

#ifdef NMGP_BIG_TRACE  // per-workgroup wall-clock phases (tools/big_trace.hip only)
__device__ unsigned long long* g_big_trace;
#define BIG_STAMP(i) \
  if (threadIdx.x == 0) g_big_trace[(blockIdx.x + gridDim.x * blockIdx.y) * 8 + (i)] = wall_clock64()
#else
#define BIG_STAMP(i)
#endif

constexpr int BBM = 128, BBN = 128, BBK = 32, BP = 36;   // tile and LDS pitch (floats, 144 B rows)
constexpr int BSTAGE = (BBM + BBN) * BP;                  // floats per LDS stage
constexpr int BSLOT = BBM * BBN;                          // floats per split-K partial tile
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4g __attribute__((ext_vector_type(4)));

struct BigGemmArgs {
  const float* A; const float* B; float* C;
  int64_t lda, ldb, sCi, sCj;
  int64_t sAb, sBb, sCb;
  int m, n, k, flags;
  int b_kcontig;            // 1: op(B)(k,j) = B[j*ldb + k]; 0: op(B)(k,j) = B[k*ldb + j]
  int a_kcontig;            // 1: op(A)(i,k) = A[i*lda + k]; 0: op(A)(i,k) = A[k*lda + i]
  float alpha, beta;
  int tiles_m, tiles_n, tiles;   // tiles per batch item (lower tiles only with OUT_LOWER)
  const int64_t* offA;      // per-batch element offsets (device arrays) instead of bat * sAb / sBb / sCb
  const int64_t* offB;
  const int64_t* offC;
  float diag_add;           // added to C(i, i) after the update (Sigma = L L^T + jitter I)
  // NMGP_EPI: C += gamma * rs[i] * E(i, j) (E(i, j) = 0 above the diagonal with NMGP_EPI_E_LOWER)
  const float* E; const int64_t* offE; int64_t sEi, sEj;
  const float* RS; const int64_t* offRS;
  float gamma;
  // NMGP_EPI with D: the raw product acc(i, j) is also stored to D(i, j) = D[offD[b] + i * sDi + j] (the KL L-bar's
  // solve form needs G21 = X22^T W21 itself besides the gradient rows it is added to)
  float* D; const int64_t* offD; int64_t sDi;
  // per-problem k range from the minibatch segment table (offsets variants): problem b runs
  // k in [seg[kseg[b]], seg[kseg[b] + kspan[b]]) -- rows of the outputs it sums over
  const int32_t* seg; const int32_t* kseg; const int32_t* kspan;
  // per-problem row range (offsets variants): problem b's rows are [seg[rseg[b]], seg[rseg[b] + rspan[b]]) of A, C
  // (and E, RS) -- the rows of the outputs it serves; m is their upper bound (tiles past a problem's rows are skipped)
  const int32_t* rseg; const int32_t* rspan;
  int koff;
  int ksplit;
  int streamk;              // 1: stream-K partition over a persistent grid (batch 1, uniform k)
  int persist;              // batched, one pass per tile: workgroup x runs work items x, x + G, ... of the
                            // (tile, problem) space, problem-major (item w: problem w % batch, tile w / batch)
  int batch, total;         // (persist) problems and work items
  float* ws; int32_t* counters;
};

template <int AUX = 0>
__device__ inline float4 ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
}

// Lower-triangle tile index -> (tile row, tile column), row-major over the lower triangle.  A tall OUT_LOWER
// output (m > n: the blocked potrf's next-panel updates) continues below the triangle with full tile rows.
__device__ inline void tile_coords(const BigGemmArgs& g, int tile, int& tm, int& tn) {
  if (g.flags & NMGP_OUT_LOWER) {
    const int T = g.tiles_n, tri = T * (T + 1) / 2;
    if (tile >= tri) {
      tm = T + (tile - tri) / T;
      tn = (tile - tri) - (tm - T) * T;
      return;
    }
    tm = (int)((sqrtf(8.0f * (float)tile + 1.0f) - 1.0f) * 0.5f);
    while ((tm + 1) * (tm + 2) / 2 <= tile) ++tm;
    while (tm * (tm + 1) / 2 > tile) --tm;
    tn = tile - tm * (tm + 1) / 2;
  } else {
    tm = tile / g.tiles_n;
    tn = tile - tm * g.tiles_n;
  }
}

// Structurally nonzero k range of a tile (triangular operands), in whole k-tiles from kbeg.
__device__ inline void tile_krange(const BigGemmArgs& g, int K, int i0, int j0, int& kbeg, int& kend) {
  kbeg = 0;
  kend = K;
  if (g.flags & NMGP_A_LOWER) kend = min(kend, i0 + BBM);
  if (g.flags & NMGP_B_UPPER) kend = min(kend, j0 + BBN);
  if (g.flags & NMGP_B_LOWER) kbeg = max(kbeg, j0);
  if (g.flags & NMGP_A_UPPER) kbeg = max(kbeg, i0);
  kbeg = (kbeg / BBK) * BBK;
}

// acc += A[i0:i0+128, kt0:kt1] op(B)[kt0:kt1, j0:j0+128] (kend bounds the masks).  AK / BK: operand
// layouts (k-contiguous or not) as compile-time variants, so each kernel carries one loader per operand.
// K / koff: the problem's k extent and first k (per-problem segment variants; g.k and g.koff otherwise) -- kept out of
// the argument struct so the kernel never writes it (a written copy lives in scratch and every operand address
// derived from it becomes a per-lane value).
// NB: 32-column accumulator blocks per wave -- 2: 4 waves (256 threads) of 64 x 64; 1: 8 waves (512 threads) of
// 64 x 32, the tile's columns split over 4 wave columns (two workgroups per CU then hold 4 waves per SIMD: a CU
// whose other workgroup is in its prologue / epilogue still has two waves per SIMD issuing MFMAs).
template <bool AK, bool BK, int MODE, int AUX = 0, int NB = 2>
__device__ __forceinline__ void big_mainloop(const BigGemmArgs& g, int K, int koff, int M, int64_t roff, float* big_smem,
                                             int64_t bat, int i0, int j0, int kend, int kt0, int kt1,
                                             f32x16 (&acc)[2][NB]) {
  constexpr int NT = 512 / NB;                 // threads
  constexpr int NQ = 1024 / NT;                // 16-byte operand loads per thread and operand (4 or 2)
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  // wave grid 2 x (4 / NB): rows 64 wr8, columns 32 NB wc8
  const int wr8 = NB == 1 ? (w >> 2) : (w >> 1), wc8 = NB == 1 ? (w & 3) : (w & 1);
  const int fl = g.flags;
  const bool aLo = fl & NMGP_A_LOWER, aUp = fl & NMGP_A_UPPER, bUp = fl & NMGP_B_UPPER, bLo = fl & NMGP_B_LOWER;
  const float* Ab = g.A + (MODE ? uniform64(g.offA[bat]) : bat * g.sAb) + (AK ? (int64_t)koff : (int64_t)koff * g.lda) +
                    (AK ? roff * g.lda : roff);
  const float* Bb = g.B + (MODE ? uniform64(g.offB[bat]) : bat * g.sBb) + (BK ? (int64_t)koff : (int64_t)koff * g.ldb);
  const __amdgpu_buffer_rsrc_t rA =
      AK ? make_rsrc(Ab, ((int64_t)(M - 1) * g.lda + K) * 4)
                  : make_rsrc(Ab, ((int64_t)(K - 1) * g.lda + M) * 4);
  const __amdgpu_buffer_rsrc_t rB =
      BK ? make_rsrc(Bb, ((int64_t)(g.n - 1) * g.ldb + K) * 4)
                  : make_rsrc(Bb, ((int64_t)(K - 1) * g.ldb + g.n) * 4);

  // loader maps: k-contiguous A / B: row t>>3 (+ NT/8 q), k 4*(t&7)
  const int lr = t >> 3, lk = (t & 7) * 4;
  // i-contiguous A / j-contiguous B: k = 4 (t & 7) + q, i or j = 4 (t >> 3) + e: each k row is read as 128
  // contiguous bytes by 8 lanes, and the thread's 4 x 4 block (k rows q, columns e) is transposed in registers
  // so the LDS image [i][k] is written with one 16-byte store per i -- the k-contiguous operands' store pattern
  // (16 single-float transposed stores per operand before: a both-transposed product ran at half the MFMA rate)
  const int jr = t & 7, jc = (t >> 3) * 4;
  // k row of load q: 4 jr + q (LDS slot 4 jr + q holds k 4 jr + q, the k-contiguous operands' order); with BOTH
  // operands k-strided the slots may hold any common permutation of k, and load q takes k = 8 q + jr instead, so
  // one wave instruction covers 8 consecutive k rows (4 KB apart) rather than rows 16 KB apart
  constexpr bool KPERM = !AK && !BK;
  // 8 waves: two k rows per thread, k = 2 (t >> 5) + q, i or j = 4 (t & 31) + e -- a wave instruction reads two
  // 512-byte k-row segments; the 2 x 4 block goes to LDS as four 8-byte stores (slot = k: the k-contiguous order)
  const int ic8 = (t & 31) * 4, kg8 = (t >> 5) * 2;
  auto krow = [&](int q) { return NB == 1 ? kg8 + q : (KPERM ? 8 * q + jr : 4 * jr + q); };
  const int jcx = NB == 1 ? ic8 : jc;
  float4 ra[NQ], rb[NQ];

  auto load = [&](int kt) {
    if constexpr (AK) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int64_t row = i0 + lr + (NT / 8) * q;
        ra[q] = ld4<AUX>(rA, (uint32_t)((row * g.lda + kt + lk) * 4));
      }
    } else {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int64_t kr = kt + krow(q);
        ra[q] = ld4<AUX>(rA, (uint32_t)((kr * g.lda + i0 + jcx) * 4));
      }
    }
    if constexpr (BK) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int64_t row = j0 + lr + (NT / 8) * q;
        rb[q] = ld4<AUX>(rB, (uint32_t)((row * g.ldb + kt + lk) * 4));
      }
    } else {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int64_t kr = kt + krow(q);
        rb[q] = ld4<AUX>(rB, (uint32_t)((kr * g.ldb + j0 + jcx) * 4));
      }
    }
  };
  auto store_lds = [&](float* st, int kt) {
    // element masks (applied here, after the current k-tile's MFMAs: masking in load() made the
    // compiler wait for the global loads before them) only on k-tiles that straddle a triangle's diagonal or the k tail
    const bool need = (kt + BBK > kend) || (aLo && kt + BBK - 1 > i0) || (bUp && kt + BBK - 1 > j0) ||
                      (bLo && kt < j0 + BBN - 1) || (aUp && kt < i0 + BBM - 1);
    if (need) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        float* a = (float*)&ra[q];
        if constexpr (AK) {
          const int i = i0 + lr + (NT / 8) * q;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int kk = kt + lk + e;
            a[e] = keep_if(a[e], kk < kend && (!aLo || kk <= i) && (!aUp || kk >= i));
          }
        } else {
          const int kk = kt + krow(q);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int i = i0 + jcx + e;
            a[e] = keep_if(a[e], kk < kend && (!aLo || kk <= i) && (!aUp || kk >= i));
          }
        }
        float* b = (float*)&rb[q];
        if constexpr (BK) {
          const int j = j0 + lr + (NT / 8) * q;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int kk = kt + lk + e;
            b[e] = keep_if(b[e], kk < kend && (!bUp || kk <= j) && (!bLo || kk >= j));
          }
        } else {
          const int kk = kt + krow(q);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int j = j0 + jcx + e;
            b[e] = keep_if(b[e], kk < kend && (!bUp || kk <= j) && (!bLo || kk >= j));
          }
        }
      }
    }
    float* As = st;
    float* Bs = st + BBM * BP;
    if constexpr (AK) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) *(float4*)&As[(lr + (NT / 8) * q) * BP + lk] = ra[q];
    } else if constexpr (NB == 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) *(float2*)&As[(ic8 + e) * BP + kg8] = make_float2(ra[0][e], ra[1][e]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        *(float4*)&As[(jc + e) * BP + 4 * jr] = make_float4(ra[0][e], ra[1][e], ra[2][e], ra[3][e]);
    }
    if constexpr (BK) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) *(float4*)&Bs[(lr + (NT / 8) * q) * BP + lk] = rb[q];
    } else if constexpr (NB == 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) *(float2*)&Bs[(ic8 + e) * BP + kg8] = make_float2(rb[0][e], rb[1][e]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        *(float4*)&Bs[(jc + e) * BP + 4 * jr] = make_float4(rb[0][e], rb[1][e], rb[2][e], rb[3][e]);
    }
  };

  if (kt0 < kt1) {
    load(kt0);
    store_lds(big_smem, kt0);
    __syncthreads();
    BIG_STAMP(1);
    int st = 0;
    const int ko = 16 * (lane >> 5), rl = lane & 31;
    for (int kt = kt0; kt < kt1; kt += BBK) {
      const bool more = kt + BBK < kt1;
      if (more) load(kt + BBK);
      const float* As = big_smem + st * BSTAGE;
      const float* Bs = As + BBM * BP;
      float4 fa[2][4], fb[NB][4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int h = 0; h < 2; ++h) fa[h][c] = *(const float4*)&As[(64 * wr8 + 32 * h + rl) * BP + ko + 4 * c];
#pragma unroll
        for (int h = 0; h < NB; ++h)
          fb[h][c] = *(const float4*)&Bs[(32 * NB * wc8 + 32 * h + rl) * BP + ko + 4 * c];
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float av = ((const float*)&fa[h][s >> 2])[s & 3];
#pragma unroll
          for (int b = 0; b < NB; ++b)
            acc[h][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, ((const float*)&fb[b][s >> 2])[s & 3], acc[h][b], 0,
                                                             0, 0);
        }
      }
      if (more) store_lds(big_smem + (st ^ 1) * BSTAGE, kt + BBK);
      lds_barrier();
      st ^= 1;
    }
  }
}

// Publish this workgroup's partial tile (slot `mine`) write-through, count arrivals on `ctr`;
// the last of the `S` contributors sums all partials in contributor order (its own from
// registers) into acc and returns true.  slot_of(c) gives contributor c's slot.
template <int NB = 2, typename SlotOf>
__device__ __forceinline__ bool big_combine(const BigGemmArgs& g, int me, int S, int32_t* ctr, SlotOf slot_of,
                                            f32x16 (&acc)[2][NB]) {
  __shared__ int s_last;
  const int t = threadIdx.x;
  constexpr int PT = 32 * NB;                // partial values per thread (a tile's 16384 over the workgroup)
  {
    const __amdgpu_buffer_rsrc_t rws = make_rsrc(g.ws + uniform64(slot_of(me)) * BSLOT, (int64_t)BSLOT * 4);
    const uint32_t off = (uint32_t)(t * PT * 4);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          u32x4g v;
          v[0] = __float_as_uint(acc[a][b][4 * q + 0]);
          v[1] = __float_as_uint(acc[a][b][4 * q + 1]);
          v[2] = __float_as_uint(acc[a][b][4 * q + 2]);
          v[3] = __float_as_uint(acc[a][b][4 * q + 3]);
          __builtin_amdgcn_raw_buffer_store_b128(v, rws, off + ((a * NB + b) * 4 + q) * 16, 0, 16 /* sc1 */);
        }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (old == S - 1);
    if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last;
  }
  __syncthreads();
  const bool last = s_last;
  __syncthreads();   // s_last is reused by the next tile of a stream-K workgroup
  if (!last) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t off = (uint32_t)(t * PT * 4);
  if (S <= 4) {
    // per half-tile (acc[a][*]) all S partials -- this workgroup's own as stored above -- are loaded at once and
    // then summed in contributor order: two memory round trips instead of S - 1 (the same sums, bit for bit)
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      u32x4g v[4][4 * NB];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c >= S) continue;
        const __amdgpu_buffer_rsrc_t rws = make_rsrc(g.ws + uniform64(slot_of(c)) * BSLOT, (int64_t)BSLOT * 4);
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            v[c][b * 4 + q] = __builtin_amdgcn_raw_buffer_load_b128(rws, off + ((a * NB + b) * 4 + q) * 16, 0, 16);
      }
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        f32x16 sum;
#pragma unroll
        for (int r = 0; r < 16; ++r) sum[r] = 0.0f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (c >= S) continue;
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) sum[4 * q + e] += __uint_as_float(v[c][b * 4 + q][e]);
        }
        acc[a][b] = sum;
      }
    }
    return true;
  }
  f32x16 sum[2][NB];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) sum[a][b][r] = 0.0f;
  for (int c = 0; c < S; ++c) {
    if (c == me) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b) sum[a][b] += acc[a][b];
      continue;
    }
    const __amdgpu_buffer_rsrc_t rws = make_rsrc(g.ws + uniform64(slot_of(c)) * BSLOT, (int64_t)BSLOT * 4);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const u32x4g v = __builtin_amdgcn_raw_buffer_load_b128(rws, off + ((a * NB + b) * 4 + q) * 16, 0, 16);
#pragma unroll
          for (int e = 0; e < 4; ++e) sum[a][b][4 * q + e] += __uint_as_float(v[e]);
        }
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = sum[a][b];
  return true;
}

// One half tile (acc[A][*], 64 x 128) of the epilogue: C and the epilogue operand gamma rs(i) E(i, j) are read
// before the half's stores, as branch-free buffer loads (an element outside the stored part reads 0 through an
// out-of-range offset; the host checks that every problem's C and E span < 2 GiB).  With per-element guards each
// load sat in its own branch and was waited on before the next, and E, read in the store loop, waited on every
// store before it (64 dependent round trips per tile in the KL L-bar product, the ECoG step's longest launch).
// E must not alias C.  A is a template parameter so every accumulator index is a constant.
template <int MODE, int A, int NB = 2>
__device__ __forceinline__ void big_epi_half(const BigGemmArgs& g, float* Cb, float* Db, __amdgpu_buffer_rsrc_t rCb,
                                             __amdgpu_buffer_rsrc_t rEb, __amdgpu_buffer_rsrc_t rRS, int M, int i0,
                                             int j0, const f32x16 (&acc)[2][NB]) {
  constexpr bool EPI = MODE == 2;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = NB == 1 ? (w >> 2) : (w >> 1), wc = NB == 1 ? (w & 3) : (w & 1);
  const bool lower = g.flags & NMGP_OUT_LOWER;
  const bool tril = MODE && (g.flags & NMGP_OUT_TRIL);
  const bool eLo = g.flags & NMGP_EPI_E_LOWER;
  const bool ldc = g.beta != 0.0f;
  const int ib = i0 + 64 * wr + 32 * A + 4 * (lane >> 5);
  f32x16 cv[2], ev[2];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int j = j0 + 32 * NB * wc + 32 * b + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = ib + (r & 3) + 8 * (r >> 2);
      // (elements that OUT_TRIL zeroes are not read: a third of C's traffic in the batched L-bar forms)
      const bool ok = i < M && j < g.n && (!lower || j <= i) && !(tril && j > i);
      cv[b][r] = ldc ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                           rCb, ok ? (uint32_t)(((int64_t)i * g.sCi + (int64_t)j * g.sCj) * 4) : 0x80000000u, 0, 0))
                     : 0.0f;
      if constexpr (EPI) {
        const bool oke = ok && !(eLo && j > i);
        const float e = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
            rEb, oke ? (uint32_t)(((int64_t)i * g.sEi + (int64_t)j * g.sEj) * 4) : 0x80000000u, 0, 0));
        const float rv = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
            rRS, i < M ? (uint32_t)(i * 4) : 0x80000000u, 0, 0));
        ev[b][r] = g.gamma * rv * e;
      } else {
        ev[b][r] = 0.0f;
      }
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int j = j0 + 32 * NB * wc + 32 * b + (lane & 31);
    f32x16 v = acc[A][b] * g.alpha;
    if (ldc) v += g.beta * cv[b];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = ib + (r & 3) + 8 * (r >> 2);
      if (i < M && j < g.n && (!lower || j <= i)) {
        float x = v[r];
        if constexpr (MODE == 1) {
          if (i == j) x += g.diag_add;
        }
        if constexpr (EPI) {
          if (!(eLo && j > i)) x += ev[b][r];
        }
        if (tril && j > i) x = 0.0f;
        Cb[(int64_t)i * g.sCi + (int64_t)j * g.sCj] = x;
        if constexpr (EPI) {
          if (Db != nullptr) Db[(int64_t)i * g.sDi + j] = acc[A][b][r];
        }
      }
    }
  }
}

// C = alpha * acc + beta * C (+ diag_add, + the KL epilogue) on the stored part of the tile.
template <int MODE, int NB = 2>
__device__ __forceinline__ void big_epilogue(const BigGemmArgs& g, float* Cb, float* Db, const float* Eb,
                                             const float* rs, int M, int i0, int j0, f32x16 (&acc)[2][NB]) {
  constexpr bool EPI = MODE == 2;
  const __amdgpu_buffer_rsrc_t rCb = make_rsrc(Cb, ((int64_t)(M - 1) * g.sCi + (int64_t)(g.n - 1) * g.sCj + 1) * 4);
  const __amdgpu_buffer_rsrc_t rEb =
      make_rsrc(EPI ? Eb : Cb, EPI ? ((int64_t)(M - 1) * g.sEi + (int64_t)(g.n - 1) * g.sEj + 1) * 4 : 0);
  const __amdgpu_buffer_rsrc_t rRS = make_rsrc(EPI ? rs : Cb, EPI ? (int64_t)M * 4 : 0);
  big_epi_half<MODE, 0, NB>(g, Cb, Db, rCb, rEb, rRS, M, i0, j0, acc);
  big_epi_half<MODE, 1, NB>(g, Cb, Db, rCb, rEb, rRS, M, i0, j0, acc);
}

// Row-vector epilogue through LDS (row-contiguous C, and E, 16-byte aligned): the accumulators (each lane holds 16
// values of ONE column) go to a 128 x 128 LDS image, then every thread owns 16 four-column row chunks -- a wave
// stores two 512-byte row segments per instruction (global_store_dwordx4) instead of 64 single floats per thread,
// and reads C / E the same way, all 16 chunks' loads before the first store.  The per-workgroup phase trace of the
// batched ECoG products (tools/big_trace_batch.hip) had the single-float epilogue at 13.3-13.5 us of a 43-65 us
// tile.  Same arithmetic, element by element, as big_epi_half.
constexpr int BCP = 136;   // LDS pitch of the C image (floats): lanes 32..63 of a column write land 32 banks over
template <int MODE, int NB = 2>
__device__ __forceinline__ void big_epilogue_rows(const BigGemmArgs& g, float* Cb, float* Db, const float* Eb,
                                                  const float* rs, int M, int i0, int j0, const f32x16 (&acc)[2][NB],
                                                  float* sm) {
  constexpr bool EPI = MODE == 2;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = NB == 1 ? (w >> 2) : (w >> 1), wc = NB == 1 ? (w & 3) : (w & 1);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        sm[(64 * wr + 32 * a + 4 * (lane >> 5) + (r & 3) + 8 * (r >> 2)) * BCP + 32 * NB * wc + 32 * b + (lane & 31)] =
            acc[a][b][r];
  __syncthreads();
  // the scalar arguments the chunk loop uses, read once (left in the argument struct, several were spilled and
  // re-read from scratch per chunk)
  const int gm = M, gn = g.n;
  const int64_t sCi = g.sCi, sEi = EPI ? g.sEi : 0;
  const float alpha = g.alpha, beta = g.beta, dadd = g.diag_add, gamma = EPI ? g.gamma : 0.0f;
  const bool lower = g.flags & NMGP_OUT_LOWER;
  const bool tril = MODE && (g.flags & NMGP_OUT_TRIL);
  const bool eLo = g.flags & NMGP_EPI_E_LOWER;
  const bool ldc = beta != 0.0f;
  const int c4 = (t & 31) * 4, rb = t >> 5;   // row rb + RS (RQ h + q): RS = threads / 32 rows apart
  constexpr int RS = 16 / NB, RQ = 4 * NB;
  const int j = j0 + c4;
  // (the pointers are wave-uniform; said explicitly, or the compiler may keep one in VGPRs and wrap every buffer
  // access in a waterfall loop)
  Cb = (float*)uniform64((int64_t)Cb);
  if constexpr (EPI) {
    Eb = (const float*)uniform64((int64_t)Eb);
    rs = (const float*)uniform64((int64_t)rs);
  }
  const __amdgpu_buffer_rsrc_t rC = make_rsrc(Cb, ((int64_t)(gm - 1) * sCi + gn) * 4);
  const __amdgpu_buffer_rsrc_t rE = make_rsrc(EPI ? Eb : Cb, EPI ? ((int64_t)(gm - 1) * sEi + gn) * 4 : 0);
  const __amdgpu_buffer_rsrc_t rR = make_rsrc(EPI ? rs : Cb, EPI ? (int64_t)gm * 4 : 0);
  const bool dst = EPI && Db != nullptr;
  const int64_t sDi = EPI ? g.sDi : 0;
  const __amdgpu_buffer_rsrc_t rD =
      make_rsrc(dst ? (float*)uniform64((int64_t)Db) : Cb, dst ? ((int64_t)(gm - 1) * sDi + gn) * 4 : 0);
  constexpr uint32_t oob = 0x80000000u;
  // 16 chunks per thread in two halves of 8 (loads of a half in flight together)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float4 cv[RQ], ev[RQ];
    float rv[RQ];
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const int i = i0 + rb + RS * (RQ * h + q);
      // a chunk is read when any of its elements keeps a computed value (not wholly above an OUT_LOWER / OUT_TRIL
      // diagonal, inside the matrix); out-of-range columns read 0 through the resource bound
      const bool rd = i < gm && j < gn && !((lower || tril) && j > i);
      cv[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rC, ldc && rd ? (uint32_t)(((int64_t)i * sCi + j) * 4) : oob, 0, 0));
      if constexpr (EPI) {
        ev[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                               rE, rd && !(eLo && j > i) ? (uint32_t)(((int64_t)i * sEi + j) * 4) : oob,
                                               0, 0));
        rv[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rR, rd ? (uint32_t)(i * 4) : oob, 0, 0));
      }
    }
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const int row = rb + RS * (RQ * h + q);
      const int i = i0 + row;
      if (i >= gm || j >= gn) continue;
      if (lower && j > i) continue;                 // wholly above the diagonal: nothing stored
      const float4 av = *(const float4*)&sm[row * BCP + c4];
      float x[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int jj = j + e;
        float v = ((const float*)&av)[e] * alpha;
        if (ldc) v += beta * ((const float*)&cv[q])[e];
        if constexpr (MODE == 1) {
          if (i == jj) v += dadd;
        }
        if constexpr (EPI) {
          if (!(eLo && jj > i)) v += gamma * rv[q] * ((const float*)&ev[q])[e];
        }
        if (tril && jj > i) v = 0.0f;
        x[e] = v;
      }
      const uint32_t off = (uint32_t)(((int64_t)i * sCi + j) * 4);
      if (dst) {
        // the raw product (D: no OUT_LOWER / OUT_TRIL masking -- the host allows D on full outputs only)
        const uint32_t offd = (uint32_t)(((int64_t)i * sDi + j) * 4);
        if (j + 3 < gn) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4g, av), rD, offd, 0, 0);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(((const float*)&av)[e]), rD,
                                                  j + e < gn ? offd + 4 * e : oob, 0, 0);
        }
      }
      if (j + 3 < gn && !(lower && j + 3 > i)) {
        u32x4g v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = __float_as_uint(x[e]);
        __builtin_amdgcn_raw_buffer_store_b128(v, rC, off, 0, 0);
      } else {
        // a chunk across the matrix edge or an OUT_LOWER diagonal: the elements that are not stored take an
        // out-of-range offset (buffer stores past the resource are dropped)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x[e]), rC,
                                                j + e < gn && !(lower && j + e > i) ? off + 4 * e : oob, 0, 0);
      }
    }
  }
  __syncthreads();   // the LDS image is the next tile's staging buffer (stream-K workgroups run several tiles)
}

template <int NB = 2>
__device__ inline void zero_acc(f32x16 (&acc)[2][NB]) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;
}

template <bool AK, bool BK, int MODE, int NB>
// second argument: waves per SIMD (two workgroups per CU: 2 with 4 waves, 4 with 8 waves -- 128 VGPRs)
__global__ __launch_bounds__(512 / NB, 4 / NB) void gemm_big_kernel(const BigGemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) float big_smem[];
  BIG_STAMP(0);
  // XCD-aware block order: hardware places block b on XCD b % 8; give each XCD a contiguous run
  int bid = blockIdx.x;
  const int nb = gridDim.x;
  if ((nb & 7) != 0) {
    // (tile counts that are not a multiple of 8 -- e.g. the 36 lower tiles of a batched SYRK -- already
    // spread each problem's tiles over the XCDs through the flattened workgroup index)
  } else if (gridDim.y == 1) {
    bid = (bid & 7) * (nb >> 3) + (bid >> 3);
  } else {
    // batched (one problem per blockIdx.y): workgroup x runs on XCD x % 8, so the contiguous-run map above
    // gave each XCD the same tile row of EVERY problem -- with triangular operands (the ECoG / HCP factor
    // products) the row with the longest k ranges landed on one XCD (144 of 480 k-tiles per problem at
    // M = 1024).  Rotating the tile index by 9 per problem walks each XCD over all tile columns instead.
    bid = (int)(((int64_t)bid + 9LL * blockIdx.y) % nb);
  }
  f32x16 acc[2][NB];
  // persistent batched grid (measured on the batched SYRK, tools/big8p_probe.hip: 2.70-2.99 -> 2.25-2.37 ms, the
  // same results bit for bit): a fixed set of co-resident workgroups walks the work items instead of one
  // workgroup per (tile, problem) -- no per-workgroup launch / LDS allocation per tile and no tail of ragged
  // triangular tiles at the end of the grid
  const int wstep = g.persist ? (int)gridDim.x : 1;
  for (int wi = g.persist ? (int)blockIdx.x : 0; wi < (g.persist ? g.total : 1); wi += wstep) {
  const int64_t bat = g.persist ? (int64_t)(wi % g.batch) : (int64_t)blockIdx.y;
  const int bidw = g.persist ? wi / g.batch : bid;
  int K = g.k, koff = g.koff;
  if constexpr (MODE != 0) {
    if (g.kseg != nullptr) {
      const int s0 = uniform32(g.kseg[bat]);
      const int k0 = uniform32(g.seg[s0]), k1 = uniform32(g.seg[s0 + uniform32(g.kspan[bat])]);
      K = max(0, k1 - k0);
      koff = k0;
    }
  }
  // this problem's rows (row-segment variants): read where needed rather than kept live across the main loop
  auto rows_of = [&](int& M, int64_t& roff) {
    M = g.m;
    roff = 0;
    if constexpr (MODE != 0) {
      if (g.rseg != nullptr) {
        const int s0 = uniform32(g.rseg[bat]);
        const int r0 = uniform32(g.seg[s0]), r1 = uniform32(g.seg[s0 + uniform32(g.rspan[bat])]);
        M = min(g.m, max(0, r1 - r0));
        roff = r0;
      }
    }
  };

  // One work segment per pass: a (tile, k-tile range).  Data-parallel / split-K grids run one
  // pass.  Stream-K (batch 1, every tile the same k range): workgroup w owns iterations
  // [lo(w), lo(w+1)) of the flattened (tile, k-tile) space, lo(w) = floor(w I / G), so every
  // workgroup does the same MFMA work whatever the tile count; a tile cut by a range boundary is
  // finished by the last of its contributors, summing partials in k order (deterministic).
  const bool sk = g.streamk;
  const int S = g.ksplit;
  const int nkt_u = (K + BBK - 1) / BBK;
  const int64_t I = (int64_t)g.tiles * nkt_u, G = nb;
  auto lo = [&](int64_t w) { return (w * I) / G; };
  auto wg_of = [&](int64_t i) { return (int)(((i + 1) * G - 1) / I); };
  int64_t it = sk ? lo(bid) : 0;
  const int64_t end = sk ? lo(bid + 1) : 1;
  while (it < end) {
    int tile, kt0, kt1, kend, nparts = 1, me = 0, c0 = 0;
    int64_t step;
    if (sk) {
      tile = (int)(it / nkt_u);
      const int ka = (int)(it - (int64_t)tile * nkt_u);
      const int kb = (int)min((int64_t)nkt_u, (int64_t)ka + (end - it));
      kend = K;
      kt0 = ka * BBK;
      kt1 = min(K, kb * BBK);
      step = kb - ka;
      if (ka > 0 || kb < nkt_u) {
        c0 = wg_of((int64_t)tile * nkt_u);
        nparts = wg_of((int64_t)tile * nkt_u + nkt_u - 1) - c0 + 1;
        me = bid - c0;
      }
    } else {
      tile = bidw / S;
      const int split = bidw - tile * S;
      int tm0, tn0, kbeg;
      tile_coords(g, tile, tm0, tn0);
      tile_krange(g, K, tm0 * BBM, tn0 * BBN, kbeg, kend);
      // a tile wholly above the diagonal of an OUT_TRIL output (offsets variants) is stored as zeros:
      // no operand loads or MFMAs (the L-bar products over the minibatch rows have long k ranges)
      if (MODE != 0 && (g.flags & NMGP_OUT_TRIL) && tn0 * BBN > tm0 * BBM + BBM - 1) kend = kbeg;
      const int nkt = kend > kbeg ? (kend - kbeg + BBK - 1) / BBK : 0;
      const int chunk = (nkt + S - 1) / S;
      kt0 = kbeg + min(split * chunk, nkt) * BBK;
      kt1 = min(kend, kbeg + min((split + 1) * chunk, nkt) * BBK);
      nparts = S;
      me = split;
      step = 1;
    }
    int tm, tn;
    tile_coords(g, tile, tm, tn);
    const int i0 = tm * BBM, j0 = tn * BBN;
    int M;
    int64_t roff;
    rows_of(M, roff);
    if (i0 >= M) {          // past this problem's rows (row-segment variants): nothing to compute or store
      it += step;
      continue;
    }
    zero_acc(acc);
    big_mainloop<AK, BK, MODE, 0, NB>(g, K, koff, M, roff, big_smem, bat, i0, j0, kend, kt0, kt1, acc);
    BIG_STAMP(2);
    bool store = true;
    if (nparts > 1) {
      const int64_t slot0 = (bat * g.tiles + tile) * (int64_t)S;
      auto slot_of = [&](int c) -> int64_t {
        if (!sk) return slot0 + c;
        const int wgc = c0 + c;
        return 2 * wgc + ((lo(wgc) / nkt_u) == tile ? 0 : 1);
      };
      int32_t* ctr = sk ? g.counters + c0 : g.counters + bat * g.tiles + tile;
      store = big_combine(g, me, nparts, ctr, slot_of, acc);
    }
    BIG_STAMP(3);
    if (store) {
      rows_of(M, roff);
      // row-vector epilogue when C (and E) rows are contiguous and 16-byte aligned (every engine product)
      constexpr bool EPI = MODE == 2;
      float* Cb = g.C + (MODE ? uniform64(g.offC[bat]) : bat * g.sCb) + roff * g.sCi;
      const float* Eb = EPI ? g.E + (g.offE ? uniform64(g.offE[bat]) : 0) + roff * g.sEi : nullptr;
      const float* rsb = EPI ? g.RS + (g.offRS ? uniform64(g.offRS[bat]) : 0) + roff : nullptr;
      float* Db = (EPI && g.D != nullptr) ? g.D + uniform64(g.offD[bat]) + roff * g.sDi : nullptr;
      const bool rows = g.sCj == 1 && (g.sCi & 3) == 0 && (((uintptr_t)Cb) & 15) == 0 &&
                        (!EPI || (g.sEj == 1 && (g.sEi & 3) == 0 && (((uintptr_t)Eb) & 15) == 0)) &&
                        (Db == nullptr || ((g.sDi & 3) == 0 && (((uintptr_t)Db) & 15) == 0));
      if (rows)
        big_epilogue_rows<MODE>(g, Cb, Db, Eb, rsb, M, i0, j0, acc, big_smem);
      else
        big_epilogue<MODE>(g, Cb, Db, Eb, rsb, M, i0, j0, acc);
    }
    it += step;
  }
  }   // persistent work items
#ifdef NMGP_BIG_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  BIG_STAMP(4);
#endif
}

// ------------------------------------------------------------------ blocked potrf: panel + lookahead
// One launch per block step j of the blocked Cholesky (chol.hip potrf_blocked, f32): workgroup i owns
// row tile i (128 rows) below the diagonal block.
//   1. L_i = A_i X_jj^T                 (k = nb; in place: the workgroup reads its rows in full first)
//      stored write-through (sc1); workgroup 0's tile L_0 (the rows of block column j+1) is published
//      with a flag once its stores drained.
//   2. every workgroup waits for the flag, then A(rows i, block column j+1) -= L_i L_0^T, its operands
//      read back with sc1 loads (L_i: its own write-through stores; L_0: workgroup 0's).
// The flag is reset by the last workgroup to finish reading, so graph replays start from zero.  Only
// workgroup 0 is waited on and it is dispatched first, so the grid need not be co-resident.
struct PotrfStepArgs {
  float* P;            // panel: A(r0, j0), rows n2, row stride lda (becomes L_j)
  float* C;            // lookahead target: A(r0, r0)
  const float* X;      // X_jj = L_jj^{-1}, ld PNB
  int64_t lda;
  int n2, nb, c1;
  int32_t* flag;       // [0] published flag, [1] readers done
};

__global__ __launch_bounds__(256, 2) void potrf_step_kernel(PotrfStepArgs pa) {
  extern __shared__ __attribute__((aligned(16))) float big_smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int i0 = blockIdx.x * BBM;
  f32x16 acc[2][2];
  // 1. panel tile
  BigGemmArgs g{};
  g.A = pa.P; g.lda = pa.lda; g.B = pa.X; g.ldb = 128; g.C = pa.P; g.sCi = pa.lda; g.sCj = 1;
  g.m = pa.n2; g.n = pa.nb; g.k = pa.nb; g.flags = NMGP_B_UPPER; g.alpha = 1.0f; g.beta = 0.0f;
  zero_acc(acc);
  big_mainloop<true, true, 0>(g, g.k, 0, g.m, 0, big_smem, 0, i0, 0, pa.nb, 0, pa.nb, acc);
  {
    const __amdgpu_buffer_rsrc_t rC = make_rsrc(pa.P, ((int64_t)(pa.n2 - 1) * pa.lda + pa.nb) * 4);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int i = i0 + 64 * wr + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const int j = 64 * wc + 32 * b + (lane & 31);
          if (i < pa.n2 && j < pa.nb)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][r]), rC,
                                                  (uint32_t)(((int64_t)i * pa.lda + j) * 4), 0, 16 /* sc1 */);
        }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (blockIdx.x == 0 && t == 0) __hip_atomic_store(pa.flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t == 0) {
    // bounded: a lost publisher must not hang the GPU (the result is then wrong, not stuck)
    bool seen = false;
    for (int spin = 0; spin < (1 << 26); ++spin) {
      if (__hip_atomic_load(pa.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
        seen = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!seen) spin_gave_up(NMGP_STATUS_POTRF_SPIN);   // surfaced by nmgp_device_status()
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // 2. lookahead: A(rows i, block column j+1) -= L_i L_0^T
  BigGemmArgs g2{};
  g2.A = pa.P; g2.lda = pa.lda; g2.B = pa.P; g2.ldb = pa.lda; g2.C = pa.C; g2.sCi = pa.lda; g2.sCj = 1;
  g2.m = pa.n2; g2.n = pa.c1; g2.k = pa.nb; g2.flags = 0; g2.alpha = -1.0f; g2.beta = 1.0f;
  zero_acc(acc);
  big_mainloop<true, true, 0, 16>(g2, g2.k, 0, g2.m, 0, big_smem, 0, i0, 0, pa.nb, 0, pa.nb, acc);
  if (t == 0) {
    const int old = __hip_atomic_fetch_add(pa.flag + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (int)gridDim.x - 1) {   // every reader is past its loads of L_0: re-arm for the next launch
      __hip_atomic_store(pa.flag, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(pa.flag + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  big_epilogue<0>(g2, g2.C, nullptr, nullptr, nullptr, g2.m, i0, 0, acc);
}

// Row-panel variant (the default): the step kernel above runs two dependent 128x128x128 products on each
// of n2/128 workgroups (<= 31 CUs busy, ~30 us per block step on the serial chain of the factorization).
// Here workgroup b owns 16 RB panel rows: 8x (RB = 1) or 4x (RB = 2) the workgroups, 1/8 or 1/4 of the
// serial MFMA work each.  Wave w owns output columns [32w, 32w + 32) as RB x 2 16x16 f32 MFMA blocks;
// k = nb = 128 in one register-resident panel: lane (li, g) loads k = 32g .. 32g + 31 of its rows (eight
// 16-byte loads per row block) and MFMA step s consumes k-slot g <-> k = 32g + s for both operands (a sum
// over k does not care about the order).  The workgroups holding the rows of block column j+1 (L_0)
// publish by counting on flag[0]; every workgroup then reads them back (sc1) for
// A(rows, block column j+1) -= L_i L_0^T.  In place: the four waves read all of their rows before the
// barrier that precedes the stores.
template <int RB>
__global__ __launch_bounds__(256) void potrf_step32_kernel(PotrfStepArgs pa) {
  constexpr int ROWS = 16 * RB;
  constexpr int LP = 128 + 4;                                   // LDS pitch of the L_i rows (floats)
  __shared__ __attribute__((aligned(16))) float Ls[ROWS * LP];
  const int t = threadIdx.x, lane = t & 63, li = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int i0 = blockIdx.x * ROWS;
  const int npub = (pa.c1 + ROWS - 1) / ROWS;                   // workgroups holding L_0
  const __amdgpu_buffer_rsrc_t rP = make_rsrc(pa.P, ((int64_t)(pa.n2 - 1) * pa.lda + pa.nb) * 4);
  const __amdgpu_buffer_rsrc_t rX = make_rsrc(pa.X, (int64_t)128 * 128 * 4);
  const __amdgpu_buffer_rsrc_t rC = make_rsrc(pa.C, ((int64_t)(pa.n2 - 1) * pa.lda + pa.c1) * 4);
  float a[RB][PS_NV], b[2][PS_NV];
  f32x4 acc[RB][2];
#pragma unroll
  for (int q = 0; q < 2 * RB; ++q) acc[q >> 1][q & 1] = f32x4{0, 0, 0, 0};
  // 1. L_i = A_i X^T: op(B)(k, j) = X[j][k], zero above the diagonal (X lower triangular)
  ps_load_rows<RB>(a, rP, i0, pa.lda, pa.n2, false);
  ps_load_rows<2>(b, rX, 32 * w, 128, pa.nb, false);
  f32x4 cv[RB][2];
  uint32_t coff[RB][2][4];
  ps_load_c<RB>(rC, i0, pa.lda, pa.n2, pa.c1, cv, coff, w);   // behind the operands: overlaps the panel product
#pragma unroll
  for (int bj = 0; bj < 2; ++bj)
#pragma unroll
    for (int s = 0; s < PS_NV; ++s) b[bj][s] = keep_if(b[bj][s], PS_NV * g + s <= 32 * w + 16 * bj + li);
  ps_mma<RB>(a, b, acc);
  __syncthreads();   // every wave has read its rows of A_i: the in-place stores may start
#pragma unroll
  for (int q = 0; q < 2 * RB; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int il = 16 * (q >> 1) + 4 * g + r, j = 32 * w + 16 * (q & 1) + li;
      const int i = i0 + il;
      Ls[il * LP + j] = acc[q >> 1][q & 1][r];
      if (i < pa.n2 && j < pa.nb)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[q >> 1][q & 1][r]), rP,
                                              (uint32_t)(((int64_t)i * pa.lda + j) * 4), 0, 16 /* sc1 */);
    }
  if (pa.c1 == 0) return;   // panel only: no lookahead column, no hand-off (the flags stay untouched)
  const bool pub = (int)blockIdx.x < npub;
  if (pub) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    if (pub) __hip_atomic_fetch_add(pa.flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // bounded: a lost publisher must not hang the GPU (the status word reports it).  The publishers are
    // the lowest block indices and wait on nobody, so the grid need not be co-resident.
    bool seen = false;
    for (int spin = 0; spin < (1 << 26); ++spin) {
      if (__hip_atomic_load(pa.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= npub) {
        seen = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!seen) spin_gave_up(NMGP_STATUS_POTRF_SPIN);
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // 2. lookahead: A(rows i, block column j+1) -= L_i L_0^T; L_i from LDS, L_0 read back write-through
#pragma unroll
  for (int q = 0; q < 2 * RB; ++q) acc[q >> 1][q & 1] = f32x4{0, 0, 0, 0};
  ps_load_rows<2>(b, rP, 32 * w, pa.lda, pa.c1, true);
#pragma unroll
  for (int bi = 0; bi < RB; ++bi)
#pragma unroll
    for (int q = 0; q < PS_NV / 4; ++q) {
      const float4 v = *(const float4*)&Ls[(16 * bi + li) * LP + PS_NV * g + 4 * q];
      a[bi][4 * q + 0] = v.x;
      a[bi][4 * q + 1] = v.y;
      a[bi][4 * q + 2] = v.z;
      a[bi][4 * q + 3] = v.w;
    }
  ps_mma<RB>(a, b, acc);
  if (t == 0) {
    const int old = __hip_atomic_fetch_add(pa.flag + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (int)gridDim.x - 1) {   // every reader is past its loads of L_0: re-arm for the next launch
      __hip_atomic_store(pa.flag, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(pa.flag + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  ps_store_c<RB>(rC, cv, coff, acc);
}

// The first block column of a trailing update on the row-panel scheme: C(i, j) -= sum_k L[i][k] L[j][k] for
// i < m, j < c1 (k = 128; the B rows are L's rows 0..c1-1).  The blocked potrf runs the column next to the
// lookahead (block column j+2 at step j) as this separate strip launch ahead of the rest of the trailing
// SYRK, so the next step kernel -- which writes that column too -- waits only for the strip.
template <int RB>
__global__ __launch_bounds__(256) void potrf_strip32_kernel(const float* L, float* C, int64_t lda, int m, int c1) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i0 = blockIdx.x * 16 * RB;
  const __amdgpu_buffer_rsrc_t rL = make_rsrc(L, ((int64_t)(m - 1) * lda + 128) * 4);
  const __amdgpu_buffer_rsrc_t rC = make_rsrc(C, ((int64_t)(m - 1) * lda + c1) * 4);
  float a[RB][PS_NV], b[2][PS_NV];
  f32x4 acc[RB][2];
#pragma unroll
  for (int q = 0; q < 2 * RB; ++q) acc[q >> 1][q & 1] = f32x4{0, 0, 0, 0};
  ps_load_rows<RB>(a, rL, i0, lda, m, false);
  ps_load_rows<2>(b, rL, 32 * w, lda, c1, false);
  f32x4 cv[RB][2];
  uint32_t coff[RB][2][4];
  ps_load_c<RB>(rC, i0, lda, m, c1, cv, coff, w);
  ps_mma<RB>(a, b, acc);
  ps_store_c<RB>(rC, cv, coff, acc);
}

// 32 rows per workgroup of the step / strip kernels (round 2: 16 rows halved the MFMA work per workgroup and
// measured the same 1.52-1.54 ms at M = 4096 -- the kernels are bound by their memory round trips and the L_0
// hand-off, not by the products)
int potrf_strip_f32(const float* L, float* C, int64_t lda, int m, int c1, hipStream_t s) {
  if (m <= 0 || c1 <= 0) return NMGP_OK;
  hipLaunchKernelGGL(potrf_strip32_kernel<2>, dim3((unsigned)((m + 31) / 32)), dim3(256), 0, s, L, C, lda, m, c1);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

// c1 = 0: the panel product only (no lookahead column)
int potrf_step_f32(float* P, float* C, const float* X, int64_t lda, int n2, int nb, int c1, int32_t* flag,
                   hipStream_t s) {
  if (n2 <= 0) return NMGP_OK;
  PotrfStepArgs pa{P, C, X, lda, n2, nb, c1, flag};
  if (nb == 128) {
    hipLaunchKernelGGL(potrf_step32_kernel<2>, dim3((unsigned)((n2 + 31) / 32)), dim3(256), 0, s, pa);
    NMGP_CHECK_LAUNCH();
    return NMGP_OK;
  }
  // (a narrower last block: the 128-row tile form)
  const size_t lds = 2 * BSTAGE * sizeof(float);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)potrf_step_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(potrf_step_kernel, dim3((unsigned)((n2 + BBM - 1) / BBM)), dim3(256), lds, s, pa);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

// Accumulator column blocks per wave of the gemm_big_kernel launches: 1 = 8 waves (512 threads) per 128 x 128 tile,
// 64 x 32 per wave (tools/big8_probe.hip: the batched SYRK 4-11 % faster than 4 waves of 64 x 64, bit-identical;
// ECoG step 0.333 -> 0.328 s, profiles/r05aa_*).  Products with BOTH operands k-strided (the KL L-bar) keep 4 waves:
// their 8-wave form spills in the staging and measured 9 % slower.
constexpr int kBigNB = 1;

// Partial slots the split-K path may use per call (workspace = slots * 64 KB + counters).
constexpr int kBigSlots = 1024;
size_t gemm_big_ws_bytes() { return (size_t)kBigSlots * BSLOT * sizeof(float) + (size_t)kBigSlots * sizeof(int32_t); }

static int cu_count() {
  static int cus = -1;
  if (cus < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess)
      cus = 256;
  }
  return cus;
}

// C(i,j) = alpha * sum_k A[i*lda + k] * op(B)(k,j) + beta * C(i,j), batched over `batch` problems.
// ws: gemm_big_ws_bytes() of device memory whose counter part is zero (the kernel leaves it zero),
// or nullptr (no split-K).
struct BigEpi {
  int a_kcontig = 1;
  const float* E = nullptr; const int64_t* offE = nullptr; int64_t sEi = 0, sEj = 0;
  const float* RS = nullptr; const int64_t* offRS = nullptr;
  float gamma = 0.0f;
  const int32_t* seg = nullptr; const int32_t* kseg = nullptr; const int32_t* kspan = nullptr;
  const int32_t* rseg = nullptr; const int32_t* rspan = nullptr;
  float* D = nullptr; const int64_t* offD = nullptr; int64_t sDi = 0;
};

static int gemm_big_f32_ex(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kcontig, float* C,
                           int64_t sCi, int64_t sCj, int m, int n, int k, int flags, float alpha, float beta,
                           int64_t sAb, int64_t sBb, int64_t sCb, const int64_t* offA, const int64_t* offB,
                           const int64_t* offC, float diag_add, int batch, void* ws, hipStream_t s,
                           const BigEpi& ep = BigEpi()) {
  if (m <= 0 || n <= 0 || batch <= 0) return NMGP_OK;
  if ((flags & NMGP_OUT_LOWER) && m < n) return -1;   // (m > n: the triangle, then full tile rows below it)
  BigGemmArgs g;
  g.A = A; g.B = B; g.C = C;
  g.offA = offA; g.offB = offB; g.offC = offC;
  g.diag_add = diag_add;
  g.a_kcontig = ep.a_kcontig;
  g.E = ep.E; g.offE = ep.offE; g.sEi = ep.sEi; g.sEj = ep.sEj;
  g.RS = ep.RS; g.offRS = ep.offRS; g.gamma = ep.gamma;
  g.seg = ep.seg; g.kseg = ep.kseg; g.kspan = ep.kspan; g.koff = 0;
  g.rseg = ep.rseg; g.rspan = ep.rspan;
  g.D = ep.D; g.offD = ep.offD; g.sDi = ep.sDi;
  if (ep.D != nullptr && (!(flags & NMGP_EPI) || ep.offD == nullptr || (flags & (NMGP_OUT_LOWER | NMGP_OUT_TRIL)) ||
                          ep.sDi < n || (int64_t)(m - 1) * ep.sDi + n >= 0x7fffffffLL / 4))
    return -1;
  if (ep.kseg != nullptr && (offA == nullptr || ep.seg == nullptr || ep.kspan == nullptr)) return -1;
  if (ep.rseg != nullptr && (offA == nullptr || ep.seg == nullptr || ep.rspan == nullptr || (flags & NMGP_OUT_LOWER)))
    return -1;
  if ((flags & NMGP_EPI) && (ep.E == nullptr || ep.RS == nullptr)) return -1;
  {
    // 32-bit buffer offsets: every problem's operand, output and epilogue spans stay below 2 GiB
    const int64_t lim = 0x7fffffffLL;
    const int64_t spanA = ep.a_kcontig ? (int64_t)(m - 1) * lda + k : (int64_t)(k - 1) * lda + m;
    const int64_t spanB = b_kcontig ? (int64_t)(n - 1) * ldb + k : (int64_t)(k - 1) * ldb + n;
    const int64_t spanC = (int64_t)(m - 1) * sCi + (int64_t)(n - 1) * sCj + 1;
    const int64_t spanE = (flags & NMGP_EPI) ? (int64_t)(m - 1) * ep.sEi + (int64_t)(n - 1) * ep.sEj + 1 : 0;
    if (spanA * 4 >= lim || spanB * 4 >= lim || spanC * 4 >= lim || spanE * 4 >= lim || sCi < 0 || sCj < 0)
      return -40;
  }
  g.lda = lda; g.ldb = ldb; g.sCi = sCi; g.sCj = sCj;
  g.sAb = sAb; g.sBb = sBb; g.sCb = sCb;
  g.m = m; g.n = n; g.k = k; g.flags = flags; g.b_kcontig = b_kcontig;
  g.alpha = alpha; g.beta = beta;
  g.tiles_m = (m + BBM - 1) / BBM;
  g.tiles_n = (n + BBN - 1) / BBN;
  g.tiles = (flags & NMGP_OUT_LOWER) ? g.tiles_n * (g.tiles_n + 1) / 2 + (g.tiles_m - g.tiles_n) * g.tiles_n
                                      : g.tiles_m * g.tiles_n;
  int S = 1, sk = 0;
  const int64_t total = (int64_t)g.tiles * batch;
  const int nkt = (k + BBK - 1) / BBK;
  const int P = 2 * cu_count();   // co-resident workgroups (the two LDS stages admit 2 per CU)
  const bool uniform_k = !(flags & (NMGP_A_LOWER | NMGP_A_UPPER | NMGP_B_UPPER | NMGP_B_LOWER));
  const int64_t dp_slots = ((total + P - 1) / P) * P;
  if (ws && batch == 1 && uniform_k && P <= kBigSlots / 2 && (double)total / (double)dp_slots < 0.9 &&
      total * nkt >= 8LL * P) {
    sk = 1;   // stream-K: 2 partial slots per workgroup, one arrival counter per workgroup
  } else if (ws && total < 2 * cu_count() && nkt >= 8) {
    S = (int)((2 * cu_count() + total - 1) / total);
    S = min(S, nkt / 4);
    S = min(S, 16);
    while (S > 1 && total * S > kBigSlots) --S;
    if (total > kBigSlots) S = 1;
  }
  g.ksplit = S;
  g.streamk = sk;
  g.batch = batch;
  g.total = (int)min(total, (int64_t)0x7fffffff);
  g.persist = (!sk && S == 1 && batch > 1) ? 1 : 0;
  g.ws = (float*)ws;
  g.counters = ws ? (int32_t*)((char*)ws + (size_t)kBigSlots * BSLOT * sizeof(float)) : nullptr;
  const size_t lds = 2 * BSTAGE * sizeof(float);
  const dim3 gd = g.persist ? dim3((unsigned)min((int64_t)P, total), 1u)
                             : dim3(sk ? (unsigned)P : (unsigned)(g.tiles * S), (unsigned)batch);
  const bool epi = flags & NMGP_EPI;
  auto go = [&](auto kern, int nb) {
    static bool attr = false;   // one per instantiation
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr = true;
    }
    hipLaunchKernelGGL(kern, gd, dim3(512 / nb), lds, s, g);
  };
  const bool offs = offA != nullptr;
  if (offs && (offB == nullptr || offC == nullptr)) return -1;
  if (!offs && (diag_add != 0.0f || (flags & NMGP_OUT_TRIL))) return -1;   // those live in the offsets variants
  if (epi) {
    // the KL L-bar forms: both operands transposed, or (the solve form's R = L21 - C21 W11) A k-contiguous
    if (!offs || g.b_kcontig) return -1;
    if (g.a_kcontig)
      go(gemm_big_kernel<true, false, 2, 2>, 2);   // (8 waves: 88 bytes of scratch per lane)
    else
      go(gemm_big_kernel<false, false, 2, 2>, 2);
  } else if (offs) {
    if (g.a_kcontig && g.b_kcontig)
      go(gemm_big_kernel<true, true, 1, kBigNB>, kBigNB);
    else if (g.a_kcontig)
      go(gemm_big_kernel<true, false, 1, kBigNB>, kBigNB);
    else if (g.b_kcontig)
      go(gemm_big_kernel<false, true, 1, kBigNB>, kBigNB);
    else
      go(gemm_big_kernel<false, false, 1, 2>, 2);
  } else {
    if (g.a_kcontig && g.b_kcontig)
      go(gemm_big_kernel<true, true, 0, kBigNB>, kBigNB);
    else if (g.a_kcontig)
      go(gemm_big_kernel<true, false, 0, kBigNB>, kBigNB);
    else if (g.b_kcontig)
      go(gemm_big_kernel<false, true, 0, kBigNB>, kBigNB);
    else
      go(gemm_big_kernel<false, false, 0, 2>, 2);
  }
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

int gemm_big_f32(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kcontig, float* C, int64_t sCi,
                 int64_t sCj, int m, int n, int k, int flags, float alpha, float beta, int64_t sAb, int64_t sBb,
                 int64_t sCb, int batch, void* ws, hipStream_t s) {
  return gemm_big_f32_ex(A, lda, B, ldb, b_kcontig, C, sCi, sCj, m, n, k, flags, alpha, beta, sAb, sBb, sCb, nullptr,
                         nullptr, nullptr, 0.0f, batch, ws, s);
}

NMGP_TU_STATUS_ACCESSOR(gemm_big)

}  // namespace nmgp

extern "C" {
int64_t nmgp_gemm_big_workspace_size(void) { return (int64_t)nmgp::gemm_big_ws_bytes(); }
int nmgp_gemm_big_f32(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kcontig, float* C, int64_t sCi,
                      int64_t sCj, int m, int n, int k, int flags, double alpha, double beta, int64_t sAb, int64_t sBb,
                      int64_t sCb, int batch, void* ws, hipStream_t s) {
  if (A == nullptr) return -1;
  if (lda < k) return -2;
  if (B == nullptr) return -3;
  if (C == nullptr) return -6;
  if (m < 0) return -9;
  if (n < 0) return -10;
  if (k < 0) return -11;
  if (batch < 0 || batch > 65535) return -18;
  return nmgp::gemm_big_f32(A, lda, B, ldb, b_kcontig, C, sCi, sCj, m, n, k, flags, (float)alpha, (float)beta, sAb,
                            sBb, sCb, batch, ws, s);
}
int nmgp_gemm_big_offsets_f32(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kcontig, float* C,
                              int64_t sCi, int64_t sCj, int m, int n, int k, int flags, double alpha, double beta,
                              double diag_add, const int64_t* offA, const int64_t* offB, const int64_t* offC,
                              int batch, void* ws, hipStream_t s) {
  if (A == nullptr) return -1;
  if (lda < k) return -2;
  if (B == nullptr) return -3;
  if (C == nullptr) return -6;
  if (m < 0) return -9;
  if (n < 0) return -10;
  if (k < 0) return -11;
  if (offA == nullptr) return -16;
  if (offB == nullptr) return -17;
  if (offC == nullptr) return -18;
  if (batch < 0 || batch > 65535) return -19;
  return nmgp::gemm_big_f32_ex(A, lda, B, ldb, b_kcontig, C, sCi, sCj, m, n, k, flags, (float)alpha, (float)beta, 0, 0,
                               0, offA, offB, offC, (float)diag_add, batch, ws, s);
}
static int big_offsets_impl(const float* A, int64_t lda, int a_kcontig, const float* B, int64_t ldb, int b_kcontig,
                            float* C, int64_t sCi, int64_t sCj, int m, int n, int k, int flags, double alpha,
                            double beta, double diag_add, const int64_t* offA, const int64_t* offB, const int64_t* offC,
                            const float* E, const int64_t* offE, int64_t sEi, int64_t sEj, const float* RS,
                            const int64_t* offRS, double gamma, const int32_t* seg, const int32_t* kseg,
                            const int32_t* kspan, const int32_t* rseg, const int32_t* rspan, int batch, void* ws,
                            hipStream_t s, float* D = nullptr, const int64_t* offD = nullptr, int64_t sDi = 0) {
  if (A == nullptr) return -1;
  if (B == nullptr) return -4;
  if (C == nullptr) return -7;
  if (m < 0) return -10;
  if (n < 0) return -11;
  if (k < 0) return -12;
  if (lda < (a_kcontig ? k : m)) return -2;
  if (offA == nullptr) return -17;
  if (offB == nullptr) return -18;
  if (offC == nullptr) return -19;
  if ((flags & NMGP_EPI) && (E == nullptr || offE == nullptr)) return -20;
  if ((flags & NMGP_EPI) && (RS == nullptr || offRS == nullptr)) return -24;
  if (batch < 0 || batch > 65535) return -30;
  nmgp::BigEpi ep;
  ep.a_kcontig = a_kcontig ? 1 : 0;
  ep.E = E; ep.offE = offE; ep.sEi = sEi; ep.sEj = sEj;
  ep.RS = RS; ep.offRS = offRS; ep.gamma = (float)gamma;
  if (kseg != nullptr && (seg == nullptr || kspan == nullptr)) return -26;
  if (rseg != nullptr && (seg == nullptr || rspan == nullptr)) return -27;
  if (rseg != nullptr && (flags & NMGP_OUT_LOWER)) return -13;
  ep.seg = seg; ep.kseg = kseg; ep.kspan = kspan;
  ep.rseg = rseg; ep.rspan = rspan;
  ep.D = D; ep.offD = offD; ep.sDi = sDi;
  return nmgp::gemm_big_f32_ex(A, lda, B, ldb, b_kcontig, C, sCi, sCj, m, n, k, flags, (float)alpha, (float)beta, 0, 0,
                               0, offA, offB, offC, (float)diag_add, batch, ws, s, ep);
}
int nmgp_gemm_big_offsets_epi_f32(const float* A, int64_t lda, int a_kcontig, const float* B, int64_t ldb,
                                  int b_kcontig, float* C, int64_t sCi, int64_t sCj, int m, int n, int k, int flags,
                                  double alpha, double beta, double diag_add, const int64_t* offA,
                                  const int64_t* offB, const int64_t* offC, const float* E, const int64_t* offE,
                                  int64_t sEi, int64_t sEj, const float* RS, const int64_t* offRS, double gamma,
                                  const int32_t* seg, const int32_t* kseg, const int32_t* kspan, int batch,
                                  void* ws, hipStream_t s) {
  return big_offsets_impl(A, lda, a_kcontig, B, ldb, b_kcontig, C, sCi, sCj, m, n, k, flags, alpha, beta, diag_add,
                          offA, offB, offC, E, offE, sEi, sEj, RS, offRS, gamma, seg, kseg, kspan, nullptr, nullptr,
                          batch, ws, s);
}
int nmgp_gemm_big_offsets_seg_f32(const float* A, int64_t lda, int a_kcontig, const float* B, int64_t ldb,
                                  int b_kcontig, float* C, int64_t sCi, int64_t sCj, int m, int n, int k, int flags,
                                  double alpha, double beta, double diag_add, const int64_t* offA,
                                  const int64_t* offB, const int64_t* offC, const float* E, const int64_t* offE,
                                  int64_t sEi, int64_t sEj, const float* RS, const int64_t* offRS, double gamma,
                                  const int32_t* seg, const int32_t* kseg, const int32_t* kspan, const int32_t* rseg,
                                  const int32_t* rspan, int batch, void* ws, hipStream_t s) {
  return big_offsets_impl(A, lda, a_kcontig, B, ldb, b_kcontig, C, sCi, sCj, m, n, k, flags, alpha, beta, diag_add,
                          offA, offB, offC, E, offE, sEi, sEj, RS, offRS, gamma, seg, kseg, kspan, rseg, rspan, batch,
                          ws, s);
}
int nmgp_gemm_big_offsets_dual_f32(const float* A, int64_t lda, int a_kcontig, const float* B, int64_t ldb,
                                   int b_kcontig, float* C, int64_t sCi, int64_t sCj, int m, int n, int k, int flags,
                                   double alpha, double beta, const int64_t* offA, const int64_t* offB,
                                   const int64_t* offC, const float* E, const int64_t* offE, int64_t sEi, int64_t sEj,
                                   const float* RS, const int64_t* offRS, double gamma, float* D, const int64_t* offD,
                                   int64_t sDi, int batch, hipStream_t s) {
  if (!(flags & NMGP_EPI)) return -13;
  if (D == nullptr) return -27;
  if (offD == nullptr) return -28;
  if (sDi < n) return -29;
  return big_offsets_impl(A, lda, a_kcontig, B, ldb, b_kcontig, C, sCi, sCj, m, n, k, flags, alpha, beta, 0.0, offA,
                          offB, offC, E, offE, sEi, sEj, RS, offRS, gamma, nullptr, nullptr, nullptr, nullptr, nullptr,
                          batch, nullptr, s, D, offD, sDi);
}
}
