// Pair-block streaming kernels (round 5): the per-coefficient-pair products of the DSVI step when every output
// owns only a few minibatch rows -- the ECoG shape (BASELINE.json configs[3]: D = 128 outputs, B = 512 rows, ~4
// rows per output, Q = 8256 pairs (i, j <= i) of M = 1024).  Each pair's sqrt_U block L_ij (M x M, lower; the
// reference's mat2ltri, code/utils.py:68-72) meets only the R rows of output i, so the products are R x M x M:
// with R ~ 4 they are bound by streaming L_ij (or its gradient block) from HBM, not by MFMA.  The grouped GEMM ran
// them as 64-row MFMA tiles (~94 % padding, a k loop per tile).  Here every problem streams its M x M lower
// triangle ONCE in 16-byte loads with the R rows' operands held on chip:
//
//   quad  C[r] = A[r] L            (MGP_d quadratic-form factors W = P_{0/1} L_ij, code/utils.py:115-120)
//                                  out[r][c] = sum_{k >= c} A[r][k] L[k][c]: rows k of L are axpy'd into the
//                                  lane-owned columns; the 4 waves of a block split k and add in wave order.
//   dot   Z[r] = W[r] L^T          (their adjoint P-bar += W-hat L^T, the autograd of the same MGP_d)
//                                  Z[r][c] = sum_{k <= c} W[r][k] L[c][k]: one dot product per row c of L,
//                                  DPP wave reductions; W's R rows live in registers.
//   rank  G += P^T W  (lower)      (L-bar of the pair, the autograd of W = P L: the gradient block's lower
//                                  triangle, read-modify-write once; the strictly upper part is not touched)
//   pbar_reduce                    P-bar_1[r] += Z_i[r] and P-bar_0[r] += Z_0[r] + ... + Z_{i-1}[r] (j order) for
//                                  row r of output i: the diagonal pair feeds the L1 prior, the others the L0 one
//
// Rows of a problem: [seg[s], seg[s+1]) of the minibatch (row index r addresses A / W / C / Z / P at row r).  R is
// read on the device (minibatch-dependent); R > RB runs in chunks of RB rows (re-streaming the block).
// Bound: HBM, M (M + 1) / 2 elements of L_ij per problem (quad, dot) or twice that (rank: read + write).
#include "common.hpp"

namespace nmgp {

constexpr int PT = 256;      // threads per block (4 waves)
constexpr int PROWS = 128;   // rows of L (dot) / of the gradient block (rank) per block

template <typename T> struct PairCfg;
template <> struct PairCfg<float> {
  static constexpr int V = 4;     // elements per 16-byte vector
  static constexpr int RB = 8;    // rows of output per pass
};
template <> struct PairCfg<double> {
  static constexpr int V = 2;
  static constexpr int RB = 4;
};
constexpr int PMAXM = 1024;       // dot / rank keep a row's W values in registers: M <= 64 V NCH

template <typename T, int V> __device__ inline void vmask(T (&v)[V], int c0, int kmax) {
#pragma unroll
  for (int e = 0; e < V; ++e) v[e] = keep_if(v[e], c0 + e <= kmax);
}

// 16 bytes through a buffer resource: an offset past the resource's extent (0x80000000) reads zeros, so a
// masked-off load needs no branch (a load under a runtime condition is sunk into its own exec-masked branch
// with a full wait, serialising the loads that should be in flight together)
template <typename T, int V> __device__ inline void vload_b(T (&v)[V], __amdgpu_buffer_rsrc_t r, uint32_t off) {
  typedef T vec_t __attribute__((ext_vector_type(V)));
  const vec_t x = __builtin_bit_cast(vec_t, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
#pragma unroll
  for (int e = 0; e < V; ++e) v[e] = x[e];
}
// ------------------------------------------------------------------------------------------------ quad
// grid (problems, column blocks of 64 V columns).  Lane l of every wave owns columns kstart + l V .. + V - 1;
// wave w takes the rows k = kstart + w + 4 i of L (k >= the block's first column: rows above contribute 0).
template <typename T>
__global__ __launch_bounds__(PT) void pair_quad_kernel(const T* __restrict__ A, const T* __restrict__ L,
                                                       T* __restrict__ C, const nmgp_pair_desc* __restrict__ descs,
                                                       const int32_t* __restrict__ seg, int M) {
  constexpr int V = PairCfg<T>::V, RB = PairCfg<T>::RB, CB = 64 * V;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const nmgp_pair_desc d = descs[blockIdx.x];
  const int r0 = seg[d.seg], R = seg[d.seg + 1] - r0;
  const int kstart = blockIdx.y * CB;
  if (R <= 0 || kstart >= M) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nk = M - kstart;
  T* sA = (T*)smem_raw;                    // nk x RB: A^T rows of the chunk
  T* red = sA + (size_t)nk * RB;           // 4 x RB x CB: wave partials
  const int c0 = kstart + lane * V;
  const bool colok = c0 < M;
  const __amdgpu_buffer_rsrc_t rL = make_rsrc(L + d.l_off, (int64_t)M * M * (int64_t)sizeof(T));
  const uint32_t lc = colok ? (uint32_t)(c0 * sizeof(T)) : 0x80000000u;   // (a column block past M reads zeros)
  for (int rc = 0; rc < R; rc += RB) {
    const int Rc = min(RB, R - rc);
    __syncthreads();                       // the previous chunk's readers are done
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) {
      const T* a = A + d.a_off + (int64_t)(r0 + rc + rr) * M + kstart;
      for (int i = tid; i < nk; i += PT) sA[i * RB + rr] = rr < Rc ? a[i] : (T)0;
    }
    __syncthreads();
    T acc[RB][V];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr)
#pragma unroll
      for (int e = 0; e < V; ++e) acc[rr][e] = (T)0;
    auto row = [&](int k, T (&l)[V]) {
      if (k < kstart + CB) vmask<T, V>(l, c0, k);        // the block's diagonal rows: columns > k are not L
      const T* ak = sA + (k - kstart) * RB;
#pragma unroll
      for (int rr = 0; rr < RB; ++rr) {
        const T a = ak[rr];
#pragma unroll
        for (int e = 0; e < V; ++e) acc[rr][e] = fma(a, l[e], acc[rr][e]);
      }
    };
    int k = kstart + w;
    for (; k + 28 < M; k += 32) {          // eight rows of this wave in flight
      T l[8][V];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        vload_b<T, V>(l[u], rL, colok ? lc + (uint32_t)((int64_t)(k + 4 * u) * M * sizeof(T)) : lc);
#pragma unroll
      for (int u = 0; u < 8; ++u) row(k + 4 * u, l[u]);
    }
    for (; k < M; k += 4) {
      T l0[V];
      vload_b<T, V>(l0, rL, colok ? lc + (uint32_t)((int64_t)k * M * sizeof(T)) : lc);
      row(k, l0);
    }
#pragma unroll
    for (int rr = 0; rr < RB; ++rr)
#pragma unroll
      for (int e = 0; e < V; ++e) red[(w * RB + rr) * CB + lane * V + e] = acc[rr][e];
    __syncthreads();
    for (int idx = tid; idx < Rc * CB; idx += PT) {
      const int rr = idx / CB, cc = idx - rr * CB, c = kstart + cc;
      if (c < M) {
        const T s = ((red[rr * CB + cc] + red[(RB + rr) * CB + cc]) + red[(2 * RB + rr) * CB + cc]) +
                    red[(3 * RB + rr) * CB + cc];
        C[d.c_off + (int64_t)(r0 + rc + rr) * M + c] = s;
      }
    }
  }
}

// --------------------------------------------------------------------------------------- dot / rank
// Both keep the R rows of W in registers: lane l holds W[r][j 64 V + l V + e] for the chunks j < NCH of a row.
template <typename T, int NCH>
__device__ inline void load_w(T (&wv)[PairCfg<T>::RB][NCH][PairCfg<T>::V], const T* W, int64_t off, int r0, int rc,
                              int Rc, int M, int lane) {
  constexpr int V = PairCfg<T>::V, RB = PairCfg<T>::RB;
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(W + off + (int64_t)(r0 + rc) * M, (int64_t)Rc * M * (int64_t)sizeof(T));
#pragma unroll
  for (int rr = 0; rr < RB; ++rr)
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int k0 = j * 64 * V + lane * V;
      vload_b<T, V>(wv[rr][j], rW, (rr < Rc && k0 < M) ? (uint32_t)(((int64_t)rr * M + k0) * sizeof(T)) : 0x80000000u);
    }
}

// grid (problems, row blocks of PROWS rows c of L).  Wave w takes rows c = base + w + 4 i (i < 32); per row its
// lanes stream L[c][0..c] in 16-byte vectors (chunks j <= c / (64 V)), dot them with the R rows of W, and DPP
// wave sums finish the R dot products.  Lane i keeps row base + w + 4 i's results; the block stores them at the end.
template <typename T, int NCH>
__global__ __launch_bounds__(PT) void pair_dot_kernel(const T* __restrict__ W, const T* __restrict__ L,
                                                      T* __restrict__ Z, const nmgp_pair_desc* __restrict__ descs,
                                                      const int32_t* __restrict__ seg, int M) {
  constexpr int V = PairCfg<T>::V, RB = PairCfg<T>::RB, CW = 64 * V;
  const nmgp_pair_desc d = descs[blockIdx.x];
  const int r0 = seg[d.seg], R = seg[d.seg + 1] - r0;
  const int base = blockIdx.y * PROWS;
  if (R <= 0 || base >= M) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const __amdgpu_buffer_rsrc_t rL = make_rsrc(L + d.l_off, (int64_t)M * M * (int64_t)sizeof(T));
  for (int rc = 0; rc < R; rc += RB) {
    const int Rc = min(RB, R - rc);
    T wv[RB][NCH][V];
    load_w<T, NCH>(wv, W, d.a_off, r0, rc, Rc, M, lane);
    T res[RB];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) res[rr] = (T)0;
    // two rows of this wave per iteration (all of both rows' loads in flight together)
    for (int i = 0; i < PROWS / 4; i += 2) {
      T l[2][NCH][V];
      int nj[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = base + w + 4 * (i + h);                  // (a row past M reads zeros, unused)
        nj[h] = c / CW + 1;                                    // chunks that hold columns <= c
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
          const int k0 = j * CW + lane * V;
          const bool ok = j < nj[h] && k0 < M && c < M;
          vload_b<T, V>(l[h][j], rL, ok ? (uint32_t)(((int64_t)c * M + k0) * sizeof(T)) : 0x80000000u);
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = base + w + 4 * (i + h);
        T acc[RB];
#pragma unroll
        for (int rr = 0; rr < RB; ++rr) acc[rr] = (T)0;
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
          if (j == nj[h] - 1) vmask<T, V>(l[h][j], j * CW + lane * V, c);
#pragma unroll
          for (int rr = 0; rr < RB; ++rr)
#pragma unroll
            for (int e = 0; e < V; ++e) acc[rr] = fma(l[h][j][e], wv[rr][j][e], acc[rr]);
        }
#pragma unroll
        for (int rr = 0; rr < RB; ++rr) {
          const T sm = wave_sum(acc[rr]);
          res[rr] = lane == i + h ? sm : res[rr];
        }
      }
    }
    const int c = base + w + 4 * lane;
    if (lane < PROWS / 4 && c < M) {
#pragma unroll
      for (int rr = 0; rr < RB; ++rr)
        if (rr < Rc) Z[d.c_off + (int64_t)(r0 + rc + rr) * M + c] = res[rr];
    }
  }
}

// grid (problems, row blocks of PROWS rows k of the gradient block).  Per row k: G[k][c] += sum_r P[r][k] W[r][c]
// for c <= k, the coefficients P[r][k] staged in LDS per block, W's rows in registers; elements above the
// diagonal are neither read nor written.
template <typename T, int NCH>
__global__ __launch_bounds__(PT) void pair_rank_kernel(const T* __restrict__ P, T* __restrict__ G,
                                                       const T* __restrict__ W, const nmgp_pair_desc* __restrict__ descs,
                                                       const int32_t* __restrict__ seg, int M) {
  constexpr int V = PairCfg<T>::V, RB = PairCfg<T>::RB, CW = 64 * V;
  __shared__ T sP[PROWS][RB];
  const nmgp_pair_desc d = descs[blockIdx.x];
  const int r0 = seg[d.seg], R = seg[d.seg + 1] - r0;
  const int base = blockIdx.y * PROWS;
  if (R <= 0 || base >= M) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  T* Gb = G + d.l_off + lane * V;
  const __amdgpu_buffer_rsrc_t rG = make_rsrc(G + d.l_off, (int64_t)M * M * (int64_t)sizeof(T));
  for (int rc = 0; rc < R; rc += RB) {
    const int Rc = min(RB, R - rc);
    __syncthreads();
    for (int idx = tid; idx < PROWS * RB; idx += PT) {
      const int rr = idx / PROWS, i = idx - rr * PROWS;
      sP[i][rr] = (rr < Rc && base + i < M) ? P[d.a_off + (int64_t)(r0 + rc + rr) * M + base + i] : (T)0;
    }
    T wv[RB][NCH][V];
    load_w<T, NCH>(wv, W, d.c_off, r0, rc, Rc, M, lane);
    __syncthreads();
    // two rows of this wave per iteration: both rows' gradient loads in flight together
    for (int i = w; i < PROWS; i += 8) {
      T g[2][NCH][V];
      int nj[2], kk[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        kk[h] = base + i + 4 * h;
        const int k = kk[h];
        nj[h] = k < M ? k / CW + 1 : 0;
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
          const int c0 = j * CW + lane * V;
          const bool ok = j < nj[h] && c0 < M;
          vload_b<T, V>(g[h][j], rG, ok ? (uint32_t)(((int64_t)k * M + c0) * sizeof(T)) : 0x80000000u);
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = kk[h];
        if (k >= M) continue;
        T coef[RB];
#pragma unroll
        for (int rr = 0; rr < RB; ++rr) coef[rr] = sP[i + 4 * h][rr];
        T* Gk = Gb + (int64_t)k * M;
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
          const int c0 = j * CW + lane * V;
          if (j < nj[h] && c0 < M) {
#pragma unroll
            for (int e = 0; e < V; ++e) {
              T sacc = g[h][j][e];
#pragma unroll
              for (int rr = 0; rr < RB; ++rr) sacc = fma(coef[rr], wv[rr][j][e], sacc);
              g[h][j][e] = sacc;
            }
            if (c0 + V - 1 <= k) {
              typedef T vec_t __attribute__((ext_vector_type(V)));
              vec_t x;
#pragma unroll
              for (int e = 0; e < V; ++e) x[e] = g[h][j][e];
              __builtin_nontemporal_store(x, (vec_t*)(Gk + j * CW));
            } else {
#pragma unroll
              for (int e = 0; e < V; ++e)
                if (c0 + e <= k) Gk[j * CW + e] = g[h][j][e];
            }
          }
        }
      }
    }
  }
}

// --------------------------------------------------------------------------------------------- mv
// mu-bar of the pair: C[c] += sum_r A[r][c] x[r] over the problem's rows r (A = P at a_off, x at l_off, C at c_off).
// One block per (problem, 1024 columns); thread t owns columns t + 256 q (coalesced single-element loads, no alignment
// requirement on the offsets); rows summed in order.  Replaces 16 64 x 64 GEMM tiles per pair with k ~ 4 (the grouped
// kernel's launch of 134 k mostly idle workgroups cost 3.3 ms per ECoG step).
template <typename T>
__global__ __launch_bounds__(256) void pair_mv_kernel(const T* __restrict__ A, const T* __restrict__ x,
                                                      T* __restrict__ C, const nmgp_pair_desc* __restrict__ descs,
                                                      const int32_t* __restrict__ seg, int M) {
  constexpr int Q = 4;
  const nmgp_pair_desc d = descs[blockIdx.x];
  const int r0 = seg[d.seg], R = seg[d.seg + 1] - r0;
  if (R <= 0) return;
  const int cb = blockIdx.y * 256 * Q + threadIdx.x;
  const T* a = A + d.a_off + (int64_t)r0 * M;
  const T* xv = x + d.l_off + r0;
  T acc[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) acc[q] = (T)0;
  for (int r = 0; r < R; ++r) {
    const T xr = xv[r];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int c = cb + 256 * q;
      if (c < M) acc[q] = fma(a[(int64_t)r * M + c], xr, acc[q]);
    }
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = cb + 256 * q;
    if (c < M) C[d.c_off + c] += acc[q];
  }
}

// ------------------------------------------------------------------------------------- pbar reduce
// One block per (row, 256 columns): row r of output i (i0 <= i < i1) gets P1[r] += Z_i[r], P0[r] += Z_0[r] + ... +
// Z_{i-1}[r], added in j order (deterministic).
template <typename T>
__global__ __launch_bounds__(256) void pair_pbar_reduce_kernel(const T* __restrict__ Z, int64_t sZ, T* __restrict__ P0,
                                                               T* __restrict__ P1, int64_t ldp,
                                                               const int32_t* __restrict__ seg, int D, int i0, int i1,
                                                               int M) {
  const int r = blockIdx.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (r >= seg[D] || c >= M) return;
  int i = 0;
  for (int q = 1; q < D; ++q) i = seg[q] <= r ? q : i;
  if (i < i0 || i >= i1) return;
  const T* z = Z + (int64_t)r * M + c;
  P1[(int64_t)r * ldp + c] += z[(int64_t)i * sZ];
  if (i > 0) {
    T acc = P0[(int64_t)r * ldp + c];
    for (int j = 0; j < i; ++j) acc += z[(int64_t)j * sZ];
    P0[(int64_t)r * ldp + c] = acc;
  }
}

template <typename T> static size_t quad_smem(int M) {
  return ((size_t)M * PairCfg<T>::RB + 4 * (size_t)PairCfg<T>::RB * 64 * PairCfg<T>::V) * sizeof(T);
}

template <typename T>
static int pair_check(const void* a, const void* b, const void* c, const nmgp_pair_desc* descs, int nprob,
                      const int32_t* seg, int M) {
  if (!a) return -1;
  if (!b) return -2;
  if (!c) return -3;
  if (nprob < 0) return -5;
  if (nprob > 0 && !descs) return -4;
  if (!seg) return -6;
  if (M <= 0 || M % PairCfg<T>::V != 0) return -7;
  return NMGP_OK;
}

template <typename T>
static int pair_quad(const T* A, const T* L, T* C, const nmgp_pair_desc* descs, int nprob, const int32_t* seg, int M,
                     hipStream_t s) {
  int rc = pair_check<T>(A, L, C, descs, nprob, seg, M);
  if (rc) return rc;
  if (quad_smem<T>(M) > 160 * 1024) return -7;
  if (nprob == 0) return NMGP_OK;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)pair_quad_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  const int ncb = (M + 64 * PairCfg<T>::V - 1) / (64 * PairCfg<T>::V);
  hipLaunchKernelGGL(pair_quad_kernel<T>, dim3((unsigned)nprob, (unsigned)ncb), dim3(PT), quad_smem<T>(M), s, A, L, C,
                     descs, seg, M);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

template <typename T>
static int pair_dot(const T* W, const T* L, T* Z, const nmgp_pair_desc* descs, int nprob, const int32_t* seg, int M,
                    hipStream_t s) {
  int rc = pair_check<T>(W, L, Z, descs, nprob, seg, M);
  if (rc) return rc;
  if (M > PMAXM) return -7;
  if (nprob == 0) return NMGP_OK;
  constexpr int NCH = PMAXM / (64 * PairCfg<T>::V);
  const dim3 grid((unsigned)nprob, (unsigned)((M + PROWS - 1) / PROWS));
  hipLaunchKernelGGL((pair_dot_kernel<T, NCH>), grid, dim3(PT), 0, s, W, L, Z, descs, seg, M);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

template <typename T>
static int pair_rank(const T* P, T* G, const T* W, const nmgp_pair_desc* descs, int nprob, const int32_t* seg, int M,
                     hipStream_t s) {
  int rc = pair_check<T>(P, G, W, descs, nprob, seg, M);
  if (rc) return rc;
  if (M > PMAXM) return -7;
  if (nprob == 0) return NMGP_OK;
  constexpr int NCH = PMAXM / (64 * PairCfg<T>::V);
  const dim3 grid((unsigned)nprob, (unsigned)((M + PROWS - 1) / PROWS));
  hipLaunchKernelGGL((pair_rank_kernel<T, NCH>), grid, dim3(PT), 0, s, P, G, W, descs, seg, M);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

template <typename T>
static int pair_mv(const T* A, const T* x, T* C, const nmgp_pair_desc* descs, int nprob, const int32_t* seg, int M,
                   hipStream_t s) {
  int rc = pair_check<T>(A, x, C, descs, nprob, seg, M);
  if (rc) return rc;
  if (nprob == 0) return NMGP_OK;
  const dim3 grid((unsigned)nprob, (unsigned)((M + 1023) / 1024));
  hipLaunchKernelGGL(pair_mv_kernel<T>, grid, dim3(256), 0, s, A, x, C, descs, seg, M);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

template <typename T>
static int pair_pbar_reduce(const T* Z, int64_t sZ, T* P0, T* P1, int64_t ldp, const int32_t* seg, int D, int i0,
                            int i1, int B, int M, hipStream_t s) {
  if (!Z) return -1;
  if (sZ < (int64_t)B * M) return -2;
  if (!P0) return -3;
  if (!P1) return -4;
  if (ldp < M) return -5;
  if (!seg) return -6;
  if (D <= 0) return -7;
  if (i0 < 0 || i1 > D || i0 > i1) return -8;
  if (B < 0) return -10;
  if (M <= 0) return -11;
  if (B == 0 || i0 == i1) return NMGP_OK;
  hipLaunchKernelGGL(pair_pbar_reduce_kernel<T>, dim3((unsigned)B, (unsigned)((M + 255) / 256)), dim3(256), 0, s, Z,
                     sZ, P0, P1, ldp, seg, D, i0, i1, M);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

}  // namespace nmgp

extern "C" {
int nmgp_pair_quad_f64(const double* A, const double* L, double* C, const nmgp_pair_desc* descs, int nprob,
                       const int32_t* seg, int M, hipStream_t s) {
  return nmgp::pair_quad<double>(A, L, C, descs, nprob, seg, M, s);
}
int nmgp_pair_quad_f32(const float* A, const float* L, float* C, const nmgp_pair_desc* descs, int nprob,
                       const int32_t* seg, int M, hipStream_t s) {
  return nmgp::pair_quad<float>(A, L, C, descs, nprob, seg, M, s);
}
int nmgp_pair_dot_f64(const double* W, const double* L, double* Z, const nmgp_pair_desc* descs, int nprob,
                      const int32_t* seg, int M, hipStream_t s) {
  return nmgp::pair_dot<double>(W, L, Z, descs, nprob, seg, M, s);
}
int nmgp_pair_dot_f32(const float* W, const float* L, float* Z, const nmgp_pair_desc* descs, int nprob,
                      const int32_t* seg, int M, hipStream_t s) {
  return nmgp::pair_dot<float>(W, L, Z, descs, nprob, seg, M, s);
}
int nmgp_pair_rank_f64(const double* P, double* G, const double* W, const nmgp_pair_desc* descs, int nprob,
                       const int32_t* seg, int M, hipStream_t s) {
  return nmgp::pair_rank<double>(P, G, W, descs, nprob, seg, M, s);
}
int nmgp_pair_rank_f32(const float* P, float* G, const float* W, const nmgp_pair_desc* descs, int nprob,
                       const int32_t* seg, int M, hipStream_t s) {
  return nmgp::pair_rank<float>(P, G, W, descs, nprob, seg, M, s);
}
int nmgp_pair_mv_f64(const double* A, const double* x, double* C, const nmgp_pair_desc* descs, int nprob,
                     const int32_t* seg, int M, hipStream_t s) {
  return nmgp::pair_mv<double>(A, x, C, descs, nprob, seg, M, s);
}
int nmgp_pair_mv_f32(const float* A, const float* x, float* C, const nmgp_pair_desc* descs, int nprob,
                     const int32_t* seg, int M, hipStream_t s) {
  return nmgp::pair_mv<float>(A, x, C, descs, nprob, seg, M, s);
}
int nmgp_pair_pbar_reduce_f64(const double* Z, int64_t sZ, double* P0, double* P1, int64_t ldp, const int32_t* seg,
                              int D, int i0, int i1, int B, int M, hipStream_t s) {
  return nmgp::pair_pbar_reduce<double>(Z, sZ, P0, P1, ldp, seg, D, i0, i1, B, M, s);
}
int nmgp_pair_pbar_reduce_f32(const float* Z, int64_t sZ, float* P0, float* P1, int64_t ldp, const int32_t* seg,
                              int D, int i0, int i1, int B, int M, hipStream_t s) {
  return nmgp::pair_pbar_reduce<float>(Z, sZ, P0, P1, ldp, seg, D, i0, i1, B, M, s);
}
}
