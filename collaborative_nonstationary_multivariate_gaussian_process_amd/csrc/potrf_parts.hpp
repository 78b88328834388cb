// Row-panel helpers of the blocked potrf's step / strip products (f32, k = 128 in one register-resident panel),
// shared by gemm_big.hip (potrf_step32_kernel, potrf_strip32_kernel) and chol.hip (potrf_fused_kernel).
// Lane (li, g) of a wave feeds 16-row blocks: it loads k = 32g .. 32g + 31 of its rows (eight 16-byte loads
// per row block) and MFMA step s consumes k-slot g <-> k = 32g + s for both operands.
#pragma once
#include "common.hpp"

namespace nmgp {

typedef unsigned int u32x4p __attribute__((ext_vector_type(4)));

constexpr int PS_NV = 32;

template <int RB>
__device__ __forceinline__ void ps_load_rows(float (&v)[RB][PS_NV], __amdgpu_buffer_rsrc_t r, int64_t row0,
                                             int64_t ld, int nrows, bool sc1) {
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
#pragma unroll
  for (int bi = 0; bi < RB; ++bi) {
    const int64_t row = row0 + 16 * bi + li;
    const uint32_t off = row < nrows ? (uint32_t)((row * ld + PS_NV * g) * 4) : 0x80000000u;
#pragma unroll
    for (int q = 0; q < PS_NV / 4; ++q) {
      const u32x4p u = sc1 ? __builtin_amdgcn_raw_buffer_load_b128(r, off, 16 * q, 16)
                           : __builtin_amdgcn_raw_buffer_load_b128(r, off, 16 * q, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[bi][4 * q + e] = __uint_as_float(u[e]);
    }
  }
}

template <int RA>
__device__ __forceinline__ void ps_mma(const float (&a)[RA][PS_NV], const float (&b)[2][PS_NV],
                                       f32x4 (&acc)[RA][2]) {
#pragma unroll
  for (int s = 0; s < PS_NV; ++s)
#pragma unroll
    for (int q = 0; q < 2 * RA; ++q)
      acc[q >> 1][q & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q >> 1][s], b[q & 1][s], acc[q >> 1][q & 1], 0, 0, 0);
}

// lookahead target of this workgroup's rows (prefetched: its other writers finished before the launch)
// (wc: this wave's 32-column group; sc1: bypass this CU's L1 -- C written by another workgroup of the launch)
template <int RB>
__device__ __forceinline__ void ps_load_c(__amdgpu_buffer_rsrc_t rC, int i0, int64_t lda, int m, int c1,
                                          f32x4 (&cv)[RB][2], uint32_t (&coff)[RB][2][4], int wc, bool sc1 = false) {
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
#pragma unroll
  for (int q = 0; q < 2 * RB; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 16 * (q >> 1) + 4 * g + r, j = 32 * wc + 16 * (q & 1) + li;
      coff[q >> 1][q & 1][r] = (i < m && j < c1) ? (uint32_t)(((int64_t)i * lda + j) * 4) : 0x80000000u;
      cv[q >> 1][q & 1][r] = __builtin_bit_cast(
          float, sc1 ? __builtin_amdgcn_raw_buffer_load_b32(rC, coff[q >> 1][q & 1][r], 0, 16)
                     : __builtin_amdgcn_raw_buffer_load_b32(rC, coff[q >> 1][q & 1][r], 0, 0));
    }
}

template <int RB>
__device__ __forceinline__ void ps_store_c(__amdgpu_buffer_rsrc_t rC, const f32x4 (&cv)[RB][2],
                                           const uint32_t (&coff)[RB][2][4], const f32x4 (&acc)[RB][2]) {
#pragma unroll
  for (int q = 0; q < 2 * RB; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (coff[q >> 1][q & 1][r] != 0x80000000u)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(cv[q >> 1][q & 1][r] - acc[q >> 1][q & 1][r]), rC,
                                              coff[q >> 1][q & 1][r], 0, 0);
}

}  // namespace nmgp
