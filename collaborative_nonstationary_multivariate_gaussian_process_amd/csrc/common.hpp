// Shared device helpers for libnmgp_hip.so (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nmgp_hip.h"

#define NMGP_CHECK_LAUNCH()                                      \
  do {                                                           \
    if (hipGetLastError() != hipSuccess) return NMGP_ERR_LAUNCH; \
  } while (0)

namespace nmgp {

constexpr int kWave = 64;

// Global-address-space pointer.  Pointers that arrive inside descriptor structs are generic, and
// generic (flat) loads count against lgkmcnt as well as vmcnt: an LDS wait would then also wait
// for every outstanding prefetch.  Casting to addrspace(1) gives global_load/store instead.
template <typename T> using GPtr = __attribute__((address_space(1))) T*;

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// 16x16x4 MFMA, one A and one B element per lane:
//   A operand lane l : A[i = l & 15][k = l >> 4]      B operand lane l : B[k = l >> 4][j = l & 15]
//   C/D register r   : col = l & 15, row = row(l, r)  (f64 and f32 differ, MI355X guide §3)
template <typename T> struct Mfma;
template <> struct Mfma<double> {
  using acc_t = f64x4;
  __device__ static inline acc_t mma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  __device__ static inline int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};
template <> struct Mfma<float> {
  using acc_t = f32x4;
  __device__ static inline acc_t mma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  __device__ static inline int row(int lane, int r) { return ((lane >> 4) << 2) + r; }
};

// Raw buffer resources: loads past num_records return 0 (checked per dword), so a buffer load is a
// bounds-checked load without a branch.  aux 16 = sc1 (bypass this CU's L1 on loads; write through
// on stores) for data handed between workgroups inside a launch.
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

template <typename T> __device__ inline T bload_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off_bytes);
template <> __device__ inline double bload_sc1<double>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 16));
}
template <> __device__ inline float bload_sc1<float>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 16));
}

template <typename T> __device__ inline void bstore_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off_bytes, T v);
template <> __device__ inline void bstore_sc1<double>(__amdgpu_buffer_rsrc_t r, uint32_t off, double v) {
  typedef unsigned int u32x2_ __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_, v), r, off, 0, 16);
}
template <> __device__ inline void bstore_sc1<float>(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, off, 0, 16);
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS traffic (lgkmcnt) but not for
// its outstanding global stores, which __syncthreads() would drain (vmcnt(0)) at every barrier.
// Only valid where waves exchange data exclusively through LDS.
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// single-problem (optionally batched) GEMM launch, defined in gemm.hip
template <typename T> int gemm_single(const nmgp_gemm_desc& d, hipStream_t s);

template <typename T> __device__ inline T shfl(T v, int src) { return __shfl(v, src, 64); }

template <typename T> __device__ inline T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide deterministic sum (blockDim.x multiple of 64, <= 1024). Result valid in all threads.
template <typename T> __device__ inline T block_sum(T v, T* scratch /* >= 16 */) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  T s = 0;
  for (int i = 0; i < nw; ++i) s += scratch[i];
  __syncthreads();
  return s;
}

template <typename T> __device__ inline T dexp(T x) { return exp(x); }
template <> __device__ inline float dexp<float>(float x) { return expf(x); }
template <typename T> __device__ inline T dlog(T x) { return log(x); }
template <> __device__ inline float dlog<float>(float x) { return logf(x); }
template <typename T> __device__ inline T dsqrt(T x) { return sqrt(x); }
template <> __device__ inline float dsqrt<float>(float x) { return sqrtf(x); }

}  // namespace nmgp
