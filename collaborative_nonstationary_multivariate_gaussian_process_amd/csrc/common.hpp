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
// A value every lane of the wave holds (e.g. loaded from a per-problem table at a wave-uniform index) moved to
// SGPRs: a buffer resource built from a VGPR base makes the compiler wrap every buffer load in a waterfall loop
// (readfirstlane, compare, exec save / restore, and a vmcnt(0) wait per load where the loop carries its result).
__device__ inline int64_t uniform64(int64_t v) {
  const uint64_t u = (uint64_t)v;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ inline int uniform32(int v) { return __builtin_amdgcn_readfirstlane(v); }
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

// Wave-wide sum on DPP (register-to-register lane moves; no LDS round trip as __shfl_xor's
// ds_bpermute has): quad swaps, half-row and row mirrors, then row_bcast:15 / row_bcast:31 carry
// the row sums into row 3; lane 63 holds the total, read back to every lane.  Fixed pattern:
// deterministic.  Disabled rows of the broadcast steps add the `old` operand, 0.
template <int CTRL, int ROWS> __device__ inline int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS> __device__ inline float dpp_t(float v) {
  return __builtin_bit_cast(float, dpp_i<CTRL, ROWS>(__builtin_bit_cast(int, v)));
}
template <int CTRL, int ROWS> __device__ inline double dpp_t(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = dpp_i<CTRL, ROWS>((int)(b & 0xffffffffLL)), hi = dpp_i<CTRL, ROWS>((int)(b >> 32));
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
template <typename T> __device__ inline T wave_total(T v);
template <> __device__ inline float wave_total<float>(float v) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
template <> __device__ inline double wave_total<double>(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), 63);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <typename T> __device__ inline T wave_sum(T v) {
  v += dpp_t<0xB1, 0xf>(v);    // quad_perm [1,0,3,2]
  v += dpp_t<0x4E, 0xf>(v);    // quad_perm [2,3,0,1]
  v += dpp_t<0x141, 0xf>(v);   // row_half_mirror
  v += dpp_t<0x140, 0xf>(v);   // row_mirror: every lane holds its 16-lane row sum
  v += dpp_t<0x142, 0xa>(v);   // row_bcast:15 into rows 1, 3
  v += dpp_t<0x143, 0xc>(v);   // row_bcast:31 into rows 2, 3
  return wave_total(v);
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

// K block-wide deterministic sums in one pass (two barriers instead of 3K); scratch >= 16*K.
template <typename T, int K> __device__ inline void block_sum_n(T (&v)[K], T* scratch) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = wave_sum(v[k]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) scratch[k * 16 + w] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    T s = 0;
    for (int i = 0; i < nw; ++i) s += scratch[k * 16 + i];
    v[k] = s;
  }
  __syncthreads();
}

// The same K sums with the result valid in thread 0 only (the caller's epilogue runs there): the
// cross-wave step is one wave, lane k summing value k's 16 wave partials, instead of every thread of
// the block re-reading all K x 16 partials from LDS (15 us of the finalize kernel at K = 20).
template <typename T, int K> __device__ inline void block_sum_n0(T (&v)[K], T* scratch) {
  static_assert(K <= 64, "one lane per value");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = wave_sum(v[k]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) scratch[k * 16 + w] = v[k];
  }
  __syncthreads();
  if (w == 0) {
    T s = 0;
    if (lane < K)
      for (int i = 0; i < nw; ++i) s += scratch[lane * 16 + i];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = shfl(s, k);
  }
  __syncthreads();
}

// v if ok else +0, bitwise: no load is sunk into a branch (loads of a batch stay in flight together)
// and a NaN in a masked-off element cannot leak through a multiply.
template <typename T> __device__ inline T keep_if(T v, bool ok);
template <> __device__ inline double keep_if<double>(double v, bool ok) {
  return __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, v) & (ok ? ~0ull : 0ull));
}
template <> __device__ inline float keep_if<float>(float v, bool ok) {
  return __builtin_bit_cast(float, __builtin_bit_cast(unsigned int, v) & (ok ? ~0u : 0u));
}

// Device status word of this translation unit: a bounded inter-workgroup spin that gives up sets its
// bit (NMGP_STATUS_* in nmgp_hip.h) instead of failing silently.  Each .hip file has its own copy
// (internal linkage, no relocatable device code); nmgp_device_status() ORs and clears them all.
static __device__ unsigned int g_nmgp_status;
__device__ inline void spin_gave_up(unsigned int bit) {
  __hip_atomic_fetch_or(&g_nmgp_status, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Host accessor of the TU's status word (read, then optionally clear).  Synchronous: called only at
// the caller's existing sync points.
#define NMGP_TU_STATUS_ACCESSOR(name)                                                        \
  int nmgp_tu_status_##name(unsigned int* v, int clear) {                                  \
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(nmgp::g_nmgp_status), sizeof(unsigned int), 0,    \
                            hipMemcpyDeviceToHost) != hipSuccess)                           \
      return NMGP_ERR_LAUNCH;                                                               \
    if (clear && *v) {                                                                      \
      const unsigned int z = 0;                                                             \
      if (hipMemcpyToSymbol(HIP_SYMBOL(nmgp::g_nmgp_status), &z, sizeof(unsigned int), 0,   \
                            hipMemcpyHostToDevice) != hipSuccess)                           \
        return NMGP_ERR_LAUNCH;                                                             \
    }                                                                                       \
    return NMGP_OK;                                                                         \
  }

template <typename T> __device__ inline T dexp(T x) { return exp(x); }
template <> __device__ inline float dexp<float>(float x) { return expf(x); }
template <typename T> __device__ inline T dlog(T x) { return log(x); }
template <> __device__ inline float dlog<float>(float x) { return logf(x); }
template <typename T> __device__ inline T dsqrt(T x) { return sqrt(x); }
template <> __device__ inline float dsqrt<float>(float x) { return sqrtf(x); }

}  // namespace nmgp
