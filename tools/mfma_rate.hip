// Issue-rate probe of the f64/f32 MFMA shapes used by the GEMM and Cholesky kernels (standalone).
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_rate.hip -o tools/bin/mfma_rate && tools/bin/mfma_rate
// One wave per SIMD; cycles per MFMA with NACC independent accumulators (s_memtime, 100 MHz x 24).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void k64(double* out, long long* cyc, int iters) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int NACC>
__global__ void k32(float* out, long long* cyc, int iters) {
  f4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f4{0, 0, 0, 0};
  float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename T>
static void run(const char* name, void (*kern)(T*, long long*, int), int nacc, void* out, long long* cyc) {
  const int iters = 1000;
  hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, (T*)out, cyc, iters);
  hipDeviceSynchronize();
  long long c;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  // s_memtime counts at 100 MHz; shader clock ~2.4 GHz
  printf("%s nacc=%d: %.1f ns per MFMA (~%.0f shader cycles at 2.4 GHz)\n", name, nacc, c * 10.0 / (iters * nacc),
         c * 10.0 * 2.4 / (iters * nacc));
}

int main() {
  void* out;
  long long* cyc;
  hipMalloc(&out, 1 << 20);
  hipMalloc(&cyc, 1024);
  run("f64 16x16x4", k64<1>, 1, out, cyc);
  run("f64 16x16x4", k64<2>, 2, out, cyc);
  run("f64 16x16x4", k64<4>, 4, out, cyc);
  run("f64 16x16x4", k64<8>, 8, out, cyc);
  run("f32 16x16x4", k32<1>, 1, out, cyc);
  run("f32 16x16x4", k32<4>, 4, out, cyc);
  run("f32 16x16x4", k32<8>, 8, out, cyc);
  return 0;
}
