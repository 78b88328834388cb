// Cycles per k-tile of the GEMM's LDS->MFMA inner step alone (standalone probe).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -I<pkg>/csrc -Iinclude \
//         tools/mma_tile_rate.hip -o tools/bin/mma_tile_rate
#include "gemm.hip"

#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void k(double* out, long long* cyc, int iters) {
  __shared__ double S[2 * nmgp::GBK * nmgp::LP];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  for (int i = t; i < 2 * nmgp::GBK * nmgp::LP; i += 256) S[i] = 1e-3 * (i % 97);
  __syncthreads();
  nmgp::f64x4 c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {
      nmgp::mma_tile<double, false, false>(S, S + nmgp::GBK * nmgp::LP, lane, wr, wc, c00, c01, c10, c11);
    } else {
      // same MFMA stream, operands already in registers
      const double a0 = S[lane], a1 = S[lane + 64], b0 = S[lane + 128], b1 = S[lane + 192];
#pragma unroll
      for (int s = 0; s < 8; ++s) nmgp::mma_step(a0 + s, a1, b0, b1, c00, c01, c10, c11);
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * 256 + t] = c00[0] + c01[1] + c10[2] + c11[3];
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* out;
  long long* cyc;
  hipMalloc(&out, 1 << 22);
  hipMalloc(&cyc, 8192);
  const int iters = 200;
  for (int mode = 0; mode < 2; ++mode) {
    for (int nb : {1, 256}) {
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(nb), dim3(256), 0, 0, out, cyc, iters);
      else hipLaunchKernelGGL(k<1>, dim3(nb), dim3(256), 0, 0, out, cyc, iters);
      hipDeviceSynchronize();
      long long c;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      printf("%s, %3d WGs: %.0f cycles per k-tile (32 MFMA; ideal 2048)\n",
             mode == 0 ? "LDS fragments (mma_tile)" : "register operands     ", nb, (double)c / iters);
    }
  }
  return 0;
}
