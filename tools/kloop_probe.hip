// Cycles per 64x64x32 f64 k-tile of the GEMM main loop with 4 waves (one per SIMD, each wave all 8
// k-steps of its 32x32 quadrant) vs 8 waves (two per SIMD, the k-steps of a tile split between the
// two waves of a quadrant) -- standalone probe for the gemm_kernel design (not in the library).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -I<pkg>/csrc \
//         tools/kloop_probe.hip -o tools/bin/kloop_probe
// A: m x K row-major (k contiguous), B: K x n row-major; the tile loop mirrors mainloop_fast.
#include "common.hpp"

#include <cstdio>
#include <vector>

using namespace nmgp;
constexpr int BM = 64, BK = 32, PL = 65, ST = 2 * BK * PL;
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

__device__ inline double ue(u4 u, int v) {
  const unsigned lo = v ? u[2] : u[0], hi = v ? u[3] : u[1];
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

template <int KH, int MODE = 0>
__global__ __launch_bounds__(256 * KH) void kloop(const double* A, const double* B, double* C, int K, int lda,
                                                   int ldb, long long* cyc) {
  __shared__ double S[2 * ST];
  constexpr int NU = 4 / KH;  // 16-B units per thread and operand
  constexpr int KS = 8 / KH;  // k-steps (of 4) per wave per tile
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, q = w & 3, h = w >> 2, wr = q >> 1, wc = q & 1;
  const int i0 = blockIdx.x * BM;
  const __amdgpu_buffer_rsrc_t rA = make_rsrc(A + (int64_t)i0 * lda, (int64_t)BM * lda * 8);
  const __amdgpu_buffer_rsrc_t rB = make_rsrc(B, (int64_t)K * ldb * 8);
  // A unit e: row (t / 16) + e * (256 * KH / 16), k pair (t % 16) * 2 ; B unit e: k (t / 32) + e * (8 * KH), cols (t % 32) * 2
  const int a_r = t >> 4, a_k = (t & 15) * 2, a_rs = 16 * KH;
  const int b_k = t >> 5, b_c = (t & 31) * 2, b_ks = 8 * KH;
  uint32_t oA = (uint32_t)((a_r * lda + a_k) * 8), oB = (uint32_t)((b_k * ldb + b_c) * 8);
  const uint32_t sA = (uint32_t)(a_rs * lda * 8), sB = (uint32_t)(b_ks * ldb * 8);
  const uint32_t stepA = BK * 8, stepB = (uint32_t)(BK * ldb * 8);
  u4 ra[NU], rb[NU];
  auto issue = [&](int e) {
    if (MODE & 1) return;
    ra[e] = __builtin_amdgcn_raw_buffer_load_b128(rA, oA + e * sA, 0, 0);
    rb[e] = __builtin_amdgcn_raw_buffer_load_b128(rB, oB + e * sB, 0, 0);
  };
  auto put = [&](double* N, int s) {  // element s = unit s/2, half s%2
    if (MODE & 2) return;
    const int e = s >> 1, v = s & 1;
    N[(a_k + v) * PL + a_r + e * a_rs] = ue(ra[e], v);
    N[BK * PL + (b_k + e * b_ks) * PL + b_c + v] = ue(rb[e], v);
  };
  f64x4 c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;
  auto mma = [&](const double* As, auto&& stage) {
    const double* pa = As + (h * KS * 4 + (lane >> 4)) * PL + wr * 32 + (lane & 15);
    const double* pb = As + BK * PL + (h * KS * 4 + (lane >> 4)) * PL + wc * 32 + (lane & 15);
    double f[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int o = u * 4 * PL;
      f[u][0] = pa[o]; f[u][1] = pa[o + 16]; f[u][2] = pb[o]; f[u][3] = pb[o + 16];
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int u = s & 1;
      const double a0 = f[u][0], a1 = f[u][1], b0 = f[u][2], b1 = f[u][3];
      if (s + 2 < KS) {
        const int o = (s + 2) * 4 * PL;
        f[u][0] = pa[o]; f[u][1] = pa[o + 16]; f[u][2] = pb[o]; f[u][3] = pb[o + 16];
      }
      c00 = Mfma<double>::mma(a0, b0, c00);
      c01 = Mfma<double>::mma(a0, b1, c01);
      c10 = Mfma<double>::mma(a1, b0, c10);
      c11 = Mfma<double>::mma(a1, b1, c11);
      stage(s);
    }
  };
  const long long t0 = __builtin_readcyclecounter();
#pragma unroll
  for (int e = 0; e < NU; ++e) issue(e);
  oA += stepA; oB += stepB;
#pragma unroll
  for (int s = 0; s < 2 * NU; ++s) put(S, s);
#pragma unroll
  for (int e = 0; e < NU; ++e) issue(e);
  oA += stepA; oB += stepB;
  lds_barrier();
  int cur = 0;
  const int nt = K / BK;
  for (int kt = 0; kt + 1 < nt; ++kt) {
    double* N = S + (cur ^ 1) * ST;
    mma(S + cur * ST, [&](int s) {
      // 2*NU elements to stage over KS k-steps
      if (KH == 1) { put(N, s); if (s & 1) issue(s >> 1); }
      else { put(N, s); if (s & 1) issue(s >> 1); }
    });
    oA += stepA; oB += stepB;
    if (!(MODE & 4)) lds_barrier();
    cur ^= 1;
  }
  mma(S + cur * ST, [](int) {});
  const long long t1 = __builtin_readcyclecounter();
  // combine the k halves (KH == 2) through LDS, then store
  if (KH == 2) {
    __syncthreads();
    double* R = S;
    if (h == 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        R[(q * 16 + 0 * 4 + r) * 64 + lane] = c00[r];
        R[(q * 16 + 1 * 4 + r) * 64 + lane] = c01[r];
        R[(q * 16 + 2 * 4 + r) * 64 + lane] = c10[r];
        R[(q * 16 + 3 * 4 + r) * 64 + lane] = c11[r];
      }
    }
    __syncthreads();
    if (h == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        c00[r] += R[(q * 16 + 0 * 4 + r) * 64 + lane];
        c01[r] += R[(q * 16 + 1 * 4 + r) * 64 + lane];
        c10[r] += R[(q * 16 + 2 * 4 + r) * 64 + lane];
        c11[r] += R[(q * 16 + 3 * 4 + r) * 64 + lane];
      }
    }
  }
  if (h == 0) {
    double* Cb = C + (int64_t)blockIdx.x * 4096 + q * 1024;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      Cb[r * 64 + lane] = c00[r];
      Cb[256 + r * 64 + lane] = c01[r];
      Cb[512 + r * 64 + lane] = c10[r];
      Cb[768 + r * 64 + lane] = c11[r];
    }
  }
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int K = 4096, n = 64;
  const int maxwg = 512;
  double *A, *B, *C;
  long long* cyc;
  hipMalloc(&A, (size_t)maxwg * 64 * K * 8);
  hipMalloc(&B, (size_t)K * n * 8);
  hipMalloc(&C, (size_t)maxwg * 4096 * 8);
  hipMalloc(&cyc, maxwg * 8);
  hipMemset(A, 0, (size_t)maxwg * 64 * K * 8);
  hipMemset(B, 0, (size_t)K * n * 8);
  for (int mode : {1, 2, 4, 3, 7}) {
    for (int nb : {1, 256}) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        switch (mode) {
          case 1: hipLaunchKernelGGL((kloop<1, 1>), dim3(nb), dim3(256), 0, 0, A, B, C, K, K, n, cyc); break;
          case 2: hipLaunchKernelGGL((kloop<1, 2>), dim3(nb), dim3(256), 0, 0, A, B, C, K, K, n, cyc); break;
          case 4: hipLaunchKernelGGL((kloop<1, 4>), dim3(nb), dim3(256), 0, 0, A, B, C, K, K, n, cyc); break;
          case 3: hipLaunchKernelGGL((kloop<1, 3>), dim3(nb), dim3(256), 0, 0, A, B, C, K, K, n, cyc); break;
          default: hipLaunchKernelGGL((kloop<1, 7>), dim3(nb), dim3(256), 0, 0, A, B, C, K, K, n, cyc); break;
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
      }
      std::vector<long long> c(nb);
      hipMemcpy(c.data(), cyc, nb * 8, hipMemcpyDeviceToHost);
      double sum = 0;
      for (long long v : c) sum += v;
      printf("4 waves, mode %d (1 no VMEM, 2 no LDS stores, 4 no barrier), %3d WGs: %.0f cycles per k-tile\n", mode, nb,
             sum / nb / (K / BK));
    }
  }
  for (int kh : {1, 2}) {
    for (int nb : {1, 128, 256, 512}) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        if (kh == 1) hipLaunchKernelGGL(kloop<1>, dim3(nb), dim3(256), 0, 0, A, B, C, K, K, n, cyc);
        else hipLaunchKernelGGL(kloop<2>, dim3(nb), dim3(512), 0, 0, A, B, C, K, K, n, cyc);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<long long> c(nb);
        hipMemcpy(c.data(), cyc, nb * 8, hipMemcpyDeviceToHost);
        double mx = 0, sum = 0;
        for (long long v : c) { mx = v > mx ? v : mx; sum += v; }
        if (rep == 1)
          printf("waves %d, %3d WGs: %.0f cycles per k-tile (mean; max %.0f; ideal 2048), kernel %.1f us, %.1f TF/s\n",
                 4 * kh, nb, sum / nb / (K / BK), mx / (K / BK), ms * 1000,
                 2.0 * 64 * 64 * (double)K * nb / (ms * 1e-3) / 1e12);
      }
    }
  }
  return 0;
}
