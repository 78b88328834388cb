// Probe (standalone; not in the library): an 8-wave variant of gemm_big_kernel's 128x128x32 tile against the
// library's 4-wave kernel on the batched ECoG SYRK (Sigma_f = L_f L_f^T, A_LOWER | B_UPPER | OUT_LOWER, both
// operands k-contiguous, per-problem offsets).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I<pkg>/csrc -Iinclude tools/big8_probe.hip -o tools/big8_probe.x
//   ./big8_probe.x [nf=512] [M=1024]
// The 8-wave tile: 512 threads, waves 2 x 4, each 64 x 32 (two 32x32x2 f32 accumulators), the same LDS images and
// k permutation.  Two workgroups per CU hold 4 waves per SIMD (the 4-wave kernel: 2), so a CU whose other
// workgroup is in its prologue / epilogue still has two waves per SIMD issuing MFMAs.  Prints the time of both
// kernels and the max |difference| of their outputs.
#include "gemm_big.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace nmgp {

template <int NT>
__device__ __forceinline__ void b8_mainloop(const float* Ab, const float* Bb, int64_t lda, int64_t ldb, int m, int n,
                                            int K, float* smem, int i0, int j0, int kend, int kt0, int kt1,
                                            f32x16 (&acc)[2]) {
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 2, wc = w & 3;
  const __amdgpu_buffer_rsrc_t rA = make_rsrc(Ab, ((int64_t)(m - 1) * lda + K) * 4);
  const __amdgpu_buffer_rsrc_t rB = make_rsrc(Bb, ((int64_t)(n - 1) * ldb + K) * 4);
  const int lr = t >> 3, lk = (t & 7) * 4;   // rows lr, lr + 64
  float4 ra[2], rb[2];
  auto load = [&](int kt) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      ra[q] = ld4<0>(rA, (uint32_t)(((int64_t)(i0 + lr + 64 * q) * lda + kt + lk) * 4));
      rb[q] = ld4<0>(rB, (uint32_t)(((int64_t)(j0 + lr + 64 * q) * ldb + kt + lk) * 4));
    }
  };
  auto store_lds = [&](float* st, int kt) {
    const bool need = (kt + BBK > kend) || (kt + BBK - 1 > i0) || (kt + BBK - 1 > j0);
    if (need) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        float* a = (float*)&ra[q];
        float* b = (float*)&rb[q];
        const int i = i0 + lr + 64 * q, j = j0 + lr + 64 * q;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int kk = kt + lk + e;
          a[e] = keep_if(a[e], kk < kend && kk <= i);
          b[e] = keep_if(b[e], kk < kend && kk <= j);
        }
      }
    }
    float* As = st;
    float* Bs = st + BBM * BP;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      *(float4*)&As[(lr + 64 * q) * BP + lk] = ra[q];
      *(float4*)&Bs[(lr + 64 * q) * BP + lk] = rb[q];
    }
  };
  if (kt0 < kt1) {
    load(kt0);
    store_lds(smem, kt0);
    __syncthreads();
    int st = 0;
    const int ko = 16 * (lane >> 5), rl = lane & 31;
    for (int kt = kt0; kt < kt1; kt += BBK) {
      const bool more = kt + BBK < kt1;
      if (more) load(kt + BBK);
      const float* As = smem + st * BSTAGE;
      const float* Bs = As + BBM * BP;
      float4 fa[2][4], fb[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int h = 0; h < 2; ++h) fa[h][c] = *(const float4*)&As[(64 * wr + 32 * h + rl) * BP + ko + 4 * c];
        fb[c] = *(const float4*)&Bs[(32 * wc + rl) * BP + ko + 4 * c];
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const float a0 = ((const float*)&fa[0][s >> 2])[s & 3], a1 = ((const float*)&fa[1][s >> 2])[s & 3];
        const float b0 = ((const float*)&fb[s >> 2])[s & 3];
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1], 0, 0, 0);
      }
      if (more) store_lds(smem + (st ^ 1) * BSTAGE, kt + BBK);
      lds_barrier();
      st ^= 1;
    }
  }
}

__global__ __launch_bounds__(512, 2) void big8_syrk_kernel(const float* __restrict__ L, float* C, const int64_t* offs,
                                                           int M, int tiles, float diag_add) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int bid = (int)(((int64_t)blockIdx.x + 9LL * blockIdx.y) % gridDim.x);
  const int64_t bat = blockIdx.y;
  const int64_t off = uniform64(offs[bat]);
  const float* Lb = L + off;
  float* Cb = C + off;
  const int T = M / BBN;
  int tm = (int)((sqrtf(8.0f * (float)bid + 1.0f) - 1.0f) * 0.5f);
  while ((tm + 1) * (tm + 2) / 2 <= bid) ++tm;
  while (tm * (tm + 1) / 2 > bid) --tm;
  const int tn = bid - tm * (tm + 1) / 2;
  const int i0 = tm * BBM, j0 = tn * BBN;
  const int kend = min(M, min(i0 + BBM, j0 + BBN));
  f32x16 acc[2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.0f;
  b8_mainloop<512>(Lb, Lb, M, M, M, M, M, smem, i0, j0, kend, 0, kend, acc);
  // row-vector epilogue through LDS (the main loop ended on a barrier)
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 2, wc = w & 3;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      smem[(64 * wr + 32 * a + 4 * (lane >> 5) + (r & 3) + 8 * (r >> 2)) * BCP + 32 * wc + (lane & 31)] = acc[a][r];
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rC = make_rsrc(Cb, (int64_t)M * M * 4);
  const int c4 = (t & 31) * 4, rb = t >> 5;
  const int j = j0 + c4;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int row = rb + 16 * q, i = i0 + row;
    if (j > i) continue;
    const float4 av = *(const float4*)&smem[row * BCP + c4];
    float x[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = ((const float*)&av)[e] + (i == j + e ? diag_add : 0.0f);
    const uint32_t o = (uint32_t)(((int64_t)i * M + j) * 4);
    if (j + 3 <= i) {
      u32x4g v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = __float_as_uint(x[e]);
      __builtin_amdgcn_raw_buffer_store_b128(v, rC, o, 0, 0);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x[e]), rC, j + e <= i ? o + 4 * e : 0x80000000u, 0, 0);
    }
  }
}

}  // namespace nmgp

int main(int argc, char** argv) {
  const int nf = argc > 1 ? atoi(argv[1]) : 512, M = argc > 2 ? atoi(argv[2]) : 1024;
  const int64_t MM = (int64_t)M * M;
  std::vector<float> h(MM);
  srand(1);
  for (int64_t i = 0; i < MM; ++i) h[i] = (float)(rand() % 2001 - 1000) * 1e-4f;
  float *L, *C1, *C2;
  hipMalloc(&L, nf * MM * 4);
  hipMalloc(&C1, nf * MM * 4);
  hipMalloc(&C2, nf * MM * 4);
  for (int f = 0; f < nf; ++f) hipMemcpy(L + f * MM, h.data(), MM * 4, hipMemcpyHostToDevice);
  hipMemset(C1, 0, nf * MM * 4);
  hipMemset(C2, 0, nf * MM * 4);
  std::vector<int64_t> off(nf);
  for (int f = 0; f < nf; ++f) off[f] = f * MM;
  int64_t* doff;
  hipMalloc(&doff, nf * 8);
  hipMemcpy(doff, off.data(), nf * 8, hipMemcpyHostToDevice);
  const int T = M / 128, tiles = T * (T + 1) / 2;
  const size_t lds = 2 * nmgp::BSTAGE * sizeof(float);
  hipFuncSetAttribute((const void*)nmgp::big8_syrk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  auto lib = [&]() {
    return nmgp_gemm_big_offsets_f32(L, M, L, M, 1, C1, M, 1, M, M, M, NMGP_A_LOWER | NMGP_B_UPPER | NMGP_OUT_LOWER,
                                     1.0, 0.0, 1e-4, doff, doff, doff, nf, nullptr, 0);
  };
  auto b8 = [&]() {
    hipLaunchKernelGGL(nmgp::big8_syrk_kernel, dim3(tiles, nf), dim3(512), lds, 0, L, C2, doff, M, tiles, 1e-4f);
    return (int)hipGetLastError();
  };
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double flop = 2.0 * nf * (double)M * M * M / 3.0;   // lower output of L L^T, triangular L: ~M^3/6 MAC
  for (int rep = 0; rep < 2; ++rep) {
    for (int v = 0; v < 2; ++v) {
      int rc = v ? b8() : lib();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) rc |= v ? b8() : lib();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= 5;
      printf("{\"kernel\": \"%s\", \"nf\": %d, \"M\": %d, \"rc\": %d, \"ms\": %.3f, \"tflops\": %.2f}\n",
             v ? "big8 (8 waves, 64x32 per wave)" : "gemm_big_kernel (4 waves, 64x64 per wave)", nf, M, rc, ms,
             flop / ms / 1e9);
    }
  }
  std::vector<float> a(MM), b(MM);
  hipMemcpy(a.data(), C1 + (nf - 1) * MM, MM * 4, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), C2 + (nf - 1) * MM, MM * 4, hipMemcpyDeviceToHost);
  double md = 0, mx = 0;
  for (int i = 0; i < M; ++i)
    for (int j = 0; j <= i; ++j) {
      md = std::max(md, (double)std::fabs(a[i * M + j] - b[i * M + j]));
      mx = std::max(mx, (double)std::fabs(a[i * M + j]));
    }
  printf("{\"max_abs_diff\": %.3e, \"max_abs\": %.3e}\n", md, mx);
  return 0;
}
