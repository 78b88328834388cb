// Probe (standalone; not in the library): a PERSISTENT 8-wave gemm_big tile loop that prefetches the next tile's
// first k-tile into registers before the current tile's epilogue, so the prologue's HBM round trip hides under the
// epilogue (tools/big_trace_batch.hip: prologue 5-11 us, epilogue 9-13 us of a 40-65 us tile in the batched ECoG
// products).  Workload: the batched SYRK Sigma_f = L_f L_f^T (A_LOWER | B_UPPER | OUT_LOWER, k-contiguous, per-problem
// offsets), against the library's launch (nmgp_gemm_big_offsets_f32, one workgroup per tile).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I<pkg>/csrc -Iinclude tools/big8p_probe.hip -o tools/big8p_probe.x
//   ./big8p_probe.x [nf=512] [M=1024]
#include "gemm_big.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace nmgp {

struct B8Pre {
  float4 ra[2], rb[2];
};

__device__ __forceinline__ void b8p_load(B8Pre& p, __amdgpu_buffer_rsrc_t r, int64_t ld, int i0, int j0, int kt) {
  const int t = threadIdx.x, lr = t >> 3, lk = (t & 7) * 4;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    p.ra[q] = ld4<0>(r, (uint32_t)(((int64_t)(i0 + lr + 64 * q) * ld + kt + lk) * 4));
    p.rb[q] = ld4<0>(r, (uint32_t)(((int64_t)(j0 + lr + 64 * q) * ld + kt + lk) * 4));
  }
}

__device__ __forceinline__ void b8p_store(float* st, B8Pre& p, int i0, int j0, int kt, int kend) {
  const int t = threadIdx.x, lr = t >> 3, lk = (t & 7) * 4;
  if ((kt + BBK > kend) || (kt + BBK - 1 > i0) || (kt + BBK - 1 > j0)) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float* a = (float*)&p.ra[q];
      float* b = (float*)&p.rb[q];
      const int i = i0 + lr + 64 * q, j = j0 + lr + 64 * q;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kk = kt + lk + e;
        a[e] = keep_if(a[e], kk < kend && kk <= i);
        b[e] = keep_if(b[e], kk < kend && kk <= j);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    *(float4*)&st[(lr + 64 * q) * BP + lk] = p.ra[q];
    *(float4*)&st[BBM * BP + (lr + 64 * q) * BP + lk] = p.rb[q];
  }
}

__device__ __forceinline__ void b8p_coords(int it, int nf, int& b, int& i0, int& j0, int& kend, int M) {
  b = it % nf;                       // consecutive work items walk the problems (spreads one problem's tiles)
  const int tile = it / nf;
  int tm = (int)((sqrtf(8.0f * (float)tile + 1.0f) - 1.0f) * 0.5f);
  while ((tm + 1) * (tm + 2) / 2 <= tile) ++tm;
  while (tm * (tm + 1) / 2 > tile) --tm;
  const int tn = tile - tm * (tm + 1) / 2;
  i0 = tm * BBM;
  j0 = tn * BBN;
  kend = min(M, min(i0 + BBM, j0 + BBN));
}

template <bool PREFETCH>
__global__ __launch_bounds__(512, 4) void big8p_syrk_kernel(const float* __restrict__ L, float* C,
                                                            const int64_t* offs, int M, int nf, int total,
                                                            float diag_add) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int ko = 16 * (lane >> 5), rl = lane & 31;
  const int64_t span = ((int64_t)(M - 1) * M + M) * 4;
  int it = blockIdx.x;
  if (it >= total) return;
  int b, i0, j0, kend;
  b8p_coords(it, nf, b, i0, j0, kend, M);
  B8Pre pre;
  {
    const __amdgpu_buffer_rsrc_t r = make_rsrc(L + uniform64(offs[b]), span);
    b8p_load(pre, r, M, i0, j0, 0);
  }
  while (true) {
    const float* Lb = L + uniform64(offs[b]);
    float* Cb = C + uniform64(offs[b]);
    const __amdgpu_buffer_rsrc_t rL = make_rsrc(Lb, span);
    f32x16 acc[2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][r] = 0.0f;
    b8p_store(smem, pre, i0, j0, 0, kend);
    __syncthreads();
    int st = 0;
    for (int kt = 0; kt < kend; kt += BBK) {
      const bool more = kt + BBK < kend;
      if (more) b8p_load(pre, rL, M, i0, j0, kt + BBK);
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
        const float b0 = ((const float*)&fb[s >> 2])[s & 3];
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(((const float*)&fa[0][s >> 2])[s & 3], b0, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(((const float*)&fa[1][s >> 2])[s & 3], b0, acc[1], 0, 0, 0);
      }
      if (more) b8p_store(smem + (st ^ 1) * BSTAGE, pre, i0, j0, kt + BBK, kend);
      lds_barrier();
      st ^= 1;
    }
    // the next work item's first k-tile goes out now and lands during this tile's epilogue
    const int nit = it + (int)gridDim.x;
    int nb = b, ni0 = i0, nj0 = j0, nkend = kend;
    if (nit < total) {
      b8p_coords(nit, nf, nb, ni0, nj0, nkend, M);
      if (PREFETCH) {
        const __amdgpu_buffer_rsrc_t rn = make_rsrc(L + uniform64(offs[nb]), span);
        b8p_load(pre, rn, M, ni0, nj0, 0);
      }
    }
    // row-vector epilogue through LDS
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
    __syncthreads();
    if (nit >= total) break;
    it = nit;
    b = nb;
    i0 = ni0;
    j0 = nj0;
    kend = nkend;
    if (!PREFETCH) {
      const __amdgpu_buffer_rsrc_t rn = make_rsrc(L + uniform64(offs[b]), span);
      b8p_load(pre, rn, M, i0, j0, 0);
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
  const int T = M / 128, tiles = T * (T + 1) / 2, total = tiles * nf;
  const size_t lds = 2 * nmgp::BSTAGE * sizeof(float);
  hipFuncSetAttribute((const void*)nmgp::big8p_syrk_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipFuncSetAttribute((const void*)nmgp::big8p_syrk_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int dev = 0, cus = 256;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  auto lib = [&]() {
    return nmgp_gemm_big_offsets_f32(L, M, L, M, 1, C1, M, 1, M, M, M, NMGP_A_LOWER | NMGP_B_UPPER | NMGP_OUT_LOWER,
                                     1.0, 0.0, 1e-4, doff, doff, doff, nf, nullptr, 0);
  };
  auto per = [&](bool pf) {
    if (pf)
      hipLaunchKernelGGL(nmgp::big8p_syrk_kernel<true>, dim3(2 * cus), dim3(512), lds, 0, L, C2, doff, M, nf, total,
                         1e-4f);
    else
      hipLaunchKernelGGL(nmgp::big8p_syrk_kernel<false>, dim3(2 * cus), dim3(512), lds, 0, L, C2, doff, M, nf, total,
                         1e-4f);
    return (int)hipGetLastError();
  };
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double flop = nf * (double)M * M * M / 3.0;   // algorithmic: lower output of L L^T, ~M^3/6 MAC per problem
  for (int rep = 0; rep < 2; ++rep) {
    for (int v = 0; v < 3; ++v) {
      auto run = [&]() { return v == 0 ? lib() : per(v == 1); };
      int rc = run();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) rc |= run();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= 5;
      printf("{\"kernel\": \"%s\", \"nf\": %d, \"M\": %d, \"rc\": %d, \"ms\": %.3f, \"algorithmic_tflops\": %.2f}\n",
             v == 1 ? "persistent 8-wave, next tile's first k-tile prefetched under the epilogue"
             : v == 2 ? "persistent 8-wave, no prefetch (first k-tile loaded after the epilogue)"
                      : "library gemm_big_kernel (8 waves, one workgroup per tile)",
             nf, M, rc, ms, flop / ms / 1e9);
    }
  }
  std::vector<float> a(MM), bb(MM);
  double md = 0, mx = 0;
  for (int f : {0, nf / 2, nf - 1}) {
    hipMemcpy(a.data(), C1 + f * MM, MM * 4, hipMemcpyDeviceToHost);
    hipMemcpy(bb.data(), C2 + f * MM, MM * 4, hipMemcpyDeviceToHost);
    for (int i = 0; i < M; ++i)
      for (int j = 0; j <= i; ++j) {
        md = std::max(md, (double)std::fabs(a[i * M + j] - bb[i * M + j]));
        mx = std::max(mx, (double)std::fabs(a[i * M + j]));
      }
  }
  printf("{\"max_abs_diff\": %.3e, \"max_abs\": %.3e}\n", md, mx);
  return 0;
}
