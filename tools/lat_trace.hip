// Cycle-stamped phases of one gemm_lat_kernel launch (standalone; not in the library).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DNMGP_LAT_TRACE -I<pkg>/csrc -Iinclude tools/lat_trace.hip \
//         -o tools/bin/lat_trace
//   ./lat_trace m n k [nprob] [transA]
// nprob copies of an m x n x k f64 GEMM (A row-major m x k, or k x m with transA; B k x n row-major) in one
// grouped launch, the PM2.5 step's shapes by default (2000 x 256 x 256, 5 problems: the quad_W / P-bar_G
// products).  Prints the launch time (events, mean of 20) and, over the workgroups' first tiles, the median /
// 90th percentile shader cycles of: descriptor lookup (0->1), operand loads landed (1->2), MFMAs (2->3),
// partials to LDS + barrier (3->4), wave-order reduction (4->5), epilogue stores issued (5->6).
#include "gemm_lat.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 2000, n = argc > 2 ? atoi(argv[2]) : 256, k = argc > 3 ? atoi(argv[3]) : 256;
  const int nprob = argc > 4 ? atoi(argv[4]) : 5;
  const int transA = argc > 5 ? atoi(argv[5]) : 0;
  double *A, *B, *C;
  hipMalloc(&A, (size_t)m * k * 8 * nprob);
  hipMalloc(&B, (size_t)k * n * 8 * nprob);
  hipMalloc(&C, (size_t)m * n * 8 * nprob);
  hipMemset(A, 0, (size_t)m * k * 8 * nprob);
  hipMemset(B, 0, (size_t)k * n * 8 * nprob);
  const int tm = (m + 31) / 32, tn = (n + 31) / 32, tiles1 = tm * tn, total = tiles1 * nprob;
  const int wgs = ((total + 7) / 8) * 8;
  unsigned long long* tr;
  hipMalloc(&tr, (size_t)wgs * 8 * 8);
  hipMemset(tr, 0, (size_t)wgs * 8 * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(nmgp::g_lat_trace), &tr, sizeof(tr));
  std::vector<nmgp_gemm_desc> hd(nprob);
  for (int p = 0; p < nprob; ++p) {
    nmgp_gemm_desc d{};
    d.A = A + (size_t)p * m * k;
    d.B = B + (size_t)p * k * n;
    d.C = C + (size_t)p * m * n;
    if (transA) { d.sA_i = 1; d.sA_k = m; } else { d.sA_i = k; d.sA_k = 1; }
    d.sB_k = n; d.sB_j = 1; d.sC_i = n; d.sC_j = 1;
    d.m = m; d.n = n; d.k = k; d.row_seg = -1; d.k_seg = -1; d.alpha = 1.0;
    d.tiles_m = tm; d.tiles_n = tn; d.tile_start = p * tiles1; d.ksplit = 1; d.batch = 1;
    hd[p] = d;
  }
  nmgp_gemm_desc* dd;
  hipMalloc(&dd, sizeof(nmgp_gemm_desc) * nprob);
  hipMemcpy(dd, hd.data(), sizeof(nmgp_gemm_desc) * nprob, hipMemcpyHostToDevice);
  for (int r = 0; r < 3; ++r) nmgp::launch_lat<double>(dd, nprob, total, nullptr, nullptr, 0, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 20; ++r) nmgp::launch_lat<double>(dd, nprob, total, nullptr, nullptr, 0, 0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h((size_t)wgs * 8);
  hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost);
  const double flop = 2.0 * m * n * (double)k * nprob;
  printf("m %d n %d k %d nprob %d transA %d: %d workgroups, %.2f us per launch, %.2f TF/s\n", m, n, k, nprob, transA, wgs,
         ms * 1e3 / 20, flop / (ms * 1e-3 / 20) / 1e12);
  const char* names[6] = {"desc lookup", "loads landed", "MFMAs", "LDS + barrier", "reduction", "epilogue"};
  for (int ph = 0; ph < 6; ++ph) {
    std::vector<long long> v;
    for (int b = 0; b < wgs; ++b) {
      const unsigned long long s0 = h[(size_t)b * 8 + ph], s1 = h[(size_t)b * 8 + ph + 1];
      if (s0 && s1 && s1 >= s0) v.push_back((long long)(s1 - s0));
    }
    if (v.empty()) continue;
    std::sort(v.begin(), v.end());
    printf("  %-14s n=%5zu  med %7lld  p90 %7lld  max %7lld cycles\n", names[ph], v.size(), v[v.size() / 2],
           v[v.size() * 9 / 10], v.back());
  }
  return 0;
}
