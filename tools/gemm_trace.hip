// Cycle-stamped phases of one gemm_kernel launch (standalone; not in the library).
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -DNMGP_GEMM_TRACE -I<pkg>/csrc -Iinclude \
//         tools/gemm_trace.hip -o tools/bin/gemm_trace
//   ./gemm_trace m n k [ksplit] [transA]
// Workgroup 0: per-k-tile shader-cycle phases.  Every workgroup: wall-clock (100 MHz) start, end of
// main loop, end of split-K publish, end -- summarised as spreads over the grid.
#include "gemm.hip"

#ifndef TT
#define TT double   // -DTT=float: the f32 kernel
#endif

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 2000, n = argc > 2 ? atoi(argv[2]) : 256, k = argc > 3 ? atoi(argv[3]) : 256;
  const int ks = argc > 4 ? atoi(argv[4]) : 1;
  const int transA = argc > 5 ? atoi(argv[5]) : 0;
  const int nprob = argc > 6 ? atoi(argv[6]) : 1;   // copies of the problem in one grouped launch
  TT *A, *B, *C, *ws;
  int32_t* ctr;
  const int tm = (m + 63) / 64, tn = (n + 63) / 64, nblk1 = tm * tn * ks, nblk = nblk1 * nprob;
  hipMalloc(&A, (size_t)m * k * sizeof(TT));
  hipMalloc(&B, (size_t)k * n * sizeof(TT));
  hipMalloc(&C, (size_t)m * n * sizeof(TT));
  hipMalloc(&ws, (size_t)tm * tn * ks * 4096 * sizeof(TT) * nprob);
  hipMalloc(&ctr, (size_t)tm * tn * 4 * nprob);
  hipMemset(ctr, 0, (size_t)tm * tn * 4 * nprob);
  hipMemset(A, 0, (size_t)m * k * sizeof(TT));
  hipMemset(B, 0, (size_t)k * n * sizeof(TT));
  const int NT = 1024 + 4 * nblk;
  unsigned long long* tr;
  hipMalloc(&tr, NT * 8);
  hipMemset(tr, 0, NT * 8);
#ifdef NMGP_GEMM_TRACE
  hipMemcpyToSymbol(HIP_SYMBOL(nmgp::g_gemm_trace), &tr, sizeof(tr));
#endif
  nmgp_gemm_desc d{};
  d.A = A; d.B = B; d.C = C;
  if (transA) { d.sA_i = 1; d.sA_k = m; } else { d.sA_i = k; d.sA_k = 1; }
  d.sB_k = n; d.sB_j = 1; d.sC_i = n; d.sC_j = 1;
  d.m = m; d.n = n; d.k = k; d.row_seg = -1; d.k_seg = -1; d.alpha = 1.0;
  d.tiles_m = tm; d.tiles_n = tn; d.tile_start = 0; d.ksplit = ks; d.ws = ws; d.counters = ctr; d.batch = 1;
  std::vector<nmgp_gemm_desc> hd(nprob, d);
  for (int p = 0; p < nprob; ++p) {
    hd[p].tile_start = p * nblk1;
    hd[p].ws = ws + (size_t)p * tm * tn * ks * 4096;
    hd[p].counters = ctr + (size_t)p * tm * tn;
  }
  nmgp_gemm_desc* dd;
  hipMalloc(&dd, sizeof(d) * nprob);
  hipMemcpy(dd, hd.data(), sizeof(d) * nprob, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int r = 0; r < 3; ++r) nmgp::launch_grouped<TT>(dd, nprob, nblk, nullptr, 0);
  hipEventRecord(e0);
  nmgp::launch_grouped<TT>(dd, nprob, nblk, nullptr, 0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
#ifndef NMGP_GEMM_TRACE
  {
    // untraced: average of 20 back-to-back launches
    hipEventRecord(e0);
    for (int r = 0; r < 20; ++r) nmgp::launch_grouped<TT>(dd, nprob, nblk, nullptr, 0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms20;
    hipEventElapsedTime(&ms20, e0, e1);
    const double fl = 2.0 * m * n * k * nprob;
    printf("nprob %d: ", nprob);
    printf("%dx%dx%d ksplit %d transA %d: %.2f us per launch (20 back-to-back), %.2f TF/s\n", m, n, k, ks, transA,
           ms20 * 50, fl / (ms20 / 20 * 1e-3) / 1e12);
    return 0;
  }
#endif
  std::vector<unsigned long long> t(NT);
  hipMemcpy(t.data(), tr, NT * 8, hipMemcpyDeviceToHost);
  printf("nprob %d: ", nprob);
  printf("%dx%dx%d ksplit %d transA %d: kernel %.2f us, %d workgroups; WG0 cycles: desc %llu, first-load-issue %llu\n",
         m, n, k, ks, transA, ms * 1000, nblk, t[1] - t[0], t[2] - t[1]);
  for (int it = 0; it < 31 && t[3 + 2 * it]; ++it)
    printf("  ktile %2d: barrier-exit %6llu  mma+stage %6llu  load %6llu  barrier %6llu\n", it,
           t[3 + 2 * it] - (it ? t[4 + 2 * (it - 1)] : t[2]), t[100 + 4 * it] - t[3 + 2 * it],
           t[101 + 4 * it] - t[100 + 4 * it], t[4 + 2 * it] - t[101 + 4 * it]);
  printf("  WG0 epilogue %llu, total %llu cycles\n", t[71] - t[70], t[71] - t[0]);
  unsigned long long t0 = ~0ull, tend = 0;
  std::vector<double> start, main, pub, red;
  for (int b = 0; b < nblk; ++b) {
    const unsigned long long* s = &t[1024 + 4 * b];
    t0 = std::min(t0, s[0]);
  }
  for (int b = 0; b < nblk; ++b) {
    const unsigned long long* s = &t[1024 + 4 * b];
    start.push_back((s[0] - t0) * 10.0);
    main.push_back((s[1] - s[0]) * 10.0);
    if (s[2]) pub.push_back((s[2] - s[1]) * 10.0);
    if (s[3]) {
      tend = std::max(tend, s[3]);
      red.push_back((s[3] - (s[2] ? s[2] : s[1])) * 10.0);
    }
  }
  auto pr = [](const char* name, std::vector<double> v) {
    if (v.empty()) return;
    std::sort(v.begin(), v.end());
    printf("  %-26s n=%5zu  min %8.0f  med %8.0f  max %8.0f ns\n", name, v.size(), v.front(), v[v.size() / 2],
           v.back());
  };
  pr("start offset", start);
  pr("desc+mainloop", main);
  pr("split-K publish+sync", pub);
  pr("reduce+store (finishers)", red);
  printf("  first start -> last end %.0f ns\n", (tend - t0) * 10.0);
  return 0;
}
