// Cycle-stamped phases of workgroup 0 of one gemm_kernel launch (standalone; not in the library).
//   hipcc -O3 --offload-arch=gfx950 -DNMGP_GEMM_TRACE -I<pkg>/csrc tools/gemm_trace.hip -o tools/bin/gemm_trace
//   ./gemm_trace m n k [ksplit-free]
#include "gemm.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 2000, n = argc > 2 ? atoi(argv[2]) : 256, k = argc > 3 ? atoi(argv[3]) : 256;
  double *A, *B, *C;
  hipMalloc(&A, (size_t)m * k * 8);
  hipMalloc(&B, (size_t)k * n * 8);
  hipMalloc(&C, (size_t)m * n * 8);
  hipMemset(A, 0, (size_t)m * k * 8);
  hipMemset(B, 0, (size_t)k * n * 8);
  unsigned long long* tr;
  hipMalloc(&tr, 128 * 8);
  hipMemset(tr, 0, 128 * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(nmgp::g_gemm_trace), &tr, sizeof(tr));
  nmgp_gemm_desc d{};
  d.A = A; d.B = B; d.C = C;
  d.sA_i = k; d.sA_k = 1; d.sB_k = n; d.sB_j = 1; d.sC_i = n; d.sC_j = 1;
  d.m = m; d.n = n; d.k = k; d.row_seg = -1; d.k_seg = -1; d.alpha = 1.0;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int r = 0; r < 3; ++r) nmgp::gemm_single<double>(d, 0);
  hipEventRecord(e0);
  nmgp::gemm_single<double>(d, 0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> t(128);
  hipMemcpy(t.data(), tr, 128 * 8, hipMemcpyDeviceToHost);
  printf("%dx%dx%d: kernel %.2f us; WG0 cycles: desc %llu, first-load-issue %llu\n", m, n, k, ms * 1000,
         t[1] - t[0], t[2] - t[1]);
  for (int it = 0; it < 31 && t[3 + 2 * it]; ++it)
    printf("  ktile %2d: wait+stage %6llu  mma %6llu\n", it, t[3 + 2 * it] - (it ? t[4 + 2 * (it - 1)] : t[2]),
           t[4 + 2 * it] - t[3 + 2 * it]);
  printf("  epilogue %llu, total %llu cycles\n", t[71] - t[70], t[71] - t[0]);
  return 0;
}
