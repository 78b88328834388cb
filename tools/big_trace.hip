// Wall-clock phases of gemm_big_kernel launches (standalone; not in the library):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DNMGP_BIG_TRACE -I<pkg>/csrc -Iinclude tools/big_trace.hip \
//         -o tools/bin/big_trace
//   ./big_trace m n k [split 0/1] [lda]
// C (m x n, OUT_LOWER, beta 1) -= L_a L_b^T with L read from a lda-wide row-major matrix, as the blocked potrf's
// k-sized updates.  Per workgroup (100 MHz wall clock): start offset, prologue (first k-tile in LDS), main loop,
// split-K combine, epilogue -- summarised as spreads over the grid -- after 3 warm-up launches.
#include "gemm_big.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 128, n = argc > 2 ? atoi(argv[2]) : 128, k = argc > 3 ? atoi(argv[3]) : 512;
  const int split = argc > 4 ? atoi(argv[4]) : 1;
  const int64_t lda = argc > 5 ? atoll(argv[5]) : 4096;
  const int64_t rows = std::max<int64_t>(m, lda);
  float *A, *ws;
  hipMalloc(&A, (size_t)rows * lda * 4);
  hipMemset(A, 0, (size_t)rows * lda * 4);
  const size_t wsb = nmgp::gemm_big_ws_bytes();
  hipMalloc(&ws, wsb);
  hipMemset(ws, 0, wsb);
  const int NT = 8 * 4096;
  unsigned long long* tr;
  hipMalloc(&tr, NT * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(nmgp::g_big_trace), &tr, sizeof(tr));
  float* L = A;                       // rows 0.., columns 0..k
  float* C = A + k;                   // C(i, j) at A[i * lda + k + j]
  auto go = [&]() {
    return nmgp::gemm_big_f32(L, lda, L, lda, 1, C, lda, 1, m, n, k, NMGP_OUT_LOWER, -1.0f, 1.0f, 0, 0, 0, 1,
                              split ? ws : nullptr, 0);
  };
  for (int r = 0; r < 3; ++r) go();
  hipDeviceSynchronize();
  hipMemset(tr, 0, NT * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  const int rc = go();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> t(NT);
  hipMemcpy(t.data(), tr, NT * 8, hipMemcpyDeviceToHost);
  int nblk = 0;
  while (nblk < NT / 8 && t[nblk * 8]) ++nblk;
  printf("%dx%dx%d split %d lda %lld: rc %d, event %.2f us, %d workgroups traced\n", m, n, k, split, (long long)lda,
         rc, ms * 1000, nblk);
  unsigned long long t0 = ~0ull, tend = 0;
  for (int b = 0; b < nblk; ++b) t0 = std::min(t0, t[b * 8]);
  std::vector<double> st, pro, mainl, comb, epi;
  for (int b = 0; b < nblk; ++b) {
    const unsigned long long* s = &t[b * 8];
    st.push_back((s[0] - t0) * 10.0);
    if (s[1]) pro.push_back((s[1] - s[0]) * 10.0);
    if (s[2]) mainl.push_back((s[2] - (s[1] ? s[1] : s[0])) * 10.0);
    if (s[3]) comb.push_back((s[3] - s[2]) * 10.0);
    if (s[4]) {
      epi.push_back((s[4] - s[3]) * 10.0);
      tend = std::max(tend, s[4]);
    }
  }
  auto pr = [](const char* name, std::vector<double> v) {
    if (v.empty()) return;
    std::sort(v.begin(), v.end());
    printf("  %-22s n=%5zu  min %8.0f  med %8.0f  max %8.0f ns\n", name, v.size(), v.front(), v[v.size() / 2],
           v.back());
  };
  pr("start offset", st);
  pr("prologue (1st k-tile)", pro);
  pr("main loop", mainl);
  pr("split-K combine", comb);
  pr("epilogue + drain", epi);
  printf("  first start -> last end %.0f ns\n", (tend - t0) * 10.0);
  return 0;
}
