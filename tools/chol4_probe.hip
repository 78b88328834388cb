// Per-step timeline of the multi-role factor+inverse kernel for matrix 0 of a batch (written for round 3's
// lookahead kernel, removed in round 4; the stamps sit in the four-role kernel's shared code paths)
// (standalone; not part of the library).  Wall clock 100 MHz (10 ns) stamps:
//   role 0 = diagonal wave: 0 column seen, 1 chain done, 2 table / L_kk in LDS;  role 1 = row wave 1:
//            0 table seen, 1 rows in LDS;  role 2 = update wave 4: 0 rows seen, 1 column k+1 spilled,
//            2 trailing update done;  roles 3 / 4 = inverse workgroups wave 0: 0 step start, 1 prefetch
//            issued, 2 step done.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DNMGP_CHOL_TRACE -I<pkg>/csrc tools/chol4_probe.hip \
//         <pkg>/csrc/gemm.hip <pkg>/csrc/gemm_big.hip -o tools/bin/chol4_probe
//   ./chol4_probe [n] [batch]          (NMGP_CHOL_4ROLE=0 times the three-role kernel, no timeline)
#include "chol.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define HC(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 256;
  const int batch = argc > 2 ? atoi(argv[2]) : 4;
  const int reps = 20;
  std::vector<double> G((size_t)n * n), A((size_t)n * n * batch);
  unsigned long long st = 12345;
  for (auto& g : G) {
    st = st * 6364136223846793005ULL + 1442695040888963407ULL;
    g = ((st >> 11) * (1.0 / 9007199254740992.0)) - 0.5;
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += G[(size_t)i * n + k] * G[(size_t)j * n + k];
      for (int b = 0; b < batch; ++b) A[(size_t)b * n * n + (size_t)i * n + j] = s / n + (i == j);
    }
  double *dA0, *dA, *dX;
  int32_t* dinfo;
  unsigned long long* dtr;
  const size_t bytes = A.size() * sizeof(double);
  HC(hipMalloc(&dA0, bytes));
  HC(hipMalloc(&dA, bytes));
  HC(hipMalloc(&dX, bytes));
  HC(hipMalloc(&dinfo, batch * sizeof(int32_t)));
  HC(hipMalloc(&dtr, 4096 * sizeof(unsigned long long)));
  HC(hipMemset(dtr, 0, 4096 * sizeof(unsigned long long)));
  HC(hipMemcpyToSymbol(HIP_SYMBOL(nmgp::g_chol_trace), &dtr, sizeof(dtr)));
  HC(hipMemcpy(dA0, A.data(), bytes, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  HC(hipEventCreate(&e0));
  HC(hipEventCreate(&e1));
  float tot = 0;
  for (int r = 0; r < reps + 3; ++r) {
    HC(hipMemcpy(dA, dA0, bytes, hipMemcpyDeviceToDevice));
    HC(hipDeviceSynchronize());
    HC(hipEventRecord(e0));
    if (nmgp::chol_inv_launch<double>(dA, n, n, (int64_t)n * n, dX, n, (int64_t)n * n, batch, dinfo, 0) != 0) return 2;
    HC(hipEventRecord(e1));
    HC(hipEventSynchronize(e1));
    float ms;
    HC(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 3) tot += ms;
  }
  std::vector<int32_t> info(batch);
  HC(hipMemcpy(info.data(), dinfo, batch * sizeof(int32_t), hipMemcpyDeviceToHost));
  std::vector<unsigned long long> tr(4096);
  HC(hipMemcpy(tr.data(), dtr, 4096 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  printf("n=%d batch=%d  launch %.2f us (event, avg of %d)  info0=%d\n", n, batch, 1000.0 * tot / reps, reps, info[0]);
  if (getenv("NMGP_CHOL_4ROLE")) {
    // four-role kernel: the factor workgroup's CHOL_STAMP(kb, p): 1 column spilled, 2 panel done, 3 publish
    // issued + next column's loads issued (relative to the first stamp)
    unsigned long long b0 = ~0ull;
    for (int i = 0; i < 256; ++i)
      if (tr[i] && tr[i] < b0) b0 = tr[i];
    printf("  k | factor: mfma+spill  polled+barrier  panel  publish\n");
    for (int k = 0; k < (n + 15) / 16; ++k) {
      auto r = [&](int p) { return tr[k * 4 + p] ? (double)(long long)(tr[k * 4 + p] - b0) / 100.0 : -1.0; };
      printf("%3d | %8.2f %8.2f %6.2f %6.2f\n", k, r(0), r(1), r(2), r(3));
    }
    return 0;
  }
  const int nt = (n + 15) / 16;
  auto T = [&](int role, int k, int ph) { return tr[2048 + role * 512 + k * 8 + ph]; };
  // every workgroup runs on its own XCD, whose wall clock is not synchronised with the others': each
  // workgroup's stamps are shown relative to its own start
  auto base = [&](int r0, int r1) {   // earliest stamp of the roles [r0, r1] (one workgroup)
    unsigned long long b = ~0ull;
    for (int r = r0; r <= r1; ++r)
      for (int i = 0; i < 512; ++i)
        if (tr[2048 + r * 512 + i] && tr[2048 + r * 512 + i] < b) b = tr[2048 + r * 512 + i];
    return b;
  };
  const unsigned long long bf = base(0, 2), b1 = base(3, 3), b2 = base(4, 4);
  auto rel = [&](unsigned long long v, unsigned long long b) { return v ? ((double)(long long)(v - b)) / 100.0 : -1.0; };
  printf("  k | diag: column  chain  table | rows: table  done | update: rows  col+1  trail | inv0: start pref  done | inv1: done\n");
  for (int k = 0; k <= nt; ++k)
    printf("%3d | %7.2f %6.2f %6.2f | %7.2f %6.2f | %7.2f %6.2f %6.2f | %7.2f %6.2f %6.2f | %6.2f\n", k, rel(T(0, k, 0), bf),
           rel(T(0, k, 1), bf), rel(T(0, k, 2), bf), rel(T(1, k, 0), bf), rel(T(1, k, 1), bf), rel(T(2, k, 0), bf),
           rel(T(2, k, 1), bf), rel(T(2, k, 2), bf), rel(T(3, k, 0), b1), rel(T(3, k, 1), b1), rel(T(3, k, 2), b1),
           rel(T(4, k, 2), b2));
  return 0;
}
