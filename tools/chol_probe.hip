// Phase-level timing of the batched potrf/trtri kernels (standalone; not part of the library).
//   hipcc -O3 --offload-arch=gfx950 -DNMGP_CHOL_TRACE -I<pkg>/csrc -Iinclude tools/chol_probe.hip <pkg>/csrc/gemm.hip -o /tmp/chol_probe
//   ./chol_probe [n] [batch]
// Prints kernel times (hipEvents, averaged) and, for potrf, the per-block-step split of wall-clock
// time between phase 1 (diagonal factor), phase 2 (panel) and phase 3 (trailing update).
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
  const int batch = argc > 2 ? atoi(argv[2]) : 6;
  const int reps = 50;
  // SPD: A = G G^T / n + I with a fixed LCG G
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
  const int nt = (n + 15) / 16;
  HC(hipMalloc(&dtr, 1024 * sizeof(unsigned long long)));
  HC(hipMemcpyToSymbol(HIP_SYMBOL(nmgp::g_chol_trace), &dtr, sizeof(dtr)));
  HC(hipMemcpy(dA0, A.data(), bytes, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  HC(hipEventCreate(&e0));
  HC(hipEventCreate(&e1));
  float tp = 0, tt = 0;
  std::vector<double> ph(4, 0.0);
  for (int r = 0; r < reps + 3; ++r) {
    HC(hipMemcpy(dA, dA0, bytes, hipMemcpyDeviceToDevice));
    HC(hipEventRecord(e0));
    if (nmgp::potrf_launch<double>(dA, n, n, (int64_t)n * n, batch, dinfo, 0) != 0) return 2;
    HC(hipEventRecord(e1));
    HC(hipEventSynchronize(e1));
    float ms;
    HC(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> tr(nt * 4);
    HC(hipMemcpy(tr.data(), dtr, tr.size() * 8, hipMemcpyDeviceToHost));
    HC(hipEventRecord(e0));
    if (nmgp::trtri_launch<double>(dA, n, n, (int64_t)n * n, dX, n, (int64_t)n * n, batch, 0) != 0) return 3;
    HC(hipEventRecord(e1));
    HC(hipEventSynchronize(e1));
    float ms2;
    HC(hipEventElapsedTime(&ms2, e0, e1));
    if (r >= 3) {
      tp += ms;
      tt += ms2;
      for (int kb = 0; kb < nt; ++kb)
        for (int p = 1; p < 4; ++p) ph[p] += (double)(tr[kb * 4 + p] - tr[kb * 4 + p - 1]) * 10.0;  // 100 MHz
    }
  }
  float tf = 0;
  for (int r = 0; r < reps + 3; ++r) {
    HC(hipMemcpy(dA, dA0, bytes, hipMemcpyDeviceToDevice));
    HC(hipEventRecord(e0));
    if (nmgp::chol_inv_launch<double>(dA, n, n, (int64_t)n * n, dX, n, (int64_t)n * n, batch, dinfo, 0) != 0)
      return 4;
    HC(hipEventRecord(e1));
    HC(hipEventSynchronize(e1));
    float ms;
    HC(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 3) tf += ms;
  }
  printf("fused chol_inv %.2f us\n", 1000 * tf / reps);
  {
    // recursive (two-level) path at the same n, graph-captured so launch gaps are as in the engine
    hipStream_t cs;
    HC(hipStreamCreate(&cs));
    for (int lvl = 0; lvl < 2; ++lvl) {
      hipGraph_t g;
      hipGraphExec_t ge;
      HC(hipStreamBeginCapture(cs, hipStreamCaptureModeGlobal));
      int rc = lvl == 0 ? nmgp::chol_inv_small<double>(dA, n, n, (int64_t)n * n, dX, n, (int64_t)n * n, batch, dinfo,
                                                       cs, 0, 1)
                        : nmgp::chol_inv_rec<double>(dA, n, n, (int64_t)n * n, dX, n, (int64_t)n * n, batch, dinfo,
                                                     cs, 0, nullptr);
      HC(hipStreamEndCapture(cs, &g));
      if (rc != 0) return 5;
      HC(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      float tg = 0;
      for (int r = 0; r < reps + 3; ++r) {
        HC(hipMemcpy(dA, dA0, bytes, hipMemcpyDeviceToDevice));
        HC(hipEventRecord(e0, cs));
        HC(hipGraphLaunch(ge, cs));
        HC(hipEventRecord(e1, cs));
        HC(hipEventSynchronize(e1));
        float ms;
        HC(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) tg += ms;
      }
      printf("%s (graph) %.2f us\n", lvl == 0 ? "chol_inv_small" : "recursive 128-leaf", 1000 * tg / reps);
      if (lvl == 0) {
        std::vector<unsigned long long> tr((nt + 1) * 4);
        HC(hipMemcpy(tr.data(), dtr, tr.size() * 8, hipMemcpyDeviceToHost));
        double q[4] = {0, 0, 0, 0};
        for (int kb = 0; kb < nt; ++kb) {
          q[0] += (tr[kb * 4 + 1] - tr[kb * 4]) * 10.0;
          q[1] += (tr[kb * 4 + 2] - tr[kb * 4 + 1]) * 10.0;
          q[2] += (tr[kb * 4 + 3] - tr[kb * 4 + 2]) * 10.0;
          q[3] += (tr[(kb + 1) * 4] - tr[kb * 4 + 3]) * 10.0;
        }
        printf("  block 0 phases (ns, summed over steps): spill %.0f  panel %.0f  publish+syrk %.0f  drain+flag %.0f"
               "  (total %.0f)\n", q[0], q[1], q[2], q[3], (tr[nt * 4] - tr[0]) * 10.0);
        std::vector<unsigned long long> t1(256 + nt * 4);
        HC(hipMemcpy(t1.data(), dtr, t1.size() * 8, hipMemcpyDeviceToHost));
        double w1 = 0, l1 = 0, a1 = 0, c1 = 0;
        for (int kb = 0; kb < nt; ++kb) {
          const unsigned long long* r1 = &t1[256 + kb * 4];
          w1 += (r1[0] - (kb ? t1[256 + (kb - 1) * 4 + 3] : tr[0])) * 10.0;
          l1 += (r1[1] - r1[0]) * 10.0;
          a1 += (r1[2] - r1[1]) * 10.0;
          c1 += (r1[3] - r1[2]) * 10.0;
        }
        {
          std::vector<unsigned long long> tx(1024);
          HC(hipMemcpy(tx.data(), dtr, tx.size() * 8, hipMemcpyDeviceToHost));
          printf("  role 0: prologue (tile loads + zeroing) %.0f ns, loop %.0f ns; inverse workgroups end %.0f / %.0f ns "
                 "after role 0 starts\n", (tx[1001] - tx[1000]) * 10.0, (tx[1002] - tx[1001]) * 10.0,
                 (tx[1006] - tx[1000]) * 10.0, (tx[1010] - tx[1000]) * 10.0);
        }
        {
          std::vector<unsigned long long> tw(1024);
          HC(hipMemcpy(tw.data(), dtr, tw.size() * 8, hipMemcpyDeviceToHost));
          double a = 0, b = 0, c = 0, d = 0;
          for (int kb = 0; kb < nt; ++kb) {
            a += (tw[512 + kb * 4] - tw[kb * 4 + 1]) * 10.0;
            b += (tw[512 + kb * 4 + 1] - tw[512 + kb * 4]) * 10.0;
            c += (tw[512 + kb * 4 + 2] - tw[512 + kb * 4 + 1]) * 10.0;
            d += (tw[kb * 4 + 2] - tw[512 + kb * 4 + 2]) * 10.0;
          }
          printf("  role 0 panel (ns, summed): colbuf load %.0f  16-column loop %.0f  LDS write %.0f  wait+barrier+flag %.0f\n",
                 a, b, c, d);
        }
        printf("  block 1 phases (ns, summed): wait-flag %.0f  load %.0f  X-row %.0f  update+store %.0f  (ends %.0f after "
               "block 0)\n", w1, l1, a1, c1, ((double)t1[256 + (nt - 1) * 4 + 3] - (double)tr[nt * 4]) * 10.0);
        printf("  per step lag (flag seen - role0 step end, ns):");
        for (int kb = 0; kb < nt; ++kb) printf(" %.0f", ((double)t1[256 + kb * 4] - (double)tr[(kb + 1) * 4]) * 10.0);
        printf("\n");
      }
    }
  }
  {
    std::vector<unsigned long long> tr((nt + 1) * 4);
    HC(hipMemcpy(tr.data(), dtr, tr.size() * 8, hipMemcpyDeviceToHost));
    double q[4] = {0, 0, 0, 0};
    for (int kb = 0; kb < nt; ++kb) {
      q[0] += (tr[kb * 4 + 1] - tr[kb * 4]) * 10.0;
      q[1] += (tr[kb * 4 + 2] - tr[kb * 4 + 1]) * 10.0;
      q[2] += (tr[kb * 4 + 3] - tr[kb * 4 + 2]) * 10.0;
      q[3] += (tr[(kb + 1) * 4] - tr[kb * 4 + 3]) * 10.0;
    }
    printf("fused phases (ns, last run, summed over steps): spill %.0f  panel %.0f  X+syrk %.0f  trtri-upd %.0f\n",
           q[0], q[1], q[2], q[3]);
    std::vector<unsigned long long> tw(1024);
    HC(hipMemcpy(tw.data(), dtr, tw.size() * 8, hipMemcpyDeviceToHost));
    printf("panel j-loop x10ns per step:");
    for (int kb = 0; kb < nt; ++kb)
      printf(" [load %llu loop %llu write %llu barrier %llu]", tw[512 + kb * 4] - tr[kb * 4 + 1],
             tw[512 + kb * 4 + 1] - tw[512 + kb * 4], tw[512 + kb * 4 + 2] - tw[512 + kb * 4 + 1],
             tr[kb * 4 + 2] - tw[512 + kb * 4 + 2]);
    printf("\n");
  }
  // residual check: L L^T vs A for matrix 0
  std::vector<double> L((size_t)n * n), X((size_t)n * n);
  HC(hipMemcpy(L.data(), dA, L.size() * 8, hipMemcpyDeviceToHost));
  HC(hipMemcpy(X.data(), dX, X.size() * 8, hipMemcpyDeviceToHost));
  double err = 0, err2 = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0, s2 = 0;
      for (int k = 0; k <= j; ++k) s += L[(size_t)i * n + k] * L[(size_t)j * n + k];
      for (int k = j; k <= i; ++k) s2 += L[(size_t)i * n + k] * X[(size_t)k * n + j];
      err = fmax(err, fabs(s - A[(size_t)i * n + j]));
      err2 = fmax(err2, fabs(s2 - (i == j)));
    }
  printf("n=%d batch=%d potrf %.2f us  trtri %.2f us  |LL^T-A|=%.3e |LX-I|=%.3e\n", n, batch, 1000 * tp / reps,
         1000 * tt / reps, err, err2);
  printf("potrf phases (ns summed over %d block steps): diag %.0f  panel %.0f  trailing %.0f\n", nt, ph[1] / reps,
         ph[2] / reps, ph[3] / reps);
  return 0;
}
