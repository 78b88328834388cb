// Wall-clock phases of the BATCHED gemm_big_kernel launches of the ECoG step (standalone; not in the library):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DNMGP_BIG_TRACE -I<pkg>/csrc -Iinclude tools/big_trace_batch.hip \
//         -o tools/bin/big_trace_batch
//   ./big_trace_batch [nf=256] [M=1024]
// Two products on nf M x M problems at per-problem offsets, as engine.py builds them for ECoG:
//   syrk:    Sigma = L L^T + j I          (A_LOWER | B_UPPER | OUT_LOWER, both operands k-contiguous)
//   kl_lbar: G = -C^-T Xs + rs(i) E(i, j) (A_UPPER | B_LOWER | OUT_TRIL | EPI, both operands k-strided, beta 1)
// Per workgroup (100 MHz wall clock): prologue (first k-tile in LDS), main loop, epilogue -- medians, and the
// main loop's time per 32-deep k-tile (sum over workgroups / sum of their k-tiles).  (Since the batched launches
// became persistent the stamps of a workgroup are those of its LAST work item: the per-k-tile figure no longer
// normalises correctly; the profiles r05t / r05u / r05aa predate that change.)
#include "gemm_big.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  const int nf = argc > 1 ? atoi(argv[1]) : 256, M = argc > 2 ? atoi(argv[2]) : 1024;
  const int64_t MM = (int64_t)M * M;
  float *A, *B, *C, *E, *RS;
  hipMalloc(&A, nf * MM * 4);
  hipMalloc(&B, nf * MM * 4);
  hipMalloc(&C, nf * MM * 4);
  hipMalloc(&E, nf * MM * 4);
  hipMalloc(&RS, (size_t)nf * M * 4);
  hipMemset(A, 0, nf * MM * 4);
  hipMemset(B, 0, nf * MM * 4);
  hipMemset(C, 0, nf * MM * 4);
  hipMemset(E, 0, nf * MM * 4);
  hipMemset(RS, 0, (size_t)nf * M * 4);
  std::vector<int64_t> off(nf), roff(nf);
  for (int f = 0; f < nf; ++f) {
    off[f] = f * MM;
    roff[f] = (int64_t)f * M;
  }
  int64_t *doff, *droff;
  hipMalloc(&doff, nf * 8);
  hipMalloc(&droff, nf * 8);
  hipMemcpy(doff, off.data(), nf * 8, hipMemcpyHostToDevice);
  hipMemcpy(droff, roff.data(), nf * 8, hipMemcpyHostToDevice);
  const int T = M / 128;
  const int NT = 8 * nf * T * T;
  unsigned long long* tr;
  hipMalloc(&tr, (size_t)NT * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(nmgp::g_big_trace), &tr, sizeof(tr));
  for (int variant = 0; variant < 2; ++variant) {
    auto go = [&]() {
      if (variant == 0)
        return nmgp_gemm_big_offsets_epi_f32(A, M, 1, A, M, 1, C, M, 1, M, M, M,
                                             NMGP_A_LOWER | NMGP_B_UPPER | NMGP_OUT_LOWER, 1.0, 0.0, 1e-4, doff, doff,
                                             doff, nullptr, nullptr, 0, 0, nullptr, nullptr, 0.0, nullptr, nullptr,
                                             nullptr, nf, nullptr, 0);
      return nmgp_gemm_big_offsets_epi_f32(A, M, 0, B, M, 0, C, M, 1, M, M, M,
                                           NMGP_A_UPPER | NMGP_B_LOWER | NMGP_OUT_TRIL | NMGP_EPI | NMGP_EPI_E_LOWER,
                                           -1.0, 1.0, 0.0, doff, doff, doff, E, doff, M, 1, RS, droff, 1.0, nullptr,
                                           nullptr, nullptr, nf, nullptr, 0);
    };
    for (int r = 0; r < 2; ++r) go();
    hipDeviceSynchronize();
    hipMemset(tr, 0, (size_t)NT * 8);
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
    hipMemcpy(t.data(), tr, (size_t)NT * 8, hipMemcpyDeviceToHost);
    // k-tiles of every launched tile (same per problem): syrk lower tiles k < (tn+1) 128; kl_lbar lower tiles
    // k in [tm 128, M), tiles above the diagonal none
    int64_t kt_per_problem = 0;
    int launched = 0;
    for (int tm = 0; tm < T; ++tm)
      for (int tn = 0; tn < T; ++tn) {
        if (variant == 0) {
          if (tn > tm) continue;
          kt_per_problem += (tn + 1) * 4;
        } else {
          if (tn <= tm) kt_per_problem += (M - tm * 128) / 32;
        }
        ++launched;
      }
    const int nblk = launched * nf;
    std::vector<double> pro, mainl, epi, tot;
    double sum_main = 0;
    unsigned long long t0 = ~0ull, tend = 0;
    for (int b = 0; b < nblk; ++b) {
      const unsigned long long* s = &t[(size_t)b * 8];
      if (!s[0]) continue;
      t0 = std::min(t0, s[0]);
      if (s[1]) pro.push_back((s[1] - s[0]) * 10.0);
      if (s[2] && s[1]) {
        mainl.push_back((s[2] - s[1]) * 10.0);
        sum_main += (s[2] - s[1]) * 10.0;
      }
      if (s[4] && s[3]) epi.push_back((s[4] - s[3]) * 10.0);
      if (s[4]) {
        tot.push_back((s[4] - s[0]) * 10.0);
        tend = std::max(tend, s[4]);
      }
    }
    auto med = [](std::vector<double> v) {
      if (v.empty()) return 0.0;
      std::sort(v.begin(), v.end());
      return v[v.size() / 2];
    };
    double sum_tot = 0;
    for (double x : tot) sum_tot += x;
    printf("{\"variant\": \"%s\", \"nf\": %d, \"M\": %d, \"rc\": %d, \"event_ms\": %.3f, \"workgroups\": %d, "
           "\"prologue_med_ns\": %.0f, \"main_med_ns\": %.0f, \"epilogue_med_ns\": %.0f, \"wg_total_med_ns\": %.0f, "
           "\"main_ns_per_ktile\": %.1f, \"main_share_of_wg_time\": %.3f, \"span_ns\": %.0f}\n",
           variant ? "kl_lbar" : "syrk", nf, M, rc, ms, nblk, med(pro), med(mainl), med(epi), med(tot),
           sum_main / (double)(kt_per_problem * nf), sum_main / sum_tot, (tend - t0) * 10.0);
  }
  return 0;
}
