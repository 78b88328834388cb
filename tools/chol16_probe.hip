// Cycles per column of the 16-column diagonal-block factorization loop that bounds every register-resident
// Cholesky in csrc/chol.hip (the pivot chain), for several formulations, on ONE wave (standalone tool).
//   V0 "ref":   chol2_potrf_role's loop: L[c][j] broadcast from lane c after scaling (readlane of a[j]).
//   V1 "la":    + pivot lookahead: d_{j+1} = a_{j+1,j+1} - (a_{j+1,j} inv_j)^2 formed from scalars read
//               before the column's scaling (chol6's diagonal wave).
//   V2 "sym":   L[c][j] = A[j][c] * inv_j read from lane j's row (the block kept symmetric): the 15 - j
//               broadcasts of a column no longer wait for its pivot.
//   V3 "lasym": V1 + V2.
// Each variant factors the same SPD 16x16 block `reps` times (data reloaded each rep, every result
// stored, so nothing is hoisted) and checks L against V0 bit for bit.
//   hipcc -O3 --offload-arch=gfx950 tools/chol16_probe.hip -o tools/bin/chol16_probe
//   ./chol16_probe [reps] [waves_per_simd]
#include <hip/hip_runtime.h>

#include <cmath>
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

__device__ inline double rl(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ inline void sqrt_recip(double d, double& s, double& inv) {
  const double y0 = __builtin_amdgcn_rsq(d);
  const double h = d * y0;
  const double r = fma(-h, y0, 1.0);
  const double y1 = fma(0.5 * y0, r, y0);
  const double s0 = d * y1;
  const double rr = fma(-s0, s0, d);
  s = fma(rr, 0.5 * y1, s0);
  const double e = fma(-s, y1, 1.0);
  inv = fma(y1, e, y1);
}

template <int V>
__device__ __attribute__((always_inline)) inline void factor16(double (&a)[16], int lane) {
  if constexpr (V == 0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const double d = rl(a[j], j);
      double sj, inv;
      sqrt_recip(d, sj, inv);
      a[j] = (lane == j) ? sj : a[j] * inv;
#pragma unroll
      for (int c = j + 1; c < 16; ++c) a[c] = fma(-a[j], rl(a[j], c), a[c]);
    }
  } else if constexpr (V == 1) {
    double d = rl(a[0], 0);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      double bn = 0, an = 0;
      if (j < 15) {
        bn = rl(a[j], j + 1);
        an = rl(a[j + 1], j + 1);
      }
      double sj, inv;
      sqrt_recip(d, sj, inv);
      if (j < 15) {
        const double ln = bn * inv;
        d = fma(-ln, ln, an);
      }
      a[j] = (lane == j) ? sj : a[j] * inv;
#pragma unroll
      for (int c = j + 1; c < 16; ++c) a[c] = fma(-a[j], rl(a[j], c), a[c]);
    }
  } else if constexpr (V == 2) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const double d = rl(a[j], j);
      double s[16];
#pragma unroll
      for (int c = j + 1; c < 16; ++c) s[c] = rl(a[c], j);     // row j, final after column j - 1
      double sj, inv;
      sqrt_recip(d, sj, inv);
      a[j] = (lane == j) ? sj : a[j] * inv;
#pragma unroll
      for (int c = j + 1; c < 16; ++c) a[c] = fma(-a[j], s[c] * inv, a[c]);
    }
  } else {
    double d = rl(a[0], 0);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      double s[16];
#pragma unroll
      for (int c = j + 1; c < 16; ++c) s[c] = rl(a[c], j);
      double sj, inv;
      sqrt_recip(d, sj, inv);
      double an = 0;
      if (j < 15) an = rl(a[j + 1], j + 1);
      a[j] = (lane == j) ? sj : a[j] * inv;
      if (j < 15) {
        const double ln = s[j + 1] * inv;
        d = fma(-ln, ln, an);
      }
#pragma unroll
      for (int c = j + 1; c < 16; ++c) a[c] = fma(-a[j], s[c] * inv, a[c]);
    }
  }
}

template <int V>
__global__ __launch_bounds__(256) void probe(const double* A, double* out, unsigned long long* cyc, int reps) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ double blk[16 * 17];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) blk[(i >> 4) * 17 + (i & 15)] = A[i];
  __syncthreads();
  double acc = 0;
  unsigned long long t0 = 0, t1 = 0;
  for (int r = 0; r < reps; ++r) {
    if (r == 1) t0 = wall_clock64();
    double a[16];
    const int row = lane & 15;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      // lanes 0..15: the symmetric block (lower part mirrored), other lanes: rows of the same block
      const int rr = (c > row) ? c : row, cc = (c > row) ? row : c;
      a[c] = blk[rr * 17 + cc] + (double)r * 1e-300;
    }
    factor16<V>(a, lane);
#pragma unroll
    for (int c = 0; c < 16; ++c) acc += a[c];
    if (r == 0 && w == 0)
#pragma unroll
      for (int c = 0; c < 16; ++c) out[lane * 16 + c] = a[c];
  }
  t1 = wall_clock64();
  if (lane == 0) cyc[w] = t1 - t0;
  if (acc == 12345.678) out[0] = acc;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 2000;
  const int waves = argc > 2 ? atoi(argv[2]) : 1;
  std::vector<double> A(256);
  unsigned long long st = 7;
  std::vector<double> G(256);
  for (auto& g : G) {
    st = st * 6364136223846793005ULL + 1442695040888963407ULL;
    g = ((st >> 11) * (1.0 / 9007199254740992.0)) - 0.5;
  }
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k < 16; ++k) s += G[i * 16 + k] * G[j * 16 + k];
      A[i * 16 + j] = s + (i == j ? 1.0 : 0.0);
    }
  double *dA, *dO;
  unsigned long long* dC;
  HC(hipMalloc(&dA, 256 * 8));
  HC(hipMalloc(&dO, 4 * 1024 * 8));
  HC(hipMalloc(&dC, 64 * 8));
  HC(hipMemcpy(dA, A.data(), 256 * 8, hipMemcpyHostToDevice));
  int clk_khz = 0;
  HC(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0));
  std::vector<double> ref(1024), got(1024);
  const char* names[4] = {"ref", "la", "sym", "lasym"};
  for (int v = 0; v < 4; ++v) {
    const int threads = 64 * waves * 4;   // waves_per_simd waves on each of the 4 SIMDs
    auto launch = [&]() {
      if (v == 0) hipLaunchKernelGGL(probe<0>, dim3(1), dim3(threads), 0, 0, dA, dO + v * 1024, dC, reps);
      if (v == 1) hipLaunchKernelGGL(probe<1>, dim3(1), dim3(threads), 0, 0, dA, dO + v * 1024, dC, reps);
      if (v == 2) hipLaunchKernelGGL(probe<2>, dim3(1), dim3(threads), 0, 0, dA, dO + v * 1024, dC, reps);
      if (v == 3) hipLaunchKernelGGL(probe<3>, dim3(1), dim3(threads), 0, 0, dA, dO + v * 1024, dC, reps);
    };
    launch();
    HC(hipDeviceSynchronize());
    launch();
    HC(hipDeviceSynchronize());
    unsigned long long cyc[64];
    HC(hipMemcpy(cyc, dC, 64 * 8, hipMemcpyDeviceToHost));
    HC(hipMemcpy(got.data(), dO + v * 1024, 1024 * 8, hipMemcpyDeviceToHost));
    if (v == 0) ref = got;
    int diff = 0;
    for (int i = 0; i < 16 * 16; ++i) {   // lanes 0..15: the factor's lower triangle
      const int l = i / 16, c = i % 16;
      if (c <= l && ref[i] != got[i]) ++diff;
    }
    const double ns = (double)cyc[0] / (clk_khz * 1e-6) / (reps - 1);   // wall clock ticks -> ns per factorization
    printf("{\"variant\": \"%s\", \"waves_per_simd\": %d, \"ns_per_block\": %.1f, \"ns_per_column\": %.1f, "
           "\"lower_diff_vs_ref\": %d}\n", names[v], waves, ns, ns / 16, diff);
  }
  return 0;
}
