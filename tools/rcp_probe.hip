// Accuracy of the gfx950 f64 reciprocal / rsqrt estimates (v_rcp_f64, v_rsq_f64), with and without
// Newton steps, against correctly rounded references -- decides how many steps the Cholesky pivot
// chain needs.   hipcc -O3 --offload-arch=gfx950 tools/rcp_probe.hip -o tools/bin/rcp_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void probe(const double* x, double* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double d = x[i];
  const double r0 = __builtin_amdgcn_rcp(d);
  const double e = fma(-d, r0, 1.0);
  const double r1 = fma(r0, e, r0);
  const double q0 = __builtin_amdgcn_rsq(d);
  double h = d * q0, t = fma(-h, q0, 1.0);
  const double q1 = fma(0.5 * q0, t, q0);
  h = d * q1;
  t = fma(-h, q1, 1.0);
  const double q2 = fma(0.5 * q1, t, q1);
  out[6 * i + 0] = r0;
  out[6 * i + 1] = r1;
  out[6 * i + 2] = q0;
  out[6 * i + 3] = q1;
  out[6 * i + 4] = q2;
  out[6 * i + 5] = d * q1;  // sqrt estimate with one step
}

int main() {
  const int n = 1 << 20;
  std::vector<double> x(n), o(6 * (size_t)n);
  unsigned long long s = 88172645463325252ULL;
  for (auto& v : x) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    v = std::ldexp(1.0 + (s >> 11) * (1.0 / 9007199254740992.0), (int)(s % 40) - 20);
  }
  double *dx, *dout;
  hipMalloc(&dx, n * 8);
  hipMalloc(&dout, 6 * (size_t)n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  probe<<<n / 256, 256>>>(dx, dout, n);
  hipMemcpy(o.data(), dout, o.size() * 8, hipMemcpyDeviceToHost);
  double m[6] = {0};
  const double ulp = std::ldexp(1.0, -52);
  for (int i = 0; i < n; ++i) {
    const double r = 1.0 / x[i], q = 1.0 / std::sqrt(x[i]), sq = std::sqrt(x[i]);
    const double ref[6] = {r, r, q, q, q, sq};
    for (int k = 0; k < 6; ++k) m[k] = std::fmax(m[k], std::fabs(o[6 * (size_t)i + k] - ref[k]) / std::fabs(ref[k]) / ulp);
  }
  printf("max rel err in ulps: rcp %.3g  rcp+1NR %.3g  rsq %.3g  rsq+1NR %.3g  rsq+2NR %.3g  sqrt(d*rsq1) %.3g\n",
         m[0], m[1], m[2], m[3], m[4], m[5]);
  return 0;
}
