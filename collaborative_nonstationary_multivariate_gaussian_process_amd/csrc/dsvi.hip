// Row / reduction kernels of the closed-form DSVI step (NMGP.forward + its autograd backward,
// code/nmgp_dsvi.py:157-301; helpers code/utils.py:106-351).  The dense contractions of the step
// go through gemm.hip / chol.hip / pairwise.hip; these kernels do everything that is per row of
// the minibatch, per variational factor, or a final reduction:
//
//   dsvi_v        v = mu_v + chol(Sigma_v + lam I) z_v, ell_Z = exp(v)        (utils.py:226-227)
//   dsvi_trow     ell_X = exp(P_t v + z_t sqrt(s2_t - rowsum(P_t o K_t12) + lam))   (:228-236)
//   dsvi_recon    per row: the Q pair samples of its output (MGP_d, :106-125), the Gibbs
//                 marginals (MGP_mu_sigma2, :128-146), F, the Gaussian log-lik (:268-272) and
//                 every per-row adjoint of the closed-form backward
//   dsvi_kl       KL_Gaussian per variational factor, with the upper=True trace quirk (:332-351)
//   dsvi_tbwd     backward of the t-row          dsvi_vbwd  backward of v through chol(Sigma_v)
//   dsvi_finalize loss, scalar hyper-parameter gradients, mu gradients of the KL terms
//   adam / philox / counter
//
// One wave (64 lanes) per minibatch row: lanes stride over the M inducing columns and reduce
// with xor-shuffles; per-output quantities live one per lane (lane d, register d>>6).
#include "common.hpp"

namespace nmgp {

using Args = nmgp_dsvi_args;
constexpr double kLogSqrt2Pi = 0.91893853320467274178;   // log(sqrt(2 pi)), code/utils.py:271

__device__ inline void pair_ij(int q, int& i, int& j) {
  int r = (int)((sqrtf(8.0f * (float)q + 1.0f) - 1.0f) * 0.5f);
  while ((r + 1) * (r + 2) / 2 <= q) ++r;
  while (r * (r + 1) / 2 > q) --r;
  i = r;
  j = q - r * (r + 1) / 2;
}
// Block index of coefficient pair (i, j <= i) in mu_U / sqrt_U / Y_0 / Y_1: the reference's dense
// D x D layout, or the packed Q-pair layout (engine.param_layout)
// (pair sharding, SURVEY §8e axis 3: a rank holds only the packed pairs [pair_q0, pair_q0 + Q) -- the
// pairs (i, j <= i) of its contiguous range of outputs -- and its blocks are numbered from pair_q0)
__device__ inline int64_t pair_blk(const nmgp_dsvi_args& a, int i, int j) {
  return a.pair_packed ? (int64_t)i * (i + 1) / 2 + j - a.pair_q0 : (int64_t)i * a.D + j;
}
// position of pair (i, j) in the Q x B pair noise (reference call order, local pair window)
__device__ inline int64_t pair_noise(const nmgp_dsvi_args& a, int i, int j) {
  return (int64_t)i * (i + 1) / 2 + j - a.pair_q0;
}
__device__ inline int64_t pair_cols(const nmgp_dsvi_args& a) {
  return a.pair_packed ? (int64_t)a.Q : (int64_t)a.D * a.D;
}

// Variational factor order: f < nW latent functions W_f (nW = n_wfac: D, or 0 on a pair-sharded rank
// that does not own KL_W) | nW <= f < nW+Q coefficient pairs (i,j) in (i, j<=i) order, packed index
// pair_q0 + f - nW | f = NF-1 the length-scale process v.  Prior slot of factor f:
// 0 = t (v), 1 = L0 (off-diagonal pairs), 2 = L1 (diagonal pairs), 3 = G (W).
__device__ inline void fac_pair(const nmgp_dsvi_args& a, int f, int& i, int& j) {
  pair_ij(f - a.n_wfac + a.pair_q0, i, j);
}
__device__ inline int prior_of(const nmgp_dsvi_args& a, int f) {
  if (f < a.n_wfac) return 3;
  if (f == a.NF - 1) return 0;
  int i, j;
  fac_pair(a, f, i, j);
  return i == j ? 2 : 1;
}

// sum_{q < cnt} p[q * stride] in a fixed order with 8 loads in flight: written as a plain loop these
// partial-sum reductions waited one L2 round trip per element (63 G12 column partials in the v backward)
// 32 loads in flight per round (round 6: the pairwise backward's 8-row tiles made the G12 column partials 250 deep at
// PM2.5, and 8 in flight left the v backward 32 round trips long); fixed summation order
template <typename T> __device__ inline T strided_sum(const T* p, int cnt, int64_t stride) {
  constexpr int U = 32;
  T acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = 0;
  for (int q = 0; q < cnt; q += U) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = (q + u < cnt) ? p[(int64_t)(q + u) * stride] : (T)0;
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] += v[u];
  }
#pragma unroll
  for (int h = U / 2; h > 0; h >>= 1)
#pragma unroll
    for (int u = 0; u < h; ++u) acc[u] += acc[u + h];
  return acc[0];
}

template <typename T> struct RowBuf {
  T* base;
  int64_t B;
  int D;
  __device__ T* mbar(int d) const { return base + (int64_t)d * B; }
  __device__ T* sbar(int s) const { return base + (int64_t)(D + s) * B; }
  __device__ T* cG() const { return base + (int64_t)(2 * D) * B; }
  __device__ T* c0() const { return base + (int64_t)(2 * D + 1) * B; }
  __device__ T* c1() const { return base + (int64_t)(2 * D + 2) * B; }
  __device__ T* tbar() const { return base + (int64_t)(2 * D + 3) * B; }
  __device__ T* varbar() const { return base + (int64_t)(2 * D + 4) * B; }
};

template <typename T> __device__ inline T hyp(const Args& a, int k) {
  return dexp(((const T*)a.theta)[a.off_hyp + k]);
}

// value of lane (d & 63), register (d >> 6), broadcast to the wave
template <typename T, int NR> __device__ inline T bcast(const T (&r)[NR], int d) {
  T v = 0;
#pragma unroll
  for (int u = 0; u < NR; ++u)
    if ((d >> 6) == u) v = shfl(r[u], d & 63);
  return v;
}
template <typename T, int NR> __device__ inline void setlane(T (&r)[NR], int d, int lane, T v) {
#pragma unroll
  for (int u = 0; u < NR; ++u)
    if ((d >> 6) == u && lane == (d & 63)) r[u] = v;
}

// Marginal variances of the sampled GPs (k11 - rowsum(P o K12) [+ ||P L||^2]).  fp64 keeps the
// reference's arithmetic exactly; in fp32 the cancellation can leave them a few ulps of k11 below 0
// and sqrt(var + 1e-4) would turn NaN on ill-conditioned K22, so they are floored at 0.
template <typename T> __device__ inline T var_floor(T v) { return v; }
template <> __device__ inline float var_floor<float>(float v) { return v > 0.f ? v : 0.f; }

// ------------------------------------------------------------------------------------ v
template <typename T>
__global__ __launch_bounds__(256) void dsvi_v_kernel(Args a) {
  const int M = a.M, lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= M) return;
  const T* zv = (const T*)a.noise;
  if (a.v64) {
    // fp32 engines: the sample from the fp64 factor, in fp64 (an fp32 factor of Sigma_v + 1e-4 I left the
    // ECoG-like fixture's compute_ELBO samples ~1e-3 off: exp(v) turns v's absolute error into relative
    // error of every Gibbs length scale)
    const double* Cv = (const double*)a.v64;
    double s = 0;
    for (int k = lane; k <= c; k += 64) s += Cv[(int64_t)c * M + k] * (double)zv[k];
    s = wave_sum(s);
    if (lane == 0) {
      const double v = (double)((const T*)a.theta)[a.off_muv + c] + s;
      const double ez = exp(v);
      ((T*)a.v)[c] = (T)v;
      ((T*)a.ellZ)[c] = (T)ez;
      ((double*)a.ellZ64)[c] = ez;
    }
    return;
  }
  const T* Cv = (const T*)a.Afac + (int64_t)(a.NF - 1) * M * M;   // C1 of the v factor (Sigma_v)
  T s = 0;
  for (int k = lane; k <= c; k += 64) s += Cv[(int64_t)c * M + k] * zv[k];
  s = wave_sum(s);
  if (lane == 0) {
    const T v = ((const T*)a.theta)[a.off_muv + c] + s;
    ((T*)a.v)[c] = v;
    ((T*)a.ellZ)[c] = dexp(v);
  }
}

// ------------------------------------------------------------------------------------ v + K_G22 (round 6)
// The v sample and the Gibbs prior's K22 + jitter I in ONE wide launch (the fused-prior schedule, engine.py
// fuse_tp): one workgroup per lower 16 x 16 tile (I, J) of K_G22 forms the v entries its rows and columns need --
// dsvi_v_kernel's arithmetic per entry, v_c = mu_v[c] + sum_k L_v[c, k] z_v[k] (code/utils.py:226-227), ell_Z = exp(v)
// -- then its 256 elements, one per thread, with pairwise_kernel's Gibbs arithmetic (code/utils.py:97-103).  The
// diagonal tiles write v / ell_Z out.  Replaces the v launch + the 32-workgroup K_G22 builder (8 exp / sqrt /
// division chains per thread) on the critical path.
template <typename T>
__global__ __launch_bounds__(256) void dsvi_vg22_kernel(Args a) {
  __shared__ T vl[32];
  const int M = a.M, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int I = (int)((sqrtf(8.0f * (float)blockIdx.x + 1.0f) - 1.0f) * 0.5f);
  while ((I + 1) * (I + 2) / 2 <= (int)blockIdx.x) ++I;
  while (I * (I + 1) / 2 > (int)blockIdx.x) --I;
  const int J = (int)blockIdx.x - I * (I + 1) / 2;
  const T* zv = (const T*)a.noise;
  const T* Cv = (const T*)a.Afac + (int64_t)(a.NF - 1) * M * M;   // L of Sigma_v (factored in place)
  // entries q < 16: rows I*16 + q; q >= 16: columns J*16 + q - 16 (I == J: the rows only)
  const int nq = I == J ? 16 : 32;
  for (int q = w; q < nq; q += 4) {
    const int c = q < 16 ? I * 16 + q : J * 16 + q - 16;
    T sacc = 0;
    if (c < M)
      for (int k = lane; k <= c; k += 64) sacc += Cv[(int64_t)c * M + k] * zv[k];
    sacc = wave_sum(sacc);
    if (lane == 0) {
      const T v = c < M ? ((const T*)a.theta)[a.off_muv + c] + sacc : (T)0;
      vl[q] = v;
      if (I == J && c < M) {
        ((T*)a.v)[c] = v;
        ((T*)a.ellZ)[c] = dexp(v);
      }
    }
  }
  __syncthreads();
  const int r = threadIdx.x >> 4, cc = threadIdx.x & 15;
  const int i = I * 16 + r, j = J * 16 + cc;
  if (i >= M || j >= M) return;
  const T* Z = (const T*)a.Z;
  const T lx = dexp(vl[r]), lz = dexp(vl[I == J ? cc : 16 + cc]);
  T r2 = 0;
  const T dd = Z[i] / (T)1 - Z[j] / (T)1;
  r2 += dd * dd;
  const T S = lx * lx + lz * lz;
  const T C = dsqrt((T)2 * (lx * lz) / S);
  T k = (T)1 * C * dexp(-r2 / S);
  if (i == j) k += (T)a.jitter;
  ((T*)a.Afac)[(int64_t)(a.NF + 3) * M * M + (int64_t)i * M + j] = k;
}

// ------------------------------------------------------------------------------------ t-row
template <typename T>
__global__ __launch_bounds__(256) void dsvi_trow_kernel(Args a) {
  const int M = a.M, B = a.B, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  const T* Pt = (const T*)a.P + (int64_t)r * M;       // slot 0 = t
  const T* Tt = (const T*)a.T + (int64_t)r * M;       // K_t12 C_t^-T: rowsum(P o K12) = ||T_row||^2
  const double* Tt64 = a.T64 ? (const double*)a.T64 + (int64_t)r * M : nullptr;
  const T* v = (const T*)a.v;
  T mean = 0;
  double q = 0;                                       // (fp64 sum of fp64 T rows in fp32 engines)
  for (int c = lane; c < M; c += 64) {
    mean += Pt[c] * v[c];
    if (Tt64) {
      const double tt = Tt64[c];
      q += tt * tt;
    } else {
      const T tt = Tt[c];
      q += (double)(tt * tt);
    }
  }
  mean = wave_sum(mean);
  q = wave_sum(q);
  if (lane == 0) {
    // k11 - ||T||^2 cancels to ~ the jitter on smooth priors: formed in fp64 when T64 is given
    const T var = var_floor((T)((double)hyp<T>(a, 0) - q));
    const T zt = ((const T*)a.noise)[M + r];
    const T tl = mean + zt * dsqrt(var + (T)a.jitter);
    ((T*)a.ellX)[r] = dexp(tl);
    ((T*)a.var_t)[r] = var;
  }
}

// ------------------------------------------------------------------------------------ recon
// training (elbo_mode 0): row r of output o uses pairs (o, s) for s <= o  -> l_r[s] = L[o,s,r]
// ELBO     (elbo_mode 1): row r uses pairs (s, o) for s >= o (column gather, nmgp_dsvi.py:361)
//
// One workgroup per row, columns across the 256 threads: the row's 3 + 4*ns dot products (ns =
// latent functions / pairs the row uses) are formed column-parallel with every load independent,
// reduced per wave then across the 4 waves in LDS; wave 0 forms the row's likelihood and per-s
// adjoints; all threads then scale the W rows and build the P-bar rows column-parallel.  Enough
// rows in flight (B workgroups, 4 waves each) to cover HBM latency.
template <typename T>
__global__ __launch_bounds__(256) void dsvi_recon_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int M = a.M, B = a.B, D = a.D;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int r = blockIdx.x;
  const bool elbo = a.elbo_mode != 0;
  const int o = a.row_out[r];
  const int slo = elbo ? o : 0, shi = elbo ? D - 1 : o, ns = shi - slo + 1;
  const int K = 3 + 4 * ns;                 // dot products of this row
  T* part = (T*)smem_raw;                   // [4 waves][K] wave partials
  T* sv = part + 4 * (3 + 4 * D);           // per-s results: fg, fp, mbar, sbar  (4 x D)
  T* scal = sv + 4 * D;                     // cg, c0, c1
  const T lam = (T)a.jitter;
  const T* th = (const T*)a.theta;
  const T s20 = hyp<T>(a, 2), s21 = hyp<T>(a, 4), s2e = hyp<T>(a, 6);
  const int64_t BM = (int64_t)B * M;
  const T* K12 = (const T*)a.K12;
  const T* P = (const T*)a.P;
  const T* PG = P + 3 * BM + (int64_t)r * M;
  const T* KG = K12 + 3 * BM + (int64_t)r * M;
  const T* P0 = P + 1 * BM + (int64_t)r * M;
  const T* K0 = K12 + 1 * BM + (int64_t)r * M;
  const T* P1 = P + 2 * BM + (int64_t)r * M;
  const T* K1 = K12 + 2 * BM + (int64_t)r * M;
  // Nystrom variances rowsum(P o K12) as ||K12 C2^-T||^2 per row: a sum of squares instead of the
  // cancellation 1 - rowsum(P o K12) of an explicit-inverse product (fp32 on smooth priors)
  const T* TG = (const T*)a.T + 3 * BM + (int64_t)r * M;
  const T* T0 = (const T*)a.T + 1 * BM + (int64_t)r * M;
  const T* T1 = (const T*)a.T + 2 * BM + (int64_t)r * M;
  T* WG = (T*)a.WG;
  T* WP = (T*)a.WP;
  const T* muW = th + a.off_muW;
  const T* muU = th + a.off_muU;
  const T* noise = (const T*)a.noise;

  // ---- phase 1: column-parallel dot products
  // (fp32 engines with T64: the three Nystrom sums in fp64 -- the variances k11 - ||T_row||^2 cancel to
  //  ~ the jitter on smooth priors -- kept as fp64 partials in qd[] and summed by wave 0 below)
  __shared__ double qd[4][3];
  if (a.T64) {
    const double* T64 = (const double*)a.T64 + (int64_t)r * M;
    double q[3] = {0, 0, 0};
    for (int c = t; c < M; c += 256) {
      const double g = T64[3 * BM + c], u0 = T64[1 * BM + c], u1 = T64[2 * BM + c];
      q[0] += g * g;
      q[1] += u0 * u0;
      q[2] += u1 * u1;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double v = wave_sum(q[k]);
      if (lane == 0) qd[w][k] = v;
    }
  } else {
    T q[3] = {0, 0, 0};
    for (int c = t; c < M; c += 256) {
      q[0] += TG[c] * TG[c];
      q[1] += T0[c] * T0[c];
      q[2] += T1[c] * T1[c];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const T v = wave_sum(q[k]);
      if (lane == 0) part[w * K + k] = v;
    }
  }
  for (int u = 0; u < ns; ++u) {
    const int s = slo + u;
    const int pi = elbo ? s : o, pj = elbo ? o : s;
    const T* Pk = (s == o) ? P1 : P0;
    const T* wg = WG + (int64_t)s * BM + (int64_t)r * M;
    const T* wp = WP + (int64_t)s * BM + (int64_t)r * M;
    const T* mw = muW + (int64_t)s * M;
    const T* mu = muU + pair_blk(a, pi, pj) * M;
    T d4[4] = {0, 0, 0, 0};
    for (int c = t; c < M; c += 256) {
      const T x = wg[c], y = wp[c];
      d4[0] += PG[c] * mw[c];
      d4[1] += x * x;
      d4[2] += Pk[c] * mu[c];
      d4[3] += y * y;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const T v = wave_sum(d4[k]);
      if (lane == 0) part[w * K + 3 + 4 * u + k] = v;
    }
  }
  __syncthreads();

  // ---- phase 2 (wave 0): likelihood of the row and the per-s adjoints
  T Rrow = 0, epart = 0, c0p = 0, c1p = 0;
  if (w == 0) {
    auto tot = [&](int k) { return part[k] + part[K + k] + part[2 * K + k] + part[3 * K + k]; };
    // residual prior variances k11 - ||T_row||^2 (G: k11 = 1); fp64 when T64 is given
    T rG, r0, r1;
    if (a.T64) {
      auto totd = [&](int k) { return qd[0][k] + qd[1][k] + qd[2][k] + qd[3][k]; };
      rG = (T)(1.0 - totd(0));
      r0 = (T)((double)s20 - totd(1));
      r1 = (T)((double)s21 - totd(2));
    } else {
      rG = (T)1 - tot(0);
      r0 = s20 - tot(1);
      r1 = s21 - tot(2);
    }
    T lm = 0, lg = 0;
    for (int u = lane; u < ns; u += 64) {
      const int s = slo + u;
      const int pi = elbo ? s : o, pj = elbo ? o : s;
      const bool diag = (s == o);
      const T m = tot(3 + 4 * u), g = rG + tot(4 + 4 * u);
      const T s2p = var_floor((diag ? r1 : r0) + tot(6 + 4 * u));
      const T sd = dsqrt(s2p + lam);
      const T zz = noise[M + B + pair_noise(a, pi, pj) * B + r];
      const T smp = tot(5 + 4 * u) + zz * sd;
      const T l = diag ? dexp(smp) : smp;
      lm += l * m;
      lg += l * l * g;
    }
    const T F = wave_sum(lm);
    lg = wave_sum(lg);
    const T sc = dsqrt(s2e);
    const T var = sc * sc;
    const T res = ((const T*)a.y)[r] - F;
    Rrow = -(res * res) / ((T)2 * var) - dlog(sc) - (T)kLogSqrt2Pi - ((T)0.5 / s2e) * lg;
    if (!elbo) {
      const T cc = -(T)a.N_over_B;
      const T Fbar = cc * res / var;
      RowBuf<T> rb{(T*)a.rowbuf, B, D};
      T cg = 0, c0 = 0, c1 = 0;
      for (int s = lane; s < D; s += 64) {
        T mbar = 0, gbar = 0, sbar = 0, s2pb = 0;
        if (s <= o) {
          const int u = s;                      // training: slo = 0
          const bool diag = (s == o);
          const T m = tot(3 + 4 * u), g = rG + tot(4 + 4 * u);
          const T s2p = var_floor((diag ? r1 : r0) + tot(6 + 4 * u));
          const T sd = dsqrt(s2p + lam);
          const T zz = noise[M + B + pair_noise(a, o, s) * B + r];
          const T smp = tot(5 + 4 * u) + zz * sd;
          const T l = diag ? dexp(smp) : smp;
          mbar = Fbar * l;
          gbar = cc * (-(l * l) / ((T)2 * s2e));
          const T lbar = Fbar * m + cc * (-(l * g) / s2e);
          sbar = diag ? lbar * l : lbar;
          s2pb = sbar * zz / ((T)2 * sd);
          cg += gbar;
          if (s < o) c0 += s2pb; else c1 = s2pb;
          sv[s] = (T)2 * gbar;
          sv[D + s] = (T)2 * s2pb;
          sv[2 * D + s] = mbar;
          sv[3 * D + s] = sbar;
        }
        rb.mbar(s)[r] = mbar;
        rb.sbar(s)[r] = sbar;
      }
      cg = wave_sum(cg);
      c0 = wave_sum(c0);
      c1 = wave_sum(c1);                        // one lane holds it
      c0p = c0;
      c1p = c1;
      epart = cc * ((res * res / (sc * sc * sc) - (T)1 / sc) / ((T)2 * sc) + (T)0.5 * lg / (s2e * s2e)) * s2e;
      if (lane == 0) {
        scal[0] = cg;
        scal[1] = c0;
        scal[2] = c1;
        rb.cG()[r] = cg;
        rb.c0()[r] = c0;
        rb.c1()[r] = c1;
      }
    }
    if (lane == 0) {
      T* rp = (T*)a.red + (int64_t)r * 4;
      rp[0] = Rrow;
      rp[1] = epart;
      rp[2] = c0p;
      rp[3] = c1p;
    }
  }
  if (elbo) return;
  __syncthreads();

  // ---- phase 3: W-hat = diag(2 adjoint) W, W / W_P scaled in place, and the P-bar initial rows.  (Rows of
  // factors s > o are neither computed by the W GEMM nor read by any backward product -- those take factor s
  // over the rows of outputs >= s only -- so they are left alone; round 3 zeroed them.)
  const T cg = scal[0], c0 = scal[1], c1 = scal[2];
  for (int s = 0; s <= o; ++s) {
    const T fg = sv[s], fp = sv[D + s];
    T* wg = WG + (int64_t)s * BM + (int64_t)r * M;
    T* wp = WP + (int64_t)s * BM + (int64_t)r * M;
    for (int c = t; c < M; c += 256) {
      wg[c] *= fg;
      wp[c] *= fp;
    }
  }
  T* PbG = (T*)a.Pbar + 3 * BM + (int64_t)r * M;
  T* Pb0 = (T*)a.Pbar + 1 * BM + (int64_t)r * M;
  T* Pb1 = (T*)a.Pbar + 2 * BM + (int64_t)r * M;
  for (int c = t; c < M; c += 256) {
    T acc = -cg * KG[c];
    for (int d = 0; d <= o; ++d) acc += sv[2 * D + d] * muW[(int64_t)d * M + c];
    PbG[c] = acc;
    acc = -c0 * K0[c];
    for (int j = 0; j < o; ++j) acc += sv[3 * D + j] * muU[pair_blk(a, o, j) * M + c];
    Pb0[c] = acc;
    Pb1[c] = sv[3 * D + o] * muU[pair_blk(a, o, o) * M + c] - c1 * K1[c];
  }
}

// ------------------------------------------------------------------------------------ KL
template <typename T> __device__ inline const T* fac_S(const Args& a, int f) {
  const T* th = (const T*)a.theta;
  const int64_t MM = (int64_t)a.M * a.M;
  if (f < a.n_wfac) return th + a.off_sW + f * MM;
  if (f == a.NF - 1) return th + a.off_sv;
  int i, j;
  fac_pair(a, f, i, j);
  return th + a.off_sU + pair_blk(a, i, j) * MM;
}
template <typename T> __device__ inline const T* fac_mu(const Args& a, int f) {
  const T* th = (const T*)a.theta;
  if (f < a.n_wfac) return th + a.off_muW + (int64_t)f * a.M;
  if (f == a.NF - 1) return th + a.off_muv;
  int i, j;
  fac_pair(a, f, i, j);
  return th + a.off_muU + pair_blk(a, i, j) * a.M;
}
template <typename T> __device__ inline const T* fac_y(const Args& a, int f) {
  const T* Y = (const T*)a.Y;
  const int D = a.D, M = a.M;
  if (f < a.n_wfac) return Y + (int64_t)f * M;
  if (f == a.NF - 1) return Y + (int64_t)D * M;
  int i, j;
  fac_pair(a, f, i, j);
  const int64_t base = (int64_t)(D + 1) * M + (i == j ? pair_cols(a) * M : 0);
  return Y + base + pair_blk(a, i, j) * M;
}

// KL per factor, parallel over (factor, 16-row slab): 16 lanes per row sum tril(S)_i. squared
// (A1_ii - lam) with independent loads, then the per-row logdet / trace-quirk / Mahalanobis terms;
// each block leaves 4 partial sums in klpart[f][slab], summed in slab order by the finalize kernel.
constexpr int KL_ROWS = 16;
template <typename T> __device__ inline T* kl_part(const Args& a) {
  return (T*)a.facbuf + a.NF + 8 * (int64_t)a.M + 4 * pair_cols(a) + (int64_t)a.NF * a.M;
}

template <typename T>
__global__ __launch_bounds__(256) void dsvi_kl_kernel(Args a) {
  __shared__ T red[4][16];
  const int M = a.M, D = a.D, NF = a.NF;
  const int64_t MM = (int64_t)M * M;
  const T lam = (T)a.jitter;
  const T* Af = (const T*)a.Afac;
  T* fb = (T*)a.facbuf;
  // blocks 0 .. kl_f1 - kl_f0 - 1: the factors of the KL range; the one after them: the v factor
  const int f = blockIdx.x < a.kl_f1 - a.kl_f0 ? a.kl_f0 + (int)blockIdx.x : NF - 1;
  const int k = prior_of(a, f), slab = blockIdx.y;
  const int q = threadIdx.x & 15, i = slab * KL_ROWS + (threadIdx.x >> 4);
  const T* S = fac_S<T>(a, f);
  T ld1 = 0, ld2 = 0, t2 = 0, t3 = 0;
  T sq = 0;
  if (i < M) {
    constexpr int V = 16 / (int)sizeof(T);
    const T* Si = S + (int64_t)i * M;
    if (M % V == 0 && (((uintptr_t)Si) & 15) == 0) {
      // 16-byte loads (the ECoG KL reads 17.6 GB of lower triangles per step: 3.1 TB/s with single elements)
      struct alignas(16) Vv { T e[V]; };
      for (int c = V * q; c <= i; c += 16 * V) {
        const Vv x = *(const Vv*)(Si + c);
#pragma unroll
        for (int e = 0; e < V; ++e) sq += (c + e <= i) ? x.e[e] * x.e[e] : (T)0;
      }
    } else {
      for (int c = q; c <= i; c += 16) {
        const T x = Si[c];
        sq += x * x;
      }
    }
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
  if (i < M && q == 0) {
    const T* C1 = Af + (int64_t)f * MM;
    const T* C2 = Af + (int64_t)(NF + k) * MM;
    const T a1 = sq + lam;
    const T c2 = C2[(int64_t)i * M + i];
    ld1 = dlog(C1[(int64_t)i * M + i]);
    ld2 = dlog(c2);
    t2 = a1 / (c2 * c2);
    t3 = fac_mu<T>(a, f)[i] * fac_y<T>(a, f)[i];
    T* ev = fb + NF + 8 * (int64_t)M + 4 * pair_cols(a) + (int64_t)f * M;
    ev[i] = (T)0.5 - (T)0.5 * a1 / (c2 * c2);   // d KL / d C2_ii * C2_ii / 2 + 1/2
  }
  // rows of this block in order: lane 0 of each 16-lane group holds one row's terms
  T v[4] = {ld1, ld2, t2, t3};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    T x = v[j];
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) x += __shfl_xor(x, o, 64);   // the 4 rows of this wave
    if ((threadIdx.x & 63) == 0) red[j][threadIdx.x >> 6] = x;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int j = threadIdx.x;
    const T tot = red[j][0] + red[j][1] + red[j][2] + red[j][3];
    kl_part<T>(a)[((int64_t)f * gridDim.y + slab) * 4 + j] = tot;
  }
}

// delta_k[i] = sum over the factors of prior k of e_f[i];  wvec_k[i] = 1 / C2_ii^2
template <typename T>
__global__ __launch_bounds__(256) void dsvi_delta_kernel(Args a) {
  const int M = a.M, D = a.D, NF = a.NF;
  const int64_t MM = (int64_t)M * M;
  const int k = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  T* fb = (T*)a.facbuf;
  const T* C2 = (const T*)a.Afac + (int64_t)(NF + k) * MM;
  const T* ev = fb + NF + 8 * (int64_t)M + 4 * pair_cols(a);
  T acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int f = 0; f < NF; f += 8) {                 // 8 loads in flight (see strided_sum)
    T v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = (f + u < NF && prior_of(a, f + u) == k) ? ev[(int64_t)(f + u) * M + i] : (T)0;
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] += v[u];
  }
  const T dl = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  const T c2 = C2[(int64_t)i * M + i];
  fb[NF + (int64_t)k * M + i] = dl;
  fb[NF + 4 * (int64_t)M + (int64_t)k * M + i] = (T)1 / (c2 * c2);
}

// ------------------------------------------------------------------------------------ t backward
template <typename T>
__global__ __launch_bounds__(256) void dsvi_tbwd_kernel(Args a) {
  __shared__ T red[16];
  const int M = a.M, B = a.B, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  T vb = 0;
  if (r < B) {
    const T* gr = (const T*)a.gib_row;    // G12 row partials (n_ct x B)
    T ex = 0;
    for (int ct = 0; ct < a.n_ct; ++ct) ex += gr[(int64_t)ct * B + r];
    const T tbar = ex * ((const T*)a.ellX)[r];
    const T sd = dsqrt(((const T*)a.var_t)[r] + (T)a.jitter);
    const T zt = ((const T*)a.noise)[M + r];
    const T varbar = tbar * zt / ((T)2 * sd);
    const T* v = (const T*)a.v;
    if (a.t64) {
      // fp32 engines: P-bar_t and varbar in fp64 from the fp64 K_t12 (the t-prior adjoints are formed
      // in fp64 from here on); the per-4-row varbar partials below go to the fp64 workspace as well
      const double* Kt = (const double*)a.K12_64 + (int64_t)r * M;
      double* Pb = (double*)a.t64 + (int64_t)r * M;
      const double tb = tbar, vb64 = varbar;
      for (int c = lane; c < M; c += 64) Pb[c] = tb * (double)v[c] - vb64 * Kt[c];
      if (lane == 0) ((double*)a.t64)[(int64_t)B * M + r] = vb64;
    } else {
      const T* Kt = (const T*)a.K12 + (int64_t)r * M;
      T* Pb = (T*)a.Pbar + (int64_t)r * M;
      for (int c = lane; c < M; c += 64) Pb[c] = tbar * v[c] - varbar * Kt[c];
    }
    if (lane == 0) {
      RowBuf<T> rb{(T*)a.rowbuf, B, a.D};
      rb.tbar()[r] = tbar;
      rb.varbar()[r] = varbar;
    }
    vb = (lane == 0) ? varbar : (T)0;
  }
  if (a.t64) {
    __shared__ double red64[16];
    const double v64 = block_sum((double)vb, red64);
    if (threadIdx.x == 0) ((double*)a.t64)[(int64_t)B * M + B + blockIdx.x] = v64;
  }
  vb = block_sum(vb, red);
  if (threadIdx.x == 0) ((T*)a.red)[(int64_t)a.nblk_rows * 4 + blockIdx.x] = vb;
}

// ------------------------------------------------------------------------------------ v backward
// vbar = P_t^T tbar (a.vbar[0:M]) + ell_Z * dL/dell_Z  -> a.vbar[M:2M];  w = C_v^T vbar ;
// Psi = Phi + Phi^T with Phi = tril(w z_v^T), diagonal halved (Cholesky backward).
// Grid over row blocks of Psi: every block rebuilds vbar (cheap, coalesced partial sums), computes w
// for its VBW_ROWS rows (one wave-reduction each) and writes those rows and the mirrored columns.
constexpr int VBW_ROWS = 8;
template <typename T>
__global__ __launch_bounds__(256) void dsvi_vbwd_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  T* vbs = (T*)smem_raw;
  T* wrow = vbs + a.M;
  const int M = a.M, B = a.B;
  const T* gcol = (const T*)a.gib_col;
  const T* grow = (const T*)a.gib_row;
  const T* ellZ = (const T*)a.ellZ;
  T* vbar = (T*)a.vbar;
  for (int c = threadIdx.x; c < M; c += blockDim.x) {
    T ez = strided_sum(gcol + c, a.n_rt, M);                                         // G12 columns
    ez += strided_sum(grow + (int64_t)a.n_ct * B + c, a.n_ct, M);                     // G22 rows
    ez += strided_sum(gcol + (int64_t)a.n_rt * M + c, a.n_rt22, M);                   // G22 cols
    const T vb = vbar[c] + ez * ellZ[c];
    vbs[c] = vb;
    if (blockIdx.x == 0) vbar[M + c] = vb;
  }
  __syncthreads();
  const T* Cv = (const T*)a.Afac + (int64_t)(a.NF - 1) * M * M;
  const int i0 = blockIdx.x * VBW_ROWS;
  {
    // w_i = sum_{k >= i} C_v[k][i] vbar[k] for the block's VBW_ROWS rows: thread t walks rows k of
    // C_v and reads the VBW_ROWS consecutive entries (i0 .. i0+7) of each (one contiguous segment per
    // row; a wave per i with lanes over k touched 64 cache lines per load), then one block reduction
    // per i in a fixed order
    T sp[VBW_ROWS];
#pragma unroll
    for (int r = 0; r < VBW_ROWS; ++r) sp[r] = 0;
    for (int k = i0 + (int)threadIdx.x; k < M; k += blockDim.x) {
      const T vk = vbs[k];
      const T* row = Cv + (int64_t)k * M + i0;
#pragma unroll
      for (int r = 0; r < VBW_ROWS; ++r)
        if (i0 + r <= k) sp[r] += row[r] * vk;
    }
    T* red = wrow + VBW_ROWS;   // 4 waves x VBW_ROWS partials
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < VBW_ROWS; ++r) {
      const T v = wave_sum(sp[r]);
      if (lane == 0) red[wv * VBW_ROWS + r] = v;
    }
    __syncthreads();
    if (threadIdx.x < VBW_ROWS) {
      const int r = threadIdx.x;
      wrow[r] = ((red[r] + red[VBW_ROWS + r]) + red[2 * VBW_ROWS + r]) + red[3 * VBW_ROWS + r];
    }
  }
  __syncthreads();
  const T* zv = (const T*)a.noise;
  T* phi = (T*)a.phi;
  for (int r = 0; r < VBW_ROWS; ++r) {
    const int i = i0 + r;
    if (i >= M) break;
    const T wi = wrow[r];
    for (int j = threadIdx.x; j <= i; j += blockDim.x) {
      const T v = wi * zv[j];
      phi[(int64_t)i * M + j] = v;     // row i, j <= i (diagonal: w_i z_i, the halved sum)
      if (j < i) phi[(int64_t)j * M + i] = v;
    }
  }
}

// ------------------------------------------------------------------------------------ mu gradients
// KL mean gradients A2^{-1} mu (Y) into the mu_W / mu_U gradient rows (live pairs j <= i only) and
// mu_v += vbar + Y_t: one grid-strided element-wise pass, launched on the side stream after the last
// writers of those rows (the mu-bar products of bwd_lbar and the v backward), off the main chain.
// values the KL mean-gradient pass updates: mu_W (D M), mu_v (M), mu_U (pair columns x M)
__device__ inline int64_t mugrad_count(const nmgp_dsvi_args& a) {
  return (int64_t)a.D * a.M + a.M + pair_cols(a) * a.M;
}
template <typename T> __device__ inline void mugrad_body(const Args& a, int64_t i0, int64_t stride) {
  const int D = a.D, M = a.M;
  T* __restrict__ gw = (T*)a.grad;
  const T* __restrict__ Y = (const T*)a.Y;
  const T* __restrict__ vbar = (const T*)a.vbar + M;   // completed by the v-backward kernel
  const int64_t DM = (int64_t)D * M, DDM = pair_cols(a) * M;
  const int64_t yu0 = (int64_t)(D + 1) * M, yu1 = yu0 + DDM;
  const int64_t n = DM + M + DDM;
  for (int64_t i = i0; i < n; i += stride) {
    if (i < DM) {
      if (a.n_wfac > 0) gw[a.off_muW + i] = gw[a.off_muW + i] + Y[i];
    } else if (i < DM + M) {
      const int64_t c = i - DM;
      gw[a.off_muv + c] += a.kl_v ? vbar[c] + Y[DM + c] : vbar[c];
    } else {
      const int64_t idx = i - DM - M;
      const int ij = (int)(idx / M);
      int pi, pj;
      if (a.pair_packed) {
        pair_ij(ij + a.pair_q0, pi, pj);
      } else {
        pi = ij / D;
        pj = ij - pi * D;
      }
      if (pj <= pi) gw[a.off_muU + idx] = gw[a.off_muU + idx] + Y[(pi == pj ? yu1 : yu0) + idx];
    }
  }
}
template <typename T>
__global__ __launch_bounds__(256) void dsvi_mugrad_kernel(Args a) {
  mugrad_body<T>(a, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

// ------------------------------------------------------------------------------------ finalize
// The recon row partials and the per-factor KL slabs are final right after recon / the KL kernel,
// long before the last backward kernels: in training steps dsvi_prefinal_kernel (side stream, after
// recon) reduces them into out[8..14], and the finalize kernel at the end of the main chain only sums
// the late partials (t-row backward, the RBF / Gibbs builder backward scalars) and adds those.
template <typename T>
__device__ inline void sum_recon_kl(const Args& a, T (&acc)[20], T* klstage) {
  const int D = a.D, M = a.M, NF = a.NF;
  const T* rp = (const T*)a.red;
  const int t = threadIdx.x;
  constexpr int RU = 4;
  const int nbr = a.nblk_rows;                                     // recon: one partial per row
  T rv[RU][4];
#pragma unroll
  for (int u = 0; u < RU; ++u) {
    const int b = min(t + u * 1024, nbr - 1);
#pragma unroll
    for (int k = 0; k < 4; ++k) rv[u][k] = rp[b * 4 + k];
  }
#pragma unroll
  for (int u = 0; u < RU; ++u)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] += keep_if(rv[u][k], t + u * 1024 < nbr);
  for (int b = t + RU * 1024; b < nbr; b += 1024)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] += rp[b * 4 + k];
  const int nslab = (M + KL_ROWS - 1) / KL_ROWS;
  const T* kp = kl_part<T>(a);
  constexpr int CH = 1024;
  const int fpc = CH / nslab;
  for (int fb = 0; fb < NF; fb += fpc) {
    const int nf = min(fpc, NF - fb), base = fb * nslab, n = nf * nslab;
    if (t < n) {
      T q[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) q[j] = kp[(int64_t)(base + t) * 4 + j];
#pragma unroll
      for (int j = 0; j < 4; ++j) klstage[t * 4 + j] = q[j];
    }
    __syncthreads();
    for (int f = fb + t; f < fb + nf; f += blockDim.x) {
      T p[4] = {0, 0, 0, 0};
      for (int sl = 0; sl < nslab; ++sl)
        for (int j = 0; j < 4; ++j) p[j] += klstage[((f - fb) * nslab + sl) * 4 + j];
      // (factors outside the KL range -- and the v factor on a rank without KL_v -- were never launched:
      //  no -M/2 constant for them either)
      const bool on = f == NF - 1 ? a.kl_v != 0 : (f >= a.kl_f0 && f < a.kl_f1);
      const T v = on ? p[1] - p[0] + (T)0.5 * (p[2] + p[3] - (T)M) : (T)0;
      ((T*)a.facbuf)[f] = v;                   // per-factor KL (kept for inspection)
      // static indices only: a computed index into acc[] put the whole array in scratch memory
      if (f < a.n_wfac) acc[5] += v;
      else if (f == NF - 1) acc[6] += v;
      else acc[7] += v;
    }
    __syncthreads();
  }
}

template <typename T>
__global__ __launch_bounds__(1024) void dsvi_prefinal_kernel(Args a) {
  __shared__ T red[16 * 20];
  __shared__ T klstage[1024 * 4];
  T acc[20];
#pragma unroll
  for (int k = 0; k < 20; ++k) acc[k] = 0;
  sum_recon_kl<T>(a, acc, klstage);
  T v8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v8[k] = acc[k];
  block_sum_n0(v8, red);
  if (threadIdx.x == 0) {
    T* out = (T*)a.out;
#pragma unroll
    for (int k = 0; k < 8; ++k) out[8 + k] = v8[k];
  }
}

template <typename T>
__global__ __launch_bounds__(1024) void dsvi_finalize_kernel(Args a) {
  // every partial sum of the step in ONE pass: 5 row-block sums, per-factor KL slabs, 12 scalar
  // partials of the RBF backward problems; all loads of a thread are independent, one multi-value
  // block reduction (fixed order, deterministic)
  __shared__ T red[16 * 20];
  __shared__ T sc[8];
  __shared__ T klstage[1024 * 4];
#ifdef NMGP_FIN_TRACE
  const unsigned long long t0 = wall_clock64();
#endif
  const T* rp = (const T*)a.red;
  const int t = threadIdx.x;
  T acc[20];
#pragma unroll
  for (int k = 0; k < 20; ++k) acc[k] = 0;
  // Loads are clamped and masked (keep_if) instead of guarded, so every partial array's first
  // strides are in flight together: one memory round trip instead of one per loop trip.
  const int nbr = a.nblk_rows;
  const int ntb = a.elbo_mode ? 0 : (a.B + 3) / 4;                 // t-row backward: per 4-row block
  const T tv = rp[(int64_t)nbr * 4 + min(t, max(ntb - 1, 0))];
  T sv[6][2][2];
  const T* sp = (const T*)a.scal_part;
  if (!a.elbo_mode) {
#pragma unroll
    for (int p = 0; p < 6; ++p)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t i = max(min(a.scal_off[p] + t + u * 1024, a.scal_off[p + 1] - 1), (int64_t)0);
        sv[p][u][0] = sp[i * 2 + 0];
        sv[p][u][1] = sp[i * 2 + 1];
      }
  }
  acc[4] += keep_if(tv, t < ntb);
  for (int b = t + 1024; b < ntb; b += 1024) acc[4] += rp[(int64_t)nbr * 4 + b];
  if (!a.elbo_mode) {
#pragma unroll
    for (int p = 0; p < 6; ++p) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const bool ok = a.scal_off[p] + t + u * 1024 < a.scal_off[p + 1];
        acc[8 + 2 * p] += keep_if(sv[p][u][0], ok);
        acc[9 + 2 * p] += keep_if(sv[p][u][1], ok);
      }
      for (int64_t i = a.scal_off[p] + t + 2048; i < a.scal_off[p + 1]; i += 1024) {
        acc[8 + 2 * p] += sp[i * 2 + 0];
        acc[9 + 2 * p] += sp[i * 2 + 1];
      }
    }
  }
  // per-factor KL from its slab partials (slab order) and the recon row partials: here only for
  // compute_ELBO samples; training steps took them from dsvi_prefinal_kernel (added after the sum)
  if (a.elbo_mode) sum_recon_kl<T>(a, acc, klstage);
#ifdef NMGP_FIN_TRACE
  const unsigned long long t1 = wall_clock64();
#endif
  block_sum_n0(acc, red);        // (valid in thread 0, which writes every output below)
  if (!a.elbo_mode && threadIdx.x == 0) {
    const T* pre = (const T*)a.out + 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += pre[k];     // acc[k] holds no early partials here: exact copy
  }
#ifdef NMGP_FIN_TRACE
  const unsigned long long t2 = wall_clock64();
#endif
  const T R = acc[0], e = acc[1], c0 = acc[2], c1 = acc[3], vs = acc[4];
  const T klw = acc[5], klv = acc[6], klu = acc[7];
  T* out = (T*)a.out;
  if (a.elbo_mode) {
    if (threadIdx.x == 0) {
      out[1] = R;
      out[2] = klw;
      out[3] = klv;
      out[4] = klu;
    }
    return;
  }
  // fp32 engines with the fp64 prior adjoints (a.scal64): the six builder partial sets (L0_12, L0_22,
  // L1_12, L1_22, t12, t22), the varbar partials and the row coefficients c0 / c1 summed in fp64 --
  // each hyper-parameter gradient cancels to ~1e-7 of its terms at ECoG length scales
  double h64[15];
#pragma unroll
  for (int k = 0; k < 15; ++k) h64[k] = 0;
  if (a.scal64) {
    __shared__ double red64[16];
    const double* s64 = (const double*)a.scal64;
#pragma unroll
    for (int q = 0; q < 6; ++q)
      for (int64_t i = a.scal_off[q] + t; i < a.scal_off[q + 1]; i += blockDim.x) {
        h64[2 * q] += s64[2 * i];
        h64[2 * q + 1] += s64[2 * i + 1];
      }
    const double* vpart = (const double*)a.t64 + (int64_t)a.B * a.M + a.B;
    for (int64_t i = t; i < ntb; i += blockDim.x) h64[12] += vpart[i];
    const T* rcrow = (const T*)a.rowbuf + (int64_t)(2 * a.D + 1) * a.B;     // c0 | c1 rows
    for (int64_t i = t; i < a.B; i += blockDim.x) {
      h64[13] += (double)rcrow[i];
      h64[14] += (double)rcrow[a.B + i];
    }
#pragma unroll
    for (int k = 0; k < 15; ++k) h64[k] = block_sum(h64[k], red64);
  }
  // L0_12 + L0_22, L1_12 + L1_22, t12 + t22 (sigma2 / length-scale partials)
  if (threadIdx.x == 0) {
    sc[0] = acc[8] + acc[10];
    sc[1] = acc[9] + acc[11];
    sc[2] = acc[12] + acc[14];
    sc[3] = acc[13] + acc[15];
    sc[4] = acc[16] + acc[18];
    sc[5] = acc[17] + acc[19];
  }
  __syncthreads();
  T* g = (T*)a.grad;
  if (threadIdx.x == 0) {
    const T cc = -(T)a.N_over_B;
    out[0] = cc * R + klw + klv + klu;
    out[1] = R;
    out[2] = klw;
    out[3] = klv;
    out[4] = klu;
    T gs[7];
    gs[0] = sc[4] + hyp<T>(a, 0) * vs;   // sigma2_tildeell_log
    gs[1] = sc[5];                        // length_scales_tildeell_log
    gs[2] = sc[0] + hyp<T>(a, 2) * c0;   // sigma2_L0_log
    gs[3] = sc[1];                        // length_scales_L0_log
    gs[4] = sc[2] + hyp<T>(a, 4) * c1;   // sigma2_L1_log
    gs[5] = sc[3];                        // length_scales_L1_log
    gs[6] = e;                            // sigma2_err_log
    if (a.scal64) {
      const T* hy = (const T*)a.theta + a.off_hyp;
      gs[0] = (T)((h64[8] + h64[10]) + exp((double)hy[0]) * h64[12]);
      gs[1] = (T)(h64[9] + h64[11]);
      gs[2] = (T)((h64[0] + h64[2]) + exp((double)hy[2]) * h64[13]);
      gs[3] = (T)(h64[1] + h64[3]);
      gs[4] = (T)((h64[4] + h64[6]) + exp((double)hy[4]) * h64[14]);
      gs[5] = (T)(h64[5] + h64[7]);
    }
    for (int k = 0; k < 7; ++k) g[a.off_hyp + k] = (a.frozen_mask >> k & 1) ? (T)0 : gs[k];
  }
  // training step: the KL mean gradients A2^{-1} mu and mu_v += vbar (round 6: here, after every other writer of those
  // rows -- bwd_lbar's mu products, nmgp_lbar_reduce, the v backward -- instead of a launch of their own) when they
  // are few (PM2.5: 5376 values); larger engines launch nmgp_dsvi_mugrad_* before finalize (one workgroup over
  // ECoG's 8.5 M values took 6.6 ms)
  if (!a.elbo_mode && mugrad_count(a) <= NMGP_MUGRAD_IN_FINALIZE_MAX) mugrad_body<T>(a, threadIdx.x, blockDim.x);
  // the optimizer step counter of a captured training step (nmgp_adam_lower_advanced_* follows): no launch of its own
  if (!a.elbo_mode && a.adam_step != nullptr && threadIdx.x == 0) a.adam_step[0] += 1;
#ifdef NMGP_FIN_TRACE
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t3 = wall_clock64();
    out[5] = (T)(t1 - t0);
    out[6] = (T)(t2 - t1);
    out[7] = (T)(t3 - t2);
  }
#endif
}

// ------------------------------------------------------------------------------------ Adam
__device__ inline unsigned long long bits_of(double x) { return __builtin_bit_cast(unsigned long long, x); }
__device__ inline unsigned int bits_of(float x) { return __builtin_bit_cast(unsigned int, x); }
// one element of torch's Adam (lerp form); returns false when grad, exp_avg and exp_avg_sq are all +0
// (the never-used strictly-upper triangles and unused (i<j) blocks of the factor parameters): the
// update would leave every value bit-identical, so nothing needs writing
template <typename T>
__device__ inline bool adam_elt(T& th, T gi, T& mi, T& vi, T lr, T b1, T b2, T eps, T bc1, T bc2s) {
  if ((bits_of(gi) | bits_of(mi) | bits_of(vi)) == 0) return false;
  mi = mi + ((T)1 - b1) * (gi - mi);          // exp_avg.lerp_(grad, 1 - beta1)
  vi = vi * b2 + ((T)1 - b2) * gi * gi;
  const T denom = dsqrt(vi) / bc2s + eps;
  th = th - (lr / bc1) * (mi / denom);
  return true;
}

// 16-byte vectors per thread (VEC) when every pointer is 16-byte aligned, grid-strided; the bias
// corrections are computed once per workgroup (a double pow per element cost more than the memory
// traffic at HCP's 670 M parameters).  Element arithmetic is unchanged, so results are bit-identical
// to the scalar form.
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void adam_kernel(T* th, const T* g, T* m, T* v, int64_t n, const int64_t* step,
                                                   T lr, T b1, T b2, T eps) {
  __shared__ T s_bc[2];
  if (threadIdx.x == 0) {
    const double t = (double)(step[0] + 1);
    s_bc[0] = (T)(1.0 - pow((double)b1, t));
    s_bc[1] = (T)sqrt(1.0 - pow((double)b2, t));
  }
  __syncthreads();
  const T bc1 = s_bc[0], bc2s = s_bc[1];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (VEC) {
    constexpr int V = 16 / (int)sizeof(T);
    struct alignas(16) P { T e[V]; };
    const int64_t nv = n / V;
    for (int64_t q = tid; q < nv; q += stride) {
      const P gq = ((const P*)g)[q];
      P mq = ((const P*)m)[q];
      P vq = ((const P*)v)[q];
      bool any = false;
#pragma unroll
      for (int e = 0; e < V; ++e) any |= (bits_of(gq.e[e]) | bits_of(mq.e[e]) | bits_of(vq.e[e])) != 0;
      if (!any) continue;
      P tq = ((P*)th)[q];
#pragma unroll
      for (int e = 0; e < V; ++e) adam_elt<T>(tq.e[e], gq.e[e], mq.e[e], vq.e[e], lr, b1, b2, eps, bc1, bc2s);
      ((P*)m)[q] = mq;
      ((P*)v)[q] = vq;
      ((P*)th)[q] = tq;
    }
    for (int64_t i = nv * V + tid; i < n; i += stride) {
      T ti = th[i], mi = m[i], vi = v[i];
      if (adam_elt<T>(ti, g[i], mi, vi, lr, b1, b2, eps, bc1, bc2s)) {
        m[i] = mi;
        v[i] = vi;
        th[i] = ti;
      }
    }
  } else {
    for (int64_t i = tid; i < n; i += stride) {
      T mi = m[i], vi = v[i];
      T ti = th[i];
      if (adam_elt<T>(ti, g[i], mi, vi, lr, b1, b2, eps, bc1, bc2s)) {
        m[i] = mi;
        v[i] = vi;
        th[i] = ti;
      }
    }
  }
}

template <typename T>
static void adam_launch(T* th, const T* g, T* m, T* v, int64_t n, const int64_t* step, T lr, T b1, T b2, T eps,
                        hipStream_t s) {
  const bool vec = ((((uintptr_t)th) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) == 0;
  const int64_t per = vec ? 16 / (int64_t)sizeof(T) : 1;
  const int64_t blocks = std::min<int64_t>((n / per + 255) / 256 + 1, 16384);
  if (vec)
    hipLaunchKernelGGL((adam_kernel<T, true>), dim3((unsigned)blocks), dim3(256), 0, s, th, g, m, v, n, step, lr, b1,
                       b2, eps);
  else
    hipLaunchKernelGGL((adam_kernel<T, false>), dim3((unsigned)blocks), dim3(256), 0, s, th, g, m, v, n, step, lr, b1,
                       b2, eps);
}

__global__ void counter_add_kernel(int64_t* c, int64_t inc) { c[0] += inc; }

// Adam over lower-triangular M x M blocks (round 5): the sqrt_W / sqrt_v / sqrt_U parameters enter the model only
// through mat2ltri (code/utils.py:68-72), so their strictly upper triangles never get a gradient and stay where
// torch's Adam leaves them (exp_avg = exp_avg_sq = 0: no move).  This form touches only the 16-byte vectors that
// hold lower-triangle elements (row r: vectors 0 .. r / V) instead of streaming g, m and v over the whole block to
// find the all-zero groups -- at the ECoG shape (8384 blocks of M = 1024) that halves the reads of the update.
// One wave per row pair (r, M - 1 - r): M + 1 elements per wave, balanced; grid-strided over the pairs.  The
// element update is adam_elt, so results are bit-identical to the dense kernel.
template <typename T>
__global__ __launch_bounds__(256) void adam_tri_kernel(T* th, const T* g, T* m, T* v, int64_t nblk, int M,
                                                       const int64_t* step, T lr, T b1, T b2, T eps) {
  __shared__ T s_bc[2];
  if (threadIdx.x == 0) {
    const double t = (double)(step[0] + 1);
    s_bc[0] = (T)(1.0 - pow((double)b1, t));
    s_bc[1] = (T)sqrt(1.0 - pow((double)b2, t));
  }
  __syncthreads();
  const T bc1 = s_bc[0], bc2s = s_bc[1];
  constexpr int V = 16 / (int)sizeof(T);
  struct alignas(16) P { T e[V]; };
  const int lane = threadIdx.x & 63;
  const int half = (M + 1) / 2;
  const int64_t npair = nblk * half;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); p < npair; p += nw) {
    const int64_t b = p / half;
    const int rp = (int)(p - b * half);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = h == 0 ? rp : M - 1 - rp;
      if (h == 1 && r == rp) break;
      const int64_t row = (b * M + r) * (int64_t)M / V;     // vector index of the row's start
      const int nv = r / V + 1;
      for (int q = lane; q < nv; q += 64) {
        const int64_t i = row + q;
        const P gq = ((const P*)g)[i];
        P mq = ((const P*)m)[i];
        P vq = ((const P*)v)[i];
        bool any = false;
#pragma unroll
        for (int e = 0; e < V; ++e) any |= (bits_of(gq.e[e]) | bits_of(mq.e[e]) | bits_of(vq.e[e])) != 0;
        if (!any) continue;
        P tq = ((P*)th)[i];
#pragma unroll
        for (int e = 0; e < V; ++e) adam_elt<T>(tq.e[e], gq.e[e], mq.e[e], vq.e[e], lr, b1, b2, eps, bc1, bc2s);
        ((P*)m)[i] = mq;
        ((P*)v)[i] = vq;
        ((P*)th)[i] = tq;
      }
    }
  }
}

// One launch over the whole flat vector (round 6): grid-strided over its 16-byte vectors in memory order; a vector
// inside one of the (up to 4) lower-triangular block ranges and wholly above its row's diagonal is skipped without a
// load, every other vector is updated with adam_elt (bit-identical to the dense kernel and to the per-range launches
// it replaces: ECoG 0.2721 -> 0.2708 s as the triangular part alone, profiles/r06zl_adam_flat_ab.txt; at PM2.5 the
// sqrt blocks' upper halves are no longer streamed and the dense gaps / ranges are one launch instead of eight).
struct AdamTri {
  int64_t off[4], len[4];   // element offset and length (blocks x M x M) of each range, ascending
  int n;
};
template <typename T>
__global__ __launch_bounds__(256) void adam_flat_kernel(T* th, const T* g, T* m, T* v, int64_t n, AdamTri tr, int M,
                                                        const int64_t* step, T lr, T b1, T b2, T eps, int sb) {
  __shared__ T s_bc[2];
  if (threadIdx.x == 0) {
    const double t = (double)(step[0] + sb);     // sb 0: the counter was already advanced for this step
    s_bc[0] = (T)(1.0 - pow((double)b1, t));
    s_bc[1] = (T)sqrt(1.0 - pow((double)b2, t));
  }
  __syncthreads();
  const T bc1 = s_bc[0], bc2s = s_bc[1];
  constexpr int V = 16 / (int)sizeof(T);
  struct alignas(16) P { T e[V]; };
  const int64_t nv = n / V;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t q = tid; q < nv; q += stride) {
    const int64_t i = q * V;
    bool skip = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k < tr.n && i >= tr.off[k] && i < tr.off[k] + tr.len[k]) {
        const int64_t loc = i - tr.off[k], rowi = loc / M;
        skip = (int)(loc - rowi * M) > (int)(rowi % M);
      }
    }
    if (skip) continue;
    const P gq = ((const P*)g)[q];
    P mq = ((const P*)m)[q];
    P vq = ((const P*)v)[q];
    bool any = false;
#pragma unroll
    for (int e = 0; e < V; ++e) any |= (bits_of(gq.e[e]) | bits_of(mq.e[e]) | bits_of(vq.e[e])) != 0;
    if (!any) continue;
    P tq = ((P*)th)[q];
#pragma unroll
    for (int e = 0; e < V; ++e) adam_elt<T>(tq.e[e], gq.e[e], mq.e[e], vq.e[e], lr, b1, b2, eps, bc1, bc2s);
    ((P*)m)[q] = mq;
    ((P*)v)[q] = vq;
    ((P*)th)[q] = tq;
  }
  for (int64_t i = nv * V + tid; i < n; i += stride) {     // (the tail past the last vector lies in no range)
    T ti = th[i], mi = m[i], vi = v[i];
    if (adam_elt<T>(ti, g[i], mi, vi, lr, b1, b2, eps, bc1, bc2s)) {
      m[i] = mi;
      v[i] = vi;
      th[i] = ti;
    }
  }
}

// the flat vector [0, n) with `ntri` ranges (offset, blocks) of lower-triangular M x M blocks: the dense kernel on
// the gaps, the triangular one on the ranges, then the step counter
template <typename T>
static int adam_lower(T* th, const T* g, T* m, T* v, int64_t n, const int64_t* tri, int ntri, int M, int64_t* step,
                      T lr, T b1, T b2, T eps, hipStream_t s, bool advanced = false) {
  if (ntri < 0 || (ntri > 0 && !tri)) return -6;
  if (M <= 0) return -8;
  constexpr int V = 16 / (int)sizeof(T);
  const bool aligned = ((((uintptr_t)th) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) == 0;
  static const bool flat = [] { const char* e = getenv("NMGP_ADAM_FLAT"); return !e || atoi(e) != 0; }();
  if ((flat || advanced) && aligned && ntri <= 4 && M % V == 0) {
    AdamTri tr{};
    tr.n = ntri;
    int64_t at = 0;
    bool ok = true;
    for (int k = 0; k < ntri; ++k) {
      const int64_t off = tri[2 * k], nb = tri[2 * k + 1];
      const int64_t len = nb * (int64_t)M * M;
      ok = ok && off >= at && nb >= 0 && off + len <= n && off % V == 0;
      tr.off[k] = off;
      tr.len[k] = len;
      at = off + len;
    }
    if (ok) {
      const int64_t blocks = std::min<int64_t>((n / V + 255) / 256 + 1, 32768);
      hipLaunchKernelGGL(adam_flat_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, s, th, g, m, v, n, tr, M, step, lr,
                         b1, b2, eps, advanced ? 0 : 1);
      NMGP_CHECK_LAUNCH();
      if (advanced) return NMGP_OK;
      hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, s, step, (int64_t)1);
      NMGP_CHECK_LAUNCH();
      return NMGP_OK;
    }
  }
  if (advanced) return -12;   // (the advanced-counter form exists only as the single launch)
  int64_t at = 0;
  for (int k = 0; k < ntri; ++k) {
    const int64_t off = tri[2 * k], nb = tri[2 * k + 1];
    const int64_t len = nb * (int64_t)M * M;
    if (off < at || nb < 0 || off + len > n) return -6;
    if (!aligned || M % V != 0 || off % V != 0) return -8;
    if (off > at) adam_launch<T>(th + at, g + at, m + at, v + at, off - at, step, lr, b1, b2, eps, s);
    if (nb > 0) {
      const int64_t pairs = nb * ((M + 1) / 2);
      const int64_t blocks = std::min<int64_t>((pairs + 3) / 4, 16384);
      hipLaunchKernelGGL(adam_tri_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, s, th + off, g + off, m + off, v + off,
                         nb, M, step, lr, b1, b2, eps);
    }
    at = off + len;
  }
  if (n > at) adam_launch<T>(th + at, g + at, m + at, v + at, n - at, step, lr, b1, b2, eps, s);
  NMGP_CHECK_LAUNCH();
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, s, step, (int64_t)1);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

// Element-wise precision conversion (grid-strided): fp32 engines factor their four GP priors in fp64
// (engine.py), the explicit-inverse projections K12 (K22 + 1e-4 I)^-1 of smooth priors lose ~cond*eps
// in an fp32 factorization.
template <typename S, typename D>
__global__ __launch_bounds__(256) void convert_kernel(const S* __restrict__ src, D* __restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = (D)src[i];
}
template <typename S, typename D>
static int convert_launch(const S* src, D* dst, int64_t n, hipStream_t s) {
  if (!src) return -1;
  if (!dst) return -2;
  if (n <= 0) return NMGP_OK;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL((convert_kernel<S, D>), dim3((unsigned)blocks), dim3(256), 0, s, src, dst, n);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

// ------------------------------------------------------------------------------------ P-bar_G reduction
// The latent P-bar of the backward (code/nmgp_dsvi.py:227-238 autograd through MGP_mu_sigma2 / MGP_d): the rows of
// output i receive sum_{d <= i} W-hat_d L_d^T.  The engine forms each factor's product once for all rows that use
// it, Z_d = W-hat_d[rows of outputs >= d] L_d^T (one grouped GEMM, k = M), and this kernel adds, per row r of
// output i, Z_0[r] + Z_1[r] + ... + Z_i[r] (in d order) onto P[r] -- instead of one k = (i + 1) M product per
// output, whose k loop (up to D M) ran on a single workgroup per output tile.  One block per (row, 256 columns).
template <typename T>
__global__ __launch_bounds__(256) void pbar_reduce_kernel(const T* __restrict__ Z, int64_t sZ, T* __restrict__ P,
                                                          int64_t ldp, const int32_t* __restrict__ seg, int D, int M) {
  const int r = blockIdx.x;
  const int j = blockIdx.y * 256 + threadIdx.x;
  if (r >= seg[D] || j >= M) return;
  int i = 0;                                   // the output of row r: the last d with seg[d] <= r
  for (int d = 1; d < D; ++d) i = seg[d] <= r ? d : i;
  T acc = P[(int64_t)r * ldp + j];
  const T* z = Z + (int64_t)r * M + j;
  for (int d = 0; d <= i; ++d) acc += z[(int64_t)d * sZ];
  P[(int64_t)r * ldp + j] = acc;
}

template <typename T>
static int pbar_reduce_launch(const T* Z, int64_t sZ, T* P, int64_t ldp, const int32_t* seg, int D, int B, int M,
                              hipStream_t s) {
  if (!Z) return -1;
  if (sZ < (int64_t)B * M) return -2;
  if (!P) return -3;
  if (ldp < M) return -4;
  if (!seg) return -5;
  if (D <= 0) return -6;
  if (B < 0) return -7;
  if (M <= 0) return -8;
  if (B == 0) return NMGP_OK;
  hipLaunchKernelGGL(pbar_reduce_kernel<T>, dim3((unsigned)B, (unsigned)((M + 255) / 256)), dim3(256), 0, s, Z, sZ, P,
                     ldp, seg, D, M);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

// ------------------------------------------------------------------------------------ L-bar reduction
// The latent factors' L-bar and mu-bar of the backward (code/nmgp_dsvi.py:198-215 autograd of W = mu + L eps and
// MGP_d's L-products): factor d collects P_G^T W-hat_d over the rows of every output i >= d.  The engine forms one
// product per (i, d) over output i's rows only, Y_{i,d} = P_G[rows of i]^T W-hat_d[rows of i] (k = the output's
// rows: every workgroup of the grouped GEMM runs a short k loop, where one product per d ran k = the rows of
// outputs d..D-1 on a single workgroup per output tile), and this kernel adds Y_{d,d} + ... + Y_{D-1,d} (in i order)
// onto factor d's gradient: the lower triangle of an M x M block at gA + d * sA (upper triangle set to 0, as the
// OUT_TRIL GEMM it replaces) and the M-vector at gB + d * sB.  Slot (i, d) is Y + (first(d) + i - d) * sY, first(d)
// = sum_{d' < d} (D - d'), matrix first, vector at offset M * M.  Blocks [0, nA) cover the matrices, the rest the
// vectors; blockIdx.y = d.
template <typename T>
__global__ __launch_bounds__(256) void lbar_reduce_kernel(const T* __restrict__ Y, int64_t sY, T* __restrict__ gA,
                                                          int64_t sA, T* __restrict__ gB, int64_t sB, int D, int M,
                                                          int nA) {
  const int d = blockIdx.y;
  const int64_t first = (int64_t)d * D - (int64_t)d * (d - 1) / 2;
  const T* y = Y + first * sY;
  const int64_t MM = (int64_t)M * M;
  if ((int)blockIdx.x < nA) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= MM) return;
    const int r = (int)(e / M), c = (int)(e % M);
    T* o = gA + (int64_t)d * sA + e;
    if (c > r) {
      *o = (T)0;
      return;
    }
    T acc = *o;
    for (int i = d; i < D; ++i) acc += y[(int64_t)(i - d) * sY + e];
    *o = acc;
  } else {
    const int e = ((int)blockIdx.x - nA) * 256 + threadIdx.x;
    if (e >= M) return;
    T* o = gB + (int64_t)d * sB + e;
    T acc = *o;
    for (int i = d; i < D; ++i) acc += y[(int64_t)(i - d) * sY + MM + e];
    *o = acc;
  }
}

template <typename T>
static int lbar_reduce_launch(const T* Y, int64_t sY, T* gA, int64_t sA, T* gB, int64_t sB, int D, int M,
                              hipStream_t s) {
  if (!Y) return -1;
  if (sY < (int64_t)M * M + M) return -2;
  if (!gA) return -3;
  if (sA < (int64_t)M * M) return -4;
  if (!gB) return -5;
  if (sB < M) return -6;
  if (D <= 0) return -7;
  if (M <= 0) return -8;
  const int64_t nA = ((int64_t)M * M + 255) / 256;
  if (nA > (1 << 30)) return -8;
  const int nB = (M + 255) / 256;
  hipLaunchKernelGGL(lbar_reduce_kernel<T>, dim3((unsigned)(nA + nB), (unsigned)D), dim3(256), 0, s, Y, sY, gA, sA, gB,
                     sB, D, M, (int)nA);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}

// ------------------------------------------------------------------------------------ batch gather
// One block: every thread reads the batch index first, the copy is grid-strided over the block,
// then (after a barrier) thread 0 advances the counter for the next step.
template <typename T>
__global__ __launch_bounds__(1024) void batch_gather_kernel(const T* Xb, const T* Yb, const int32_t* Ib,
                                                            const int32_t* Sb, int64_t B, int64_t nseg, int64_t nbatch,
                                                            int64_t* ctr, T* x, T* y, int32_t* ro, int32_t* seg) {
  const int64_t b = ctr[0] % nbatch;
  const T* xs = Xb + b * B;
  const T* ys = Yb + b * B;
  const int32_t* is = Ib + b * B;
  for (int64_t i = threadIdx.x; i < B; i += blockDim.x) {
    x[i] = xs[i];
    y[i] = ys[i];
    ro[i] = is[i];
  }
  for (int64_t i = threadIdx.x; i < nseg; i += blockDim.x) seg[i] = Sb[b * nseg + i];
  __syncthreads();
  if (threadIdx.x == 0) ctr[0] += 1;
}

// ------------------------------------------------------------------------------------ Philox
__device__ inline void philox_round(uint32_t (&c)[4], uint32_t (&k)[2]) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
  const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
  c[0] = h1 ^ c[1] ^ k[0];
  c[1] = l1;
  c[2] = h0 ^ c[3] ^ k[1];
  c[3] = l0;
  k[0] += 0x9E3779B9u;
  k[1] += 0xBB67AE85u;
}

// normals 4t .. 4t+3 of the Philox-4x32-10 stream (key = seed, counter = (t, base)), Box-Muller
template <typename T>
__device__ inline void normal_quad(T* out, int64_t n, uint64_t seed, uint64_t base, int64_t t) {
  uint32_t c[4] = {(uint32_t)t, (uint32_t)((uint64_t)t >> 32), (uint32_t)base, (uint32_t)(base >> 32)};
  uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
#pragma unroll
  for (int r = 0; r < 10; ++r) philox_round(c, k);
  const double inv = 2.3283064365386963e-10;   // 2^-32
  double u[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) u[q] = ((double)c[q] + 0.5) * inv;
  const double two_pi = 6.283185307179586;
  const double r0 = sqrt(-2.0 * log(u[0])), r1 = sqrt(-2.0 * log(u[2]));
  double z[4] = {r0 * cos(two_pi * u[1]), r0 * sin(two_pi * u[1]), r1 * cos(two_pi * u[3]), r1 * sin(two_pi * u[3])};
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (t * 4 + q < n) out[t * 4 + q] = (T)z[q];
}

template <typename T>
__global__ void normal_kernel(T* out, int64_t n, uint64_t seed, const int64_t* counter, int64_t offset) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t * 4 >= n) return;
  normal_quad<T>(out, n, seed, (uint64_t)(counter ? counter[0] : 0) + (uint64_t)offset, t);
}

// Start of a graph-replayed training step in ONE launch (was: minibatch gather, Philox noise, noise
// counter advance, gradient zeroing -- four dependent launches): block 0 gathers the minibatch and
// advances the batch counter; every block draws its share of the noise from the counter value it read
// at entry and zeroes its share of the gradient; the last block to finish advances the noise counter
// (so every block has read it) and re-arms the arrival word.  Same values as the separate kernels.
template <typename T>
__global__ __launch_bounds__(256) void step_begin_kernel(const T* Xb, const T* Yb, const int32_t* Ib,
                                                         const int32_t* Sb, int64_t B, int64_t nseg, int64_t nbatch,
                                                         int64_t* bctr, T* x, T* y, int32_t* ro, int32_t* seg,
                                                         T* noise, int64_t nnoise, uint64_t seed, int64_t* nctr,
                                                         int32_t* done, T* grad, int64_t ngrad) {
  const uint64_t base = (uint64_t)nctr[0];
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t q = tid; q * 4 < nnoise; q += stride) normal_quad<T>(noise, nnoise, seed, base, q);
  if ((((uintptr_t)grad) & 15) == 0) {      // 16-byte stores
    constexpr int V = 16 / (int)sizeof(T);
    struct alignas(16) Z { T e[V]; };
    const Z z{};
    const int64_t nv = ngrad / V;
    for (int64_t i = tid; i < nv; i += stride) ((Z*)grad)[i] = z;
    for (int64_t i = nv * V + tid; i < ngrad; i += stride) grad[i] = (T)0;
  } else {
    for (int64_t i = tid; i < ngrad; i += stride) grad[i] = (T)0;
  }
  if (blockIdx.x == 0) {
    const int64_t b = bctr[0] % nbatch;
    for (int64_t i = threadIdx.x; i < B; i += blockDim.x) {
      x[i] = Xb[b * B + i];
      y[i] = Yb[b * B + i];
      ro[i] = Ib[b * B + i];
    }
    for (int64_t i = threadIdx.x; i < nseg; i += blockDim.x) seg[i] = Sb[b * nseg + i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (blockIdx.x == 0) bctr[0] += 1;
    const int old = __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (int)gridDim.x - 1) {
      nctr[0] += 1;
      __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

static inline unsigned blocks_rows(int B) { return (unsigned)((B + 3) / 4); }

}  // namespace nmgp

using nmgp::Args;

#define CHECK_ARGS(a)              \
  do {                             \
    if ((a) == nullptr) return -1; \
  } while (0)

namespace nmgp {
// One definition per entry point, instantiated below for f64 and f32 (extern "C" wrappers).
template <typename T> static int dsvi_hyper(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  hipLaunchKernelGGL(dsvi_v_kernel<T>, dim3(blocks_rows(a->M)), dim3(256), 0, s, *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T> static int dsvi_vg22(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  const int nt = (a->M + 15) / 16;
  hipLaunchKernelGGL(dsvi_vg22_kernel<T>, dim3((unsigned)(nt * (nt + 1) / 2)), dim3(256), 0, s, *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T> static int dsvi_trow(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  hipLaunchKernelGGL(dsvi_trow_kernel<T>, dim3(blocks_rows(a->B)), dim3(256), 0, s, *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T> static int dsvi_recon(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  if (a->D > 128) return -1;
  const size_t sm = (size_t)(4 * (3 + 4 * a->D) + 4 * a->D + 4) * sizeof(T);
  hipLaunchKernelGGL(dsvi_recon_kernel<T>, dim3((unsigned)a->B), dim3(256), sm, s, *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T> static int dsvi_kl(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  // the factors of the KL range, then the v factor (last in the factor list) unless this rank has no KL_v
  if (a->kl_f0 < 0 || a->kl_f1 > a->NF - 1 || a->kl_f0 > a->kl_f1) return -1;
  const int nf = a->kl_f1 - a->kl_f0 + (a->kl_v ? 1 : 0);
  if (nf <= 0) return NMGP_OK;
  hipLaunchKernelGGL(dsvi_kl_kernel<T>, dim3(nf, (a->M + KL_ROWS - 1) / KL_ROWS), dim3(256), 0, s, *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T> static int dsvi_delta(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  hipLaunchKernelGGL(dsvi_delta_kernel<T>, dim3((unsigned)((a->M + 255) / 256), 4), dim3(256), 0, s, *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T> static int dsvi_tbwd(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  hipLaunchKernelGGL(dsvi_tbwd_kernel<T>, dim3(blocks_rows(a->B)), dim3(256), 0, s, *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T> static int dsvi_vbwd(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  const size_t sm = (size_t)(a->M + 5 * VBW_ROWS) * sizeof(T);   // vbar | w rows | 4 x VBW_ROWS wave partials
  hipLaunchKernelGGL(dsvi_vbwd_kernel<T>, dim3((a->M + VBW_ROWS - 1) / VBW_ROWS), dim3(256), sm, s, *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T> static int dsvi_mugrad(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  const int64_t n = (int64_t)a->D * a->M + a->M + (a->pair_packed ? (int64_t)a->Q : (int64_t)a->D * a->D) * a->M;
  hipLaunchKernelGGL(dsvi_mugrad_kernel<T>, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 2048)), dim3(256), 0, s,
                     *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T> static int dsvi_prefinal(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  if (a->M > 16384) return -2;
  hipLaunchKernelGGL(dsvi_prefinal_kernel<T>, dim3(1), dim3(1024), 0, s, *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T> static int dsvi_finalize(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  if (a->M > 16384) return -2;
  hipLaunchKernelGGL(dsvi_finalize_kernel<T>, dim3(1), dim3(1024), 0, s, *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T>
static int normal_launch(T* out, int64_t n, uint64_t seed, const int64_t* counter, int64_t offset, hipStream_t s) {
  if (!out) return -1;
  if (n <= 0) return NMGP_OK;
  const int64_t nt = (n + 3) / 4;
  hipLaunchKernelGGL(normal_kernel<T>, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, out, n, seed, counter,
                     offset);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T>
static int batch_gather(const T* Xb, const T* Yb, const int32_t* Ib, const int32_t* Sb, int64_t B, int64_t nseg,
                        int64_t nbatch, int64_t* ctr, T* x, T* y, int32_t* ro, int32_t* seg, hipStream_t s) {
  if (!Xb || !Yb || !Ib || !Sb) return -1;
  if (B <= 0 || nseg <= 0 || nbatch <= 0) return -5;
  if (!ctr) return -8;
  if (!x || !y || !ro || !seg) return -9;
  hipLaunchKernelGGL(batch_gather_kernel<T>, dim3(1), dim3(1024), 0, s, Xb, Yb, Ib, Sb, B, nseg, nbatch, ctr, x, y, ro,
                     seg);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
// status words of the kernel files with bounded inter-workgroup spins (common.hpp)
int nmgp_tu_status_gemm(unsigned int* v, int clear);
int nmgp_tu_status_gemm_big(unsigned int* v, int clear);
int nmgp_tu_status_chol(unsigned int* v, int clear);
}  // namespace nmgp

extern "C" {
int nmgp_device_status(uint32_t* out, int clear) {
  if (!out) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return NMGP_ERR_LAUNCH;
  unsigned int acc = 0;
  int (*const parts[])(unsigned int*, int) = {nmgp::nmgp_tu_status_gemm, nmgp::nmgp_tu_status_gemm_big,
                                              nmgp::nmgp_tu_status_chol};
  for (auto fn : parts) {
    unsigned int v = 0;
    const int rc = fn(&v, clear);
    if (rc != NMGP_OK) return rc;
    acc |= v;
  }
  *out = acc;
  return NMGP_OK;
}
#define NMGP_DSVI_ENTRY(name)                                                                  \
  int nmgp_dsvi_##name##_f64(const Args* a, hipStream_t s) { return nmgp::dsvi_##name<double>(a, s); } \
  int nmgp_dsvi_##name##_f32(const Args* a, hipStream_t s) { return nmgp::dsvi_##name<float>(a, s); }
NMGP_DSVI_ENTRY(hyper)
NMGP_DSVI_ENTRY(vg22)
NMGP_DSVI_ENTRY(trow)
NMGP_DSVI_ENTRY(recon)
NMGP_DSVI_ENTRY(kl)
NMGP_DSVI_ENTRY(delta)
NMGP_DSVI_ENTRY(tbwd)
NMGP_DSVI_ENTRY(vbwd)
NMGP_DSVI_ENTRY(finalize)
NMGP_DSVI_ENTRY(prefinal)
NMGP_DSVI_ENTRY(mugrad)
#undef NMGP_DSVI_ENTRY
int nmgp_adam_lower_f64(double* th, const double* g, double* m, double* v, int64_t n, const int64_t* tri, int ntri,
                        int M, int64_t* step, double lr, double b1, double b2, double eps, hipStream_t s) {
  if (!th) return -1;
  if (!g) return -2;
  if (!m) return -3;
  if (!v) return -4;
  if (!step) return -9;
  if (n <= 0) return NMGP_OK;
  return nmgp::adam_lower<double>(th, g, m, v, n, tri, ntri, M, step, lr, b1, b2, eps, s);
}
int nmgp_adam_lower_f32(float* th, const float* g, float* m, float* v, int64_t n, const int64_t* tri, int ntri, int M,
                        int64_t* step, double lr, double b1, double b2, double eps, hipStream_t s) {
  if (!th) return -1;
  if (!g) return -2;
  if (!m) return -3;
  if (!v) return -4;
  if (!step) return -9;
  if (n <= 0) return NMGP_OK;
  return nmgp::adam_lower<float>(th, g, m, v, n, tri, ntri, M, step, (float)lr, (float)b1, (float)b2, (float)eps, s);
}
int nmgp_adam_lower_advanced_f64(double* th, const double* g, double* m, double* v, int64_t n, const int64_t* tri,
                                 int ntri, int M, const int64_t* step, double lr, double b1, double b2, double eps,
                                 hipStream_t s) {
  if (!th) return -1;
  if (!g) return -2;
  if (!m) return -3;
  if (!v) return -4;
  if (!step) return -9;
  if (n <= 0) return NMGP_OK;
  return nmgp::adam_lower<double>(th, g, m, v, n, tri, ntri, M, const_cast<int64_t*>(step), lr, b1, b2, eps, s, true);
}
int nmgp_adam_lower_advanced_f32(float* th, const float* g, float* m, float* v, int64_t n, const int64_t* tri, int ntri,
                                 int M, const int64_t* step, double lr, double b1, double b2, double eps,
                                 hipStream_t s) {
  if (!th) return -1;
  if (!g) return -2;
  if (!m) return -3;
  if (!v) return -4;
  if (!step) return -9;
  if (n <= 0) return NMGP_OK;
  return nmgp::adam_lower<float>(th, g, m, v, n, tri, ntri, M, const_cast<int64_t*>(step), (float)lr, (float)b1,
                                 (float)b2, (float)eps, s, true);
}
int nmgp_adam_f64(double* th, const double* g, double* m, double* v, int64_t n, int64_t* step, double lr,
                  double b1, double b2, double eps, hipStream_t s) {
  if (!th) return -1;
  if (!g) return -2;
  if (!m) return -3;
  if (!v) return -4;
  if (!step) return -6;
  if (n <= 0) return NMGP_OK;
  nmgp::adam_launch<double>(th, g, m, v, n, step, lr, b1, b2, eps, s);
  NMGP_CHECK_LAUNCH();
  hipLaunchKernelGGL(nmgp::counter_add_kernel, dim3(1), dim3(1), 0, s, step, (int64_t)1);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
int nmgp_adam_f32(float* th, const float* g, float* m, float* v, int64_t n, int64_t* step, double lr, double b1,
                  double b2, double eps, hipStream_t s) {
  if (!th) return -1;
  if (!g) return -2;
  if (!m) return -3;
  if (!v) return -4;
  if (!step) return -6;
  if (n <= 0) return NMGP_OK;
  nmgp::adam_launch<float>(th, g, m, v, n, step, (float)lr, (float)b1, (float)b2, (float)eps, s);
  NMGP_CHECK_LAUNCH();
  hipLaunchKernelGGL(nmgp::counter_add_kernel, dim3(1), dim3(1), 0, s, step, (int64_t)1);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
int nmgp_normal_f64(double* out, int64_t n, uint64_t seed, const int64_t* counter, int64_t offset, hipStream_t s) {
  return nmgp::normal_launch<double>(out, n, seed, counter, offset, s);
}
int nmgp_normal_f32(float* out, int64_t n, uint64_t seed, const int64_t* counter, int64_t offset, hipStream_t s) {
  return nmgp::normal_launch<float>(out, n, seed, counter, offset, s);
}
#define NMGP_STEP_BEGIN(T, sfx)                                                                                 \
  int nmgp_step_begin_##sfx(const T* Xb, const T* Yb, const int32_t* Ib, const int32_t* Sb, int64_t B, int64_t nseg, \
                            int64_t nbatch, int64_t* bctr, T* x, T* y, int32_t* ro, int32_t* seg, T* noise,          \
                            int64_t nnoise, uint64_t seed, int64_t* nctr, int32_t* done, T* grad, int64_t ngrad,      \
                            hipStream_t s) {                                                                         \
    if (!Xb || !Yb || !Ib || !Sb) return -1;                                                                        \
    if (B <= 0 || nseg <= 0 || nbatch <= 0) return -5;                                                              \
    if (!bctr) return -8;                                                                                           \
    if (!x || !y || !ro || !seg) return -9;                                                                         \
    if (!noise || nnoise < 0 || !nctr || !done) return -13;                                                         \
    if (!grad || ngrad < 0) return -18;                                                                             \
    const int64_t work = std::max((nnoise + 3) / 4, ngrad);                                                         \
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 256));             \
    hipLaunchKernelGGL(nmgp::step_begin_kernel<T>, dim3(blocks), dim3(256), 0, s, Xb, Yb, Ib, Sb, B, nseg, nbatch,   \
                       bctr, x, y, ro, seg, noise, nnoise, seed, nctr, done, grad, ngrad);                           \
    NMGP_CHECK_LAUNCH();                                                                                            \
    return NMGP_OK;                                                                                                 \
  }
NMGP_STEP_BEGIN(double, f64)
NMGP_STEP_BEGIN(float, f32)
#undef NMGP_STEP_BEGIN
int nmgp_batch_gather_f64(const double* Xb, const double* Yb, const int32_t* Ib, const int32_t* Sb, int64_t B,
                          int64_t nseg, int64_t nbatch, int64_t* ctr, double* x, double* y, int32_t* ro, int32_t* seg,
                          hipStream_t s) {
  return nmgp::batch_gather<double>(Xb, Yb, Ib, Sb, B, nseg, nbatch, ctr, x, y, ro, seg, s);
}
int nmgp_batch_gather_f32(const float* Xb, const float* Yb, const int32_t* Ib, const int32_t* Sb, int64_t B,
                          int64_t nseg, int64_t nbatch, int64_t* ctr, float* x, float* y, int32_t* ro, int32_t* seg,
                          hipStream_t s) {
  return nmgp::batch_gather<float>(Xb, Yb, Ib, Sb, B, nseg, nbatch, ctr, x, y, ro, seg, s);
}
int nmgp_convert_f32_to_f64(const float* src, double* dst, int64_t n, hipStream_t s) {
  return nmgp::convert_launch<float, double>(src, dst, n, s);
}
int nmgp_convert_f64_to_f32(const double* src, float* dst, int64_t n, hipStream_t s) {
  return nmgp::convert_launch<double, float>(src, dst, n, s);
}
int nmgp_pbar_reduce_f64(const double* Z, int64_t sZ, double* P, int64_t ldp, const int32_t* seg, int D, int B, int M,
                         hipStream_t s) {
  return nmgp::pbar_reduce_launch<double>(Z, sZ, P, ldp, seg, D, B, M, s);
}
int nmgp_pbar_reduce_f32(const float* Z, int64_t sZ, float* P, int64_t ldp, const int32_t* seg, int D, int B, int M,
                         hipStream_t s) {
  return nmgp::pbar_reduce_launch<float>(Z, sZ, P, ldp, seg, D, B, M, s);
}
int nmgp_lbar_reduce_f64(const double* Y, int64_t sY, double* gA, int64_t sA, double* gB, int64_t sB, int D, int M,
                         hipStream_t s) {
  return nmgp::lbar_reduce_launch<double>(Y, sY, gA, sA, gB, sB, D, M, s);
}
int nmgp_lbar_reduce_f32(const float* Y, int64_t sY, float* gA, int64_t sA, float* gB, int64_t sB, int D, int M,
                         hipStream_t s) {
  return nmgp::lbar_reduce_launch<float>(Y, sY, gA, sA, gB, sB, D, M, s);
}
int nmgp_counter_add(int64_t* c, int64_t inc, hipStream_t s) {
  if (!c) return -1;
  hipLaunchKernelGGL(nmgp::counter_add_kernel, dim3(1), dim3(1), 0, s, c, inc);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
}
