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
// Variational factor order: f < D latent functions W_f | D <= f < D+Q coefficient pairs (i,j) in
// (i, j<=i) order | f = D+Q (= NF-1) the length-scale process v.  Prior slot of factor f:
// 0 = t (v), 1 = L0 (off-diagonal pairs), 2 = L1 (diagonal pairs), 3 = G (W).
__device__ inline int prior_of(int f, int D) {
  const int Q = D * (D + 1) / 2;
  if (f < D) return 3;
  if (f == D + Q) return 0;
  int i, j;
  pair_ij(f - D, i, j);
  return i == j ? 2 : 1;
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
  const T* Cv = (const T*)a.Afac + (int64_t)(a.NF - 1) * M * M;   // C1 of the v factor (Sigma_v)
  const T* zv = (const T*)a.noise;
  T s = 0;
  for (int k = lane; k <= c; k += 64) s += Cv[(int64_t)c * M + k] * zv[k];
  s = wave_sum(s);
  if (lane == 0) {
    const T v = ((const T*)a.theta)[a.off_muv + c] + s;
    ((T*)a.v)[c] = v;
    ((T*)a.ellZ)[c] = dexp(v);
  }
}

// ------------------------------------------------------------------------------------ t-row
template <typename T>
__global__ __launch_bounds__(256) void dsvi_trow_kernel(Args a) {
  const int M = a.M, B = a.B, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  const T* Pt = (const T*)a.P + (int64_t)r * M;       // slot 0 = t
  const T* Kt = (const T*)a.K12 + (int64_t)r * M;
  const T* v = (const T*)a.v;
  T mean = 0, q = 0;
  for (int c = lane; c < M; c += 64) {
    const T p = Pt[c];
    mean += p * v[c];
    q += p * Kt[c];
  }
  mean = wave_sum(mean);
  q = wave_sum(q);
  if (lane == 0) {
    const T var = var_floor(hyp<T>(a, 0) - q);
    const T zt = ((const T*)a.noise)[M + r];
    const T tl = mean + zt * dsqrt(var + (T)a.jitter);
    ((T*)a.ellX)[r] = dexp(tl);
    ((T*)a.var_t)[r] = var;
  }
}

// ------------------------------------------------------------------------------------ recon
// training (elbo_mode 0): row r of output o uses pairs (o, s) for s <= o  -> l_r[s] = L[o,s,r]
// ELBO     (elbo_mode 1): row r uses pairs (s, o) for s >= o (column gather, nmgp_dsvi.py:361)
template <typename T, int NR>
__global__ __launch_bounds__(256) void dsvi_recon_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  __shared__ T red[16];
  T* rowacc_all = (T*)smem_raw;
  const int M = a.M, B = a.B, D = a.D;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = blockIdx.x * 4 + w;
  const bool elbo = a.elbo_mode != 0;
  T Rrow = 0, epart = 0, c0p = 0, c1p = 0;
  if (r < B) {
    const int o = a.row_out[r];
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
    T* WG = (T*)a.WG;
    T* WP = (T*)a.WP;
    const T* muW = th + a.off_muW;
    const T* muU = th + a.off_muU;
    const T* noise = (const T*)a.noise;
    const int slo = elbo ? o : 0, shi = elbo ? D - 1 : o;

    T qG = 0, q0 = 0, q1 = 0;
    for (int c = lane; c < M; c += 64) {
      qG += PG[c] * KG[c];
      q0 += P0[c] * K0[c];
      q1 += P1[c] * K1[c];
    }
    qG = wave_sum(qG);
    q0 = wave_sum(q0);
    q1 = wave_sum(q1);

    T mreg[NR], greg[NR], lreg[NR], sdreg[NR], zreg[NR];
#pragma unroll
    for (int u = 0; u < NR; ++u) mreg[u] = greg[u] = lreg[u] = sdreg[u] = zreg[u] = 0;
    for (int s = slo; s <= shi; ++s) {
      // latent function s: m = P_G mu_W[s], g = 1 - rowsum(P_G o K_G12) + ||P_G L_W[s]||^2
      const T* wg = WG + (int64_t)s * BM + (int64_t)r * M;
      const T* mw = muW + (int64_t)s * M;
      T sm = 0, sq = 0;
      for (int c = lane; c < M; c += 64) {
        sm += PG[c] * mw[c];
        const T x = wg[c];
        sq += x * x;
      }
      sm = wave_sum(sm);
      sq = wave_sum(sq);
      setlane(mreg, s, lane, sm);
      setlane(greg, s, lane, (T)1 - qG + sq);
      // coefficient pair: training (o, s), ELBO (s, o)
      const int pi = elbo ? s : o, pj = elbo ? o : s;
      const bool diag = (s == o);
      const T* Pk = diag ? P1 : P0;
      const T* mu = muU + ((int64_t)pi * D + pj) * M;
      const T* wp = WP + (int64_t)s * BM + (int64_t)r * M;
      T pm = 0, pq = 0;
      for (int c = lane; c < M; c += 64) {
        pm += Pk[c] * mu[c];
        const T x = wp[c];
        pq += x * x;
      }
      pm = wave_sum(pm);
      pq = wave_sum(pq);
      const T s2p = var_floor((diag ? s21 : s20) - (diag ? q1 : q0) + pq);
      const T sd = dsqrt(s2p + lam);
      const T zz = noise[M + B + (int64_t)(pi * (pi + 1) / 2 + pj) * B + r];
      const T smp = pm + zz * sd;
      setlane(lreg, s, lane, diag ? dexp(smp) : smp);
      setlane(sdreg, s, lane, sd);
      setlane(zreg, s, lane, zz);
    }
    T lm = 0, lg = 0;
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      lm += lreg[u] * mreg[u];
      lg += lreg[u] * lreg[u] * greg[u];
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
      T mbar[NR], gbar[NR], sbar[NR], s2pb[NR];
      T cg = 0, c0 = 0;
#pragma unroll
      for (int u = 0; u < NR; ++u) {
        const int s = lane + 64 * u;
        const bool inr = s <= o;
        mbar[u] = inr ? Fbar * lreg[u] : (T)0;
        gbar[u] = inr ? cc * (-(lreg[u] * lreg[u]) / ((T)2 * s2e)) : (T)0;
        const T lbar = Fbar * mreg[u] + cc * (-(lreg[u] * greg[u]) / s2e);
        const T sb = inr ? (s == o ? lbar * lreg[u] : lbar) : (T)0;
        sbar[u] = sb;
        s2pb[u] = inr ? sb * zreg[u] / ((T)2 * sdreg[u]) : (T)0;
        cg += gbar[u];
        if (s < o) c0 += s2pb[u];
      }
      cg = wave_sum(cg);
      c0 = wave_sum(c0);
      const T c1 = bcast(s2pb, o);
      c0p = c0;
      c1p = c1;
      // d loss / d log s2_err  (Normal_logprob with scale sqrt(s2e), then the -0.5/s2e sum)
      epart = cc * ((res * res / (sc * sc * sc) - (T)1 / sc) / ((T)2 * sc) + (T)0.5 * lg / (s2e * s2e)) * s2e;
      // W-hat: scale the quadratic-form rows in place by 2*adjoint
      for (int s = 0; s <= o; ++s) {
        const T fg = (T)2 * bcast(gbar, s);
        const T fp = (T)2 * bcast(s2pb, s);
        T* wg = WG + (int64_t)s * BM + (int64_t)r * M;
        T* wp = WP + (int64_t)s * BM + (int64_t)r * M;
        for (int c = lane; c < M; c += 64) {
          wg[c] *= fg;
          wp[c] *= fp;
        }
      }
      // rows of the latent functions s > o are not computed by the W GEMM (l_s = 0 there) but the
      // k-concatenated P-bar GEMM reads them: store exact zeros
      for (int s = o + 1; s < D; ++s) {
        T* wg = WG + (int64_t)s * BM + (int64_t)r * M;
        for (int c = lane; c < M; c += 64) wg[c] = (T)0;
      }
      // P-bar initial rows (the rank-<=D mean terms and the -c*K12 diagonal term)
      T* acc = rowacc_all + (int64_t)w * M;
      T* PbG = (T*)a.Pbar + 3 * BM + (int64_t)r * M;
      T* Pb0 = (T*)a.Pbar + 1 * BM + (int64_t)r * M;
      T* Pb1 = (T*)a.Pbar + 2 * BM + (int64_t)r * M;
      for (int c = lane; c < M; c += 64) acc[c] = -cg * KG[c];
      for (int d = 0; d <= o; ++d) {
        const T mb = bcast(mbar, d);
        const T* mw = muW + (int64_t)d * M;
        for (int c = lane; c < M; c += 64) acc[c] += mb * mw[c];
      }
      for (int c = lane; c < M; c += 64) PbG[c] = acc[c];
      for (int c = lane; c < M; c += 64) acc[c] = -c0 * K0[c];
      for (int j = 0; j < o; ++j) {
        const T sb = bcast(sbar, j);
        const T* mu = muU + ((int64_t)o * D + j) * M;
        for (int c = lane; c < M; c += 64) acc[c] += sb * mu[c];
      }
      for (int c = lane; c < M; c += 64) Pb0[c] = acc[c];
      {
        const T sb = bcast(sbar, o);
        const T* mu = muU + ((int64_t)o * D + o) * M;
        for (int c = lane; c < M; c += 64) Pb1[c] = sb * mu[c] - c1 * K1[c];
      }
      RowBuf<T> rb{(T*)a.rowbuf, B, D};
#pragma unroll
      for (int u = 0; u < NR; ++u) {
        const int s = lane + 64 * u;
        if (s < D) {
          rb.mbar(s)[r] = mbar[u];
          rb.sbar(s)[r] = sbar[u];
        }
      }
      if (lane == 0) {
        rb.cG()[r] = cg;
        rb.c0()[r] = c0;
        rb.c1()[r] = c1;
      }
    }
  }
  if ((threadIdx.x & 63) != 0) Rrow = epart = c0p = c1p = 0;   // every lane holds the row's value
  Rrow = block_sum(Rrow, red);
  epart = block_sum(epart, red);
  c0p = block_sum(c0p, red);
  c1p = block_sum(c1p, red);
  if (threadIdx.x == 0) {
    T* rp = (T*)a.red + (int64_t)blockIdx.x * 4;
    rp[0] = Rrow;
    rp[1] = epart;
    rp[2] = c0p;
    rp[3] = c1p;
  }
}

// ------------------------------------------------------------------------------------ KL
template <typename T> __device__ inline const T* fac_S(const Args& a, int f) {
  const T* th = (const T*)a.theta;
  const int64_t MM = (int64_t)a.M * a.M;
  if (f < a.D) return th + a.off_sW + f * MM;
  if (f == a.NF - 1) return th + a.off_sv;
  int i, j;
  pair_ij(f - a.D, i, j);
  return th + a.off_sU + ((int64_t)i * a.D + j) * MM;
}
template <typename T> __device__ inline const T* fac_mu(const Args& a, int f) {
  const T* th = (const T*)a.theta;
  if (f < a.D) return th + a.off_muW + (int64_t)f * a.M;
  if (f == a.NF - 1) return th + a.off_muv;
  int i, j;
  pair_ij(f - a.D, i, j);
  return th + a.off_muU + ((int64_t)i * a.D + j) * a.M;
}
template <typename T> __device__ inline const T* fac_y(const Args& a, int f) {
  const T* Y = (const T*)a.Y;
  const int D = a.D, M = a.M;
  if (f < D) return Y + (int64_t)f * M;
  if (f == a.NF - 1) return Y + (int64_t)D * M;
  int i, j;
  pair_ij(f - D, i, j);
  const int64_t base = (int64_t)(D + 1) * M + (i == j ? (int64_t)D * D * M : 0);
  return Y + base + ((int64_t)i * D + j) * M;
}

// KL per factor, parallel over (factor, 16-row slab): 16 lanes per row sum tril(S)_i. squared
// (A1_ii - lam) with independent loads, then the per-row logdet / trace-quirk / Mahalanobis terms;
// each block leaves 4 partial sums in klpart[f][slab], summed in slab order by the finalize kernel.
constexpr int KL_ROWS = 16;
template <typename T> __device__ inline T* kl_part(const Args& a) {
  return (T*)a.facbuf + a.NF + 8 * (int64_t)a.M + 4 * (int64_t)a.D * a.D + (int64_t)a.NF * a.M;
}

template <typename T>
__global__ __launch_bounds__(256) void dsvi_kl_kernel(Args a) {
  __shared__ T red[4][16];
  const int M = a.M, D = a.D, NF = a.NF;
  const int64_t MM = (int64_t)M * M;
  const T lam = (T)a.jitter;
  const T* Af = (const T*)a.Afac;
  T* fb = (T*)a.facbuf;
  const int f = blockIdx.x, k = prior_of(f, D), slab = blockIdx.y;
  const int q = threadIdx.x & 15, i = slab * KL_ROWS + (threadIdx.x >> 4);
  const T* S = fac_S<T>(a, f);
  T ld1 = 0, ld2 = 0, t2 = 0, t3 = 0;
  T sq = 0;
  if (i < M) {
    for (int c = q; c <= i; c += 16) {
      const T x = S[(int64_t)i * M + c];
      sq += x * x;
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
    T* ev = fb + NF + 8 * (int64_t)M + 4 * (int64_t)D * D + (int64_t)f * M;
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
  const T* ev = fb + NF + 8 * (int64_t)M + 4 * (int64_t)D * D;
  T dl = 0;
  for (int f = 0; f < NF; ++f)
    if (prior_of(f, D) == k) dl += ev[(int64_t)f * M + i];
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
    const T* Kt = (const T*)a.K12 + (int64_t)r * M;
    T* Pb = (T*)a.Pbar + (int64_t)r * M;
    for (int c = lane; c < M; c += 64) Pb[c] = tbar * v[c] - varbar * Kt[c];
    if (lane == 0) {
      RowBuf<T> rb{(T*)a.rowbuf, B, a.D};
      rb.tbar()[r] = tbar;
      rb.varbar()[r] = varbar;
    }
    vb = (lane == 0) ? varbar : (T)0;
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
    T ez = 0;
    for (int rt = 0; rt < a.n_rt; ++rt) ez += gcol[(int64_t)rt * M + c];                 // G12 columns
    for (int ct = 0; ct < a.n_ct; ++ct) ez += grow[(int64_t)a.n_ct * B + (int64_t)ct * M + c];   // G22 rows
    for (int rt = 0; rt < a.n_rt22; ++rt) ez += gcol[(int64_t)a.n_rt * M + (int64_t)rt * M + c];  // G22 cols
    const T vb = vbar[c] + ez * ellZ[c];
    vbs[c] = vb;
    if (blockIdx.x == 0) vbar[M + c] = vb;
  }
  __syncthreads();
  const T* Cv = (const T*)a.Afac + (int64_t)(a.NF - 1) * M * M;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i0 = blockIdx.x * VBW_ROWS;
  for (int r = wv; r < VBW_ROWS; r += 4) {
    const int i = i0 + r;
    T s = 0;
    if (i < M)
      for (int k = i + lane; k < M; k += 64) s += Cv[(int64_t)k * M + i] * vbs[k];
    s = wave_sum(s);
    if (lane == 0) wrow[r] = s;
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

// ------------------------------------------------------------------------------------ finalize
template <typename T>
__global__ __launch_bounds__(256) void dsvi_finalize_kernel(Args a) {
  __shared__ T red[16];
  __shared__ T sc[8];
  const int D = a.D, M = a.M, NF = a.NF;
  const T* rp = (const T*)a.red;
  const T* fb = (const T*)a.facbuf;
  T R = 0, e = 0, c0 = 0, c1 = 0, vs = 0;
  for (int b = threadIdx.x; b < a.nblk_rows; b += blockDim.x) {
    R += rp[b * 4 + 0];
    e += rp[b * 4 + 1];
    c0 += rp[b * 4 + 2];
    c1 += rp[b * 4 + 3];
    if (!a.elbo_mode) vs += rp[(int64_t)a.nblk_rows * 4 + b];
  }
  R = block_sum(R, red);
  e = block_sum(e, red);
  c0 = block_sum(c0, red);
  c1 = block_sum(c1, red);
  vs = block_sum(vs, red);
  T klw = 0, klv = 0, klu = 0;
  const int nslab = (M + KL_ROWS - 1) / KL_ROWS;
  const T* kp = kl_part<T>(a);
  for (int f = threadIdx.x; f < NF; f += blockDim.x) {
    T p[4] = {0, 0, 0, 0};
    for (int sl = 0; sl < nslab; ++sl)
      for (int j = 0; j < 4; ++j) p[j] += kp[((int64_t)f * nslab + sl) * 4 + j];
    const T v = p[1] - p[0] + (T)0.5 * (p[2] + p[3] - (T)M);
    ((T*)a.facbuf)[f] = v;                       // per-factor KL (kept for inspection)
    if (f < D) klw += v; else if (f == NF - 1) klv += v; else klu += v;
  }
  klw = block_sum(klw, red);
  klv = block_sum(klv, red);
  klu = block_sum(klu, red);
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
  // scalar partials of the RBF backward problems: L0_12, L0_22, L1_12, L1_22, t12, t22
  const T* sp = (const T*)a.scal_part;
  for (int p = 0; p < 6; ++p) {
    T s0 = 0, s1 = 0;
    for (int64_t t = a.scal_off[p] + threadIdx.x; t < a.scal_off[p + 1]; t += blockDim.x) {
      s0 += sp[t * 2 + 0];
      s1 += sp[t * 2 + 1];
    }
    s0 = block_sum(s0, red);
    s1 = block_sum(s1, red);
    if (threadIdx.x == 0) {
      if (p == 0) { sc[0] = s0; sc[1] = s1; }
      else if (p == 1) { sc[0] += s0; sc[1] += s1; }
      else if (p == 2) { sc[2] = s0; sc[3] = s1; }
      else if (p == 3) { sc[2] += s0; sc[3] += s1; }
      else if (p == 4) { sc[4] = s0; sc[5] = s1; }
      else { sc[4] += s0; sc[5] += s1; }
    }
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
    for (int k = 0; k < 7; ++k) g[a.off_hyp + k] = (a.frozen_mask >> k & 1) ? (T)0 : gs[k];
  }
  // KL mean gradients A2^{-1} mu (Y) and mu_v += vbar
  const T* Y = (const T*)a.Y;
  for (int64_t idx = threadIdx.x; idx < (int64_t)D * M; idx += blockDim.x) g[a.off_muW + idx] += Y[idx];
  const T* vbar = (const T*)a.vbar + M;   // completed by the v-backward kernel
  for (int c = threadIdx.x; c < M; c += blockDim.x) g[a.off_muv + c] += vbar[c] + Y[(int64_t)D * M + c];
  const int64_t yu0 = (int64_t)(D + 1) * M, yu1 = yu0 + (int64_t)D * D * M;
  for (int64_t idx = threadIdx.x; idx < (int64_t)D * D * M; idx += blockDim.x) {
    const int ij = (int)(idx / M);
    const int i = ij / D, j = ij - i * D;
    if (j > i) continue;
    g[a.off_muU + idx] += (i == j ? Y[yu1 + idx] : Y[yu0 + idx]);
  }
}

// ------------------------------------------------------------------------------------ Adam
template <typename T>
__global__ void adam_kernel(T* th, const T* g, T* m, T* v, int64_t n, const int64_t* step, T lr, T b1, T b2,
                            T eps) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double t = (double)(step[0] + 1);
  const T bc1 = (T)(1.0 - pow((double)b1, t));
  const T bc2s = (T)sqrt(1.0 - pow((double)b2, t));
  const T gi = g[i];
  T mi = m[i];
  mi = mi + ((T)1 - b1) * (gi - mi);          // exp_avg.lerp_(grad, 1 - beta1)
  const T vi = v[i] * b2 + ((T)1 - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  const T denom = dsqrt(vi) / bc2s + eps;
  th[i] = th[i] - (lr / bc1) * (mi / denom);
}

__global__ void counter_add_kernel(int64_t* c, int64_t inc) { c[0] += inc; }

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

template <typename T>
__global__ void normal_kernel(T* out, int64_t n, uint64_t seed, const int64_t* counter, int64_t offset) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t * 4 >= n) return;
  const uint64_t base = (uint64_t)(counter ? counter[0] : 0) + (uint64_t)offset;
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
template <typename T> static int dsvi_trow(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  hipLaunchKernelGGL(dsvi_trow_kernel<T>, dim3(blocks_rows(a->B)), dim3(256), 0, s, *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T> static int dsvi_recon(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  if (a->D > 128) return -1;
  const size_t sm = (size_t)4 * a->M * sizeof(T);
  if (a->D <= 64)
    hipLaunchKernelGGL((dsvi_recon_kernel<T, 1>), dim3(blocks_rows(a->B)), dim3(256), sm, s, *a);
  else
    hipLaunchKernelGGL((dsvi_recon_kernel<T, 2>), dim3(blocks_rows(a->B)), dim3(256), sm, s, *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T> static int dsvi_kl(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  hipLaunchKernelGGL(dsvi_kl_kernel<T>, dim3(a->NF, (a->M + KL_ROWS - 1) / KL_ROWS), dim3(256), 0, s, *a);
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
  const size_t sm = (size_t)2 * a->M * sizeof(T);
  hipLaunchKernelGGL(dsvi_vbwd_kernel<T>, dim3((a->M + VBW_ROWS - 1) / VBW_ROWS), dim3(256), sm, s, *a);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
template <typename T> static int dsvi_finalize(const Args* a, hipStream_t s) {
  CHECK_ARGS(a);
  hipLaunchKernelGGL(dsvi_finalize_kernel<T>, dim3(1), dim3(256), 0, s, *a);
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
}  // namespace nmgp

extern "C" {
#define NMGP_DSVI_ENTRY(name)                                                                     \
  int nmgp_dsvi_##name##_f64(const Args* a, hipStream_t s) { return nmgp::dsvi_##name<double>(a, s); } \
  int nmgp_dsvi_##name##_f32(const Args* a, hipStream_t s) { return nmgp::dsvi_##name<float>(a, s); }
NMGP_DSVI_ENTRY(hyper)
NMGP_DSVI_ENTRY(trow)
NMGP_DSVI_ENTRY(recon)
NMGP_DSVI_ENTRY(kl)
NMGP_DSVI_ENTRY(delta)
NMGP_DSVI_ENTRY(tbwd)
NMGP_DSVI_ENTRY(vbwd)
NMGP_DSVI_ENTRY(finalize)
#undef NMGP_DSVI_ENTRY
int nmgp_adam_f64(double* th, const double* g, double* m, double* v, int64_t n, int64_t* step, double lr,
                  double b1, double b2, double eps, hipStream_t s) {
  if (!th) return -1;
  if (!g) return -2;
  if (!m) return -3;
  if (!v) return -4;
  if (!step) return -6;
  if (n <= 0) return NMGP_OK;
  hipLaunchKernelGGL(nmgp::adam_kernel<double>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, th, g, m, v, n,
                     step, lr, b1, b2, eps);
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
  hipLaunchKernelGGL(nmgp::adam_kernel<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, th, g, m, v, n,
                     step, (float)lr, (float)b1, (float)b2, (float)eps);
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
int nmgp_counter_add(int64_t* c, int64_t inc, hipStream_t s) {
  if (!c) return -1;
  hipLaunchKernelGGL(nmgp::counter_add_kernel, dim3(1), dim3(1), 0, s, c, inc);
  NMGP_CHECK_LAUNCH();
  return NMGP_OK;
}
}
