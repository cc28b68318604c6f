#include <cstdlib>
// Train-mode BatchNorm, Dropout2d masks and the element-wise backward kernels of the ROI path
// (gfx950).  All of them are HBM-streaming passes over NHWC activations: f32 arithmetic,
// storage in the compute dtype, statistics as deterministic per-split partials (no atomics)
// combined in double precision by a one-thread-per-channel finalize.
#include "common.h"
#include "hiseg_train.h"

namespace hiseg {

constexpr int kBnSplits = 1024;  // pixel splits of the statistics passes (4 blocks per CU)

template <typename T>
__device__ __forceinline__ float ld(const void* p, long long i) { return Elem<T>::load(p, i); }
template <typename T>
__device__ __forceinline__ void st(void* p, long long i, float v) { Elem<T>::store(p, i, v); }

__device__ __forceinline__ float act_grad(float y, int act) {
  switch (act) {
    case HISEG_ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case HISEG_ACT_SIGMOID: return y * (1.f - y);
    default: return 1.f;
  }
}

// Pixel range of split s.
__device__ __forceinline__ void split_range(long long P, int s, int S, long long& b, long long& e) {
  b = P * s / S;
  e = P * (s + 1) / S;
}

// ---------------------------------------------------------------------------------------- stats
// Block layout: CT = min(C, 256) channel lanes x R = 256/CT pixel rows; channel block blockIdx.y.
template <typename T>
__global__ void __launch_bounds__(256) bn_stats_kernel(const void* z, long long P, int C, int cs, int coff,
                                                       float* partial) {
  __shared__ float sh_n[256], sh_m[256], sh_q[256];
  const int CT = C < 256 ? C : 256;
  const int R = 256 / CT;
  const int t = threadIdx.x;
  const int cl = t % CT, r = t / CT;
  const int c = blockIdx.y * 256 + cl;
  long long b, e;
  split_range(P, blockIdx.x, gridDim.x, b, e);
  float n = 0.f, mean = 0.f, m2 = 0.f;
  if (r < R && c < C) {
    for (long long p = b + r; p < e; p += R) {
      const float x = ld<T>(z, p * cs + coff + c);
      n += 1.f;
      const float d = x - mean;
      mean += d / n;
      m2 += d * (x - mean);
    }
  }
  sh_n[t] = n; sh_m[t] = mean; sh_q[t] = m2;
  __syncthreads();
  if (r == 0 && c < C) {
    for (int rr = 1; rr < R; ++rr) {
      const int o = rr * CT + cl;
      const float nb = sh_n[o];
      if (nb == 0.f) continue;
      const float na = n, nt = na + nb;
      const float d = sh_m[o] - mean;
      mean += d * (nb / nt);
      m2 += sh_q[o] + d * d * (na * nb / nt);
      n = nt;
    }
    float* out = partial + (long long)blockIdx.x * 3 * C;
    out[c] = n; out[C + c] = mean; out[2 * C + c] = m2;
  }
}

// ---------------------------------------------------------------------------------------- apply
template <typename T>
__global__ void __launch_bounds__(256) bn_apply_kernel(hiseg_bn_apply_desc d) {
  const long long n = d.P * d.C;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long p = i / d.C;
    const int c = (int)(i - p * d.C);
    const long long tc = d.per_sample ? (p / d.HW) * d.C + c : c;
    float v = ld<T>(d.z, p * d.z_cstride + d.z_coff + c) * d.scale[tc] + d.shift[tc];
    if (d.residual) v += ld<T>(d.residual, p * d.r_cstride + d.r_coff + c);
    v = apply_act(v, d.act, d.act_beta);
    if (d.chan_mul) v *= d.chan_mul[(p / d.HW) * d.C + c];
    st<T>(d.y, p * d.y_cstride + d.y_coff + c, v);
  }
}

// ---------------------------------------------------------------------------------------- backward
__device__ __forceinline__ float silu_grad_pre(const hiseg_bn_bwd_desc& d, float z, int c) {
  const float v = (z - d.mean[c]) * d.invstd[c] * (d.gamma ? d.gamma[c] : 1.f) + (d.beta ? d.beta[c] : 0.f);
  const float s = 1.f / (1.f + expf(-v));
  return s * (1.f + v * (1.f - s));
}

// The derivative is taken at the forward's own pre-activation z*fwd_scale + fwd_shift (+ residual) when the
// folded affine is given and the activation needs it (smooth ones; ReLU after a residual add with the residual).
__host__ __device__ __forceinline__ bool bn_pre_path(const hiseg_bn_bwd_desc& d) {
  return d.fwd_scale && (act_smooth(d.act) || (d.act == HISEG_ACT_RELU && (!d.dres || d.residual)));
}

template <typename T>
__device__ __forceinline__ float bn_g(const hiseg_bn_bwd_desc& d, long long p, int c) {
  float g = ld<T>(d.dy, p * d.dy_cstride + d.dy_coff + c);
  if (d.chan_mul) g *= d.chan_mul[(p / d.HW) * d.C + c];
  if (bn_pre_path(d)) {
    float v = ld<T>(d.z, p * d.z_cstride + d.z_coff + c) * d.fwd_scale[c] + d.fwd_shift[c];
    if (d.residual) v += ld<T>(d.residual, p * d.r_cstride + d.r_coff + c);
    g *= act_grad_pre(v, d.act, d.act_beta);
  } else if (d.act == HISEG_ACT_SILU) g *= silu_grad_pre(d, ld<T>(d.z, p * d.z_cstride + d.z_coff + c), c);
  else if (d.act != HISEG_ACT_NONE) g *= act_grad(ld<T>(d.y, p * d.y_cstride + d.y_coff + c), d.act);
  return g;
}

template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(hiseg_bn_bwd_desc d) {
  __shared__ float sa[256], sb[256], sc[256];
  const int C = d.C;
  const int CT = C < 256 ? C : 256;
  const int R = 256 / CT;
  const int t = threadIdx.x;
  const int cl = t % CT, r = t / CT;
  const int c = blockIdx.y * 256 + cl;
  long long b, e;
  split_range(d.P, blockIdx.x, gridDim.x, b, e);
  float s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (r < R && c < C) {
    const float mu = d.mean[c], inv = d.invstd[c];
    for (long long p = b + r; p < e; p += R) {
      const float g = bn_g<T>(d, p, c);
      const float xh = (ld<T>(d.z, p * d.z_cstride + d.z_coff + c) - mu) * inv;
      s1 += g; s2 += g * xh; s3 += xh;
    }
  }
  sa[t] = s1; sb[t] = s2; sc[t] = s3;
  __syncthreads();
  if (r == 0 && c < C) {
    for (int rr = 1; rr < R; ++rr) {
      s1 += sa[rr * CT + cl]; s2 += sb[rr * CT + cl]; s3 += sc[rr * CT + cl];
    }
    float* out = d.partial + (long long)blockIdx.x * 3 * C;
    out[c] = s1; out[C + c] = s2; out[2 * C + c] = s3;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(hiseg_bn_bwd_desc d, int S) {
  const int C = d.C;
  const float* coef = d.partial + (long long)S * 3 * C;
  const long long n = d.P * C;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long p = i / C;
    const int c = (int)(i - p * C);
    const float g = bn_g<T>(d, p, c);
    const float xh = (ld<T>(d.z, p * d.z_cstride + d.z_coff + c) - d.mean[c]) * d.invstd[c];
    st<T>(d.dz, p * d.dz_cstride + d.dz_coff + c, coef[c] * (g - coef[C + c] - xh * coef[2 * C + c]));
    if (d.dres) {
      const long long o = p * d.dres_cstride + d.dres_coff + c;
      st<T>(d.dres, o, d.dres_accumulate ? ld<T>(d.dres, o) + g : g);
    }
  }
}

// ---------------------------------------------------------------------------------------- vectorised
// The same passes with one 16-B chunk (8 bf16 / 4 f32 channels) per thread per pixel: a wavefront
// reads 64 x 16 B = 1 KiB per load instruction, pixel rows of a block are contiguous in HBM (NHWC),
// so every pass streams at HBM rate.  Block = CT chunk lanes x R pixel rows (CT = min(C/VEC, 256)).
// Used whenever channels, strides and offsets are multiples of the chunk (all hiseg activations).
template <typename T>
__device__ __forceinline__ void ldv(const void* p, long long i, float* v) {
  Chunk<T>::unpack(*reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(p) + i), v);
}
template <typename T>
__device__ __forceinline__ void stv(void* p, long long i, const float* v) {
  *reinterpret_cast<uint4*>(reinterpret_cast<T*>(p) + i) = Chunk<T>::pack(v);
}

template <typename T>
__global__ void __launch_bounds__(256) bn_stats_vec_kernel(const void* z, long long P, int C, int cs, int coff,
                                                           float* partial) {
  constexpr int V = Chunk<T>::N;
  __shared__ float sh[256 * (2 * V + 1)];
  const int NCH = C / V;
  const int CT = NCH < 256 ? NCH : 256;
  const int R = 256 / CT;
  const int t = threadIdx.x;
  const int cl = t % CT, r = t / CT;
  const int ch = blockIdx.y * 256 + cl;
  const bool live = r < R && ch < NCH;
  long long b, e;
  split_range(P, blockIdx.x, gridDim.x, b, e);
  float n = 0.f, mean[V], m2[V];
#pragma unroll
  for (int k = 0; k < V; ++k) mean[k] = m2[k] = 0.f;
  if (live) {
    // four pixels' loads in flight before their Welford updates (the updates are a dependent chain; the loads are
    // not): the small deep layers give each thread tens of pixels at L2 / HBM latency.  Same update order as one by one.
    auto upd = [&](const float* x) __attribute__((always_inline)) {
      n += 1.f;
      const float rn = 1.f / n;
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const float d = x[k] - mean[k];
        mean[k] += d * rn;
        m2[k] += d * (x[k] - mean[k]);
      }
    };
    long long p = b + r;
    for (; p + 3 * R < e; p += 4 * R) {
      float x0[V], x1[V], x2[V], x3[V];
      ldv<T>(z, p * cs + coff + ch * V, x0);
      ldv<T>(z, (p + R) * cs + coff + ch * V, x1);
      ldv<T>(z, (p + 2 * R) * cs + coff + ch * V, x2);
      ldv<T>(z, (p + 3 * R) * cs + coff + ch * V, x3);
      upd(x0); upd(x1); upd(x2); upd(x3);
    }
    for (; p < e; p += R) {
      float x[V];
      ldv<T>(z, p * cs + coff + ch * V, x);
      upd(x);
    }
  }
  float* my = sh + t * (2 * V + 1);
  my[0] = n;
#pragma unroll
  for (int k = 0; k < V; ++k) { my[1 + k] = mean[k]; my[1 + V + k] = m2[k]; }
  // pairwise (tree) merge of the R pixel rows, fixed order: the one-thread walk over R - 1 rows was a dependent chain
  // of divisions (R = 128 for the 16-channel decoder layers: 31 us per 26 MB layer)
  for (int step = 1; step < R; step <<= 1) {
    __syncthreads();
    if (r % (2 * step) == 0 && r + step < R && ch < NCH) {
      const float* o = sh + ((r + step) * CT + cl) * (2 * V + 1);
      const float nb = o[0];
      if (nb != 0.f) {
        const float na = n, nt = na + nb;
#pragma unroll
        for (int k = 0; k < V; ++k) {
          const float d = o[1 + k] - mean[k];
          mean[k] += d * (nb / nt);
          m2[k] += o[1 + V + k] + d * d * (na * nb / nt);
        }
        n = nt;
        my[0] = n;
#pragma unroll
        for (int k = 0; k < V; ++k) { my[1 + k] = mean[k]; my[1 + V + k] = m2[k]; }
      }
    }
  }
  if (r == 0 && ch < NCH) {
    float* out = partial + (long long)blockIdx.x * 3 * C + ch * V;
#pragma unroll
    for (int k = 0; k < V; ++k) { out[k] = n; out[C + k] = mean[k]; out[2 * C + k] = m2[k]; }
  }
}

// Split groups of a large split count (the conv epilogue's fused statistics: one split per (pixel tile, wave), 12 288
// for a 256-ROI 64x48 layer): one block per (64 channels, KPRE consecutive splits), 4 rows x 64 channel lanes
// (coalesced loads across the lanes).  Row r sums every 4th split of the group as (n, sum n mean, sum M2 + n mean^2)
// in double -- no division in the loop -- and the 4 rows' sums are added in a fixed order; the group's (n, mean, M2)
// overwrites its own first split row (read by this block only), so bn_finalize_par_kernel merges S / KPRE rows at a
// stride of KPRE rows.  (One block per channel reading S strided rows: 85 us per 256-channel layer on 12 288 splits;
// this kernel with a Chan merge per split: 17 us.)
constexpr int KPRE = 64;
__global__ void __launch_bounds__(256) bn_premerge_kernel(float* partial, int S, int C) {
  __shared__ double sn[4][64], s1[4][64], s2[4][64];
  const int t = threadIdx.x, l = t & 63, r = t >> 6;
  const int c = blockIdx.x * 64 + l;
  const int s0 = blockIdx.y * KPRE;
  double n = 0, a = 0, b = 0;
  if (c < C) {
#pragma unroll 4
    for (int i = r; i < KPRE; i += 4) {
      if (s0 + i >= S) break;
      const float* p = partial + (long long)(s0 + i) * 3 * C;
      const double ni = p[c], mi = p[C + c], qi = p[2 * C + c];
      n += ni;
      a = fma(ni, mi, a);
      b += qi + ni * mi * mi;
    }
  }
  sn[r][l] = n; s1[r][l] = a; s2[r][l] = b;
  __syncthreads();
  if (r == 0 && c < C) {
    n = (sn[0][l] + sn[1][l]) + (sn[2][l] + sn[3][l]);
    a = (s1[0][l] + s1[1][l]) + (s1[2][l] + s1[3][l]);
    b = (s2[0][l] + s2[1][l]) + (s2[2][l] + s2[3][l]);
    const double mean = n > 0 ? a / n : 0.0;
    const double m2 = n > 0 ? fmax(b - a * mean, 0.0) : 0.0;
    float* o = partial + (long long)s0 * 3 * C;
    o[c] = (float)n;
    o[C + c] = (float)mean;
    o[2 * C + c] = (float)m2;
  }
}

// One block per channel: 256 threads merge the S split partials (rows `rs` floats apart; Chan, double), tree-combined
// in LDS.
__global__ void __launch_bounds__(256) bn_finalize_par_kernel(const float* partial, int S, int C, long long P,
                                                              const float* gamma, const float* beta, float eps,
                                                              float momentum, float* rm, float* rv, float* mean_o,
                                                              float* invstd_o, float* scale, float* shift,
                                                              long long rs) {
  __shared__ double sn[256], sm[256], sq[256];
  const int c = blockIdx.x, t = threadIdx.x;
  double n = 0, mean = 0, m2 = 0;
  // a thread's (up to four) partials loaded before its merges: one round of load latency instead of four
  for (int s0 = t; s0 < S; s0 += 1024) {
    float pn[4], pm[4], pq[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int s = s0 + 256 * u;
      const float* p = partial + (long long)(s < S ? s : 0) * rs;
      pn[u] = s < S ? p[c] : 0.f;
      pm[u] = p[C + c];
      pq[u] = p[2 * C + c];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double nb = pn[u];
      if (nb == 0) continue;
      const double d = pm[u] - mean, nt = n + nb;
      mean += d * nb / nt;
      m2 += pq[u] + d * d * n * nb / nt;
      n = nt;
    }
  }
  sn[t] = n; sm[t] = mean; sq[t] = m2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
      const double na = sn[t], nb = sn[t + w];
      if (nb > 0) {
        const double nt = na + nb, d = sm[t + w] - sm[t];
        sm[t] += d * nb / nt;
        sq[t] += sq[t + w] + d * d * na * nb / nt;
        sn[t] = nt;
      }
    }
    __syncthreads();
  }
  if (t == 0) {
    const double var = sq[0] / sn[0];
    const double inv = 1.0 / sqrt(var + (double)eps);
    const double mu = sm[0];
    const float g = gamma ? gamma[c] : 1.f, bb = beta ? beta[c] : 0.f;
    mean_o[c] = (float)mu;
    invstd_o[c] = (float)inv;
    scale[c] = (float)(g * inv);
    shift[c] = (float)(bb - mu * g * inv);
    if (rm) rm[c] = (float)((1.0 - momentum) * rm[c] + momentum * mu);
    if (rv) rv[c] = (float)((1.0 - momentum) * rv[c] + momentum * (P > 1 ? var * (double)P / (double)(P - 1) : var));
  }
}

// The same merge as 16 channel lanes x 16 split rows per block (round 6): row r sums splits r, r + 16, ... of its
// channel as (n, sum n mean, sum M2 + n mean^2) in double, four splits' loads in flight, no division in the loop
// (bn_premerge_kernel's form); the 16 rows are added in a fixed order.  C / 16 blocks instead of C: the per-channel
// kernel's 256-thread block and eight-level double Chan tree per channel cost ~7 us a call whatever S, on ~58 calls
// of the distillation student's forward.  Within f32 rounding of the Chan merge (test_bn_finalize_n_matches_f64_merge).
__global__ void __launch_bounds__(256) bn_finalize_rows_kernel(const float* partial, int S, int C, long long P,
                                                               const float* gamma, const float* beta, float eps,
                                                               float momentum, float* rm, float* rv, float* mean_o,
                                                               float* invstd_o, float* scale, float* shift,
                                                               long long rs) {
  __shared__ double sn[16][16], sa[16][16], sb[16][16];
  const int l = threadIdx.x & 15, r = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + l;
  double n = 0, a = 0, b = 0;
  if (c < C) {
    int s = r;
    for (; s + 48 < S; s += 64) {
      float pn[4], pm[4], pq[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* p = partial + (long long)(s + 16 * u) * rs;
        pn[u] = p[c];
        pm[u] = p[C + c];
        pq[u] = p[2 * C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double ni = pn[u], mi = pm[u];
        n += ni;
        a = fma(ni, mi, a);
        b += (double)pq[u] + ni * mi * mi;
      }
    }
    for (; s < S; s += 16) {
      const float* p = partial + (long long)s * rs;
      const double ni = p[c], mi = p[C + c];
      n += ni;
      a = fma(ni, mi, a);
      b += (double)p[2 * C + c] + ni * mi * mi;
    }
  }
  sn[r][l] = n; sa[r][l] = a; sb[r][l] = b;
  __syncthreads();
  if (r != 0 || c >= C) return;
  for (int q = 1; q < 16; ++q) { n += sn[q][l]; a += sa[q][l]; b += sb[q][l]; }
  const double mu = n > 0 ? a / n : 0.0;
  const double var = n > 0 ? fmax(b - a * mu, 0.0) / n : 0.0;
  const double inv = 1.0 / sqrt(var + (double)eps);
  const float g = gamma ? gamma[c] : 1.f, bb = beta ? beta[c] : 0.f;
  mean_o[c] = (float)mu;
  invstd_o[c] = (float)inv;
  scale[c] = (float)(g * inv);
  shift[c] = (float)(bb - mu * g * inv);
  if (rm) rm[c] = (float)((1.0 - momentum) * rm[c] + momentum * mu);
  if (rv) rv[c] = (float)((1.0 - momentum) * rv[c] + momentum * (P > 1 ? var * (double)P / (double)(P - 1) : var));
}

// Element-wise passes: block = CT chunk lanes x R pixel rows (as the reductions), blocks stride over pixel
// rows; 32-bit pixel indices (P < 2^31, checked on the host), no per-element 64-bit division.
template <typename T, int U = 1>
__global__ void __launch_bounds__(256) bn_apply_vec_kernel(hiseg_bn_apply_desc d) {
  constexpr int V = Chunk<T>::N;
  const int NCH = d.C / V;
  const int CT = NCH < 256 ? NCH : 256;
  const int R = 256 / CT;
  const int t = threadIdx.x;
  const int cl = t % CT, r = t / CT;
  const int ch = blockIdx.y * 256 + cl;
  if (r >= R || ch >= NCH) return;
  const int c = ch * V;
  const int P = (int)d.P;
  float sc[V], sf[V];
#pragma unroll
  for (int k = 0; k < V; ++k) { sc[k] = d.per_sample ? 0.f : d.scale[c + k]; sf[k] = d.per_sample ? 0.f : d.shift[c + k]; }
  // U pixels per iteration, their loads issued together (the pixels and the per-element arithmetic are U = 1's)
  const int stride = gridDim.x * R;
  for (int p0 = blockIdx.x * R + r; p0 < P; p0 += U * stride) {
    float v[U][V], rr[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + u * stride;
      if (p >= P) continue;
      ldv<T>(d.z, (long long)p * d.z_cstride + d.z_coff + c, v[u]);
      if (d.residual) ldv<T>(d.residual, (long long)p * d.r_cstride + d.r_coff + c, rr[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + u * stride;
      if (p >= P) continue;
      const float* cm = d.chan_mul ? d.chan_mul + (long long)(p / d.HW) * d.C + c : nullptr;
      if (d.per_sample) {   // LayerNorm2d: the sample's folded tables
        const long long tb = (long long)(p / d.HW) * d.C + c;
#pragma unroll
        for (int k = 0; k < V; ++k) { sc[k] = d.scale[tb + k]; sf[k] = d.shift[tb + k]; }
      }
#pragma unroll
      for (int k = 0; k < V; ++k) {
        float x = v[u][k] * sc[k] + sf[k];
        if (d.residual) x += rr[u][k];
        x = apply_act(x, d.act, d.act_beta);
        if (cm) x *= cm[k];
        v[u][k] = x;
      }
      stv<T>(d.y, (long long)p * d.y_cstride + d.y_coff + c, v[u]);
    }
  }
}

// How the backward pass gets act'(.) (bn_bwd_mode on the host; a template argument so the per-element loop
// carries no activation switch and the per-channel tables live in registers, loaded once per thread):
//   kGNone  identity;  kGY  act'(y) from the stored output (ReLU / Sigmoid, no folded affine given);
//   kGReLU  ReLU mask at the forward's pre-activation z*fwd_scale + fwd_shift (+ residual);
//   kGPre   any activation's derivative at that pre-activation (smooth ones; SiLU without the forward's tables
//           folds them here from mean / invstd / gamma / beta).
enum { kGNone = 0, kGY = 1, kGReLU = 2, kGPre = 3 };

__host__ __device__ __forceinline__ int bn_bwd_mode(const hiseg_bn_bwd_desc& d) {
  if (d.act == HISEG_ACT_NONE) return kGNone;
  if (bn_pre_path(d)) return d.act == HISEG_ACT_RELU ? kGReLU : kGPre;
  if (d.act == HISEG_ACT_SILU) return kGPre;
  return kGY;
}

// the pre-activation's per-channel affine of chunk c (modes kGReLU / kGPre)
template <int V>
__device__ __forceinline__ void bn_pre_tables(const hiseg_bn_bwd_desc& d, int c, float* fs, float* fh) {
#pragma unroll
  for (int k = 0; k < V; ++k) {
    if (d.fwd_scale) {
      fs[k] = d.fwd_scale[c + k];
      fh[k] = d.fwd_shift[c + k];
    } else {
      const float kk = d.invstd[c + k] * (d.gamma ? d.gamma[c + k] : 1.f);
      fs[k] = kk;
      fh[k] = (d.beta ? d.beta[c + k] : 0.f) - d.mean[c + k] * kk;
    }
  }
}

// g = dy (* chan_mul) * act'(.) for one 16-B chunk; z = the chunk's pre-BN values (already loaded)
template <typename T, int MODE>
__device__ __forceinline__ void bn_gv(const hiseg_bn_bwd_desc& d, int p, int c, float* g, const float* z,
                                      const float* fs, const float* fh) {
  constexpr int V = Chunk<T>::N;
  ldv<T>(d.dy, (long long)p * d.dy_cstride + d.dy_coff + c, g);
  if (d.chan_mul) {
    const float* cm = d.chan_mul + (long long)(p / d.HW) * d.C + c;
#pragma unroll
    for (int k = 0; k < V; ++k) g[k] *= cm[k];
  }
  if constexpr (MODE == kGReLU || MODE == kGPre) {
    float rr[V];
    if (d.residual) ldv<T>(d.residual, (long long)p * d.r_cstride + d.r_coff + c, rr);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float v = z[k] * fs[k] + fh[k];
      if (d.residual) v += rr[k];
      if constexpr (MODE == kGReLU) g[k] = v > 0.f ? g[k] : 0.f;
      else g[k] *= act_grad_pre(v, d.act, d.act_beta);
    }
  } else if constexpr (MODE == kGY) {
    float y[V];
    ldv<T>(d.y, (long long)p * d.y_cstride + d.y_coff + c, y);
#pragma unroll
    for (int k = 0; k < V; ++k) g[k] *= act_grad(y[k], d.act);
  }
}

template <typename T, int MODE>
__global__ void __launch_bounds__(256) bn_bwd_reduce_vec_kernel(hiseg_bn_bwd_desc d) {
  constexpr int V = Chunk<T>::N;
  __shared__ float sh[256 * 3 * V];
  const int C = d.C;
  const int NCH = C / V;
  const int CT = NCH < 256 ? NCH : 256;
  const int R = 256 / CT;
  const int t = threadIdx.x;
  const int cl = t % CT, r = t / CT;
  const int ch = blockIdx.y * 256 + cl;
  const int c = ch * V;
  long long b, e;
  split_range(d.P, blockIdx.x, gridDim.x, b, e);
  float s1[V], s2[V], s3[V];
#pragma unroll
  for (int k = 0; k < V; ++k) s1[k] = s2[k] = s3[k] = 0.f;
  if (r < R && ch < NCH) {
    float mu[V], inv[V], fs[V], fh[V];
#pragma unroll
    for (int k = 0; k < V; ++k) { mu[k] = d.mean[c + k]; inv[k] = d.invstd[c + k]; }
    if constexpr (MODE == kGReLU || MODE == kGPre) bn_pre_tables<V>(d, c, fs, fh);
    // (a four-way unroll here measured slower: 75 -> 91 and 103 -> 146 us on the train step's 256-channel layers)
    for (int p = (int)b + r; p < (int)e; p += R) {
      float g[V], z[V];
      ldv<T>(d.z, (long long)p * d.z_cstride + d.z_coff + c, z);
      bn_gv<T, MODE>(d, p, c, g, z, fs, fh);
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const float xh = (z[k] - mu[k]) * inv[k];
        s1[k] += g[k]; s2[k] += g[k] * xh; s3[k] += xh;
      }
    }
  }
  float* my = sh + t * 3 * V;
#pragma unroll
  for (int k = 0; k < V; ++k) { my[k] = s1[k]; my[V + k] = s2[k]; my[2 * V + k] = s3[k]; }
  // pairwise (tree) sum of the R pixel rows, fixed order (was one thread walking R - 1 rows)
  for (int step = 1; step < R; step <<= 1) {
    __syncthreads();
    if (r % (2 * step) == 0 && r + step < R && ch < NCH) {
      const float* o = sh + ((r + step) * CT + cl) * 3 * V;
#pragma unroll
      for (int k = 0; k < V; ++k) { s1[k] += o[k]; s2[k] += o[V + k]; s3[k] += o[2 * V + k]; }
#pragma unroll
      for (int k = 0; k < V; ++k) { my[k] = s1[k]; my[V + k] = s2[k]; my[2 * V + k] = s3[k]; }
    }
  }
  if (r == 0 && ch < NCH) {
    float* out = d.partial + (long long)blockIdx.x * 3 * C + c;
#pragma unroll
    for (int k = 0; k < V; ++k) { out[k] = s1[k]; out[C + k] = s2[k]; out[2 * C + k] = s3[k]; }
  }
}

__global__ void __launch_bounds__(256) bn_bwd_finalize_par_kernel(hiseg_bn_bwd_desc d, int S) {
  __shared__ double a1[256], a2[256], a3[256];
  const int c = blockIdx.x, t = threadIdx.x, C = d.C;
  double s1 = 0, s2 = 0, s3 = 0;
  for (int s0 = t; s0 < S; s0 += 1024) {   // (up to four partials' loads in flight, then the sums in order)
    float v1[4], v2[4], v3[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int s = s0 + 256 * u;
      const float* p = d.partial + (long long)(s < S ? s : 0) * 3 * C;
      v1[u] = s < S ? p[c] : 0.f;
      v2[u] = s < S ? p[C + c] : 0.f;
      v3[u] = s < S ? p[2 * C + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) { s1 += v1[u]; s2 += v2[u]; s3 += v3[u]; }
  }
  a1[t] = s1; a2[t] = s2; a3[t] = s3;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) { a1[t] += a1[t + w]; a2[t] += a2[t + w]; a3[t] += a3[t + w]; }
    __syncthreads();
  }
  if (t == 0) {
    s1 = a1[0]; s2 = a2[0]; s3 = a3[0];
    const double P = (double)d.P;
    const double k = (d.gamma ? d.gamma[c] : 1.0) * d.invstd[c];
    float* coef = d.partial + (long long)S * 3 * C;
    coef[c] = (float)k;
    coef[C + c] = (float)(s1 / P);
    coef[2 * C + c] = (float)(s2 / P);
    if (d.dgamma) d.dgamma[c] = (float)(d.accumulate_params ? d.dgamma[c] + s2 : s2);
    if (d.dbeta) d.dbeta[c] = (float)(d.accumulate_params ? d.dbeta[c] + s1 : s1);
    if (d.dconv_bias) {
      const double sdz = k * (s1 - P * (s1 / P) - s3 * (s2 / P));
      d.dconv_bias[c] = (float)(d.accumulate_params ? d.dconv_bias[c] + sdz : sdz);
    }
  }
}

template <typename T, int MODE, int U = 1>
__global__ void __launch_bounds__(256) bn_bwd_apply_vec_kernel(hiseg_bn_bwd_desc d, int S) {
  constexpr int V = Chunk<T>::N;
  const int C = d.C;
  const int NCH = C / V;
  const int CT = NCH < 256 ? NCH : 256;
  const int R = 256 / CT;
  const int t = threadIdx.x;
  const int cl = t % CT, r = t / CT;
  const int ch = blockIdx.y * 256 + cl;
  if (r >= R || ch >= NCH) return;
  const int c = ch * V;
  const float* coef = d.partial + (long long)S * 3 * C;
  float k0[V], k1[V], k2[V], mu[V], inv[V], fs[V], fh[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    k0[k] = coef[c + k]; k1[k] = coef[C + c + k]; k2[k] = coef[2 * C + c + k];
    mu[k] = d.mean[c + k]; inv[k] = d.invstd[c + k];
  }
  if constexpr (MODE == kGReLU || MODE == kGPre) bn_pre_tables<V>(d, c, fs, fh);
  const int P = (int)d.P;
  const int stride = gridDim.x * R;
  for (int p0 = blockIdx.x * R + r; p0 < P; p0 += U * stride) {
    float g[U][V], z[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {   // U pixels' loads together (bn_gv loads dy / y / residual)
      const int p = p0 + u * stride;
      if (p >= P) continue;
      ldv<T>(d.z, (long long)p * d.z_cstride + d.z_coff + c, z[u]);
      bn_gv<T, MODE>(d, p, c, g[u], z[u], fs, fh);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + u * stride;
      if (p >= P) continue;
      float o[V];
#pragma unroll
      for (int k = 0; k < V; ++k) o[k] = k0[k] * (g[u][k] - k1[k] - (z[u][k] - mu[k]) * inv[k] * k2[k]);
      stv<T>(d.dz, (long long)p * d.dz_cstride + d.dz_coff + c, o);
      if (d.dres) {
        const long long off = (long long)p * d.dres_cstride + d.dres_coff + c;
        if (d.dres_accumulate) {
          float rv[V];
          ldv<T>(d.dres, off, rv);
#pragma unroll
          for (int k = 0; k < V; ++k) g[u][k] += rv[k];
        }
        stv<T>(d.dres, off, g[u]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------- dropout
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void dropout2d_mask_kernel(int n, float p, unsigned long long seed, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float u = (float)(splitmix64(seed ^ splitmix64((unsigned long long)i)) >> 40) * (1.0f / 16777216.0f);
  out[i] = u < p ? 0.f : 1.f / (1.f - p);
}

// Device-resident seed: seed = (base * 0x9E3779B1 + offset) masked to 48 bits, base read from device memory, so
// a captured step replays with fresh masks once hiseg_seed_advance (captured with it) moved the base on.
__global__ void dropout2d_mask_dev_kernel(int n, float p, const unsigned long long* base, unsigned long long offset,
                                          float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long seed = (base[0] * 0x9E3779B1ull + offset) & 0xFFFFFFFFFFFFull;
  const float u = (float)(splitmix64(seed ^ splitmix64((unsigned long long)i)) >> 40) * (1.0f / 16777216.0f);
  out[i] = u < p ? 0.f : 1.f / (1.f - p);
}

__global__ void seed_advance_kernel(unsigned long long* base) {
  if (threadIdx.x == 0) base[0] += 1ull;
}

// ---------------------------------------------------------------------------------------- element-wise
#define EW_LOOP(P, C)                                                                                   \
  const long long n_ = (P) * (C);                                                                      \
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n_; i += (long long)gridDim.x * 256)

__device__ __forceinline__ long long vi(const hiseg_ew_view& v, long long p, int c) { return p * v.cstride + v.coff + c; }

template <typename T>
__global__ void __launch_bounds__(256) relu_bwd_kernel(long long P, int HW, int C, hiseg_ew_view dy, hiseg_ew_view y,
                                                       const float* mul, hiseg_ew_view dz) {
  EW_LOOP(P, C) {
    const long long p = i / C;
    const int c = (int)(i - p * C);
    float g = ld<T>(dy.p, vi(dy, p, c));
    if (mul) g *= mul[(p / HW) * C + c];
    st<T>(dz.p, vi(dz, p, c), ld<T>(y.p, vi(y, p, c)) > 0.f ? g : 0.f);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) sigmoid_bwd_kernel(long long P, int C, hiseg_ew_view dy, hiseg_ew_view s,
                                                          hiseg_ew_view dz) {
  EW_LOOP(P, C) {
    const long long p = i / C;
    const int c = (int)(i - p * C);
    const float v = ld<T>(s.p, vi(s, p, c));
    st<T>(dz.p, vi(dz, p, c), ld<T>(dy.p, vi(dy, p, c)) * v * (1.f - v));
  }
}

template <typename T>
__global__ void __launch_bounds__(256) gate_fwd_kernel(long long P, int C, hiseg_ew_view a, hiseg_ew_view g,
                                                       hiseg_ew_view out) {
  EW_LOOP(P, C) {
    const long long p = i / C;
    const int c = (int)(i - p * C);
    st<T>(out.p, vi(out, p, c), ld<T>(a.p, vi(a, p, c)) * ld<T>(g.p, vi(g, p, c)));
  }
}

template <typename T>
__global__ void __launch_bounds__(256) gate_bwd_kernel(long long P, int C, hiseg_ew_view dy, hiseg_ew_view a,
                                                       hiseg_ew_view g, hiseg_ew_view da, int acc, hiseg_ew_view dzg) {
  EW_LOOP(P, C) {
    const long long p = i / C;
    const int c = (int)(i - p * C);
    const float gy = ld<T>(dy.p, vi(dy, p, c));
    const float gv = ld<T>(g.p, vi(g, p, c));
    const float av = ld<T>(a.p, vi(a, p, c));
    if (da.p) {
      const long long o = vi(da, p, c);
      st<T>(da.p, o, acc ? ld<T>(da.p, o) + gy * gv : gy * gv);
    }
    if (dzg.p) st<T>(dzg.p, vi(dzg, p, c), gy * av * gv * (1.f - gv));
  }
}

// Vector form of gate_bwd_kernel: 16-B chunks, (channel chunk, pixel lane) threads as bn_apply_vec_kernel.
template <typename T>
__global__ void __launch_bounds__(256) gate_bwd_vec_kernel(int P, int C, hiseg_ew_view dy, hiseg_ew_view a,
                                                           hiseg_ew_view g, hiseg_ew_view da, int acc,
                                                           hiseg_ew_view dzg) {
  constexpr int V = Chunk<T>::N;
  const int NCH = C / V;
  const int CT = NCH < 256 ? NCH : 256;
  const int R = 256 / CT;
  const int cl = threadIdx.x % CT, r = threadIdx.x / CT;
  const int ch = blockIdx.y * 256 + cl;
  if (r >= R || ch >= NCH) return;
  const int c = ch * V;
  for (int p = blockIdx.x * R + r; p < P; p += gridDim.x * R) {
    float gy[V], gv[V], o[V];
    ldv<T>(dy.p, (long long)p * dy.cstride + dy.coff + c, gy);
    ldv<T>(g.p, (long long)p * g.cstride + g.coff + c, gv);
    if (da.p) {
      const long long off = (long long)p * da.cstride + da.coff + c;
      if (acc) ldv<T>(da.p, off, o);
#pragma unroll
      for (int k = 0; k < V; ++k) o[k] = acc ? o[k] + gy[k] * gv[k] : gy[k] * gv[k];
      stv<T>(da.p, off, o);
    }
    if (dzg.p) {
      float av[V];
      ldv<T>(a.p, (long long)p * a.cstride + a.coff + c, av);
#pragma unroll
      for (int k = 0; k < V; ++k) o[k] = gy[k] * av[k] * gv[k] * (1.f - gv[k]);
      stv<T>(dzg.p, (long long)p * dzg.cstride + dzg.coff + c, o);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) act_bwd_cvt_kernel(long long P, int C, hiseg_ew_view dy, hiseg_ew_view y, int act,
                                                          hiseg_ew_view dz, int acc) {
  EW_LOOP(P, C) {
    const long long p = i / C;
    const int c = (int)(i - p * C);
    float g = ld<float>(dy.p, vi(dy, p, c));
    if (act != HISEG_ACT_NONE) g *= act_grad(ld<float>(y.p, vi(y, p, c)), act);
    const long long o = vi(dz, p, c);
    st<T>(dz.p, o, acc ? ld<T>(dz.p, o) + g : g);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) add_kernel(long long P, int C, hiseg_ew_view dst, hiseg_ew_view src) {
  EW_LOOP(P, C) {
    const long long p = i / C;
    const int c = (int)(i - p * C);
    const long long o = vi(dst, p, c);
    st<T>(dst.p, o, ld<T>(dst.p, o) + ld<T>(src.p, vi(src, p, c)));
  }
}

template <typename T>
__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const void* x, int N, int H, int W, int C, const void* dy,
                                                          void* dx, int acc) {
  const int Ho = H / 2, Wo = W / 2;
  const long long n_ = (long long)N * Ho * Wo * C;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n_; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long long q = i / C;
    const int ox = (int)(q % Wo);
    const long long t2 = q / Wo;
    const int oy = (int)(t2 % Ho);
    const long long n = t2 / Ho;
    long long idx[4];
    float best = -INFINITY;
    int arg = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      idx[k] = ((n * H + 2 * oy + (k >> 1)) * W + 2 * ox + (k & 1)) * C + c;
      const float v = ld<T>(x, idx[k]);
      if (v > best || v != v) { best = v; arg = k; }
    }
    const float g = ld<T>(dy, q * C + c);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float add = k == arg ? g : 0.f;
      st<T>(dx, idx[k], acc ? ld<T>(dx, idx[k]) + add : add);
    }
  }
}

// PyTorch bilinear (align_corners=False) source index of output o: max(0, (o+0.5)*scale-0.5).
__device__ __forceinline__ void bl_src(int o, float scale, int in, int& i0, int& i1, float& l1) {
  float s = scale * (o + 0.5f) - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = s - i0;
}

__global__ void __launch_bounds__(256) resize_bwd_kernel(const float* dy, int NC, int h, int w, int H, int W, float* dx) {
  const long long n_ = (long long)NC * h * w;
  const float sh = (float)h / H, sw = (float)w / W;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n_; i += (long long)gridDim.x * 256) {
    const int ix = (int)(i % w);
    const int iy = (int)((i / w) % h);
    const long long pl = i / ((long long)h * w);
    const int oy_lo = max(0, (int)floorf((iy - 1.5f) / sh)), oy_hi = min(H - 1, (int)ceilf((iy + 1.5f) / sh));
    const int ox_lo = max(0, (int)floorf((ix - 1.5f) / sw)), ox_hi = min(W - 1, (int)ceilf((ix + 1.5f) / sw));
    float acc = 0.f;
    for (int oy = oy_lo; oy <= oy_hi; ++oy) {
      int y0, y1; float ly;
      bl_src(oy, sh, h, y0, y1, ly);
      const float wy = (y0 == iy ? 1.f - ly : 0.f) + (y1 == iy ? ly : 0.f);
      if (wy == 0.f) continue;
      for (int ox = ox_lo; ox <= ox_hi; ++ox) {
        int x0, x1; float lx;
        bl_src(ox, sw, w, x0, x1, lx);
        const float wx = (x0 == ix ? 1.f - lx : 0.f) + (x1 == ix ? lx : 0.f);
        if (wx != 0.f) acc += wy * wx * dy[(pl * H + oy) * W + ox];
      }
    }
    dx[i] = acc;
  }
}

// dx (+)= 2x2 sum of dy (nearest-x2 upsample backward), one 16-B chunk per thread
template <typename T>
__global__ void __launch_bounds__(256) up2_bwd_kernel(long long N, int h, int w, int C, hiseg_ew_view dy,
                                                      hiseg_ew_view dx, int accumulate) {
  constexpr int V = Chunk<T>::N;
  const int nch = C / V;
  const long long n_el = N * h * w * nch;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n_el; i += (long long)gridDim.x * 256) {
    const int ch = (int)(i % nch);
    const long long q = i / nch;            // low-res pixel
    const int x = (int)(q % w);
    const long long r = q / w;
    const int y = (int)(r % h);
    const long long n = r / h;
    float acc[V], v[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long long fp = (n * 2 * h + 2 * y + (j >> 1)) * (2 * w) + 2 * x + (j & 1);
      Chunk<T>::unpack(*reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(dy.p) + fp * dy.cstride + dy.coff +
                                                       ch * V), v);
#pragma unroll
      for (int k = 0; k < V; ++k) acc[k] += v[k];
    }
    T* dst = reinterpret_cast<T*>(dx.p) + q * dx.cstride + dx.coff + ch * V;
    if (accumulate) {
      Chunk<T>::unpack(*reinterpret_cast<const uint4*>(dst), v);
#pragma unroll
      for (int k = 0; k < V; ++k) acc[k] += v[k];
    }
    *reinterpret_cast<uint4*>(dst) = Chunk<T>::pack(acc);
  }
}

inline unsigned ew_blocks(long long n) {
  long long b = (n + 255) / 256;
  return (unsigned)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}


// ---------------------------------------------------------------------------------------- LayerNorm2d
// model.py:18-38: per sample n, mean / biased variance over (C, H, W), eps; y = (z - mean) * invstd * w + b.
// Statistics in double (per-thread sums of the sample's values), sample n's HW pixels split into Sp
// contiguous slices, one block per (slice, sample): CT channel-chunk lanes x R pixel rows, V channels per
// chunk (a 16-B chunk, or 1 on the scalar path).  The forward apply is hiseg_bn_apply with per-sample tables.
template <typename T, int V>
__device__ __forceinline__ void ldn(const void* p, long long i, float* v) {
  if constexpr (V == 1) v[0] = ld<T>(p, i);
  else ldv<T>(p, i, v);
}
template <typename T, int V>
__device__ __forceinline__ void stn(void* p, long long i, const float* v) {
  if constexpr (V == 1) st<T>(p, i, v[0]);
  else stv<T>(p, i, v);
}

__device__ __forceinline__ void ln_layout(int C, int V, int& NCH, int& CT, int& R) {
  NCH = C / V;
  CT = NCH < 256 ? NCH : 256;
  R = 256 / CT;
}

template <typename T, int V>
__global__ void __launch_bounds__(256) ln_stats_kernel(const void* z, int HW, int C, int cs, int coff, double* part) {
  __shared__ double s1[256], s2[256];
  int NCH, CT, R;
  ln_layout(C, V, NCH, CT, R);
  const int t = threadIdx.x, cl = t % CT, r = t / CT;
  const int n = blockIdx.y, Sp = gridDim.x;
  const long long b = (long long)HW * blockIdx.x / Sp, e = (long long)HW * (blockIdx.x + 1) / Sp;
  const long long p0 = (long long)n * HW;
  double a1 = 0.0, a2 = 0.0;
  if (r < R) {
    for (long long p = b + r; p < e; p += R)
      for (int ch = cl; ch < NCH; ch += CT) {
        float v[V];
        ldn<T, V>(z, (p0 + p) * cs + coff + ch * V, v);
#pragma unroll
        for (int k = 0; k < V; ++k) { a1 += v[k]; a2 += (double)v[k] * v[k]; }
      }
  }
  s1[t] = a1; s2[t] = a2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) { s1[t] += s1[t + w]; s2[t] += s2[t + w]; }
    __syncthreads();
  }
  if (t == 0) {
    double* o = part + ((long long)n * Sp + blockIdx.x) * 2;
    o[0] = s1[0]; o[1] = s2[0];
  }
}

__global__ void __launch_bounds__(256) ln_finalize_kernel(const double* part, int Sp, int C, int HW, const float* gamma,
                                                          const float* beta, float eps, float* mean, float* invstd,
                                                          float* scale, float* shift) {
  __shared__ double s1[256], s2[256];
  __shared__ float s_m, s_i;
  const int n = blockIdx.x, t = threadIdx.x;
  double a1 = 0.0, a2 = 0.0;
  for (int s = t; s < Sp; s += 256) { a1 += part[((long long)n * Sp + s) * 2]; a2 += part[((long long)n * Sp + s) * 2 + 1]; }
  s1[t] = a1; s2[t] = a2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) { s1[t] += s1[t + w]; s2[t] += s2[t + w]; }
    __syncthreads();
  }
  if (t == 0) {
    const double M = (double)C * HW;
    const double m = s1[0] / M;
    double var = s2[0] / M - m * m;
    if (var < 0.0) var = 0.0;
    s_m = (float)m;
    s_i = (float)(1.0 / sqrt(var + (double)eps));
    mean[n] = s_m;
    invstd[n] = s_i;
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    const float k = (gamma ? gamma[c] : 1.f) * s_i;
    scale[(long long)n * C + c] = k;
    shift[(long long)n * C + c] = (beta ? beta[c] : 0.f) - s_m * k;
  }
}

// Backward.  g = dy * chan_mul * act'(pre), pre = z*scale[n][c] + shift[n][c] (+ residual), xhat = (z - mean_n)
// * invstd_n; per block and channel: G = sum g, GX = sum g*xhat, X = sum xhat (blocks never straddle samples)
//   per sample:  a_n = sum_c w_c G_nc / M,  b_n = sum_c w_c GX_nc / M   (M = C*HW)
//   dz = invstd_n * (g*w_c - a_n - xhat*b_n),  dw_c = sum GX, db_c = sum G,
//   dconv_bias_c = sum_n invstd_n * (w_c G_nc - HW a_n - X_nc b_n)
template <typename T, int V>
__device__ __forceinline__ void ln_g(const hiseg_ln_bwd_desc& d, long long p, int n, int c, const float* z, float* g) {
  ldn<T, V>(d.dy, p * d.dy_cstride + d.dy_coff + c, g);
  float rr[V];
  if (d.residual) ldn<T, V>(d.residual, p * d.r_cstride + d.r_coff + c, rr);
  const long long tb = (long long)n * d.C + c;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    if (d.chan_mul) g[k] *= d.chan_mul[tb + k];
    if (d.act != HISEG_ACT_NONE) {
      float v = z[k] * d.scale[tb + k] + d.shift[tb + k];
      if (d.residual) v += rr[k];
      g[k] *= act_grad_pre(v, d.act, d.act_beta);
    }
  }
}

template <typename T, int V>
__global__ void __launch_bounds__(256) ln_bwd_reduce_kernel(hiseg_ln_bwd_desc d, float* part) {
  int NCH, CT, R;
  ln_layout(d.C, V, NCH, CT, R);
  const int t = threadIdx.x, cl = t % CT, r = t / CT;
  const int n = blockIdx.y, Sp = gridDim.x, C = d.C;
  const long long b = (long long)d.HW * blockIdx.x / Sp, e = (long long)d.HW * (blockIdx.x + 1) / Sp;
  const long long p0 = (long long)n * d.HW;
  const float mu = d.mean[n], inv = d.invstd[n];
  float* out = part + ((long long)n * Sp + blockIdx.x) * 3 * C;
  __shared__ float sh[3][256][V];
  for (int cg = 0; cg < NCH; cg += CT) {   // channel groups of CT chunks
    const int ch = cg + cl;
    float s1[V], s2[V], s3[V];
#pragma unroll
    for (int k = 0; k < V; ++k) s1[k] = s2[k] = s3[k] = 0.f;
    if (r < R && ch < NCH) {
      for (long long p = b + r; p < e; p += R) {
        float z[V], g[V];
        ldn<T, V>(d.z, (p0 + p) * d.z_cstride + d.z_coff + ch * V, z);
        ln_g<T, V>(d, p0 + p, n, ch * V, z, g);
#pragma unroll
        for (int k = 0; k < V; ++k) {
          const float xh = (z[k] - mu) * inv;
          s1[k] += g[k]; s2[k] += g[k] * xh; s3[k] += xh;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < V; ++k) { sh[0][t][k] = s1[k]; sh[1][t][k] = s2[k]; sh[2][t][k] = s3[k]; }
    __syncthreads();
    if (r == 0 && ch < NCH) {
      for (int rr = 1; rr < R; ++rr) {
#pragma unroll
        for (int k = 0; k < V; ++k) {
          s1[k] += sh[0][rr * CT + cl][k]; s2[k] += sh[1][rr * CT + cl][k]; s3[k] += sh[2][rr * CT + cl][k];
        }
      }
#pragma unroll
      for (int k = 0; k < V; ++k) { out[ch * V + k] = s1[k]; out[C + ch * V + k] = s2[k]; out[2 * C + ch * V + k] = s3[k]; }
    }
    __syncthreads();
  }
}

// per sample: the Sp slices' sums -> nc [N][3][C] and coef [N][2] = (a_n, b_n)
__global__ void __launch_bounds__(256) ln_bwd_sample_kernel(hiseg_ln_bwd_desc d, const float* part, int Sp, float* nc,
                                                            float* coef) {
  __shared__ double sa[256], sb[256];
  const int n = blockIdx.x, t = threadIdx.x, C = d.C;
  double a = 0.0, bb = 0.0;
  for (int c = t; c < C; c += 256) {
    double G = 0.0, GX = 0.0, X = 0.0;
    for (int s = 0; s < Sp; ++s) {
      const float* q = part + ((long long)n * Sp + s) * 3 * C;
      G += q[c]; GX += q[C + c]; X += q[2 * C + c];
    }
    float* o = nc + (long long)n * 3 * C;
    o[c] = (float)G; o[C + c] = (float)GX; o[2 * C + c] = (float)X;
    const double w = d.gamma ? d.gamma[c] : 1.0;
    a += w * G; bb += w * GX;
  }
  sa[t] = a; sb[t] = bb;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) { sa[t] += sa[t + w]; sb[t] += sb[t + w]; }
    __syncthreads();
  }
  if (t == 0) {
    const double M = (double)C * d.HW;
    coef[n * 2] = (float)(sa[0] / M);
    coef[n * 2 + 1] = (float)(sb[0] / M);
  }
}

// per channel: dw, db, dconv_bias over the samples
__global__ void __launch_bounds__(256) ln_bwd_channel_kernel(hiseg_ln_bwd_desc d, const float* nc, const float* coef) {
  const int c = blockIdx.x * 256 + threadIdx.x, C = d.C;
  if (c >= C) return;
  const double w = d.gamma ? d.gamma[c] : 1.0;
  double G = 0.0, GX = 0.0, DB = 0.0;
  for (int n = 0; n < d.N; ++n) {
    const float* o = nc + (long long)n * 3 * C;
    G += o[c]; GX += o[C + c];
    DB += (double)d.invstd[n] * (w * o[c] - (double)d.HW * coef[n * 2] - (double)o[2 * C + c] * coef[n * 2 + 1]);
  }
  if (d.dgamma) d.dgamma[c] = (float)(d.accumulate_params ? d.dgamma[c] + GX : GX);
  if (d.dbeta) d.dbeta[c] = (float)(d.accumulate_params ? d.dbeta[c] + G : G);
  if (d.dconv_bias) d.dconv_bias[c] = (float)(d.accumulate_params ? d.dconv_bias[c] + DB : DB);
}

template <typename T, int V>
__global__ void __launch_bounds__(256) ln_bwd_apply_kernel(hiseg_ln_bwd_desc d, const float* coef) {
  int NCH, CT, R;
  ln_layout(d.C, V, NCH, CT, R);
  const int t = threadIdx.x, cl = t % CT, r = t / CT;
  if (r >= R) return;
  const long long P = (long long)d.N * d.HW;
  for (long long p = (long long)blockIdx.x * R + r; p < P; p += (long long)gridDim.x * R) {
    const int n = (int)(p / d.HW);
    const float mu = d.mean[n], inv = d.invstd[n], an = coef[n * 2], bn = coef[n * 2 + 1];
    for (int ch = cl; ch < NCH; ch += CT) {
      const int c = ch * V;
      float z[V], g[V], o[V];
      ldn<T, V>(d.z, p * d.z_cstride + d.z_coff + c, z);
      ln_g<T, V>(d, p, n, c, z, g);
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const float w = d.gamma ? d.gamma[c + k] : 1.f;
        o[k] = inv * (g[k] * w - an - (z[k] - mu) * inv * bn);
      }
      stn<T, V>(d.dz, p * d.dz_cstride + d.dz_coff + c, o);
      if (d.dres) {
        const long long off = p * d.dres_cstride + d.dres_coff + c;
        if (d.dres_accumulate) {
          float q[V];
          ldn<T, V>(d.dres, off, q);
#pragma unroll
          for (int k = 0; k < V; ++k) g[k] += q[k];
        }
        stn<T, V>(d.dres, off, g);
      }
    }
  }
}

// dz (+)= dy * act'(z) for an activation applied without normalisation (the fg_gate convs with GELU / Swish /
// SiLU: the conv writes the pre-activation, hiseg_bn_apply with unit tables the activation).
template <typename T>
__global__ void __launch_bounds__(256) act_bwd_pre_kernel(long long P, int C, hiseg_ew_view dy, hiseg_ew_view z, int act,
                                                          float beta, hiseg_ew_view dz, int accumulate) {
  EW_LOOP(P, C) {
    const long long p = i / C;
    const int c = (int)(i - p * C);
    float g = ld<T>(dy.p, vi(dy, p, c)) * act_grad_pre(ld<T>(z.p, vi(z, p, c)), act, beta);
    if (accumulate) g += ld<T>(dz.p, vi(dz, p, c));
    st<T>(dz.p, vi(dz, p, c), g);
  }
}
}  // namespace hiseg

using namespace hiseg;

#define DISPATCH_T(dtype, ...)                       \
  do {                                               \
    if ((dtype) == HISEG_BF16) {                     \
      using T = bf16_t;                              \
      __VA_ARGS__;                                   \
    } else {                                         \
      using T = float;                               \
      __VA_ARGS__;                                   \
    }                                                \
  } while (0)

extern "C" int hiseg_bn_partials(void) { return kBnSplits; }

// pixels per iteration of the element-wise BN passes (HISEG_BN_U, read per call: A/B timing; same results).  Two
// measured no faster (tools/bn_bench.py, profiles/r4_bn_bench.txt: apply 5.1-5.4 TB/s, backward 4.3-4.7 TB/s of
// algorithmic bytes at U = 1 -- 0.7-0.85 of the ~6.3 TB/s a copy reaches), so U = 1 stays
static int bn_unroll() {
  const char* e = getenv("HISEG_BN_U");
  return e && atoi(e) == 2 ? 2 : 1;
}

// 16-B chunk path eligibility: channel count, strides and offsets in whole chunks, aligned base.
static bool vec_ok(int dtype, int C, const void* p, int cs, int coff) {
  const int v = dtype == HISEG_BF16 ? 8 : 4;
  return p == nullptr || (C % v == 0 && cs % v == 0 && coff % v == 0 && al16(p));
}

// Grid of the element-wise passes: pixel-row blocks (<= 2048 -> 8 waves per SIMD), channel groups in y.
static dim3 vec_grid(long long P, int C, int dtype) {
  const int nch = C / (dtype == HISEG_BF16 ? 8 : 4);
  const int ct = nch < 256 ? nch : 256, R = 256 / ct;
  long long bx = (P + R - 1) / R;
  if (bx > 2048) bx = 2048;
  return dim3((unsigned)(bx < 1 ? 1 : bx), (unsigned)((nch + 255) / 256));
}

static int splits_for(long long P) { return (int)(P < kBnSplits ? (P > 0 ? P : 1) : kBnSplits); }

// Pixel splits of the statistics / backward-reduce passes: >= 32 pixels per split, at most kBnSplits (4 blocks per
// CU).  The deep low-resolution layers (the distillation student's 4 x 20 x 20 = 1 600-pixel stages) used to take
// 1 024 one- or two-pixel splits whose merge was most of their BN time.  A function of P alone, so hiseg_bn_stats and
// hiseg_bn_finalize agree.
static int stat_splits(long long P) {
  const long long s = P / 32;
  return (int)(s < 1 ? 1 : s > kBnSplits ? kBnSplits : s);
}
static dim3 fin_grid(int C) { return dim3((unsigned)C); }   // one block per channel

// HISEG_BN_FIN (read per call): 1 bn_finalize_rows_kernel, 0 the per-channel Chan-tree kernel, 2 (default) the rows
// kernel up to 256 splits (a row walks S / 16 of them; more take the per-channel kernel's one round of loads)
static bool bn_fin_rows(int S) {
  const char* e = getenv("HISEG_BN_FIN");
  const int m = e ? atoi(e) : 2;
  return m == 1 || (m == 2 && S <= 256);
}

static void bn_fin_launch(const float* partial, int S, int C, long long P, const float* gamma, const float* beta,
                          float eps, float momentum, float* rm, float* rv, float* mean, float* invstd, float* scale,
                          float* shift, hipStream_t stream, long long rs) {
  if (bn_fin_rows(S))
    hipLaunchKernelGGL(bn_finalize_rows_kernel, dim3((unsigned)((C + 15) / 16)), dim3(256), 0, stream, partial, S, C,
                       P, gamma, beta, eps, momentum, rm, rv, mean, invstd, scale, shift, rs);
  else
    hipLaunchKernelGGL(bn_finalize_par_kernel, fin_grid(C), dim3(256), 0, stream, partial, S, C, P, gamma, beta, eps,
                       momentum, rm, rv, mean, invstd, scale, shift, rs);
}

extern "C" int hiseg_bn_stats(int dtype, const void* z, long long P, int C, int cstride, int coff, float* partial,
                              hiseg_stream_t stream) {
  HISEG_REQUIRE(z && partial && P > 0 && C > 0 && cstride >= C, HISEG_ERR_BAD_ARG, "bn_stats: bad arguments");
  HISEG_REQUIRE(dtype == HISEG_F32 || dtype == HISEG_BF16, HISEG_ERR_BAD_DTYPE, "bn_stats: dtype");
  const int S = stat_splits(P);   // empty splits write n = 0
  if (vec_ok(dtype, C, z, cstride, coff)) {
    const int V = dtype == HISEG_BF16 ? 8 : 4;
    dim3 grid(S, (C / V + 255) / 256);
    DISPATCH_T(dtype, hipLaunchKernelGGL(bn_stats_vec_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream, z, P, C,
                                         cstride, coff, partial));
    return hiseg_check_launch("bn_stats");
  }
  dim3 grid(S, (C + 255) / 256);
  DISPATCH_T(dtype, hipLaunchKernelGGL(bn_stats_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream, z, P, C, cstride,
                                       coff, partial));
  return hiseg_check_launch("bn_stats");
}

extern "C" int hiseg_bn_finalize(const float* partial, int C, long long P, const float* gamma, const float* beta,
                                 float eps, float momentum, float* running_mean, float* running_var, float* mean,
                                 float* invstd, float* scale, float* shift, hiseg_stream_t stream) {
  HISEG_REQUIRE(partial && mean && invstd && scale && shift && C > 0, HISEG_ERR_BAD_ARG, "bn_finalize: null");
  bn_fin_launch(partial, stat_splits(P), C, P, gamma, beta, eps, momentum, running_mean, running_var, mean, invstd, scale,
                shift, (hipStream_t)stream, 3ll * C);
  return hiseg_check_launch("bn_finalize");
}

// The same merge over an explicit split count (the fused upsample_bg_fg statistics, train_head.hip: 1 024 splits).
int bn_finalize_splits(const float* partial, int S, int C, long long P, const float* gamma, const float* beta,
                       float eps, float momentum, float* running_mean, float* running_var, float* mean, float* invstd,
                       float* scale, float* shift, hipStream_t stream, long long rs = 0) {
  bn_fin_launch(partial, S, C, P, gamma, beta, eps, momentum, running_mean, running_var, mean, invstd, scale, shift, stream,
                rs ? rs : 3ll * C);
  return hiseg_check_launch("bn_finalize");
}

extern "C" int hiseg_bn_finalize_n(float* partial, int S, int C, long long P, const float* gamma,
                                   const float* beta, float eps, float momentum, float* running_mean,
                                   float* running_var, float* mean, float* invstd, float* scale, float* shift,
                                   hiseg_stream_t stream) {
  HISEG_REQUIRE(partial && mean && invstd && scale && shift && C > 0 && S > 0 && P > 0, HISEG_ERR_BAD_ARG,
                "bn_finalize_n: bad arguments");
  long long rs = 3ll * C;
  if (S > 4 * KPRE) {   // the conv epilogue's split counts: pre-merged in groups of KPRE first, in place
    const int G = (S + KPRE - 1) / KPRE;
    hipLaunchKernelGGL(bn_premerge_kernel, dim3((C + 63) / 64, G), dim3(256), 0, (hipStream_t)stream, partial, S, C);
    const int e = hiseg_check_launch("bn_premerge");
    if (e) return e;
    S = G;
    rs *= KPRE;
  }
  return bn_finalize_splits(partial, S, C, P, gamma, beta, eps, momentum, running_mean, running_var, mean, invstd,
                            scale, shift, (hipStream_t)stream, rs);
}

extern "C" int hiseg_bn_apply(const hiseg_bn_apply_desc* d, hiseg_stream_t stream) {
  HISEG_REQUIRE(d && d->z && d->y && d->scale && d->shift && d->P > 0 && d->C > 0 && d->HW > 0, HISEG_ERR_BAD_ARG,
                "bn_apply: bad arguments");
  HISEG_REQUIRE(d->P < (1ll << 31), HISEG_ERR_BAD_SHAPE, "bn_apply: too many pixels");
  if (vec_ok(d->dtype, d->C, d->z, d->z_cstride, d->z_coff) && vec_ok(d->dtype, d->C, d->y, d->y_cstride, d->y_coff) &&
      vec_ok(d->dtype, d->C, d->residual, d->r_cstride, d->r_coff)) {
    if (bn_unroll() == 2)
      DISPATCH_T(d->dtype, hipLaunchKernelGGL((bn_apply_vec_kernel<T, 2>), vec_grid(d->P, d->C, d->dtype), dim3(256),
                                              0, (hipStream_t)stream, *d));
    else
      DISPATCH_T(d->dtype, hipLaunchKernelGGL((bn_apply_vec_kernel<T, 1>), vec_grid(d->P, d->C, d->dtype), dim3(256),
                                              0, (hipStream_t)stream, *d));
    return hiseg_check_launch("bn_apply");
  }
  DISPATCH_T(d->dtype, hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(ew_blocks(d->P * d->C)), dim3(256), 0,
                                          (hipStream_t)stream, *d));
  return hiseg_check_launch("bn_apply");
}

// Group sums of the data-gradient epilogue's backward-reduction partials (hiseg_bn_bwd_desc.partial_splits): block
// (64 channels, KPRE splits), 4 rows x 64 channel lanes, row r summing every 4th split, the rows added in a fixed
// order; group g's sums go to row g of `out` (a region after the partials).
__global__ void __launch_bounds__(256) bn_bwd_premerge_kernel(const float* partial, int S, int C, float* out) {
  __shared__ float a1[4][64], a2[4][64], a3[4][64];
  const int t = threadIdx.x, l = t & 63, r = t >> 6;
  const int c = blockIdx.x * 64 + l;
  const int s0 = blockIdx.y * KPRE;
  float x1 = 0.f, x2 = 0.f, x3 = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int i = r; i < KPRE; i += 4) {
      if (s0 + i >= S) break;
      const float* p = partial + (long long)(s0 + i) * 3 * C;
      x1 += p[c];
      x2 += p[C + c];
      x3 += p[2 * C + c];
    }
  }
  a1[r][l] = x1; a2[r][l] = x2; a3[r][l] = x3;
  __syncthreads();
  if (r == 0 && c < C) {
    float* o = out + (long long)blockIdx.y * 3 * C;
    o[c] = (a1[0][l] + a1[1][l]) + (a1[2][l] + a1[3][l]);
    o[C + c] = (a2[0][l] + a2[1][l]) + (a2[2][l] + a2[3][l]);
    o[2 * C + c] = (a3[0][l] + a3[1][l]) + (a3[2][l] + a3[3][l]);
  }
}

extern "C" int hiseg_bn_bwd(const hiseg_bn_bwd_desc* d_in, hiseg_stream_t stream) {
  HISEG_REQUIRE(d_in, HISEG_ERR_BAD_ARG, "bn_bwd: null descriptor");
  hiseg_bn_bwd_desc dd = *d_in;
  const hiseg_bn_bwd_desc* d = &dd;
  HISEG_REQUIRE(d && d->dy && d->z && d->dz && d->mean && d->invstd && d->partial && d->P > 0 && d->C > 0 && d->HW > 0,
                HISEG_ERR_BAD_ARG, "bn_bwd: bad arguments");
  const bool pre = d->fwd_scale && d->fwd_shift &&
                   (act_smooth(d->act) || (d->act == HISEG_ACT_RELU && (!d->dres || d->residual)));
  HISEG_REQUIRE(pre || d->act == HISEG_ACT_NONE || d->act == HISEG_ACT_SILU || d->y, HISEG_ERR_BAD_ARG,
                "bn_bwd: activation needs y");
  HISEG_REQUIRE(pre || (d->act != HISEG_ACT_GELU && d->act != HISEG_ACT_SWISH), HISEG_ERR_BAD_ARG,
                "bn_bwd: GELU / Swish need the forward's fwd_scale / fwd_shift");
  HISEG_REQUIRE(!d->dres || !act_smooth(d->act) || (pre && d->residual), HISEG_ERR_BAD_ARG,
                "bn_bwd: a smooth activation after a residual add needs the residual (pre-activation)");
  HISEG_REQUIRE(d->P < (1ll << 31), HISEG_ERR_BAD_SHAPE, "bn_bwd: too many pixels");
  hipStream_t s = (hipStream_t)stream;
  int S = stat_splits(d->P);
  const int dt = d->dtype, C = d->C;
  // the reduction already done by the data-gradient conv's epilogue (hiseg_conv2d_desc.bnb_partial): more than
  // 4 KPRE splits are summed in groups first, into the region after them
  const bool pre_red = d->partial_splits > 0;
  if (pre_red) {
    S = d->partial_splits;
    if (S > 4 * KPRE) {
      const int G = (S + KPRE - 1) / KPRE;
      float* grp = dd.partial + (long long)S * 3 * C;
      hipLaunchKernelGGL(bn_bwd_premerge_kernel, dim3((C + 63) / 64, G), dim3(256), 0, s, d->partial, S, C, grp);
      const int e = hiseg_check_launch("bn_bwd_premerge");
      if (e) return e;
      dd.partial = grp;
      S = G;
    }
  }
  if (vec_ok(dt, C, d->dy, d->dy_cstride, d->dy_coff) && vec_ok(dt, C, d->y, d->y_cstride, d->y_coff) &&
      vec_ok(dt, C, d->z, d->z_cstride, d->z_coff) && vec_ok(dt, C, d->dz, d->dz_cstride, d->dz_coff) &&
      vec_ok(dt, C, d->dres, d->dres_cstride, d->dres_coff) && vec_ok(dt, C, d->residual, d->r_cstride, d->r_coff)) {
    const int V = dt == HISEG_BF16 ? 8 : 4;
    const dim3 rgrid(S, (C / V + 255) / 256), agrid = vec_grid(d->P, C, dt);
    const int mode = bn_bwd_mode(*d);
#define BN_BWD_VEC(M)                                                                                         \
  do {                                                                                                        \
    if (!pre_red)                                                                                             \
      DISPATCH_T(dt, hipLaunchKernelGGL((bn_bwd_reduce_vec_kernel<T, M>), rgrid, dim3(256), 0, s, *d));       \
    hipLaunchKernelGGL(bn_bwd_finalize_par_kernel, fin_grid(C), dim3(256), 0, s, *d, S);                          \
    if (bn_unroll() == 2)                                                                                     \
      DISPATCH_T(dt, hipLaunchKernelGGL((bn_bwd_apply_vec_kernel<T, M, 2>), agrid, dim3(256), 0, s, *d, S));  \
    else                                                                                                      \
      DISPATCH_T(dt, hipLaunchKernelGGL((bn_bwd_apply_vec_kernel<T, M, 1>), agrid, dim3(256), 0, s, *d, S));  \
  } while (0)
    switch (mode) {
      case kGNone: BN_BWD_VEC(kGNone); break;
      case kGY: BN_BWD_VEC(kGY); break;
      case kGReLU: BN_BWD_VEC(kGReLU); break;
      default: BN_BWD_VEC(kGPre); break;
    }
#undef BN_BWD_VEC
    return hiseg_check_launch("bn_bwd");
  }
  if (!pre_red)
    DISPATCH_T(d->dtype, hipLaunchKernelGGL(bn_bwd_reduce_kernel<T>, dim3(S, (d->C + 255) / 256), dim3(256), 0, s, *d));
  hipLaunchKernelGGL(bn_bwd_finalize_par_kernel, fin_grid(C), dim3(256), 0, s, *d, S);
  DISPATCH_T(d->dtype, hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(ew_blocks(d->P * d->C)), dim3(256), 0, s, *d, S));
  return hiseg_check_launch("bn_bwd");
}

extern "C" int hiseg_dropout2d_mask_dev(int N, int C, float p, const unsigned long long* seed_base,
                                        unsigned long long offset, float* out, hiseg_stream_t stream) {
  HISEG_REQUIRE(seed_base && out && N > 0 && C > 0 && p >= 0.f && p < 1.f, HISEG_ERR_BAD_ARG, "dropout2d_mask_dev: bad args");
  const int n = N * C;
  hipLaunchKernelGGL(dropout2d_mask_dev_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, p,
                     seed_base, offset, out);
  return hiseg_check_launch("dropout2d_mask_dev");
}

extern "C" int hiseg_seed_advance(unsigned long long* seed_base, hiseg_stream_t stream) {
  HISEG_REQUIRE(seed_base, HISEG_ERR_BAD_ARG, "seed_advance: null");
  hipLaunchKernelGGL(seed_advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, seed_base);
  return hiseg_check_launch("seed_advance");
}

extern "C" int hiseg_dropout2d_mask(int N, int C, float p, unsigned long long seed, float* out, hiseg_stream_t stream) {
  HISEG_REQUIRE(out && N > 0 && C > 0 && p >= 0.f && p < 1.f, HISEG_ERR_BAD_ARG, "dropout2d_mask: bad arguments");
  const int n = N * C;
  hipLaunchKernelGGL(dropout2d_mask_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, p, seed, out);
  return hiseg_check_launch("dropout2d_mask");
}

extern "C" int hiseg_relu_bwd(int dtype, long long P, int HW, int C, hiseg_ew_view dy, hiseg_ew_view y,
                              const float* chan_mul, hiseg_ew_view dz, hiseg_stream_t stream) {
  HISEG_REQUIRE(dy.p && y.p && dz.p && P > 0 && C > 0 && HW > 0, HISEG_ERR_BAD_ARG, "relu_bwd: bad arguments");
  DISPATCH_T(dtype, hipLaunchKernelGGL(relu_bwd_kernel<T>, dim3(ew_blocks(P * C)), dim3(256), 0, (hipStream_t)stream,
                                       P, HW, C, dy, y, chan_mul, dz));
  return hiseg_check_launch("relu_bwd");
}

extern "C" int hiseg_sigmoid_bwd(int dtype, long long P, int C, hiseg_ew_view dy, hiseg_ew_view s, hiseg_ew_view dz,
                                 hiseg_stream_t stream) {
  HISEG_REQUIRE(dy.p && s.p && dz.p && P > 0 && C > 0, HISEG_ERR_BAD_ARG, "sigmoid_bwd: bad arguments");
  DISPATCH_T(dtype, hipLaunchKernelGGL(sigmoid_bwd_kernel<T>, dim3(ew_blocks(P * C)), dim3(256), 0,
                                       (hipStream_t)stream, P, C, dy, s, dz));
  return hiseg_check_launch("sigmoid_bwd");
}

extern "C" int hiseg_gate_fwd(int dtype, long long P, int C, hiseg_ew_view a, hiseg_ew_view g, hiseg_ew_view out,
                              hiseg_stream_t stream) {
  HISEG_REQUIRE(a.p && g.p && out.p && P > 0 && C > 0, HISEG_ERR_BAD_ARG, "gate_fwd: bad arguments");
  DISPATCH_T(dtype, hipLaunchKernelGGL(gate_fwd_kernel<T>, dim3(ew_blocks(P * C)), dim3(256), 0, (hipStream_t)stream,
                                       P, C, a, g, out));
  return hiseg_check_launch("gate_fwd");
}

extern "C" int hiseg_gate_bwd(int dtype, long long P, int C, hiseg_ew_view dy, hiseg_ew_view a, hiseg_ew_view g,
                              hiseg_ew_view da, int da_accumulate, hiseg_ew_view dzg, hiseg_stream_t stream) {
  HISEG_REQUIRE(dy.p && a.p && g.p && P > 0 && C > 0, HISEG_ERR_BAD_ARG, "gate_bwd: bad arguments");
  if (P < (1ll << 31) && vec_ok(dtype, C, dy.p, dy.cstride, dy.coff) && vec_ok(dtype, C, a.p, a.cstride, a.coff) &&
      vec_ok(dtype, C, g.p, g.cstride, g.coff) && vec_ok(dtype, C, da.p, da.cstride, da.coff) &&
      vec_ok(dtype, C, dzg.p, dzg.cstride, dzg.coff)) {
    DISPATCH_T(dtype, hipLaunchKernelGGL(gate_bwd_vec_kernel<T>, vec_grid(P, C, dtype), dim3(256), 0,
                                         (hipStream_t)stream, (int)P, C, dy, a, g, da, da_accumulate, dzg));
    return hiseg_check_launch("gate_bwd");
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(gate_bwd_kernel<T>, dim3(ew_blocks(P * C)), dim3(256), 0, (hipStream_t)stream,
                                       P, C, dy, a, g, da, da_accumulate, dzg));
  return hiseg_check_launch("gate_bwd");
}

extern "C" int hiseg_act_bwd_cvt(int dtype, long long P, int C, hiseg_ew_view dy, hiseg_ew_view y, int act,
                                 hiseg_ew_view dz, int accumulate, hiseg_stream_t stream) {
  HISEG_REQUIRE(dy.p && dz.p && P > 0 && C > 0 && (act == HISEG_ACT_NONE || y.p), HISEG_ERR_BAD_ARG,
                "act_bwd_cvt: bad arguments");
  DISPATCH_T(dtype, hipLaunchKernelGGL(act_bwd_cvt_kernel<T>, dim3(ew_blocks(P * C)), dim3(256), 0, (hipStream_t)stream,
                                       P, C, dy, y, act, dz, accumulate));
  return hiseg_check_launch("act_bwd_cvt");
}

extern "C" int hiseg_add_inplace(int dtype, long long P, int C, hiseg_ew_view dst, hiseg_ew_view src,
                                 hiseg_stream_t stream) {
  HISEG_REQUIRE(dst.p && src.p && P > 0 && C > 0, HISEG_ERR_BAD_ARG, "add_inplace: bad arguments");
  DISPATCH_T(dtype, hipLaunchKernelGGL(add_kernel<T>, dim3(ew_blocks(P * C)), dim3(256), 0, (hipStream_t)stream, P, C,
                                       dst, src));
  return hiseg_check_launch("add_inplace");
}

extern "C" int hiseg_maxpool2x2_bwd(int dtype, const void* x, int N, int H, int W, int C, const void* dy, void* dx,
                                    int accumulate, hiseg_stream_t stream) {
  HISEG_REQUIRE(x && dy && dx && N > 0 && H % 2 == 0 && W % 2 == 0 && C > 0, HISEG_ERR_BAD_ARG,
                "maxpool2x2_bwd: bad arguments");
  DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_bwd_kernel<T>, dim3(ew_blocks((long long)N * H * W * C / 4)), dim3(256),
                                       0, (hipStream_t)stream, x, N, H, W, C, dy, dx, accumulate));
  return hiseg_check_launch("maxpool2x2_bwd");
}

extern "C" int hiseg_upsample2x_bwd(int dtype, long long N, int h, int w, int C, hiseg_ew_view dy, hiseg_ew_view dx,
                                    int accumulate, hiseg_stream_t stream) {
  HISEG_REQUIRE(dy.p && dx.p && N > 0 && h > 0 && w > 0 && C > 0, HISEG_ERR_BAD_ARG, "upsample2x_bwd: bad arguments");
  HISEG_REQUIRE(vec_ok(dtype, C, dy.p, dy.cstride, dy.coff) && vec_ok(dtype, C, dx.p, dx.cstride, dx.coff),
                HISEG_ERR_BAD_SHAPE, "upsample2x_bwd: channels/strides must be whole 16-B chunks");
  const long long n = N * h * w * (C / (dtype == HISEG_BF16 ? 8 : 4));
  DISPATCH_T(dtype, hipLaunchKernelGGL(up2_bwd_kernel<T>, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, N, h, w,
                                       C, dy, dx, accumulate));
  return hiseg_check_launch("upsample2x_bwd");
}

extern "C" int hiseg_resize_bilinear_bwd(const float* dy, int NC, int h, int w, int H, int W, float* dx,
                                         hiseg_stream_t stream) {
  HISEG_REQUIRE(dy && dx && NC > 0 && h > 0 && w > 0 && H > 0 && W > 0, HISEG_ERR_BAD_ARG, "resize_bwd: bad arguments");
  hipLaunchKernelGGL(resize_bwd_kernel, dim3(ew_blocks((long long)NC * h * w)), dim3(256), 0, (hipStream_t)stream, dy,
                     NC, h, w, H, W, dx);
  return hiseg_check_launch("resize_bilinear_bwd");
}

// ---------------------------------------------------------------------------------------- LayerNorm2d host side
static int ln_splits(int N, int HW) {
  int sp = (2048 + N - 1) / N;
  const int cap = HW / 16 > 0 ? HW / 16 : 1;
  if (sp > cap) sp = cap;
  if (sp > 256) sp = 256;
  return sp < 1 ? 1 : sp;
}

extern "C" long long hiseg_ln_ws(int N, int HW, int C) {
  const long long sp = ln_splits(N, HW);
  const long long stats = (long long)N * sp * 4;                                  // doubles as float pairs
  const long long bwd = (long long)N * sp * 3 * C + (long long)N * 3 * C + 2LL * N;
  return stats > bwd ? stats : bwd;
}

extern "C" int hiseg_ln_fwd_stats(int dtype, const void* z, int N, int HW, int C, int cstride, int coff,
                                  const float* gamma, const float* beta, float eps, float* ws, float* mean,
                                  float* invstd, float* scale, float* shift, hiseg_stream_t stream) {
  HISEG_REQUIRE(z && ws && mean && invstd && scale && shift && N > 0 && HW > 0 && C > 0 && cstride >= coff + C,
                HISEG_ERR_BAD_ARG, "ln_fwd_stats: bad arguments");
  HISEG_REQUIRE(dtype == HISEG_F32 || dtype == HISEG_BF16, HISEG_ERR_BAD_DTYPE, "ln_fwd_stats: dtype");
  HISEG_REQUIRE(al16(ws), HISEG_ERR_BAD_ARG, "ln_fwd_stats: workspace must be 16-B aligned");
  hipStream_t s = (hipStream_t)stream;
  const int sp = ln_splits(N, HW);
  double* part = reinterpret_cast<double*>(ws);
  if (vec_ok(dtype, C, z, cstride, coff)) {
    DISPATCH_T(dtype, hipLaunchKernelGGL((ln_stats_kernel<T, Chunk<T>::N>), dim3(sp, N), dim3(256), 0, s, z, HW, C,
                                         cstride, coff, part));
  } else {
    DISPATCH_T(dtype, hipLaunchKernelGGL((ln_stats_kernel<T, 1>), dim3(sp, N), dim3(256), 0, s, z, HW, C, cstride, coff,
                                         part));
  }
  hipLaunchKernelGGL(ln_finalize_kernel, dim3(N), dim3(256), 0, s, part, sp, C, HW, gamma, beta, eps, mean, invstd,
                     scale, shift);
  return hiseg_check_launch("ln_fwd_stats");
}

extern "C" int hiseg_ln_bwd(const hiseg_ln_bwd_desc* d, hiseg_stream_t stream) {
  HISEG_REQUIRE(d && d->dy && d->z && d->dz && d->mean && d->invstd && d->scale && d->shift && d->ws && d->N > 0 &&
                    d->HW > 0 && d->C > 0,
                HISEG_ERR_BAD_ARG, "ln_bwd: bad arguments");
  HISEG_REQUIRE(d->dtype == HISEG_F32 || d->dtype == HISEG_BF16, HISEG_ERR_BAD_DTYPE, "ln_bwd: dtype");
  hipStream_t s = (hipStream_t)stream;
  const int sp = ln_splits(d->N, d->HW), dt = d->dtype, C = d->C;
  float* part = d->ws;
  float* nc = part + (long long)d->N * sp * 3 * C;
  float* coef = nc + (long long)d->N * 3 * C;
  const bool vec = vec_ok(dt, C, d->dy, d->dy_cstride, d->dy_coff) && vec_ok(dt, C, d->z, d->z_cstride, d->z_coff) &&
                   vec_ok(dt, C, d->dz, d->dz_cstride, d->dz_coff) &&
                   vec_ok(dt, C, d->dres, d->dres_cstride, d->dres_coff) &&
                   vec_ok(dt, C, d->residual, d->r_cstride, d->r_coff);
  long long bx = ((long long)d->N * d->HW + 7) / 8;
  if (bx > 4096) bx = 4096;
  if (vec) {
    DISPATCH_T(dt, hipLaunchKernelGGL((ln_bwd_reduce_kernel<T, Chunk<T>::N>), dim3(sp, d->N), dim3(256), 0, s, *d, part));
  } else {
    DISPATCH_T(dt, hipLaunchKernelGGL((ln_bwd_reduce_kernel<T, 1>), dim3(sp, d->N), dim3(256), 0, s, *d, part));
  }
  hipLaunchKernelGGL(ln_bwd_sample_kernel, dim3(d->N), dim3(256), 0, s, *d, part, sp, nc, coef);
  hipLaunchKernelGGL(ln_bwd_channel_kernel, dim3((C + 255) / 256), dim3(256), 0, s, *d, nc, coef);
  if (vec) {
    DISPATCH_T(dt, hipLaunchKernelGGL((ln_bwd_apply_kernel<T, Chunk<T>::N>), dim3((unsigned)bx), dim3(256), 0, s, *d,
                                      coef));
  } else {
    DISPATCH_T(dt, hipLaunchKernelGGL((ln_bwd_apply_kernel<T, 1>), dim3((unsigned)bx), dim3(256), 0, s, *d, coef));
  }
  return hiseg_check_launch("ln_bwd");
}

extern "C" int hiseg_act_bwd_pre(int dtype, long long P, int C, hiseg_ew_view dy, hiseg_ew_view z, int act,
                                 float act_beta, hiseg_ew_view dz, int accumulate, hiseg_stream_t stream) {
  HISEG_REQUIRE(dy.p && z.p && dz.p && P > 0 && C > 0, HISEG_ERR_BAD_ARG, "act_bwd_pre: bad arguments");
  DISPATCH_T(dtype, hipLaunchKernelGGL(act_bwd_pre_kernel<T>, dim3(ew_blocks(P * C)), dim3(256), 0, (hipStream_t)stream,
                                       P, C, dy, z, act, act_beta, dz, accumulate));
  return hiseg_check_launch("act_bwd_pre");
}
