// RefinedHierarchicalLoss forward / backward on gfx950 (see include/hiseg_loss.h).
//
// Pass structure (all per mask pixel, f32 math, deterministic partial sums):
//   targets : boundary weight (3x3 window holds >= 2 labels, refinement.py:389-431), raw contour
//             target (max(|dy|,|dx|) of the class-1 mask with replicate padding, :1002-1015), class
//             counts -> [targets2] dilated contour target (box count of the raw contour > 0.1, :1018-1038)
//             -> 5 x distance iteration d += (1-d)*maxpool3(d)*0.5 (:1058-1066)
//   weights : one thread: dynamic class weights, clamps, EMA in double (hierarchical_segmentation.py
//             :227-255,286-309), kept in the device state
//   main    : per ROI x split partial sums of every loss term, dice statistics and metrics
//   finalize: loss values, clamps (refinement.py:936,948,980), loss-dict outputs, backward coefficients
//   bwd     : per pixel gradients w.r.t. all five inputs
#include "common.h"
#include "hiseg_loss.h"

namespace hiseg {

constexpr int kSpl = 16;      // pixel splits per ROI in the main pass
constexpr int kNS = 14;       // sums per partial
constexpr int kG = 18;        // loss_finalize_kernel's row groups (kG * kNS <= 256)
constexpr int kCntBlocks = 256;
constexpr int kCoef = 32;     // global coefficient slots

struct LossWS {
  float *bw, *ct, *craw, *dA, *dB, *cnt, *part, *coef, *dice;  // dice: [N][2]
};

__host__ __device__ inline LossWS loss_ws(float* ws, int N, long long NP) {
  LossWS w;
  w.bw = ws; w.ct = ws + NP; w.craw = ws + 2 * NP; w.dA = ws + 3 * NP; w.dB = ws + 4 * NP;
  w.cnt = ws + 5 * NP;
  w.part = w.cnt + kCntBlocks * 4;
  w.coef = w.part + (long long)N * kSpl * kNS;
  w.dice = w.coef + kCoef;
  return w;
}

// coef slots
enum { C_WBF0 = 0, C_WBF1, C_WTN0, C_WTN1, C_TNACT, C_KBF, C_KTN, C_KF, C_KBA, C_KCONS, C_KDICE, C_KCT, C_KD, C_FGCNT };

__global__ void __launch_bounds__(256) loss_targets_kernel(const long long* tg, int N, int H, int W, float* bw,
                                                           float* craw, float* dA, float* cnt) {
  __shared__ float red[4][256];
  const long long NP = (long long)N * H * W;
  float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
  for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < NP; p += (long long)gridDim.x * 256) {
    const int x = (int)(p % W);
    const long long t = p / W;
    const int y = (int)(t % H);
    const long long n = t / H;
    const long long* img = tg + n * H * W;
    const long long v = img[(long long)y * W + x];
    // boundary: >= 2 distinct labels in the clipped 3x3 window
    bool bnd = false;
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int yy = y + dy, xx = x + dx;
        if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
        if (img[(long long)yy * W + xx] != v) bnd = true;
      }
    bw[p] = bnd ? 2.f : 1.f;
    // raw contour of class 1: dy/dx differences, replicate padding at the last row / column
    const float t1 = v == 1 ? 1.f : 0.f;
    const int yy = y < H - 1 ? y : y - 1, xx = x < W - 1 ? x : x - 1;
    float gy = 0.f, gx = 0.f;
    if (H > 1) {
      const float a = img[(long long)yy * W + x] == 1 ? 1.f : 0.f, b = img[(long long)(yy + 1) * W + x] == 1 ? 1.f : 0.f;
      gy = fabsf(b - a);
    }
    if (W > 1) {
      const float a = img[(long long)y * W + xx] == 1 ? 1.f : 0.f, b = img[(long long)y * W + xx + 1] == 1 ? 1.f : 0.f;
      gx = fabsf(b - a);
    }
    craw[p] = fmaxf(gy, gx);
    dA[p] = t1;
    c0 += v == 0 ? 1.f : 0.f;
    c1 += v > 0 ? 1.f : 0.f;
    c2 += v == 1 ? 1.f : 0.f;
    c3 += v == 2 ? 1.f : 0.f;
  }
  const int t = threadIdx.x;
  red[0][t] = c0; red[1][t] = c1; red[2][t] = c2; red[3][t] = c3;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s)
      for (int k = 0; k < 4; ++k) red[k][t] += red[k][t + s];
    __syncthreads();
  }
  if (t < 4) cnt[blockIdx.x * 4 + t] = red[t][0];
}

// dilated contour target: (sum of raw contour over ks x ks window, zero padded) / ks^2 > 0.1
__global__ void __launch_bounds__(256) loss_contour_kernel(const float* craw, int N, int H, int W, int ks, float* ct) {
  const long long NP = (long long)N * H * W;
  const float w = 1.f / (float)(ks * ks);
  for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < NP; p += (long long)gridDim.x * 256) {
    if (ks <= 1) { ct[p] = craw[p]; continue; }
    const int x = (int)(p % W);
    const long long t = p / W;
    const int y = (int)(t % H);
    const long long n = t / H;
    const int r = ks / 2;
    float s = 0.f;
    for (int dy = -r; dy <= r; ++dy) {
      const int yy = y + dy;
      if (yy < 0 || yy >= H) continue;
      for (int dx = -r; dx <= r; ++dx) {
        const int xx = x + dx;
        if (xx < 0 || xx >= W) continue;
        s += craw[(n * H + yy) * W + xx] * w;
      }
    }
    ct[p] = s > 0.1f ? 1.f : 0.f;
  }
}

// one distance iteration: out = d + (1 - d) * maxpool3(d) * 0.5
__global__ void __launch_bounds__(256) loss_dist_kernel(const float* d, int N, int H, int W, float* out) {
  const long long NP = (long long)N * H * W;
  for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < NP; p += (long long)gridDim.x * 256) {
    const int x = (int)(p % W);
    const long long t = p / W;
    const int y = (int)(t % H);
    const long long n = t / H;
    float m = -INFINITY;
    for (int dy = -1; dy <= 1; ++dy) {
      const int yy = y + dy;
      if (yy < 0 || yy >= H) continue;
      for (int dx = -1; dx <= 1; ++dx) {
        const int xx = x + dx;
        if (xx < 0 || xx >= W) continue;
        m = fmaxf(m, d[(n * H + yy) * W + xx]);
      }
    }
    const float v = d[p];
    out[p] = v + (1.f - v) * m * 0.5f;
  }
}

__device__ __forceinline__ double clampd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }

// the 4 class pixel counts (bg, fg, target, non-target) of this batch -> counts[4]
__global__ void loss_counts_kernel(const float* cnt, int nblk, double* counts) {
  if (threadIdx.x != 0) return;
  double c[4] = {0, 0, 0, 0};
  for (int b = 0; b < nblk; ++b)
    for (int k = 0; k < 4; ++k) c[k] += cnt[b * 4 + k];
  for (int k = 0; k < 4; ++k) counts[k] = c[k];
}

// class weights + EMA update from counts (this batch's, or their all-reduced sum over data-parallel ranks);
// local_fg = this batch's foreground count (the loss terms' own normalisation)
__global__ void loss_weights_kernel(hiseg_loss_cfg cfg, const double* counts, const double* local, double* st,
                                    float* coef) {
  if (threadIdx.x != 0) return;
  const double bg = counts[0], fg = counts[1], tc = counts[2], nt = counts[3];
  const double fg_local = local[1];
  float wb0, wb1;
  if (cfg.use_dynamic_weights) {
    const double tot = bg + fg;
    const float bw = (float)clampd((float)(tot / (2.0 * (bg > 1 ? bg : 1))), 0.5, 3.0);
    const float fw = (float)clampd((float)((float)(tot / (2.0 * (fg > 1 ? fg : 1))) * cfg.target_weight), 0.5, 3.0);
    st[0] = 0.9 * st[0] + 0.1 * (double)bw;
    st[1] = 0.9 * st[1] + 0.1 * (double)fw;
    wb0 = (float)st[0]; wb1 = (float)st[1];
  } else {
    wb0 = 1.f; wb1 = cfg.target_weight;
  }
  coef[C_WBF0] = wb0; coef[C_WBF1] = wb1;
  float active = 0.f, wt0 = 1.f, wt1 = 1.f;
  if (fg > 0 && tc + nt > 0) {
    active = 1.f;
    if (cfg.use_dynamic_weights) {
      const double ftot = tc + nt;
      const float tw = (float)clampd((float)(ftot / (2.0 * (tc > 1 ? tc : 1))), 0.5, 3.0);
      const float ntw = (float)clampd((float)(ftot / (2.0 * (nt > 1 ? nt : 1))), 0.5, 3.0);
      if (st[4] == 0.0) { st[2] = tw; st[3] = ntw; st[4] = 1.0; }
      else { st[2] = 0.9 * st[2] + 0.1 * (double)tw; st[3] = 0.9 * st[3] + 0.1 * (double)ntw; }
      st[5] = st[2]; st[6] = st[3];
      wt0 = (float)st[2]; wt1 = (float)st[3];
    } else {
      st[5] = 1.0; st[6] = 1.0;
    }
  }
  coef[C_WTN0] = wt0; coef[C_WTN1] = wt1; coef[C_TNACT] = active;
  coef[C_FGCNT] = (float)fg_local;
  st[7] += 1.0;
}

__device__ __forceinline__ void softmax3(const float* v, float* p) {
  const float m = fmaxf(v[0], fmaxf(v[1], v[2]));
  const float e0 = __expf(v[0] - m), e1 = __expf(v[1] - m), e2 = __expf(v[2] - m);
  const float s = e0 + e1 + e2;
  p[0] = e0 / s; p[1] = e1 / s; p[2] = e2 / s;
}

__device__ __forceinline__ float lse2(float a, float b) { const float m = fmaxf(a, b); return m + logf(__expf(a - m) + __expf(b - m)); }
__device__ __forceinline__ float lse3(float a, float b, float c) {
  const float m = fmaxf(a, fmaxf(b, c));
  return m + logf(__expf(a - m) + __expf(b - m) + __expf(c - m));
}

// grid (kSpl, N): partial sums [n][split][kNS]
__global__ void __launch_bounds__(256) loss_main_kernel(hiseg_loss_cfg cfg, int N, int H, int W, const float* pred,
                                                        const float* bgfg, const float* tn, const float* cont,
                                                        const float* dist, const long long* tg, LossWS w) {
  __shared__ float red[kNS][256];
  const int n = blockIdx.y;
  const long long plane = (long long)H * W;
  const long long b = plane * blockIdx.x / kSpl, e = plane * (blockIdx.x + 1) / kSpl;
  const float wb0 = w.coef[C_WBF0], wb1 = w.coef[C_WBF1], wt0 = w.coef[C_WTN0], wt1 = w.coef[C_WTN1];
  const bool tn_on = w.coef[C_TNACT] > 0.f;
  float s[kNS];
#pragma unroll
  for (int k = 0; k < kNS; ++k) s[k] = 0.f;
  for (long long q = b + threadIdx.x; q < e; q += 256) {
    const long long p = n * plane + q;
    const int y = (int)tg[p];
    const float* P = pred + n * 3 * plane + q;
    const float* G = bgfg + n * 2 * plane + q;
    const float v[3] = {P[0], P[plane], P[2 * plane]};
    const float g0 = G[0], g1 = G[plane];
    const int fg = y > 0 ? 1 : 0;
    const float nll_bf = lse2(g0, g1) - (fg ? g1 : g0);
    const float wy = fg ? wb1 : wb0;
    s[0] += wy * nll_bf;
    s[1] += wy;
    if (tn_on && fg) {
      const float* T = tn + n * 2 * plane + q;
      const int yt = y == 2 ? 1 : 0;
      s[2] += (yt ? wt1 : wt0) * (lse2(T[0], T[plane]) - (yt ? T[plane] : T[0]));
    }
    const float nll_f = lse3(v[0], v[1], v[2]) - v[y];
    s[3] += nll_f;
    float pf[3];
    softmax3(v, pf);
    const float pb1 = 1.f / (1.f + __expf(g0 - g1));
    const float dcon = pb1 - (pf[1] + pf[2]);
    s[4] += dcon * dcon;
    const float t1 = y == 1 ? 1.f : 0.f;
    s[5] += pf[1] * t1;
    s[6] += pf[1];
    s[7] += t1;
    if (cfg.use_boundary_aware) s[8] += nll_f * w.bw[p];
    if (cfg.use_contour && cont) {
      const float x = cont[p], t = w.ct[p];
      s[9] += fmaxf(x, 0.f) - x * t + log1pf(__expf(-fabsf(x)));
    }
    if (cfg.use_distance && dist) s[10] += fabsf(dist[p] - w.dB[p]);
    const int pr = g1 > g0 ? 1 : 0;
    s[11] += pr == fg ? 1.f : 0.f;
    s[12] += (pr == 1 && fg) ? 1.f : 0.f;
    s[13] += (pr == 1 || fg) ? 1.f : 0.f;
  }
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < kNS; ++k) red[k][t] = s[k];
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (t < st)
      for (int k = 0; k < kNS; ++k) red[k][t] += red[k][t + st];
    __syncthreads();
  }
  if (t < kNS) w.part[((long long)n * kSpl + blockIdx.x) * kNS + t] = red[t][0];
}

__global__ void __launch_bounds__(256) loss_finalize_kernel(hiseg_loss_cfg cfg, int N, int H, int W, LossWS w,
                                                            const double* st, float* out) {
  __shared__ double tot[kNS];
  __shared__ double gsum[kG * kNS];
  __shared__ double dsum;
  const int t = threadIdx.x;
  // the N x kSpl partial rows summed by kG groups of kNS threads (row i to group i % kG, four accumulators each),
  // then the groups in order: one thread per sum walked all N x 16 rows, a dependent chain of double adds at load
  // latency (0.52 ms of the B0 train step at 256 ROIs)
  if (t < kG * kNS) {
    const int g = t / kNS, k = t % kNS, rows = N * kSpl;
    double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    int i = g;
    for (; i + 3 * kG < rows; i += 4 * kG) {
      a0 += w.part[(long long)i * kNS + k];
      a1 += w.part[(long long)(i + kG) * kNS + k];
      a2 += w.part[(long long)(i + 2 * kG) * kNS + k];
      a3 += w.part[(long long)(i + 3 * kG) * kNS + k];
    }
    for (; i < rows; i += kG) a0 += w.part[(long long)i * kNS + k];
    gsum[t] = (a0 + a1) + (a2 + a3);
  }
  if (t == 0) dsum = 0;
  __syncthreads();
  if (t < kNS) {
    double s = 0;
    for (int g = 0; g < kG; ++g) s += gsum[g * kNS + t];
    tot[t] = s;
  }
  __syncthreads();
  // per-ROI dice (thread per ROI, strided)
  double my = 0;
  for (int n = t; n < N; n += 256) {
    double I = 0, Ps = 0, Ts = 0;
    for (int k = 0; k < kSpl; ++k) {
      const float* pp = w.part + ((long long)n * kSpl + k) * kNS;
      I += pp[5]; Ps += pp[6]; Ts += pp[7];
    }
    const double sm = 1e-6, D = Ps + Ts + sm;
    my += 1.0 - (2 * I + sm) / D;
    w.dice[n * 2] = (float)(-2.0 / D);
    w.dice[n * 2 + 1] = (float)((2 * I + sm) / (D * D));
  }
  atomicAdd(&dsum, my);  // one double atomic per thread on LDS (order-independent up to rounding of <= 256 terms)
  __syncthreads();
  if (t != 0) return;
  const double P = (double)N * H * W;
  const double fgc = w.coef[C_FGCNT];
  const double bf = tot[0] / tot[1];
  const bool tn_on = w.coef[C_TNACT] > 0.f;
  const double tnl = tn_on ? tot[2] / (fgc > 1 ? fgc : 1) : 0.0;
  const double fin = tot[3] / P, cons = tot[4] / P, dice = dsum / N;
  double total = cfg.bg_weight * bf + cfg.fg_weight * tnl + cfg.ce_weight * fin + cfg.dice_weight * dice +
                 cfg.consistency_weight * cons;
  out[HISEG_LOSS_NOUT] = (float)total;  // the base HierarchicalLoss total (loss_dict['total_loss'])
  double ba = 0, ct = 0, dl = 0;
  float mba = 0.f, mct = 0.f, md = 0.f;
  if (cfg.use_boundary_aware) { ba = tot[8] / P; mba = ba <= 10.0 ? 1.f : 0.f; ba = ba < 10.0 ? ba : 10.0; total += cfg.boundary_aware_weight * ba; }
  if (cfg.use_contour) { ct = tot[9] / P; mct = ct <= 10.0 ? 1.f : 0.f; ct = ct < 10.0 ? ct : 10.0; total += cfg.contour_weight * ct; }
  if (cfg.use_distance) { dl = tot[10] / P; md = dl <= 10.0 ? 1.f : 0.f; dl = dl < 10.0 ? dl : 10.0; total += cfg.distance_weight * dl; }
  out[HISEG_LOSS_TOTAL] = (float)total;
  out[HISEG_LOSS_BGFG] = (float)bf;
  out[HISEG_LOSS_TN] = (float)tnl;
  out[HISEG_LOSS_FINAL] = (float)fin;
  out[HISEG_LOSS_CONS] = (float)cons;
  out[HISEG_LOSS_DICE] = (float)dice;
  out[HISEG_LOSS_BA] = (float)ba;
  out[HISEG_LOSS_CONTOUR] = (float)ct;
  out[HISEG_LOSS_DIST] = (float)dl;
  out[HISEG_LOSS_ACC] = (float)(tot[11] / P);
  out[HISEG_LOSS_IOU] = (float)(tot[12] / (tot[13] > 1 ? tot[13] : 1));
  out[HISEG_LOSS_W_BG] = cfg.use_dynamic_weights ? (float)st[0] : 1.f;
  out[HISEG_LOSS_W_FG] = cfg.use_dynamic_weights ? (float)st[1] : cfg.target_weight;
  out[HISEG_LOSS_W_T] = (float)st[5];
  out[HISEG_LOSS_W_NT] = (float)st[6];
  float* c = w.coef;
  c[C_KBF] = (float)(cfg.bg_weight / tot[1]);
  c[C_KTN] = tn_on ? (float)(cfg.fg_weight / (fgc > 1 ? fgc : 1)) : 0.f;
  c[C_KF] = (float)(cfg.ce_weight / P);
  c[C_KBA] = (float)(cfg.boundary_aware_weight * mba / P);
  c[C_KCONS] = (float)(2.0 * cfg.consistency_weight / P);
  c[C_KDICE] = (float)(cfg.dice_weight / N);
  c[C_KCT] = (float)(cfg.contour_weight * mct / P);
  c[C_KD] = (float)(cfg.distance_weight * md / P);
}

__global__ void __launch_bounds__(256) loss_bwd_kernel(hiseg_loss_cfg cfg, int N, int H, int W, const float* pred,
                                                       const float* bgfg, const float* tn, const float* cont,
                                                       const float* dist, const long long* tg, LossWS w,
                                                       const float* gout, float* dpred, float* dbgfg, float* dtn,
                                                       float* dcont, float* ddist) {
  const long long plane = (long long)H * W, NP = (long long)N * plane;
  const float* c = w.coef;
  const float go = gout ? gout[0] : 1.f;
  for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < NP; p += (long long)gridDim.x * 256) {
    const long long n = p / plane, q = p - n * plane;
    const int y = (int)tg[p];
    const int fg = y > 0 ? 1 : 0;
    const float* P = pred + n * 3 * plane + q;
    const float* G = bgfg + n * 2 * plane + q;
    const float v[3] = {P[0], P[plane], P[2 * plane]};
    const float g0 = G[0], g1 = G[plane];
    float pf[3];
    softmax3(v, pf);
    const float pb1 = 1.f / (1.f + __expf(g0 - g1)), pb0 = 1.f - pb1;
    const float dcon = pb1 - (pf[1] + pf[2]);
    const float kcons = c[C_KCONS] * dcon;  // dL/dpb1 ; dL/ds = -kcons
    if (dbgfg) {
      const float wy = fg ? c[C_WBF1] : c[C_WBF0];
      const float kb = c[C_KBF] * wy;
      float d0 = kb * (pb0 - (fg ? 0.f : 1.f));
      float d1 = kb * (pb1 - (fg ? 1.f : 0.f));
      const float j = kcons * pb1 * pb0;
      d0 -= j; d1 += j;
      dbgfg[n * 2 * plane + q] = go * d0;
      dbgfg[n * 2 * plane + plane + q] = go * d1;
    }
    if (dtn) {
      float d0 = 0.f, d1 = 0.f;
      if (fg && c[C_TNACT] > 0.f) {
        const float* T = tn + n * 2 * plane + q;
        const int yt = y == 2 ? 1 : 0;
        const float p1 = 1.f / (1.f + __expf(T[0] - T[plane])), p0 = 1.f - p1;
        const float k = c[C_KTN] * (yt ? c[C_WTN1] : c[C_WTN0]);
        d0 = k * (p0 - (yt ? 0.f : 1.f));
        d1 = k * (p1 - (yt ? 1.f : 0.f));
      }
      dtn[n * 2 * plane + q] = go * d0;
      dtn[n * 2 * plane + plane + q] = go * d1;
    }
    if (dpred) {
      const float kf = c[C_KF] + (cfg.use_boundary_aware ? c[C_KBA] * w.bw[p] : 0.f);
      float d[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) d[j] = kf * (pf[j] - (j == y ? 1.f : 0.f));
      // consistency: s = 1 - pf0, dL/ds = -kcons; ds/dv_j = -pf0 (delta_0j - pf_j)
      const float ks = -kcons;
      d[0] += ks * (-pf[0] * (1.f - pf[0]));
      d[1] += ks * (pf[0] * pf[1]);
      d[2] += ks * (pf[0] * pf[2]);
      // dice: dL/dpf1 = kdice * (A_n * t1 + B_n)
      const float t1 = y == 1 ? 1.f : 0.f;
      const float kd = c[C_KDICE] * (w.dice[n * 2] * t1 + w.dice[n * 2 + 1]);
#pragma unroll
      for (int j = 0; j < 3; ++j) d[j] += kd * pf[1] * ((j == 1 ? 1.f : 0.f) - pf[j]);
      dpred[n * 3 * plane + q] = go * d[0];
      dpred[n * 3 * plane + plane + q] = go * d[1];
      dpred[n * 3 * plane + 2 * plane + q] = go * d[2];
    }
    if (dcont) {
      float d = 0.f;
      if (cfg.use_contour && cont) {
        const float x = cont[p];
        d = c[C_KCT] * (1.f / (1.f + __expf(-x)) - w.ct[p]);
      }
      dcont[p] = go * d;
    }
    if (ddist) {
      float d = 0.f;
      if (cfg.use_distance && dist) {
        const float r = dist[p] - w.dB[p];
        d = c[C_KD] * (r > 0.f ? 1.f : (r < 0.f ? -1.f : 0.f));
      }
      ddist[p] = go * d;
    }
  }
}

__global__ void loss_state_init_kernel(double* st) {
  if (threadIdx.x == 0) {
    st[0] = 1.0; st[1] = 1.0; st[2] = 1.0; st[3] = 1.0; st[4] = 0.0; st[5] = 1.0; st[6] = 1.0; st[7] = 0.0;
  }
}

inline unsigned gblocks(long long n) {
  long long b = (n + 255) / 256;
  return (unsigned)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

}  // namespace hiseg

using namespace hiseg;

extern "C" int hiseg_loss_state_init(double* state, hiseg_stream_t stream) {
  HISEG_REQUIRE(state, HISEG_ERR_BAD_ARG, "loss_state_init: null");
  hipLaunchKernelGGL(loss_state_init_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, state);
  return hiseg_check_launch("loss_state_init");
}

extern "C" long long hiseg_loss_ws(int N, int H, int W) {
  const long long NP = (long long)N * H * W;
  return 5 * NP + kCntBlocks * 4 + (long long)N * kSpl * kNS + kCoef + 2LL * N + 10;   // + local counts (double[4])
}

static double* local_counts(float* ws, int N, int H, int W) {   // after the partials, 8-B aligned (ws is)
  const long long n = hiseg_loss_ws(N, H, W) - 10;
  return reinterpret_cast<double*>(ws + ((n + 1) & ~1LL));
}

extern "C" int hiseg_loss_fwd(const hiseg_loss_cfg* cfg, int N, int H, int W, const float* pred, const float* bgfg,
                              const float* tn, const float* cont, const float* dist, const long long* targets,
                              double* state, float* ws, float* out, hiseg_stream_t stream) {
  HISEG_REQUIRE(cfg && pred && bgfg && tn && targets && state && ws && out && N > 0 && H > 0 && W > 0,
                HISEG_ERR_BAD_ARG, "loss_fwd: bad arguments");
  HISEG_REQUIRE(!cfg->use_contour || cont, HISEG_ERR_BAD_ARG, "loss_fwd: contour term needs cont");
  HISEG_REQUIRE(!cfg->use_distance || dist, HISEG_ERR_BAD_ARG, "loss_fwd: distance term needs dist");
  int r = hiseg_loss_fwd_begin(cfg, N, H, W, targets, ws, nullptr, stream);
  if (r) return r;
  return hiseg_loss_fwd_end(cfg, N, H, W, pred, bgfg, tn, cont, dist, targets, nullptr, state, ws, out, stream);
}

extern "C" int hiseg_loss_fwd_begin(const hiseg_loss_cfg* cfg, int N, int H, int W, const long long* targets, float* ws,
                                    double* counts, hiseg_stream_t stream) {
  HISEG_REQUIRE(cfg && targets && ws && N > 0 && H > 0 && W > 0, HISEG_ERR_BAD_ARG, "loss_fwd_begin: bad arguments");
  HISEG_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 7) == 0, HISEG_ERR_BAD_ARG, "loss_fwd_begin: ws alignment");
  hipStream_t s = (hipStream_t)stream;
  const long long NP = (long long)N * H * W;
  LossWS w = loss_ws(ws, N, NP);
  double* lc = local_counts(ws, N, H, W);
  hipLaunchKernelGGL(loss_targets_kernel, dim3(kCntBlocks), dim3(256), 0, s, targets, N, H, W, w.bw, w.craw, w.dA, w.cnt);
  hipLaunchKernelGGL(loss_counts_kernel, dim3(1), dim3(64), 0, s, w.cnt, kCntBlocks, lc);
  if (counts) (void)hipMemcpyAsync(counts, lc, 4 * sizeof(double), hipMemcpyDeviceToDevice, s);
  if (cfg->use_contour)
    hipLaunchKernelGGL(loss_contour_kernel, dim3(gblocks(NP)), dim3(256), 0, s, w.craw, N, H, W, cfg->contour_ks, w.ct);
  if (cfg->use_distance) {
    for (int it = 0; it < 5; ++it) {  // dA -> dB -> dA -> dB -> dA -> dB: the target ends in dB
      float* src = (it & 1) ? w.dB : w.dA;
      float* dst = (it & 1) ? w.dA : w.dB;
      hipLaunchKernelGGL(loss_dist_kernel, dim3(gblocks(NP)), dim3(256), 0, s, src, N, H, W, dst);
    }
  }
  return hiseg_check_launch("loss_fwd_begin");
}

extern "C" int hiseg_loss_fwd_end(const hiseg_loss_cfg* cfg, int N, int H, int W, const float* pred, const float* bgfg,
                                  const float* tn, const float* cont, const float* dist, const long long* targets,
                                  const double* counts, double* state, float* ws, float* out, hiseg_stream_t stream) {
  HISEG_REQUIRE(cfg && pred && bgfg && tn && targets && state && ws && out && N > 0 && H > 0 && W > 0,
                HISEG_ERR_BAD_ARG, "loss_fwd_end: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  const long long NP = (long long)N * H * W;
  LossWS w = loss_ws(ws, N, NP);
  const double* lc = local_counts(ws, N, H, W);
  hipLaunchKernelGGL(loss_weights_kernel, dim3(1), dim3(64), 0, s, *cfg, counts ? counts : lc, lc, state, w.coef);
  hipLaunchKernelGGL(loss_main_kernel, dim3(kSpl, N), dim3(256), 0, s, *cfg, N, H, W, pred, bgfg, tn, cont, dist,
                     targets, w);
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, s, *cfg, N, H, W, w, state, out);
  return hiseg_check_launch("loss_fwd");
}

extern "C" int hiseg_loss_bwd(const hiseg_loss_cfg* cfg, int N, int H, int W, const float* pred, const float* bgfg,
                              const float* tn, const float* cont, const float* dist, const long long* targets,
                              const float* ws, const float* grad_out, float* dpred, float* dbgfg, float* dtn,
                              float* dcont, float* ddist, hiseg_stream_t stream) {
  HISEG_REQUIRE(cfg && pred && bgfg && tn && targets && ws && N > 0 && H > 0 && W > 0, HISEG_ERR_BAD_ARG,
                "loss_bwd: bad arguments");
  const long long NP = (long long)N * H * W;
  LossWS w = loss_ws(const_cast<float*>(ws), N, NP);
  hipLaunchKernelGGL(loss_bwd_kernel, dim3(gblocks(NP)), dim3(256), 0, (hipStream_t)stream, *cfg, N, H, W, pred, bgfg,
                     tn, cont, dist, targets, w, grad_out, dpred, dbgfg, dtn, dcont, ddist);
  return hiseg_check_launch("loss_bwd");
}
