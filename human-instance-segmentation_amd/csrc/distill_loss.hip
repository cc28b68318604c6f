// UNetDistillationLoss forward/backward (include/hiseg_distill.h) on gfx950.
//
// Three launches per forward: a per-(sample, split) partial reduction of the five per-pixel sums
// (binary KL, squared error, weighted BCE, and the Dice sums I = sum p y, P = sum p, Y = sum y),
// a one-block finalize that combines them in double precision into the loss values and the
// gradient coefficients (left in the workspace), and -- in the backward -- one element-wise pass
// that writes d total / d student.  Every stage is an HBM stream over the B x H x W logits; no host
// synchronisation (the reference reads each term back with .item()).
#include <math.h>

#include "common.h"
#include "hiseg_distill.h"

namespace hiseg {

constexpr int kDistSplits = 64;   // splits per sample
constexpr int kDistQ = 6;         // partial quantities
constexpr float kEps = 1e-5f;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// torch.clamp semantics: NaN stays NaN (fminf / fmaxf alone would return a bound)
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return x != x ? x : fminf(fmaxf(x, lo), hi); }

// A captured step's schedule values live on the device (hiseg_distill_cfg.dev_scalars).
__device__ __forceinline__ void load_dev_scalars(hiseg_distill_cfg& c) {
  if (c.dev_scalars) {
    c.temperature = c.dev_scalars[0];
    c.kl_weight = c.dev_scalars[1];
    c.task_weight = c.dev_scalars[2];
    c.pos_weight = c.dev_scalars[3];
  }
}

__global__ void __launch_bounds__(256) distill_partial_kernel(hiseg_distill_cfg c, long long HW, const float* s,
                                                              const float* te, const float* y, float* ws) {
  load_dev_scalars(c);
  __shared__ float red[kDistQ][256];
  const int b = blockIdx.y, sp = blockIdx.x, S = gridDim.x, t = threadIdx.x;
  const long long beg = HW * sp / S, end = HW * (sp + 1) / S;
  const float* sb = s + (long long)b * HW;
  const float* tb = te + (long long)b * HW;
  const float* yb = y ? y + (long long)b * HW : nullptr;
  const float invT = 1.f / c.temperature;
  float q[kDistQ] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (long long i = beg + t; i < end; i += 256) {
    const float x = sb[i];
    if (c.distill_terms) {
      const float tv = tb[i];
      const float ps = clampf(sigm(clampf(x, -10.f, 10.f) * invT), kEps, 1.f - kEps);
      const float pt = clampf(sigm(clampf(tv, -10.f, 10.f) * invT), kEps, 1.f - kEps);
      q[0] += pt * (logf(pt + kEps) - logf(ps + kEps)) + (1.f - pt) * (logf(1.f - pt + kEps) - logf(1.f - ps + kEps));
      const float d = x - tv;
      q[1] += d * d;
    }
    if (c.has_target) {
      const float yv = yb[i];
      q[2] += (1.f - yv) * x + (1.f + (c.pos_weight - 1.f) * yv) * (log1pf(expf(-fabsf(x))) + fmaxf(-x, 0.f));
      const float p = sigm(x);
      q[3] += p * yv;
      q[4] += p;
      q[5] += yv;
    }
  }
#pragma unroll
  for (int k = 0; k < kDistQ; ++k) red[k][t] = q[k];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
#pragma unroll
      for (int k = 0; k < kDistQ; ++k) red[k][t] += red[k][t + w];
    }
    __syncthreads();
  }
  if (t < kDistQ) ws[((long long)b * S + sp) * kDistQ + t] = red[t][0];
}

// Coefficient block (after the B*S*Q partials): [0] c_kl, [1] c_mse, [2] c_bce, [3] c_dice,
// then per sample u_b = 2 / D_b and v_b = N_b / D_b^2 (d coeff_b / d p = y u_b - v_b).
__global__ void distill_finalize_kernel(hiseg_distill_cfg c, int B, int S, long long HW, float* ws, float* out) {
  load_dev_scalars(c);
  __shared__ double per[256][3];
  const int t = threadIdx.x;
  double acc[3] = {0, 0, 0};
  if (t < B) {
    for (int sp = 0; sp < S; ++sp) {
      const float* p = ws + ((long long)t * S + sp) * kDistQ;
      acc[0] += p[3]; acc[1] += p[4]; acc[2] += p[5];
    }
  }
  per[t][0] = acc[0]; per[t][1] = acc[1]; per[t][2] = acc[2];
  __syncthreads();
  if (t != 0) return;
  double kl = 0, mse = 0, bce = 0;
  for (long long i = 0; i < (long long)B * S; ++i) {
    const float* p = ws + i * kDistQ;
    kl += p[0]; mse += p[1]; bce += p[2];
  }
  const double n = (double)B * (double)HW;
  kl /= n; mse /= n; bce /= n;
  // The reference's KL fallback (kl NaN/Inf -> 0.1 mean|pt - ps|, :560-564) is reachable only through a NaN
  // probability (the clamped probabilities keep every finite term bounded), where |pt - ps| is NaN as well: kl
  // stays NaN either way.  clamp(kl, 0, 5) keeps a NaN (:570).
  const bool kl_pass = kl >= 0.0 && kl <= 5.0;
  const double klc = kl != kl ? kl : (kl < 0.0 ? 0.0 : (kl > 5.0 ? 5.0 : kl));
  const double sm = 1e-5;
  double coeff = 0;
  float* cf = ws + (long long)B * S * kDistQ;
  for (int b = 0; b < B; ++b) {
    const double I = per[b][0], P = per[b][1], Y = per[b][2];
    const double Nb = 2.0 * I + sm, Db = P + Y + sm;
    coeff += Nb / Db;
    cf[4 + 2 * b] = (float)(2.0 / Db);
    cf[5 + 2 * b] = (float)(Nb / (Db * Db));
  }
  const double dice = 1.0 - coeff / B;
  const double kl_v = c.distill_terms ? klc : 0.0, mse_v = c.distill_terms ? mse : 0.0;
  const double task = c.use_dice ? 0.7 * bce + 0.3 * dice : bce;
  const double kw = c.kl_weight, tw = c.task_weight;
  const double dist = c.distill_in_total ? kw * kl_v + (1.0 - kw) * mse_v : 0.0;
  double total = c.has_target ? tw * task + (1.0 - tw) * dist : dist;
  // Final safety check (:650-659): a non-finite total falls back to the task loss (targets, task not NaN), else
  // to the MSE term (not NaN), else to a constant 1.0 that carries no gradient.
  int mode = 0;
  if (!isfinite(total)) {
    if (c.has_target && task == task) { mode = 1; total = task; }
    else if (mse_v == mse_v) { mode = 2; total = mse_v; }
    else { mode = 3; total = 1.0; }
  }
  auto nz = [](double v) { return v != v ? 0.f : (float)v; };   // loss_dict: NaN reported as 0.0
  out[HISEG_DISTILL_TOTAL] = (float)total;
  out[HISEG_DISTILL_KL] = nz(kl_v);
  out[HISEG_DISTILL_MSE] = nz(mse_v);
  out[HISEG_DISTILL_BCE] = c.has_target ? nz(bce) : 0.f;
  out[HISEG_DISTILL_DICE] = (c.has_target && c.use_dice) ? nz(dice) : 0.f;
  const double wd = c.has_target ? 1.0 - tw : 1.0;
  const bool dterms = c.distill_terms && c.distill_in_total;
  const double wt = mode == 1 ? 1.0 : tw;   // weight of the task terms in the differentiated total
  cf[0] = (mode == 0 && dterms && kl_pass) ? (float)(wd * kw / n) : 0.f;
  cf[1] = mode == 0 ? (dterms ? (float)(wd * (1.0 - kw) * 2.0 / n) : 0.f)
                    : ((mode == 2 && c.distill_terms) ? (float)(2.0 / n) : 0.f);
  cf[2] = (c.has_target && mode <= 1) ? (float)(wt * (c.use_dice ? 0.7 : 1.0) / n) : 0.f;
  cf[3] = (c.has_target && c.use_dice && mode <= 1) ? (float)(-wt * 0.3 / B) : 0.f;
}

__global__ void __launch_bounds__(256) distill_grad_kernel(hiseg_distill_cfg c, int B, int S, long long HW,
                                                           const float* s, const float* te, const float* y,
                                                           const float* ws, const float* gout, float* ds) {
  load_dev_scalars(c);
  const float* cf = ws + (long long)B * S * kDistQ;
  const float ckl = cf[0], cmse = cf[1], cbce = cf[2], cdice = cf[3];
  const float go = gout[0];
  const float invT = 1.f / c.temperature;
  const long long n = (long long)B * HW;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float x = s[i];
    float g = 0.f;
    if (ckl != 0.f || cmse != 0.f) {
      const float tv = te[i];
      if (ckl != 0.f && x >= -10.f && x <= 10.f) {
        const float sig = sigm(x * invT);
        if (sig >= kEps && sig <= 1.f - kEps) {
          const float pt = clampf(sigm(clampf(tv, -10.f, 10.f) * invT), kEps, 1.f - kEps);
          const float dterm = -pt / (sig + kEps) + (1.f - pt) / (1.f - sig + kEps);
          g += ckl * dterm * sig * (1.f - sig) * invT;
        }
      }
      g += cmse * (x - tv);
    }
    if (cbce != 0.f || cdice != 0.f) {
      const float yv = y[i];
      if (cbce != 0.f) g += cbce * ((1.f - yv) - (1.f + (c.pos_weight - 1.f) * yv) * sigm(-x));
      if (cdice != 0.f) {
        const int b = (int)(i / HW);
        const float p = sigm(x);
        g += cdice * (yv * cf[4 + 2 * b] - cf[5 + 2 * b]) * p * (1.f - p);
      }
    }
    ds[i] = g * go;
  }
}

static int dist_splits(long long HW) {
  long long s = (HW + 1023) / 1024;
  return (int)(s < 1 ? 1 : (s > kDistSplits ? kDistSplits : s));
}

}  // namespace hiseg

using namespace hiseg;

extern "C" long long hiseg_distill_ws(int B, int H, int W) {
  return (long long)B * kDistSplits * kDistQ + 4 + 2 * (long long)B;
}

extern "C" int hiseg_distill_loss_fwd(const hiseg_distill_cfg* cfg, int B, int H, int W, const float* student,
                                      const float* teacher, const float* target, float* ws, float* out,
                                      hiseg_stream_t stream) {
  HISEG_REQUIRE(cfg && student && teacher && ws && out && B > 0 && H > 0 && W > 0, HISEG_ERR_BAD_ARG,
                "distill_loss_fwd: bad arguments");
  HISEG_REQUIRE(B <= 256, HISEG_ERR_BAD_SHAPE, "distill_loss_fwd: at most 256 samples per call");
  HISEG_REQUIRE(!cfg->has_target || target, HISEG_ERR_BAD_ARG, "distill_loss_fwd: has_target needs target");
  HISEG_REQUIRE(cfg->temperature > 0.f, HISEG_ERR_BAD_ARG, "distill_loss_fwd: temperature must be > 0");
  const long long HW = (long long)H * W;
  const int S = dist_splits(HW);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(distill_partial_kernel, dim3(S, B), dim3(256), 0, s, *cfg, HW, student, teacher,
                     cfg->has_target ? target : nullptr, ws);
  hipLaunchKernelGGL(distill_finalize_kernel, dim3(1), dim3(256), 0, s, *cfg, B, S, HW, ws, out);
  return hiseg_check_launch("distill_loss_fwd");
}

extern "C" int hiseg_distill_loss_bwd(const hiseg_distill_cfg* cfg, int B, int H, int W, const float* student,
                                      const float* teacher, const float* target, const float* ws,
                                      const float* grad_out, float* dstudent, hiseg_stream_t stream) {
  HISEG_REQUIRE(cfg && student && teacher && ws && grad_out && dstudent && B > 0 && H > 0 && W > 0,
                HISEG_ERR_BAD_ARG, "distill_loss_bwd: bad arguments");
  HISEG_REQUIRE(!cfg->has_target || target, HISEG_ERR_BAD_ARG, "distill_loss_bwd: has_target needs target");
  const long long HW = (long long)H * W;
  const long long n = (long long)B * HW;
  long long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(distill_grad_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, *cfg, B,
                     dist_splits(HW), HW, student, teacher, cfg->has_target ? target : nullptr, ws, grad_out,
                     dstudent);
  return hiseg_check_launch("distill_loss_bwd");
}
