// Flat-parameter-space optimiser step (gfx950): gradient norm partials, clip_grad_norm_ scaling
// and the AdamW update in one streaming pass (include/hiseg_train.h).  HBM-bound: reads p, g, m,
// v and writes p, g, m, v once (28 B per parameter).
#include "common.h"
#include "hiseg_train.h"

namespace hiseg {

constexpr int kOptBlocks = 1024;

__global__ void __launch_bounds__(256) grad_norm_kernel(const float* g, long long n, float* partial) {
  __shared__ float red[256];
  float s = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) s += g[i] * g[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) adamw_kernel(float* p, float* g, float* m, float* v, long long n, float lr,
                                                    float b1, float b2, float eps, float wd, float bc1, float bc2,
                                                    const float* partial, float max_norm, float* norm_out) {
  __shared__ float coef;
  if (threadIdx.x == 0) {
    float c = 1.f;
    if (partial) {
      double s = 0;
      for (int b = 0; b < kOptBlocks; ++b) s += partial[b];
      const float total = (float)sqrt(s);
      if (norm_out && blockIdx.x == 0) norm_out[0] = total;
      if (max_norm > 0.f) {
        const float cc = max_norm / (total + 1e-6f);
        c = cc < 1.f ? cc : 1.f;
      }
    }
    coef = c;
  }
  __syncthreads();
  const float c = coef;
  const float step = lr / bc1;
  const float sbc2 = sqrtf(bc2);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float gi = g[i];
    if (partial && max_norm > 0.f) { gi *= c; g[i] = gi; }
    float pi = p[i] * (1.f - lr * wd);
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi -= step * mi / (sqrtf(vi) / sbc2 + eps);
    p[i] = pi;
  }
}

// Guarded step (include/hiseg_train.h, hiseg_adamw_step_guarded): every block derives the total norm, the
// skip decision and the bias corrections from the partials and the device step count itself.
__global__ void __launch_bounds__(256) adamw_guarded_kernel(float* p, float* g, float* m, float* v, long long n,
                                                            float lr, float b1, float b2, float eps, float wd,
                                                            const float* partial, float max_norm, float* norm_out,
                                                            int* steps, int parity, int* skipped) {
  __shared__ float s_coef, s_step, s_sbc2;
  __shared__ int s_skip;
  if (threadIdx.x == 0) {
    double acc = 0;
    for (int b = 0; b < kOptBlocks; ++b) acc += partial[b];
    const float total = (float)sqrt(acc);
    const bool finite = isfinite(total);
    const int t_prev = steps[parity];
    const int t = t_prev + 1;
    float c = 1.f;
    if (max_norm > 0.f && finite) {
      const float cc = max_norm / (total + 1e-6f);
      c = cc < 1.f ? cc : 1.f;
    }
    const double bc1 = 1.0 - pow((double)b1, (double)t), bc2 = 1.0 - pow((double)b2, (double)t);
    s_coef = c;
    s_step = (float)((double)lr / bc1);
    s_sbc2 = (float)sqrt(bc2);
    s_skip = finite ? 0 : 1;
    if (blockIdx.x == 0) {
      if (norm_out) norm_out[0] = total;
      steps[parity ^ 1] = finite ? t : t_prev;
      if (!finite) skipped[0] += 1;
    }
  }
  __syncthreads();
  if (s_skip) return;
  const float c = s_coef, step = s_step, sbc2 = s_sbc2;
  const bool clip = max_norm > 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float gi = g[i];
    if (clip) { gi *= c; g[i] = gi; }
    float pi = p[i] * (1.f - lr * wd);
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi -= step * mi / (sqrtf(vi) / sbc2 + eps);
    p[i] = pi;
  }
}

// Commit the new step count into the slot the next step reads (the graph-safe form: the host never flips parity).
__global__ void adamw_commit_kernel(int* steps, int parity) {
  if (threadIdx.x == 0) steps[parity] = steps[parity ^ 1];
}

constexpr int kMaxSeg = 256;

// Per-segment step counts (hiseg_adamw_step_segmented): the bias corrections of segment s come from its own
// count; each thread walks its grid-stride indices upwards, so its segment index only advances.
__global__ void __launch_bounds__(256) adamw_seg_kernel(float* p, float* g, float* m, float* v, long long n, float lr,
                                                        float b1, float b2, float omb1, float omb2, float decay,
                                                        float eps, const float* partial,
                                                        float max_norm, float* norm_out, const long long* seg_start,
                                                        int nseg, int* steps, int parity, int* skipped,
                                                        const float* lr_decay) {
  if (lr_decay) {   // device-resident schedule values (hiseg_adamw_step_segmented_dev): a replayed graph reads them
    lr = lr_decay[0];
    decay = lr_decay[1];
  }
  __shared__ float s_step[kMaxSeg], s_sbc2[kMaxSeg];
  __shared__ long long s_seg[kMaxSeg + 1];
  __shared__ float s_coef;
  __shared__ int s_skip;
  if (threadIdx.x == 0) {
    double acc = 0;
    for (int b = 0; b < kOptBlocks; ++b) acc += partial[b];
    const float total = (float)sqrt(acc);
    const bool finite = isfinite(total);
    float c = 1.f;
    if (max_norm > 0.f && finite) {
      const float cc = max_norm / (total + 1e-6f);
      c = cc < 1.f ? cc : 1.f;
    }
    s_coef = c;
    s_skip = finite ? 0 : 1;
    if (blockIdx.x == 0) {
      if (norm_out) norm_out[0] = total;
      if (!finite) skipped[0] += 1;
    }
  }
  for (int k = threadIdx.x; k <= nseg; k += blockDim.x) s_seg[k] = seg_start[k];
  for (int k = threadIdx.x; k < nseg; k += blockDim.x) {
    const int t = steps[parity * nseg + k] + 1;
    const double bc1 = 1.0 - pow((double)b1, (double)t), bc2 = 1.0 - pow((double)b2, (double)t);
    s_step[k] = (float)((double)lr / bc1);
    s_sbc2[k] = (float)sqrt(bc2);
  }
  __syncthreads();
  if (blockIdx.x == 0)
    for (int k = threadIdx.x; k < nseg; k += blockDim.x)
      steps[(parity ^ 1) * nseg + k] = steps[parity * nseg + k] + (s_skip ? 0 : 1);
  if (s_skip) return;
  const float c = s_coef;
  const bool clip = max_norm > 0.f;
  int sg = 0;
  // torch.optim.AdamW's multi-tensor arithmetic, op for op: p *= 1 - lr wd; m = lerp(m, g, 1 - b1);
  // v = v b2 + (1 - b2) g g; p -= (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps)  (complements from the host in double)
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    while (sg + 1 < nseg && i >= s_seg[sg + 1]) ++sg;
    const float step = s_step[sg], sbc2 = s_sbc2[sg];
    float gi = g[i];
    if (clip) { gi *= c; g[i] = gi; }
    const float pi = __fmul_rn(p[i], decay);
    const float m0 = m[i];
    const float mi = omb1 < 0.5f ? __fadd_rn(m0, __fmul_rn(omb1, __fsub_rn(gi, m0)))
                                 : __fsub_rn(gi, __fmul_rn(__fsub_rn(gi, m0), __fsub_rn(1.f, omb1)));
    const float vi = __fadd_rn(__fmul_rn(v[i], b2), __fmul_rn(__fmul_rn(omb2, gi), gi));
    m[i] = mi;
    v[i] = vi;
    const float den = __fadd_rn(__fdiv_rn(__fsqrt_rn(vi), sbc2), eps);
    p[i] = __fadd_rn(pi, __fmul_rn(-step, __fdiv_rn(mi, den)));
  }
}

__global__ void adamw_seg_commit_kernel(int* steps, int nseg, int parity) {
  for (int k = threadIdx.x; k < nseg; k += blockDim.x) steps[parity * nseg + k] = steps[(parity ^ 1) * nseg + k];
}

}  // namespace hiseg

using namespace hiseg;

extern "C" int hiseg_adamw_max_segments(void) { return kMaxSeg; }

extern "C" int hiseg_adamw_step_segmented(float* p, float* g, float* m, float* v, long long n, float lr, float beta1,
                                          float beta2, float one_minus_beta1, float one_minus_beta2, float decay,
                                          float eps, const float* partial, float max_norm, float* norm_out,
                                          const long long* seg_start, int nseg, int* steps, int parity,
                                          int* skipped, hiseg_stream_t stream) {
  HISEG_REQUIRE(p && g && m && v && n > 0 && partial && seg_start && steps && skipped && (parity == 0 || parity == 1),
                HISEG_ERR_BAD_ARG, "adamw_step_segmented: bad arguments");
  HISEG_REQUIRE(nseg >= 1 && nseg <= kMaxSeg, HISEG_ERR_BAD_SHAPE, "adamw_step_segmented: 1..256 segments");
  hipLaunchKernelGGL(adamw_seg_kernel, dim3(kOptBlocks), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr, beta1,
                     beta2, one_minus_beta1, one_minus_beta2, decay, eps, partial, max_norm, norm_out, seg_start, nseg,
                     steps, parity, skipped, (const float*)nullptr);
  hipLaunchKernelGGL(adamw_seg_commit_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, steps, nseg, parity);
  return hiseg_check_launch("adamw_step_segmented");
}

extern "C" int hiseg_adamw_step_segmented_dev(float* p, float* g, float* m, float* v, long long n,
                                              const float* lr_decay, float beta1, float beta2, float one_minus_beta1,
                                              float one_minus_beta2, float eps, const float* partial, float max_norm,
                                              float* norm_out, const long long* seg_start, int nseg, int* steps,
                                              int parity, int* skipped, hiseg_stream_t stream) {
  HISEG_REQUIRE(p && g && m && v && n > 0 && lr_decay && partial && seg_start && steps && skipped &&
                    (parity == 0 || parity == 1),
                HISEG_ERR_BAD_ARG, "adamw_step_segmented_dev: bad arguments");
  HISEG_REQUIRE(nseg >= 1 && nseg <= kMaxSeg, HISEG_ERR_BAD_SHAPE, "adamw_step_segmented_dev: 1..256 segments");
  hipLaunchKernelGGL(adamw_seg_kernel, dim3(kOptBlocks), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, 0.f, beta1,
                     beta2, one_minus_beta1, one_minus_beta2, 0.f, eps, partial, max_norm, norm_out, seg_start, nseg,
                     steps, parity, skipped, lr_decay);
  hipLaunchKernelGGL(adamw_seg_commit_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, steps, nseg, parity);
  return hiseg_check_launch("adamw_step_segmented_dev");
}

extern "C" int hiseg_adamw_step_guarded(float* p, float* g, float* m, float* v, long long n, float lr, float beta1,
                                        float beta2, float eps, float weight_decay, const float* partial, float max_norm,
                                        float* norm_out, int* steps, int parity, int* skipped, hiseg_stream_t stream) {
  HISEG_REQUIRE(p && g && m && v && n > 0 && partial && steps && skipped && (parity == 0 || parity == 1),
                HISEG_ERR_BAD_ARG, "adamw_step_guarded: bad arguments");
  hipLaunchKernelGGL(adamw_guarded_kernel, dim3(kOptBlocks), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr,
                     beta1, beta2, eps, weight_decay, partial, max_norm, norm_out, steps, parity, skipped);
  hipLaunchKernelGGL(adamw_commit_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, steps, parity);
  return hiseg_check_launch("adamw_step_guarded");
}

extern "C" int hiseg_optim_blocks(void) { return kOptBlocks; }

extern "C" int hiseg_grad_norm_partials(const float* g, long long n, float* partial, hiseg_stream_t stream) {
  HISEG_REQUIRE(g && partial && n > 0, HISEG_ERR_BAD_ARG, "grad_norm_partials: bad arguments");
  hipLaunchKernelGGL(grad_norm_kernel, dim3(kOptBlocks), dim3(256), 0, (hipStream_t)stream, g, n, partial);
  return hiseg_check_launch("grad_norm_partials");
}

extern "C" int hiseg_adamw_step(float* p, float* g, float* m, float* v, long long n, float lr, float beta1, float beta2,
                                float eps, float weight_decay, float bc1, float bc2, const float* partial,
                                float max_norm, float* norm_out, hiseg_stream_t stream) {
  HISEG_REQUIRE(p && g && m && v && n > 0 && bc1 > 0.f && bc2 > 0.f, HISEG_ERR_BAD_ARG, "adamw_step: bad arguments");
  hipLaunchKernelGGL(adamw_kernel, dim3(kOptBlocks), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr, beta1, beta2,
                     eps, weight_decay, bc1, bc2, partial, max_norm, norm_out);
  return hiseg_check_launch("adamw_step");
}
