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

}  // namespace hiseg

using namespace hiseg;

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
