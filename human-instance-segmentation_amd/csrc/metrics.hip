// Per-sample (target, prediction) histograms for the validation metrics (include/hiseg_metrics.h).
//
// One HBM pass over the logits (or predicted labels) and the int64 targets: grid (splits, samples), each
// thread classifies 4 consecutive pixels per step (16-B loads per channel plane and per target pair),
// keeps its histogram in registers (K = (C+2)(C+1) counters, a compare-add per counter per pixel --
// well inside the VALU budget of a 4*C+8 byte/pixel stream), then the block reduces it (cross-lane
// shuffles, LDS) and adds it to conf with one 64-bit atomic per counter.  Integer counts: the result is
// exact and independent of the launch shape.
#include "common.h"
#include "hiseg_metrics.h"

namespace hiseg {

constexpr int kMetPx = 2048;   // pixels per block (256 threads x 4 pixels x 2 steps)

template <int C>
__device__ __forceinline__ int argmax_c(const float* v) {
  float best = v[0];
  int bi = 0;
#pragma unroll
  for (int c = 1; c < C; ++c) {
    if (best == best && (v[c] != v[c] || v[c] > best)) {  // first maximum; NaN is the maximum
      best = v[c];
      bi = c;
    }
  }
  return bi;
}

template <int C>
__device__ __forceinline__ int row_of(long long t) { return t >= 0 ? (t < C ? (int)t : C) : C + 1; }

template <int C>
__device__ __forceinline__ int col_of(long long p) { return (p >= 0 && p < C) ? (int)p : C; }

template <int K>
__device__ __forceinline__ void count(unsigned (&cnt)[K], int k) {
#pragma unroll
  for (int j = 0; j < K; ++j) cnt[j] += (k == j) ? 1u : 0u;
}

template <typename T, int C, bool LABELS>
__global__ void __launch_bounds__(256) seg_confusion_kernel(const void* logits, const long long* labels,
                                                            const long long* target, long long HW, int vec,
                                                            unsigned long long* conf) {
  constexpr int K = (C + 2) * (C + 1);
  __shared__ unsigned red[K];
  const int n = blockIdx.y, t = threadIdx.x;
  if (t < K) red[t] = 0u;
  unsigned cnt[K];
#pragma unroll
  for (int j = 0; j < K; ++j) cnt[j] = 0u;

  const long long beg = (long long)blockIdx.x * kMetPx;
  const long long end = beg + kMetPx < HW ? beg + kMetPx : HW;
  const long long* tg = target + (long long)n * HW;
  const long long* lb = LABELS ? labels + (long long)n * HW : nullptr;
  const T* lg = LABELS ? nullptr : reinterpret_cast<const T*>(logits) + (long long)n * C * HW;

  if (vec) {   // HW % 4 == 0 and 16-B (f32) / 8-B (bf16) aligned planes
    // two 4-pixel groups per thread and iteration, every load of both issued before the counting
    for (long long i0 = beg + 4 * t; i0 < end; i0 += 8 * 256) {
      long long tv[2][4];
      float v[2][4][C];
      long long lv[2][4];
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const long long i = i0 + g * 1024;
        if (g == 1 && i >= end) break;
        const longlong2 t01 = *reinterpret_cast<const longlong2*>(tg + i);
        const longlong2 t23 = *reinterpret_cast<const longlong2*>(tg + i + 2);
        tv[g][0] = t01.x; tv[g][1] = t01.y; tv[g][2] = t23.x; tv[g][3] = t23.y;
        if constexpr (LABELS) {
          const longlong2 l01 = *reinterpret_cast<const longlong2*>(lb + i);
          const longlong2 l23 = *reinterpret_cast<const longlong2*>(lb + i + 2);
          lv[g][0] = l01.x; lv[g][1] = l01.y; lv[g][2] = l23.x; lv[g][3] = l23.y;
        } else {
#pragma unroll
          for (int c = 0; c < C; ++c) {
            if constexpr (sizeof(T) == 4) {
              const float4 q = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(lg) + (long long)c * HW + i);
              v[g][0][c] = q.x; v[g][1][c] = q.y; v[g][2][c] = q.z; v[g][3][c] = q.w;
            } else {
              const uint2 q = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(lg) + (long long)c * HW + i);
              v[g][0][c] = __uint_as_float(q.x << 16); v[g][1][c] = __uint_as_float(q.x & 0xffff0000u);
              v[g][2][c] = __uint_as_float(q.y << 16); v[g][3][c] = __uint_as_float(q.y & 0xffff0000u);
            }
          }
        }
      }
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        if (g == 1 && i0 + 1024 >= end) break;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int col;
          if constexpr (LABELS) col = col_of<C>(lv[g][e]);
          else col = argmax_c<C>(v[g][e]);
          count<K>(cnt, row_of<C>(tv[g][e]) * (C + 1) + col);
        }
      }
    }
  } else {
    for (long long i = beg + t; i < end; i += 256) {
      int col;
      if constexpr (LABELS) {
        col = col_of<C>(lb[i]);
      } else {
        float v[C];
#pragma unroll
        for (int c = 0; c < C; ++c) v[c] = Elem<T>::load(lg, (long long)c * HW + i);
        col = argmax_c<C>(v);
      }
      count<K>(cnt, row_of<C>(tg[i]) * (C + 1) + col);
    }
  }

  // wave sums, then the block's sum in LDS, then one atomic per counter
#pragma unroll
  for (int j = 0; j < K; ++j) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cnt[j] += __shfl_xor(cnt[j], off, 64);
  }
  __syncthreads();
  if ((t & 63) == 0) {
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (cnt[j]) atomicAdd(&red[j], cnt[j]);
  }
  __syncthreads();
  if (t < K && red[t]) atomicAdd(conf + (long long)n * K + t, (unsigned long long)red[t]);
}

}  // namespace hiseg

using namespace hiseg;

template <typename T, bool LABELS>
static void conf_launch(int C, dim3 g, hipStream_t s, const void* lg, const long long* lb, const long long* tg,
                        long long HW, int vec, unsigned long long* conf) {
  switch (C) {
    case 2: hipLaunchKernelGGL((seg_confusion_kernel<T, 2, LABELS>), g, dim3(256), 0, s, lg, lb, tg, HW, vec, conf); break;
    case 3: hipLaunchKernelGGL((seg_confusion_kernel<T, 3, LABELS>), g, dim3(256), 0, s, lg, lb, tg, HW, vec, conf); break;
    default: hipLaunchKernelGGL((seg_confusion_kernel<T, 4, LABELS>), g, dim3(256), 0, s, lg, lb, tg, HW, vec, conf); break;
  }
}

extern "C" int hiseg_seg_confusion(const void* logits, int dtype, const long long* pred_labels,
                                   const long long* target, int N, int C, long long HW, unsigned long long* conf,
                                   hiseg_stream_t stream) {
  HISEG_REQUIRE(target && conf && (logits || pred_labels), HISEG_ERR_BAD_ARG, "seg_confusion: null");
  HISEG_REQUIRE(N > 0 && N <= 65535 && HW > 0 && C >= 2 && C <= 4, HISEG_ERR_BAD_SHAPE,
                "seg_confusion: N %d C %d HW %lld", N, C, HW);
  HISEG_REQUIRE(pred_labels || dtype == HISEG_F32 || dtype == HISEG_BF16, HISEG_ERR_BAD_DTYPE,
                "seg_confusion: dtype %d", dtype);
  const long long splits = (HW + kMetPx - 1) / kMetPx;
  HISEG_REQUIRE(splits <= 0x7fffffffll, HISEG_ERR_BAD_SHAPE, "seg_confusion: HW %lld too large", HW);
  const dim3 g((unsigned)splits, (unsigned)N);
  hipStream_t s = (hipStream_t)stream;
  const uintptr_t align_mask = (pred_labels || dtype == HISEG_F32) ? 15 : 7;
  const int vec = (HW % 4 == 0) && ((reinterpret_cast<uintptr_t>(target) & 15) == 0) &&
                  ((reinterpret_cast<uintptr_t>(pred_labels ? (const void*)pred_labels : logits) & align_mask) == 0);
  if (pred_labels) conf_launch<float, true>(C, g, s, nullptr, pred_labels, target, HW, vec, conf);
  else if (dtype == HISEG_F32) conf_launch<float, false>(C, g, s, logits, nullptr, target, HW, vec, conf);
  else conf_launch<bf16_t, false>(C, g, s, logits, nullptr, target, HW, vec, conf);
  return hiseg_check_launch("seg_confusion");
}
