// Training data path on the GPU (include/hiseg_data.h): PIL-exact bilinear resize of 8-bit images and the
// fused 3-class ROI target gather.  Both are byte-stream passes (HBM / L2 bound): one thread per output
// pixel (resize: all channels of the pixel; targets: one class id), integer arithmetic with the same
// fixed-point weights and rounding as Pillow, so the results are bit-identical to the host library.
#include <math.h>

#include <vector>

#include "common.h"
#include "hiseg_data.h"

namespace hiseg {

constexpr int kPilBits = 22;   // Pillow Resample.c PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ int clip8(int v) {   // Pillow clip8: lookups[v >> PRECISION_BITS], clamped to [0, 255]
  const int q = v >> kPilBits;
  return q < 0 ? 0 : (q > 255 ? 255 : q);
}

template <int C>
__global__ void __launch_bounds__(256) pil_h_kernel(const uint8_t* src, int H, int W, int y_first, int rows, int Wout,
                                                    int ksize, const int* bounds, const int* kk, uint8_t* tmp) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (idx >= (long long)rows * Wout) return;
  const int xx = (int)(idx % Wout), yy = (int)(idx / Wout);
  const int xmin = bounds[2 * xx], xmax = bounds[2 * xx + 1];
  const int* k = kk + (long long)xx * ksize;
  const uint8_t* row = src + (((long long)b * H + yy + y_first) * W + xmin) * C;
  int ss[C];
#pragma unroll
  for (int c = 0; c < C; ++c) ss[c] = 1 << (kPilBits - 1);
  for (int x = 0; x < xmax; ++x) {
    const int w = k[x];
#pragma unroll
    for (int c = 0; c < C; ++c) ss[c] += (int)row[x * C + c] * w;
  }
  uint8_t* o = tmp + (((long long)b * rows + yy) * Wout + xx) * C;
#pragma unroll
  for (int c = 0; c < C; ++c) o[c] = (uint8_t)clip8(ss[c]);
}

template <int C, bool F32>
__global__ void __launch_bounds__(256) pil_v_kernel(const uint8_t* tmp, int rows, int W, int Hout, int ksize,
                                                    const int* bounds, const int* kk, void* out) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (idx >= (long long)Hout * W) return;
  const int xx = (int)(idx % W), yy = (int)(idx / W);
  const int ymin = bounds[2 * yy], ymax = bounds[2 * yy + 1];
  const int* k = kk + (long long)yy * ksize;
  const uint8_t* col = tmp + (((long long)b * rows + ymin) * W + xx) * C;
  int ss[C];
#pragma unroll
  for (int c = 0; c < C; ++c) ss[c] = 1 << (kPilBits - 1);
  for (int y = 0; y < ymax; ++y) {
    const int w = k[y];
#pragma unroll
    for (int c = 0; c < C; ++c) ss[c] += (int)col[(long long)y * W * C + c] * w;
  }
  if constexpr (F32) {   // image.astype(float32) / 255 (dataset.py:282), CHW
    float* o = reinterpret_cast<float*>(out);
#pragma unroll
    for (int c = 0; c < C; ++c) o[(((long long)b * C + c) * Hout + yy) * W + xx] = (float)clip8(ss[c]) / 255.0f;
  } else {
    uint8_t* o = reinterpret_cast<uint8_t*>(out) + (((long long)b * Hout + yy) * W + xx) * C;
#pragma unroll
    for (int c = 0; c < C; ++c) o[c] = (uint8_t)clip8(ss[c]);
  }
}

// cv2.resize(..., INTER_NEAREST) source index (OpenCV resizeNN): min(floor(x / (dst / src)), src - 1)
__device__ __forceinline__ int nn_src(int x, int src, int dst) {
  const double ifx = 1.0 / ((double)dst / (double)src);
  const int s = (int)floor((double)x * ifx);
  return s < src - 1 ? s : src - 1;
}

__global__ void __launch_bounds__(256) roi_targets_kernel(const uint8_t* masks, const hiseg_roi_target_desc* descs,
                                                          int mh, int mw, long long* out) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (idx >= mh * mw) return;
  const hiseg_roi_target_desc d = descs[b];
  const int i = idx / mw, j = idx - (idx / mw) * mw;
  const int rh = d.y2 - d.y1, rw = d.x2 - d.x1;
  const int yi = d.y1 + nn_src(i, rh, mh), xi = d.x1 + nn_src(j, rw, mw);    // dataset.py:272 (ROI -> mask)
  const int y0 = nn_src(yi, d.h0, d.img_h), x0 = nn_src(xi, d.w0, d.img_w);  // dataset.py:117 (orig -> image)
  const long long plane = (long long)d.h0 * d.w0;
  const uint8_t* m = masks + d.mask_offset + (long long)y0 * d.w0 + x0;
  long long cls = 0;
  if (m[(long long)d.target * plane] > 0) {
    cls = 1;                                                                    // dataset.py:153
  } else {
    for (int k = 0; k < d.n_inst; ++k)
      if (k != d.target && m[(long long)k * plane] > 0) { cls = 2; break; }     // dataset.py:156-160
  }
  out[(long long)b * mh * mw + idx] = cls;
}

inline unsigned nblk(long long n) { return (unsigned)((n + 255) / 256); }

}  // namespace hiseg

using namespace hiseg;

// Pillow libImaging/Resample.c precompute_coeffs + normalize_coeffs_8bpc for the bilinear filter
// (support 1), box [0, in_size].
extern "C" int hiseg_pil_bilinear_table(int in_size, int out_size, int* ksize_out, int* bounds, int* kk) {
  HISEG_REQUIRE(in_size > 0 && out_size > 0 && ksize_out, HISEG_ERR_BAD_ARG, "pil_bilinear_table: sizes %d -> %d",
                in_size, out_size);
  double filterscale, scale;
  filterscale = scale = (double)((float)in_size - 0.0f) / out_size;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = 1.0 * filterscale;
  const int ksize = (int)ceil(support) * 2 + 1;
  *ksize_out = ksize;
  if (!bounds || !kk) return HISEG_OK;
  std::vector<double> k(ksize);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = 0.0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    int x = 0;
    for (; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      const double w = t < 1.0 ? 1.0 - t : 0.0;
      k[x] = w;
      ww += w;
    }
    for (x = 0; x < xmax; ++x)
      if (ww != 0.0) k[x] /= ww;
    for (; x < ksize; ++x) k[x] = 0;
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
    for (x = 0; x < ksize; ++x)
      kk[(long long)xx * ksize + x] = k[x] < 0 ? (int)(-0.5 + k[x] * (1 << kPilBits)) : (int)(0.5 + k[x] * (1 << kPilBits));
  }
  return HISEG_OK;
}

#define PIL_C_DISPATCH(C, ...)                          \
  switch (C) {                                          \
    case 1: { constexpr int CC = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int CC = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int CC = 3; __VA_ARGS__; } break; \
    default: { constexpr int CC = 4; __VA_ARGS__; } break; \
  }

extern "C" int hiseg_pil_resample_h(const unsigned char* src, int B, int H, int W, int C, int y_first, int rows,
                                    int Wout, int ksize, const int* bounds, const int* kk, unsigned char* tmp,
                                    hiseg_stream_t stream) {
  HISEG_REQUIRE(src && bounds && kk && tmp, HISEG_ERR_BAD_ARG, "pil_resample_h: null");
  HISEG_REQUIRE(B > 0 && B <= 65535 && H > 0 && W > 0 && C >= 1 && C <= 4 && Wout > 0 && ksize > 0 && rows > 0 &&
                    y_first >= 0 && y_first + rows <= H,
                HISEG_ERR_BAD_SHAPE, "pil_resample_h: shape");
  const dim3 g(nblk((long long)rows * Wout), (unsigned)B);
  PIL_C_DISPATCH(C, hipLaunchKernelGGL(pil_h_kernel<CC>, g, dim3(256), 0, (hipStream_t)stream, src, H, W, y_first,
                                       rows, Wout, ksize, bounds, kk, tmp));
  return hiseg_check_launch("pil_resample_h");
}

extern "C" int hiseg_pil_resample_v(const unsigned char* tmp, int B, int rows, int W, int C, int Hout, int ksize,
                                    const int* bounds, const int* kk, int out_f32, void* out, hiseg_stream_t stream) {
  HISEG_REQUIRE(tmp && bounds && kk && out, HISEG_ERR_BAD_ARG, "pil_resample_v: null");
  HISEG_REQUIRE(B > 0 && B <= 65535 && rows > 0 && W > 0 && C >= 1 && C <= 4 && Hout > 0 && ksize > 0,
                HISEG_ERR_BAD_SHAPE, "pil_resample_v: shape");
  const dim3 g(nblk((long long)Hout * W), (unsigned)B);
  hipStream_t s = (hipStream_t)stream;
  if (out_f32) {
    PIL_C_DISPATCH(C, hipLaunchKernelGGL((pil_v_kernel<CC, true>), g, dim3(256), 0, s, tmp, rows, W, Hout, ksize,
                                         bounds, kk, out));
  } else {
    PIL_C_DISPATCH(C, hipLaunchKernelGGL((pil_v_kernel<CC, false>), g, dim3(256), 0, s, tmp, rows, W, Hout, ksize,
                                         bounds, kk, out));
  }
  return hiseg_check_launch("pil_resample_v");
}

extern "C" int hiseg_roi_targets(const unsigned char* masks, const hiseg_roi_target_desc* descs, int B, int mh,
                                 int mw, long long* out, hiseg_stream_t stream) {
  HISEG_REQUIRE(masks && descs && out, HISEG_ERR_BAD_ARG, "roi_targets: null");
  HISEG_REQUIRE(B > 0 && B <= 65535 && mh > 0 && mw > 0 && (long long)mh * mw < (1ll << 31), HISEG_ERR_BAD_SHAPE,
                "roi_targets: shape");
  hipLaunchKernelGGL(roi_targets_kernel, dim3(nblk((long long)mh * mw), (unsigned)B), dim3(256), 0,
                     (hipStream_t)stream, masks, descs, mh, mw, out);
  return hiseg_check_launch("roi_targets");
}
