// EfficientNet depthwise convolution in training (timm conv_dw: groups = C, bias-free, k 3/5, stride 1/2,
// "same" padding k/2), NHWC, weights in the parameter's own layout [C][k*k] f32 (no per-step repack).
// HBM-bound passes, one 16-B channel chunk per thread (include/hiseg_train.h, hiseg_dw_*):
//   fwd         out[n,oy,ox,c] = sum_t w[c,t] x[n, oy*s-p+ky, ox*s-p+kx, c]      (raw: train-mode BN follows)
//   bwd_data    dx[n,iy,ix,c] (+)= sum over taps whose output (oy, ox) maps onto (iy, ix)
//   bwd_weight  dw[c,t] (+)= sum_{n,oy,ox} dy[n,oy,ox,c] x[n,iy,ix,c]  -- per-split partials, then a reduce
#include "common.h"
#include "hiseg_train.h"

namespace hiseg {

template <typename T>
__device__ __forceinline__ void ldc(const void* p, long long i, float* v) {
  Chunk<T>::unpack(*reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(p) + i), v);
}

template <typename T>
__global__ void __launch_bounds__(256) dw_fwd_kernel(const void* x, int N, int H, int W, int C, int K, int s,
                                                     const float* w, void* out, int Ho, int Wo) {
  constexpr int V = Chunk<T>::N;
  const int nch = C / V, pad = K / 2, KK = K * K;
  const long long n_el = (long long)N * Ho * Wo * nch;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n_el; i += (long long)gridDim.x * 256) {
    const int ch = (int)(i % nch);
    const long long q = i / nch;
    const int ox = (int)(q % Wo);
    const long long r = q / Wo;
    const int oy = (int)(r % Ho);
    const int n = (int)(r / Ho);
    const int c = ch * V;
    float acc[V], v[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    for (int ky = 0; ky < K; ++ky) {
      const int iy = oy * s - pad + ky;
      if ((unsigned)iy >= (unsigned)H) continue;
      for (int kx = 0; kx < K; ++kx) {
        const int ix = ox * s - pad + kx;
        if ((unsigned)ix >= (unsigned)W) continue;
        ldc<T>(x, (((long long)n * H + iy) * W + ix) * C + c, v);
        const int t = ky * K + kx;
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += v[e] * w[(c + e) * KK + t];
      }
    }
    *reinterpret_cast<uint4*>(reinterpret_cast<T*>(out) + q * C + c) = Chunk<T>::pack(acc);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) dw_bwd_data_kernel(const void* dy, int N, int H, int W, int C, int K, int s,
                                                          const float* w, int Ho, int Wo, void* dx, int accumulate) {
  constexpr int V = Chunk<T>::N;
  const int nch = C / V, pad = K / 2, KK = K * K;
  const long long n_el = (long long)N * H * W * nch;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n_el; i += (long long)gridDim.x * 256) {
    const int ch = (int)(i % nch);
    const long long q = i / nch;
    const int ix = (int)(q % W);
    const long long r = q / W;
    const int iy = (int)(r % H);
    const int n = (int)(r / H);
    const int c = ch * V;
    float acc[V], v[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    for (int ky = 0; ky < K; ++ky) {
      const int ny = iy + pad - ky;
      if (ny < 0 || ny % s) continue;
      const int oy = ny / s;
      if (oy >= Ho) continue;
      for (int kx = 0; kx < K; ++kx) {
        const int nx = ix + pad - kx;
        if (nx < 0 || nx % s) continue;
        const int ox = nx / s;
        if (ox >= Wo) continue;
        ldc<T>(dy, (((long long)n * Ho + oy) * Wo + ox) * C + c, v);
        const int t = ky * K + kx;
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += v[e] * w[(c + e) * KK + t];
      }
    }
    T* dst = reinterpret_cast<T*>(dx) + q * C + c;
    if (accumulate) {
      Chunk<T>::unpack(*reinterpret_cast<const uint4*>(dst), v);
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] += v[e];
    }
    *reinterpret_cast<uint4*>(dst) = Chunk<T>::pack(acc);
  }
}

// grid (S = dw_wsplits, ceil(tasks / TPB)), tasks = (channel chunk, filter row ky) pairs, TPB = min(tasks, 256) of them per
// block and R = 256 / TPB pixel lanes each: thread (task, r) walks pixels b + r, b + r + R, ... of its split with
// incrementally advanced (n, oy, ox) (32-bit; no per-pixel division), K x V accumulators (one per kx and channel),
// then the R lanes of a task are summed in LDS in lane order.  (The first form gave each task ONE thread walking
// its split's P / 128 pixels with three 64-bit divisions per pixel: the B0 student's 16- and 24-channel layers at
// 320 x 320 ran 6-12 tasks per block, 128 blocks -- 6.6 ms of the unfrozen distillation step.)
template <typename T>
__global__ void __launch_bounds__(256) dw_bwd_weight_kernel(const void* x, const void* dy, int N, int H, int W, int C,
                                                            int K, int s, int Ho, int Wo, int TPB, float* ws) {
  constexpr int V = Chunk<T>::N;
  __shared__ float red[256 * V];
  const int nch = C / V, pad = K / 2, KK = K * K;
  const int R = 256 / TPB;
  const int tl = threadIdx.x % TPB, r = threadIdx.x / TPB;
  const int task = blockIdx.y * TPB + tl;
  const bool live = task < nch * K && r < R;
  const int ch = live ? task / K : 0, ky = live ? task - ch * K : 0;
  const int c = ch * V;
  const int P = N * Ho * Wo;
  const int b = (int)((long long)P * blockIdx.x / gridDim.x), e = (int)((long long)P * (blockIdx.x + 1) / gridDim.x);
  float acc[5][V];
#pragma unroll
  for (int kx = 0; kx < 5; ++kx)
#pragma unroll
    for (int k = 0; k < V; ++k) acc[kx][k] = 0.f;
  int q = b + r;
  if (live && q < e) {
    int ox = q % Wo, t2 = q / Wo, oy = t2 % Ho, n = t2 / Ho;
    const int dx = R % Wo, dyr = R / Wo;
    for (; q < e; q += R) {
      const int iy = oy * s - pad + ky;
      if ((unsigned)iy < (unsigned)H) {
        float g[V], v[V];
        ldc<T>(dy, (long long)q * C + c, g);
        const long long rowb = ((long long)n * H + iy) * W;
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) {
          if (kx >= K) break;
          const int ix = ox * s - pad + kx;
          if ((unsigned)ix >= (unsigned)W) continue;
          ldc<T>(x, (rowb + ix) * C + c, v);
#pragma unroll
          for (int k = 0; k < V; ++k) acc[kx][k] += g[k] * v[k];
        }
      }
      ox += dx;
      oy += dyr;
      if (ox >= Wo) { ox -= Wo; ++oy; }
      while (oy >= Ho) { oy -= Ho; ++n; }
    }
  }
  float* out = ws + (long long)blockIdx.x * C * KK;
#pragma unroll
  for (int kx = 0; kx < 5; ++kx) {
    if (kx >= K) break;
#pragma unroll
    for (int k = 0; k < V; ++k) red[threadIdx.x * V + k] = acc[kx][k];
    __syncthreads();
    if (r == 0 && live) {
      float sum[V];
#pragma unroll
      for (int k = 0; k < V; ++k) sum[k] = red[tl * V + k];
      for (int rr = 1; rr < R; ++rr)
#pragma unroll
        for (int k = 0; k < V; ++k) sum[k] += red[(rr * TPB + tl) * V + k];
#pragma unroll
      for (int k = 0; k < V; ++k) out[(c + k) * KK + ky * K + kx] = sum[k];
    }
    __syncthreads();
  }
}

// dw[i] += sum_s ws[s][i]: a block = 64 outputs x 4 split groups (group g sums splits g, g + 4, ... in order, four
// loads in flight), the groups combined in LDS in order.  The sums run in double (up to 1024 split partials per weight
// on the large-pixel layers of the unfrozen encoder; the loads, not the adds, bound this pass).  (One thread per output
// walking every split in double was 33 us per call on the 288-output layers.)
__global__ void __launch_bounds__(256) dw_weight_reduce_kernel(const float* ws, int S, int n, float* dw) {
  __shared__ double red[4][64];
  const int ol = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + ol;
  double acc = 0.0;
  if (i < n) {
    int sp = g;
    for (; sp + 12 < S; sp += 16) {
      const float a0 = ws[(long long)sp * n + i], a1 = ws[(long long)(sp + 4) * n + i];
      const float a2 = ws[(long long)(sp + 8) * n + i], a3 = ws[(long long)(sp + 12) * n + i];
      acc += a0; acc += a1; acc += a2; acc += a3;
    }
    for (; sp < S; sp += 4) acc += ws[(long long)sp * n + i];
  }
  red[g][ol] = acc;
  __syncthreads();
  if (g == 0 && i < n) dw[i] = (float)((double)dw[i] + (((red[0][ol] + red[1][ol]) + red[2][ol]) + red[3][ol]));
}

// pixel splits of the weight gradient: about 32 pixels per thread (R pixel lanes per task), at most kDwMaxSplits
static int dw_wsplits(long long P, int C, int K, int V) {
  const int tasks = (C / V) * K, TPB = tasks < 256 ? tasks : 256, R = 256 / TPB;
  long long sp = P / (32ll * R);
  if (sp < 1) sp = 1;
  if (sp > 1024) sp = 1024;
  return (int)sp;
}

inline unsigned dw_blocks(long long n) {
  const long long b = (n + 255) / 256;
  return (unsigned)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

}  // namespace hiseg

using namespace hiseg;

#define DW_DISPATCH(dtype, KERNEL, ...)                                                 \
  do {                                                                                  \
    if ((dtype) == HISEG_BF16) hipLaunchKernelGGL(KERNEL<bf16_t>, __VA_ARGS__);         \
    else hipLaunchKernelGGL(KERNEL<float>, __VA_ARGS__);                                \
  } while (0)

static int dw_check(int dtype, int N, int H, int W, int C, int K, int stride, int Ho, int Wo) {
  HISEG_REQUIRE(dtype == HISEG_BF16 || dtype == HISEG_F32, HISEG_ERR_BAD_DTYPE, "dw: dtype %d", dtype);
  HISEG_REQUIRE(N > 0 && H > 0 && W > 0 && K >= 1 && K <= 5 && K % 2 == 1 && (stride == 1 || stride == 2),
                HISEG_ERR_BAD_SHAPE, "dw: shape (K %d stride %d)", K, stride);
  HISEG_REQUIRE(C > 0 && C % (dtype == HISEG_BF16 ? 8 : 4) == 0, HISEG_ERR_BAD_SHAPE, "dw: C %d not chunk-aligned", C);
  HISEG_REQUIRE(Ho == (H + 2 * (K / 2) - K) / stride + 1 && Wo == (W + 2 * (K / 2) - K) / stride + 1,
                HISEG_ERR_BAD_SHAPE, "dw: output %dx%d does not match", Ho, Wo);
  return HISEG_OK;
}

extern "C" int hiseg_dw_train_fwd(int dtype, const void* x, int N, int H, int W, int C, int K, int stride,
                                  const float* w, void* out, int Ho, int Wo, hiseg_stream_t stream) {
  HISEG_REQUIRE(x && w && out, HISEG_ERR_BAD_ARG, "dw_train_fwd: null");
  const int r = dw_check(dtype, N, H, W, C, K, stride, Ho, Wo);
  if (r) return r;
  const long long n = (long long)N * Ho * Wo * (C / (dtype == HISEG_BF16 ? 8 : 4));
  DW_DISPATCH(dtype, dw_fwd_kernel, dim3(dw_blocks(n)), dim3(256), 0, (hipStream_t)stream, x, N, H, W, C, K, stride, w,
              out, Ho, Wo);
  return hiseg_check_launch("dw_train_fwd");
}

extern "C" int hiseg_dw_bwd_data(int dtype, const void* dy, int N, int H, int W, int C, int K, int stride,
                                 const float* w, int Ho, int Wo, void* dx, int accumulate, hiseg_stream_t stream) {
  HISEG_REQUIRE(dy && w && dx, HISEG_ERR_BAD_ARG, "dw_bwd_data: null");
  const int r = dw_check(dtype, N, H, W, C, K, stride, Ho, Wo);
  if (r) return r;
  const long long n = (long long)N * H * W * (C / (dtype == HISEG_BF16 ? 8 : 4));
  DW_DISPATCH(dtype, dw_bwd_data_kernel, dim3(dw_blocks(n)), dim3(256), 0, (hipStream_t)stream, dy, N, H, W, C, K,
              stride, w, Ho, Wo, dx, accumulate);
  return hiseg_check_launch("dw_bwd_data");
}

extern "C" long long hiseg_dw_bwd_weight_ws(int dtype, int N, int Ho, int Wo, int C, int K) {
  return (long long)dw_wsplits((long long)N * Ho * Wo, C, K, dtype == HISEG_BF16 ? 8 : 4) * C * K * K;
}

extern "C" int hiseg_dw_bwd_weight(int dtype, const void* x, const void* dy, int N, int H, int W, int C, int K,
                                   int stride, int Ho, int Wo, float* ws, float* dw, hiseg_stream_t stream) {
  HISEG_REQUIRE(x && dy && ws && dw, HISEG_ERR_BAD_ARG, "dw_bwd_weight: null");
  const int r = dw_check(dtype, N, H, W, C, K, stride, Ho, Wo);
  if (r) return r;
  const int nch = C / (dtype == HISEG_BF16 ? 8 : 4);
  HISEG_REQUIRE((long long)N * H * W * C < (1ll << 31) && (long long)N * Ho * Wo < (1ll << 31), HISEG_ERR_BAD_SHAPE,
                "dw_bwd_weight: tensor too large");
  hipStream_t s = (hipStream_t)stream;
  const int tasks = nch * K, TPB = tasks < 256 ? tasks : 256;
  const int S = dw_wsplits((long long)N * Ho * Wo, C, K, dtype == HISEG_BF16 ? 8 : 4);
  DW_DISPATCH(dtype, dw_bwd_weight_kernel, dim3(S, (tasks + TPB - 1) / TPB), dim3(256), 0, s, x, dy, N, H, W,
              C, K, stride, Ho, Wo, TPB, ws);
  const int n = C * K * K;
  hipLaunchKernelGGL(dw_weight_reduce_kernel, dim3((n + 63) / 64), dim3(256), 0, s, ws, S, n, dw);
  return hiseg_check_launch("dw_bwd_weight");
}
