#include <cstdlib>
// Training kernels of the refined hierarchical head's non-conv ops (gfx950):
//   * SpatialAttentionModule (attention_modules.py:67-113) train forward (+ Dropout2d) / backward
//   * ChannelAttentionModule (attention_modules.py:10-64) train forward (+ Dropout2d) / backward
//   * upsample_bg_fg [ConvT 2->32, BatchNorm(train), ReLU, 1x1 32->2] + softmax + hierarchical
//     combine + the target branch's last 1x1 (refinement.py:501-506,559-596) forward / backward
//   * the target branch's last 1x1 conv (Ct -> 2) backward
// All are HBM-streaming kernels; reductions go through deterministic per-block partials and a
// finalize kernel (no atomics).
#include <float.h>
#include "common.h"
#include "hiseg_train.h"
#include "hiseg_head_train.h"

namespace hiseg {

template <typename T>
__device__ __forceinline__ float ldT(const void* p, long long i) { return Elem<T>::load(p, i); }
template <typename T>
__device__ __forceinline__ void stT(void* p, long long i, float v) { Elem<T>::store(p, i, v); }

static inline unsigned nb(long long n, int bs) { return (unsigned)((n + bs - 1) / bs); }
static inline unsigned capb(long long n) {
  long long b = (n + 255) / 256;
  return (unsigned)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

// ======================================================================================= spatial attention
// stats[p] = (mean_c x, max_c x), argmax[p] = first channel attaining the max.
template <typename T>
__global__ void __launch_bounds__(256) sa_stats_kernel(const void* x, long long P, int C, float* stats, int* argmax) {
  constexpr int K = Chunk<T>::N;
  constexpr int G = 16;
  const int nch = C / K;
  const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long pix = gid / G;
  const int l = (int)(gid % G);
  float s = 0.f, m = -FLT_MAX, v[K];
  int am = 0x7fffffff;
  if (pix < P) {
    const uint4* src = reinterpret_cast<const uint4*>(x) + pix * nch;
    for (int ch = l; ch < nch; ch += G) {
      Chunk<T>::unpack(src[ch], v);
#pragma unroll
      for (int e = 0; e < K; ++e) {
        s += v[e];
        if (v[e] > m) { m = v[e]; am = ch * K + e; }
      }
    }
  }
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) {
    s += __shfl_xor(s, off, G);
    const float mo = __shfl_xor(m, off, G);
    const int ao = __shfl_xor(am, off, G);
    if (mo > m || (mo == m && ao < am)) { m = mo; am = ao; }
  }
  if (pix < P && l == 0) {
    stats[pix * 2] = s / (float)C;
    stats[pix * 2 + 1] = m;
    argmax[pix] = am;
  }
}

__global__ void __launch_bounds__(256) sa_map_kernel(const float* stats, int N, int H, int W, const float* w, int k,
                                                     float* att) {
  const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (long long)N * H * W) return;
  const int x = (int)(gid % W);
  const long long t = gid / W;
  const int y = (int)(t % H);
  const int n = (int)(t / H);
  const int r = k / 2;
  float acc = 0.f;
  for (int c = 0; c < 2; ++c)
    for (int ky = 0; ky < k; ++ky) {
      const int yy = y + ky - r;
      if (yy < 0 || yy >= H) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int xx = x + kx - r;
        if (xx < 0 || xx >= W) continue;
        acc += w[(c * k + ky) * k + kx] * stats[(((long long)n * H + yy) * W + xx) * 2 + c];
      }
    }
  att[gid] = sigmoidf_(acc);
}

// out = x * att[p] * mul[n][c]
template <typename T>
__global__ void __launch_bounds__(256) sa_apply_kernel(const void* x, long long P, int HW, int C, const float* att,
                                                       const float* mul, void* out) {
  constexpr int K = Chunk<T>::N;
  const int nch = C / K;
  const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= P * nch) return;
  const long long p = gid / nch;
  const int ch = (int)(gid - p * nch);
  const float a = att[p];
  float v[K];
  Chunk<T>::unpack(reinterpret_cast<const uint4*>(x)[gid], v);
  const float* m = mul ? mul + (p / HW) * C + ch * K : nullptr;
#pragma unroll
  for (int e = 0; e < K; ++e) v[e] *= m ? a * m[e] : a;
  reinterpret_cast<uint4*>(out)[gid] = Chunk<T>::pack(v);
}

// dpre[p] = (sum_c dout*mul*x) * att * (1 - att)
template <typename T>
__global__ void __launch_bounds__(256) sa_bwd1_kernel(const void* x, const void* dout, long long P, int HW, int C,
                                                      const float* att, const float* mul, float* dpre) {
  constexpr int K = Chunk<T>::N;
  constexpr int G = 16;
  const int nch = C / K;
  const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long pix = gid / G;
  const int l = (int)(gid % G);
  float s = 0.f, v[K], g[K];
  if (pix < P) {
    const uint4* xs = reinterpret_cast<const uint4*>(x) + pix * nch;
    const uint4* ds = reinterpret_cast<const uint4*>(dout) + pix * nch;
    const float* m = mul ? mul + (pix / HW) * C : nullptr;
    for (int ch = l; ch < nch; ch += G) {
      Chunk<T>::unpack(xs[ch], v);
      Chunk<T>::unpack(ds[ch], g);
#pragma unroll
      for (int e = 0; e < K; ++e) s += g[e] * v[e] * (m ? m[ch * K + e] : 1.f);
    }
  }
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, G);
  if (pix < P && l == 0) {
    const float a = att[pix];
    dpre[pix] = s * a * (1.f - a);
  }
}

// dstats[p][c] = sum_taps w[c][ky][kx] * dpre[y - ky + r][x - kx + r]   (adjoint of the 7x7 correlation)
__global__ void __launch_bounds__(256) sa_bwd2_kernel(const float* dpre, int N, int H, int W, const float* w, int k,
                                                      float* dstats) {
  const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (long long)N * H * W) return;
  const int x = (int)(gid % W);
  const long long t = gid / W;
  const int y = (int)(t % H);
  const int n = (int)(t / H);
  const int r = k / 2;
  float a0 = 0.f, a1 = 0.f;
  for (int ky = 0; ky < k; ++ky) {
    const int yy = y - ky + r;
    if (yy < 0 || yy >= H) continue;
    for (int kx = 0; kx < k; ++kx) {
      const int xx = x - kx + r;
      if (xx < 0 || xx >= W) continue;
      const float d = dpre[((long long)n * H + yy) * W + xx];
      a0 += w[ky * k + kx] * d;
      a1 += w[(k + ky) * k + kx] * d;
    }
  }
  dstats[gid * 2] = a0;
  dstats[gid * 2 + 1] = a1;
}

// dw partial per image row: part[(n*H + y)][c*k*k + ky*k + kx] = sum_x dpre[y][x] * stats[y+ky-r][x+kx-r][c]
__global__ void __launch_bounds__(256) sa_dw_kernel(const float* dpre, const float* stats, int N, int H, int W, int k,
                                                    float* part) {
  const int row = blockIdx.x;  // n*H + y
  const int n = row / H, y = row - n * H;
  const int t = threadIdx.x;
  const int nw = 2 * k * k;
  if (t >= nw) return;
  const int c = t / (k * k), ky = (t / k) % k, kx = t % k;
  const int r = k / 2;
  const int yy = y + ky - r;
  float acc = 0.f;
  if (yy >= 0 && yy < H) {
    for (int x = 0; x < W; ++x) {
      const int xx = x + kx - r;
      if (xx < 0 || xx >= W) continue;
      acc += dpre[((long long)n * H + y) * W + x] * stats[(((long long)n * H + yy) * W + xx) * 2 + c];
    }
  }
  part[(long long)row * nw + t] = acc;
}

// out[c] (+)= sum_r part[r*ld + c], c < cols
__global__ void __launch_bounds__(128) sum_rows_kernel(const float* part, int rows, int ld, int cols, float* out, int acc) {
  const int c = blockIdx.x * 128 + threadIdx.x;
  if (c >= cols) return;
  double s = 0;
  for (int r = 0; r < rows; ++r) s += part[(long long)r * ld + c];
  out[c] = acc ? (float)(out[c] + s) : (float)s;
}

// First level of sum_rows for tall inputs: split s (rows [s*R, s*R+R)) of a 64-column tile, 4 row lanes per
// column; the split's sum overwrites its first row (read only by this block), so the second level sums
// ceil(rows/R) rows of stride R*ld.  part is scratch: its contents are consumed.
__global__ void __launch_bounds__(256) sum_rows_split_kernel(float* part, int rows, int ld, int cols, int R) {
  __shared__ double red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), lane = threadIdx.x >> 6;
  const long long r0 = (long long)blockIdx.y * R;
  const long long r1 = r0 + R < rows ? r0 + R : rows;
  double s = 0;
  if (c < cols)
    for (long long r = r0 + lane; r < r1; r += 4) s += part[r * ld + c];
  red[lane][threadIdx.x & 63] = s;
  __syncthreads();
  if (lane == 0 && c < cols)
    part[r0 * ld + c] = (float)(red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// out[c] (+)= sum_r part[r*ld + c]; consumes part (scratch) when rows > 64
static void sum_rows(float* part, int rows, int ld, int cols, float* out, int acc, hipStream_t s) {
  if (rows <= 64) {
    hipLaunchKernelGGL(sum_rows_kernel, dim3((cols + 127) / 128), dim3(128), 0, s, part, rows, ld, cols, out, acc);
    return;
  }
  int R = (rows + 63) / 64;
  R = R < 64 ? 64 : R;
  const int S = (rows + R - 1) / R;
  hipLaunchKernelGGL(sum_rows_split_kernel, dim3((cols + 63) / 64, S), dim3(256), 0, s, part, rows, ld, cols, R);
  hipLaunchKernelGGL(sum_rows_kernel, dim3((cols + 127) / 128), dim3(128), 0, s, part, S, R * ld, cols, out, acc);
}

// dx = dout*mul*att + dstats0 / C + [c == argmax] * dstats1
template <typename T>
__global__ void __launch_bounds__(256) sa_bwd3_kernel(const void* dout, long long P, int HW, int C, const float* att,
                                                      const float* mul, const float* dstats, const int* argmax, void* dx) {
  constexpr int K = Chunk<T>::N;
  const int nch = C / K;
  const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= P * nch) return;
  const long long p = gid / nch;
  const int ch = (int)(gid - p * nch);
  const float a = att[p], d0 = dstats[p * 2] / (float)C, d1 = dstats[p * 2 + 1];
  const int am = argmax[p];
  const float* m = mul ? mul + (p / HW) * C + ch * K : nullptr;
  float g[K];
  Chunk<T>::unpack(reinterpret_cast<const uint4*>(dout)[gid], g);
#pragma unroll
  for (int e = 0; e < K; ++e) {
    float v = g[e] * a * (m ? m[e] : 1.f) + d0;
    if (ch * K + e == am) v += d1;
    g[e] = v;
  }
  reinterpret_cast<uint4*>(dx)[gid] = Chunk<T>::pack(g);
}

// ======================================================================================= channel attention
// Global-average-pool partials part[n][s][c] over S pixel splits per image, S = ca_splits(N, HW) <= kGapSplits (the
// workspace size).  (Round 5: S was a fixed 16 -- N x 16 blocks, 64 for the distillation student's 4 images -- and
// channel counts whose chunk count does not divide 256 (96, 144, 240, 480, 672, 1152: most SqueezeExcite layers) took
// a one-thread-per-channel kernel with 2-byte loads: the SE forward and backward pools were most of the unfrozen
// distillation step's SE time.)
constexpr int kGapSplits = 64;

static int ca_splits(int N, int HW) {
  int s = 1024 / (N > 0 ? N : 1);
  const int cap = HW / 16 > 0 ? HW / 16 : 1;   // >= 16 pixels per split
  if (s > cap) s = cap;
  if (s > kGapSplits) s = kGapSplits;
  return s < 1 ? 1 : s;
}

// part[n][s][c] = sum_{p in split s of image n} x[p][c] (* dout[p][c] * mul[n][c] if dout).  16-B loads: 256 threads =
// R = 256 / CT pixel lanes x CT channel chunks (CT = min(nch, 256); blockIdx.z: the chunk group), lanes reduced in LDS
// in lane order.
template <typename T>
__global__ void __launch_bounds__(256) ca_gap_vec_kernel(const void* x, const void* dout, const float* mul, int HW,
                                                         int C, int S, float* part) {
  constexpr int K = Chunk<T>::N;
  __shared__ float red[256 * K];   // [R][CT * K]
  const int n = blockIdx.x, sp = blockIdx.y;
  const int nch = C / K;
  const int CT = nch < 256 ? nch : 256, R = 256 / CT;
  const int cl = threadIdx.x % CT, lane = threadIdx.x / CT;
  const int ch = blockIdx.z * 256 + cl;
  const bool live = lane < R && ch < nch;
  const int p0 = (int)((long long)HW * sp / S), p1 = (int)((long long)HW * (sp + 1) / S);
  float acc[K], v[K], g[K];
#pragma unroll
  for (int e = 0; e < K; ++e) acc[e] = 0.f;
  if (live) {
    const uint4* xs = reinterpret_cast<const uint4*>(x) + (long long)n * HW * nch + ch;
    const uint4* ds = dout ? reinterpret_cast<const uint4*>(dout) + (long long)n * HW * nch + ch : nullptr;
    for (int p = p0 + lane; p < p1; p += R) {
      Chunk<T>::unpack(xs[(long long)p * nch], v);
      if (ds) {
        Chunk<T>::unpack(ds[(long long)p * nch], g);
#pragma unroll
        for (int e = 0; e < K; ++e) v[e] *= g[e];
      }
#pragma unroll
      for (int e = 0; e < K; ++e) acc[e] += v[e];
    }
    if (ds && mul) {
#pragma unroll
      for (int e = 0; e < K; ++e) acc[e] *= mul[(long long)n * C + ch * K + e];
    }
  }
  if (lane < R) {
#pragma unroll
    for (int e = 0; e < K; ++e) red[lane * CT * K + cl * K + e] = acc[e];
  }
  __syncthreads();
  const int cols = CT * K;
  for (int c = threadIdx.x; c < cols; c += 256) {
    const int cc = blockIdx.z * 256 * K + c;
    if (cc >= C) continue;
    float s = 0.f;
    for (int l = 0; l < R; ++l) s += red[l * cols + c];
    part[((long long)n * S + sp) * C + cc] = s;
  }
}

template <typename T>
static int ca_gap(const void* x, const void* dout, const float* mul, int N, int HW, int C, float* part, hipStream_t s) {
  const int nch = C / Chunk<T>::N;
  const int S = ca_splits(N, HW);
  hipLaunchKernelGGL(ca_gap_vec_kernel<T>, dim3(N, S, (nch + 255) / 256), dim3(256), 0, s, x, dout, mul, HW, C, S, part);
  return S;
}

__device__ __forceinline__ float act_f(float v, int act, float beta) { return apply_act(v, act, beta); }
__device__ __forceinline__ float act_d(float pre, int act, float beta) { return act_grad_pre(pre, act, beta); }

// out = x * gate[n][c] * mul[n][c]   (NHWC, C channels contiguous).  Block = (256 / nch) pixel lanes x nch
// channel chunks over a pixel range of image blockIdx.y (blockIdx.x = range): the chunk's gate factors stay
// in registers across the thread's pixels.  Falls back to one chunk per thread when nch does not divide 256.
static unsigned ca_ranges(int N, int HW) {   // pixel ranges per image: ~8k blocks, >= 64 pixels per range
  long long r = (8192 + N - 1) / N;
  const long long cap = HW / 64 > 0 ? HW / 64 : 1;
  if (r > cap) r = cap;
  return (unsigned)(r < 1 ? 1 : (r > 65535 ? 65535 : r));
}

template <typename T>
__global__ void __launch_bounds__(256) ca_apply_kernel(const void* x, int N, int HW, int C, const float* gate,
                                                       const float* mul, void* out) {
  constexpr int K = Chunk<T>::N;
  const int nch = C / K;
  const long long n = blockIdx.y;
  if (nch <= 256 && 256 % nch == 0) {
    const int R = 256 / nch, ch = threadIdx.x % nch, lane = threadIdx.x / nch;
    float g[K];
#pragma unroll
    for (int e = 0; e < K; ++e) g[e] = gate[n * C + ch * K + e] * (mul ? mul[n * C + ch * K + e] : 1.f);
    const int p0 = (int)((long long)HW * blockIdx.x / gridDim.x), p1 = (int)((long long)HW * (blockIdx.x + 1) / gridDim.x);
    const uint4* xs = reinterpret_cast<const uint4*>(x) + n * HW * nch + ch;
    uint4* os = reinterpret_cast<uint4*>(out) + n * HW * nch + ch;
    for (int p = p0 + lane; p < p1; p += R) {
      float v[K];
      Chunk<T>::unpack(xs[(long long)p * nch], v);
#pragma unroll
      for (int e = 0; e < K; ++e) v[e] *= g[e];
      os[(long long)p * nch] = Chunk<T>::pack(v);
    }
    return;
  }
  for (int li = blockIdx.x * 256 + threadIdx.x; li < HW * nch; li += gridDim.x * 256) {
    const int ch = li % nch;
    const long long gid = n * HW * nch + li;
    float v[K];
    Chunk<T>::unpack(reinterpret_cast<const uint4*>(x)[gid], v);
    const float* gg = gate + n * C + ch * K;
    const float* m = mul ? mul + n * C + ch * K : nullptr;
#pragma unroll
    for (int e = 0; e < K; ++e) v[e] *= gg[e] * (m ? m[e] : 1.f);
    reinterpret_cast<uint4*>(out)[gid] = Chunk<T>::pack(v);
  }
}

// per image: ds = dgate * g (1-g); dh; dgap; per-image weight-gradient rows
// The channel-attention / SqueezeExcite MLP over the pooled vector, as three wide launches (round 5: one block per
// image did it all -- 4 blocks for the distillation student's SE layers, 45 us forward / 66 us backward per call):
//   colsum:  out[n][c] = (sum_k part[n][k][c]) * HW^-1 (forward: the pool)  or  * g (1 - g) (backward: ds)
//   rowdot:  one 32-lane group per (n, r): s = sum_c W[r ldr + c ldc] v[n][c] (lane-strided, butterfly-reduced)
//            forward: hpre = s + b1, h = act(hpre);  backward: dh = s * act'(hpre)
//   coldot:  one thread per (n, c): s = sum_r W[c ldc + r ldr] v[n][r]
//            forward: gate = sigmoid(s + b2);  backward: dgap = s
__global__ void __launch_bounds__(256) ca_colsum_kernel(const float* part, int S, int C, float inv_hw, const float* gate,
                                                        float* out, int out_ld, int out_off, float* out2) {
  const int n = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const float* p = part + (long long)n * S * C + c;
  float s = 0.f;
  int k = 0;
  for (; k + 3 < S; k += 4) {
    const float a0 = p[(long long)k * C], a1 = p[(long long)(k + 1) * C], a2 = p[(long long)(k + 2) * C],
                a3 = p[(long long)(k + 3) * C];
    s += a0; s += a1; s += a2; s += a3;
  }
  for (; k < S; ++k) s += p[(long long)k * C];
  float v;
  if (gate) {
    const float g = gate[(long long)n * C + c];
    v = s * g * (1.f - g);
  } else {
    v = s * inv_hw;
  }
  out[(long long)n * out_ld + out_off + c] = v;
  if (out2) out2[(long long)n * C + c] = v;
}

__global__ void __launch_bounds__(256) ca_rowdot_kernel(const float* W, long long ldr, long long ldc, const float* v,
                                                        int v_ld, int v_off, int C, int Cr, const float* b1, int act,
                                                        float beta, float* hpre, float* out, int out_ld, int fwd) {
  const int n = blockIdx.y, r = blockIdx.x * 8 + (threadIdx.x >> 5), l = threadIdx.x & 31;
  float s = 0.f;
  if (r < Cr) {
    const float* vv = v + (long long)n * v_ld + v_off;
    for (int c = l; c < C; c += 32) s += W[r * ldr + c * ldc] * vv[c];
  }
#pragma unroll
  for (int m = 16; m > 0; m >>= 1) s += __shfl_xor(s, m, 64);
  if (l == 0 && r < Cr) {
    if (fwd) {
      const float pre = s + (b1 ? b1[r] : 0.f);
      hpre[(long long)n * Cr + r] = pre;
      out[(long long)n * out_ld + r] = act_f(pre, act, beta);
    } else {
      out[(long long)n * out_ld + r] = s * act_d(hpre[(long long)n * Cr + r], act, beta);
    }
  }
}

__global__ void __launch_bounds__(256) ca_coldot_kernel(const float* W, long long ldc, long long ldr, const float* v,
                                                        int v_ld, int C, int Cr, const float* b2, int fwd, float* out) {
  const int n = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const float* vv = v + (long long)n * v_ld;
  float s = 0.f;
  for (int r = 0; r < Cr; ++r) s += W[c * ldc + r * ldr] * vv[r];
  out[(long long)n * C + c] = fwd ? sigmoidf_(s + (b2 ? b2[c] : 0.f)) : s;
}

// forward: gap [N][C], hpre [N][Cr], gate [N][C]; h [N][Cr] in scratch
static void ca_mlp_fwd(const float* part, int S, int N, int HW, int C, int Cr, const float* w1, const float* w2, int act,
                       float beta, float* gap, float* hpre, float* gate, const float* b1, const float* b2, float* h,
                       hipStream_t s) {
  const dim3 cg((C + 255) / 256, N), rg((Cr + 7) / 8, N);
  hipLaunchKernelGGL(ca_colsum_kernel, cg, dim3(256), 0, s, part, S, C, 1.f / (float)HW, nullptr, gap, C, 0, nullptr);
  hipLaunchKernelGGL(ca_rowdot_kernel, rg, dim3(256), 0, s, w1, (long long)C, 1ll, gap, C, 0, C, Cr, b1, act, beta, hpre,
                     h, Cr, 1);
  hipLaunchKernelGGL(ca_coldot_kernel, cg, dim3(256), 0, s, w2, (long long)Cr, 1ll, h, Cr, C, Cr, b2, 1, gate);
}

// backward: sd [N][Cr + C] = (dh, ds), dgap [N][C]
static void ca_mlp_bwd(const float* part, int S, int N, int C, int Cr, const float* w1, const float* w2, int act,
                       float beta, const float* hpre, const float* gate, float* dgap, float* sd, hipStream_t s) {
  const dim3 cg((C + 255) / 256, N), rg((Cr + 7) / 8, N);
  hipLaunchKernelGGL(ca_colsum_kernel, cg, dim3(256), 0, s, part, S, C, 0.f, gate, sd, Cr + C, Cr, nullptr);
  hipLaunchKernelGGL(ca_rowdot_kernel, rg, dim3(256), 0, s, w2, 1ll, (long long)Cr, sd, Cr + C, Cr, C, Cr, nullptr, act,
                     beta, const_cast<float*>(hpre), sd, Cr + C, 0);
  hipLaunchKernelGGL(ca_coldot_kernel, cg, dim3(256), 0, s, w1, 1ll, (long long)C, sd, Cr + C, C, Cr, nullptr, 0, dgap);
}

// dW1[r][c] += sum_n dh[n][r] gap[n][c]; dW2[c][r] += sum_n ds[n][c] act(hpre[n][r]); db1 += sum_n dh; db2 += sum_n ds
// (images in order).  One thread per output element over many blocks -- the per-image rows were written by one block
// per image and summed by four more launches (the distillation student's SE layers: 4 blocks for up to 2 x 55 k
// outputs).
__global__ void __launch_bounds__(256) ca_wgrad_kernel(int N, int C, int Cr, const float* sd, const float* gap,
                                                       const float* hpre, int act, float beta, float* dw1, float* dw2,
                                                       float* db1, float* db2) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long n1 = (long long)C * Cr;
  const int ld = Cr + C;
  if (i < n1) {
    const int r = (int)(i / C), c = (int)(i - (long long)r * C);
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += sd[(long long)n * ld + r] * gap[(long long)n * C + c];
    dw1[i] += s;
  } else if (i < 2 * n1) {
    const long long j = i - n1;
    const int c = (int)(j / Cr), r = (int)(j - (long long)c * Cr);
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += sd[(long long)n * ld + Cr + c] * act_f(hpre[(long long)n * Cr + r], act, beta);
    dw2[j] += s;
  } else if (i < 2 * n1 + Cr) {
    const int r = (int)(i - 2 * n1);
    if (db1) {
      float s = 0.f;
      for (int n = 0; n < N; ++n) s += sd[(long long)n * ld + r];
      db1[r] += s;
    }
  } else if (i < 2 * n1 + Cr + C) {
    const int c = (int)(i - 2 * n1 - Cr);
    if (db2) {
      float s = 0.f;
      for (int n = 0; n < N; ++n) s += sd[(long long)n * ld + Cr + c];
      db2[c] += s;
    }
  }
}

static void ca_wgrad(int N, int C, int Cr, const float* sd, const float* gap, const float* hpre, int act, float beta,
                     float* dw1, float* dw2, float* db1, float* db2, hipStream_t s) {
  const long long n = 2ll * C * Cr + Cr + C;
  hipLaunchKernelGGL(ca_wgrad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, N, C, Cr, sd, gap, hpre, act,
                     beta, dw1, dw2, db1, db2);
}

// dx = dout*mul*gate + dgap/HW, same block layout as ca_apply_kernel
template <typename T>
__global__ void __launch_bounds__(256) ca_dx_kernel(const void* dout, int N, int HW, int C, const float* gate,
                                                    const float* mul, const float* dgap, void* dx) {
  constexpr int K = Chunk<T>::N;
  const int nch = C / K;
  const long long n = blockIdx.y;
  const float inv = 1.f / (float)HW;
  if (nch <= 256 && 256 % nch == 0) {
    const int R = 256 / nch, ch = threadIdx.x % nch, lane = threadIdx.x / nch;
    float g[K], d[K];
#pragma unroll
    for (int e = 0; e < K; ++e) {
      const long long i = n * C + ch * K + e;
      g[e] = gate[i] * (mul ? mul[i] : 1.f);
      d[e] = dgap[i] * inv;
    }
    const int p0 = (int)((long long)HW * blockIdx.x / gridDim.x), p1 = (int)((long long)HW * (blockIdx.x + 1) / gridDim.x);
    const uint4* ds = reinterpret_cast<const uint4*>(dout) + n * HW * nch + ch;
    uint4* os = reinterpret_cast<uint4*>(dx) + n * HW * nch + ch;
    for (int p = p0 + lane; p < p1; p += R) {
      float v[K];
      Chunk<T>::unpack(ds[(long long)p * nch], v);
#pragma unroll
      for (int e = 0; e < K; ++e) v[e] = v[e] * g[e] + d[e];
      os[(long long)p * nch] = Chunk<T>::pack(v);
    }
    return;
  }
  for (int li = blockIdx.x * 256 + threadIdx.x; li < HW * nch; li += gridDim.x * 256) {
    const int ch = li % nch;
    const long long gid = n * HW * nch + li;
    float v[K];
    Chunk<T>::unpack(reinterpret_cast<const uint4*>(dout)[gid], v);
#pragma unroll
    for (int e = 0; e < K; ++e) {
      const long long i = n * C + ch * K + e;
      v[e] = v[e] * gate[i] * (mul ? mul[i] : 1.f) + dgap[i] * inv;
    }
    reinterpret_cast<uint4*>(dx)[gid] = Chunk<T>::pack(v);
  }
}

// ======================================================================================= upsample_bg_fg + combine
struct UbfArgs {
  const float* low; int N, h, w;
  const float* ut_w; const float* ut_b;     // ConvT [2][32][2][2], bias [32]
  const float* scale; const float* shift;   // norm fold: a = act(z*scale + shift); [32] (BN) or [N][32] (LN)
  const float* mean; const float* invstd; const float* gamma;   // [32] (BN) or [N] (LN)
  const float* u1_w; const float* u1_b;     // [2][32], [2]
  int act; float beta; int ln;
};

__device__ __forceinline__ float ubf_z(const UbfArgs& u, float l0, float l1, int c, int q) {
  return l0 * u.ut_w[(c * 2 + (q >> 1)) * 2 + (q & 1)] + l1 * u.ut_w[((32 + c) * 2 + (q >> 1)) * 2 + (q & 1)] + u.ut_b[c];
}

// BN statistics of z = ConvT(low) over all N*2h*2w pixels: partial [S][3][32] (Welford), block = 8 rows x 32 ch
__global__ void __launch_bounds__(256) ubf_stats_kernel(UbfArgs u, float* partial) {
  __shared__ float sn[256], sm[256], sq[256];
  const int t = threadIdx.x, c = t & 31, r = t >> 5;
  const long long P = (long long)u.N * u.h * u.w;
  const long long b = P * blockIdx.x / gridDim.x, e = P * (blockIdx.x + 1) / gridDim.x;
  float n = 0.f, mean = 0.f, m2 = 0.f;
  for (long long p = b + r; p < e; p += 8) {
    const float l0 = u.low[p * 2], l1 = u.low[p * 2 + 1];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float x = ubf_z(u, l0, l1, c, q);
      n += 1.f;
      const float d = x - mean;
      mean += d / n;
      m2 += d * (x - mean);
    }
  }
  sn[t] = n; sm[t] = mean; sq[t] = m2;
  __syncthreads();
  if (r == 0) {
    for (int rr = 1; rr < 8; ++rr) {
      const int o = rr * 32 + c;
      const float nb2 = sn[o];
      if (nb2 == 0.f) continue;
      const float nt = n + nb2, d = sm[o] - mean;
      mean += d * (nb2 / nt);
      m2 += sq[o] + d * d * (n * nb2 / nt);
      n = nt;
    }
    float* out = partial + (long long)blockIdx.x * 96;
    out[c] = n; out[32 + c] = mean; out[64 + c] = m2;
  }
}

// per mask pixel: bg/fg logits, target logits (fused Ct->2 1x1), softmax, hierarchical combine
template <typename T>
__global__ void __launch_bounds__(256) ubf_fwd_kernel(UbfArgs u, const void* tfeat, int Ct, const float* t_w,
                                                      const float* t_b, float* logits, float* bgfg, float* tn) {
  __shared__ float s_tw[2 * 512];
  for (int i = threadIdx.x; i < 2 * Ct; i += 256) s_tw[i] = t_w[i];
  __syncthreads();
  const int H = 2 * u.h, W = 2 * u.w;
  const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (long long)u.N * H * W) return;
  const int X = (int)(gid % W);
  const long long tt = gid / W;
  const int Y = (int)(tt % H);
  const int n = (int)(tt / H);
  const int q = (Y & 1) * 2 + (X & 1);
  const float* lo = u.low + (((long long)n * u.h + (Y >> 1)) * u.w + (X >> 1)) * 2;
  const float l0 = lo[0], l1 = lo[1];
  float b0 = u.u1_b[0], b1 = u.u1_b[1];
  const float* sc = u.scale + (u.ln ? n * 32 : 0);
  const float* sh = u.shift + (u.ln ? n * 32 : 0);
  for (int c = 0; c < 32; ++c) {
    const float a = apply_act(ubf_z(u, l0, l1, c, q) * sc[c] + sh[c], u.act, u.beta);
    b0 += u.u1_w[c] * a;
    b1 += u.u1_w[32 + c] * a;
  }
  constexpr int K = Chunk<T>::N;
  float t0 = t_b[0], t1 = t_b[1], v[K];
  const uint4* tf = reinterpret_cast<const uint4*>(tfeat) + gid * (Ct / K);
  for (int ch = 0; ch < Ct / K; ++ch) {
    Chunk<T>::unpack(tf[ch], v);
#pragma unroll
    for (int e = 0; e < K; ++e) {
      t0 += s_tw[ch * K + e] * v[e];
      t1 += s_tw[Ct + ch * K + e] * v[e];
    }
  }
  const float mx = fmaxf(b0, b1);
  const float e0 = __expf(b0 - mx), e1 = __expf(b1 - mx);
  const float pf = e1 / (e0 + e1);
  const long long plane = (long long)H * W, pp = (long long)Y * W + X;
  float* L = logits + (long long)n * 3 * plane + pp;
  L[0] = b0;
  L[plane] = b1 + t0 * pf;
  L[2 * plane] = b1 + t1 * pf;
  float* G = bgfg + (long long)n * 2 * plane + pp;
  G[0] = b0; G[plane] = b1;
  float* Tn = tn + (long long)n * 2 * plane + pp;
  Tn[0] = t0; Tn[plane] = t1;
}

// pass 1 (8 pixel rows x 32 channels per block): combine backward -> db, dtn per pixel (written by c == 0);
// per channel: sum g, sum g*xhat, sum xhat (BN bwd), dW1[k][c] = sum db_k * a_c; db1.
// partial layout per block: [32 g][32 gx][32 x][64 dW1][2 db1]  (162)
// LayerNorm (u.ln): sb blocks per sample, block j of sample n covers a slice of that sample only, so the
// per-block channel sums add up to per-(sample, channel) sums.
template <bool U2>
__global__ void __launch_bounds__(256) ubf_bwd1_kernel(UbfArgs u, const float* dlogits, const float* dbgfg_ext,
                                                       const float* dtn_ext, const float* bgfg, const float* tn,
                                                       float* db_out, float* dtn_out, float* partial, int sb) {
  __shared__ float red[8][162];
  const int t = threadIdx.x, c = t & 31, r = t >> 5;
  const int H = 2 * u.h, W = 2 * u.w;
  const long long P = (long long)u.N * H * W, plane = (long long)H * W;
  long long b, e;
  int ns = 0;
  if (u.ln) {
    ns = blockIdx.x / sb;
    const int j = blockIdx.x % sb;
    b = ns * plane + plane * j / sb;
    e = ns * plane + plane * (j + 1) / sb;
  } else {
    b = P * blockIdx.x / gridDim.x;
    e = P * (blockIdx.x + 1) / gridDim.x;
  }
  const float mu = u.ln ? u.mean[ns] : u.mean[c], inv = u.ln ? u.invstd[ns] : u.invstd[c];
  const float scc = u.ln ? u.scale[ns * 32 + c] : u.scale[c], shc = u.ln ? u.shift[ns * 32 + c] : u.shift[c];
  const float w0 = u.u1_w[c], w1 = u.u1_w[32 + c];
  // the thread's ConvTranspose weights for the 4 sub-pixels and its bias, loaded once (U2; the U1 form re-reads them
  // per pixel through ubf_z: the stores below may alias them as far as the compiler knows)
  float zw0[4], zw1[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    zw0[q] = u.ut_w[(c * 2 + (q >> 1)) * 2 + (q & 1)];
    zw1[q] = u.ut_w[((32 + c) * 2 + (q >> 1)) * 2 + (q & 1)];
  }
  const float zb = u.ut_b[c];
  float sg = 0.f, sgx = 0.f, sx = 0.f, dw0 = 0.f, dw1 = 0.f, db0s = 0.f, db1s = 0.f;
  // (n, Y, X) of p advanced incrementally by the row stride 8: the 64-bit div / mod per pixel dominated the loop
  int X, Y;
  long long n;
  {
    const long long p0 = b + r, tt = p0 / W;
    X = (int)(p0 - tt * W);
    Y = (int)(tt % H);
    n = tt / H;
  }
  struct In { float g0, g1, t0, t1, dL0, dL1, dL2, e0, e1, f0, f1, l0, l1; long long pp, n; int X, Y; };
  auto load = [&](long long nn, int YY, int XX) __attribute__((always_inline)) -> In {
    In v;
    const long long pp = (long long)YY * W + XX;
    const float* G = bgfg + nn * 2 * plane + pp;
    const float* Tn = tn + nn * 2 * plane + pp;
    const float* dL = dlogits + nn * 3 * plane + pp;
    v.g0 = G[0]; v.g1 = G[plane]; v.t0 = Tn[0]; v.t1 = Tn[plane];
    v.dL0 = dL[0]; v.dL1 = dL[plane]; v.dL2 = dL[2 * plane];
    v.e0 = dbgfg_ext ? dbgfg_ext[nn * 2 * plane + pp] : 0.f;
    v.e1 = dbgfg_ext ? dbgfg_ext[nn * 2 * plane + plane + pp] : 0.f;
    v.f0 = dtn_ext ? dtn_ext[nn * 2 * plane + pp] : 0.f;
    v.f1 = dtn_ext ? dtn_ext[nn * 2 * plane + plane + pp] : 0.f;
    const float* lo = u.low + ((nn * u.h + (YY >> 1)) * u.w + (XX >> 1)) * 2;
    v.l0 = lo[0]; v.l1 = lo[1];
    v.pp = pp; v.n = nn; v.X = XX; v.Y = YY;
    return v;
  };
  auto body = [&](const In& v, long long p) __attribute__((always_inline)) {
    const float mx = fmaxf(v.g0, v.g1);
    const float ex0 = __expf(v.g0 - mx), ex1 = __expf(v.g1 - mx);
    const float pf = ex1 / (ex0 + ex1);
    const float dpf = v.dL1 * v.t0 + v.dL2 * v.t1;
    const float dsg = dpf * pf * (1.f - pf);
    float db0 = v.dL0 - dsg, db1 = v.dL1 + v.dL2 + dsg;
    float dt0 = v.dL1 * pf, dt1 = v.dL2 * pf;
    if (dbgfg_ext) { db0 += v.e0; db1 += v.e1; }
    if (dtn_ext) { dt0 += v.f0; dt1 += v.f1; }
    if (c == 0) {
      db_out[p * 2] = db0; db_out[p * 2 + 1] = db1;
      dtn_out[p * 2] = dt0; dtn_out[p * 2 + 1] = dt1;
      db0s += db0; db1s += db1;
    }
    const int q = (v.Y & 1) * 2 + (v.X & 1);
    const float z = U2 ? v.l0 * zw0[q] + v.l1 * zw1[q] + zb : ubf_z(u, v.l0, v.l1, c, q);
    const float pre = z * scc + shc;
    const float a = apply_act(pre, u.act, u.beta);
    const float g = (w0 * db0 + w1 * db1) * act_grad_pre(pre, u.act, u.beta);
    const float xh = (z - mu) * inv;
    sg += g; sgx += g * xh; sx += xh;
    dw0 += db0 * a; dw1 += db1 * a;
  };
  auto step = [&]() __attribute__((always_inline)) {
    X += 8;
    while (X >= W) {
      X -= W;
      if (++Y == H) { Y = 0; ++n; }
    }
  };
  long long p = b + r;
  while (X >= W) {   // (b + r may start past a row end only through the initial decomposition: never; kept for form)
    X -= W;
    if (++Y == H) { Y = 0; ++n; }
  }
  if (U2) {
    // two pixels per iteration, both pixels' loads issued before either's arithmetic; the sums in pixel order
    for (; p + 8 < e; p += 16) {
      const In va = load(n, Y, X);
      step();
      const In vb = load(n, Y, X);
      step();
      body(va, p);
      body(vb, p + 8);
    }
  }
  for (; p < e; p += 8) {
    const In va = load(n, Y, X);
    step();
    body(va, p);
  }
  red[r][c] = sg; red[r][32 + c] = sgx; red[r][64 + c] = sx; red[r][96 + c] = dw0; red[r][128 + c] = dw1;
  if (c == 0) { red[r][160] = db0s; red[r][161] = db1s; }
  __syncthreads();
  if (t < 162) {
    float s = 0.f;
    for (int rr = 0; rr < 8; ++rr) s += red[rr][t];
    partial[(long long)blockIdx.x * 162 + t] = s;
  }
}

// finalize 1: BN coefficients + dgamma/dbeta/dW1/db1 (accumulate into the parameter gradients)
// coef: [32 k][32 mean g][32 mean gx]
__global__ void ubf_fin1_kernel(UbfArgs u, const float* partial, int nblk, long long P, float* coef, float* dgamma,
                                float* dbeta, float* du1_w, float* du1_b, float* dut_b_analytic) {
  const int t = threadIdx.x;
  if (t >= 162) return;
  // 8 independent partial sums, 16 loads in flight per thread: the serial dependent loop over 2048 block rows
  // was latency-bound (0.5 ms for one 192-thread block)
  double s8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int b = 0;
  for (; b + 16 <= nblk; b += 16) {
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = partial[(long long)(b + i) * 162 + t];
#pragma unroll
    for (int i = 0; i < 16; ++i) s8[i & 7] += v[i];
  }
  for (; b < nblk; ++b) s8[0] += partial[(long long)b * 162 + t];
  const double s = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
  __shared__ double S[162];
  S[t] = s;
  __syncthreads();
  if (t < 32) {
    const double k = u.ln ? 0.0 : (u.gamma ? u.gamma[t] : 1.0) * u.invstd[t];   // BN coefficients only
    coef[t] = (float)k;
    coef[32 + t] = (float)(S[t] / P);
    coef[64 + t] = (float)(S[32 + t] / P);
    dgamma[t] += (float)S[32 + t];
    dbeta[t] += (float)S[t];
    if (dut_b_analytic) dut_b_analytic[t] += (float)(k * (S[t] - P * (S[t] / P) - S[64 + t] * (S[32 + t] / P)));
  }
  if (t >= 96 && t < 160) du1_w[t - 96] += (float)S[t];
  if (t >= 160) du1_b[t - 160] += (float)S[t];
}

// LayerNorm finalize (grid N, 32 lanes): the sample's sb block partials -> G, GX, X per channel,
// coef_ln[n] = (a_n, b_n), dbias[n][c] = invstd_n (gamma_c G - HWm a_n - X b_n) (the ConvTranspose bias gradient)
__global__ void ubf_ln_fin_kernel(UbfArgs u, const float* partial, int sb, float* coef_ln, float* dbias) {
  __shared__ float sa[32], sbb[32];
  const int n = blockIdx.x, c = threadIdx.x;
  double G = 0, GX = 0, X = 0;
  for (int j = 0; j < sb; ++j) {
    const float* q = partial + ((long long)n * sb + j) * 162;
    G += q[c]; GX += q[32 + c]; X += q[64 + c];
  }
  const float gam = u.gamma ? u.gamma[c] : 1.f;
  sa[c] = (float)(gam * G); sbb[c] = (float)(gam * GX);
  __syncthreads();
  double A = 0, B = 0;
  for (int i = 0; i < 32; ++i) { A += sa[i]; B += sbb[i]; }
  const double HWm = 4.0 * u.h * u.w, M = 32.0 * HWm;
  const double an = A / M, bn = B / M;
  if (c == 0) { coef_ln[n * 2] = (float)an; coef_ln[n * 2 + 1] = (float)bn; }
  dbias[n * 32 + c] = (float)(u.invstd[n] * (gam * G - HWm * an - X * bn));
}

// pass 2 (per low pixel, 8 rows x 32 channels): dz of the 4 children, dlow, dWt partial [ci][c][q] (256)
// LayerNorm: coef_ln [N][2] = (a_n, b_n); dz = invstd_n * (gamma_c g - a_n - xhat b_n)
__global__ void __launch_bounds__(256) ubf_bwd2_kernel(UbfArgs u, const float* db_in, const float* coef,
                                                       const float* coef_ln, float* dlow, float* partial) {
  __shared__ float red[8][256];
  const int t = threadIdx.x, c = t & 31, r = t >> 5;
  const long long PL = (long long)u.N * u.h * u.w;
  const long long b = PL * blockIdx.x / gridDim.x, e = PL * (blockIdx.x + 1) / gridDim.x;
  const float k = u.ln ? 0.f : coef[c], m1 = u.ln ? 0.f : coef[32 + c], m2 = u.ln ? 0.f : coef[64 + c];
  const float gam = u.gamma ? u.gamma[c] : 1.f;
  const float w0 = u.u1_w[c], w1 = u.u1_w[32 + c];
  const int W = 2 * u.w;
  float dw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) dw[i] = 0.f;
  int x, y;
  long long n;
  {
    const long long p0 = b + r, tt = p0 / u.w;
    x = (int)(p0 - tt * u.w);
    y = (int)(tt % u.h);
    n = tt / u.h;
  }
  for (long long p = b + r; p < e; p += 8, x += 8) {
    while (x >= u.w) {
      x -= u.w;
      if (++y == u.h) { y = 0; ++n; }
    }
    const float l0 = u.low[p * 2], l1 = u.low[p * 2 + 1];
    const float mu = u.ln ? u.mean[n] : u.mean[c], inv = u.ln ? u.invstd[n] : u.invstd[c];
    const float scc = u.ln ? u.scale[n * 32 + c] : u.scale[c], shc = u.ln ? u.shift[n * 32 + c] : u.shift[c];
    float dl0 = 0.f, dl1 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long long P = (n * (2 * u.h) + 2 * y + (q >> 1)) * W + 2 * x + (q & 1);
      const float z = ubf_z(u, l0, l1, c, q);
      const float pre = z * scc + shc;
      const float g = (w0 * db_in[P * 2] + w1 * db_in[P * 2 + 1]) * act_grad_pre(pre, u.act, u.beta);
      const float dz = u.ln ? inv * (gam * g - coef_ln[n * 2] - (z - mu) * inv * coef_ln[n * 2 + 1])
                            : k * (g - m1 - (z - mu) * inv * m2);
      const float wa = u.ut_w[(c * 2 + (q >> 1)) * 2 + (q & 1)];
      const float wb = u.ut_w[((32 + c) * 2 + (q >> 1)) * 2 + (q & 1)];
      dl0 += wa * dz;
      dl1 += wb * dz;
      dw[q] += l0 * dz;
      dw[4 + q] += l1 * dz;
    }
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) {
      dl0 += __shfl_xor(dl0, off, 32);
      dl1 += __shfl_xor(dl1, off, 32);
    }
    if (c == 0) { dlow[p * 2] = dl0; dlow[p * 2 + 1] = dl1; }
  }
  // layout [ci][c][q] -> index (ci*32 + c)*4 + q
#pragma unroll
  for (int q = 0; q < 4; ++q) { red[r][(0 * 32 + c) * 4 + q] = dw[q]; red[r][(1 * 32 + c) * 4 + q] = dw[4 + q]; }
  __syncthreads();
  float s = 0.f;
  for (int rr = 0; rr < 8; ++rr) s += red[rr][t];
  partial[(long long)blockIdx.x * 256 + t] = s;
}

// ======================================================================================= last 1x1 (Ct -> 2) backward
// dt[p][c] = sum_k dtn[p][k] * w[k][c]; dW[k][c] = sum_p dtn[p][k] * t[p][c]; db[k] = sum_p dtn[p][k]
// block: 16 pixel rows x (Ct/K) chunk lanes
template <typename T>
__global__ void __launch_bounds__(256) pw2_bwd_kernel(const void* tfeat, long long P, int Ct, const float* dtn,
                                                      const float* w, void* dt, float* partial) {
  constexpr int K = Chunk<T>::N;
  extern __shared__ float red[];  // [R][2*Ct + 2]
  const int nch = Ct / K;
  const int R = 256 / nch;
  const int t = threadIdx.x, ch = t % nch, r = t / nch;
  const long long b = P * blockIdx.x / gridDim.x, e = P * (blockIdx.x + 1) / gridDim.x;
  float a0[K], a1[K], v[K], wk0[K], wk1[K];
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int i = 0; i < K; ++i) { a0[i] = 0.f; a1[i] = 0.f; wk0[i] = w[ch * K + i]; wk1[i] = w[Ct + ch * K + i]; }
  if (r < R) {
    for (long long p = b + r; p < e; p += R) {
      const float d0 = dtn[p * 2], d1 = dtn[p * 2 + 1];
      Chunk<T>::unpack(reinterpret_cast<const uint4*>(tfeat)[p * nch + ch], v);
      float o[K];
#pragma unroll
      for (int i = 0; i < K; ++i) {
        a0[i] += d0 * v[i];
        a1[i] += d1 * v[i];
        o[i] = d0 * wk0[i] + d1 * wk1[i];
      }
      reinterpret_cast<uint4*>(dt)[p * nch + ch] = Chunk<T>::pack(o);
      if (ch == 0) { s0 += d0; s1 += d1; }
    }
  }
  const int cols = 2 * Ct + 2;
  if (r < R) {
#pragma unroll
    for (int i = 0; i < K; ++i) { red[r * cols + ch * K + i] = a0[i]; red[r * cols + Ct + ch * K + i] = a1[i]; }
    if (ch == 0) { red[r * cols + 2 * Ct] = s0; red[r * cols + 2 * Ct + 1] = s1; }
  }
  __syncthreads();
  for (int i = t; i < cols; i += 256) {
    float s = 0.f;
    for (int rr = 0; rr < R; ++rr) s += red[rr * cols + i];
    partial[(long long)blockIdx.x * cols + i] = s;
  }
}

}  // namespace hiseg

using namespace hiseg;

#define DISPATCH_T(dtype, ...)        \
  do {                                \
    if ((dtype) == HISEG_BF16) {      \
      using T = bf16_t;               \
      __VA_ARGS__;                    \
    } else {                          \
      using T = float;                \
      __VA_ARGS__;                    \
    }                                 \
  } while (0)

static int chunk_of(int dtype) { return dtype == HISEG_BF16 ? 8 : 4; }

// train_norm.hip: the BatchNorm statistics merge over an explicit split count
int bn_finalize_splits(const float* partial, int S, int C, long long P, const float* gamma, const float* beta,
                       float eps, float momentum, float* running_mean, float* running_var, float* mean, float* invstd,
                       float* scale, float* shift, hipStream_t stream, long long rs = 0);

extern "C" int hiseg_attn_spatial_train_fwd(int dtype, const void* x, int N, int H, int W, int C, const float* w7, int k,
                                            const float* chan_mul, float* stats, int* argmax, float* att, void* out,
                                            hiseg_stream_t stream) {
  HISEG_REQUIRE(x && w7 && stats && argmax && att && out && N > 0 && H > 0 && W > 0 && (k & 1), HISEG_ERR_BAD_ARG,
                "attn_spatial_train_fwd: bad args");
  HISEG_REQUIRE(C > 0 && C % chunk_of(dtype) == 0, HISEG_ERR_BAD_SHAPE, "attn_spatial_train_fwd: C alignment");
  hipStream_t s = (hipStream_t)stream;
  const long long P = (long long)N * H * W;
  DISPATCH_T(dtype, hipLaunchKernelGGL(sa_stats_kernel<T>, dim3(nb(P * 16, 256)), dim3(256), 0, s, x, P, C, stats, argmax));
  hipLaunchKernelGGL(sa_map_kernel, dim3(nb(P, 256)), dim3(256), 0, s, stats, N, H, W, w7, k, att);
  DISPATCH_T(dtype, hipLaunchKernelGGL(sa_apply_kernel<T>, dim3(nb(P * (C / chunk_of(dtype)), 256)), dim3(256), 0, s, x,
                                       P, H * W, C, att, chan_mul, out));
  return hiseg_check_launch("attn_spatial_train_fwd");
}

extern "C" int hiseg_attn_spatial_ws(int N, int H, int W, int k) {
  // floats: dpre [P] + dstats [2P] + dw partial [N*H][2k^2]
  const long long P = (long long)N * H * W;
  return (int)(3 * P + (long long)N * H * 2 * k * k);
}

extern "C" int hiseg_attn_spatial_bwd(int dtype, const void* x, int N, int H, int W, int C, const float* w7, int k,
                                      const float* chan_mul, const float* stats, const int* argmax, const float* att,
                                      const void* dout, void* dx, float* ws, float* dw7, hiseg_stream_t stream) {
  HISEG_REQUIRE(x && w7 && stats && argmax && att && dout && dx && ws && dw7, HISEG_ERR_BAD_ARG, "attn_spatial_bwd: null");
  HISEG_REQUIRE(C > 0 && C % chunk_of(dtype) == 0 && (k & 1) && 2 * k * k <= 256, HISEG_ERR_BAD_SHAPE,
                "attn_spatial_bwd: shape");
  hipStream_t s = (hipStream_t)stream;
  const long long P = (long long)N * H * W;
  float* dpre = ws;
  float* dstats = ws + P;
  float* part = ws + 3 * P;
  DISPATCH_T(dtype, hipLaunchKernelGGL(sa_bwd1_kernel<T>, dim3(nb(P * 16, 256)), dim3(256), 0, s, x, dout, P, H * W, C,
                                       att, chan_mul, dpre));
  hipLaunchKernelGGL(sa_bwd2_kernel, dim3(nb(P, 256)), dim3(256), 0, s, dpre, N, H, W, w7, k, dstats);
  hipLaunchKernelGGL(sa_dw_kernel, dim3(N * H), dim3(256), 0, s, dpre, stats, N, H, W, k, part);
  sum_rows(part, N * H, 2 * k * k, 2 * k * k, dw7, 1, s);
  DISPATCH_T(dtype, hipLaunchKernelGGL(sa_bwd3_kernel<T>, dim3(nb(P * (C / chunk_of(dtype)), 256)), dim3(256), 0, s,
                                       dout, P, H * W, C, att, chan_mul, dstats, argmax, dx));
  return hiseg_check_launch("attn_spatial_bwd");
}

extern "C" int hiseg_attn_channel_ws(int N, int C, int Cr) {
  return N * kGapSplits * C + N * C + N * 2 * C * Cr;  // floats: gap partials, dgap, per-image weight grads
}

extern "C" int hiseg_attn_channel_train_fwd(int dtype, const void* x, int N, int HW, int C, const float* w1, int Cr,
                                            const float* w2, int act, float act_beta, const float* chan_mul, float* ws,
                                            float* gap, float* hpre, float* gate, void* out, hiseg_stream_t stream) {
  HISEG_REQUIRE(x && w1 && w2 && ws && gap && hpre && gate && out && N > 0 && HW > 0 && Cr > 0, HISEG_ERR_BAD_ARG,
                "attn_channel_train_fwd: bad args");
  HISEG_REQUIRE(C > 0 && C % chunk_of(dtype) == 0, HISEG_ERR_BAD_SHAPE, "attn_channel_train_fwd: C alignment");
  hipStream_t s = (hipStream_t)stream;
  int S = 0;
  DISPATCH_T(dtype, S = ca_gap<T>(x, nullptr, nullptr, N, HW, C, ws, s));
  ca_mlp_fwd(ws, S, N, HW, C, Cr, w1, w2, act, act_beta, gap, hpre, gate, nullptr, nullptr,
             ws + (long long)N * kGapSplits * C, s);   // h in the dgap region
  DISPATCH_T(dtype, hipLaunchKernelGGL(ca_apply_kernel<T>, dim3(ca_ranges(N, HW), N),
                                       dim3(256), 0, s, x, N, HW, C, gate, chan_mul, out));
  return hiseg_check_launch("attn_channel_train_fwd");
}

extern "C" int hiseg_attn_channel_bwd(int dtype, const void* x, int N, int HW, int C, const float* w1, int Cr,
                                      const float* w2, int act, float act_beta, const float* chan_mul,
                                      const float* gap, const float* hpre, const float* gate, const void* dout, void* dx,
                                      float* ws, float* dw1, float* dw2, hiseg_stream_t stream) {
  HISEG_REQUIRE(x && w1 && w2 && gap && hpre && gate && dout && dx && ws && dw1 && dw2, HISEG_ERR_BAD_ARG,
                "attn_channel_bwd: null");
  HISEG_REQUIRE(C > 0 && C % chunk_of(dtype) == 0, HISEG_ERR_BAD_SHAPE, "attn_channel_bwd: C alignment");
  hipStream_t s = (hipStream_t)stream;
  float* part = ws;
  float* dgap = ws + (long long)N * kGapSplits * C;
  float* wpart = dgap + (long long)N * C;
  int S = 0;
  DISPATCH_T(dtype, S = ca_gap<T>(x, dout, chan_mul, N, HW, C, part, s));
  ca_mlp_bwd(part, S, N, C, Cr, w1, w2, act, act_beta, hpre, gate, dgap, wpart, s);   // wpart holds sd [N][Cr + C]
  ca_wgrad(N, C, Cr, wpart, gap, hpre, act, act_beta, dw1, dw2, nullptr, nullptr, s);
  DISPATCH_T(dtype, hipLaunchKernelGGL(ca_dx_kernel<T>, dim3(ca_ranges(N, HW), N),
                                       dim3(256), 0, s, dout, N, HW, C, gate, chan_mul, dgap, dx));
  return hiseg_check_launch("attn_channel_bwd");
}

// timm SqueezeExcite (EfficientNet MBConv: GAP -> conv_reduce + bias -> SiLU -> conv_expand + bias -> sigmoid)
// in train mode: the channel-attention kernels with biases.  fwd writes gap / hpre / gate and out = x * gate
// (the projection conv's input, materialised so its weight gradient sees it); bwd from d(out).
extern "C" long long hiseg_se_train_ws(int N, int C, int Cr) {
  return (long long)N * kGapSplits * C + (long long)N * C + (long long)N * 2 * C * Cr + (long long)N * (Cr + C);
}

extern "C" int hiseg_se_train_fwd(int dtype, const void* x, int N, int HW, int C, const float* w1, const float* b1,
                                  int Cr, const float* w2, const float* b2, int act, float* ws, float* gap,
                                  float* hpre, float* gate, void* out, hiseg_stream_t stream) {
  HISEG_REQUIRE(x && w1 && b1 && w2 && b2 && ws && gap && hpre && gate && out && N > 0 && HW > 0 && Cr > 0,
                HISEG_ERR_BAD_ARG, "se_train_fwd: bad args");
  HISEG_REQUIRE(C > 0 && C % chunk_of(dtype) == 0, HISEG_ERR_BAD_SHAPE, "se_train_fwd: C alignment");
  hipStream_t s = (hipStream_t)stream;
  int S = 0;
  DISPATCH_T(dtype, S = ca_gap<T>(x, nullptr, nullptr, N, HW, C, ws, s));
  ca_mlp_fwd(ws, S, N, HW, C, Cr, w1, w2, act, 1.f, gap, hpre, gate, b1, b2, ws + (long long)N * kGapSplits * C, s);
  DISPATCH_T(dtype, hipLaunchKernelGGL(ca_apply_kernel<T>, dim3(ca_ranges(N, HW), N),
                                       dim3(256), 0, s, x, N, HW, C, gate, nullptr, out));
  return hiseg_check_launch("se_train_fwd");
}

extern "C" int hiseg_se_train_bwd(int dtype, const void* x, int N, int HW, int C, const float* w1, int Cr,
                                  const float* w2, int act, const float* gap, const float* hpre, const float* gate,
                                  const void* dout, void* dx, float* ws, float* dw1, float* db1, float* dw2, float* db2,
                                  hiseg_stream_t stream) {
  HISEG_REQUIRE(x && w1 && w2 && gap && hpre && gate && dout && dx && ws && dw1 && db1 && dw2 && db2,
                HISEG_ERR_BAD_ARG, "se_train_bwd: null");
  HISEG_REQUIRE(C > 0 && C % chunk_of(dtype) == 0, HISEG_ERR_BAD_SHAPE, "se_train_bwd: C alignment");
  hipStream_t s = (hipStream_t)stream;
  float* part = ws;
  float* dgap = ws + (long long)N * kGapSplits * C;
  float* wpart = dgap + (long long)N * C;
  float* bpart = wpart + (long long)N * 2 * C * Cr;
  int S = 0;
  DISPATCH_T(dtype, S = ca_gap<T>(x, dout, nullptr, N, HW, C, part, s));
  ca_mlp_bwd(part, S, N, C, Cr, w1, w2, act, 1.f, hpre, gate, dgap, bpart, s);
  ca_wgrad(N, C, Cr, bpart, gap, hpre, act, 1.f, dw1, dw2, db1, db2, s);
  DISPATCH_T(dtype, hipLaunchKernelGGL(ca_dx_kernel<T>, dim3(ca_ranges(N, HW), N),
                                       dim3(256), 0, s, dout, N, HW, C, gate, nullptr, dgap, dx));
  return hiseg_check_launch("se_train_bwd");
}

static UbfArgs ubf_args(const hiseg_ubf_desc* d) {
  UbfArgs u;
  u.low = d->low; u.N = d->N; u.h = d->h; u.w = d->w;
  u.ut_w = d->ut_w; u.ut_b = d->ut_b;
  u.scale = d->scale; u.shift = d->shift; u.mean = d->mean; u.invstd = d->invstd; u.gamma = d->gamma;
  u.u1_w = d->u1_w; u.u1_b = d->u1_b;
  u.act = d->act; u.beta = d->act_beta; u.ln = d->layernorm;
  return u;
}

// blocks of the pass-1 reduction: kUbfBlocks pixel ranges (BN), or sb ranges per sample (LN)
static int ubf_sb(int N) { const int sb = 2048 / (N > 0 ? N : 1); return sb < 1 ? 1 : sb; }

static const int kUbfBlocks = 2048;   // 8 workgroups per CU: the per-pixel loops are latency-bound

extern "C" int hiseg_ubf_ws(int N) {
  const long long nb1 = (long long)N * ubf_sb(N);
  const long long part = nb1 * 162 > (long long)kUbfBlocks * 256 ? nb1 * 162 : (long long)kUbfBlocks * 256;
  const long long bwd = part + 96 + (long long)N * 34;
  const long long fwd = (long long)hiseg_bn_partials() * 96;
  return (int)(bwd > fwd ? bwd : fwd);
}

extern "C" int hiseg_ubf_train_fwd(const hiseg_ubf_desc* d, float eps, float momentum, float* running_mean,
                                   float* running_var, float* ws, hiseg_stream_t stream) {
  HISEG_REQUIRE(d && d->low && d->ut_w && d->ut_b && d->u1_w && d->u1_b && d->tfeat && d->t_w && d->t_b && d->logits &&
                    d->bgfg && d->tn && ws && d->scale && d->shift && d->mean && d->invstd,
                HISEG_ERR_BAD_ARG, "ubf_train_fwd: null argument");
  HISEG_REQUIRE(d->Ct > 0 && d->Ct <= 512 && d->Ct % chunk_of(d->dtype) == 0, HISEG_ERR_BAD_SHAPE, "ubf: Ct");
  HISEG_REQUIRE(d->act >= HISEG_ACT_NONE && d->act <= HISEG_ACT_SWISH, HISEG_ERR_BAD_ARG, "ubf: activation");
  hipStream_t s = (hipStream_t)stream;
  const UbfArgs u = ubf_args(d);
  const long long Pm = (long long)d->N * 4 * d->h * d->w;
  if (d->layernorm) {   // per-sample statistics; no running statistics
    int r = hiseg_ubf_ln_tables(d->low, d->N, d->h, d->w, d->ut_w, d->ut_b, d->gamma, d->beta, eps, 0,
                                const_cast<float*>(d->mean), const_cast<float*>(d->invstd), const_cast<float*>(d->scale),
                                const_cast<float*>(d->shift), stream);
    if (r) return r;
  } else {
    const int S = hiseg_bn_partials();
    hipLaunchKernelGGL(ubf_stats_kernel, dim3(S), dim3(256), 0, s, u, ws);
    int r = bn_finalize_splits(ws, S, 32, Pm, d->gamma, d->beta, eps, momentum, running_mean, running_var,
                               const_cast<float*>(d->mean), const_cast<float*>(d->invstd), const_cast<float*>(d->scale),
                               const_cast<float*>(d->shift), s);
    if (r) return r;
  }
  DISPATCH_T(d->dtype, hipLaunchKernelGGL(ubf_fwd_kernel<T>, dim3(nb(Pm, 256)), dim3(256), 0, s, u, d->tfeat, d->Ct,
                                          d->t_w, d->t_b, d->logits, d->bgfg, d->tn));
  return hiseg_check_launch("ubf_train_fwd");
}

extern "C" int hiseg_ubf_train_bwd(const hiseg_ubf_desc* d, const float* dlogits, const float* dbgfg_ext,
                                   const float* dtn_ext, float* db_buf, float* dtn_out, float* dlow, float* ws,
                                   const hiseg_ubf_grads* g, hiseg_stream_t stream) {
  HISEG_REQUIRE(d && dlogits && db_buf && dtn_out && dlow && ws && g && g->dut_w && g->dut_b && g->dgamma && g->dbeta &&
                    g->du1_w && g->du1_b,
                HISEG_ERR_BAD_ARG, "ubf_train_bwd: null argument");
  hipStream_t s = (hipStream_t)stream;
  const UbfArgs u = ubf_args(d);
  const long long Pm = (long long)d->N * 4 * d->h * d->w, PL = (long long)d->N * d->h * d->w;
  const int sb = ubf_sb(d->N);
  const int nb1 = d->layernorm ? d->N * sb : kUbfBlocks;
  const long long part_len = (long long)nb1 * 162 > (long long)kUbfBlocks * 256 ? (long long)nb1 * 162
                                                                                  : (long long)kUbfBlocks * 256;
  float* part = ws;                          // [nb1][162] (pass 1), then [kUbfBlocks][256] (pass 2)
  float* coef = ws + part_len;               // [96] (BN)
  float* coef_ln = coef + 96;                // [N][2] (LN)
  float* dbias = coef_ln + 2LL * d->N;       // [N][32] (LN)
  // HISEG_UBF_U2=0: the one-pixel loop with per-pixel weight reads (A/B timing; same results)
  const char* ue = getenv("HISEG_UBF_U2");
  if (!(ue && atoi(ue) == 0))
    hipLaunchKernelGGL(ubf_bwd1_kernel<true>, dim3(nb1), dim3(256), 0, s, u, dlogits, dbgfg_ext, dtn_ext, d->bgfg,
                       d->tn, db_buf, dtn_out, part, sb);
  else
    hipLaunchKernelGGL(ubf_bwd1_kernel<false>, dim3(nb1), dim3(256), 0, s, u, dlogits, dbgfg_ext, dtn_ext, d->bgfg,
                       d->tn, db_buf, dtn_out, part, sb);
  if (d->layernorm)
    hipLaunchKernelGGL(ubf_ln_fin_kernel, dim3(d->N), dim3(32), 0, s, u, part, sb, coef_ln, dbias);
  hipLaunchKernelGGL(ubf_fin1_kernel, dim3(1), dim3(192), 0, s, u, part, nb1, Pm, coef, g->dgamma, g->dbeta,
                     g->du1_w, g->du1_b, d->layernorm ? nullptr : g->dut_b);
  if (d->layernorm) sum_rows(dbias, d->N, 32, 32, g->dut_b, 1, s);
  hipLaunchKernelGGL(ubf_bwd2_kernel, dim3(kUbfBlocks), dim3(256), 0, s, u, db_buf, coef, coef_ln, dlow, part);
  // dWt [ci][c][q] in the ConvTranspose2d layout [2][32][2][2] == (ci*32 + c)*4 + q
  sum_rows(part, kUbfBlocks, 256, 256, g->dut_w, 1, s);
  (void)PL;
  return hiseg_check_launch("ubf_train_bwd");
}

static const int kPw2Blocks = 512;
extern "C" int hiseg_pw2_ws(int Ct) { return kPw2Blocks * (2 * Ct + 2); }

extern "C" int hiseg_pw2_bwd(int dtype, const void* tfeat, long long P, int Ct, const float* dtn, const float* w,
                             void* dt, float* ws, float* dw, float* db, hiseg_stream_t stream) {
  HISEG_REQUIRE(tfeat && dtn && w && dt && ws && dw && db && P > 0, HISEG_ERR_BAD_ARG, "pw2_bwd: null argument");
  HISEG_REQUIRE(Ct % chunk_of(dtype) == 0 && Ct / chunk_of(dtype) <= 256, HISEG_ERR_BAD_SHAPE, "pw2_bwd: Ct");
  hipStream_t s = (hipStream_t)stream;
  const int nch = Ct / chunk_of(dtype);
  const int R = 256 / nch;
  const size_t lds = (size_t)R * (2 * Ct + 2) * sizeof(float);
  DISPATCH_T(dtype, hipLaunchKernelGGL(pw2_bwd_kernel<T>, dim3(kPw2Blocks), dim3(256), lds, s, tfeat, P, Ct, dtn, w, dt, ws));
  sum_rows(ws, kPw2Blocks, 2 * Ct + 2, 2 * Ct, dw, 1, s);
  sum_rows(ws + 2 * Ct, kPw2Blocks, 2 * Ct + 2, 2, db, 1, s);
  return hiseg_check_launch("pw2_bwd");
}
