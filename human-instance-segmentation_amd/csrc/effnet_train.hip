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

// LDS-tiled weight gradient (bf16; round 6).  dw_bwd_weight_kernel re-reads every input chunk K x K times through
// L1 / L2 with K + 1 16-B loads per (task, pixel).  Here a block takes TPB consecutive 8 x 16 output tiles (flattened
// over the images) x 64 channels: per tile the (7 ST + K) x (15 ST + K) input window and the 8 x 16 dy tile go to LDS
// once (zeros outside the image, past Ho / Wo and past C), then thread (channel pair cp, tile row ry) holds its row's
// 16 dy pairs and all K x K tap accumulators (packed f32 pairs) and sweeps the window rows it needs: each window
// value feeds the <= K taps whose outputs read it.  After its tiles the block sums the 8 rows in LDS in row order
// and writes one partial per (tile range, channel, tap) -- ws[range][c * K * K + t] -- reduced in double by
// dw_wpart_kernel / dw_weight_reduce_kernel.  Different summation order from dw_bwd_weight_kernel (f32 partials
// per tile row, then double): equal within f32 re-association.
constexpr int kWgTH = 8, kWgTW = 16, kWgCG = 64, kWgPS = kWgCG * 2 + 8;

__host__ __device__ constexpr int wg_win_bytes(int KS, int ST) {
  return ((kWgTH - 1) * ST + KS) * ((kWgTW - 1) * ST + KS) * kWgPS;
}
__host__ __device__ constexpr int wg_lds_bytes(int KS, int ST) {
  return (wg_win_bytes(KS, ST) + kWgTH * kWgTW * kWgPS) > kWgTH * KS * KS * kWgCG * 4
             ? wg_win_bytes(KS, ST) + kWgTH * kWgTW * kWgPS
             : kWgTH * KS * KS * kWgCG * 4;
}

template <int KS, int ST>
__global__ void __launch_bounds__(256) dw_wgrad_tile_kernel(const void* x, const void* dy, int H, int W, int C,
                                                            int Ho, int Wo, int ntiles, int TPB, float* ws) {
  constexpr int IH = (kWgTH - 1) * ST + KS, IW = (kWgTW - 1) * ST + KS, KK = KS * KS;
  extern __shared__ __attribute__((aligned(16))) char wgs[];
  char* const win = wgs;
  char* const dyl = wgs + wg_win_bytes(KS, ST);
  const int t = threadIdx.x;
  const int g0 = blockIdx.y * kWgCG;
  const int nch = C >> 3;
  const int ntx = (Wo + kWgTW - 1) / kWgTW, tpi = ((Ho + kWgTH - 1) / kWgTH) * ntx;   // tiles per image
  const int cp = t & 31, ry = t >> 5;
  const int c = g0 + cp * 2;
  typedef float f2v __attribute__((ext_vector_type(2)));
  f2v acc[KK];
#pragma unroll
  for (int k = 0; k < KK; ++k) acc[k] = f2v{0.f, 0.f};
  const int tb = blockIdx.x * TPB, te = tb + TPB < ntiles ? tb + TPB : ntiles;
  for (int ti = tb; ti < te; ++ti) {
    const int n = ti / tpi, bt = ti - n * tpi;
    const int ty = bt / ntx, tx = bt - ty * ntx;
    const int oy0 = ty * kWgTH, ox0 = tx * kWgTW;
    const int iy0 = oy0 * ST - KS / 2, ix0 = ox0 * ST - KS / 2;
    const uint4* src = reinterpret_cast<const uint4*>(x) + (long long)n * H * W * nch;
    const uint4* dsrc = reinterpret_cast<const uint4*>(dy) + (long long)n * Ho * Wo * nch;
    // ---- window + dy tile -> LDS: 8 chunks (128 B) per pixel, batches of 8 loads in flight per thread
    constexpr int NLW = IH * IW * 8, NLD = kWgTH * kWgTW * 8, NL = NLW + NLD, NB = (NL + 255) / 256;
    __syncthreads();   // the previous tile's window / dy are no longer read
#pragma unroll
    for (int b0 = 0; b0 < NB; b0 += 8) {
      uint4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = t + 256 * (b0 + u);
        v[u] = make_uint4(0u, 0u, 0u, 0u);
        if (b0 + u < NB && idx < NL) {
          const int j = idx < NLW ? idx : idx - NLW;
          const int pix = j >> 3, ch = (g0 >> 3) + (j & 7);
          if (idx < NLW) {
            const int hy = pix / IW, hx = pix - hy * IW;
            const int iy = iy0 + hy, ix = ix0 + hx;
            if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W && ch < nch)
              v[u] = src[((long long)iy * W + ix) * nch + ch];
          } else {
            const int oy = oy0 + (pix >> 4), ox = ox0 + (pix & 15);
            if (oy < Ho && ox < Wo && ch < nch) v[u] = dsrc[((long long)oy * Wo + ox) * nch + ch];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = t + 256 * (b0 + u);
        if (b0 + u < NB && idx < NL) {
          char* base = idx < NLW ? win + (idx >> 3) * kWgPS + (idx & 7) * 16
                                 : dyl + ((idx - NLW) >> 3) * kWgPS + ((idx - NLW) & 7) * 16;
          *reinterpret_cast<uint4*>(base) = v[u];
        }
      }
    }
    __syncthreads();
    // ---- this thread's 16 dy pairs of tile row ry, then the window rows ry * ST + ky
    f2v d[kWgTW];
#pragma unroll
    for (int ox = 0; ox < kWgTW; ++ox) {
      const unsigned raw = *reinterpret_cast<const unsigned*>(dyl + (ry * kWgTW + ox) * kWgPS + cp * 4);
      d[ox] = f2v{__uint_as_float(raw << 16), __uint_as_float(raw & 0xffff0000u)};
    }
#pragma unroll
    for (int ky = 0; ky < KS; ++ky) {
      const char* row = win + ((ry * ST + ky) * IW) * kWgPS + cp * 4;
#pragma unroll
      for (int j = 0; j < IW; ++j) {
        const unsigned raw = *reinterpret_cast<const unsigned*>(row + j * kWgPS);
        const f2v xv{__uint_as_float(raw << 16), __uint_as_float(raw & 0xffff0000u)};
#pragma unroll
        for (int ox = 0; ox < kWgTW; ++ox) {
          const int kx = j - ox * ST;
          if (kx < 0 || kx >= KS) continue;
          acc[ky * KS + kx] = __builtin_elementwise_fma(d[ox], xv, acc[ky * KS + kx]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // ---- the 8 tile rows summed in row order: LDS red[ry][tap][64 channels]
  __syncthreads();
  float* red = reinterpret_cast<float*>(wgs);
#pragma unroll
  for (int k = 0; k < KK; ++k) {
    red[(ry * KK + k) * kWgCG + cp * 2] = acc[k].x;
    red[(ry * KK + k) * kWgCG + cp * 2 + 1] = acc[k].y;
  }
  __syncthreads();
  float* out = ws + (long long)blockIdx.x * C * KK + (long long)g0 * KK;
  const int lim = (C - g0 < kWgCG ? C - g0 : kWgCG) * KK;
  for (int i = t; i < lim; i += 256) {
    const int cl = i / KK, k = i - cl * KK;
    float sum = red[k * kWgCG + cl];
#pragma unroll
    for (int r = 1; r < kWgTH; ++r) sum += red[(r * KK + k) * kWgCG + cl];
    out[i] = sum;
  }
  (void)c;
}

// Stride-2 data gradient, LDS-tiled (bf16; round 6).  dw_bwd_data_kernel gives each thread one 8-channel chunk of one
// input pixel: K x K tap tests, 64-bit index divisions, a 16-B dy load per valid tap and 8 strided weight loads per
// tap.  Here a block owns an 8 x 16 tile of dx (one image, 64 channels); the dy window under it ((K + 7) / 2 + 1 rows
// x (K + 15) / 2 + 1 columns, zeros outside the dy grid / past C) goes to LDS once.  Thread (channel pair cp, tile row
// ry) holds its 2 channels' K x K weights and writes 16 dx pairs; the rows are dealt so a wave's two rows share their
// parity (rows w, w + 4 of wave w), so the valid ky taps are wave-uniform and the kx taps compile-time per column.
// Per output the taps run in dw_bwd_data_kernel's order (ky, then kx, skipping the invalid ones).
constexpr int kDgTH = 8, kDgTW = 16, kDgCG = 64, kDgPS = kDgCG * 2 + 8;

template <int KS, int PAR>
__device__ __forceinline__ void dg_row(const char* dyw, int DW, int rloc, int cp, const float (&w)[KS * KS][2],
                                       float (&o)[kDgTW][2]) {
  // dx row with parity PAR: ky valid when (iy + p - ky) is even; its dy row (iy + p - ky) / 2 is window row
  // (rloc + p - ky) / 2 where rloc = iy - iy0 + 2 * (iy0 / 2 - DY0) (even-based local row)
  constexpr int P = KS / 2;
#pragma unroll
  for (int ox = 0; ox < kDgTW; ++ox) o[ox][0] = o[ox][1] = 0.f;
#pragma unroll
  for (int ky = 0; ky < KS; ++ky) {
    if (((PAR + P - ky) & 1) != 0) continue;
    const char* row = dyw + ((rloc + P - ky) >> 1) * DW * kDgPS + cp * 4;
#pragma unroll
    for (int ox = 0; ox < kDgTW; ++ox) {
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        if (((ox + P - kx) & 1) != 0) continue;
        const int col = (ox + P - kx + (KS == 5 ? 2 : 0)) >> 1;   // window column (the window starts one column
                                                                // left of ix0 / 2 for k5)
        const unsigned raw = *reinterpret_cast<const unsigned*>(row + col * kDgPS);
        o[ox][0] = __builtin_fmaf(__uint_as_float(raw << 16), w[ky * KS + kx][0], o[ox][0]);
        o[ox][1] = __builtin_fmaf(__uint_as_float(raw & 0xffff0000u), w[ky * KS + kx][1], o[ox][1]);
      }
    }
  }
}

template <int KS>
__global__ void __launch_bounds__(256) dw_dgrad_s2_tile_kernel(const void* dy, int H, int W, int C, const float* wt,
                                                               int Ho, int Wo, void* dx, int accumulate) {
  constexpr int P = KS / 2;
  // window rows / cols: (ry + 2P - ky) / 2 over the valid (even) numerators -> 0 .. (7 + 2P) / 2, (15 + 2P) / 2
  constexpr int DH = (kDgTH - 1 + 2 * P) / 2 + 1, DW = (kDgTW - 1 + 2 * P) / 2 + 1;
  __shared__ __attribute__((aligned(16))) char dyw[DH * DW * kDgPS];
  const int t = threadIdx.x;
  const int n = blockIdx.y, g0 = blockIdx.z * kDgCG;
  const int ntx = (W + kDgTW - 1) / kDgTW;
  const int ty = blockIdx.x / ntx, tx = blockIdx.x - ty * ntx;
  const int iy0 = ty * kDgTH, ix0 = tx * kDgTW;   // both even
  // dy rows / cols under the tile: (iy + P - ky) / 2 over iy in [iy0, iy0 + 7], ky in [0, K - 1], even numerators
  const int DY0 = iy0 / 2 - (KS == 5 ? 1 : 0), DX0 = ix0 / 2 - (KS == 5 ? 1 : 0);
  const int nch = C >> 3;
  const uint4* src = reinterpret_cast<const uint4*>(dy) + (long long)n * Ho * Wo * nch;
  for (int idx = t; idx < DH * DW * 8; idx += 256) {
    const int pix = idx >> 3, ch = (g0 >> 3) + (idx & 7);
    const int hy = pix / DW, hx = pix - hy * DW;
    const int oy = DY0 + hy, ox = DX0 + hx;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if ((unsigned)oy < (unsigned)Ho && (unsigned)ox < (unsigned)Wo && ch < nch)
      v = src[((long long)oy * Wo + ox) * nch + ch];
    *reinterpret_cast<uint4*>(dyw + pix * kDgPS + (idx & 7) * 16) = v;
  }
  const int cp = t & 31, ry = (t >> 6) + 4 * ((t >> 5) & 1);   // a wave's two rows: w and w + 4 (same parity)
  const int c = g0 + cp * 2;
  const bool live = c < C;
  const int cc = live ? c : 0;
  float w[KS * KS][2];
#pragma unroll
  for (int k = 0; k < KS * KS; ++k) {
    w[k][0] = wt[(long long)cc * KS * KS + k];
    w[k][1] = wt[(long long)(cc + 1) * KS * KS + k];
  }
  __syncthreads();
  const int iy = iy0 + ry;
  if (!live || iy >= H) return;
  float o[kDgTW][2];
  // local even-based row: window row of dy row (iy + P - ky) / 2 is that minus DY0; rloc = iy - 2 * DY0
  const int rloc = iy - 2 * DY0;
  if (ry & 1) dg_row<KS, 1>(dyw, DW, rloc, cp, w, o);
  else dg_row<KS, 0>(dyw, DW, rloc, cp, w, o);
  unsigned* dst = reinterpret_cast<unsigned*>(dx) + ((long long)(n * H + iy) * W) * (C >> 1) + (c >> 1);
#pragma unroll
  for (int ox = 0; ox < kDgTW; ++ox) {
    if (ix0 + ox >= W) break;
    unsigned* d = dst + (long long)(ix0 + ox) * (C >> 1);
    float a = o[ox][0], b = o[ox][1];
    if (accumulate) {
      const unsigned prev = *d;
      a += __uint_as_float(prev << 16);
      b += __uint_as_float(prev & 0xffff0000u);
    }
    *d = f2bf2(a, b);
  }
}

// first pass of the split reduction when there are many splits: part[g][i] = sum of splits [g * 256, (g + 1) * 256)
// of output i in double (a block = 64 outputs x 4 lanes, lane l the splits l, l + 4, ... of the chunk with 16 loads
// in flight, the lanes combined in order)
__global__ void __launch_bounds__(256) dw_wpart_kernel(const float* ws, int S, int n, double* part) {
  __shared__ double red[4][64];
  const int ol = threadIdx.x & 63, l = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + ol;
  const int s0 = blockIdx.y * 256, s1 = s0 + 256 < S ? s0 + 256 : S;
  double acc = 0.0;
  if (i < n) {
    for (int sb = s0 + l; sb < s1; sb += 64) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = sb + 4 * u < s1 ? ws[(long long)(sb + 4 * u) * n + i] : 0.f;
#pragma unroll
      for (int u = 0; u < 16; ++u) acc += v[u];
    }
  }
  red[l][ol] = acc;
  __syncthreads();
  if (l == 0 && i < n) part[(long long)blockIdx.y * n + i] = ((red[0][ol] + red[1][ol]) + red[2][ol]) + red[3][ol];
}

// second pass: dw[i] += sum_g part[g][i], in order
__global__ void __launch_bounds__(256) dw_wpart_final_kernel(const double* part, int G, int n, float* dw) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double acc = 0.0;
  for (int g = 0; g < G; ++g) acc += part[(long long)g * n + i];
  dw[i] = (float)((double)dw[i] + acc);
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

// HISEG_DW_DGRAD_TILE (read per call): 1 (default) the LDS-tiled stride-2 data gradient on bf16 layers, 0 the
// per-pixel kernel
static bool dw_dg_tiled() {
  const char* e = getenv("HISEG_DW_DGRAD_TILE");
  return !(e && e[0] == '0');
}

extern "C" int hiseg_dw_bwd_data(int dtype, const void* dy, int N, int H, int W, int C, int K, int stride,
                                 const float* w, int Ho, int Wo, void* dx, int accumulate, hiseg_stream_t stream) {
  HISEG_REQUIRE(dy && w && dx, HISEG_ERR_BAD_ARG, "dw_bwd_data: null");
  const int r = dw_check(dtype, N, H, W, C, K, stride, Ho, Wo);
  if (r) return r;
  if (dtype == HISEG_BF16 && stride == 2 && (K == 3 || K == 5) && dw_dg_tiled()) {
    const dim3 grid(((H + kDgTH - 1) / kDgTH) * ((W + kDgTW - 1) / kDgTW), N, (C + kDgCG - 1) / kDgCG);
    if (K == 3)
      hipLaunchKernelGGL(dw_dgrad_s2_tile_kernel<3>, grid, dim3(256), 0, (hipStream_t)stream, dy, H, W, C, w, Ho, Wo,
                         dx, accumulate);
    else
      hipLaunchKernelGGL(dw_dgrad_s2_tile_kernel<5>, grid, dim3(256), 0, (hipStream_t)stream, dy, H, W, C, w, Ho, Wo,
                         dx, accumulate);
    return hiseg_check_launch("dw_bwd_data");
  }
  const long long n = (long long)N * H * W * (C / (dtype == HISEG_BF16 ? 8 : 4));
  DW_DISPATCH(dtype, dw_bwd_data_kernel, dim3(dw_blocks(n)), dim3(256), 0, (hipStream_t)stream, dy, N, H, W, C, K,
              stride, w, Ho, Wo, dx, accumulate);
  return hiseg_check_launch("dw_bwd_data");
}

// the LDS-tiled weight gradient's tile ranges: TPB tiles per block, about 2048 blocks over the channel groups
static void dw_wg_ranges(int N, int Ho, int Wo, int C, int* ntiles, int* tpb, int* S) {
  const int T = N * ((Ho + kWgTH - 1) / kWgTH) * ((Wo + kWgTW - 1) / kWgTW), groups = (C + kWgCG - 1) / kWgCG;
  long long b = ((long long)T * groups + 2047) / 2048;
  const int p = (int)(b < 1 ? 1 : b);
  *ntiles = T;
  *tpb = p;
  *S = (T + p - 1) / p;
}

// HISEG_DW_WGRAD_TILE (read per call): 1 (default) the LDS-tiled weight gradient on bf16 layers, 0 the split kernel
static bool dw_wg_tiled(int dtype) {
  const char* e = getenv("HISEG_DW_WGRAD_TILE");
  return dtype == HISEG_BF16 && !(e && e[0] == '0');
}

extern "C" long long hiseg_dw_bwd_weight_ws(int dtype, int N, int Ho, int Wo, int C, int K) {
  // floats; room for either path (the choice is read per call): the split kernel's partials, or the tiled kernel's
  // per-range partials followed by the first reduction pass's double partials
  const long long old = (long long)dw_wsplits((long long)N * Ho * Wo, C, K, dtype == HISEG_BF16 ? 8 : 4) * C * K * K;
  int T, p, S;
  dw_wg_ranges(N, Ho, Wo, C, &T, &p, &S);
  const long long n = (long long)C * K * K, G = (S + 255) / 256;
  const long long tiled = (long long)S * n + 2 * G * n + 4;
  return old > tiled ? old : tiled;
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
  if (dw_wg_tiled(dtype)) {
    int T, p, S;
    dw_wg_ranges(N, Ho, Wo, C, &T, &p, &S);
    const dim3 grid(S, (C + kWgCG - 1) / kWgCG);
#define WG_L(KS, ST)                                                                                                 \
  do {                                                                                                               \
    static bool attr = false;                                                                                        \
    if (!attr) {                                                                                                     \
      (void)hipFuncSetAttribute((const void*)dw_wgrad_tile_kernel<KS, ST>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                wg_lds_bytes(KS, ST));                                                               \
      attr = true;                                                                                                   \
    }                                                                                                                \
    hipLaunchKernelGGL((dw_wgrad_tile_kernel<KS, ST>), grid, dim3(256), wg_lds_bytes(KS, ST), s, x, dy, H, W, C, Ho,  \
                       Wo, T, p, ws);                                                                                \
  } while (0)
    if (K == 3 && stride == 1) WG_L(3, 1);
    else if (K == 3) WG_L(3, 2);
    else if (K == 5 && stride == 1) WG_L(5, 1);
    else if (K == 5) WG_L(5, 2);
    else HISEG_REQUIRE(false, HISEG_ERR_BAD_SHAPE, "dw_bwd_weight: tiled form takes k3 / k5 (K %d)", K);
#undef WG_L
    const int n = C * K * K;
    if (S <= 256) {
      hipLaunchKernelGGL(dw_weight_reduce_kernel, dim3((n + 63) / 64), dim3(256), 0, s, ws, S, n, dw);
    } else {
      const int G = (S + 255) / 256;
      double* part = reinterpret_cast<double*>(ws + (((long long)S * n + 1) & ~1ll));
      hipLaunchKernelGGL(dw_wpart_kernel, dim3((n + 63) / 64, G), dim3(256), 0, s, ws, S, n, part);
      hipLaunchKernelGGL(dw_wpart_final_kernel, dim3((n + 255) / 256), dim3(256), 0, s, part, G, n, dw);
    }
    return hiseg_check_launch("dw_bwd_weight");
  }
  const int tasks = nch * K, TPB = tasks < 256 ? tasks : 256;
  const int S = dw_wsplits((long long)N * Ho * Wo, C, K, dtype == HISEG_BF16 ? 8 : 4);
  DW_DISPATCH(dtype, dw_bwd_weight_kernel, dim3(S, (tasks + TPB - 1) / TPB), dim3(256), 0, s, x, dy, N, H, W,
              C, K, stride, Ho, Wo, TPB, ws);
  const int n = C * K * K;
  hipLaunchKernelGGL(dw_weight_reduce_kernel, dim3((n + 63) / 64), dim3(256), 0, s, ws, S, n, dw);
  return hiseg_check_launch("dw_bwd_weight");
}
