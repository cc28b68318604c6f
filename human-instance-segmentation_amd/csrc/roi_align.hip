// Dynamic RoIAlign forward (reference: src/human_edge_detection/dynamic_roi_align.py:56-171).
//
// One thread per output pixel (roi n, row i, col j); the sampling point and the four bilinear
// weights are computed once and reused for every channel.  The coordinate arithmetic follows
// the reference op for op in f32 with no FMA contraction (each product/sum rounded as torch
// rounds it on the CPU):
//   linspace(0,1,S)[j] = j < S/2 ? step*j : 1 - step*(S-1-j),  step = 1/(S-1)   (:110-111)
//   fx = x1 + gx*(x2-x1), x1 = roi_x1*scale_w                                    (:83-93,133)
//   nx = fx/(W-1)*2-1 (aligned) | fx/W*2-1                                       (:139-146)
//   grid_sample unnormalise (CPU vectorised form): (nx+1)*((W-1)/2) | (nx+1)*(W/2)-0.5
//   bilinear with zero padding: taps outside [0,W-1]x[0,H-1] contribute 0       (:163-169)
// Feature maps are read in place through the roi's batch index; the reference's
// index_select copy of N full maps (:156) is not materialised.
#include <cstdlib>

#include "common.h"
#include "hiseg_head_train.h"

// hipcc contracts a*b+c into an FMA by default (-ffp-contract=fast-honor-pragmas), and __fmul_rn / __fadd_rn are
// plain operators in this header set: without this pragma the sample coordinate x1 + g*(x2-x1) and the bilinear sum
// were fused, one rounding fewer than torch's CPU ops, which moved the taps' weights by an ulp (1e-5 relative on
// the ROI patches, amplified ~100x by train-mode BatchNorm).
#pragma clang fp contract(off)

namespace hiseg {

// plain operators under the pragma above: the header's __fmul_rn / __fadd_rn carry the contractable flag of the
// header's own code, and after inlining the backend fused them (x2*sw - x1, x1 + g*len, (n+1)*s - 0.5)
__device__ __forceinline__ float fmul(float a, float b) { return a * b; }
__device__ __forceinline__ float fadd(float a, float b) { return a + b; }
__device__ __forceinline__ float fsub(float a, float b) { return a - b; }

__device__ __forceinline__ float linspace01(int idx, int steps) {
  if (steps == 1) return 0.f;
  const float step = __fdiv_rn(1.0f, (float)(steps - 1));
  const int halfway = steps / 2;
  if (idx < halfway) return fmul(step, (float)idx);
  return fsub(1.0f, fmul(step, (float)(steps - idx - 1)));
}

// Returns the unnormalised source coordinate along one axis.
__device__ __forceinline__ float src_coord(float lo, float len, float g, int size, int aligned) {
  const float f = fadd(lo, fmul(g, len));
  if (aligned) {
    const float nrm = fsub(fmul(__fdiv_rn(f, (float)(size - 1)), 2.0f), 1.0f);
    return fmul(fadd(nrm, 1.0f), __fdiv_rn((float)(size - 1), 2.0f));
  }
  const float nrm = fsub(fmul(__fdiv_rn(f, (float)size), 2.0f), 1.0f);
  return fsub(fmul(fadd(nrm, 1.0f), __fdiv_rn((float)size, 2.0f)), 0.5f);
}

template <typename TO, bool VEC>
__global__ void __launch_bounds__(256) roi_align_kernel(hiseg_roi_align_desc d) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)d.N * d.oh * d.ow;
  if (gid >= total) return;
  const int j = (int)(gid % d.ow);
  const long long t = gid / d.ow;
  const int i = (int)(t % d.oh);
  const int n = (int)(t / d.oh);

  const float* roi = d.rois + (long long)n * 5;
  const float bf = roi[0];
  const long long b = (long long)bf;  // .long(): truncation toward zero
  const float x1 = fmul(roi[1], d.scale_w), y1 = fmul(roi[2], d.scale_h);
  const float x2 = fmul(roi[3], d.scale_w), y2 = fmul(roi[4], d.scale_h);
  const float ix = src_coord(x1, fsub(x2, x1), linspace01(j, d.ow), d.W, d.aligned);
  const float iy = src_coord(y1, fsub(y2, y1), linspace01(i, d.oh), d.H, d.aligned);

  const float xw = floorf(ix), yn = floorf(iy);
  const float wgt_w = fsub(ix, xw), wgt_e = fsub(1.f, wgt_w);
  const float wgt_n = fsub(iy, yn), wgt_s = fsub(1.f, wgt_n);
  const float w_nw = fmul(wgt_s, wgt_e), w_ne = fmul(wgt_s, wgt_w);
  const float w_sw = fmul(wgt_n, wgt_e), w_se = fmul(wgt_n, wgt_w);
  // integer tap positions (clamped to a safe range before the int conversion)
  const float xwc = fminf(fmaxf(xw, -2.f), (float)d.W + 1.f);
  const float ync = fminf(fmaxf(yn, -2.f), (float)d.H + 1.f);
  const int x0 = (int)xwc, y0 = (int)ync;
  const bool bvalid = (b >= 0 && b < d.B) && (ix == ix) && (iy == iy);
  const bool vx0 = x0 >= 0 && x0 < d.W, vx1 = x0 + 1 >= 0 && x0 + 1 < d.W;
  const bool vy0 = y0 >= 0 && y0 < d.H, vy1 = y0 + 1 >= 0 && y0 + 1 < d.H;

  const int Cout = d.aff_w ? d.n_aff : d.C;
  const long long plane = (long long)d.H * d.W;
  const bool aff = d.aff_w != nullptr;
  const float* src0 = d.feat + (bvalid ? b : 0) * d.C * plane;
  const long long o_nw = (long long)y0 * d.W + x0;   // tap offsets, used only where valid
  auto value = [&](int c) __attribute__((always_inline)) -> float {
    if (!bvalid) return 0.f;
    const float* src = src0 + (aff ? 0 : (long long)c * plane);
    float aw = 1.f, ab = 0.f;
    if (aff) { aw = d.aff_w[c]; ab = d.aff_b ? d.aff_b[c] : 0.f; }
    auto tap = [&](bool ok, long long off) -> float {
      if (!ok) return 0.f;
      const float u = src[off];
      return aff ? fadd(fmul(aw, u), ab) : u;
    };
    const float v_nw = tap(vy0 && vx0, o_nw);
    const float v_ne = tap(vy0 && vx1, o_nw + 1);
    const float v_sw = tap(vy1 && vx0, o_nw + d.W);
    const float v_se = tap(vy1 && vx1, o_nw + d.W + 1);
    return fadd(fadd(fadd(fmul(v_nw, w_nw), fmul(v_ne, w_ne)), fmul(v_sw, w_sw)), fmul(v_se, w_se));
  };
  if (d.o_nchw) {
    for (int c = 0; c < Cout; ++c)
      reinterpret_cast<float*>(d.out)[(((long long)n * Cout + c) * d.oh + i) * d.ow + j] = value(c);
    return;
  }
  if (VEC) {
    // the whole padded pixel (channels, then zeros up to zero_to == o_cstride) as 16-B stores: one per 8 bf16 /
    // 4 f32 channels instead of one 2- / 4-B store per channel, each lane's pixel 16-B aligned (checked on the host)
    constexpr int K = Chunk<TO>::N;
    uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<TO*>(d.out) + gid * d.o_cstride);
    for (int q = 0; q < d.o_cstride / K; ++q) {
      float v[K];
#pragma unroll
      for (int e = 0; e < K; ++e) v[e] = q * K + e < Cout ? value(q * K + e) : 0.f;
      dst[q] = Chunk<TO>::pack(v);
    }
    return;
  }
  for (int c = 0; c < Cout; ++c) Elem<TO>::store(d.out, gid * d.o_cstride + d.o_coff + c, value(c));
  for (int c = Cout; c < d.zero_to; ++c) Elem<TO>::store(d.out, gid * d.o_cstride + d.o_coff + c, 0.f);
}

// Backward into the output_conv affine (see hiseg_roi_align_bwd_affine): per sample, the same taps
// and weights as the forward; partial sums [block][4] = (dw0, dw1, db0, db1), n_aff == 2.
constexpr int kRoiBwdBlocks = 512;

template <typename TG>
__global__ void __launch_bounds__(256) roi_align_bwd_affine_kernel(hiseg_roi_align_desc d, const void* g, int gcs,
                                                                   int gco, float* part) {
  __shared__ float red[4][256];
  const long long total = (long long)d.N * d.oh * d.ow;
  float a0 = 0.f, a1 = 0.f, b0 = 0.f, b1 = 0.f;
  for (long long gid = (long long)blockIdx.x * 256 + threadIdx.x; gid < total; gid += (long long)gridDim.x * 256) {
    const int j = (int)(gid % d.ow);
    const long long t = gid / d.ow;
    const int i = (int)(t % d.oh);
    const int n = (int)(t / d.oh);
    const float* roi = d.rois + (long long)n * 5;
    const long long b = (long long)roi[0];
    const float x1 = fmul(roi[1], d.scale_w), y1 = fmul(roi[2], d.scale_h);
    const float x2 = fmul(roi[3], d.scale_w), y2 = fmul(roi[4], d.scale_h);
    const float ix = src_coord(x1, fsub(x2, x1), linspace01(j, d.ow), d.W, d.aligned);
    const float iy = src_coord(y1, fsub(y2, y1), linspace01(i, d.oh), d.H, d.aligned);
    const float xw = floorf(ix), yn = floorf(iy);
    const float wgt_w = fsub(ix, xw), wgt_e = fsub(1.f, wgt_w);
    const float wgt_n = fsub(iy, yn), wgt_s = fsub(1.f, wgt_n);
    const int x0 = (int)fminf(fmaxf(xw, -2.f), (float)d.W + 1.f), y0 = (int)fminf(fmaxf(yn, -2.f), (float)d.H + 1.f);
    if (!((b >= 0 && b < d.B) && (ix == ix) && (iy == iy))) continue;
    const bool vx0 = x0 >= 0 && x0 < d.W, vx1 = x0 + 1 >= 0 && x0 + 1 < d.W;
    const bool vy0 = y0 >= 0 && y0 < d.H, vy1 = y0 + 1 >= 0 && y0 + 1 < d.H;
    const float* src = d.feat + (long long)b * d.C * d.H * d.W;
    float vu = 0.f, ws = 0.f;
    auto tap = [&](bool ok, int yy, int xx, float w) {
      if (!ok) return;
      vu += w * src[(long long)yy * d.W + xx];
      ws += w;
    };
    tap(vy0 && vx0, y0, x0, fmul(wgt_s, wgt_e));
    tap(vy0 && vx1, y0, x0 + 1, fmul(wgt_s, wgt_w));
    tap(vy1 && vx0, y0 + 1, x0, fmul(wgt_n, wgt_e));
    tap(vy1 && vx1, y0 + 1, x0 + 1, fmul(wgt_n, wgt_w));
    const float g0 = Elem<TG>::load(g, gid * gcs + gco), g1 = Elem<TG>::load(g, gid * gcs + gco + 1);
    a0 += g0 * vu; a1 += g1 * vu; b0 += g0 * ws; b1 += g1 * ws;
  }
  const int t = threadIdx.x;
  red[0][t] = a0; red[1][t] = a1; red[2][t] = b0; red[3][t] = b1;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) {
#pragma unroll
      for (int k = 0; k < 4; ++k) red[k][t] += red[k][t + s];
    }
    __syncthreads();
  }
  if (t < 4) part[blockIdx.x * 4 + t] = red[t][0];
}

__global__ void roi_bwd_sum_kernel(const float* part, int nblk, float* dw, float* db) {
  const int t = threadIdx.x;
  if (t >= 4) return;
  double s = 0;
  for (int b = 0; b < nblk; ++b) s += part[b * 4 + t];
  if (t < 2) dw[t] += (float)s;
  else if (db) db[t - 2] += (float)s;
}

}  // namespace hiseg

using namespace hiseg;

static bool getenv_flag(const char* name, int dflt) {   // read per call (A/B timing, the equivalence test)
  const char* e = getenv(name);
  return e ? atoi(e) != 0 : dflt != 0;
}

extern "C" int hiseg_roi_align_ws(int N) { (void)N; return kRoiBwdBlocks * 4; }

extern "C" int hiseg_roi_align_bwd_affine(const hiseg_roi_align_desc* d, const void* g, int g_dtype, int g_cstride,
                                          int g_coff, float* ws, float* dw, float* db, hiseg_stream_t stream) {
  HISEG_REQUIRE(d && g && ws && dw, HISEG_ERR_BAD_ARG, "roi_align_bwd_affine: null argument");
  HISEG_REQUIRE(d->N > 0 && d->feat && d->rois && d->C == 1 && d->aff_w && d->n_aff == 2, HISEG_ERR_BAD_SHAPE,
                "roi_align_bwd_affine: expects the 1->2 output_conv over a 1-channel map");
  hipStream_t s = (hipStream_t)stream;
  if (g_dtype == HISEG_BF16)
    hipLaunchKernelGGL(roi_align_bwd_affine_kernel<bf16_t>, dim3(kRoiBwdBlocks), dim3(256), 0, s, *d, g, g_cstride, g_coff, ws);
  else
    hipLaunchKernelGGL(roi_align_bwd_affine_kernel<float>, dim3(kRoiBwdBlocks), dim3(256), 0, s, *d, g, g_cstride, g_coff, ws);
  hipLaunchKernelGGL(roi_bwd_sum_kernel, dim3(1), dim3(64), 0, s, ws, kRoiBwdBlocks, dw, db);
  return hiseg_check_launch("roi_align_bwd_affine");
}

extern "C" int hiseg_roi_align_fwd(const hiseg_roi_align_desc* d, hiseg_stream_t stream) {
  HISEG_REQUIRE(d != nullptr, HISEG_ERR_BAD_ARG, "roi_align: null descriptor");
  HISEG_REQUIRE(d->N >= 0, HISEG_ERR_BAD_SHAPE, "roi_align: negative N");
  if (d->N == 0) return HISEG_OK;  // empty ROI list (empty tensors carry null pointers)
  HISEG_REQUIRE(d->feat && d->rois && d->out, HISEG_ERR_BAD_ARG, "roi_align: null pointer");
  HISEG_REQUIRE(d->B > 0 && d->C > 0 && d->H > 0 && d->W > 0 && d->oh > 0 && d->ow > 0 && d->N >= 0,
                HISEG_ERR_BAD_SHAPE, "roi_align: bad shape");
  HISEG_REQUIRE(!d->aligned || (d->H > 1 && d->W > 1), HISEG_ERR_BAD_SHAPE, "roi_align: aligned needs H,W > 1");
  HISEG_REQUIRE(!d->aff_w || d->n_aff > 0, HISEG_ERR_BAD_ARG, "roi_align: n_aff");
  HISEG_REQUIRE(!d->o_nchw || d->out_dtype == HISEG_F32, HISEG_ERR_BAD_DTYPE, "roi_align: NCHW output is f32 only");
  const int Cout = d->aff_w ? d->n_aff : d->C;
  HISEG_REQUIRE(d->o_nchw || d->o_cstride >= d->o_coff + (d->zero_to > Cout ? d->zero_to : Cout), HISEG_ERR_BAD_SHAPE,
                "roi_align: o_cstride too small");
  if (d->N == 0) return HISEG_OK;
  const long long total = (long long)d->N * d->oh * d->ow;
  dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
  // whole-pixel 16-B stores: NHWC output written from channel 0 through the padding (zero_to == o_cstride), pixel
  // stride a whole number of 16-B chunks, 16-B aligned base
  const int esz = d->out_dtype == HISEG_BF16 ? 2 : 4;
  const bool vec = !d->o_nchw && d->o_coff == 0 && d->zero_to == d->o_cstride && (d->o_cstride * esz) % 16 == 0 &&
                   (reinterpret_cast<uintptr_t>(d->out) & 15) == 0 && getenv_flag("HISEG_ROI_VEC", 1);
#define ROI_L(TO)                                                                          \
  do {                                                                                     \
    if (vec) hipLaunchKernelGGL((roi_align_kernel<TO, true>), grid, dim3(256), 0, s, *d);  \
    else hipLaunchKernelGGL((roi_align_kernel<TO, false>), grid, dim3(256), 0, s, *d);     \
  } while (0)
  if (d->out_dtype == HISEG_BF16) ROI_L(bf16_t);
  else ROI_L(float);
#undef ROI_L
  return hiseg_check_launch("roi_align");
}
