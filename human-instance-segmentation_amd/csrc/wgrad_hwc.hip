// Halo-tiled weight gradient of 3x3 stride-1 convolutions on 32x32x16 MFMA (gfx950, bf16): the ROI head's 64- to
// 256-channel ResidualBlock layers (refinement.py:31-55), trained by train_advanced.py:680-762.
//
//   dW[co][tap][ci] = sum_p dY[p][co] * X[p + tap][ci]        (tap = (ky, kx), p over the output pixels)
//
// The transposed-read kernels (train_conv.hip, wgrad_wide.hip) run this as a GEMM over K = 9 Cin columns: every tap
// of a pixel block re-stages the same X pixels and the same dY block from L2 into LDS, once per 128- / 256-column K
// tile.  Here a workgroup owns 64 Cout x 64 Cin x all 9 taps and walks pixel tiles of 8 rows x 16 columns: per tile
// the dY tile (128 pixels x 64 Cout) and the X halo (10 x 18 pixels x 64 Cin) are LDS-DMA'd once, double-buffered,
// and each wave (32 Cout x 32 Cin) walks the 10 halo rows: halo row hr's B fragments (16 pixels x 32 Cin, one per
// kx) feed the 3 ky taps of output rows hr - ky, whose A fragments (32 Cout x 16 pixels of one output row) stay in a
// 4-row register ring (the next row read ahead) -- 9 MFMAs per 3 + 1 fragment reads, each fragment two ds_read_b64_tr_b16 (the LDS images are
// pixel-major, channels contiguous, as the DMA delivers them).  The 9 tap accumulators (32 x 32 f32 each, 144
// registers) persist over the workgroup's pixel tiles; the loop issues no vector-memory instruction but the next
// tile's DMA, so its one wait per tile (vmcnt(0) + barrier) covers a whole tile of MFMAs.
//
// Split-K over pixel tiles into the f32 partial planes ws[split][Cg][Kg] (k = tap Cin + ci) that
// hiseg_conv2d_wgrad_reduce sums, the GEMM-bias column k = Ktot (sum of dY, the conv bias gradient) from one more
// MFMA per output row against a ones fragment in the Cin-tile-0 waves.  Accumulation order: the workgroup's pixel
// tiles in order, rows in order, 16 pixels per MFMA -- deterministic and independent of placement (the layer rules
// below depend on shapes only), but not the transposed-read kernels' order: wgrad_geometry gives these layers a
// split count of their own.
#include "hiseg_train.h"
#include "wgrad_common.h"

namespace hiseg {

typedef short wh_v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) wh_v4s_t wh_lds_v4s_t;
typedef __attribute__((address_space(3))) void wh_lds_void_t;
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef short wh_v8s_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void wh_dma16(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, unsigned voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(__builtin_amdgcn_readfirstlane(lds_addr)), "v"(voff), "s"(rsrc) : "memory");
}

typedef __attribute__((address_space(3))) char wh_lds_char_t;
__device__ __forceinline__ wh_v4s_t wh_tr(const wh_lds_char_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((wh_lds_v4s_t*)p);
}

__device__ __forceinline__ bf16x8_t wh_cat(wh_v4s_t lo, wh_v4s_t hi) {
  const wh_v8s_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// LDS image rows are 128 B (64 channels, 8 chunks of 16 B); chunk c of row r sits at slot c ^ 4 ((r >> 1) & 1): the
// 4 rows x 4 chunks a 32-lane half reads per ds_read_b64_tr_b16 (4 consecutive rows) land in distinct banks.
constexpr int WH_TR = 8, WH_TW = 16, WH_HWD = 18, WH_NHP = (WH_TR + 2) * WH_HWD;   // 180 halo pixels
constexpr int WH_DY_B = WH_TR * WH_TW * 128;                                        // 16 KiB
constexpr int WH_XI = (WH_NHP + 7) / 8;                                             // 23 DMA pieces of 8 rows
constexpr int WH_STAGE = WH_DY_B + WH_XI * 1024;                                    // 39 936 B
constexpr int WH_LDS = 2 * WH_STAGE;                                                // two per CU fit 160 KiB

// VAR (timing variants, HISEG_WGRAD_HWC_VAR): bit 0 MFMA rows at raised wave priority (s_setprio 1); bit 1 the second
// workgroup of each CU (dispatch order) starts half a pixel tile late, so the two workgroups sharing each SIMD reach
// their barriers out of phase
template <bool BIAS, int VAR = 0>
__global__ void __launch_bounds__(256, 2) conv_wgrad_hwc_kernel(WgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wco = w & 1, wci = w >> 1;   // the wave's 32-Cout / 32-Cin half of the 64 x 64 tile
  const int nco = d.Cout / 64, nci = a.Cin / 64;
  const int ntx = (d.W + WH_TW - 1) / WH_TW, nty = (d.H + WH_TR - 1) / WH_TR;
  const int NT = d.N * nty * ntx;
  // XCD-major bijective remap: the (Cout, Cin) tiles of one split -- the same pixel tiles -- run on one XCD
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = orig & 7, loc = orig >> 3;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int tile = wg % (nco * nci), split = wg / (nco * nci);
  const int co0 = (tile % nco) * 64, ci0 = (tile / nco) * 64;
  const int tps = (NT + a.splits - 1) / a.splits;
  const int t0 = split * tps, t1 = t0 + tps < NT ? t0 + tps : NT;

  const unsigned OOB = 0x80000000u;
  // the workgroup's 64 input channels lie in one source (Ca and Cb multiples of 64): source A, or the concat's B
  const bool srcb = ci0 >= d.Ca;
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(srcb ? d.srcB : d.srcA), (short)0, d.N * d.H * d.W * (srcb ? d.b_cstride : d.a_cstride) * 2,
      0x00020000);
  const int x_cs = srcb ? d.b_cstride : d.a_cstride, x_c0 = srcb ? d.b_coff + ci0 - d.Ca : d.a_coff + ci0;
  const __amdgpu_buffer_rsrc_t rY = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(a.dy), (short)0, (a.M * a.dy_cs + a.dy_coff + d.Cout) * 2, 0x00020000);
  const unsigned lds_base = (unsigned)(uintptr_t)(wh_lds_void_t*)smem;

  // ---- DMA of pixel tile tt into stage buffer sb: dY rows (16 pieces, 4 per wave), X halo rows (23 pieces)
  auto dma = [&](int tt, int sb) __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int tx = tt % ntx, rest = tt / ntx, ty = rest % nty, n = rest / nty;
    const int y0 = ty * WH_TR, x0 = tx * WH_TW;
    const int slot = ln & 7;
    const unsigned sbase = lds_base + (unsigned)(sb * WH_STAGE);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = w + 4 * k;
      const int row = 8 * i + (ln >> 3);
      const int c = slot ^ (((row >> 1) & 1) << 2);
      const int y = y0 + (row >> 4), x = x0 + (row & 15);
      const unsigned off = (y < d.H && x < d.W)
                               ? (unsigned)((((n * d.H + y) * d.W + x) * a.dy_cs + a.dy_coff + co0 + 8 * c) * 2)
                               : OOB;
      wh_dma16(rY, sbase + (unsigned)(i * 1024), off);
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int i = w + 4 * k;
      if (i < WH_XI) {
        const int hp = 8 * i + (ln >> 3);
        const int c = slot ^ (((hp >> 1) & 1) << 2);
        const int hy = hp / WH_HWD, hx = hp - WH_HWD * hy;
        const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
        const bool ok = hp < WH_NHP && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
        const unsigned off =
            ok ? (unsigned)((((n * d.H + iy) * d.W + ix) * x_cs + x_c0 + 8 * c) * 2) : OOB;
        wh_dma16(rX, sbase + (unsigned)(WH_DY_B + i * 1024), off);
      }
    }
  };

  // ---- per-lane fragment-read bases.  ds_read_b64_tr_b16: lane 4q + p of a 16-lane group g supplies row q, columns
  // 4p .. 4p + 3 of the group's 4 x 16 block and receives column (lane & 15) of the 4 rows.  A = dY^T (rows Cout,
  // k = pixels): group g reads Cout 16 (g & 1) .. + 15 of the wave's 32, pixels 8 (g >> 1) + 4 j + q of an output row
  // (j = 0, 1: the two reads).  B = X (k = pixels, columns Cin): the same with halo pixels and Cin.
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int ca = 4 * wco + 2 * (g & 1) + (p >> 1);   // dY chunk (Cout / 8 within the 64-Cout tile)
  const int cb = 4 * wci + 2 * (g & 1) + (p >> 1);   // X chunk
  // dY row = 16 r + 8 (g >> 1) + 4 j + q: its swizzle bit is q's
  const unsigned a_lane = (unsigned)((8 * (g >> 1) + q) * 128 + ((ca ^ (((q >> 1) & 1) << 2)) << 4) + 8 * (p & 1));
  // X halo row = 18 hr + kx + 8 (g >> 1) + 4 j + q: its swizzle bit depends on m = (18 hr + kx) mod 4 = (2 hr + kx) % 4
  unsigned b_lane[4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
    b_lane[m] = (unsigned)((8 * (g >> 1) + q) * 128 + ((cb ^ ((((m + q) >> 1) & 1) << 2)) << 4) + 8 * (p & 1));

  floatx16 acc[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  floatx16 accb;
#pragma unroll
  for (int e = 0; e < 16; ++e) accb[e] = 0.f;
  const bool do_bias = BIAS && ci0 == 0 && wci == 0;   // wave-uniform
  const bf16x8_t ones = __builtin_bit_cast(bf16x8_t, wh_v8s_t{0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80,
                                                             0x3f80, 0x3f80});

  const wh_lds_char_t* lds = (const wh_lds_char_t*)smem;
  const wh_lds_char_t* pa = lds + a_lane;
  const wh_lds_char_t* pb[4] = {lds + b_lane[0], lds + b_lane[1], lds + b_lane[2], lds + b_lane[3]};
  auto compute = [&](int sb) __attribute__((always_inline)) {
    const int so = sb * WH_STAGE;
    const wh_lds_char_t* qa = pa + so;
    const wh_lds_char_t* qb[4] = {pb[0] + so, pb[1] + so, pb[2] + so, pb[3] + so};
    auto rdA = [&](int r) __attribute__((always_inline)) -> bf16x8_t {
      const wh_lds_char_t* ad = qa + r * 16 * 128;
      return wh_cat(wh_tr(ad), wh_tr(ad + 4 * 128));
    };
    auto rdB = [&](int hr, int kx) __attribute__((always_inline)) -> bf16x8_t {
      const wh_lds_char_t* ad = qb[(2 * hr + kx) & 3] + (WH_DY_B + (WH_HWD * hr + kx) * 128);
      return wh_cat(wh_tr(ad), wh_tr(ad + 4 * 128));
    };
    bf16x8_t ar[4], br[2][3];   // A ring of 4: row hr + 1 is read while row hr - 2 still feeds ky = 2
    br[0][0] = rdB(0, 0); br[0][1] = rdB(0, 1); br[0][2] = rdB(0, 2);
    ar[0] = rdA(0);
#pragma unroll
    for (int hr = 0; hr < WH_TR + 2; ++hr) {
      const int cur = hr & 1;
      if (hr + 1 < WH_TR + 2) {   // the next halo row's fragments ahead of this row's MFMAs
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) br[cur ^ 1][kx] = rdB(hr + 1, kx);
        if (hr + 1 < WH_TR) ar[(hr + 1) & 3] = rdA(hr + 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((VAR & 1) != 0) __builtin_amdgcn_s_setprio(1);
      if (hr < WH_TR && do_bias)
        accb = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[hr & 3], ones, accb, 0, 0, 0);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int r = hr - ky;
        if (r >= 0 && r < WH_TR) {
#pragma unroll
          for (int kx = 0; kx < 3; ++kx)
            acc[ky][kx] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[r & 3], br[cur][kx], acc[ky][kx], 0, 0, 0);
        }
      }
      if constexpr ((VAR & 1) != 0) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  if constexpr ((VAR & 2) != 0) {
    if (orig >= 256 && orig < 512) __builtin_amdgcn_s_sleep(72);
  }
  if (t0 < t1) {
    dma(t0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int tt = t0; tt < t1; ++tt) {
      const int sb = (tt - t0) & 1;
      if (tt + 1 < t1) dma(tt + 1, sb ^ 1);
      compute(sb);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  // ---- partial planes: D[m = Cout][n = Cin], lane column n = lane & 31, row m = (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
  const long long plane = (long long)a.Cg * a.Kg;
  float* base = a.ws + (long long)split * plane;
  const int ci = ci0 + 32 * wci + (lane & 31);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int co = co0 + 32 * wco + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
    float* row = base + (long long)co * a.Kg;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) row[(ky * 3 + kx) * a.Cin + ci] = acc[ky][kx][e];
    if (do_bias && (lane & 31) == 0) row[a.Ktot] = accb[e];
  }
}

// The layer rules (shapes only, so the choice never depends on where the allocator put the operands): bf16, 3x3,
// stride 1, pad 1, sources at full resolution (one, or a concat A ++ B: each Cin tile reads one source through a
// resource of its own), Ca, Cb and Cout multiples of 64, 8-channel-aligned views, every buffer resource under 2^31
// bytes.
bool wgrad_hwc_shape_ok(const hiseg_conv2d_desc* d) {
  const char* e = getenv("HISEG_WGRAD_HWC");
  if (e && atoi(e) == 0) return false;
  if (d->dtype != HISEG_BF16 || d->convT || d->a_up != 1) return false;
  if (d->KH != 3 || d->KW != 3 || d->stride != 1 || d->pad != 1 || d->Ho != d->H || d->Wo != d->W) return false;
  if (d->Ca % 64 || d->Cb % 64 || d->Cout % 64 || d->a_cstride % 8 || d->a_coff % 8) return false;
  if ((long long)d->N * d->H * d->W * d->a_cstride * 2 >= 0x7fffffffll) return false;
  if (d->Cb && (d->srcB == nullptr || d->b_cstride % 8 || d->b_coff % 8 ||
                (long long)d->N * d->H * d->W * d->b_cstride * 2 >= 0x7fffffffll))
    return false;
  return true;
}

// Split count of the layers this kernel takes: one round of two workgroups per CU (512 workgroups; two rounds of
// half the pixel tiles each measured no faster and doubled the partial planes), at most 256 splits (the reduce of a
// 64 -> 64 layer's 512 planes took longer than its weight gradient) and at least 4 pixel tiles per split.
int wgrad_hwc_splits(const hiseg_conv2d_desc* d) {
  const long long NT = (long long)d->N * ((d->H + WH_TR - 1) / WH_TR) * ((d->W + WH_TW - 1) / WH_TW);
  const int tiles = (d->Cout / 64) * ((d->Ca + d->Cb) / 64);
  long long sp = 512 / tiles;
  if (sp > 256) sp = 256;
  if (sp > NT / 4) sp = NT / 4;
  if (sp < 1) sp = 1;
  return (int)sp;
}

// 1 = launched, 0 = the layer does not qualify (the caller takes another kernel, with the same split count), <0 error.
// Any split count works (split s takes pixel tiles [s tps, (s + 1) tps); an empty split writes zeros).
int wgrad_hwc_try(const WgradArgs& a, hipStream_t s) {
  const hiseg_conv2d_desc& d = a.d;
  if (!wgrad_hwc_shape_ok(&d)) return 0;
  if (a.dy_cs % 8 || a.dy_coff % 8 || a.Cin != d.Ca + d.Cb) return 0;
  if (((long long)a.M * a.dy_cs + a.dy_coff + d.Cout) * 2 >= 0x7fffffffll) return 0;
  if (a.Kg < a.Ktot + (a.want_bias ? 1 : 0)) return 0;
  const int nwg = (d.Cout / 64) * (a.Cin / 64) * a.splits;
  auto launch = [&](auto kern) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, WH_LDS);
      attr = true;
    }
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(256), WH_LDS, s, a);
  };
  // default: the stagger (tools/wgrad_bench.py, same box, two alternating runs: 256 -> 256 0.819 vs 0.826 ms,
  // 128 -> 128 @128x96 0.850 vs 0.861; the raised MFMA priority alone or with it: no gain; profiles/r5_wgrad_hwc.txt)
  static const int var = [] { const char* e = getenv("HISEG_WGRAD_HWC_VAR"); return e ? atoi(e) : 2; }();
  switch (var) {
    case 1: a.want_bias ? launch(conv_wgrad_hwc_kernel<true, 1>) : launch(conv_wgrad_hwc_kernel<false, 1>); break;
    case 2: a.want_bias ? launch(conv_wgrad_hwc_kernel<true, 2>) : launch(conv_wgrad_hwc_kernel<false, 2>); break;
    case 3: a.want_bias ? launch(conv_wgrad_hwc_kernel<true, 3>) : launch(conv_wgrad_hwc_kernel<false, 3>); break;
    default: a.want_bias ? launch(conv_wgrad_hwc_kernel<true>) : launch(conv_wgrad_hwc_kernel<false>);
  }
  const int r = hiseg_check_launch("conv_wgrad_hwc");
  return r < 0 ? r : 1;
}

}  // namespace hiseg
