// Wide-tile weight gradient on CDNA4 MFMA (gfx950, bf16): the ROI head's 128- and 256-channel 3x3 layers
// (refinement.py:31-55 ResidualBlock and the mask-grid blocks, trained by train_advanced.py:680-762).
//
// GEMM (include/hiseg_train.h, hiseg_conv2d_wgrad):  D[k][j] = sum_p X[p][k] * dY[p][j], contracted over pixels.
// train_conv.hip's conv_wgrad_tr_kernel runs it on 128 x 128 workgroup tiles with 64 x 64 wave tiles, two
// workgroups per CU: per 64-pixel stage every workgroup moves 32 KiB from L2 into LDS for 128 MFMAs per SIMD,
// 128 B/clk per CU at two workgroups -- twice an XCD's L2 share per CU -- and each MFMA needs 512 B of
// transposed LDS reads.  It held 0.28-0.30 of the bf16 peak on the 256-channel class (1.24 ms per launch vs
// 0.65 ms for the forward conv of the same FLOPs, profiles/r3_*).
//
// Here one 256-thread workgroup per CU computes a 256 (K) x 256 (C) tile (NW = 4; the kernel is written for
// BC = 128 and NW = 8 too, both measured slower): each wave a 128 x 128 quarter held in AGPRs (64 16x16
// accumulators), the operands of a 64-pixel stage as 128-column
// transposed-read images (the T10 (b) swizzle of conv_wgrad_tr_kernel: two for X, BC / 128 for dY) filled by
// LDS-DMA, a two-stage ring with one barrier per stage.  Per MFMA the L2 -> LDS traffic is a quarter of the
// 128 x 128 tile's and the LDS reads half (128 x 128 wave tiles), wave K-half wk reads X image wk only.
// Split-K over pixel blocks with f32 partial tiles, reduced by wgrad_reduce_kernel exactly as before; the
// per-lane source addressing (two sources, upsampled source A, GEMM-bias column, halo taps through
// out-of-range offsets) is conv_wgrad_tr_kernel's.  Results equal it up to f32 re-association (the same
// pixel partition into splits is not guaranteed: the split count follows this tile's grid).
#include <cstdlib>

#include "hiseg_train.h"
#include "wgrad_common.h"

namespace hiseg {

typedef short ww_v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) ww_v4s_t ww_lds_v4s_t;
typedef __attribute__((address_space(3))) void ww_lds_void_t;
typedef unsigned ww_v4u_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) ww_v4u_t ww_lds_v4u_t;

__device__ __forceinline__ unsigned ww_swz(int row, int ch) {
  return 256u * (unsigned)row + 16u * (unsigned)(ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ void ww_dma16(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, unsigned voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(lds_addr), "v"(voff), "s"(rsrc) : "memory");
}

__device__ __forceinline__ ww_v4s_t ww_tr(unsigned byte_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((ww_lds_v4s_t*)(uintptr_t)byte_addr);
}

// SHT 1: one source and 256-multiple Cin -- both 128-column X images of a K tile lie in the same tap (their channel
// offsets 128 apart, both valid or both not), so a row block's tap position, bounds and pixel offset are computed
// once for the two (the per-stage DMA address math was ~60 % of the wave's VALU instructions,
// profiles/r4_wgrad_counters.txt).  SHT 2, also stride 1, no upsampled source and Ho x Wo = H x W: the X and dY
// byte offsets of a row block advance by a uniform PB pixels' stride per stage, kept in registers -- the per-stage
// math is the two bounds compares.
// TOG: image-major ring (image m of stage s at (m STAGES + s) IMG, so the stage is address bit 14) and per-lane
// fragment-read addresses held in registers, flipped once per stage -- each LDS read is a register + an immediate
// k-step offset instead of a v_add per read
template <int BC, int NW, int PB, int STAGES, bool BPRE = false, int SHT = 0, bool TOG = false>
__global__ void __launch_bounds__(NW * 64, 1) conv_wgrad_wide_kernel(WgradArgs a) {
  constexpr int BK = 256;
  constexpr int KS = PB / 32;              // 32-pixel k-steps per stage
  constexpr int NXH = 2, NYH = BC / 128;   // 128-column images per stage
  constexpr int NI = PB / (4 * NW);        // DMA instructions per image per wave (4 rows each, PB rows)
  constexpr int NLW = NI * (NXH + NYH);    // DMA instructions per wave per stage
  constexpr int WCN = NW / 2;              // waves along C
  constexpr int WCOLS = BC / WCN;          // a wave's C columns
  constexpr int TM = 8, TN = WCOLS / 16;   // wave tile 128 (K) x WCOLS (C)
  constexpr int IMG = PB * 256;
  constexpr int STAGE = (NXH + NYH) * IMG;
  static_assert((BC == 128 || BC == 256) && (NW == 4 || NW == 8) && TN >= 1 && NI >= 1 && (KS == 1 || KS == 2) &&
                STAGES >= 2, "tile");
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wk = w / WCN, wc = w % WCN;
  // XCD-major bijective remap (conv_wgrad_tr_kernel's): the K / C tiles of one pixel split run on one XCD
  const int nkt = (a.Kg + BK - 1) / BK, nct = (a.Cg + BC - 1) / BC;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = orig & 7, loc = orig >> 3;
  const int wgi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int k0 = (wgi % nkt) * BK, j0 = ((wgi / nkt) % nct) * BC, split = wgi / (nkt * nct);
  // blocks_per_split counts 64-pixel blocks (wgrad_geometry); stages of PB pixels
  const int pb_begin = split * a.blocks_per_split * (64 / PB);
  const int nblocks = (a.M + PB - 1) / PB;
  int pb_end = pb_begin + a.blocks_per_split * (64 / PB);
  if (pb_end > nblocks) pb_end = nblocks;
  const int nit = pb_end > pb_begin ? pb_end - pb_begin : 0;

  // one buffer resource over both X sources from the lower address (the launcher checked the span)
  const char* const pa = reinterpret_cast<const char*>(d.srcA);
  const char* const pb = d.Cb ? reinterpret_cast<const char*>(d.srcB) : pa;
  const char* const xbase = pa < pb ? pa : pb;
  const unsigned dA = (unsigned)(pa - xbase), dB = (unsigned)(pb - xbase);
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(xbase), (short)0, 0x7fffffff,
                                                                       0x00020000);
  const __amdgpu_buffer_rsrc_t rY = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.dy), (short)0, 0x7fffffff,
                                                                       0x00020000);
  const unsigned OOB = 0x80000000u;

  // per-lane DMA state: instruction i of an image fills rows 4(w + 4i) .. +3; this lane row (lane >> 4), slot
  // lane & 15.  Packed to keep the 256-column tile's state in registers: xo = channel offset (-1: zero column),
  // xk = ky | kx << 4 | upsampling shift << 8 | source B << 9; yo = dY channel offset (-1: zero) | sub-pixel q << 28
  int xo[NXH][NI], xk[NXH][NI], yo[NYH][NI];
  int pn[NI], py[NI], px[NI], pp[NI];
  unsigned bias_lanes = 0;   // bit NI h + i: this lane's chunk of X image h, instruction i is the GEMM-bias column's
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int r = 4 * (w + NW * i) + (lane >> 4);
    const int c = (lane & 15) ^ (((r & 3) << 2) | ((r >> 2) & 3));
#pragma unroll
    for (int h = 0; h < NXH; ++h) {
      const int k = k0 + 128 * h + 8 * c;
      const int tap = k / a.Cin;
      const int ci = k - tap * a.Cin;
      const bool la = d.Cb == 0 || ci < d.Ca;
      xo[h][i] = k < a.Ktot ? (la ? d.a_coff + ci : d.b_coff + ci - d.Ca) : -1;
      const int kyv = tap / d.KW, kxv = tap - kyv * d.KW;
      xk[h][i] = kyv | (kxv << 4) | ((la && d.a_up == 2) ? 1 << 8 : 0) | (la ? 0 : 1 << 9);
      if (a.want_bias && k == a.Ktot) bias_lanes |= 1u << (NI * h + i);
    }
#pragma unroll
    for (int hh = 0; hh < NYH; ++hh) {
      const int j = j0 + 128 * hh + 8 * c;
      if (d.convT) {
        const int C = d.Cout >> 2, q = j / C;
        yo[hh][i] = j < d.Cout ? (a.dy_coff + (j - q * C)) | (q << 28) : -1;
      } else {
        yo[hh][i] = j < d.Cout ? a.dy_coff + j : -1;
      }
    }
    const int p = pb_begin * PB + r;
    pp[i] = p;
    px[i] = p % d.Wo;
    const int tt = p / d.Wo;
    py[i] = tt % d.Ho;
    pn[i] = tt / d.Ho;
  }
  // SHT 2: byte offsets of row block i's X source pixel (tap-shifted, image 0's channel) and dY pixel
  unsigned ob[NI], yb[NI];
  if constexpr (SHT == 2) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int kk = xk[0][i];
      const int toff = ((kk & 15) - d.pad) * d.W + ((kk >> 4) & 15) - d.pad;
      ob[i] = dA + 2u * (unsigned)xo[0][i] + 2u * (unsigned)(pp[i] + toff) * (unsigned)d.a_cstride;
      yb[i] = 2u * (unsigned)pp[i] * (unsigned)a.dy_cs;
    }
  }
  const unsigned ob_step = 2u * PB * (unsigned)d.a_cstride, yb_step = 2u * PB * (unsigned)a.dy_cs;
  const int adv_x = PB % d.Wo, adv_y = PB / d.Wo;
  const unsigned lds_base = (unsigned)(uintptr_t)(ww_lds_void_t*)smem;
  static_assert(!TOG || (STAGES == 2 && IMG == 16384 && BPRE && KS == 2), "toggled fragment addressing");
  auto img_off = [&](int s, int m) __attribute__((always_inline)) -> unsigned {
    return TOG ? (unsigned)((m * STAGES + s) * IMG) : (unsigned)(s * STAGE + m * IMG);
  };

  // DMA of a stage in 2 NI parts (part p: row block i = p / 2 of the X images if p is even, of the dY images if odd;
  // the odd part advances the row block's pixels), interleaved with the previous stage's MFMA rows so the DMA
  // issue (about 100 cycles per 1-KiB piece) hides under them
  auto issue_part = [&](int s, int p) __attribute__((always_inline)) {
    const int i = p >> 1;
    const unsigned row_base = 256u * (unsigned)(4 * (w + NW * i));
    if ((p & 1) == 0 && SHT == 2) {
      const int kk = xk[0][i];
      const int iy = py[i] - d.pad + (kk & 15);
      const int ix = px[i] - d.pad + ((kk >> 4) & 15);
      const bool ok = xo[0][i] >= 0 && pp[i] < a.M && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
      ww_dma16(rX, lds_base + img_off(s, 0) + row_base, ok ? ob[i] : OOB);
      ww_dma16(rX, lds_base + img_off(s, 1) + row_base, ok ? ob[i] + 256u : OOB);
    } else if ((p & 1) == 0 && SHT == 1) {
      const int kk = xk[0][i];
      const int iy = py[i] * d.stride - d.pad + (kk & 15);
      const int ix = px[i] * d.stride - d.pad + ((kk >> 4) & 15);
      const bool ok = pp[i] < a.M && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
      const int sh = (kk >> 8) & 1, Hs = d.H >> sh, Ws = d.W >> sh;
      const unsigned pix = (unsigned)(((pn[i] * Hs + (iy >> sh)) * Ws + (ix >> sh)) * d.a_cstride);
#pragma unroll
      for (int h = 0; h < NXH; ++h) {
        const unsigned offx = ok && xo[h][i] >= 0 ? dA + (pix + (unsigned)xo[h][i]) * 2u : OOB;
        ww_dma16(rX, lds_base + img_off(s, h) + row_base, offx);
      }
    } else if ((p & 1) == 0) {
#pragma unroll
      for (int h = 0; h < NXH; ++h) {
        const int kk = xk[h][i];
        const int iy = py[i] * d.stride - d.pad + (kk & 15);
        const int ix = px[i] * d.stride - d.pad + ((kk >> 4) & 15);
        const bool okx = xo[h][i] >= 0 && pp[i] < a.M && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
        const int sh = (kk >> 8) & 1, Hs = d.H >> sh, Ws = d.W >> sh;
        const bool fb = (kk >> 9) & 1;
        const unsigned offx = okx ? (fb ? dB : dA) + (unsigned)((((pn[i] * Hs + (iy >> sh)) * Ws + (ix >> sh)) *
                                                                  (fb ? d.b_cstride : d.a_cstride) + xo[h][i]) * 2)
                                  : OOB;
        ww_dma16(rX, lds_base + img_off(s, h) + row_base, offx);
      }
    } else {
#pragma unroll
      for (int hh = 0; hh < NYH; ++hh) {
        const int yv = yo[hh][i];
        const bool oky = yv >= 0 && pp[i] < a.M;
        int yp = pp[i];
        if (d.convT) {
          const int qq = (yv >> 28) & 3;
          yp = (pn[i] * (2 * d.Ho) + 2 * py[i] + (qq >> 1)) * (2 * d.Wo) + 2 * px[i] + (qq & 1);
        }
        unsigned offy = oky ? (unsigned)((yp * a.dy_cs + (yv & 0x0fffffff)) * 2) : OOB;
        if constexpr (SHT == 2) offy = oky ? yb[i] + 2u * (unsigned)yv : OOB;
        ww_dma16(rY, lds_base + img_off(s, NXH + hh) + row_base, offy);
      }
      if constexpr (SHT == 2) {
        ob[i] += ob_step;
        yb[i] += yb_step;
      }
      pp[i] += PB;
      px[i] += adv_x;
      py[i] += adv_y;
      if (px[i] >= d.Wo) { px[i] -= d.Wo; ++py[i]; }
      while (py[i] >= d.Ho) { py[i] -= d.Ho; ++pn[i]; }
    }
  };
  auto issue = [&](int s) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < 2 * NI; ++p) issue_part(s, p);
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // fragment reads: group g = lane >> 4 takes pixel rows 8g..8g+7 of a 32-pixel k-step; lane 4q+p of the group
  // addresses row q, columns 4p..4p+3 of its 16-column block
  const int g = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  // this wave's X image (K half wk) and dY image / column base
  const int yimg = (wc * WCOLS) / 128;
  const int ych0 = ((wc * WCOLS) % 128) / 8;

  // TOG: rows 8g + q (+ 4) of a k-step (k-step 1's rows 32 below: the swizzle repeats every 16 rows), channel pair
  // 2i (+ 1), this wave's X / dY image, stage 0
  unsigned oX[TOG ? TM : 1][2], oY[TOG ? TN : 1][2];
  if constexpr (TOG) {
#pragma unroll
    for (int hi = 0; hi < 2; ++hi) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        oX[i][hi] = lds_base + img_off(0, wk) + ww_swz(8 * g + q + 4 * hi, 2 * i + (pq >> 1)) + 8u * (pq & 1);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        oY[j][hi] = lds_base + img_off(0, NXH + yimg) + ww_swz(8 * g + q + 4 * hi, ych0 + 2 * j + (pq >> 1)) +
                    8u * (pq & 1);
    }
  }

#pragma unroll
  for (int s0 = 0; s0 < STAGES - 1; ++s0)
    if (s0 < nit) issue(s0);
  for (int it = 0; it < nit; ++it) {
    const int cur = it % STAGES;
    if (STAGES > 2 && it + STAGES - 2 < nit) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NLW * (STAGES - 2)) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (bias_lanes) {   // the GEMM-bias column: X = 1 in every row, written over the landed DMA zeros
#pragma unroll
      for (int h = 0; h < NXH; ++h)
#pragma unroll
        for (int i = 0; i < NI; ++i)
          if (bias_lanes & (1u << (NI * h + i)))
            *reinterpret_cast<ww_lds_v4u_t*>(
                (uintptr_t)(lds_base + img_off(cur, h) + 256u * (unsigned)(4 * (w + NW * i)) + 16u * (unsigned)lane)) =
                ww_v4u_t{0x3f80u, 0u, 0u, 0u};
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // stage it landed everywhere; every wave left stage it-1's buffer
    asm volatile("" ::: "memory");
    const int nxt = it + STAGES - 1;   // the stage whose DMA this iteration issues (into stage it-1's buffer)
    const bool more = nxt < nit;

    const unsigned sX = lds_base + img_off(cur, wk);
    const unsigned sY = lds_base + img_off(cur, NXH + yimg);
    // k-step 0 fragments, then per A row i: its MFMAs, after which af[i] takes row i of k-step 1 (the reads land
    // under the remaining rows' MFMAs); k-step 1's B fragments after the last row
    bf16x8_t af[TM], bfr[TN];
    auto rdA = [&](int ks, int i) __attribute__((always_inline)) -> bf16x8_t {
      if constexpr (TOG) {
        const ww_v4s_t lo = ww_tr(oX[i][0] + (unsigned)(ks * 32 * 256));
        const ww_v4s_t hi = ww_tr(oX[i][1] + (unsigned)(ks * 32 * 256));
        return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
      const int r0 = ks * 32 + 8 * g + q, ch = 2 * i + (pq >> 1);
      const ww_v4s_t lo = ww_tr(sX + ww_swz(r0, ch) + 8u * (pq & 1));
      const ww_v4s_t hi = ww_tr(sX + ww_swz(r0 + 4, ch) + 8u * (pq & 1));
      return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    auto rdB = [&](int ks, int j) __attribute__((always_inline)) -> bf16x8_t {
      if constexpr (TOG) {
        const ww_v4s_t lo = ww_tr(oY[j][0] + (unsigned)(ks * 32 * 256));
        const ww_v4s_t hi = ww_tr(oY[j][1] + (unsigned)(ks * 32 * 256));
        return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
      const int r0 = ks * 32 + 8 * g + q, ch = ych0 + 2 * j + (pq >> 1);
      const ww_v4s_t lo = ww_tr(sY + ww_swz(r0, ch) + 8u * (pq & 1));
      const ww_v4s_t hi = ww_tr(sY + ww_swz(r0 + 4, ch) + 8u * (pq & 1));
      return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = rdB(0, j);
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = rdA(0, i);
    if constexpr (BPRE && KS == 2) {
      // k-step 1's B fragments read into a second set during k-step 0's first rows (two per row), so k-step 1's
      // first MFMAs do not wait for them; A as before (row i of k-step 1 after row i of k-step 0)
      static_assert(TN <= 2 * TM, "B prefetch spread");
      bf16x8_t bnx[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        af[i] = rdA(1, i);
        if (2 * i < TN) bnx[2 * i] = rdB(1, 2 * i);
        if (2 * i + 1 < TN) bnx[2 * i + 1] = rdB(1, 2 * i + 1);
        if (more && i < 2 * NI) issue_part(nxt % STAGES, i);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bnx[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (TOG) {   // the next stage's buffer
#pragma unroll
        for (int hi = 0; hi < 2; ++hi) {
#pragma unroll
          for (int i = 0; i < TM; ++i) oX[i][hi] ^= (unsigned)IMG;
#pragma unroll
          for (int j = 0; j < TN; ++j) oY[j][hi] ^= (unsigned)IMG;
        }
      }
      continue;
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (ks + 1 < KS) af[i] = rdA(1, i);
        if (ks == 0 && more && i < 2 * NI) issue_part(nxt % STAGES, i);
      }
      if (ks + 1 < KS) {
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = rdB(1, j);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  float* ws = a.ws + (long long)split * a.Cg * a.Kg;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int k = k0 + wk * 128 + i * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int jj = j0 + wc * WCOLS + j * 16 + (lane & 15);
      if (k < a.Kg && jj < a.Cg) *reinterpret_cast<floatx4*>(ws + (long long)jj * a.Kg + k) = acc[i][j];
    }
  }
}

// HISEG_WGRAD_WIDE=0 keeps every layer on conv_wgrad_tr_kernel (A/B timing only)
static bool wide_mode() {
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("HISEG_WGRAD_WIDE");
    mode = e ? atoi(e) : 1;
  }
  return mode != 0;
}

// The wide tile for a layer: 256 or 128 (C tile), 0 when it does not apply.  bf16, 128-multiple GEMM columns
// (no ConvTranspose), the transposed-read kernel's alignment rules, every X source within one 2^31-byte buffer
// resource, and a K extent of at least two 128-column images.
int wgrad_wide_bc(const hiseg_conv2d_desc* d, int Cg, int Kg, int Cin, int M, int dy_cs, int dy_coff) {
  if (!wide_mode() || d->dtype != HISEG_BF16 || d->convT) return 0;
  if (Cg % 128 || Kg < 256) return 0;
  if (d->Ca % 8 || Cin % 8 || d->a_cstride % 8 || d->a_coff % 8) return 0;
  if (d->Cb && (d->b_cstride % 8 || d->b_coff % 8)) return 0;
  if (dy_cs >= 0 && (dy_cs % 8 || dy_coff % 8)) return 0;
  const long long span_a = (long long)d->N * d->H * d->W * d->a_cstride * 2;
  const long long span_b = d->Cb ? (long long)d->N * d->H * d->W * d->b_cstride * 2 : 0;
  if (span_a >= 0x7fffffffll || span_b >= 0x7fffffffll) return 0;
  if (dy_cs >= 0 && ((long long)M * dy_cs + dy_coff + Cg) * 2 >= 0x7fffffffll) return 0;
  if (d->Cb) {
    const long long pa = (long long)(uintptr_t)d->srcA, pb = (long long)(uintptr_t)d->srcB;
    const long long lo = pa < pb ? pa : pb;
    if (pa - lo + span_a >= 0x7fffffffll || pb - lo + span_b >= 0x7fffffffll || hiseg_force_far()) {
      if (dy_cs >= 0) hiseg_note_placement("wgrad_wide declined (sources far apart)", d);
      return 0;
    }
  }
  // (the 256 x 128 tile measured slower than the 128 x 128 kernel; so was this tile on Cin = 128: 128 -> 256 @64x48 x
  // 256 ROIs 1.078 vs 0.656 ms, its K tiles straddling two taps, profiles/r5_wgrad_hwc.txt)
  if (Cin % 256) return 0;
  return Cg % 256 == 0 ? 256 : 0;
}

template <int BC, int NW, int PB, int STAGES, bool BPRE = false, int SHT = 0, bool TOG = false>
static int wide_launch(const WgradArgs& a, hipStream_t s) {
  constexpr size_t lds = (size_t)STAGES * (2 + BC / 128) * PB * 256;
  auto kern = conv_wgrad_wide_kernel<BC, NW, PB, STAGES, BPRE, SHT, TOG>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  const int nwg = ((a.Kg + 255) / 256) * ((a.Cg + BC - 1) / BC) * a.splits;
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(NW * 64), lds, s, a);
  return hiseg_check_launch("conv_wgrad_wide");
}

// 1 = launched, 0 = the layer does not take the wide tile
int wgrad_wide_try(const WgradArgs& a, hipStream_t s) {
  const int bc = wgrad_wide_bc(&a.d, a.Cg, a.Kg, a.Cin, a.M, a.dy_cs, a.dy_coff);
  if (bc == 0) return 0;
  // four waves, one per SIMD, 128 x 128 wave tiles in AGPRs.  (Eight waves at two per SIMD with 128 x 64 wave tiles
  // spill 76 B per lane and ran 1.74 ms on the 256-channel class; this form 1.19 ms, conv_wgrad_tr_kernel 1.31 ms,
  // same box, tools/wgrad_bench.py.)
  // (32-pixel stages in a 4-deep ring, the same kernel at <256, 4, 32, 4>: 1.229 vs 1.212 ms, same box -- the
  // DMA lookahead is not what holds it at ~0.31 of peak)
  // k-step 1's B fragments prefetched during k-step 0 (1.2075 vs 1.2225 ms on the 256-channel class, same checksum;
  // HISEG_WGRAD_BPRE=0 restores the late reads for A/B timing)
  static const int bpre = [] { const char* e = getenv("HISEG_WGRAD_BPRE"); return e ? atoi(e) : 1; }();
  // (Counters, profiles/r4_wgrad_counters.txt: the MFMA pipe is busy 33 % of the kernel's cycles; per 64-pixel stage a
  // wave issues 128 MFMAs and ~270 other VALU, ~140 SALU, 64 LDS and 16 DMA instructions, and waits 26 % of its
  // cycles at s_waitcnt / the barrier and 29 % issue-stalled -- one wave per SIMD has no partner to fill them.  The
  // eight-wave form that would give it one still needs 256 VGPRs + 36 spilled for its 128 accumulators plus the
  // hoisted fragment / DMA addresses, as in round 3.)
  // Shared-tap DMA addressing (SHT above; HISEG_WGRAD_SHT=1 / 0 for A/B timing, read per call): 1.19 -> 1.12 (SHT 1)
  // -> 1.04 ms (SHT 2) on the 256-channel class, same checksum (profiles/r4_wgrad_sht.txt).  (Folding the fragment
  // reads' stage / k-step offsets into immediates -- image-major ring, stage loop unrolled by two -- spilled 104
  // VGPRs: the remaining one v_add per LDS read stays.)
  const char* e = getenv("HISEG_WGRAD_SHT");
  int sht = e ? atoi(e) : 2;
  if (a.d.Cb != 0 || a.Cin % 256 != 0) sht = 0;
  if (sht >= 2 && !(a.d.stride == 1 && a.d.a_up == 1 && a.d.Ho == a.d.H && a.d.Wo == a.d.W)) sht = 1;
  const char* et = getenv("HISEG_WGRAD_TOG");
  const bool tog = !(et && atoi(et) == 0);
  const int r = !bpre ? wide_launch<256, 4, 64, 2>(a, s)
              : sht >= 2 && tog ? wide_launch<256, 4, 64, 2, true, 2, true>(a, s)
              : sht >= 2 ? wide_launch<256, 4, 64, 2, true, 2>(a, s)
              : sht == 1 ? wide_launch<256, 4, 64, 2, true, 1>(a, s)
                         : wide_launch<256, 4, 64, 2, true>(a, s);
  return r < 0 ? r : 1;
}

}  // namespace hiseg
