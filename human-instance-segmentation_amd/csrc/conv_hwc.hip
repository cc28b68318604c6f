// Halo-tiled 3x3 convolution, Cout-split waves (gfx950, bf16): the dominant class of the ROI head (256->256 /
// 128->128 / 128->256 3x3 layers, refinement.py:31-55 ResidualBlock, rgb.py:657-673).
//
// conv_hwr.hip gives each wave a 64 Cout x 128-pixel tile (half of the workgroup's 16 x 16 pixels), so every weight
// fragment is loaded from L2/L1 into registers by the two pixel waves of its Cout group, 4 KiB per wave per K step.
// Timing ablations of conv_hwr (tools/conv_bench.py, DIAG variants 110+, profiles/r5_hwr_ablation.txt): 0.79 ms on
// 256->256 @64x48 x 256 ROIs; without its MFMAs 0.55 ms, without the in-loop weight loads 0.63 ms, without the halo
// DMA 0.65, without both 0.54 (= the MFMA-only time): the vector-memory stream, three quarters of it the weight
// fragments, is what the MFMAs fail to hide.
//
// Here a wave owns 32 output channels of ALL 256 pixels of the tile: 2 x 16 accumulators of v_mfma_f32_16x16x32_bf16
// (the same 128 registers), 2 weight fragments (2 KiB) per K step instead of 4, and no fragment loaded twice in a
// workgroup -- half the weight traffic per FLOP.  The B side reads more LDS instead: per (32-channel slice, kx) the
// wave walks the 18 halo rows of its window once, each row's B fragment (16 pixels x 32 channels, one ds_read_b128)
// feeding the 3 ky taps x 2 Cout fragments it meets (output rows r - ky), so each fragment is read once per (slice,
// kx) and a slice costs 54 fragment reads per wave (6 per K step).  The weights of the three ky taps of a kx are
// loaded one (slice, kx) block ahead.  The halo of the next slice is LDS-DMA'd during the first two kx blocks of a
// slice into the other buffer; one barrier per slice.
//
// Per output element the accumulation order is conv_hwr's (slices in order; within a slice kx-major, ky inner; one
// 32-channel MFMA per (slice, tap)), so results equal conv_hwr / conv_hw variant 86 bit for bit.
//
// NW (waves = 32-Cout groups per workgroup): 4 -> 128 Cout x 256 pixels, two workgroups per CU; 8 -> 256 Cout x 256
// pixels, one workgroup per CU (the 256-Cout layers read each halo once instead of once per 128-Cout workgroup).
#include "conv_common.h"

namespace hiseg {

#ifndef HISEG_CONV_HWC_MT
#define HISEG_CONV_HWC_MT 3   // work items per multi-tile workgroup (variants 109 / 102)
#endif

typedef unsigned hc_u4 __attribute__((ext_vector_type(4)));
typedef unsigned hc_u2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void hc_lds_void;

__device__ __forceinline__ void hc_dma16(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, unsigned voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(__builtin_amdgcn_readfirstlane(lds_addr)), "v"(voff), "s"(rsrc) : "memory");
}

// ABL (DIAG builds only, timing ablations -- wrong results): bit 0 no weight loads after the prologue, bit 1 no halo
// DMA after the prologue, bit 2 no B-fragment LDS reads, bit 3 no slice barrier, bit 4 no MFMAs, bit 5 no epilogue
// (accumulators stored straight, unconverted)
// RP (NW 4): residual prefetch.  The workgroup takes 80 KiB of LDS instead of 64 (two per CU still fit the 160 KiB):
// the epilogue tile is bytes [0, 64K) and the two halo buffers sit at [56K, 80K) (X) and [32K, 56K) (Y), the last
// slice always in X.  The residual rows of tile rows 0..127 ([0, 32K), never a halo) are LDS-DMA'd during slice 0, rows
// 128..223 ([32K, 56K) = Y, free in the last slice) during the last slice in place of the (absent) next halo, and only
// rows 224..255 ([56K, 64K), inside X) after the last barrier -- while rows 0..223 are converted.  Without it the
// whole 64-KiB residual tile was fetched after the last barrier with every wave waiting on it.
// (Measured and not kept, same box, 256->256 @64x48 x 256 ROIs: weights loaded two kx blocks ahead, 0.698 vs 0.698 ms;
// a progressive epilogue storing each output row from the accumulators as soon as its last MFMA ran, 8-B stores
// straight to HBM, 0.728 vs 0.698 ms -- bit-identical both.)
// (Also measured and not kept: the halo pieces and the residual tile through registers -- buffer_load_dwordx4, then
// ds_write_b128 -- instead of LDS-DMA, 0.710 vs 0.695 ms.)
// ST: BatchNorm batch statistics of the output fused into the epilogue (train mode, the conv feeding a BatchNorm: no
// activation, no residual; advanced/normalization_comparison.py:181-182).  The epilogue's store loop already moves
// every bf16 output chunk through registers: each thread accumulates shifted sums of its 8 channels over the 16
// pixels it stores, the 4 threads of a chunk in a wave are Chan-merged in a fixed order, and each wave writes count,
// mean and M2 per channel as split (pixel tile, wave) of d.stats_partial [S][3][Cout] (S = hiseg_conv2d_stats_tiles),
// the layout hiseg_bn_finalize_n merges -- the separate statistics pass (one read of z) is gone.  (Measured first
// forms: statistics from the accumulators spilled 65 registers in the K loop, conv forward +15 %; a Welford update per
// pixel plus a cross-wave LDS merge and barrier, conv forward +6 %.)
// TWB (pixel blocks per workgroup): 1 -- the workgroup's NW waves are NW 32-Cout groups over one 16 x 16 pixel block
// (BCO = 32 NW); 2 -- NW / 2 Cout groups over two 16 x 16 blocks side by side (a 16 x 32 tile, one 18 x 34 halo per
// slice; BCO = 16 NW: the 64-Cout layers).  A wave's tile and loop are the same either way.
// BR (round 5): the BatchNorm backward reduction of the layer whose output gradient this data-gradient conv writes
// (d.bnb_partial, include/hiseg.h), from the same store loop as ST: each thread's 16 stored bf16 values g of its 8
// channels, g masked by the ReLU of that BatchNorm's forward (bnb_z * bnb_scale + bnb_shift > 0, bnb_z loaded beside
// the store), summed as g, g * xhat and xhat (xhat = (bnb_z - mean) * invstd); the wave's threads of one chunk are
// added in a fixed butterfly order and each wave writes one split [3][Cout] -- the reduction pass over (dy, z) is gone.
// R3 (variant 108, round 6): a ring of three halo buffers (72 KiB of LDS, two workgroups per CU still fit): slice
// sl + 2's halo is LDS-DMA'd during slice sl, so each slice's pieces have a whole slice more to land before the barrier
// that needs them.
template <int ACT, bool RES, int NW, bool UP = false, int ABL = 0, bool RP = false, bool ST = false, int TWB = 1,
          bool BR = false, bool R3 = false>
__global__ void __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) conv_hwc_kernel(ConvArgs a) {
  constexpr int NCG = NW / TWB;                      // Cout groups of 32
  constexpr int BCO = 32 * NCG, TM = 2, NR = 16;    // wave tile: 32 Cout x (16 rows x 16 columns)
  constexpr int TW = 16 * TWB, HWD = TW + 2;
  constexpr int NHR = 18 * HWD;                       // halo rows (pixels) of a slice
  constexpr int PPW = ((NHR + 15) / 16 + NW - 1) / NW;   // halo pieces (16 rows, 1 KiB) per wave per slice
  // pieces issued in kx block 0 (the rest in block 1); DIAG ABL 512: all in block 0, ABL 1024: issued at row 0
  constexpr int PH = (ABL & 512) ? PPW : (PPW + 1) / 2;
  constexpr int PROW = (ABL & 1024) ? 0 : 3;
  constexpr int HB = PPW * NW * 1024;                 // bytes of one halo buffer
  constexpr int NPX = 256 * TWB;                      // output pixels of the tile
  static_assert((NW == 4 || NW == 8) && (TWB == 1 || (TWB == 2 && NW == 4 && !RP)), "configuration");
  static_assert(!R3 || (NW == 4 && !RP && TWB == 1 && !ST && !BR), "R3: the plain / residual 128-Cout form");
  // halo pieces the last wave issues per slice (the fewest of any wave): the vmcnt bound that still waits for every
  // piece of an older slice
  constexpr int NPMIN = ((NHR + 15) / 16 - 1 - (NW - 1)) / NW + 1;
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wc = w % NCG, pb = w / NCG;   // the wave's 32-Cout group and 16-column pixel block

  // ---- XCD-major bijective remap; Cout tiles fastest (the tiles of one pixel block share its halo in L2)
  const int nco = d.Cout_pad / BCO;
  const int ntx = (d.W + TW - 1) / TW, nty = (d.H + 15) >> 4;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = orig & 7, loc = orig >> 3;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int co0 = (wg % nco) * BCO;
  int tl = wg / nco;
  const int tx = tl % ntx;
  tl /= ntx;
  const int ty = tl % nty;
  const int n = tl / nty;
  const int y0 = ty * 16, x0 = tx * TW;

  const unsigned OOB = 0x80000000u;   // >= num_records: loads return zeros
  const int nsl = a.Cin >> 5;         // 32-channel slices (even: Cin % 64 == 0)
  const int ncb = a.Cin >> 6;
  const __amdgpu_buffer_rsrc_t rF = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(d.weight_frag), (short)0, d.Cout_pad * 9 * a.Cin * 2, 0x00020000);
  constexpr int USH = UP ? 1 : 0;
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(d.srcA), (short)0, d.N * (d.H >> USH) * (d.W >> USH) * d.a_cstride * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(d.Cb ? d.srcB : d.srcA), (short)0, d.Cb ? d.N * d.H * d.W * d.b_cstride * 2 : 0, 0x00020000);

  // ---- A fragments (hiseg.ops.frag_pack): (16-row Cout tile ct, slice sl, tap) at
  // ((((ct * ncb + sl / 2) * 9 + tap) * 2 + sl % 2) * 64 + lane) * 16 B; the wave's two tiles are ct0, ct0 + 1
  const unsigned a_ct = (unsigned)((co0 + wc * 32) >> 4) * (unsigned)ncb * 18u * 1024u;
  const unsigned a_ct_step = (unsigned)ncb * 18u * 1024u;
  // the weights of taps (ky, kx), ky = 0..2, of slice sl: 6 loads (the wave-uniform part in the SGPR offset)
  auto load_blk = [&](hc_u4 (&af)[3][TM], int sl, int kx) __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const unsigned a_lane = a_ct + (unsigned)ln * 16u;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const unsigned so = __builtin_amdgcn_readfirstlane(
          (((unsigned)(sl >> 1) * 9u + (unsigned)(ky * 3 + kx)) * 2u + (unsigned)(sl & 1)) * 1024u);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[ky][i] = __builtin_amdgcn_raw_buffer_load_b128(rF, a_lane + (unsigned)i * a_ct_step, so, 0);
    }
  };

  // ---- halo layout (conv_hwr's): row hr = hy * 18 + hx (64 B = 32 channels), 16-B chunk c at slot c ^ swz(hx),
  // swz(hx) = 2 ((hx >> 2) & 1); conflict-free B-fragment reads for every column shift kx.  Piece p of wave w = halo
  // rows 16 (NW p + w) + lane / 4 (one LDS-DMA of 1 KiB).
  const unsigned lds_base = (unsigned)(uintptr_t)(hc_lds_void*)smem;
  // halo buffer of slice sl (byte offset in LDS)
  auto hbuf = [&](int sl) __attribute__((always_inline)) -> int {
    if constexpr (RP) return ((nsl - 1 - sl) & 1) ? 32 * 1024 : 56 * 1024;
    else if constexpr (R3) return (sl % 3) * HB;
    else return (sl & 1) * HB;
  };
  // source byte offset of halo piece p's lane at slice sl (src A: sl < Ca / 32; src B: the concatenated rest)
  auto piece_off = [&](int p, int sl) __attribute__((always_inline)) -> unsigned {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int hr = 16 * (NW * p + w) + (ln >> 2);
    const int hy = hr / HWD, hx = hr - HWD * hy;
    const int iy = y0 + hy - 1, ix = x0 + hx - 1;
    const bool ok = hr < NHR && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
    const int chunk = (ln & 3) ^ (((hx >> 2) & 1) << 1);
    const bool fb = 32 * sl >= d.Ca;
    const int cs = fb ? d.b_cstride : d.a_cstride, coff = fb ? d.b_coff + 32 * sl - d.Ca : d.a_coff + 32 * sl;
    if constexpr (UP) {
      const int ush = fb ? 0 : 1;
      return ok ? (unsigned)((((n * (d.H >> ush) + (iy >> ush)) * (d.W >> ush) + (ix >> ush)) * cs + coff + chunk * 8) * 2)
                : OOB;
    } else {
      return ok ? (unsigned)((((n * d.H + iy) * d.W + ix) * cs + coff + chunk * 8) * 2) : OOB;
    }
  };
  // Each piece's src-A offset at slice 0, computed once: a src-A slice adds 64 B (an out-of-tile lane keeps OOB +
  // 64 sl >= 2^31 > num_records).  The per-slice address arithmetic (a division by the halo width, three 32-bit
  // multiplies, the bounds tests: ~30 instructions per piece, issued between two MFMA rows) is gone from the K loop
  // for every src-A slice; src-B slices (the decoder's concatenated skip) keep it.
  unsigned pofA[PPW];
#pragma unroll
  for (int p = 0; p < PPW; ++p) pofA[p] = 16 * (NW * p + w) < NHR ? piece_off(p, 0) : OOB;
  auto halo_dma = [&](int p, int sl, int boff) __attribute__((always_inline)) {
    if (16 * (NW * p + w) >= NHR) return;   // a piece wholly past the halo (wave-uniform): nothing to load
    const bool fb = 32 * sl >= d.Ca;
    const unsigned off = fb ? piece_off(p, sl) : pofA[p] + 64u * (unsigned)sl;
    hc_dma16(fb ? rB : rA, lds_base + (unsigned)(boff + 1024 * (NW * p + w)), off);
  };
  const char* lds_c = reinterpret_cast<const char*>(smem);
  // B fragment of halo row r at column shift kx: pixels (r, kx + lane % 16), channels 8 (lane / 16) .. + 7
  auto rdB = [&](int ln, int boff, int kx, int r) __attribute__((always_inline)) -> hc_u4 {
    const int hx = (ln & 15) + kx + 16 * pb;
    return *reinterpret_cast<const hc_u4*>(lds_c + boff + (r * HWD + hx) * 64 +
                                           (((ln >> 4) ^ (((hx >> 2) & 1) << 1)) << 4));
  };

  floatx4 acc[TM][NR];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // ---- epilogue geometry (conv_hwr's): 256 pixel rows x BCO bf16, 16-B chunk c of row r at slot c ^ (r & SWM);
  // tile row r = pixel (y0 + r / 16, x0 + r % 16).  Residual piece q (RPI rows, 1 KiB) = rows RPI q .. + RPI - 1,
  // issued by wave q % NW as its piece k = q / NW.
  constexpr int EROWB = BCO * 2;
  constexpr int CPR = BCO / 8;        // 16-B chunks per row
  constexpr int RPI = 64 / CPR;       // rows per wave instruction
  constexpr int SWM = CPR - 1;
  constexpr int NRI = NPX / (RPI * NW);   // residual pieces per wave
  auto px_of = [&](int r) __attribute__((always_inline)) -> int {
    const int y = y0 + r / TW, x = x0 + r % TW;
    return (y < d.Ho && x < d.Wo) ? (n * d.Ho + y) * d.Wo + x : -1;
  };
  const __amdgpu_buffer_rsrc_t rR = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(RES ? d.residual : d.out), (short)0, RES ? a.M * d.r_cstride * 2 : 0, 0x00020000);
  auto res_dma = [&](int k) __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int c = ln % CPR;
    const int r = RPI * (w + NW * k) + ln / CPR;
    const int px = px_of(r);
    const unsigned off = px >= 0 ? (unsigned)((px * d.r_cstride + d.r_coff + co0 + ((c ^ (r & SWM)) * 8)) * 2) : OOB;
    hc_dma16(rR, lds_base + (unsigned)(RPI * (w + NW * k) * EROWB), off);
  };
  static_assert(!RP || (NW == 4 && NRI == 16), "residual prefetch layout: 128-Cout tiles");

  // ABL 64 / 128 (DIAG): the second workgroup of each CU in the first dispatch round starts half / a quarter of a
  // slice late, so the two workgroups sharing each SIMD reach their barriers and DMA waits out of phase
  if constexpr ((ABL & 192) != 0) {
    if (orig >= 256 && orig < 512) {
      if constexpr ((ABL & 64) != 0) __builtin_amdgcn_s_sleep(36);
      else __builtin_amdgcn_s_sleep(18);
    }
  }
  // ABL 2048 / 4096 (DIAG): the first round's workgroups start in 4 phases (by dispatch index), 0 .. 3 x ~3 / ~1.5 us
  // apart, so that the grid's epilogues (every workgroup's at once: an HBM burst) spread over time
  if constexpr ((ABL & 6144) != 0) {
    if (orig < 512) {
      const int ph = (orig >> 3) & 3;
      for (int i = 0; i < ((ABL & 2048) ? 2 : 1) * ph; ++i) __builtin_amdgcn_s_sleep(94);
    }
  }
  // ---- prologue: slice 0's halo, the weights of block (slice 0, kx 0)
  hc_u4 af[3][TM], an[3][TM];
#pragma unroll
  for (int p = 0; p < PPW; ++p) halo_dma(p, 0, hbuf(0));
  if constexpr (R3) {
    if (nsl > 1) {
#pragma unroll
      for (int p = 0; p < PPW; ++p) halo_dma(p, 1, hbuf(1));
    }
  }
  load_blk(af, 0, 0);
  if constexpr (R3) {   // slice 0's pieces (slice 1's, younger, may fly)
    if (nsl > 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(6 + NPMIN) : "memory");
    else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");    // the halo pieces (older than the 6 weight loads)
  }
  __syncthreads();

  // One (slice, kx) block: the next block's weights are loaded first; halo pieces of slice sl + 1 ride in blocks
  // kx 0 and 1; then the 18 halo rows, each B fragment read two rows ahead and used for the (up to) 3 ky taps x 2
  // Cout fragments whose output row r - ky lies in the tile.
  auto block = [&](int sl, auto kxc) __attribute__((always_inline)) {
    constexpr int KX = decltype(kxc)::value;
    const int buf = hbuf(sl);
    const bool more = sl + 1 < nsl;
    if ((ABL & 1) == 0 && (KX < 2 || more)) load_blk(an, KX < 2 ? sl : sl + 1, KX < 2 ? KX + 1 : 0);
    // This block's LDS-DMA pieces (the next slice's halo; RP: residual rows), issued after row 2's MFMAs.  The
    // compiler does not see the asm DMA in its vmcnt accounting, so a piece issued before its wait for a weight
    // fragment of this block would make that wait cover the weight loads issued at the start of this block (measured:
    // a stall per block); after row 2 every fragment of the block has been waited for, and the pieces get the rest of
    // this block to land (they are older than the next block's weight loads).
    auto pieces = [&]() __attribute__((always_inline)) {
      if constexpr ((ABL & 2) != 0) {
      } else if constexpr (R3 && KX < 2) {   // slice sl + 2's halo into the third buffer
        if (sl + 2 < nsl) {
#pragma unroll
          for (int p = KX * PH; p < (KX == 0 ? PH : PPW); ++p) halo_dma(p, sl + 2, hbuf(sl + 2));
        }
      } else if constexpr (KX < 2) {
        if (more) {
#pragma unroll
          for (int p = KX * PH; p < (KX == 0 ? PH : PPW); ++p) halo_dma(p, sl + 1, hbuf(sl + 1));
        } else if constexpr (RP && RES) {   // last slice: residual rows 128..223 into the free buffer Y
#pragma unroll
          for (int k = 8 + 3 * KX; k < 11 + 3 * KX; ++k) res_dma(k);
        }
      }
      if constexpr (RP && RES) {   // slice 0: residual rows 0..127 (pieces 0..7 of each wave: 3, 3, 2 per block)
        if (sl == 0) {
#pragma unroll
          for (int k = 3 * KX; k < (KX == 2 ? 8 : 3 * KX + 3); ++k) res_dma(k);
        }
      }
    };
    int ln = lane;
    asm volatile("" : "+v"(ln));
    hc_u4 bq[3];
    if constexpr ((ABL & 4) == 0) {
      bq[0] = rdB(ln, buf, KX, 0);
      bq[1] = rdB(ln, buf, KX, 1);
    } else {
      bq[0] = bq[1] = bq[2] = af[0][0];
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = 0; r < NR + 2; ++r) {
      if (r == PROW) {
        __builtin_amdgcn_s_setprio(0);
        pieces();
        __builtin_amdgcn_s_setprio(1);
      }
      if ((ABL & 4) == 0 && r + 2 < NR + 2) bq[(r + 2) % 3] = rdB(ln, buf, KX, r + 2);
      // keep row r + 2's fragment read ahead of row r's MFMAs (left alone, the scheduler sinks each read next to its
      // use, and every other row waits out an LDS latency)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int j = r - ky;
        if (j >= 0 && j < NR) {
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            if constexpr ((ABL & 16) == 0)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[ky][i]),
                                                                   __builtin_bit_cast(bf16x8_t, bq[r % 3]), acc[i][j], 0,
                                                                   0, 0);
            else
              acc[i][j][0] += __builtin_bit_cast(float, af[ky][i][0]) + __builtin_bit_cast(float, bq[r % 3][1]);
          }
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (KX == 2 && (ABL & 8) == 0) {
      if constexpr (R3) {
        // slice sl + 1's pieces were issued during slice sl - 1: older than this slice's 18 weight loads and its
        // slice-(sl + 2) pieces, which may fly
        if (sl + 2 < nsl) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(18 + NPMIN) : "memory");
        else if (more) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        if (more) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // every halo piece (the next weights may fly)
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();   // slice sl+1's halo is in LDS; every wave is done reading slice sl's buffer
    }
    if constexpr ((ABL & 1) == 0) {
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int i = 0; i < TM; ++i) af[ky][i] = an[ky][i];
    }
  };
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  using K2 = std::integral_constant<int, 2>;
  for (int sl = 0; sl < nsl; ++sl) {
    block(sl, K0{});
    block(sl, K1{});
    block(sl, K2{});
  }

  // ---- epilogue through LDS (conv_hwr's): 256 pixel rows x BCO bf16, 16-B chunk c of row r at slot c ^ (r & SWM);
  // the residual tile arrives there by LDS-DMA, each lane turns its accumulator quads into bf16 output quads in
  // place, whole rows leave by 16-B stores.  Tile row r = pixel (y0 + r / 16, x0 + r % 16).
  if constexpr ((ABL & 32) != 0) {
    float* o = reinterpret_cast<float*>(d.out) + (long long)wg * 64 * 64 * NW + t;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) o[(i * NR + j) * 64 * NW] = acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    return;
  }
  char* tile = reinterpret_cast<char*>(smem);
  if constexpr (RES && !RP) {
#pragma unroll
    for (int k = 0; k < NRI; ++k) res_dma(k);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else if constexpr (RES) {   // rows 224..255 (pieces 14, 15 of each wave), into buffer X now that it is free
    res_dma(14);
    res_dma(15);
  }
  // BR: this thread's 16 chunks of the BatchNorm input z (the rows and channels it will store), loaded now so their
  // latency overlaps the conversion and the barrier (in the store loop they cost more than the reduction pass saved)
  constexpr int NSTZ = NPX * CPR / (NW * 64);
  uint4 zpre[BR ? NSTZ : 1];
  if constexpr (BR) {
#pragma unroll
    for (int k = 0; k < NSTZ; ++k) {
      const int idx = t + NW * 64 * k;
      const int r = idx / CPR, c = idx % CPR;
      const int px = px_of(r), co = co0 + 8 * c;
      zpre[k] = (px >= 0 && co < d.Cout)
                    ? *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(d.bnb_z) +
                                                      (long long)px * d.bnb_z_cstride + d.bnb_z_coff + co)
                    : make_uint4(0u, 0u, 0u, 0u);
    }
  }
  floatx4 sc[TM], sh[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int cl = wc * 32 + i * 16 + (lane >> 4) * 4;
    const int cc = co0 + cl < d.Cout ? co0 + cl : 0;
    sc[i] = *reinterpret_cast<const floatx4*>(d.scale + cc);
    sh[i] = *reinterpret_cast<const floatx4*>(d.shift + cc);
  }
  // accumulator rows j0 .. j1 - 1 (tile rows 16 j + lane % 16) -> bf16 output quads in place
  auto convert = [&](auto j0c, auto j1c) __attribute__((always_inline)) {
    constexpr int J0 = decltype(j0c)::value, J1 = decltype(j1c)::value;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = J0; j < J1; ++j) {
        const int cl = wc * 32 + i * 16 + (lane >> 4) * 4;
        const int r = j * TW + 16 * pb + (lane & 15);
        char* q = tile + r * EROWB + ((((cl >> 3) ^ (r & SWM)) << 4) | ((cl & 4) << 1));
        const floatx4 ac = acc[i][j];
        float v[4];
        uint2 rv = make_uint2(0u, 0u);
        if constexpr (RES) rv = *reinterpret_cast<const uint2*>(q);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = ac[e] * sc[i][e] + sh[i][e];
          if constexpr (RES) v[e] += Quad<bf16_t>::get(rv, e);
          if constexpr (ACT == HISEG_ACT_RELU) v[e] = v[e] > 0.f ? v[e] : 0.f;
        }
        uint2 o;
        o.x = f2bf2(v[0], v[1]);
        o.y = f2bf2(v[2], v[3]);
        *reinterpret_cast<uint2*>(q) = o;
      }
  };
  if constexpr (RES && RP) {
    convert(std::integral_constant<int, 0>{}, std::integral_constant<int, 14>{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // rows 224..255 of the residual landed (every wave's pieces)
    convert(std::integral_constant<int, 14>{}, std::integral_constant<int, NR>{});
  } else {
    convert(std::integral_constant<int, 0>{}, std::integral_constant<int, NR>{});
  }
  __syncthreads();
  constexpr int NST = NPX * CPR / (NW * 64);   // NPX rows x CPR chunks over the workgroup's threads
  // ST: thread t stores chunk t % CPR (8 channels) of rows t / CPR + 16 k: 16 pixels of those channels pass through its
  // registers; it sums them shifted by its first valid value (shifted sums: no division in the loop, no cancellation
  // over 16 values), then the 4 threads of a chunk in the wave are Chan-merged (fixed order) and the wave writes its
  // partial as split (pixel tile, wave) -- no cross-wave merge, no extra barrier
  float sk[8], s1[8], s2[8];
  int sn = 0;
  float bfs[8], bfh[8], bmu[8], binv[8];
  if constexpr (BR) {
    static_assert(!RES && !ST && ACT == HISEG_ACT_NONE && NW == 4 && (CPR == 16 || CPR == 8), "fused BN backward");
    const int cb = co0 + 8 * (t % CPR);   // this thread's 8 channels (the same in every store-loop iteration)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int ch = cb + e < d.Cout ? cb + e : 0;
      bfs[e] = d.bnb_scale[ch];
      bfh[e] = d.bnb_shift[ch];
      bmu[e] = d.bnb_mean[ch];
      binv[e] = d.bnb_invstd[ch];
      sk[e] = s1[e] = s2[e] = 0.f;
    }
  }
  if constexpr (ST) {
    static_assert(!RES && ACT == HISEG_ACT_NONE && NW == 4, "fused statistics: the conv feeding a BatchNorm");
    static_assert(CPR == 16 || CPR == 8, "fused statistics: a wave's threads of one chunk are lanes CPR apart");
#pragma unroll
    for (int e = 0; e < 8; ++e) sk[e] = s1[e] = s2[e] = 0.f;
  }
  // All NST chunks leave LDS first (the accumulators are dead, their registers free), then go out by buffer stores
  // whose out-of-tile lanes carry an offset past num_records (dropped by the hardware): no LDS latency per store, no
  // branch, 32-bit offsets (conv_hwc_applies bounds the output span).
  uint4 sv[NST];
#pragma unroll
  for (int k = 0; k < NST; ++k) {
    const int idx = t + NW * 64 * k;
    const int r = idx / CPR, c = idx % CPR;
    sv[k] = *reinterpret_cast<const uint4*>(tile + r * EROWB + ((c ^ (r & SWM)) << 4));
  }
  const __amdgpu_buffer_rsrc_t rO = __builtin_amdgcn_make_buffer_rsrc(d.out, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int k = 0; k < NST; ++k) {
    const int idx = t + NW * 64 * k;
    const int r = idx / CPR, c = idx % CPR;
    const int px = px_of(r), co = co0 + 8 * c;
    const uint4 v = sv[k];
    __builtin_amdgcn_raw_buffer_store_b128(
        __builtin_bit_cast(hc_u4, v), rO,
        (px >= 0 && co < d.Cout) ? (unsigned)((px * d.o_cstride + d.o_coff + co) * 2) : OOB, 0, 0);
    if constexpr (BR) {
      if (px >= 0 && co < d.Cout) {
        const uint4 zq = zpre[BR ? k : 0];
        const unsigned wv[4] = {v.x, v.y, v.z, v.w}, zw[4] = {zq.x, zq.y, zq.z, zq.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float g0 = __builtin_bit_cast(float, (e & 1) ? (wv[e >> 1] & 0xffff0000u) : (wv[e >> 1] << 16));
          const float zf = __builtin_bit_cast(float, (e & 1) ? (zw[e >> 1] & 0xffff0000u) : (zw[e >> 1] << 16));
          const float g = (d.bnb_act == HISEG_ACT_RELU && !(zf * bfs[e] + bfh[e] > 0.f)) ? 0.f : g0;
          const float xh = (zf - bmu[e]) * binv[e];
          sk[e] += g;
          s1[e] = fmaf(g, xh, s1[e]);
          s2[e] += xh;
        }
      }
    }
    if constexpr (ST) {
      if (px >= 0) {
        const unsigned wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = __builtin_bit_cast(float, (e & 1) ? (wv[e >> 1] & 0xffff0000u) : (wv[e >> 1] << 16));
          if (sn == 0) sk[e] = x;
          const float dx = x - sk[e];
          s1[e] += dx;
          s2[e] = fmaf(dx, dx, s2[e]);
        }
        ++sn;
      }
    }
  }
  if constexpr (ST) {
    float nn = (float)sn, mu[8], q2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mu[e] = sn ? sk[e] + s1[e] / nn : 0.f;
      q2[e] = sn ? fmaxf(s2[e] - s1[e] * s1[e] / nn, 0.f) : 0.f;
    }
#pragma unroll
    for (int m = CPR; m < 64; m <<= 1) {   // lanes ^ CPR .. ^ 32: the wave's threads of the chunk
      const float nb = __shfl_xor(nn, m, 64);
      const float nt = nn + nb;
      const float fb = nt > 0.f ? nb / nt : 0.f, fab = nt > 0.f ? nn * nb / nt : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float mb = __shfl_xor(mu[e], m, 64), qb = __shfl_xor(q2[e], m, 64);
        const float dd = mb - mu[e];
        mu[e] += dd * fb;
        q2[e] += qb + dd * dd * fab;
      }
      nn = nt;
    }
    if (lane < CPR) {
      const long long C = d.Cout;
      float* part = a.d.stats_partial + ((long long)((n * nty + ty) * ntx + tx) * NW + w) * 3 * C;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ch = co0 + 8 * lane + e;
        part[ch] = nn;
        part[C + ch] = mu[e];
        part[2 * C + ch] = q2[e];
      }
    }
  }
  if constexpr (BR) {
#pragma unroll
    for (int m = CPR; m < 64; m <<= 1) {   // lanes ^ CPR .. ^ 32: the wave's threads of the chunk, fixed order
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sk[e] += __shfl_xor(sk[e], m, 64);
        s1[e] += __shfl_xor(s1[e], m, 64);
        s2[e] += __shfl_xor(s2[e], m, 64);
      }
    }
    if (lane < CPR) {
      const long long C = d.Cout;
      float* part = a.d.bnb_partial + ((long long)((n * nty + ty) * ntx + tx) * NW + w) * 3 * C;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ch = co0 + 8 * lane + e;
        if (ch < C) {
          part[ch] = sk[e];
          part[C + ch] = s1[e];
          part[2 * C + ch] = s2[e];
        }
      }
    }
  }
}

template <int ACT, bool RES, int NW, bool UP = false, int ABL = 0, bool RP = false, bool ST = false, int TWB = 1,
          bool BR = false, bool R3 = false>
static int launch_hwc(const ConvArgs& a, hipStream_t s) {
  const hiseg_conv2d_desc& d = a.d;
  constexpr int BCO = 32 * NW / TWB, TW = 16 * TWB;
  constexpr int PPW = ((18 * (TW + 2) + 15) / 16 + NW - 1) / NW;
  constexpr size_t halo2 = (size_t)2 * PPW * NW * 1024, epi = (size_t)256 * TWB * BCO * 2;
  const int tiles = d.N * ((d.H + 15) / 16) * ((d.W + TW - 1) / TW);
  const int nco = d.Cout_pad / BCO;
  const size_t halo = R3 ? halo2 / 2 * 3 : halo2;
  const size_t lds = RP ? (size_t)80 * 1024 : (halo > epi ? halo : epi);
  auto kern = conv_hwc_kernel<ACT, RES, NW, UP, ABL, RP, ST, TWB, BR, R3>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3(tiles * nco), dim3(NW * 64), lds, s, a);
  return hiseg_check_launch("conv_hwc");
}

// MT (variants 109 / 102, round 6): multi-tile workgroups.  conv_hwc_kernel's wave tile, slice loop and per-element
// accumulation order (so the outputs are bit-identical to it), but each workgroup walks MT work items (pixel tile x
// Cout tile) -- item wg, wg + G, wg + 2G, ... (G = the grid: at any moment the concurrent workgroups hold adjacent
// items, as in the one-tile grid) -- and the tile boundary is pipelined: during the last slice of a tile (odd, buffer
// 1) the NEXT tile's slice-0 halo is LDS-DMA'd into buffer 0 and its first weight block loaded, so the next tile
// starts without a prologue.  The epilogue therefore must not touch buffer 0: it runs in two halves of NPX / 2 rows
// through a 32-KiB region E at [HB, HB + 32K) (over buffer 1, free after the last slice; TWB 1 takes 56 KiB of LDS,
// TWB 2 the 80 KiB of its two buffers -- two workgroups per CU either way).  No fused statistics / residual prefetch / ring of three.
template <int ACT, bool RES, int TWB, int MT>
__global__ void __launch_bounds__(256, 2) conv_hwc_mt_kernel(ConvArgs a) {
  constexpr int NW = 4, NCG = NW / TWB;
  constexpr int BCO = 32 * NCG, TM = 2, NR = 16;
  constexpr int TW = 16 * TWB, HWD = TW + 2;
  constexpr int NHR = 18 * HWD;
  constexpr int PPW = ((NHR + 15) / 16 + NW - 1) / NW;
  constexpr int PH = (PPW + 1) / 2;
  constexpr int HB = PPW * NW * 1024;
  constexpr int NPX = 256 * TWB, HALF = NPX / 2;
  constexpr int EOFF = HB;
  static_assert(MT >= 2 && (TWB == 1 || TWB == 2), "multi-tile configuration");
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wc = w % NCG, pb = w / NCG;

  const int nco = d.Cout_pad / BCO;
  const int ntx = (d.W + TW - 1) / TW, nty = (d.H + 15) >> 4;
  const int total = d.N * nty * ntx * nco;   // work items
  const int G = gridDim.x;
  const int orig = blockIdx.x;
  const int q8 = G >> 3, r8 = G & 7, xcd = orig & 7, loc = orig >> 3;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;

  const unsigned OOB = 0x80000000u;
  const int nsl = a.Cin >> 5;
  const int ncb = a.Cin >> 6;
  const __amdgpu_buffer_rsrc_t rF = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(d.weight_frag), (short)0, d.Cout_pad * 9 * a.Cin * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(d.srcA), (short)0, d.N * d.H * d.W * d.a_cstride * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(d.Cb ? d.srcB : d.srcA), (short)0, d.Cb ? d.N * d.H * d.W * d.b_cstride * 2 : 0, 0x00020000);
  const unsigned a_ct_step = (unsigned)ncb * 18u * 1024u;

  // tile geometry of work item i (Cout tiles fastest, as conv_hwc_kernel's remap)
  struct Geo { int co0, n, y0, x0; unsigned a_ct; };
  auto geo = [&](int i) __attribute__((always_inline)) -> Geo {
    Geo g;
    g.co0 = (i % nco) * BCO;
    int tl = i / nco;
    g.x0 = (tl % ntx) * TW;
    tl /= ntx;
    g.y0 = (tl % nty) * 16;
    g.n = tl / nty;
    g.a_ct = (unsigned)((g.co0 + wc * 32) >> 4) * (unsigned)ncb * 18u * 1024u;
    return g;
  };
  auto load_blk = [&](hc_u4 (&af)[3][TM], unsigned a_ct, int sl, int kx) __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const unsigned a_lane = a_ct + (unsigned)ln * 16u;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const unsigned so = __builtin_amdgcn_readfirstlane(
          (((unsigned)(sl >> 1) * 9u + (unsigned)(ky * 3 + kx)) * 2u + (unsigned)(sl & 1)) * 1024u);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[ky][i] = __builtin_amdgcn_raw_buffer_load_b128(rF, a_lane + (unsigned)i * a_ct_step, so, 0);
    }
  };
  auto piece_off = [&](const Geo& g, int p, int sl) __attribute__((always_inline)) -> unsigned {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int hr = 16 * (NW * p + w) + (ln >> 2);
    const int hy = hr / HWD, hx = hr - HWD * hy;
    const int iy = g.y0 + hy - 1, ix = g.x0 + hx - 1;
    const bool ok = hr < NHR && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
    const int chunk = (ln & 3) ^ (((hx >> 2) & 1) << 1);
    const bool fb = 32 * sl >= d.Ca;
    const int cs = fb ? d.b_cstride : d.a_cstride, coff = fb ? d.b_coff + 32 * sl - d.Ca : d.a_coff + 32 * sl;
    return ok ? (unsigned)((((g.n * d.H + iy) * d.W + ix) * cs + coff + chunk * 8) * 2) : OOB;
  };
  const unsigned lds_base = (unsigned)(uintptr_t)(hc_lds_void*)smem;
  auto hbuf = [&](int sl) __attribute__((always_inline)) -> int { return (sl & 1) * HB; };
  unsigned pofA[PPW];
  auto set_pof = [&](const Geo& g) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < PPW; ++p) pofA[p] = 16 * (NW * p + w) < NHR ? piece_off(g, p, 0) : OOB;
  };
  auto halo_dma = [&](const Geo& g, int p, int sl, int boff) __attribute__((always_inline)) {
    if (16 * (NW * p + w) >= NHR) return;
    const bool fb = 32 * sl >= d.Ca;
    const unsigned off = fb ? piece_off(g, p, sl) : pofA[p] + 64u * (unsigned)sl;
    hc_dma16(fb ? rB : rA, lds_base + (unsigned)(boff + 1024 * (NW * p + w)), off);
  };
  // the next tile's slice-0 pieces (its offsets computed here, once per tile)
  auto halo_dma0 = [&](const Geo& g, int p) __attribute__((always_inline)) {
    if (16 * (NW * p + w) >= NHR) return;
    hc_dma16(rA, lds_base + (unsigned)(1024 * (NW * p + w)), piece_off(g, p, 0));
  };
  const char* lds_c = reinterpret_cast<const char*>(smem);
  auto rdB = [&](int ln, int boff, int kx, int r) __attribute__((always_inline)) -> hc_u4 {
    const int hx = (ln & 15) + kx + 16 * pb;
    return *reinterpret_cast<const hc_u4*>(lds_c + boff + (r * HWD + hx) * 64 +
                                           (((ln >> 4) ^ (((hx >> 2) & 1) << 1)) << 4));
  };

  floatx4 acc[TM][NR];
  constexpr int EROWB = BCO * 2;
  constexpr int CPR = BCO / 8;
  constexpr int RPI = 64 / CPR;
  constexpr int SWM = CPR - 1;
  constexpr int NRI = NPX / (RPI * NW);
  static_assert(HALF * EROWB == 32 * 1024 && EOFF + HALF * EROWB <= 80 * 1024 && 2 * HB <= 80 * 1024 && NRI % 2 == 0,
                "epilogue halves");
  const __amdgpu_buffer_rsrc_t rR = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(RES ? d.residual : d.out), (short)0, RES ? a.M * d.r_cstride * 2 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rO = __builtin_amdgcn_make_buffer_rsrc(d.out, (short)0, 0x7fffffff, 0x00020000);
  char* E = reinterpret_cast<char*>(smem) + EOFF;

  int item = wg;
  Geo g = geo(item);
  set_pof(g);
  hc_u4 af[3][TM], an[3][TM];
#pragma unroll
  for (int p = 0; p < PPW; ++p) halo_dma(g, p, 0, hbuf(0));
  load_blk(af, g.a_ct, 0, 0);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  __syncthreads();

#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // one loop over (tile, slice): the epilogue runs after each tile's last slice (a single loop level keeps the
  // compiler from hoisting per-slice scalars out of an outer tile loop -- SGPR spills)
  int it = 0, sl = 0;
  int nitem = item + G;
  bool has_next = 1 < MT && nitem < total;   // workgroup-uniform
  for (;;) {

    auto block = [&](int sl, auto kxc) __attribute__((always_inline)) {
      constexpr int KX = decltype(kxc)::value;
      const int buf = hbuf(sl);
      const bool more = sl + 1 < nsl;
      if (KX < 2 || more) load_blk(an, g.a_ct, KX < 2 ? sl : sl + 1, KX < 2 ? KX + 1 : 0);
      auto pieces = [&]() __attribute__((always_inline)) {
        if constexpr (KX < 2) {
          if (more) {
#pragma unroll
            for (int p = KX * PH; p < (KX == 0 ? PH : PPW); ++p) halo_dma(g, p, sl + 1, hbuf(sl + 1));
          } else if (has_next) {   // last slice (buffer 1): the next tile's slice 0 into buffer 0
            const Geo gn = geo(nitem);
#pragma unroll
            for (int p = KX * PH; p < (KX == 0 ? PH : PPW); ++p) halo_dma0(gn, p);
          }
        }
      };
      int ln = lane;
      asm volatile("" : "+v"(ln));
      hc_u4 bq[3];
      bq[0] = rdB(ln, buf, KX, 0);
      bq[1] = rdB(ln, buf, KX, 1);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int r = 0; r < NR + 2; ++r) {
        if (r == 3) {
          __builtin_amdgcn_s_setprio(0);
          pieces();
          __builtin_amdgcn_s_setprio(1);
        }
        if (r + 2 < NR + 2) bq[(r + 2) % 3] = rdB(ln, buf, KX, r + 2);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int j = r - ky;
          if (j >= 0 && j < NR) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[ky][i]),
                                                                 __builtin_bit_cast(bf16x8_t, bq[r % 3]), acc[i][j], 0,
                                                                 0, 0);
          }
        }
      }
      __builtin_amdgcn_s_setprio(0);
      if constexpr (KX == 2) {
        if (more) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // halo pieces (the next weights may fly)
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (last slice: the next tile's slice-0 pieces)
        __syncthreads();
      }
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int i = 0; i < TM; ++i) af[ky][i] = an[ky][i];
    };
    using K0 = std::integral_constant<int, 0>;
    using K1 = std::integral_constant<int, 1>;
    using K2 = std::integral_constant<int, 2>;
    block(sl, K0{});
    block(sl, K1{});
    block(sl, K2{});
    if (++sl < nsl) continue;

    // ---- epilogue in two halves through E (buffer 0 holds the next tile's slice-0 halo).  Its lane-derived addresses
    // come from an opaque copy of the lane id, so the compiler cannot hoist them out of the tile loop (live registers)
    int eln = lane;
    asm volatile("" : "+v"(eln));
    const int et = w * 64 + eln;
    auto px_of = [&](int r) __attribute__((always_inline)) -> int {
      const int y = g.y0 + r / TW, x = g.x0 + r % TW;
      return (y < d.Ho && x < d.Wo) ? (g.n * d.Ho + y) * d.Wo + x : -1;
    };
    floatx4 sc[TM], sh[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int cl = wc * 32 + i * 16 + (eln >> 4) * 4;
      const int cc = g.co0 + cl < d.Cout ? g.co0 + cl : 0;
      sc[i] = *reinterpret_cast<const floatx4*>(d.scale + cc);
      sh[i] = *reinterpret_cast<const floatx4*>(d.shift + cc);
    }
    constexpr int NST = NPX * CPR / (NW * 64);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if constexpr (RES) {
#pragma unroll
        for (int k = h * NRI / 2; k < (h + 1) * NRI / 2; ++k) {
          int ln = lane;
          asm volatile("" : "+v"(ln));
          const int c = ln % CPR;
          const int r = RPI * (w + NW * k) + ln / CPR;
          const int px = px_of(r);
          const unsigned off =
              px >= 0 ? (unsigned)((px * d.r_cstride + d.r_coff + g.co0 + ((c ^ (r & SWM)) * 8)) * 2) : OOB;
          hc_dma16(rR, lds_base + (unsigned)(EOFF + (RPI * (w + NW * k) - h * HALF) * EROWB), off);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = h * NR / 2; j < (h + 1) * NR / 2; ++j) {
          const int cl = wc * 32 + i * 16 + (eln >> 4) * 4;
          const int r = j * TW + 16 * pb + (eln & 15);
          char* q = E + (r - h * HALF) * EROWB + ((((cl >> 3) ^ (r & SWM)) << 4) | ((cl & 4) << 1));
          const floatx4 ac = acc[i][j];
          float v[4];
          uint2 rv = make_uint2(0u, 0u);
          if constexpr (RES) rv = *reinterpret_cast<const uint2*>(q);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = ac[e] * sc[i][e] + sh[i][e];
            if constexpr (RES) v[e] += Quad<bf16_t>::get(rv, e);
            if constexpr (ACT == HISEG_ACT_RELU) v[e] = v[e] > 0.f ? v[e] : 0.f;
          }
          uint2 o;
          o.x = f2bf2(v[0], v[1]);
          o.y = f2bf2(v[2], v[3]);
          *reinterpret_cast<uint2*>(q) = o;
        }
      __syncthreads();
      uint4 sv[NST / 2];
#pragma unroll
      for (int k = 0; k < NST / 2; ++k) {
        const int idx = et + NW * 64 * (k + h * NST / 2);
        const int r = idx / CPR, c = idx % CPR;
        sv[k] = *reinterpret_cast<const uint4*>(E + (r - h * HALF) * EROWB + ((c ^ (r & SWM)) << 4));
      }
#pragma unroll
      for (int k = 0; k < NST / 2; ++k) {
        const int idx = et + NW * 64 * (k + h * NST / 2);
        const int r = idx / CPR, c = idx % CPR;
        const int px = px_of(r), co = g.co0 + 8 * c;
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(hc_u4, sv[k]), rO,
            (px >= 0 && co < d.Cout) ? (unsigned)((px * d.o_cstride + d.o_coff + co) * 2) : OOB, 0, 0);
      }
      // the next tile's first weight block, in flight during the second half (its registers were free)
      if (h == 0 && has_next) load_blk(af, geo(nitem).a_ct, 0, 0);
      __syncthreads();   // E free again (next half; the next tile's slice-1 halo lands over it)
    }
    if (!has_next) break;
    item = nitem;
    g = geo(item);
    set_pof(g);
    sl = 0;
    ++it;
    nitem = item + G;
    has_next = it + 1 < MT && nitem < total;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
}

template <int ACT, bool RES, int TWB, int MT>
static int launch_hwc_mt(const ConvArgs& a, hipStream_t s) {
  const hiseg_conv2d_desc& d = a.d;
  constexpr int BCO = 128 / TWB, TW = 16 * TWB;
  constexpr int PPW = ((18 * (TW + 2) + 15) / 16 + 3) / 4;
  constexpr size_t hb = (size_t)PPW * 4 * 1024;   // one halo buffer; E = [hb, hb + 32K) over buffer 1
  constexpr size_t lds = 2 * hb > hb + 32 * 1024 ? 2 * hb : hb + 32 * 1024;
  const long long items = (long long)d.N * ((d.H + 15) / 16) * ((d.W + TW - 1) / TW) * (d.Cout_pad / BCO);
  const int grid = (int)((items + MT - 1) / MT);
  auto kern = conv_hwc_mt_kernel<ACT, RES, TWB, MT>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, s, a);
  return hiseg_check_launch("conv_hwc_mt");
}

template <int TWB, int MT>
static int launch_hwc_mt_act(const ConvArgs& a, hipStream_t s) {
  const bool res = a.d.residual != nullptr, relu = a.d.act == HISEG_ACT_RELU;
  return res ? (relu ? launch_hwc_mt<HISEG_ACT_RELU, true, TWB, MT>(a, s) : launch_hwc_mt<HISEG_ACT_NONE, true, TWB, MT>(a, s))
             : (relu ? launch_hwc_mt<HISEG_ACT_RELU, false, TWB, MT>(a, s)
                     : launch_hwc_mt<HISEG_ACT_NONE, false, TWB, MT>(a, s));
}

template <int NW, bool RP = false, int TWB = 1, bool R3 = false>
static int launch_hwc_nw(const ConvArgs& a, hipStream_t s) {
  const hiseg_conv2d_desc& d = a.d;
  if (d.a_up == 2)   // (conv_hwc_try checked the form)
    return launch_hwc<HISEG_ACT_RELU, false, NW, true, 0, false, false, TWB, false, R3>(a, s);
  const bool res = d.residual != nullptr, relu = d.act == HISEG_ACT_RELU;
  return res ? (relu ? launch_hwc<HISEG_ACT_RELU, true, NW, false, 0, RP, false, TWB, false, R3>(a, s)
                     : launch_hwc<HISEG_ACT_NONE, true, NW, false, 0, RP, false, TWB, false, R3>(a, s))
             : (relu ? launch_hwc<HISEG_ACT_RELU, false, NW, false, 0, false, false, TWB, false, R3>(a, s)
                     : launch_hwc<HISEG_ACT_NONE, false, NW, false, 0, false, false, TWB, false, R3>(a, s));
}

// Whether variant `variant` takes the layer (the layer rules are conv_hwr_try's: the same operands, weight fragments and
// halo; with d.stats_partial the fused-statistics form: variant 104 / 107, no activation, no residual).
static bool conv_hwc_applies(const ConvArgs& a, int variant) {
  const hiseg_conv2d_desc& d = a.d;
  if (((variant < 104 || variant > 109) && variant != 102) || d.weight_frag == nullptr) return false;
  // 109 / 102: the multi-tile workgroups (no upsampled source, no fused statistics / BatchNorm-backward reduction)
  if ((variant == 109 || variant == 102) && (d.a_up != 1 || d.stats_partial || d.bnb_partial)) return false;
  if (d.dtype != HISEG_BF16 || d.out_dtype != HISEG_BF16) return false;
  if ((d.a_up != 1 && d.a_up != 2) || d.in_scale != nullptr || d.convT || d.mul != nullptr || d.out2 != nullptr)
    return false;
  if (d.KH != 3 || d.KW != 3 || d.stride != 1 || d.pad != 1 || d.Ho != d.H || d.Wo != d.W) return false;
  if (d.act != HISEG_ACT_NONE && d.act != HISEG_ACT_RELU) return false;
  if (d.Ca % 32 != 0 || d.Cb % 32 != 0 || (d.Ca + d.Cb) % 64 != 0 || d.Ca < 64 || d.K_pad != 9 * (d.Ca + d.Cb))
    return false;
  if ((d.a_cstride | d.a_coff) & 7) return false;
  if (d.Cb && (d.srcB == nullptr || ((d.b_cstride | d.b_coff) & 7))) return false;
  if ((d.Cout & (variant == 105 ? 255 : (variant == 107 || variant == 102) ? 63 : 127)) || d.Cout_pad != d.Cout ||
      ((d.o_cstride | d.o_coff) & 7) ||
      (d.residual && ((d.r_cstride | d.r_coff) & 7)))
    return false;
  if ((((uintptr_t)d.scale | (uintptr_t)d.shift | (uintptr_t)d.out | (uintptr_t)d.residual |
        (uintptr_t)d.weight_frag) & 15))
    return false;
  const long long span_a = (long long)d.N * (d.H / d.a_up) * (d.W / d.a_up) * d.a_cstride * 2;
  const long long span_b = d.Cb ? (long long)d.N * d.H * d.W * d.b_cstride * 2 : 0;
  const long long span_w = (long long)d.Cout_pad * d.K_pad * 2;
  const long long span_r = d.residual ? (long long)a.M * d.r_cstride * 2 : 0;
  const long long span_o = (long long)a.M * d.o_cstride * 2;   // the epilogue's 32-bit buffer-store offsets
  if (span_a >= 0x7fffffffll || span_b >= 0x7fffffffll || span_w >= 0x7fffffffll || span_r >= 0x7fffffffll ||
      span_o >= 0x7fffffffll)
    return false;
  if ((long long)d.N * d.H * d.W >= (1ll << 29)) return false;
  // upsampled src A: the smp decoder conv1 form only (ReLU, or no activation when the conv feeds a train-mode BN)
  if (d.a_up == 2 && (d.residual || d.act != (d.stats_partial ? HISEG_ACT_NONE : HISEG_ACT_RELU))) return false;
  if (d.stats_partial && ((variant != 104 && variant != 107) || d.residual || d.act != HISEG_ACT_NONE)) return false;
  if (d.bnb_partial &&
      ((variant != 104 && variant != 107) || d.residual || d.act != HISEG_ACT_NONE || d.stats_partial || d.a_up != 1 ||
       d.bnb_z == nullptr || ((d.bnb_z_cstride | d.bnb_z_coff) & 7) || ((uintptr_t)d.bnb_z & 15) ||
       !d.bnb_scale || !d.bnb_shift || !d.bnb_mean || !d.bnb_invstd ||
       (d.bnb_act != HISEG_ACT_RELU && d.bnb_act != HISEG_ACT_NONE)))
    return false;
  return true;
}

// BatchNorm statistics partials the automatic choice would fuse into this layer's epilogue (0: none): the pixel tiles
int conv_hwc_stats_tiles(const ConvArgs& a) {
  ConvArgs b = a;
  float dummy;
  if (b.d.bnb_partial == nullptr) b.d.stats_partial = &dummy;   // (a data gradient with bnb_partial: that form)
  const int tw = conv_hwc_applies(b, 104) ? 16 : conv_hwc_applies(b, 107) ? 32 : 0;
  if (tw == 0) return 0;
  return a.d.N * ((a.d.H + 15) / 16) * ((a.d.W + tw - 1) / tw) * 4;   // (pixel tile, wave) splits
}

// 1 = launched, 0 = the layer does not qualify (caller falls back), <0 on error.  Variant 104: 128-Cout workgroups
// (four waves, two per CU); 105: 256-Cout workgroups (eight waves, one per CU; Cout a multiple of 256); 106: 104 with
// the residual prefetch (RP); 107: 64-Cout workgroups over 16 x 32-pixel tiles (TWB 2; Cout a multiple of 64).  The layer
// rules are conv_hwr_try's (the same operands, weight fragments and halo).
int conv_hwc_try(const ConvArgs& a, hipStream_t s, int variant) {
  const hiseg_conv2d_desc& d = a.d;
#ifdef HISEG_DIAG
  if (variant >= 150 && variant < 4300) {   // timing ablations of variant 104 (res + ReLU only; output buffer as
                                          // scratch: the ABL 32 store writes one float per thread and MFMA row)
    if (d.weight_frag == nullptr || !d.residual || d.act != HISEG_ACT_RELU || d.a_up != 1 || d.Cout % 128) return 0;
    int r;
    switch (variant - 150) {
      case 1: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 1>(a, s); break;
      case 2: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 2>(a, s); break;
      case 3: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 3>(a, s); break;
      case 4: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 4>(a, s); break;
      case 8: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 8>(a, s); break;
      case 15: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 15>(a, s); break;
      case 16: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 16>(a, s); break;
      case 32: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 32>(a, s); break;
      case 47: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 47>(a, s); break;
      case 64: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 64>(a, s); break;
      case 128: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 128>(a, s); break;
      case 512: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 512>(a, s); break;
      case 1024: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 1024>(a, s); break;
      case 1536: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 1536>(a, s); break;
      case 2048: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 2048>(a, s); break;
      case 4096: r = launch_hwc<HISEG_ACT_RELU, true, 4, false, 4096>(a, s); break;
      default: return 0;
    }
    return r < 0 ? r : 1;
  }
#endif
  if (!conv_hwc_applies(a, variant)) return 0;
  if (d.bnb_partial) {   // the fused BatchNorm-backward reduction (variants 104 / 107; conv_hwc_applies checked it)
    const int r = variant == 107 ? launch_hwc<HISEG_ACT_NONE, false, 4, false, 0, false, false, 2, true>(a, s)
                                 : launch_hwc<HISEG_ACT_NONE, false, 4, false, 0, false, false, 1, true>(a, s);
    return r < 0 ? r : 1;
  }
  if (d.stats_partial) {   // the fused-statistics epilogue (variants 104 / 107; conv_hwc_applies checked the form)
    int r;
    if (variant == 107)
      r = d.a_up == 2 ? launch_hwc<HISEG_ACT_NONE, false, 4, true, 0, false, true, 2>(a, s)
                      : launch_hwc<HISEG_ACT_NONE, false, 4, false, 0, false, true, 2>(a, s);
    else
      r = d.a_up == 2 ? launch_hwc<HISEG_ACT_NONE, false, 4, true, 0, false, true>(a, s)
                      : launch_hwc<HISEG_ACT_NONE, false, 4, false, 0, false, true>(a, s);
    return r < 0 ? r : 1;
  }
  const int r = variant == 109 ? launch_hwc_mt_act<1, HISEG_CONV_HWC_MT>(a, s)
              : variant == 102 ? launch_hwc_mt_act<2, HISEG_CONV_HWC_MT>(a, s)
              : variant == 107 ? launch_hwc_nw<4, false, 2>(a, s)
              : variant == 108 ? launch_hwc_nw<4, false, 1, true>(a, s)
              : variant == 105 ? launch_hwc_nw<8>(a, s)
              : variant == 106 ? launch_hwc_nw<4, true>(a, s)
                               : launch_hwc_nw<4>(a, s);
  return r < 0 ? r : 1;
}

}  // namespace hiseg
