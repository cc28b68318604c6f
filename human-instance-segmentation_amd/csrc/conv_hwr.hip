// Halo-tiled 3x3 convolution with register-streamed weights (gfx950, bf16): the dominant class of the ROI head
// (256->256 / 128->128 / 128->256 3x3 layers, refinement.py:31-55 ResidualBlock, rgb.py:657-673).
//
// conv_hw.hip streams the weights through a 4-stage LDS ring by LDS-DMA and synchronises the workgroup once per
// K stage of 32 (one tap of one 32-channel slice): 72 barriers and 144 weight pieces per wave for a 256-channel
// layer, 32 MFMAs per barrier.  Counters (profiles/r3_*): the MFMA pipe was busy about half of the kernel's
// cycles, the waves spending the rest issue-stalled or parked at the per-stage waits.  Here the weights never
// touch LDS: they are packed in MFMA A-fragment order (hiseg.ops.frag_pack: one 16-row x 32-k fragment = 1 KiB
// contiguous) and every wave loads its own four fragments per K step straight into registers with
// buffer_load_dwordx4 (fully coalesced; the two pixel waves of a Cout group read the same bytes, the second from
// L1), one K step ahead.  LDS holds only the activations: an 18 x 18 halo per 32-channel slice, double-buffered,
// written from registers (six 1 KiB pieces per wave per slice, loaded two taps before they are stored), so the
// workgroup synchronises once per slice -- 8 barriers for 256 channels, 288 MFMAs per barrier per wave.
//
// Tile: 128 Cout x 256 pixels (a 16 x 16 block of one image), 4 waves as 2 (Cout) x 2 (pixel rows 0-7 / 8-15),
// 64 x 128 per wave (4 x 8 accumulators of v_mfma_f32_16x16x32_bf16 in VGPRs), two workgroups per CU (64 KiB of
// LDS each: the halo buffers, then the LDS-staged epilogue of conv_hw).  K order: channel-major (slice, then its
// 9 taps), the same as conv_hw, so results equal conv_hw's bit for bit.
#include "conv_common.h"

namespace hiseg {

typedef unsigned hr_u4 __attribute__((ext_vector_type(4)));


__device__ __forceinline__ int hr_hswz(int r) { return ((r >> 2) & 1) << 1; }   // halo rows (any start)

__device__ __forceinline__ void hr_dma16(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, unsigned voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(__builtin_amdgcn_readfirstlane(lds_addr)), "v"(voff), "s"(rsrc) : "memory");
}

typedef __attribute__((address_space(3))) void hr_lds_void;

// SCH (schedule of a K step): bit 1 -- s_setprio 1 around the MFMA groups (the co-resident workgroup's wave yields
// its issue slots to them); bit 2 -- B-fragment reuse across ky (below).  Bit 0 is unused (an earlier interleaving
// of the B reads between the last group's MFMAs measured slower: the variant numbers stay for the A/B record).
// UP: src A is the nearest-x2 upsampled low-resolution map of an smp decoder conv1 (halo pixel (iy, ix) reads
// source pixel (iy / 2, ix / 2)); a template flag so the dominant class's code is untouched.
// WCO x TWB: waves along Cout (BCO = 64 WCO) x 16-column pixel blocks of the tile (TW = 16 TWB): (2, 1) is the
// 128-Cout x 16 x 16 workgroup of four waves; (1, 2) a 64-Cout x 16 x 32 workgroup of four waves (the 64-channel
// layers: every wave keeps the 64 x 128 wave tile); (2, 2) 128 Cout x 16 x 32 with eight waves.  The per-element
// accumulation order is the same for every configuration: results are bit-identical across them.
// ABL (DIAG builds only, timing ablations -- wrong results): bit 0 no A loads in the K loop, bit 1 no halo DMA after
// the prologue, bit 2 no B-fragment LDS reads after the prologue, bit 3 no slice barrier, bit 4 no MFMAs.
template <int ACT, bool RES, int SCH, bool UP = false, int WCO = 2, int TWB = 1, int ABL = 0>
__global__ void __launch_bounds__(WCO * TWB * 128, (WCO * TWB > 2) ? 1 : 2) conv_hwr_kernel(ConvArgs a) {
  constexpr int BCO = 64 * WCO, TM = 4, TN = 8;
  constexpr int TW = 16 * TWB, NPW = 2 * TWB, NW = WCO * NPW, HWD = TW + 2;
  constexpr int NHR = 18 * HWD;                          // halo rows (pixels) of a slice
  constexpr int PPW = ((NHR + 15) / 16 + NW - 1) / NW;   // halo pieces (16 rows, 1 KiB) per wave per slice
  constexpr int HB = PPW * NW * 1024;                    // bytes of one halo buffer
  constexpr int NPX = 16 * TW;                           // output pixels of the tile
  static_assert(PPW <= 12 && (WCO == 1 || WCO == 2) && (TWB == 1 || TWB == 2), "configuration");
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wco = w / NPW, wpx = w % NPW;   // pixel wave: tile rows 8 (wpx & 1) .. + 7, columns 16 (wpx >> 1) .. + 15

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

  // ---- A fragments: (Cout tile ct, slice sl, tap) at ((((ct * ncb + sl / 2) * 9 + tap) * 2 + sl % 2) * 64 + lane) * 16 B:
  // the lane / Cout-tile part in 4 VGPRs, the wave-uniform (slice, tap) part as the SGPR offset of the load
  // (recomputed per step from an opaque copy of the lane id: kept live across the unrolled slice, these loop
  // invariants -- with the halo and B-fragment bases below -- push the kernel past 256 registers and spill)
  const unsigned a_ct = (unsigned)((co0 + wco * 64) >> 4) * (unsigned)ncb * 18u * 1024u;
  const unsigned a_ct_step = (unsigned)ncb * 18u * 1024u;
  auto load_a = [&](hr_u4 (&af)[TM], int sl, int tap) __attribute__((always_inline)) {
    const unsigned so = __builtin_amdgcn_readfirstlane((((unsigned)(sl >> 1) * 9u + (unsigned)tap) * 2u + (unsigned)(sl & 1)) * 1024u);
#pragma unroll
    for (int i = 0; i < TM; ++i)
      af[i] = __builtin_amdgcn_raw_buffer_load_b128(rF, a_ct + (unsigned)i * a_ct_step + (unsigned)lane * 16u, so, 0);
  };

  // ---- halo layout: row hr = hy * 18 + hx (64 B = 32 channels), 16-B chunk c stored at slot c ^ swz(hx),
  // swz(hx) = 2 ((hx >> 2) & 1).  A B-fragment read (16 consecutive hx of one hy, 4 chunks) is conflict-free for
  // every column shift kx (checked for all hy / kx by brute force over the ds_read_b128 lane groups), and the
  // swizzle depends on the column only: a fragment's address is a per-lane base for its kx plus the row offset
  // (j + ky) * 1152 as the instruction's immediate -- no per-read address arithmetic.
  // Halo pieces: piece p (0..5) of wave w = halo rows hr = 16 (4p + w) + lane / 4, one LDS-DMA (1 KiB) each; lane l
  // lands at byte 16 l of the piece = row hr, slot l % 4, so it fetches chunk (l % 4) ^ swz(hr % 18).  Per piece,
  // once: the source pixel (-1 outside the image / past row 324) and that chunk.
  const unsigned lds_base = (unsigned)(uintptr_t)(hr_lds_void*)smem;
  auto halo_dma = [&](int p, int sl, int buf) __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int hr = 16 * (NW * p + w) + (ln >> 2);
    const int hy = hr / HWD, hx = hr - HWD * hy;
    const int iy = y0 + hy - 1, ix = x0 + hx - 1;
    const bool ok = hr < NHR && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
    const int chunk = (ln & 3) ^ (((hx >> 2) & 1) << 1);
    const bool fb = 32 * sl >= d.Ca;
    const int cs = fb ? d.b_cstride : d.a_cstride, coff = fb ? d.b_coff + 32 * sl - d.Ca : d.a_coff + 32 * sl;
    unsigned off;
    if constexpr (UP) {
      const int ush = fb ? 0 : 1;
      off = ok ? (unsigned)((((n * (d.H >> ush) + (iy >> ush)) * (d.W >> ush) + (ix >> ush)) * cs + coff + chunk * 8) * 2)
               : OOB;
    } else {
      off = ok ? (unsigned)((((n * d.H + iy) * d.W + ix) * cs + coff + chunk * 8) * 2) : OOB;
    }
    hr_dma16(fb ? rB : rA, lds_base + (unsigned)(buf * HB + 1024 * (NW * p + w)), off);
  };
  char* lds_c = reinterpret_cast<char*>(smem);
  // B fragment: pixel (tile row wpx*8 + j, column lane % 16) at tap (ky, kx), channels 8 (lane / 16) .. + 7:
  // halo row (wpx * 8 + j + ky, lane % 16 + kx)
  auto bsw = [&](int ln, int kx) __attribute__((always_inline)) -> int {
    const int hx = (ln & 15) + kx + 16 * (wpx >> 1);
    return ((wpx & 1) * TN * HWD + hx) * 64 + (((ln >> 4) ^ (((hx >> 2) & 1) << 1)) << 4);
  };
  auto rdB = [&](int ln, int buf, int tap, int j) __attribute__((always_inline)) -> hr_u4 {
    const int ky = tap / 3, kx = tap - 3 * (tap / 3);
    return *reinterpret_cast<const hr_u4*>(lds_c + bsw(ln, kx) + buf * HB + (j + ky) * HWD * 64);
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: slice 0's halo into buffer 0, the first A fragments
  constexpr int NBMAX = TN + 2;
  hr_u4 af[TM], bf[NBMAX];
#pragma unroll
  for (int p = 0; p < PPW; ++p) halo_dma(p, 0, 0);
  load_a(af, 0, 0);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // the halo pieces (older than the 4 A loads)
  __syncthreads();
#pragma unroll
  for (int k = 0; k < ((SCH & 4) ? TN + 2 : TN); ++k) bf[k] = rdB(lane, 0, 0, k);

  // One K step (slice sl, tap), Cout fragment by Cout fragment: A fragment i's 8 MFMAs, then (registers free) the
  // next step's fragment i is loaded into it; the last fragment's MFMAs replace the B fragments column by column
  // with the next tap's (the next slice's first tap's come after the slice barrier).  The halo of slice sl+1:
  // piece p by LDS-DMA at the end of tap p (p = 0..5), after that step's A loads -- vmcnt counts in issue order,
  // so a piece is first waited for (by the compiler's wait for an A fragment issued after it) two steps later;
  // before the slice barrier every wave's pieces have landed (vmcnt(4): only the next slice's A loads may stay).
  // REUSE (SCH & 4): steps run kx-major (step s: kx = s / 3, ky = s % 3), so the three ky steps of a kx read the
  // halo tile rows j + ky of ONE set of 10 B fragments (rows 0..9 of the wave's window) kept in registers: 10
  // fragment reads per three steps instead of 24 (conv_hw.hip's REUSE; the same accumulation order as its
  // variant 86).  Without it step s is tap s (ky-major, variant 82's order).
  constexpr bool REUSE = (SCH & 4) != 0;
  constexpr int NB = REUSE ? TN + 2 : TN;
  auto tap_of = [](int st) constexpr { return REUSE ? (st % 3) * 3 + st / 3 : st; };
  auto step = [&](int sl, auto tapc) __attribute__((always_inline)) {
    constexpr int st = decltype(tapc)::value;
    constexpr int KY = REUSE ? st % 3 : 0;          // B register shift of this step
    constexpr bool read_b = REUSE ? (KY == 2 && st < 8) : st < 8;
    const int buf = sl & 1;
    const bool more = sl + 1 < nsl;
    const int nsl_ = st < 8 ? sl : sl + 1, ntap = st < 8 ? tap_of(st + 1) : 0;
    const unsigned so = __builtin_amdgcn_readfirstlane(
        (((unsigned)(nsl_ >> 1) * 9u + (unsigned)ntap) * 2u + (unsigned)(nsl_ & 1)) * 1024u);
    const bool load_next = st < 8 || more;
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const unsigned a_lane = a_ct + (unsigned)ln * 16u;
    if constexpr ((SCH & 2) != 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if constexpr ((ABL & 16) == 0) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                               __builtin_bit_cast(bf16x8_t, bf[j + KY]), acc[i][j], 0, 0, 0);
      } else {
        acc[i][0][0] += __builtin_bit_cast(float, af[i][0]) + __builtin_bit_cast(float, bf[KY][1]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if ((ABL & 1) == 0 && load_next)
        af[i] = __builtin_amdgcn_raw_buffer_load_b128(rF, a_lane + (unsigned)i * a_ct_step, so, 0);
    }
    if constexpr ((SCH & 2) != 0) __builtin_amdgcn_s_setprio(0);
    if constexpr (read_b && (ABL & 4) == 0) {
      if constexpr (REUSE) {   // the next kx's window: rows 0..9 at column shift kx + 1
#pragma unroll
        for (int k = 0; k < NB; ++k) bf[k] = rdB(ln, buf, st / 3 + 1, k);
      } else {
#pragma unroll
        for (int j = 0; j < TN; ++j) bf[j] = rdB(ln, buf, st + 1, j);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (st < 6 && (ABL & 2) == 0) {   // pieces st, st + 6 of slice sl + 1's halo
      if (more) {
#pragma unroll
        for (int p = st; p < PPW; p += 6) halo_dma(p, sl + 1, buf ^ 1);
      }
    }
    if constexpr (st == 8) {
      if constexpr ((ABL & 8) == 0) {
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        __syncthreads();   // slice sl+1's halo is in LDS; every wave is done reading slice sl's buffer
      }
      if (more && (ABL & 4) == 0) {
#pragma unroll
        for (int k = 0; k < NB; ++k) bf[k] = rdB(ln, buf ^ 1, 0, k);
      }
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  using I5 = std::integral_constant<int, 5>;
  using I6 = std::integral_constant<int, 6>;
  using I7 = std::integral_constant<int, 7>;
  using I8 = std::integral_constant<int, 8>;
  for (int sl = 0; sl < nsl; ++sl) {
    step(sl, I0{}); step(sl, I1{}); step(sl, I2{}); step(sl, I3{}); step(sl, I4{});
    step(sl, I5{}); step(sl, I6{}); step(sl, I7{}); step(sl, I8{});
  }

  // ---- epilogue through LDS (conv_hw's): 256 pixel rows x 128 bf16, 16-B chunk c of row r at slot c ^ (r & 15);
  // the residual tile arrives there by LDS-DMA, each lane turns its accumulator quads into bf16 output quads in
  // place, whole rows leave by 16-B stores.  Tile row r = pixel (y0 + r / 16, x0 + r % 16).
  constexpr int EROWB = BCO * 2;
  constexpr int CPR = BCO / 8;        // 16 chunks per row
  constexpr int RPI = 64 / CPR;       // rows per wave instruction
  constexpr int SWM = CPR - 1;
  char* tile = reinterpret_cast<char*>(smem);
  auto px_of = [&](int r) __attribute__((always_inline)) -> int {
    const int y = y0 + r / TW, x = x0 + r % TW;
    return (y < d.Ho && x < d.Wo) ? (n * d.Ho + y) * d.Wo + x : -1;
  };
  if constexpr (RES) {
    const int nrec_r = a.M * d.r_cstride * 2;
    const __amdgpu_buffer_rsrc_t rR = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.residual), (short)0, nrec_r,
                                                                       0x00020000);
    constexpr int NRI = NPX / (RPI * NW);
    const int c = lane % CPR;
#pragma unroll
    for (int k = 0; k < NRI; ++k) {
      const int r = RPI * (w + NW * k) + lane / CPR;
      const int px = px_of(r);
      const unsigned off = px >= 0 ? (unsigned)((px * d.r_cstride + d.r_coff + co0 + ((c ^ (r & SWM)) * 8)) * 2) : OOB;
      hr_dma16(rR, lds_base + (unsigned)(RPI * (w + NW * k) * EROWB), off);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  floatx4 sc[TM], sh[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int cl = wco * TM * 16 + i * 16 + (lane >> 4) * 4;
    const int cc = co0 + cl < d.Cout ? co0 + cl : 0;
    sc[i] = *reinterpret_cast<const floatx4*>(d.scale + cc);
    sh[i] = *reinterpret_cast<const floatx4*>(d.shift + cc);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = wco * TM * 16 + i * 16 + (lane >> 4) * 4;
      const int r = ((wpx & 1) * TN + j) * TW + 16 * (wpx >> 1) + (lane & 15);
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
  __syncthreads();
  constexpr int NST = NPX * CPR / (NW * 64);   // NPX rows x CPR chunks over the workgroup's threads
#pragma unroll 4
  for (int k = 0; k < NST; ++k) {
    const int idx = t + NW * 64 * k;
    const int r = idx / CPR, c = idx % CPR;
    const int px = px_of(r), co = co0 + 8 * c;
    const uint4 v = *reinterpret_cast<const uint4*>(tile + r * EROWB + ((c ^ (r & SWM)) << 4));
    if (px >= 0 && co < d.Cout)
      *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(d.out) + (long long)px * d.o_cstride + d.o_coff + co) = v;
  }
}

template <int ACT, bool RES, int SCH, bool UP = false, int WCO = 2, int TWB = 1, int ABL = 0>
static int launch_hwr(const ConvArgs& a, hipStream_t s) {
  const hiseg_conv2d_desc& d = a.d;
  constexpr int BCO = 64 * WCO, TW = 16 * TWB, NW = WCO * 2 * TWB;
  constexpr int PPW = ((18 * (TW + 2) + 15) / 16 + NW - 1) / NW;
  constexpr size_t halo2 = (size_t)2 * PPW * NW * 1024, epi = (size_t)16 * TW * BCO * 2;
  const int tiles = d.N * ((d.H + 15) / 16) * ((d.W + TW - 1) / TW);
  const int nco = d.Cout_pad / BCO;
  const size_t lds = halo2 > epi ? halo2 : epi;
  auto kern = conv_hwr_kernel<ACT, RES, SCH, UP, WCO, TWB, ABL>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3(tiles * nco), dim3(NW * 64), lds, s, a);
  return hiseg_check_launch("conv_hwr");
}

template <int SCH>
static int launch_hwr_sch(const ConvArgs& a, hipStream_t s) {
  const hiseg_conv2d_desc& d = a.d;
  if constexpr (SCH == 6) {
    if (d.a_up == 2) return launch_hwr<HISEG_ACT_RELU, false, 6, true>(a, s);   // (conv_hwr_try checked the form)
  }
  const bool res = d.residual != nullptr, relu = d.act == HISEG_ACT_RELU;
  return res ? (relu ? launch_hwr<HISEG_ACT_RELU, true, SCH>(a, s) : launch_hwr<HISEG_ACT_NONE, true, SCH>(a, s))
             : (relu ? launch_hwr<HISEG_ACT_RELU, false, SCH>(a, s) : launch_hwr<HISEG_ACT_NONE, false, SCH>(a, s));
}

// the 16 x 32-pixel configurations (SCH 6): ReLU / none, residual or not, upsampled src A (decoder conv1 form)
template <int WCO>
static int launch_hwr_wide(const ConvArgs& a, hipStream_t s) {
  const hiseg_conv2d_desc& d = a.d;
  if (d.a_up == 2) return launch_hwr<HISEG_ACT_RELU, false, 6, true, WCO, 2>(a, s);
  const bool res = d.residual != nullptr, relu = d.act == HISEG_ACT_RELU;
  return res ? (relu ? launch_hwr<HISEG_ACT_RELU, true, 6, false, WCO, 2>(a, s)
                     : launch_hwr<HISEG_ACT_NONE, true, 6, false, WCO, 2>(a, s))
             : (relu ? launch_hwr<HISEG_ACT_RELU, false, 6, false, WCO, 2>(a, s)
                     : launch_hwr<HISEG_ACT_NONE, false, 6, false, WCO, 2>(a, s));
}

// 1 = launched, 0 = the layer does not qualify (caller falls back), <0 on error.  Variants 92..95 = SCH 0..3,
// 96 = SCH 4 (B reuse across ky), 97 = SCH 6 (reuse + priority); 100 = SCH 6 on 64-Cout x 16 x 32-pixel tiles
// (64-multiple Cout), 101 = SCH 6 on 128-Cout x 16 x 32-pixel tiles with eight waves.
int conv_hwr_try(const ConvArgs& a, hipStream_t s, int variant) {
  const hiseg_conv2d_desc& d = a.d;
#ifdef HISEG_DIAG
  if (variant >= 110 && variant < 142) {   // timing ablations of the automatic configuration (res + ReLU only)
    if (d.weight_frag == nullptr || !d.residual || d.act != HISEG_ACT_RELU || d.a_up != 1) return 0;
    int r;
    switch (variant - 110) {
      case 1: r = launch_hwr<HISEG_ACT_RELU, true, 6, false, 2, 1, 1>(a, s); break;
      case 2: r = launch_hwr<HISEG_ACT_RELU, true, 6, false, 2, 1, 2>(a, s); break;
      case 4: r = launch_hwr<HISEG_ACT_RELU, true, 6, false, 2, 1, 4>(a, s); break;
      case 8: r = launch_hwr<HISEG_ACT_RELU, true, 6, false, 2, 1, 8>(a, s); break;
      case 15: r = launch_hwr<HISEG_ACT_RELU, true, 6, false, 2, 1, 15>(a, s); break;
      case 16: r = launch_hwr<HISEG_ACT_RELU, true, 6, false, 2, 1, 16>(a, s); break;
      case 7: r = launch_hwr<HISEG_ACT_RELU, true, 6, false, 2, 1, 7>(a, s); break;
      case 3: r = launch_hwr<HISEG_ACT_RELU, true, 6, false, 2, 1, 3>(a, s); break;
      default: return 0;
    }
    return r < 0 ? r : 1;
  }
#endif
  if (!((variant >= 92 && variant <= 97) || variant == 100 || variant == 101) || d.weight_frag == nullptr) return 0;
  if (d.dtype != HISEG_BF16 || d.out_dtype != HISEG_BF16) return 0;
  if ((d.a_up != 1 && d.a_up != 2) || d.in_scale != nullptr || d.convT || d.mul != nullptr || d.out2 != nullptr)
    return 0;
  if (d.KH != 3 || d.KW != 3 || d.stride != 1 || d.pad != 1 || d.Ho != d.H || d.Wo != d.W) return 0;
  if (d.act != HISEG_ACT_NONE && d.act != HISEG_ACT_RELU) return 0;
  if (d.Ca % 32 != 0 || d.Cb % 32 != 0 || (d.Ca + d.Cb) % 64 != 0 || d.Ca < 64 || d.K_pad != 9 * (d.Ca + d.Cb))
    return 0;
  if ((d.a_cstride | d.a_coff) & 7) return 0;
  if (d.Cb && (d.srcB == nullptr || ((d.b_cstride | d.b_coff) & 7))) return 0;
  if ((d.Cout & (variant == 100 ? 63 : 127)) || d.Cout_pad != d.Cout || ((d.o_cstride | d.o_coff) & 7) ||
      (d.residual && ((d.r_cstride | d.r_coff) & 7)))
    return 0;
  if ((((uintptr_t)d.scale | (uintptr_t)d.shift | (uintptr_t)d.out | (uintptr_t)d.residual |
        (uintptr_t)d.weight_frag) & 15))
    return 0;
  const long long span_a = (long long)d.N * (d.H / d.a_up) * (d.W / d.a_up) * d.a_cstride * 2;
  const long long span_b = d.Cb ? (long long)d.N * d.H * d.W * d.b_cstride * 2 : 0;
  const long long span_w = (long long)d.Cout_pad * d.K_pad * 2;
  const long long span_r = d.residual ? (long long)a.M * d.r_cstride * 2 : 0;
  if (span_a >= 0x7fffffffll || span_b >= 0x7fffffffll || span_w >= 0x7fffffffll || span_r >= 0x7fffffffll) return 0;
  if ((long long)d.N * d.H * d.W >= (1ll << 29)) return 0;   // halo source pixel packed with its chunk in 31 bits
  // upsampled src A: the smp decoder conv1 form only (ReLU, no residual), automatic schedule (variant 97)
  if (d.a_up == 2 && (variant < 97 || d.residual || d.act != HISEG_ACT_RELU)) return 0;
  int r;
  switch (variant) {
    case 100: r = launch_hwr_wide<1>(a, s); break;
    case 101: r = launch_hwr_wide<2>(a, s); break;
    case 92: r = launch_hwr_sch<0>(a, s); break;
    case 93: r = launch_hwr_sch<1>(a, s); break;
    case 94: r = launch_hwr_sch<2>(a, s); break;
    case 95: r = launch_hwr_sch<3>(a, s); break;
    case 96: r = launch_hwr_sch<4>(a, s); break;
    default: r = launch_hwr_sch<6>(a, s); break;
  }
  return r < 0 ? r : 1;
}

}  // namespace hiseg
