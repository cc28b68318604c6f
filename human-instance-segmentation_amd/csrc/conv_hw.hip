// Halo-tiled wide convolution for 3x3 / stride 1 / pad 1 bf16 layers (gfx950): the wide-tile kernel's
// MFMA structure (conv_wide.hip: one 256-thread workgroup per CU, a BCO (Cout) x 256 (pixel) tile, 4 waves
// as 2 x 2, accumulators in AGPRs) with the activations loaded ONCE per 32-channel slice instead of once per
// (tap, slice) stage.
//
// Why (profiles/r2_*): the wide kernel's K stage costs ~1 850 cycles against 1 024 for its 64
// MFMAs per wave; the gap is its 8 LDS-DMA pieces per wave per stage (4 weight + 4 activation rows), each
// costing ~100 issue cycles inside an MFMA phase.  Here the pixel tile is a 16 x 16 block of one image, so
// the 9 taps of a 32-channel slice read shifted windows of ONE 18 x 18 halo tile (324 rows x 64 B) kept in
// LDS: 21 DMA pieces per slice for all 9 taps instead of 36 -- per wave per stage 4 weight pieces + 0.67
// halo pieces.
//
// K order: channel-major (slice c = channels 32c..32c+31, then its 9 taps), so the accumulation order
// differs from the generic kernel's tap-major one (results within bf16 rounding, not bit-identical).
// Weights stream through a 4-deep ring of 16 KiB stages (BCO rows x 64 B) exactly as in conv_wide; the halo
// tiles are double-buffered by slice: slice c+1's halo rides in the DMA sets of taps 3..8 of slice c (one
// piece per wave per set: 24 pieces, the 3 past row 324 read zeros into padding), issued after every wave
// finished reading slice c-1's halo (the barrier of the hand-over into tap 0 of slice c) and landed by the
// hand-over into tap 8.  Halo rows are swizzled chunk c -> slot c ^ 2((r >> 2) & 1), conflict-free for a
// ds_read_b128 fragment read of 16 consecutive rows from any start (a tap's window starts anywhere).
//
// Built twice (Makefile): this file (HISEG_HW_PART 1: BCO 256, accumulators in AGPRs, and conv_hw_try) and
// conv_hw128.hip (HISEG_HW_PART 2: BCO 128 and 64 with -amdgpu-mfma-vgpr-form -- 128 accumulators in VGPRs keep
// every configuration at two waves per SIMD; the AGPR form allocates 192 AGPRs and drops the B-reuse
// residual kernels to one).  BCO 64 arranges the 4 waves as 1 (Cout) x 4 (pixel): 64 Cout x 64 pixels per wave,
// one weight piece per wave per stage, the same halo.
#include <type_traits>

#include "conv_common.h"

#ifndef HISEG_HW_PART
#define HISEG_HW_PART 1
#endif

namespace hiseg {

typedef __attribute__((address_space(3))) void lds_void_h;

__device__ __forceinline__ void dma16h(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, unsigned voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(__builtin_amdgcn_readfirstlane(lds_addr)), "v"(voff), "s"(rsrc) : "memory");
}

template <int N>
__device__ __forceinline__ void hvm() {
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

__device__ __forceinline__ int hwswz(int r) { return (-(r >> 2)) & 3; }        // weight rows (16-aligned reads)
__device__ __forceinline__ int hhswz(int r) { return ((r >> 2) & 1) << 1; }     // halo rows (any start)

constexpr int kHaloRows = 324;             // 18 x 18
constexpr int kHaloBytes = 24 * 1024;      // 24 pieces of 16 rows x 64 B (rows 324..383: padding)

// REUSE: taps ordered kx-major within a slice (tap t = (kx = t / 3, ky = t % 3)), so the three ky taps of a
// kx read the same 10 halo rows shifted by one row each: the wave keeps B fragments for tile rows 0..9 in
// registers across them and reads 10 per three stages instead of 24 (LDS read traffic per MFMA -39 % at
// BCO 128, where the fragment reads are what bounds the two co-resident workgroups).
template <int BCO, int ACT, bool RES, bool REUSE>
__global__ void __launch_bounds__(256, 1) conv_hw_kernel(ConvArgs a) {
  constexpr int STAGES = 4;
  constexpr int WPX = BCO == 64 ? 4 : 2;   // pixel waves (BCO 64: 1 x 4 waves, else 2 x 2)
  constexpr int TM = BCO * WPX / 64;  // A (Cout) fragments per wave
  constexpr int TN = 16 / WPX;        // B (pixel) fragments per wave: TN tile rows of 16 pixels
  constexpr int J0 = TN >= 8 ? 3 : 1, J1 = TN >= 8 ? 5 : 2;   // columns of group 3 issuing DMA slots 0 / 1
  constexpr int GA = TM / 4;          // A fragments per MFMA group
  constexpr int NAI = BCO / 64;       // weight DMA pieces per wave per stage
  constexpr int STAGE_BYTES = BCO * 64;
  constexpr int RING = STAGES * STAGE_BYTES;
  static_assert(GA >= 1 && TM % 4 == 0 && NAI <= 4, "tile");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wco = w / WPX, wpx = w % WPX;

  // ---- XCD-major bijective remap; Cout tiles fastest, then the 16 x 16 pixel tiles of an image row-major
  const int nco = (d.Cout_pad + BCO - 1) / BCO;   // (BCO 64 over 16 / 32 / 48 columns: one partial tile)
  const int ntx = (d.W + 15) >> 4, nty = (d.H + 15) >> 4;
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
  const int y0 = ty * 16, x0 = tx * 16;

  const int lrow = lane >> 2, slot = lane & 3;
  // weight rows: piece i of wave w fills rows 16 (w + 4i) + lane / 4 of the stage, chunk slot lane % 4
  unsigned woff[NAI];
#pragma unroll
  for (int i = 0; i < NAI; ++i) {
    const int r = 16 * (w + 4 * i) + lrow;
    woff[i] = ((unsigned)(co0 + r) * (unsigned)d.K_pad + (unsigned)((slot ^ hwswz(r)) * 8)) * 2u;
  }
  const unsigned OOB = 0x80000000u;   // >= num_records: the DMA returns zeros
  // halo rows: piece h (0..23) = rows 16h + lane / 4; piece 4p + w belongs to wave w (p = 0..5).  The lane's
  // byte offset for piece p (slice 0; OOB outside the image / past row 324), computed where needed: a
  // precomputed array indexed by the stage's piece number would live in scratch
  // slice sl of a two-source layer (the EnhancedUNet decoder concat) comes from src B once 32 sl >= Ca
  auto halo_off = [&](int p, int sl) __attribute__((always_inline)) -> unsigned {
    const int hr = 16 * (4 * p + w) + lrow;
    const int hy = hr / 18, hx = hr - 18 * hy;
    const int iy = y0 + hy - 1, ix = x0 + hx - 1;
    const bool ok = hr < kHaloRows && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
    const bool fb = 32 * sl >= d.Ca;
    const int cs = fb ? d.b_cstride : d.a_cstride, coff = fb ? d.b_coff + 32 * sl - d.Ca : d.a_coff + 32 * sl;
    // src A of an smp decoder conv1 is the nearest-x2 upsampled low-resolution map: halo pixel (iy, ix) reads
    // source pixel (iy / 2, ix / 2) of the (H / 2, W / 2) grid
    const int ush = (!fb && d.a_up == 2) ? 1 : 0;
    const int sy = iy >> ush, sx = ix >> ush, sH = d.H >> ush, sW = d.W >> ush;
    return ok ? (unsigned)((((n * sH + sy) * sW + sx) * cs + coff + (slot ^ hhswz(hr)) * 8) * 2) : OOB;
  };
  const int nrec_w = d.Cout_pad * d.K_pad * 2;
  const int nrec_a = d.N * (d.H / d.a_up) * (d.W / d.a_up) * d.a_cstride * 2;
  const int nrec_b = d.Cb ? d.N * d.H * d.W * d.b_cstride * 2 : 0;
  const int nsl = a.Cin >> 5;          // 32-channel slices
  const int nS = 9 * nsl;
  const unsigned lds_base = (unsigned)(uintptr_t)(lds_void_h*)smem;
  const unsigned halo_base = lds_base + (unsigned)RING;
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.weight), (short)0, nrec_w,
                                                                     0x00020000);
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.srcA), (short)0, nrec_a,
                                                                     0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.Cb ? d.srcB : d.srcA), (short)0,
                                                                     nrec_b, 0x00020000);

  // ---- the DMA set to be issued next: stage (n_sl, n_tap); weights of that stage, plus, for taps 3..8 of
  // every slice but the last, halo piece (tap - 3) of slice n_sl + 1
  int n_sl = 0, n_tap = 0;
  unsigned p_sbase = lds_base, p_voff[NAI], p_hdst = halo_base, p_hoff = OOB;
  bool p_halo = false, p_hb = false;
#pragma unroll
  for (int k = 0; k < NAI; ++k) p_voff[k] = OOB;
  auto prepare_live = [&](int s) __attribute__((always_inline)) {
    p_sbase = lds_base + (unsigned)((s & (STAGES - 1)) * STAGE_BYTES);
    const int wtap = REUSE ? (n_tap % 3) * 3 + n_tap / 3 : n_tap;   // packed weights: tap = ky * 3 + kx
    const unsigned kofs = (unsigned)(wtap * a.Cin + 32 * n_sl) * 2u;
#pragma unroll
    for (int k = 0; k < NAI; ++k) p_voff[k] = woff[k] + kofs;
    p_halo = n_tap >= 3 && n_sl + 1 < nsl;
    const int hp = n_tap >= 3 ? n_tap - 3 : 0;
    p_hoff = halo_off(hp, n_sl + 1);
    p_hb = 32 * (n_sl + 1) >= d.Ca;
    p_hdst = halo_base + (unsigned)(((n_sl + 1) & 1) * kHaloBytes + 1024 * (4 * hp + w));
    const int tp = n_tap + 1;
    const bool wrap = tp == 9;
    n_tap = wrap ? 0 : tp;
    n_sl += wrap ? 1 : 0;
  };
  auto prepare_dead = [&](int s) __attribute__((always_inline)) {
    p_sbase = lds_base + (unsigned)((s & (STAGES - 1)) * STAGE_BYTES);
#pragma unroll
    for (int k = 0; k < NAI; ++k) p_voff[k] = OOB;
    p_halo = false;
  };
  auto prepare = [&](int s) __attribute__((always_inline)) {
    if (s < nS) prepare_live(s);
    else prepare_dead(s);
  };
  // DMA slot k of the pending set: k < NAI weight piece k, k == NAI the halo piece (when the set has one)
  auto slot_dma = [&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    if constexpr (k < NAI) {
      dma16h(rW, p_sbase + (unsigned)(1024 * (w + 4 * k)), p_voff[k]);
    } else if constexpr (k == NAI) {
      if (p_halo) dma16h(p_hb ? rB : rA, p_hdst, p_hoff);
    }
  };
  // halo of a set: the hand-over waits count one DMA more when the set following the awaited one carries one
  auto set_has_halo = [&](int s) __attribute__((always_inline)) -> bool {
    const int sl = s / 9, tp = s - 9 * (s / 9);
    return s < nS && tp >= 3 && sl + 1 < nsl;
  };

  // ---- fragment reads.  A: weight ring (16-aligned rows).  B: pixel (row j of the wave's 8 tile rows, column
  // lane % 16) at tap (ky, kx) = halo row (wpx*8 + j + ky) * 18 + (lane % 16) + kx, chunk lane / 16
  const char* lds_c = reinterpret_cast<const char*>(smem);
  const int a_lane_off = (lane & 15) * 64 + (((lane >> 4) ^ hwswz(lane & 15)) << 4);
  auto rdA = [&](int s, int i) __attribute__((always_inline)) {
    return *reinterpret_cast<const uint4*>(lds_c + (s & (STAGES - 1)) * STAGE_BYTES + (wco * TM * 16 + i * 16) * 64 +
                                           a_lane_off);
  };
  const int bcol = lane & 15, bch = lane >> 4;
  // B fragment of halo tile row k (= output tile row + ky) at column shift kx
  auto rdBk = [&](int sl, int kx, int k) __attribute__((always_inline)) {
    const int hr = (wpx * TN + k) * 18 + bcol + kx;
    return *reinterpret_cast<const uint4*>(lds_c + RING + (sl & 1) * kHaloBytes + hr * 64 + ((bch ^ hhswz(hr)) << 4));
  };
  auto rdB = [&](int sl, int tap, int j) __attribute__((always_inline)) {
    const int ky = tap / 3, kx = tap - 3 * (tap / 3);
    return rdBk(sl, kx, j + ky);
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: slice 0's halo (6 pieces per wave), sets 0 and 1 whole, slots 0..1 of set 2
#pragma unroll
  for (int p = 0; p < 6; ++p)
    dma16h(rA, halo_base + (unsigned)(1024 * (4 * p + w)), halo_off(p, 0));
#pragma unroll
  for (int s = 0; s < STAGES - 2; ++s) {
    prepare(s);
    slot_dma(std::integral_constant<int, 0>{}); slot_dma(std::integral_constant<int, 1>{});
    slot_dma(std::integral_constant<int, 2>{}); slot_dma(std::integral_constant<int, 3>{});
    slot_dma(std::integral_constant<int, 4>{});
  }
  prepare(STAGES - 2);
  slot_dma(std::integral_constant<int, 0>{}); slot_dma(std::integral_constant<int, 1>{});
  // halo 0 and set 0 landed; set 1 (NAI, tap 1: no halo) and set 2's slots 0..1 (min(NAI, 2) weight pieces:
  // tap 2 has no halo piece) may stay in flight
  hvm<NAI + (NAI < 2 ? NAI : 2)>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  constexpr int NB = REUSE ? TN + 2 : TN;
  uint4 af[TM], bf[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) bf[j] = rdBk(0, 0, j);
#pragma unroll
  for (int i = 0; i < GA; ++i) af[i] = rdA(0, i);

  // MFMA of A fragment i and output column group j at B register b (j + ky under REUSE, else j)
  auto mfma = [&](int i, int j, int b) __attribute__((always_inline)) {
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                         __builtin_bit_cast(bf16x8_t, bf[b]), acc[i][j], 0, 0, 0);
  };

  // the stage whose B fragments are read next (stage s + 1 during body(s); REUSE: the next kx group during
  // its last stage): slice / tap counters
  int r_sl = 0, r_tap = REUSE ? 3 : 1;
  // One K stage s.  Groups 0..2: A fragments of the next group read ahead; DMA slots 2..NAI of set s+2 go out
  // after groups 0 and 1.  Hand-over: set s+1 landed (set s+2 may stay in flight: NAI or NAI + 1 DMAs),
  // barrier (every wave is done with stage s-1's ring buffer and, at tap 0, with the previous slice's halo),
  // set s+3 prepared.  Group 3: stage s+1's B fragments read column by column, slots 0..1 of set s+3.
  auto body = [&](int s, auto tailc, auto kyc) __attribute__((always_inline)) {
    constexpr bool TAIL = decltype(tailc)::value;
    constexpr int KY = decltype(kyc)::value;          // REUSE: the stage's ky (B register shift); else 0
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int i = 0; i < GA; ++i) mfma(g * GA + i, j, j + KY);
        if (j == 1) {
#pragma unroll
          for (int i = 0; i < GA; ++i) af[(g + 1) * GA + i] = rdA(s, (g + 1) * GA + i);
        }
      }
      __builtin_amdgcn_s_setprio(0);
      if (g == 0) { slot_dma(std::integral_constant<int, 2>{}); slot_dma(std::integral_constant<int, 3>{}); }
      if (g == 1) slot_dma(std::integral_constant<int, 4>{});
    }
    if (set_has_halo(s + 2)) hvm<NAI + 1>();
    else hvm<NAI>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (TAIL) prepare_dead(s + STAGES - 1);
    else prepare_live(s + STAGES - 1);
    const int rsl = r_sl, rtp = r_tap;
    __builtin_amdgcn_s_setprio(1);
    if constexpr (REUSE && KY == 2) {   // the next kx group's 10 rows: 0..1 now (unused by ky 2), k + 2 after column k
      bf[0] = rdBk(rsl, rtp / 3, 0);
      bf[1] = rdBk(rsl, rtp / 3, 1);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int i = 0; i < GA; ++i) mfma(3 * GA + i, j, j + KY);
      if constexpr (!REUSE) bf[j] = rdB(rsl, rtp, j);
      else if constexpr (KY == 2) bf[j + 2] = rdBk(rsl, rtp / 3, j + 2);
      if (j == 1) {
#pragma unroll
        for (int i = 0; i < GA; ++i) af[i] = rdA(s + 1, i);
      }
      if (j == J0) slot_dma(std::integral_constant<int, 0>{});
      if (j == J1) slot_dma(std::integral_constant<int, 1>{});
    }
    __builtin_amdgcn_s_setprio(0);
    if (!REUSE || KY == 2) {
      const int tp = r_tap + (REUSE ? 3 : 1);
      r_tap = tp == 9 ? 0 : tp;
      r_sl += tp == 9 ? 1 : 0;
    }
  };
  using F = std::false_type;
  using T = std::true_type;
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  using K2 = std::integral_constant<int, 2>;
  if constexpr (REUSE) {   // kx groups of three stages; the last group prepares the sets past the end
    for (int s = 0; s < nS - 3; s += 3) {
      body(s, F{}, K0{});
      body(s + 1, F{}, K1{});
      body(s + 2, F{}, K2{});
    }
    body(nS - 3, T{}, K0{});
    body(nS - 2, T{}, K1{});
    body(nS - 1, T{}, K2{});
  } else {
    for (int s = 0; s < nS - (STAGES - 1); ++s) body(s, F{}, K0{});
#pragma unroll
    for (int q = STAGES - 1; q >= 1; --q) body(nS - q, T{}, K0{});
  }
  hvm<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // ---- epilogue through LDS (as conv_wide's non-prefetching path): the output tile as 256 pixel rows x BCO
  // bf16, 16-B chunk c of row r at slot c ^ (r & SWM) (SWM = min(BCO / 8, 16) - 1); the residual tile arrives there by LDS-DMA, each lane
  // turns its accumulator quads into bf16 output quads in place, whole rows leave by 16-B stores.  Tile row
  // r = pixel (y0 + r / 16, x0 + r % 16); rows outside the image are neither read nor written.
  constexpr int EROWB = BCO * 2;
  constexpr int CPR = BCO / 8;
  constexpr int RPI = 64 / CPR;
  constexpr int SWM = (CPR < 16 ? CPR : 16) - 1;   // chunk swizzle mask (stays inside the row)
  char* tile = reinterpret_cast<char*>(smem);
  auto px_of = [&](int r) __attribute__((always_inline)) -> int {   // GEMM row of tile row r, or -1
    const int y = y0 + (r >> 4), x = x0 + (r & 15);
    return (y < d.Ho && x < d.Wo) ? (n * d.Ho + y) * d.Wo + x : -1;
  };
  if constexpr (RES) {
    const int nrec_r = a.M * d.r_cstride * 2;
    const __amdgpu_buffer_rsrc_t rR = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.residual), (short)0, nrec_r,
                                                                       0x00020000);
    constexpr int NRI = 256 / (RPI * 4);
    const int c = lane % CPR;
#pragma unroll
    for (int k = 0; k < NRI; ++k) {
      const int r = RPI * (w + 4 * k) + lane / CPR;
      const int px = px_of(r);
      const unsigned off = px >= 0 ? (unsigned)((px * d.r_cstride + d.r_coff + co0 + ((c ^ (r & SWM)) * 8)) * 2) : OOB;
      dma16h(rR, lds_base + (unsigned)(RPI * (w + 4 * k) * EROWB), off);
    }
    hvm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
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
      const int r = wpx * TN * 16 + j * 16 + (lane & 15);
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
  constexpr int NST = 256 * CPR / 256;
#pragma unroll 4
  for (int k = 0; k < NST; ++k) {
    const int idx = t + 256 * k;
    const int r = idx / CPR, c = idx % CPR;
    const int px = px_of(r), co = co0 + 8 * c;
    const uint4 v = *reinterpret_cast<const uint4*>(tile + r * EROWB + ((c ^ (r & SWM)) << 4));
    if (px >= 0 && co < d.Cout)
      *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(d.out) + (long long)px * d.o_cstride + d.o_coff + co) = v;
  }
}

template <int BCO, bool REUSE>
static int launch_hw(const ConvArgs& a, hipStream_t s) {
  const hiseg_conv2d_desc& d = a.d;
  const int tiles = d.N * ((d.H + 15) / 16) * ((d.W + 15) / 16);
  const int nco = (d.Cout_pad + BCO - 1) / BCO;
  const size_t ring_halo = (size_t)4 * BCO * 64 + 2 * kHaloBytes;
  const size_t epi = (size_t)256 * BCO * 2;
  const size_t lds = ring_halo > epi ? ring_halo : epi;
  const bool res = d.residual != nullptr;
  const bool relu = d.act == HISEG_ACT_RELU;
  auto kern = res ? (relu ? conv_hw_kernel<BCO, HISEG_ACT_RELU, true, REUSE> : conv_hw_kernel<BCO, HISEG_ACT_NONE, true, REUSE>)
                  : (relu ? conv_hw_kernel<BCO, HISEG_ACT_RELU, false, REUSE>
                          : conv_hw_kernel<BCO, HISEG_ACT_NONE, false, REUSE>);
  static bool attr_set[2][2] = {};
  bool& done = attr_set[res ? 1 : 0][relu ? 1 : 0];
  if (!done) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    done = true;
  }
  hipLaunchKernelGGL(kern, dim3(tiles * nco), dim3(256), lds, s, a);
  return hiseg_check_launch("conv_hw");
}

#if HISEG_HW_PART == 2
int launch_hw128(const ConvArgs& a, hipStream_t s, bool reuse) {
  return reuse ? launch_hw<128, true>(a, s) : launch_hw<128, false>(a, s);
}
int launch_hw64(const ConvArgs& a, hipStream_t s, bool reuse) {
  return reuse ? launch_hw<64, true>(a, s) : launch_hw<64, false>(a, s);
}
#else
int launch_hw128(const ConvArgs& a, hipStream_t s, bool reuse);   // conv_hw128.hip
int launch_hw64(const ConvArgs& a, hipStream_t s, bool reuse);

// Returns 1 if launched, 0 if the layer does not qualify (caller falls back), <0 on error.
// variant 80 = BCO 256 (Cout a multiple of 256), 82 = BCO 128; 84 / 86 the same with the kx-major tap order and
// B-fragment reuse across ky; 88 / 89 = BCO 64 (1 x 4 waves of 64 Cout x 64 pixels; 64-multiple Cout) without /
// with the reuse.
int conv_hw_try(const ConvArgs& a, hipStream_t s, int variant) {
  const hiseg_conv2d_desc& d = a.d;
  if (d.dtype != HISEG_BF16 || d.out_dtype != HISEG_BF16) return 0;
  if (d.in_scale != nullptr || d.convT || d.mul != nullptr || d.out2 != nullptr) return 0;
  if (d.KH != 3 || d.KW != 3 || d.stride != 1 || d.pad != 1 || d.Ho != d.H || d.Wo != d.W) return 0;
  if (d.act != HISEG_ACT_NONE && d.act != HISEG_ACT_RELU) return 0;
  // src A nearest-x2 upsampled (smp decoder conv1): even grid (conv2d_impl checks)
  if (d.a_up != 1 && d.a_up != 2) return 0;
  // two sources (concat): each whole 32-channel slice from one of them
  // (K_pad is only the packed weight rows' stride: a 32-multiple Cin padded to a 64-multiple K is fine)
  if (d.Ca % 32 != 0 || d.Cb % 32 != 0 || d.Ca < 64 || d.K_pad < 9 * (d.Ca + d.Cb)) return 0;
  if ((d.a_cstride | d.a_coff) & 7) return 0;
  if (d.Cb && (d.srcB == nullptr || ((d.b_cstride | d.b_coff) & 7))) return 0;
  // BCO 64 also takes a partial last tile of 16 / 32 / 48 output columns (16..48 columns alone, or the B7-ultra
  // head's 96 / 160-channel layers): weight rows past Cout_pad read zeros (exact num_records), columns past Cout
  // are neither scaled from real tables nor stored
  const int cmul = variant >= 88 ? 63 : 127;
  const bool narrow = variant >= 88 && d.Cout % 16 == 0;
  if (((d.Cout & cmul) && !narrow) || ((d.o_cstride | d.o_coff) & 7) || (d.residual && ((d.r_cstride | d.r_coff) & 7)))
    return 0;
  if ((((uintptr_t)d.scale | (uintptr_t)d.shift | (uintptr_t)d.out | (uintptr_t)d.residual) & 15)) return 0;
  const long long span_a = (long long)d.N * (d.H / d.a_up) * (d.W / d.a_up) * d.a_cstride * 2;
  const long long span_b = d.Cb ? (long long)d.N * d.H * d.W * d.b_cstride * 2 : 0;
  const long long span_w = (long long)d.Cout_pad * d.K_pad * 2;
  const long long span_r = d.residual ? (long long)a.M * d.r_cstride * 2 : 0;
  if (span_a >= 0x7fffffffll || span_b >= 0x7fffffffll || span_w >= 0x7fffffffll || span_r >= 0x7fffffffll) return 0;
  int r;
  switch (variant) {
    case 80: if (d.Cout % 256) return 0; r = launch_hw<256, false>(a, s); break;
    case 82: r = launch_hw128(a, s, false); break;
    case 84: if (d.Cout % 256) return 0; r = launch_hw<256, true>(a, s); break;
    case 86: r = launch_hw128(a, s, true); break;
    case 88: r = launch_hw64(a, s, false); break;
    case 89: r = launch_hw64(a, s, true); break;
    default: return 0;
  }
  return r < 0 ? r : 1;
}
#endif

}  // namespace hiseg
