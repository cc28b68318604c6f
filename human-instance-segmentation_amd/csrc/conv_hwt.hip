// Halo-tiled 3x3 convolution, one wave per SIMD with 64 x 256 wave tiles (gfx950, bf16): the dominant class of the
// ROI head (256->256 / 128->128 / 128->256 3x3 layers, refinement.py:31-55 ResidualBlock, rgb.py:657-673).
//
// conv_hwr.hip runs two workgroups per CU (two waves per SIMD, 64 x 128 wave tiles, 256 VGPRs each): the weight
// (A) fragments reach the registers from L2 one K step ahead, and its counters put the MFMA pipe at 0.59 busy with
// the idle cycles in waits for those loads -- there is no register room for a second A buffer.  Here one workgroup
// holds the CU (four waves, one per SIMD, 512 registers each): every wave computes 64 Cout x 256 pixels (16 pixel
// rows x 16 columns, 4 x 16 accumulators of v_mfma_f32_16x16x32_bf16 = 256 AGPRs), so each A fragment feeds 16
// MFMAs instead of 8 (half the A traffic per FLOP), and the A fragments are double-buffered two K steps ahead.
// Workgroup tile: 128 Cout x 32 x 16 pixels (waves: 2 Cout halves x 2 row halves); the 34 x 18 halo of a 32-channel
// slice is DMA'd once per slice into one of two 40 KiB LDS buffers, one barrier per slice.  B fragments are reused
// across ky (kx-major steps: the 18 fragment rows of a column shift serve its three ky steps).  The K order and the
// MFMA shape are conv_hwr's, so the results are bit-identical to it (and to conv_hw's variant 86).
#include "conv_common.h"

namespace hiseg {

typedef unsigned ht_u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void ht_lds_void;

__device__ __forceinline__ void ht_dma16(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, unsigned voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(__builtin_amdgcn_readfirstlane(lds_addr)), "v"(voff), "s"(rsrc) : "memory");
}

template <int ACT, bool RES>
__global__ void __launch_bounds__(256, 1) conv_hwt_kernel(ConvArgs a) {
  constexpr int BCO = 128, TM = 4, TN = 16, NB = TN + 2;
  constexpr int TH = 32, TW = 16, HWD = TW + 2, NW = 4;
  constexpr int NHR = (TH + 2) * HWD;                      // 612 halo rows (pixels) of a slice
  constexpr int PPW = ((NHR + 15) / 16 + NW - 1) / NW;     // 10 pieces (16 rows, 1 KiB) per wave per slice
  constexpr int HB = PPW * NW * 1024;                      // 40 KiB per halo buffer
  constexpr int NPX = TH * TW;                             // 512 output pixels
  static_assert(PPW == 10, "the halo schedule below issues two pieces in each of the first five steps");
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wco = w >> 1, wpx = w & 1;   // Cout half (64 columns); pixel rows 16 wpx .. + 15 of the tile

  // ---- XCD-major bijective remap; Cout tiles fastest (the two Cout tiles of a pixel tile share its halo in L2)
  const int nco = d.Cout_pad / BCO;
  const int ntx = (d.W + TW - 1) / TW, nty = (d.H + TH - 1) / TH;
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
  const int y0 = ty * TH, x0 = tx * TW;

  const unsigned OOB = 0x80000000u;   // >= num_records: loads return zeros
  const int nsl = a.Cin >> 5;         // 32-channel slices (even: Cin % 64 == 0)
  const int ncb = a.Cin >> 6;
  const __amdgpu_buffer_rsrc_t rF = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(d.weight_frag), (short)0, d.Cout_pad * 9 * a.Cin * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(d.srcA), (short)0, d.N * d.H * d.W * d.a_cstride * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(d.Cb ? d.srcB : d.srcA), (short)0, d.Cb ? d.N * d.H * d.W * d.b_cstride * 2 : 0, 0x00020000);

  // ---- A fragments (hiseg.ops.frag_pack): (Cout tile ct, slice sl, tap) at
  // ((((ct * ncb + sl / 2) * 9 + tap) * 2 + sl % 2) * 64 + lane) * 16 B; the wave-uniform (slice, tap) part is the SGPR
  // offset of the load
  const unsigned a_ct = (unsigned)((co0 + wco * 64) >> 4) * (unsigned)ncb * 18u * 1024u;
  const unsigned a_ct_step = (unsigned)ncb * 18u * 1024u;

  // ---- halo layout (conv_hwr's): row hr = hy * 18 + hx (64 B = 32 channels), 16-B chunk c at slot
  // c ^ 2 ((hx >> 2) & 1): a B-fragment read (16 consecutive hx of one hy) is conflict-free for every column shift.
  // Piece p of wave w = halo rows 16 (4 p + w) + lane / 4 (one 1 KiB LDS-DMA), lane l -> row hr, slot l % 4.
  const unsigned lds_base = (unsigned)(uintptr_t)(ht_lds_void*)smem;
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
    const unsigned off = ok ? (unsigned)((((n * d.H + iy) * d.W + ix) * cs + coff + chunk * 8) * 2) : OOB;
    ht_dma16(fb ? rB : rA, lds_base + (unsigned)(buf * HB + 1024 * (NW * p + w)), off);
  };
  const char* lds_c = reinterpret_cast<const char*>(smem);
  // B fragment k of column shift kx: pixel row 16 wpx + k (halo row + ky), column lane % 16 + kx, channels
  // 8 (lane / 16) .. + 7
  auto rdB = [&](int ln, int buf, int kx, int k) __attribute__((always_inline)) -> ht_u4 {
    const int hx = (ln & 15) + kx;
    const int o = (16 * wpx * HWD + hx) * 64 + (((ln >> 4) ^ (((hx >> 2) & 1) << 1)) << 4);
    return *reinterpret_cast<const ht_u4*>(lds_c + o + buf * HB + k * HWD * 64);
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // K step (slice sl, position st; kx-major: kx = st / 3, ky = st % 3, tap = 3 ky + kx)
  auto a_soff = [&](int sl, int tap) __attribute__((always_inline)) -> unsigned {
    return __builtin_amdgcn_readfirstlane((((unsigned)(sl >> 1) * 9u + (unsigned)tap) * 2u + (unsigned)(sl & 1)) * 1024u);
  };
  ht_u4 af[2][TM], bf[NB];

  // ---- prologue: slice 0's halo into buffer 0, A fragments of steps 0 and 1 (taps 0 and 3)
#pragma unroll
  for (int p = 0; p < PPW; ++p) halo_dma(p, 0, 0);
  {
    const unsigned s0 = a_soff(0, 0), s1 = a_soff(0, 3);
#pragma unroll
    for (int i = 0; i < TM; ++i)
      af[0][i] = __builtin_amdgcn_raw_buffer_load_b128(rF, a_ct + (unsigned)i * a_ct_step + (unsigned)lane * 16u, s0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
      af[1][i] = __builtin_amdgcn_raw_buffer_load_b128(rF, a_ct + (unsigned)i * a_ct_step + (unsigned)lane * 16u, s1, 0);
  }
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // the halo pieces (older than the 8 A loads)
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NB; ++k) bf[k] = rdB(lane, 0, 0, k);

  // One K step: A fragment by A fragment, its 16 MFMAs, then the fragment of the step two ahead is loaded into its
  // registers.  Slice sl + 1's halo: pieces 2 st, 2 st + 1 at steps st = 0..4 of slice sl (after that step's A loads);
  // at st = 8 every piece has landed once at most the 8 A loads of the last two steps are pending (vmcnt(8)), then the
  // slice barrier.  B fragments: after the ky = 2 step of a column shift, the next shift's 18 rows; after the barrier,
  // the next slice's first shift.  AB = A buffer of the step, SB = halo buffer of the slice (both compile-time: the
  // loop runs two slices, 18 steps, per iteration).
  auto tap_of = [](int st) constexpr { return 3 * (st % 3) + st / 3; };
  auto step = [&](int sl, auto stc, auto abc, auto sbc) __attribute__((always_inline)) {
    constexpr int st = decltype(stc)::value;
    constexpr int AB = decltype(abc)::value;
    constexpr int SB = decltype(sbc)::value;
    constexpr int KY = st % 3;
    const bool more = sl + 1 < nsl;
    constexpr bool NEXT_SL = st + 2 >= 9;                  // the step two ahead is in the next slice
    const bool load_next = !NEXT_SL || more;
    const unsigned so = a_soff(NEXT_SL ? sl + 1 : sl, tap_of((st + 2) % 9));
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const unsigned a_lane = a_ct + (unsigned)ln * 16u;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[AB][i]),
                                                             __builtin_bit_cast(bf16x8_t, bf[j + KY]), acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (load_next) af[AB][i] = __builtin_amdgcn_raw_buffer_load_b128(rF, a_lane + (unsigned)i * a_ct_step, so, 0);
    }
    if constexpr (KY == 2 && st < 8) {   // the next column shift's window rows
#pragma unroll
      for (int k = 0; k < NB; ++k) bf[k] = rdB(ln, SB, st / 3 + 1, k);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (st < 5) {
      if (more) {
        halo_dma(2 * st, sl + 1, SB ^ 1);
        halo_dma(2 * st + 1, sl + 1, SB ^ 1);
      }
    }
    if constexpr (st == 8) {
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      __syncthreads();   // slice sl+1's halo is in LDS; every wave is done reading slice sl's buffer
      if (more) {
#pragma unroll
        for (int k = 0; k < NB; ++k) bf[k] = rdB(ln, SB ^ 1, 0, k);
      }
    }
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  using S3 = std::integral_constant<int, 3>;
  using S4 = std::integral_constant<int, 4>;
  using S5 = std::integral_constant<int, 5>;
  using S6 = std::integral_constant<int, 6>;
  using S7 = std::integral_constant<int, 7>;
  using S8 = std::integral_constant<int, 8>;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  for (int sl = 0; sl < nsl; sl += 2) {   // nsl is even (Cin % 64 == 0)
    step(sl, S0{}, I0{}, I0{}); step(sl, S1{}, I1{}, I0{}); step(sl, S2{}, I0{}, I0{}); step(sl, S3{}, I1{}, I0{});
    step(sl, S4{}, I0{}, I0{}); step(sl, S5{}, I1{}, I0{}); step(sl, S6{}, I0{}, I0{}); step(sl, S7{}, I1{}, I0{});
    step(sl, S8{}, I0{}, I0{});
    step(sl + 1, S0{}, I1{}, I1{}); step(sl + 1, S1{}, I0{}, I1{}); step(sl + 1, S2{}, I1{}, I1{});
    step(sl + 1, S3{}, I0{}, I1{}); step(sl + 1, S4{}, I1{}, I1{}); step(sl + 1, S5{}, I0{}, I1{});
    step(sl + 1, S6{}, I1{}, I1{}); step(sl + 1, S7{}, I0{}, I1{}); step(sl + 1, S8{}, I1{}, I1{});
  }

  // ---- epilogue through LDS: 512 pixel rows x 128 bf16, 16-B chunk c of row r at slot c ^ (r & 15); the residual
  // tile arrives there by LDS-DMA, each lane turns its accumulator quads into bf16 output quads in place, whole rows
  // leave by 16-B stores.  Tile row r = pixel (y0 + r / 16, x0 + r % 16).
  constexpr int EROWB = BCO * 2;   // 256 B per row
  constexpr int CPR = BCO / 8;     // 16 chunks per row
  constexpr int RPI = 64 / CPR;    // 4 rows per wave instruction
  constexpr int SWM = CPR - 1;
  char* tile = reinterpret_cast<char*>(smem);
  auto px_of = [&](int r) __attribute__((always_inline)) -> int {
    const int y = y0 + r / TW, x = x0 + r % TW;
    return (y < d.Ho && x < d.Wo) ? (n * d.Ho + y) * d.Wo + x : -1;
  };
  __syncthreads();   // every wave is done with the halo buffers
  if constexpr (RES) {
    const int nrec_r = a.M * d.r_cstride * 2;
    const __amdgpu_buffer_rsrc_t rR = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.residual), (short)0, nrec_r,
                                                                       0x00020000);
    constexpr int NRI = NPX / (RPI * NW);   // 32 pieces per wave
    const int c = lane % CPR;
#pragma unroll 8
    for (int k = 0; k < NRI; ++k) {
      const int r = RPI * (w + NW * k) + lane / CPR;
      const int px = px_of(r);
      const unsigned off = px >= 0 ? (unsigned)((px * d.r_cstride + d.r_coff + co0 + ((c ^ (r & SWM)) * 8)) * 2) : OOB;
      ht_dma16(rR, lds_base + (unsigned)(RPI * (w + NW * k) * EROWB), off);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int cl = wco * TM * 16 + i * 16 + (lane >> 4) * 4;
    const int cc = co0 + cl < d.Cout ? co0 + cl : 0;
    const floatx4 sc = *reinterpret_cast<const floatx4*>(d.scale + cc);
    const floatx4 sh = *reinterpret_cast<const floatx4*>(d.shift + cc);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int r = (16 * wpx + j) * TW + (lane & 15);
      char* q = tile + r * EROWB + ((((cl >> 3) ^ (r & SWM)) << 4) | ((cl & 4) << 1));
      const floatx4 ac = acc[i][j];
      float v[4];
      uint2 rv = make_uint2(0u, 0u);
      if constexpr (RES) rv = *reinterpret_cast<const uint2*>(q);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = ac[e] * sc[e] + sh[e];
        if constexpr (RES) v[e] += Quad<bf16_t>::get(rv, e);
        if constexpr (ACT == HISEG_ACT_RELU) v[e] = v[e] > 0.f ? v[e] : 0.f;
      }
      uint2 o;
      o.x = f2bf2(v[0], v[1]);
      o.y = f2bf2(v[2], v[3]);
      *reinterpret_cast<uint2*>(q) = o;
    }
  }
  __syncthreads();
  constexpr int NST = NPX * CPR / (NW * 64);   // 32 stores per thread
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

template <int ACT, bool RES>
static int launch_hwt(const ConvArgs& a, hipStream_t s) {
  const hiseg_conv2d_desc& d = a.d;
  constexpr size_t lds = (size_t)512 * 256;   // the epilogue tile (> the two 40 KiB halo buffers)
  const int tiles = d.N * ((d.H + 31) / 32) * ((d.W + 15) / 16);
  const int nco = d.Cout_pad / 128;
  auto kern = conv_hwt_kernel<ACT, RES>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3(tiles * nco), dim3(256), lds, s, a);
  return hiseg_check_launch("conv_hwt");
}

// 1 = launched, 0 = the layer does not qualify (caller falls back), <0 on error.  Variant 103.  The form conv_hwr
// takes with 128-multiple Cout (single-source or whole-slice two-source 3x3, ReLU / none, optional residual), not
// the upsampled decoder form.
int conv_hwt_try(const ConvArgs& a, hipStream_t s, int variant) {
  const hiseg_conv2d_desc& d = a.d;
  if (variant != 103 || d.weight_frag == nullptr) return 0;
  if (d.dtype != HISEG_BF16 || d.out_dtype != HISEG_BF16) return 0;
  if (d.a_up != 1 || d.in_scale != nullptr || d.convT || d.mul != nullptr || d.out2 != nullptr) return 0;
  if (d.KH != 3 || d.KW != 3 || d.stride != 1 || d.pad != 1 || d.Ho != d.H || d.Wo != d.W) return 0;
  if (d.act != HISEG_ACT_NONE && d.act != HISEG_ACT_RELU) return 0;
  if (d.Ca % 32 != 0 || d.Cb % 32 != 0 || (d.Ca + d.Cb) % 64 != 0 || d.Ca < 64 || d.K_pad != 9 * (d.Ca + d.Cb))
    return 0;
  if ((d.a_cstride | d.a_coff) & 7) return 0;
  if (d.Cb && (d.srcB == nullptr || ((d.b_cstride | d.b_coff) & 7))) return 0;
  if ((d.Cout & 127) || d.Cout_pad != d.Cout || ((d.o_cstride | d.o_coff) & 7) ||
      (d.residual && ((d.r_cstride | d.r_coff) & 7)))
    return 0;
  if ((((uintptr_t)d.scale | (uintptr_t)d.shift | (uintptr_t)d.out | (uintptr_t)d.residual |
        (uintptr_t)d.weight_frag) & 15))
    return 0;
  const long long span_a = (long long)d.N * d.H * d.W * d.a_cstride * 2;
  const long long span_b = d.Cb ? (long long)d.N * d.H * d.W * d.b_cstride * 2 : 0;
  const long long span_w = (long long)d.Cout_pad * d.K_pad * 2;
  const long long span_r = d.residual ? (long long)a.M * d.r_cstride * 2 : 0;
  if (span_a >= 0x7fffffffll || span_b >= 0x7fffffffll || span_w >= 0x7fffffffll || span_r >= 0x7fffffffll) return 0;
  const bool res = d.residual != nullptr, relu = d.act == HISEG_ACT_RELU;
  const int r = res ? (relu ? launch_hwt<HISEG_ACT_RELU, true>(a, s) : launch_hwt<HISEG_ACT_NONE, true>(a, s))
                    : (relu ? launch_hwt<HISEG_ACT_RELU, false>(a, s) : launch_hwt<HISEG_ACT_NONE, false>(a, s));
  return r < 0 ? r : 1;
}

}  // namespace hiseg
