// 3x3 / stride-1 convolution, warp-specialised: 8 compute waves + loader waves (bf16, gfx950).
//
// conv_halo2 measured the in-order vmcnt trap: a wave that issues the long-latency (HBM) halo
// loads of the next channel block and then the short-latency (L2) weight loads of the next taps
// cannot wait for those weights without also waiting for the halo (vmcnt retires in issue
// order, MI355X_MICROARCH.md "s_waitcnt vmcnt(N)").  Here the two streams live in different
// waves:
//   * loader waves move the (TH+2) x (W+2) x 64-channel input halo of channel block cb+1 into
//     LDS by LDS-DMA (one 1 KiB buffer_load ... lds per 8 rows; out-of-image taps read zeros via
//     an out-of-range voffset; 128-B rows, XOR swizzle applied on the source address) while the
//     compute waves run the 9 taps of block cb; they wait vmcnt(0) and join the block barrier;
//   * compute waves stream only weights (fragment-ordered, 3 K blocks ahead in registers; every
//     wait is hipcc's own exact counted vmcnt) and read B fragments from the halo.
// One barrier per 64-channel block, none per K block.
#include "conv_common.h"

namespace hiseg {

constexpr int H3_BPX = 192;

__device__ __forceinline__ void dma16_h3(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, unsigned voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(lds_addr), "v"(voff), "s"(rsrc) : "memory");
}

// 8 compute waves (WCO x WPX) + NLW loader waves.
template <int BCO, int WCO, int WPX, int NLW, int HMAX>
__global__ void __launch_bounds__(64 * (8 + NLW)) conv_halo3_kernel(ConvArgs a) {
  constexpr int TMW = BCO / (16 * WCO);
  constexpr int TN = H3_BPX / (16 * WPX);
  constexpr int HBUF = HMAX * 128;             // bytes per halo buffer (128-B rows, XOR swizzle)
  constexpr int JG = TN > 6 ? TN / 2 : TN;
  static_assert(WCO * WPX == 8 && TMW >= 1 && TN >= 1 && HMAX % 8 == 0, "tile");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* const lds = reinterpret_cast<char*>(smem);
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int W = d.W, H = d.H, W2 = d.W + 2;
  const int TH = H3_BPX / W;

  const int nco = d.Cout_pad / BCO;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = orig & 7, loc = orig >> 3;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int co0 = (wg % nco) * BCO;
  const int px0 = (wg / nco) * H3_BPX;
  const int n = px0 / (H * W);
  const int y0 = (px0 - n * H * W) / W;
  const int ncb = a.Cin >> 6;

  if (w >= 8) {
    // ------------------------------------------------------------ loader waves: halo DMA only
    const int L = w - 8;
    const int R = (TH + 2) * W2;
    const int NHI = (R + 7) >> 3;  // 8-row DMA instructions per halo
    const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)smem;
    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.srcA), (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.srcB ? d.srcB : d.srcA), (short)0, 0x7fffffff, 0x00020000);
    const int slot = lane & 7;
    auto issue = [&](int cb) __attribute__((always_inline)) {
      const int ci0 = cb << 6;
      const bool fromA = ci0 < d.Ca;
      const int cs = fromA ? d.a_cstride : d.b_cstride;
      const int cbase = fromA ? d.a_coff + ci0 : d.b_coff + ci0 - d.Ca;
      const unsigned base = lds0 + (unsigned)((cb & 1) * HBUF);
      for (int h = L; h < NHI; h += NLW) {
        const int r = 8 * h + (lane >> 3);
        const int hy = r / W2, hx = r - (r / W2) * W2;
        const int iy = y0 - 1 + hy, ix = hx - 1;
        const bool ok = r < R && iy >= 0 && iy < H && ix >= 0 && ix < W;
        const int c = slot ^ ((r >> 1) & 7);
        const unsigned off = ok ? ((unsigned)(((n * H + iy) * W + ix) * cs + cbase) + (unsigned)c * 8u) * 2u : 0x80000000u;
        dma16_h3(fromA ? rA : rB, base + (unsigned)h * 1024u, off);
      }
    };
    issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int cb = 0; cb + 1 < ncb; ++cb) {
      issue(cb + 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    return;
  }

  // -------------------------------------------------------------- compute waves
  const int wco = w / WPX, wpx = w % WPX;
  int fbrow[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int p = wpx * (TN * 16) + j * 16 + (lane & 15);
    fbrow[j] = (p / W) * W2 + (p - (p / W) * W);
  }
  const int qk = lane >> 4;  // chunk (k group) of this lane for k-step 0; k-step 1 is qk + 4
  const int nK = ncb * 9;
  const char* wbase = reinterpret_cast<const char*>(d.weight_frag) +
                      ((size_t)(co0 / 16 + wco * TMW) * nK * 2) * 1024 + lane * 16;
  const size_t ct_stride = (size_t)nK * 2 * 1024;
  uint4 wreg[3][TMW][2];
  auto load_w = [&](int st, int kb) __attribute__((always_inline)) {
#pragma unroll
    for (int ti = 0; ti < TMW; ++ti)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        wreg[st][ti][s] = *reinterpret_cast<const uint4*>(wbase + ti * ct_stride + ((size_t)kb * 2 + s) * 1024);
  };

  floatx4 acc[TMW][TN];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  load_w(0, 0);
  load_w(1, 1 < nK ? 1 : nK - 1);
  load_w(2, 2 < nK ? 2 : nK - 1);

  for (int cb = 0; cb < ncb; ++cb) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // halo(cb) landed (loader waited vmcnt(0)); halo(cb-1) reads done
    asm volatile("" ::: "memory");
    const char* hb = lds + (cb & 1) * HBUF;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kb = cb * 9 + tap;
      const int st = tap % 3;
      const int dt = (tap / 3) * W2 + (tap % 3);
      int addr0[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = fbrow[j] + dt;
        addr0[j] = r * 128 + ((qk ^ ((r >> 1) & 7)) << 4);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int j0 = 0; j0 < TN; j0 += JG) {
          uint4 bfr[JG];
#pragma unroll
          for (int j = 0; j < JG; ++j) bfr[j] = *reinterpret_cast<const uint4*>(hb + (addr0[j0 + j] ^ (s << 6)));
#pragma unroll
          for (int ti = 0; ti < TMW; ++ti)
#pragma unroll
            for (int j = 0; j < JG; ++j)
              acc[ti][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  __builtin_bit_cast(bf16x8_t, wreg[st][ti][s]), __builtin_bit_cast(bf16x8_t, bfr[j]),
                  acc[ti][j0 + j], 0, 0, 0);
        }
      }
      load_w(st, kb + 3 < nK ? kb + 3 : nK - 1);
    }
  }

#pragma clang loop unroll(full)
  for (int ti = 0; ti < TMW; ++ti)
#pragma clang loop unroll(full)
    for (int j = 0; j < TN; ++j) {
      const int px = px0 + wpx * TN * 16 + j * 16 + (lane & 15);
      const int co = co0 + wco * TMW * 16 + ti * 16 + (lane >> 4) * 4;
      conv_epilogue<bf16_t, bf16_t>(a, px, co, acc[ti][j]);
    }
}

template <int BCO, int WCO, int WPX, int NLW, int HMAX>
static int launch_halo3(const ConvArgs& a, hipStream_t s) {
  const int ntile = a.M / H3_BPX;
  const int nco = a.d.Cout_pad / BCO;
  const size_t lds = (size_t)2 * HMAX * 128;
  auto kern = conv_halo3_kernel<BCO, WCO, WPX, NLW, HMAX>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(ntile * nco), dim3(64 * (8 + NLW)), lds, s, a);
  return hiseg_check_launch("conv_halo3");
}

// 1 if launched, 0 if not applicable, <0 on error.  variant: 0 auto, 30+ forced.
int conv_halo3_try(const ConvArgs& a, hipStream_t s, int variant) {
  const hiseg_conv2d_desc& d = a.d;
  if (!d.weight_frag) return 0;
  if (d.dtype != HISEG_BF16 || d.out_dtype != HISEG_BF16 || d.convT) return 0;
  if (d.KH != 3 || d.KW != 3 || d.stride != 1 || d.pad != 1 || d.a_up != 1 || d.in_scale) return 0;
  if (d.Ca % 64 || d.Cb % 64 || d.K_pad != 9 * a.Cin) return 0;
  if (((d.a_cstride | d.a_coff) & 7) || (d.Cb && ((d.b_cstride | d.b_coff) & 7))) return 0;
  if (H3_BPX % d.W) return 0;
  const int TH = H3_BPX / d.W;
  if (d.H % TH) return 0;
  const int R = (TH + 2) * (d.W + 2);
  const long long span = (long long)d.N * d.H * d.W * (d.a_cstride > d.b_cstride ? d.a_cstride : d.b_cstride) * 2;
  if (span >= 0x7fffffffll) return 0;
  if (R > 448) return 0;
  if (variant == 0 || variant < 30) {
    if (d.Cout_pad % 128 == 0) variant = 30;
    else if (d.Cout_pad % 64 == 0) variant = 31;
    else return 0;
  }
  int r;
  switch (variant) {
    case 30: if (d.Cout_pad % 128) return 0; r = launch_halo3<128, 4, 2, 2, 448>(a, s); break;
    case 31: if (d.Cout_pad % 64) return 0; r = launch_halo3<64, 2, 4, 2, 448>(a, s); break;
    case 32: if (d.Cout_pad % 128) return 0; r = launch_halo3<128, 4, 2, 1, 448>(a, s); break;
    case 33: if (d.Cout_pad % 128) return 0; r = launch_halo3<128, 8, 1, 2, 448>(a, s); break;
    default: return 0;
  }
  return r < 0 ? r : 1;
}

}  // namespace hiseg
