// 3x3 / stride-1 convolution with an LDS-resident input halo (bf16, gfx950).
//
// The implicit-GEMM kernels gather each input pixel once per filter tap (9x for 3x3).  Here a
// workgroup owns a 192-pixel output tile made of TH = 192/W complete rows of one image, loads
// the (TH+2) x (W+2) input halo of a 64-channel block into LDS once, and runs all 9 taps of that
// channel block out of it: the tap only shifts the LDS row each lane reads.  Per 9 K blocks the
// LDS-DMA traffic is 9 weight blocks (BCO x 128 B, L2-resident) + one halo (<= NH*64 rows x
// 128 B) instead of 9 weight + 9 activation blocks, ~3x fewer DMA instructions per FLOP.
//
// Pipelines: the halo of channel block cb+1 is prefetched a whole channel block ahead into the
// second halo buffer; weights stream through a WS-deep ring.  Waits are exact counted vmcnt
// values (the halo issue interleaves with the weight stream; see the `outstanding` rule below),
// barriers are raw s_barrier, LDS-DMA is inline asm (hipcc's waitcnt pass would otherwise drain
// vmcnt(0) before every ds_read).  8 waves = 2 (Cout) x 4 (pixels); wave tile (BCO/2) x 48.
#include "conv_common.h"

namespace hiseg {

typedef __attribute__((address_space(3))) void lds_void2;

__device__ __forceinline__ void dma16h(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, unsigned voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(lds_addr), "v"(voff), "s"(rsrc) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

constexpr int HALO_BPX = 192;

template <int BCO, int NH, int WS>
__global__ void __launch_bounds__(512) conv_halo_kernel(ConvArgs a) {
  constexpr int NW = 8, WPX = 4;
  constexpr int TM = BCO / 32;             // 16-row Cout tiles per wave (2 Cout waves)
  constexpr int TN = HALO_BPX / (WPX * 16);  // = 3 pixel tiles per wave
  constexpr int NB = BCO / (8 * NW);       // weight DMA instructions per wave per K block
  constexpr int HROWS = NH * 8 * NW;       // halo rows per buffer (padded)
  constexpr int WSTAGE = BCO * 8;          // 16-B slots per weight stage
  constexpr int HSTAGE = HROWS * 8;        // 16-B slots per halo buffer
  static_assert(NB >= 1 && TM >= 1, "tile");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  uint4* const sWbase = smem;                        // WS weight stages
  uint4* const sHbase = smem + WS * WSTAGE;          // 2 halo buffers
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wco = w / WPX, wpx = w % WPX;
  const int W = d.W, H = d.H, W2 = d.W + 2;
  const int TH = HALO_BPX / W;

  // ---- XCD-major bijective remap, Cout tiles fastest
  const int nco = d.Cout_pad / BCO;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int q = nwg >> 3, r8 = nwg & 7, xcd = orig & 7, loc = orig >> 3;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + loc;
  const int co0 = (wg % nco) * BCO;
  const int px0 = (wg / nco) * HALO_BPX;          // tile = TH whole rows of one image
  const int n = px0 / (H * W);
  const int y0 = (px0 - n * H * W) / W;

  // ---- halo DMA lanes: instruction h = w + NW*i covers halo rows 8h..8h+7
  const int lrow = lane >> 3, slot = lane & 7;
  const int R = (TH + 2) * W2;
  int hpix[NH], hch[NH];
  bool hok[NH];
#pragma unroll
  for (int i = 0; i < NH; ++i) {
    const int r = 8 * (w + NW * i) + lrow;
    const int hy = r / W2, hx = r - (r / W2) * W2;
    const int iy = y0 - 1 + hy, ix = hx - 1;
    hok[i] = r < R && iy >= 0 && iy < H && ix >= 0 && ix < W;
    hpix[i] = (n * H + iy) * W + ix;
    hch[i] = slot ^ ((r >> 1) & 7);
  }
  unsigned woff[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int r = 8 * (w + NW * i) + lrow;
    woff[i] = ((unsigned)(co0 + r) * (unsigned)d.K_pad + (unsigned)(slot ^ ((r >> 1) & 7)) * 8u) * 2u;
  }
  // ---- fragment rows of this lane in the halo (tap (0,0)): pixel p -> (p/W)*(W+2) + p%W
  int frow[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int p = wpx * (TN * 16) + j * 16 + (lane & 15);
    frow[j] = (p / W) * W2 + (p - (p / W) * W);
  }

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.srcA), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.srcB ? d.srcB : d.srcA), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.weight), (short)0, 0x7fffffff, 0x00020000);
  const unsigned OOB = 0x80000000u;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_void2*)smem;
  const int Cin = a.Cin;
  const int ncb = Cin >> 6;
  const int nK = ncb * 9;

  auto issue_w = [&](int kb) __attribute__((always_inline)) {
    const int cb = kb / 9, tap = kb - (kb / 9) * 9;
    const unsigned kofs = (unsigned)(tap * Cin + cb * 64) * 2u;
    const unsigned base = lds0 + (unsigned)((kb % WS) * WSTAGE) * 16u;
#pragma unroll
    for (int i = 0; i < NB; ++i) dma16h(rW, base + (unsigned)(64 * (w + NW * i)) * 16u, woff[i] + kofs);
  };
  auto issue_h = [&](int cb) __attribute__((always_inline)) {
    const int ci0 = cb << 6;
    const bool fromA = ci0 < d.Ca;
    const int cs = fromA ? d.a_cstride : d.b_cstride;
    const int cbase = fromA ? d.a_coff + ci0 : d.b_coff + ci0 - d.Ca;
    const unsigned base = lds0 + (unsigned)(WS * WSTAGE + (cb & 1) * HSTAGE) * 16u;
#pragma unroll
    for (int i = 0; i < NH; ++i) {
      const unsigned off = hok[i] ? ((unsigned)(hpix[i] * cs + cbase) + (unsigned)hch[i] * 8u) * 2u : OOB;
      dma16h(fromA ? rA : rB, base + (unsigned)(64 * (w + NW * i)) * 16u, off);
    }
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  issue_h(0);
#pragma unroll
  for (int s = 0; s < WS - 1; ++s)
    if (s < nK) issue_w(s);

  for (int kb = 0; kb < nK; ++kb) {
    const int cb = kb / 9, tap = kb - (kb / 9) * 9;
    // VMEM ops issued after W(kb) that may still be in flight:
    //   weights W(kb+1 .. kb+WS-2) and the halo H(cb+1) if it was issued (at tap 0 of this
    //   channel block, right after W(cb*9 + WS-1)) after W(kb), i.e. when 1 <= tap <= WS-1.
    const int wAfter = (nK - 1 - kb) < (WS - 2) ? (nK - 1 - kb) : (WS - 2);
    const bool hAfter = tap >= 1 && tap <= WS - 1 && cb + 1 < ncb;
    if constexpr (WS == 2) {
      if (hAfter) wait_vm<NH>(); else wait_vm<0>();
    } else {
      static_assert(WS == 3, "WS 2 or 3");
      if (wAfter == 1) { if (hAfter) wait_vm<NB + NH>(); else wait_vm<NB>(); }
      else { if (hAfter) wait_vm<NH>(); else wait_vm<0>(); }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kb + WS - 1 < nK) issue_w(kb + WS - 1);
    if (tap == 0 && cb + 1 < ncb) issue_h(cb + 1);

    const uint4* sW = sWbase + (kb % WS) * WSTAGE;
    const uint4* sH = sHbase + (cb & 1) * HSTAGE;
    const int ky = tap / 3, kx = tap - (tap / 3) * 3;
    const int dtap = ky * W2 + kx;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s * 4 + (lane >> 4);
      uint4 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = sW[swz(wco * TM * 16 + i * 16 + (lane & 15), ch)];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = sH[swz(frow[j] + dtap, ch)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                              __builtin_bit_cast(bf16x8_t, bfr[j]), acc[i][j], 0, 0, 0);
    }
  }

#pragma clang loop unroll(full)
  for (int i = 0; i < TM; ++i)
#pragma clang loop unroll(full)
    for (int j = 0; j < TN; ++j) {
      const int px = px0 + wpx * TN * 16 + j * 16 + (lane & 15);
      const int co = co0 + wco * TM * 16 + i * 16 + (lane >> 4) * 4;
      conv_epilogue<bf16_t, bf16_t>(a, px, co, acc[i][j]);
    }
}

template <int BCO, int NH, int WS>
static int launch_halo(const ConvArgs& a, hipStream_t s) {
  const int ntile = a.M / HALO_BPX;
  const int nco = a.d.Cout_pad / BCO;
  const size_t lds = (size_t)(WS * BCO + 2 * NH * 64) * 8 * 16;
  auto kern = conv_halo_kernel<BCO, NH, WS>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(ntile * nco), dim3(512), lds, s, a);
  return hiseg_check_launch("conv_halo");
}

// 1 if launched, 0 if not applicable, <0 on error.  variant: 0 = auto, 10+ = forced config.
int conv_halo_try(const ConvArgs& a, hipStream_t s, int variant) {
  const hiseg_conv2d_desc& d = a.d;
  if (d.dtype != HISEG_BF16 || d.out_dtype != HISEG_BF16 || d.convT) return 0;
  if (d.KH != 3 || d.KW != 3 || d.stride != 1 || d.pad != 1 || d.a_up != 1 || d.in_scale) return 0;
  if (d.Ca % 64 || d.Cb % 64 || d.K_pad != 9 * a.Cin) return 0;
  if (((d.a_cstride | d.a_coff) & 7) || (d.Cb && ((d.b_cstride | d.b_coff) & 7))) return 0;
  if (HALO_BPX % d.W) return 0;
  const int TH = HALO_BPX / d.W;
  if (d.H % TH) return 0;
  const int R = (TH + 2) * (d.W + 2);
  const long long span = (long long)d.N * d.H * d.W * (d.a_cstride > d.b_cstride ? d.a_cstride : d.b_cstride) * 2;
  if (span >= 0x7fffffffll || (long long)d.Cout_pad * d.K_pad * 2 >= 0x7fffffffll) return 0;
  int r;
  if (variant == 0 || variant < 10) {
    if (d.Cout_pad % 256 == 0 && R <= 5 * 64) variant = 10;
    else if (d.Cout_pad % 128 == 0 && R <= 7 * 64) variant = 11;
    else return 0;
  }
  switch (variant) {
    case 10: if (d.Cout_pad % 256 || R > 5 * 64) return 0; r = launch_halo<256, 5, 2>(a, s); break;
    case 11: if (d.Cout_pad % 128 || R > 7 * 64) return 0; r = launch_halo<128, 7, 3>(a, s); break;
    case 12: if (d.Cout_pad % 128 || R > 5 * 64) return 0; r = launch_halo<128, 5, 3>(a, s); break;
    case 13: if (d.Cout_pad % 64 || R > 7 * 64) return 0; r = launch_halo<64, 7, 3>(a, s); break;
    default: return 0;
  }
  return r < 0 ? r : 1;
}

}  // namespace hiseg
