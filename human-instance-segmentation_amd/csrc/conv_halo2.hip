// 3x3 / stride-1 convolution: LDS-resident input halo + weights streamed into registers
// (bf16, gfx950).  The kernel the ROI head's 256/128/64-channel 3x3 layers run on.
//
// Why this shape (measured on the LDS-ring kernels, conv_fast/conv_halo): with both operands
// staged through LDS the workgroup spends >50 % of its wave cycles in s_waitcnt — the bytes a
// CU can keep in flight are capped by LDS capacity, not by bandwidth.  Here
//   * the activation operand is a (TH+2) x (W+2) halo of one 64-channel block (TH = 192/W whole
//     output rows of one image), loaded ONCE per channel block for all 9 taps, double buffered
//     and prefetched a whole channel block (9 K blocks) ahead through registers;
//   * the weight operand never touches LDS: the host packs it in MFMA-fragment order so each
//     wave loads its A fragments with one contiguous 1 KiB global_load_dwordx4 per
//     (16-row tile, k-step), prefetched 3 K blocks ahead in registers (the register file, not
//     LDS, holds the in-flight bytes);
//   * one barrier per channel block (halo buffer hand-over), none per K block; every load is a
//     plain compiler-visible load, so hipcc's own counted vmcnt waits are exact.
// Halo rows are 160 B (128 B + 32 B pad, a stride of 10 16-B bank slots): for every row base
// (the tap shift) the four ds_read_b128 lane groups of a B-fragment read (MI355X_MICROARCH.md
// §LDS) hit 16 distinct slots (checked exhaustively; 128-B rows with the XOR swizzle are 2-way
// for odd bases, 144-B rows 2-way), so the per-tap shift is a plain address add.  8 waves = WCO (Cout) x WPX (pixels).
#include "conv_common.h"

namespace hiseg {

constexpr int H2_BPX = 192;
constexpr int H2_ROWB = 160;  // 128 B + 32 B pad: row stride of 10 bank slots

template <int BCO, int WCO, int WPX, int NHL>
__global__ void __launch_bounds__(512) conv_halo2_kernel(ConvArgs a) {
  constexpr int TMW = BCO / (16 * WCO);
  constexpr int TN = H2_BPX / (16 * WPX);
  constexpr int MAXR = NHL * 512 / 8;          // halo rows per buffer
  constexpr int HBUF = MAXR * H2_ROWB;         // bytes per halo buffer
  constexpr int JG = TN > 6 ? TN / 2 : TN;     // B fragments live at a time
  static_assert(WCO * WPX == 8 && TMW >= 1 && TN >= 1, "tile");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* const lds = reinterpret_cast<char*>(smem);
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wco = w / WPX, wpx = w % WPX;
  const int W = d.W, H = d.H, W2 = d.W + 2;
  const int TH = H2_BPX / W;

  const int nco = d.Cout_pad / BCO;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int q = nwg >> 3, r8 = nwg & 7, xcd = orig & 7, loc = orig >> 3;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + loc;
  const int co0 = (wg % nco) * BCO;
  const int px0 = (wg / nco) * H2_BPX;
  const int n = px0 / (H * W);
  const int y0 = (px0 - n * H * W) / W;

  // ---- halo chunks owned by this thread: g = t + 512 i  ->  row g>>3, chunk g&7
  const int R = (TH + 2) * W2;
  int hpix[NHL], hlds[NHL];
  bool hok[NHL], hin[NHL];
#pragma unroll
  for (int i = 0; i < NHL; ++i) {
    const int g = t + 512 * i;
    const int r = g >> 3, c = g & 7;
    const int hy = r / W2, hx = r - (r / W2) * W2;
    const int iy = y0 - 1 + hy, ix = hx - 1;
    hin[i] = r < R;
    hok[i] = hin[i] && iy >= 0 && iy < H && ix >= 0 && ix < W;
    hpix[i] = (n * H + iy) * W + ix;
    hlds[i] = r * H2_ROWB + c * 16;
  }
  // ---- B-fragment row base (tap (0,0)) of this lane, per pixel tile
  int fb[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int p = wpx * (TN * 16) + j * 16 + (lane & 15);
    fb[j] = ((p / W) * W2 + (p - (p / W) * W)) * H2_ROWB + (lane >> 4) * 16;
  }

  const int Cin = a.Cin;
  const int ncb = Cin >> 6;
  const int nK = ncb * 9;
  // fragment-ordered weights: block (ct, kb, s) = 1 KiB at ((ct*nK + kb)*2 + s) KiB
  const char* wbase = reinterpret_cast<const char*>(d.weight_frag) +
                      ((size_t)(co0 / 16 + wco * TMW) * nK * 2) * 1024 + lane * 16;
  const size_t ct_stride = (size_t)nK * 2 * 1024;

  uint4 wreg[3][TMW][2];
  uint4 hreg[NHL];

  auto load_w = [&](int st, int kb) __attribute__((always_inline)) {
#pragma unroll
    for (int ti = 0; ti < TMW; ++ti)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        wreg[st][ti][s] = *reinterpret_cast<const uint4*>(wbase + ti * ct_stride + ((size_t)kb * 2 + s) * 1024);
  };
  // Every load and LDS store below is unconditional (out-of-image / padding chunks load from a
  // valid address and are zeroed at store time): loads under exec-masked branches make hipcc's
  // waitcnt pass fall back to vmcnt(0), which would drain the weight prefetch every few taps.
  auto load_h = [&](int cb) __attribute__((always_inline)) {
    const int ci0 = cb << 6;
    const bool fromA = ci0 < d.Ca;
    const char* src = reinterpret_cast<const char*>(fromA ? d.srcA : d.srcB);
    const int cs = fromA ? d.a_cstride : d.b_cstride;
    const int cbase = fromA ? d.a_coff + ci0 : d.b_coff + ci0 - d.Ca;
#pragma unroll
    for (int i = 0; i < NHL; ++i) {
      const int c = (t + 512 * i) & 7;
      const size_t off = hok[i] ? ((size_t)hpix[i] * cs + cbase + c * 8) * 2 : (size_t)(cbase + c * 8) * 2;
      hreg[i] = *reinterpret_cast<const uint4*>(src + off);
    }
  };
  auto store_h = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NHL; ++i) {
      const uint4 z = make_uint4(0u, 0u, 0u, 0u);
      *reinterpret_cast<uint4*>(lds + buf * HBUF + hlds[i]) = hok[i] ? hreg[i] : z;
    }
  };

  floatx4 acc[TMW][TN];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  load_w(0, 0);
  load_w(1, 1 < nK ? 1 : nK - 1);
  load_w(2, 2 < nK ? 2 : nK - 1);
  load_h(0);
  store_h(0);

  for (int cb = 0; cb < ncb; ++cb) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool more = cb + 1 < ncb;
    if (more) load_h(cb + 1);
    const char* hb = lds + (cb & 1) * HBUF;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kb = cb * 9 + tap;
      const int st = tap % 3;
      const int dt = ((tap / 3) * W2 + (tap % 3)) * H2_ROWB;
      int addr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) addr[j] = fb[j] + dt;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int j0 = 0; j0 < TN; j0 += JG) {
          uint4 bfr[JG];
#pragma unroll
          for (int j = 0; j < JG; ++j) bfr[j] = *reinterpret_cast<const uint4*>(hb + addr[j0 + j] + s * 64);
#pragma unroll
          for (int ti = 0; ti < TMW; ++ti)
#pragma unroll
            for (int j = 0; j < JG; ++j)
              acc[ti][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  __builtin_bit_cast(bf16x8_t, wreg[st][ti][s]), __builtin_bit_cast(bf16x8_t, bfr[j]),
                  acc[ti][j0 + j], 0, 0, 0);
        }
      }
      load_w(st, kb + 3 < nK ? kb + 3 : nK - 1);  // tail: harmless reload, keeps the stream branch-free
      if (tap == 5 && more) store_h((cb + 1) & 1);
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

template <int BCO, int WCO, int WPX, int NHL>
static int launch_halo2(const ConvArgs& a, hipStream_t s) {
  const int ntile = a.M / H2_BPX;
  const int nco = a.d.Cout_pad / BCO;
  const size_t lds = (size_t)2 * (NHL * 512 / 8) * H2_ROWB;
  auto kern = conv_halo2_kernel<BCO, WCO, WPX, NHL>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(ntile * nco), dim3(512), lds, s, a);
  return hiseg_check_launch("conv_halo2");
}

// 1 if launched, 0 if not applicable, <0 on error.  variant: 0 auto, 20+ forced.
int conv_halo2_try(const ConvArgs& a, hipStream_t s, int variant) {
  const hiseg_conv2d_desc& d = a.d;
  if (!d.weight_frag) return 0;
  if (d.dtype != HISEG_BF16 || d.out_dtype != HISEG_BF16 || d.convT) return 0;
  if (d.KH != 3 || d.KW != 3 || d.stride != 1 || d.pad != 1 || d.a_up != 1 || d.in_scale) return 0;
  if (d.Ca % 64 || d.Cb % 64 || d.K_pad != 9 * a.Cin) return 0;
  if (((d.a_cstride | d.a_coff) & 7) || (d.Cb && ((d.b_cstride | d.b_coff) & 7))) return 0;
  if (H2_BPX % d.W) return 0;
  const int TH = H2_BPX / d.W;
  if (d.H % TH) return 0;
  const int R = (TH + 2) * (d.W + 2);
  if (variant == 0 || variant < 20) {
    if (d.Cout_pad % 256 == 0 && R <= 320) variant = 20;
    else if (d.Cout_pad % 128 == 0) variant = R <= 320 ? 22 : 21;
    else if (d.Cout_pad % 64 == 0) variant = R <= 320 ? 24 : 23;
    else return 0;
  }
  int r;
  switch (variant) {
    case 20: if (d.Cout_pad % 256 || R > 320) return 0; r = launch_halo2<256, 8, 1, 5>(a, s); break;
    case 21: if (d.Cout_pad % 128 || R > 448) return 0; r = launch_halo2<128, 4, 2, 7>(a, s); break;
    case 22: if (d.Cout_pad % 128 || R > 320) return 0; r = launch_halo2<128, 4, 2, 5>(a, s); break;
    case 23: if (d.Cout_pad % 64 || R > 448) return 0; r = launch_halo2<64, 2, 4, 7>(a, s); break;
    case 24: if (d.Cout_pad % 64 || R > 320) return 0; r = launch_halo2<64, 2, 4, 5>(a, s); break;
    case 25: if (d.Cout_pad % 128 || R > 320) return 0; r = launch_halo2<128, 8, 1, 5>(a, s); break;
    default: return 0;
  }
  return r < 0 ? r : 1;
}

}  // namespace hiseg
