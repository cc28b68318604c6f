// Pointwise (1x1 / stride 1) convolution and the ConvTranspose2d(k=2, s=2) GEMM on gfx950, bf16.
//
// These layers are HBM streams: K <= 288 input channels, so a 256-column output tile costs
// 2 * K * 256 flops per pixel against (K + 256) * 2 bytes of activations -- at most ~250 flop/B,
// far below the MFMA/HBM ridge (~310 flop/B).  The LDS-DMA ring kernels run them at 2.6-2.8 TB/s
// (tools/conv_bench.py): every 128x128 or 256x256 workgroup tile re-stages its weight block and pays
// a ring prologue and an LDS epilogue for only 8-9 K stages.
//
// Here one persistent workgroup per CU keeps its 256-column weight tile (<= 147 KiB) in LDS for the
// whole launch and streams pixels: each wave owns 32-pixel blocks (block b, b + #waves, ...), loads the
// block's activations straight into MFMA B-fragment registers (a lane's 8 consecutive channels of one
// pixel are 16 contiguous bytes of the NHWC row), prefetches the next block's while the current one's
// 16 x 2 x NKS MFMAs run (A = weight fragments read from LDS), and stores the epilogue straight from
// the accumulators (4 consecutive output channels = 8 bytes per lane).  Weight rows are padded by 16 B
// in LDS (row stride = 33 / 37 chunks), which makes the 16 rows of a fragment read hit distinct banks.
//
// ConvTranspose2d: GEMM column j = q * C + co (q = 2 dy + dx) of input pixel (n, y, x) lands at output
// pixel (n, 2y + dy, 2x + dx), channel co; a 512-column layer runs as two column tiles.
#include "conv_common.h"

namespace hiseg {

constexpr int kPwCT = 256;     // output columns per workgroup tile
constexpr int kPwBlk = 32;     // pixels per wave block (two 16-pixel MFMA columns)

// f2bf without the early return (a select, so the epilogue stays free of exec-mask branches)
__device__ __forceinline__ uint32_t pw_bf(float f) {
  const uint32_t u = __float_as_uint(f);
  const uint32_t r = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
  return (u & 0x7fffffffu) > 0x7f800000u ? ((u >> 16) | 0x40u) : r;
}

typedef unsigned pw_u4 __attribute__((ext_vector_type(4)));
typedef unsigned pw_u2 __attribute__((ext_vector_type(2)));

// NKS k-steps of 32 channels; NKS == 9: k-steps 0..7 from source A (Ca == 256), k-step 8 from source B
// (Cb <= 32 channels, the rest zero).  Every global access is a buffer instruction whose out-of-range lanes
// (pixel tail, channel tail, the block past the last) carry an offset beyond num_records: loads return zeros,
// stores are dropped -- no divergent branches, so the compiler's vmcnt waits stay counted.
// EPI: 0 plain, 1 residual added before the activation, 2 mul applied after it (include/hiseg.h epilogue).
template <int NKS, int EPI, int ACT, bool CONVT>
__global__ void __launch_bounds__(256, 1) conv_pw_kernel(ConvArgs a, int nct) {
  constexpr bool RES = EPI == 1, MUL = EPI == 2, XOP = EPI != 0;
  constexpr int RB = kPwCT / 16;               // 16-row blocks of the column tile
  constexpr int ROWC = NKS * 4 + 1;            // LDS row stride in 16-B chunks (one chunk of padding)
  constexpr int NA = NKS == 9 ? 8 : NKS;       // k-steps from source A
  constexpr unsigned OOB = 0x80000000u;
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int ct = blockIdx.x % nct;             // column tile
  const int grp = blockIdx.x / nct, ngrp = gridDim.x / nct;
  const int c0 = ct * kPwCT;

  // ---- weights of the column tile -> LDS (row r, chunk c at r * ROWC + c); scale / shift after them
  uint4* wl = smem;
  float* ssc = reinterpret_cast<float*>(smem + kPwCT * ROWC);
  float* ssh = ssc + kPwCT;
  const uint4* wg = reinterpret_cast<const uint4*>(d.weight);
  const int kc = d.K_pad >> 3;                 // 16-B chunks per global weight row
  for (int i = t; i < kPwCT * NKS * 4; i += 256) {
    const int r = i / (NKS * 4), c = i - r * (NKS * 4);
    wl[r * ROWC + c] = wg[(long long)(c0 + r) * kc + c];
  }
  for (int i = t; i < kPwCT; i += 256) {
    const int j = c0 + i < d.Cout ? c0 + i : 0;
    ssc[i] = d.scale[j];
    ssh[i] = d.shift[j];
  }
  __syncthreads();

  const int M = a.M;
  const int nblk = (M + kPwBlk - 1) / kPwBlk;
  const int g = lane >> 4, pl = lane & 15;
  const long long out_px = (long long)M * (CONVT ? 4 : 1);
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(d.srcA), (short)0, (int)((long long)M * d.a_cstride * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(NKS == 9 ? d.srcB : d.srcA), (short)0, NKS == 9 ? (int)((long long)M * d.b_cstride * 2) : 0,
      0x00020000);
  const __amdgpu_buffer_rsrc_t rO = __builtin_amdgcn_make_buffer_rsrc(d.out, (short)0,
                                                                     (int)(out_px * d.o_cstride * 2), 0x00020000);
  // the extra epilogue operand (residual or mul), same layout rules as the output
  const void* xp = RES ? d.residual : MUL ? d.mul : d.out;
  const int x_cs = RES ? d.r_cstride : d.m_cstride, x_coff = RES ? d.r_coff : d.m_coff;
  const __amdgpu_buffer_rsrc_t rR = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(xp), (short)0, XOP ? (int)(out_px * x_cs * 2) : 0, 0x00020000);
  const bool bch_ok = NKS == 9 && 8 * g < d.Cb;   // this lane's chunk of the source-B k-step holds channels

  // B fragments of block b: lane (g, pl) holds pixel b*32 + 16j + pl, channels 32 ks + 8 g .. + 7
  auto load_ks = [&](int b, int ks, uint4 (&bk)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int p = b * kPwBlk + 16 * j + pl;
      pw_u4 v;
      if (ks < NA) {
        const unsigned off = p < M ? (unsigned)((p * d.a_cstride + d.a_coff + 32 * ks + 8 * g) * 2) : OOB;
        v = __builtin_amdgcn_raw_buffer_load_b128(rA, off, 0, 0);
      } else {
        const unsigned off = (p < M && bch_ok) ? (unsigned)((p * d.b_cstride + d.b_coff + 8 * g) * 2) : OOB;
        v = __builtin_amdgcn_raw_buffer_load_b128(rB, off, 0, 0);
      }
      bk[j] = make_uint4(v.x, v.y, v.z, v.w);
    }
  };

  // byte offset of (input pixel p, tile column c0 + 16 i + 4 g) in a view (cs, coff), OOB if outside
  int pbase[2];            // per pixel column j: pixel row index (or its output-grid base for ConvTranspose)
  auto set_block = [&](int b) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int p = b * kPwBlk + 16 * j + pl;
      if constexpr (CONVT) {
        const int x = p % d.Wo, tt = p / d.Wo, y = tt % d.Ho, n = tt / d.Ho;
        pbase[j] = p < M ? (n * (2 * d.Ho) + 2 * y) * (2 * d.Wo) + 2 * x : -1;
      } else {
        pbase[j] = p < M ? p : -1;
      }
    }
  };
  auto offset = [&](int j, int i, int cs, int coff) __attribute__((always_inline)) -> unsigned {
    const int col = c0 + 16 * i + 4 * g;
    if (pbase[j] < 0 || col >= d.Cout) return OOB;
    if constexpr (CONVT) {
      const int C = d.Cout >> 2, q = col / C, co = col - q * C;
      const int op = pbase[j] + (q >> 1) * (2 * d.Wo) + (q & 1);
      return (unsigned)((op * cs + coff + co) * 2);
    } else {
      return (unsigned)((pbase[j] * cs + coff + col) * 2);
    }
  };

  // blocks of this wave: grp * 4 + w, then strides of all waves of the column tile's groups.  Two B buffers
  // in a loop unrolled by two: block b computes from one while block b + stride's fragments load into the
  // other (past the last block the loads are OOB zeros), so the loads have a whole block of MFMAs and its
  // epilogue to land and every wait is a counted vmcnt.
  const int stride = ngrp * 4;
  int b = grp * 4 + w;
  uint4 b0[NKS][2], b1[NKS][2];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) load_ks(b, ks, b0[ks]);
  auto process = [&](int b, const uint4 (&bf)[NKS][2], uint4 (&bn)[NKS][2]) __attribute__((always_inline)) {
    const int nb = b + stride;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) load_ks(nb, ks, bn[ks]);
    set_block(b);
    pw_u2 rv[XOP ? RB : 1][2];
    if constexpr (XOP) {
#pragma unroll
      for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) rv[i][j] = __builtin_amdgcn_raw_buffer_load_b64(rR, offset(j, i, x_cs, x_coff), 0, 0);
    }
    // the weight fragments are loop-invariant: an opaque base per block keeps the compiler from hoisting all
    // 16 x NKS of them (64 registers each k-step) out of the pixel loop
    int wofs = pl * ROWC + g;   // (an index, not a pointer: the asm would turn an LDS pointer into a flat one)
    asm volatile("" : "+v"(wofs));
    const uint4* wrow = smem + wofs;
    floatx4 acc[RB][2];
#pragma unroll
    for (int i = 0; i < RB; ++i) acc[i][0] = acc[i][1] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const uint4 af = wrow[16 * i * ROWC + 4 * ks];
        acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af),
                                                            __builtin_bit_cast(bf16x8_t, bf[ks][0]), acc[i][0], 0, 0, 0);
        acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af),
                                                            __builtin_bit_cast(bf16x8_t, bf[ks][1]), acc[i][1], 0, 0, 0);
      }
    }
    // epilogue: lane holds columns 16 i + 4 g .. + 3 of pixel 16 j + pl
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int cl = 16 * i + 4 * g;
      const floatx4 sc = *reinterpret_cast<const floatx4*>(ssc + cl);
      const floatx4 sh = *reinterpret_cast<const floatx4*>(ssh + cl);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[i][j][e] * sc[e] + sh[e];
          if constexpr (RES) v[e] += Quad<bf16_t>::get(make_uint2(rv[i][j].x, rv[i][j].y), e);
          v[e] = apply_act(v[e], ACT);
          if constexpr (MUL) v[e] *= Quad<bf16_t>::get(make_uint2(rv[i][j].x, rv[i][j].y), e);
        }
        pw_u2 q;
        q.x = pw_bf(v[0]) | (pw_bf(v[1]) << 16);
        q.y = pw_bf(v[2]) | (pw_bf(v[3]) << 16);
        __builtin_amdgcn_raw_buffer_store_b64(q, rO, offset(j, i, d.o_cstride, d.o_coff), 0, 0);
      }
    }
  };
  for (; b < nblk; b += 2 * stride) {
    process(b, b0, b1);
    if (b + stride >= nblk) break;
    process(b + stride, b1, b0);
  }
}

static int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <int NKS, int EPI, int ACT, bool CONVT>
static int launch_pw(const ConvArgs& a, hipStream_t s) {
  const hiseg_conv2d_desc& d = a.d;
  const size_t lds = (size_t)kPwCT * (NKS * 4 + 1) * 16 + 2 * kPwCT * 4;
  auto kern = conv_pw_kernel<NKS, EPI, ACT, CONVT>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int nct = d.Cout_pad / kPwCT;
  const int nblk = (a.M + kPwBlk - 1) / kPwBlk;
  int groups = cu_count() / nct;                       // one workgroup per CU in all
  const int need = (nblk + 3) / 4;
  if (groups > need) groups = need;
  if (groups < 1) groups = 1;
  hipLaunchKernelGGL(kern, dim3(groups * nct), dim3(256), lds, s, a, nct);
  return hiseg_check_launch("conv_pw");
}

template <int NKS>
static int launch_pw_k(const ConvArgs& a, hipStream_t s) {
  const hiseg_conv2d_desc& d = a.d;
  constexpr int N = HISEG_ACT_NONE, R = HISEG_ACT_RELU, S = HISEG_ACT_SIGMOID;
  const int act = d.act;
  if constexpr (NKS == 9) {   // the 256 + 8 combiner: plain outputs only (the other forms would spill)
    return act == R ? launch_pw<NKS, 0, R, false>(a, s) : launch_pw<NKS, 0, N, false>(a, s);
  } else {
    if (d.convT) return act == R ? launch_pw<NKS, 0, R, true>(a, s) : launch_pw<NKS, 0, N, true>(a, s);
    if (d.residual) return act == R ? launch_pw<NKS, 1, R, false>(a, s) : launch_pw<NKS, 1, N, false>(a, s);
    if (d.mul) return act == S ? launch_pw<NKS, 2, S, false>(a, s) : launch_pw<NKS, 2, N, false>(a, s);
    return act == R ? launch_pw<NKS, 0, R, false>(a, s)
         : act == S ? launch_pw<NKS, 0, S, false>(a, s) : launch_pw<NKS, 0, N, false>(a, s);
  }
}

// Returns 1 if launched, 0 if the layer does not qualify (caller falls back), <0 on error.  variant 90.
int conv_pw_try(const ConvArgs& a, hipStream_t s, int variant) {
  const hiseg_conv2d_desc& d = a.d;
  if (variant != 90) return 0;
  if (d.dtype != HISEG_BF16 || d.out_dtype != HISEG_BF16) return 0;
  if (d.KH != 1 || d.KW != 1 || d.stride != 1 || d.pad != 0 || d.a_up != 1) return 0;
  if (d.in_scale || d.out2) return 0;
  if (d.residual && d.mul) return 0;
  if (d.act == HISEG_ACT_SIGMOID ? (d.convT || d.residual) : (d.act != HISEG_ACT_NONE && d.act != HISEG_ACT_RELU))
    return 0;
  if (d.mul && (d.act == HISEG_ACT_RELU || d.convT || ((d.m_cstride | d.m_coff) & 3))) return 0;
  if (d.convT && d.residual) return 0;
  if (d.Ca % 32 || d.Cb % 8 || d.Cout % 4 || d.Cout_pad % kPwCT) return 0;
  if (d.convT && (d.Cout / 4) % 4) return 0;
  const int nks = (a.Cin + 31) / 32;
  if (d.K_pad < nks * 32) return 0;
  if (nks == 9 ? (d.Ca != 256 || d.Cb > 32 || d.convT || d.residual || d.mul || d.act == HISEG_ACT_SIGMOID) : d.Cb != 0)
    return 0;
  const long long out_px = (long long)a.M * (d.convT ? 4 : 1);
  const long long lim = 0x7fffffffll;
  if ((long long)a.M * d.a_cstride * 2 >= lim || (d.Cb && (long long)a.M * d.b_cstride * 2 >= lim) ||
      out_px * d.o_cstride * 2 >= lim || (d.residual && out_px * d.r_cstride * 2 >= lim) ||
      (d.mul && out_px * d.m_cstride * 2 >= lim))
    return 0;
  if ((d.a_cstride | d.a_coff) & 7) return 0;
  if (d.Cb && ((d.b_cstride | d.b_coff) & 7)) return 0;
  if (((d.o_cstride | d.o_coff) & 3) || (d.residual && ((d.r_cstride | d.r_coff) & 3))) return 0;
  if (((uintptr_t)d.out | (uintptr_t)d.residual | (uintptr_t)d.mul) & 7) return 0;
  int r;
  switch (nks) {
    case 4: r = launch_pw_k<4>(a, s); break;
    case 8: r = launch_pw_k<8>(a, s); break;
    case 9: r = launch_pw_k<9>(a, s); break;
    default: return 0;
  }
  return r < 0 ? r : 1;
}

}  // namespace hiseg
