// Pointwise (1x1 / stride 1) convolution and the ConvTranspose2d(k=2, s=2) GEMM on gfx950, bf16.
//
// These layers are HBM streams: K <= 288 input channels, so a 256-column output tile costs
// 2 * K * 256 flops per pixel against (K + 256) * 2 bytes of activations -- at most ~250 flop/B,
// far below the MFMA/HBM ridge (~310 flop/B).  The LDS-DMA ring kernels run them at 2.6-2.8 TB/s
// (tools/conv_bench.py): every 128x128 or 256x256 workgroup tile re-stages its weight block and pays
// a ring prologue and an LDS epilogue for only 8-9 K stages.
//
// Here persistent workgroups keep their column tile of the weights (<= 147 KiB) in LDS for the whole
// launch and stream pixels: each wave owns 32-pixel blocks (block b, b + #waves, ...), loads the block's
// activations straight into MFMA B-fragment registers (a lane's 8 consecutive channels of one pixel are 16
// contiguous bytes of the NHWC row), prefetches the next block's while the current one's RB x 2 x nks MFMAs
// run (A = weight fragments read from LDS), and stores the epilogue straight from the accumulators (4
// consecutive output channels = 8 bytes per lane).  Weight rows are padded by 16 B in LDS (row stride =
// 4 NKS + 1 chunks), which makes the 16 rows of a fragment read hit distinct banks.
//
// Column tiles of CT = 16 RB columns: RB = 16 for the head's 256-multiple layers; the EfficientNet encoder's
// 1x1 layers (timm InvertedResidual conv_pw / conv_pwl, DepthwiseSeparableConv conv_pw; efficientnet.py in
// timm 1.0.19) have 16..1152 columns and 16..240 input channels (K <= 256: nks <= 8 k-steps, a runtime count
// up to the template's NKS): RB 1..8 for narrow projections, RB 16 with ragged last tiles for the wide
// expansions (672 = 3 tiles, the third half empty).  Input channel tails (Ca a multiple of 8, not of 32) read
// zeros through out-of-range offsets.  INS: the squeeze-excite gate of the projection's input (in_scale
// [N][Ca], f32) is staged in LDS once per workgroup and applied to each fragment in registers, rounded to
// bf16 exactly as the generic kernel's loader does (conv_igemm.hip gather), so results stay bit-identical.
//
// ConvTranspose2d: GEMM column j = q * C + co (q = 2 dy + dx) of input pixel (n, y, x) lands at output
// pixel (n, 2y + dy, 2x + dx), channel co; a 512-column layer runs as two column tiles.
//
// Built twice (Makefile): this file (HISEG_PW_PART 1: RB 16, and conv_pw_try) and conv_pw_n.hip
// (HISEG_PW_PART 2: RB 1, 2, 4, 8; up to 10 k-steps at RB <= 4).
#include "conv_common.h"

#ifndef HISEG_PW_PART
#define HISEG_PW_PART 1
#endif

namespace hiseg {

constexpr int kPwBlk = 32;     // pixels per wave block (two 16-pixel MFMA columns)
constexpr int kPwActRt = -1;   // ACT template value: activation read from the descriptor at run time

typedef unsigned pw_u4 __attribute__((ext_vector_type(4)));
typedef unsigned pw_u2 __attribute__((ext_vector_type(2)));

// NKS: k-steps of 32 channels held in registers (nks <= NKS of them used); NKS == 9:
// k-steps 0..7 from source A (Ca == 256), k-step 8 from source B (Cb <= 32 channels, the rest zero).  Every
// global access is a buffer instruction whose out-of-range lanes (pixel tail, channel tail, the block past
// the last) carry an offset beyond num_records: loads return zeros, stores are dropped -- no divergent
// branches, so the compiler's vmcnt waits stay counted.
// EPI: 0 plain, 1 residual added before the activation, 2 mul applied after it (include/hiseg.h epilogue).
template <int NKSA, int EPI, int ACT, bool CONVT, int RB, bool INS>
__global__ void __launch_bounds__(256, 1) conv_pw_kernel(ConvArgs a, int nct, int nks_arg) {
  // NKSA > 0: exactly NKSA k-steps (the head's layers: no run-time guards, which cost the residual / mul
  // forms registers); NKSA < 0: a run-time count nks_arg <= -NKSA
  constexpr int NKS = NKSA < 0 ? -NKSA : NKSA;
  const int nks = NKSA < 0 ? nks_arg : NKSA;
  constexpr bool RES = EPI == 1, MUL = EPI == 2, XOP = EPI != 0;
  constexpr int CT = 16 * RB;                  // output columns per workgroup tile
  constexpr int ROWC = NKS * 4 + 1;            // LDS row stride in 16-B chunks (one chunk of padding)
  constexpr int NA = NKS == 9 ? 8 : NKS;       // k-steps from source A
  constexpr unsigned OOB = 0x80000000u;
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int ct = blockIdx.x % nct;             // column tile
  const int grp = blockIdx.x / nct, ngrp = gridDim.x / nct;
  const int c0 = ct * CT;
  const int act = ACT == kPwActRt ? d.act : ACT;
#ifdef HISEG_DIAG
  const int abl = a.abl;   // timing ablations (variants 190-221): 1 staging, 2 loads, 4 MFMAs, 8 epilogue math, 16 stores
#else
  constexpr int abl = 0;
#endif

  // ---- weights of the column tile -> LDS (row r, chunk c at r * ROWC + c; rows past Cout_pad zero); scale /
  // shift after them, then (INS) the gate table [N][Ca]
  uint4* wl = smem;
  float* ssc = reinterpret_cast<float*>(smem + CT * ROWC);
  float* ssh = ssc + CT;
  float* gl = ssh + CT;
  // Staged kPwStage chunks per thread at a time, all loads of a round issued before its LDS stores: a rolled
  // load -> store loop waits out one L2/HBM latency per 16-B chunk, 28 times over for a 224-channel 256-column
  // tile, which cost the EfficientNet layers (a few 32-pixel blocks per wave) 20-40 us per launch.  Loads past
  // the tile (or past Cout_pad) are OOB buffer reads: zeros, no branches.
  constexpr int kPwStage = 8;
  const int kc = d.K_pad >> 3;                 // 16-B chunks per global weight row
  const int wch = nks * 4;                     // chunks per row that are used
  const int nchunk = CT * wch;
  {
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(d.weight), (short)0, (int)((long long)d.Cout_pad * kc * 16), 0x00020000);
    for (int i0 = t; i0 < ((abl & 1) ? 0 : nchunk); i0 += 256 * kPwStage) {
      pw_u4 v[kPwStage];
#pragma unroll
      for (int u = 0; u < kPwStage; ++u) {
        const int i = i0 + 256 * u;
        const int r = i / wch, c = i - r * wch;
        const unsigned off = i < nchunk ? (unsigned)(((c0 + r) * kc + c) * 16) : 0x80000000u;
        v[u] = __builtin_amdgcn_raw_buffer_load_b128(rW, off, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kPwStage; ++u) {
        const int i = i0 + 256 * u;
        const int r = i / wch, c = i - r * wch;
        if (i < nchunk) wl[r * ROWC + c] = make_uint4(v[u].x, v[u].y, v[u].z, v[u].w);
      }
    }
  }
  for (int i = t; i < CT; i += 256) {
    const int j = c0 + i < d.Cout ? c0 + i : 0;
    ssc[i] = d.scale[j];
    ssh[i] = d.shift[j];
  }
  if constexpr (INS) {   // the gate table [N][Ca] f32, 16-B aligned, N Ca a multiple of 8: float4 chunks, staged
    const int n4 = d.N * d.Ca / 4;
    const __amdgpu_buffer_rsrc_t rG = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(d.in_scale), (short)0, (int)(n4 * 16), 0x00020000);
    float4* gl4 = reinterpret_cast<float4*>(gl);
    for (int i0 = t; i0 < n4; i0 += 256 * kPwStage) {
      pw_u4 v[kPwStage];
#pragma unroll
      for (int u = 0; u < kPwStage; ++u) {
        const int i = i0 + 256 * u;
        v[u] = __builtin_amdgcn_raw_buffer_load_b128(rG, i < n4 ? (unsigned)(i * 16) : 0x80000000u, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kPwStage; ++u) {
        const int i = i0 + 256 * u;
        if (i < n4) gl4[i] = __builtin_bit_cast(float4, v[u]);
      }
    }
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
    if (abl & 2) {
      bk[0] = bk[1] = make_uint4(0u, 0u, 0u, 0u);
      return;
    }
    const bool ch_ok = 32 * ks + 8 * g < d.Ca;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int p = b * kPwBlk + 16 * j + pl;
      pw_u4 v;
      if (ks < NA) {
        const unsigned off = (p < M && ch_ok) ? (unsigned)((p * d.a_cstride + d.a_coff + 32 * ks + 8 * g) * 2) : OOB;
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
  const int hw = d.H * d.W;

  // blocks of this wave: grp * 4 + w, then strides of all waves of the column tile's groups.  Two B buffers
  // in a loop unrolled by two: block b computes from one while block b + stride's fragments load into the
  // other (past the last block the loads are OOB zeros), so the loads have a whole block of MFMAs and its
  // epilogue to land and every wait is a counted vmcnt.
  const int stride = ngrp * 4;
  int b = grp * 4 + w;
  uint4 b0[NKS][2], b1[NKS][2];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks)
    if (ks < nks) load_ks(b, ks, b0[ks]);
  auto process = [&](int b, uint4 (&bf)[NKS][2], uint4 (&bn)[NKS][2]) __attribute__((always_inline)) {
    const int nb = b + stride;
    if constexpr (INS) {   // gate the current block's fragments before the next block's loads reuse registers
      int gofs[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int p = b * kPwBlk + 16 * j + pl;
        const int n = p < M ? p / hw : 0;
        gofs[j] = n * d.Ca;
      }
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        if (ks >= nks) continue;
        const int ch = 32 * ks + 8 * g < d.Ca ? 32 * ks + 8 * g : d.Ca - 8;   // masked lanes hold zeros
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float4* gp = reinterpret_cast<const float4*>(gl + gofs[j] + ch);
          const float4 s0 = gp[0], s1 = gp[1];
          float f[8];
          Chunk<bf16_t>::unpack(bf[ks][j], f);
          f[0] *= s0.x; f[1] *= s0.y; f[2] *= s0.z; f[3] *= s0.w;
          f[4] *= s1.x; f[5] *= s1.y; f[6] *= s1.z; f[7] *= s1.w;
          bf[ks][j] = Chunk<bf16_t>::pack(f);
        }
      }
    }
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      if (ks < nks) load_ks(nb, ks, bn[ks]);
    set_block(b);
    pw_u2 rv[XOP ? RB : 1][2];
    if constexpr (XOP) {
#pragma unroll
      for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) rv[i][j] = __builtin_amdgcn_raw_buffer_load_b64(rR, offset(j, i, x_cs, x_coff), 0, 0);
    }
    // the weight fragments are loop-invariant: an opaque base per block keeps the compiler from hoisting all
    // RB x NKS of them (4 registers each) out of the pixel loop
    int wofs = pl * ROWC + g;   // (an index, not a pointer: the asm would turn an LDS pointer into a flat one)
    asm volatile("" : "+v"(wofs));
    const uint4* wrow = smem + wofs;
    floatx4 acc[RB][2];
#pragma unroll
    for (int i = 0; i < RB; ++i) acc[i][0] = acc[i][1] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (ks >= nks) continue;
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        if (abl & 4) continue;
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
          if (abl & 8) {
            v[e] = acc[i][j][e];
            continue;
          }
          v[e] = acc[i][j][e] * sc[e] + sh[e];
          if constexpr (RES) v[e] += Quad<bf16_t>::get(make_uint2(rv[i][j].x, rv[i][j].y), e);
          v[e] = apply_act(v[e], act);
          if constexpr (MUL) v[e] *= Quad<bf16_t>::get(make_uint2(rv[i][j].x, rv[i][j].y), e);
        }
        pw_u2 q;
        q.x = f2bf2(v[0], v[1]);
        q.y = f2bf2(v[2], v[3]);
        if (!(abl & 16)) __builtin_amdgcn_raw_buffer_store_b64(q, rO, offset(j, i, d.o_cstride, d.o_coff), 0, 0);
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

static size_t pw_lds_bytes(int NKS, int RB, bool ins, const hiseg_conv2d_desc& d) {
  return (size_t)16 * RB * (NKS * 4 + 1) * 16 + 2 * 16 * RB * 4 + (ins ? (size_t)d.N * d.Ca * 4 : 0);
}

template <int NKSA, int EPI, int ACT, bool CONVT, int RB, bool INS>
static int launch_pw(const ConvArgs& a, hipStream_t s, int nks) {
  const hiseg_conv2d_desc& d = a.d;
  const size_t lds = pw_lds_bytes(NKSA < 0 ? -NKSA : NKSA, RB, INS, d);
  auto kern = conv_pw_kernel<NKSA, EPI, ACT, CONVT, RB, INS>;
  static int occ = 0;   // resident workgroups per CU at the largest LDS request seen (the gate table varies)
  static size_t occ_lds = 0;
  if (lds > occ_lds) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)kern, 256, lds) != hipSuccess || nb < 1) nb = 1;
    occ = nb > 4 ? 4 : nb;
    occ_lds = lds;
  }
  const int nct = (d.Cout_pad + 16 * RB - 1) / (16 * RB);
  const int nblk = (a.M + kPwBlk - 1) / kPwBlk;
  int groups = cu_count() * occ / nct;                  // every resident slot of the chip in all
  const int need = (nblk + 3) / 4;
  if (groups > need) groups = need;
  if (groups < 1) groups = 1;
  hipLaunchKernelGGL(kern, dim3(groups * nct), dim3(256), lds, s, a, nct, nks);
  return hiseg_check_launch("conv_pw");
}

// narrow column tiles (conv_pw_n.hip): RB 1, 2, 4 or 8; plain / residual epilogue, optional SE gate
int launch_pw_narrow(const ConvArgs& a, hipStream_t s, int rb, int nks_max, int nks);

#if HISEG_PW_PART == 2
// The activation is a template argument for the forms the encoder / head layers use (identity: the projections,
// SE-gated or not; ReLU: the head; SiLU: the EfficientNet expansions) and a run-time switch otherwise: with the switch
// inlined per output element the RB 4 kernels were 40-50 KB of code against ~15 KB.
template <int RB, int NKS>
static int launch_pw_n2(const ConvArgs& a, hipStream_t s, int nks) {
  const hiseg_conv2d_desc& d = a.d;
  constexpr int N = HISEG_ACT_NONE, R = HISEG_ACT_RELU, SI = HISEG_ACT_SILU, RT = kPwActRt;
  const bool ins = d.in_scale != nullptr;
  const int act = d.act;
  if (ins) {
    if (d.residual) return act == N ? launch_pw<-NKS, 1, N, false, RB, true>(a, s, nks)
                                    : launch_pw<-NKS, 1, RT, false, RB, true>(a, s, nks);
    return act == N ? launch_pw<-NKS, 0, N, false, RB, true>(a, s, nks)
                    : launch_pw<-NKS, 0, RT, false, RB, true>(a, s, nks);
  }
  if (d.residual) return act == N ? launch_pw<-NKS, 1, N, false, RB, false>(a, s, nks)
                       : act == R ? launch_pw<-NKS, 1, R, false, RB, false>(a, s, nks)
                                  : launch_pw<-NKS, 1, RT, false, RB, false>(a, s, nks);
  return act == N ? launch_pw<-NKS, 0, N, false, RB, false>(a, s, nks)
       : act == R ? launch_pw<-NKS, 0, R, false, RB, false>(a, s, nks)
       : act == SI ? launch_pw<-NKS, 0, SI, false, RB, false>(a, s, nks)
                   : launch_pw<-NKS, 0, RT, false, RB, false>(a, s, nks);
}
template <int RB>
static int launch_pw_n1(const ConvArgs& a, hipStream_t s, int nks_max, int nks) {
  if (nks_max == 2) return launch_pw_n2<RB, 2>(a, s, nks);
  if (nks_max == 4) return launch_pw_n2<RB, 4>(a, s, nks);
  if constexpr (RB <= 4) {
    if (nks_max == 10) return launch_pw_n2<RB, 10>(a, s, nks);
  }
  return launch_pw_n2<RB, 8>(a, s, nks);
}
int launch_pw_narrow(const ConvArgs& a, hipStream_t s, int rb, int nks_max, int nks) {
  switch (rb) {
    case 1: return launch_pw_n1<1>(a, s, nks_max, nks);
    case 2: return launch_pw_n1<2>(a, s, nks_max, nks);
    case 4: return launch_pw_n1<4>(a, s, nks_max, nks);
    default: return launch_pw_n1<8>(a, s, nks_max, nks);
  }
}
#else
template <int NKS>
static int launch_pw_k(const ConvArgs& a, hipStream_t s, int nks) {
  const hiseg_conv2d_desc& d = a.d;
  constexpr int N = HISEG_ACT_NONE, R = HISEG_ACT_RELU, S = HISEG_ACT_SIGMOID, SI = HISEG_ACT_SILU;
  const int act = d.act;
  if constexpr (NKS == 9) {   // the 256 + 8 combiner: plain outputs only (the other forms would spill)
    return act == R ? launch_pw<NKS, 0, R, false, 16, false>(a, s, nks) : launch_pw<NKS, 0, N, false, 16, false>(a, s, nks);
  } else {
    if (nks != NKS) {   // a k-step count below the register tile: plain epilogue (EfficientNet expansions)
      HISEG_REQUIRE(!(d.convT || d.residual || d.mul), HISEG_ERR_BAD_ARG,
                    "conv_pw: residual / mul / ConvTranspose forms need 2, 4 or 8 k-steps (pw_plan declines them)");
      return act == R ? launch_pw<-NKS, 0, R, false, 16, false>(a, s, nks)
           : act == S ? launch_pw<-NKS, 0, S, false, 16, false>(a, s, nks)
           : act == SI ? launch_pw<-NKS, 0, SI, false, 16, false>(a, s, nks)
                       : launch_pw<-NKS, 0, N, false, 16, false>(a, s, nks);
    }
    if (d.convT) return act == R ? launch_pw<NKS, 0, R, true, 16, false>(a, s, nks)
                                 : launch_pw<NKS, 0, N, true, 16, false>(a, s, nks);
    if (d.residual) return act == R ? launch_pw<NKS, 1, R, false, 16, false>(a, s, nks)
                                    : launch_pw<NKS, 1, N, false, 16, false>(a, s, nks);
    if (d.mul) return act == S ? launch_pw<NKS, 2, S, false, 16, false>(a, s, nks)
                               : launch_pw<NKS, 2, N, false, 16, false>(a, s, nks);
    return act == R ? launch_pw<NKS, 0, R, false, 16, false>(a, s, nks)
         : act == S ? launch_pw<NKS, 0, S, false, 16, false>(a, s, nks)
         : act == SI ? launch_pw<NKS, 0, SI, false, 16, false>(a, s, nks)
                     : launch_pw<NKS, 0, N, false, 16, false>(a, s, nks);
  }
}

// The pointwise kernel's plan for a layer: false when it does not qualify (caller falls back).
static constexpr long long kPwGateBytes = 64 * 1024;   // LDS bytes for an SE gate [N][Ca] f32
static bool pw_plan(const ConvArgs& a, int& rb, int& nks, int& nks_max) {
  const hiseg_conv2d_desc& d = a.d;
  if (d.dtype != HISEG_BF16 || d.out_dtype != HISEG_BF16) return false;
  if (d.KH != 1 || d.KW != 1 || d.stride != 1 || d.pad != 0 || d.a_up != 1) return false;
  if (d.out2) return false;
  if (d.residual && d.mul) return false;
  if (d.Ca % 8 || d.Cb % 8 || d.Cout % 4) return false;
  if (d.convT && (d.Cout / 4) % 4) return false;
  if (d.convT && d.residual) return false;
  nks = (a.Cin + 31) / 32;
  if (d.K_pad < nks * 32 || nks > 10) return false;
  // HISEG_PW_EFF=0 restores the round-2 v5 coverage (256-multiple columns, 4 / 8 / 9 k-steps of whole 32-channel
  // slices, no SE gate) for same-box A/B timing
  static const bool eff = [] { const char* e = getenv("HISEG_PW_EFF"); return !(e && atoi(e) == 0); }();
  if (!eff && (d.Cout_pad % 256 || d.Ca % 32 || d.in_scale || (nks != 4 && nks != 8 && nks != 9))) return false;
  // 9 k-steps at 256-column tiles: the 256 + 8 combiner only; 9..10 k-steps at narrow tiles: a single source of
  // up to 320 channels (the B7 encoder's 288-channel SE-gated projections)
  rb = 16;
  if (d.Cout_pad <= 128) rb = d.Cout_pad <= 16 ? 1 : d.Cout_pad <= 32 ? 2 : d.Cout_pad <= 64 ? 4 : 8;
  {
    // Wide layers over few pixels (the EfficientNet expansions of the distillation teacher / student, M <= 128 Ki
    // pixels: a 256-column tile gives each wave one or two 32-pixel blocks behind a 115-135 KiB weight staging, one
    // workgroup per CU) take 64-column tiles: four workgroups per CU, a quarter of the staging each, and less
    // padding in the last column tile (288 = 4.5 x 64, not 1.1 x 256).  Same accumulation order per output element,
    // so bit-identical (tools/pw_probe.py, profiles/r6_pw_rb_sweep.txt: 224 -> 1344 @ 4 x 40 x 40 25.1 -> 17.9 us,
    // 48 -> 288 @ 4 x 160 x 160 29.6 -> 24.6, 160 -> 960 @ 4 x 40 x 40 13.6 -> 12.1; the head's 786 Ki-pixel layers keep
    // 256 columns, 193 vs 318 us).  HISEG_PW_RB=1|2|4|8|16 (read once; A/B timing) forces the width.
    static const int force_rb = [] { const char* e = getenv("HISEG_PW_RB"); return e ? atoi(e) : 0; }();
    const bool narrow_ok = !d.convT && !d.mul && d.act != HISEG_ACT_SWISH && d.Cb == 0;
    if (rb == 16 && narrow_ok) {
      int want = force_rb ? force_rb : (a.M <= 131072 ? 4 : 16);
      if (want != 1 && want != 2 && want != 4 && want != 8) want = 16;
      if (!(want > 4 && nks > 8)) rb = want;
    }
  }
  const bool comb = rb == 16 && nks == 9;
  if ((rb == 16 && nks > 9) || (rb > 4 && nks > 8)) return false;   // (registers: 2 x 10 B fragment sets)
  if (comb ? (d.Ca != 256 || d.Cb > 32 || d.convT || d.residual || d.mul || d.in_scale ||
              (d.act != HISEG_ACT_NONE && d.act != HISEG_ACT_RELU))
           : d.Cb != 0)
    return false;
  if (rb == 16) {
    // the head's forms (ReLU / sigmoid / none; residual, mul, ConvTranspose) and the EfficientNet expansion
    // (SiLU); no SE gate at 256-column tiles
    if (d.in_scale) return false;
    if (d.act == HISEG_ACT_SIGMOID ? (d.convT || d.residual)
                                   : (d.act != HISEG_ACT_NONE && d.act != HISEG_ACT_RELU &&
                                      !(d.act == HISEG_ACT_SILU && !d.convT && !d.residual && !d.mul)))
      return false;
    if (d.mul && (d.act == HISEG_ACT_RELU || d.convT || ((d.m_cstride | d.m_coff) & 3))) return false;
  } else {
    // narrow tiles: plain or residual epilogue with any elementwise activation, optional SE gate
    if (d.convT || d.mul || d.act == HISEG_ACT_SWISH) return false;
    if (d.in_scale && (((uintptr_t)d.in_scale & 15) || (long long)d.N * d.Ca * 4 > kPwGateBytes)) return false;
  }
  const long long out_px = (long long)a.M * (d.convT ? 4 : 1);
  const long long lim = 0x7fffffffll;
  if ((long long)a.M * d.a_cstride * 2 >= lim || (d.Cb && (long long)a.M * d.b_cstride * 2 >= lim) ||
      out_px * d.o_cstride * 2 >= lim || (d.residual && out_px * d.r_cstride * 2 >= lim) ||
      (d.mul && out_px * d.m_cstride * 2 >= lim))
    return false;
  if ((d.a_cstride | d.a_coff) & 7) return false;
  if (d.Cb && ((d.b_cstride | d.b_coff) & 7)) return false;
  if (((d.o_cstride | d.o_coff) & 3) || (d.residual && ((d.r_cstride | d.r_coff) & 3))) return false;
  if (((uintptr_t)d.out | (uintptr_t)d.residual | (uintptr_t)d.mul) & 7) return false;
  nks_max = comb ? 9 : nks <= 2 ? 2 : nks <= 4 ? 4 : nks <= 8 ? 8 : 10;
  // 256-column tiles at a k-step count below the register tile exist for the plain epilogue only (launch_pw_k):
  // the residual / mul / ConvTranspose forms need exactly 2, 4 or 8 k-steps (ConvTranspose 144 -> 72 and 192 -> 96,
  // the B1 / B7 EnhancedUNet up-convolutions, have 5 / 6 and take the LDS-DMA ring kernel)
  if (rb == 16 && !comb && nks != nks_max && (d.convT || d.residual || d.mul)) return false;
  return true;
}

bool conv_pw_applies(const ConvArgs& a) {
  int rb, nks, nks_max;
  return pw_plan(a, rb, nks, nks_max);
}

// SE-gated layers stage the gate of every image of the launch in LDS ([N][Ca] f32, kPwGateBytes at most), so the
// plan depends on the batch.  The images a pointwise launch may take for this layer when the gate alone makes it
// decline (0: the layer does not qualify anyway or fits as it is): conv2d_impl then runs it in image ranges of that
// many, so a pixel's kernel -- and its accumulation order -- never depends on the batch it comes in.
int conv_pw_gate_images(const ConvArgs& a) {
  const hiseg_conv2d_desc& d = a.d;
  if (!d.in_scale || d.Ca <= 0 || (long long)d.N * d.Ca * 4 <= kPwGateBytes) return 0;
  const int per = (int)(kPwGateBytes / (4ll * d.Ca));
  if (per < 1) return 0;
  ConvArgs one = a;
  one.d.N = per;
  one.M = per * d.Ho * d.Wo;
  int rb, nks, nks_max;
  return pw_plan(one, rb, nks, nks_max) ? per : 0;
}

// Returns 1 if launched, 0 if the layer does not qualify (caller falls back), <0 on error.  variant 90.
int conv_pw_try(const ConvArgs& a0, hipStream_t s, int variant) {
#ifdef HISEG_DIAG
  const bool diag = variant >= 190 && variant < 222;   // variant 90 with ablation bits variant - 190
#else
  const bool diag = false;
#endif
  if (variant != 90 && !diag) return 0;
  ConvArgs a = a0;
  a.abl = diag ? variant - 190 : 0;
  int rb, nks, nks_max;
  if (!pw_plan(a, rb, nks, nks_max)) return 0;
  int r;
  if (rb < 16) {
    r = launch_pw_narrow(a, s, rb, nks_max, nks);
  } else {
    switch (nks_max) {
      case 2: r = launch_pw_k<2>(a, s, nks); break;
      case 4: r = launch_pw_k<4>(a, s, nks); break;
      case 8: r = launch_pw_k<8>(a, s, nks); break;
      default: r = launch_pw_k<9>(a, s, nks); break;
    }
  }
  return r < 0 ? r : 1;
}
#endif

}  // namespace hiseg
