// Implicit-GEMM convolution on CDNA4 MFMA (gfx950).
//
// GEMM view (see include/hiseg.h, hiseg_conv2d_fwd):   D[co][px] = sum_k W[co][k] * X[px][k]
//   rows of the MFMA "A" operand  = output channels (weights, K-contiguous, packed by the host)
//   cols of the MFMA "B" operand  = output pixels   (gathered on the fly from NHWC activations)
// With this orientation every lane ends up holding 4 consecutive output channels of one
// pixel (16x16 accumulator map: col = lane&15, row = 4*(lane>>4)+r), which is what the
// channel-contiguous NHWC epilogue stores.
//
// bf16: v_mfma_f32_16x16x32_bf16 (8 k-values per lane per fragment = one 16-B chunk).
// f32 : v_mfma_f32_16x16x4_f32 (exact f32, parity mode); a 16-B chunk holds 4 k-values and
//       is consumed by 4 MFMAs (the k order inside a chunk is permuted identically for both
//       operands, so the contraction is unchanged).
//
// Tiling: one workgroup = 256 threads = 4 waves, output tile BCO x BPX, K block = 8 chunks
// (64 bf16 / 32 f32).  Both operand tiles are staged through LDS as 128-B rows of 8 chunks,
// chunk c of row r stored at slot c ^ ((r>>1)&7): conflict-free for the ds_read_b128 lane
// groups of the fragment reads (MI355X_MICROARCH.md §LDS) and for the row-wise stores.
// Two LDS stages; the next K block is gathered into registers while the current one feeds
// the MFMAs (register-staged double buffering, one barrier per K block).
#include <cstdlib>
#include "conv_common.h"

namespace hiseg {

// SPLIT: split-K (grid.z = splits, a.kper K blocks each) for small grids with long K loops -- the SE-gated
// EfficientNet projections at the deep stages (B7: 2304 -> 384 over 4 x 20 x 20 pixels = 39 tiles of 128 x 128
// for 36 K blocks: one global round trip per K block on one workgroup per CU).  Each split stores its raw f32
// tile to the caller's workspace [split][M][Cout_pad]; conv_splitk_reduce_kernel sums the splits in order and
// applies the epilogue (deterministic; within f32 re-association of the unsplit kernel).
typedef unsigned ig_u4 __attribute__((ext_vector_type(4)));

// LIN (bf16; 1x1, pad 0, one source, no upsampling; the launcher checks every tensor fits one 2^31-byte buffer
// resource): a chunk's source pixel and channel never change along the K loop except by whole K blocks, so its
// activation, gate and weight byte offsets are computed once and each K block's loads are buffer loads at those
// offsets + a wave-uniform (SGPR) K-block offset -- the per-block 64-bit (n, y, x) -> address products and bounds
// checks were most of the gather's VALU work, the SE-gated layers' more.  Rows outside the GEMM and chunks past
// Cin load zeros through out-of-range offsets; the same values land in LDS as in the general gather.
// LIN 2 (bf16; any KH x KW <= 32 taps and stride, ungated, one un-upsampled source): each thread stages one chunk
// column, so its (tap, channel) is per thread -- per K block one byte delta ((ky Ws + kx) Cstride + ci) 2 is added
// to each row's tap-(0, 0) offset, and a per-row tap mask (bit ky KW + kx: the tap lies inside the image) replaces
// the bounds checks.
template <typename T, typename TO, int BCO, int BPX, int WCO, int WPX, bool SPLIT = false, int LIN = 0>
__global__ void __launch_bounds__(256) conv_igemm_kernel(ConvArgs a) {
  constexpr int KCH = Chunk<T>::N;
  constexpr int BK = 8 * KCH;
  constexpr int TM = BCO / (WCO * 16);
  constexpr int TN = BPX / (WPX * 16);
  constexpr int A_CH = (BPX * 8 + 255) / 256;
  constexpr int W_CH = (BCO * 8 + 255) / 256;
  constexpr int STAGE = (BCO + BPX) * 8;  // uint4 slots per stage
  constexpr bool A_FULL = (BPX * 8) % 256 == 0;  // every thread owns A_CH act chunks
  constexpr bool W_FULL = (BCO * 8) % 256 == 0;
  static_assert(WCO * WPX == 4, "4 waves");
  static_assert(TM >= 1 && TN >= 1, "tile");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];

  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int wco = wave / WPX;
  const int wpx = wave % WPX;
  const int px0 = blockIdx.x * BPX;
  const int co0 = blockIdx.y * BCO;
  const int c = t & 7;  // the chunk this thread stages, every row, every K block

  // ---- per-row pixel decode for the activation gather ----
  int rn[A_CH], riy[A_CH], rix[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int r = (t >> 3) + 32 * i;
    const int m = px0 + r;
    if ((A_FULL || r < BPX) && m < a.M) {
      const int ox = m % d.Wo;
      const int tt = m / d.Wo;
      const int oy = tt % d.Ho;
      rn[i] = tt / d.Ho;
      riy[i] = oy * d.stride - d.pad;
      rix[i] = ox * d.stride - d.pad;
    } else {
      rn[i] = -1; riy[i] = 0; rix[i] = 0;
    }
  }
  // K range of this workgroup (split-K: blocks [kb0, kb1))
  const int kb0 = SPLIT ? (int)blockIdx.z * a.kper : 0;
  const int kb1 = SPLIT ? (kb0 + a.kper < a.nK ? kb0 + a.kper : a.nK) : a.nK;
  // K state of this thread's chunk: k = kb*BK + c*KCH  ->  (ky, kx, ci)
  int ci, ky, kx;
  {
    const int k = kb0 * BK + c * KCH;
    const int tap = k / a.Cin;
    ci = k - tap * a.Cin;
    ky = tap / d.KW;
    kx = tap - ky * d.KW;
  }
  const int Cin = a.Cin;
  const int KW = d.KW;
  static_assert(!LIN || sizeof(T) == 2, "LIN: bf16");
  const unsigned OOB = 0x80000000u;
  unsigned voff_a[LIN ? A_CH : 1], voff_g[LIN ? A_CH : 1], voff_w[LIN ? W_CH : 1];
  __amdgpu_buffer_rsrc_t rsA, rsG, rsW;
  if constexpr (LIN == 2) {
    rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.srcA), (short)0, 0x7fffffff, 0x00020000);
    rsW = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.weight), (short)0, 0x7fffffff, 0x00020000);
    const int ci0 = kb0 * BK + c * KCH;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {   // voff_a: tap-(0, 0) byte offset (wrapping); voff_g: the row's tap mask
      unsigned msk = 0u;
      if (rn[i] >= 0) {
        for (int ky2 = 0; ky2 < d.KH; ++ky2)
          for (int kx2 = 0; kx2 < d.KW; ++kx2) {
            const int iy = riy[i] + ky2, ix = rix[i] + kx2;
            if (iy >= 0 && iy < d.H && ix >= 0 && ix < d.W) msk |= 1u << (ky2 * d.KW + kx2);
          }
      }
      voff_g[i] = msk;
      voff_a[i] = (unsigned)(((rn[i] * a.Hs + riy[i]) * a.Ws + rix[i]) * d.a_cstride + d.a_coff) * 2u;
    }
#pragma unroll
    for (int i = 0; i < W_CH; ++i) {
      const int r = (t >> 3) + 32 * i;
      voff_w[i] = co0 + r < d.Cout_pad ? (unsigned)(((co0 + r) * d.K_pad + ci0) * 2) : OOB;
    }
  }
  if constexpr (LIN == 1) {
    rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.srcA), (short)0, 0x7fffffff, 0x00020000);
    rsG = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(d.in_scale ? d.in_scale : reinterpret_cast<const float*>(d.srcA)),
                                            (short)0, 0x7fffffff, 0x00020000);
    rsW = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.weight), (short)0, 0x7fffffff, 0x00020000);
    const int ci0 = kb0 * BK + c * KCH;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const bool ok = rn[i] >= 0 && riy[i] >= 0 && riy[i] < d.H && rix[i] >= 0 && rix[i] < d.W;
      voff_a[i] = ok ? (unsigned)((((rn[i] * a.Hs + riy[i]) * a.Ws + rix[i]) * d.a_cstride + d.a_coff + ci0) * 2) : OOB;
      voff_g[i] = ok ? (unsigned)((rn[i] * d.Ca + ci0) * 4) : OOB;
    }
#pragma unroll
    for (int i = 0; i < W_CH; ++i) {
      const int r = (t >> 3) + 32 * i;
      voff_w[i] = co0 + r < d.Cout_pad ? (unsigned)(((co0 + r) * d.K_pad + ci0) * 2) : OOB;
    }
  }

  uint4 ra[A_CH], rw[W_CH];
#pragma unroll
  for (int i = 0; i < W_CH; ++i) rw[i] = make_uint4(0u, 0u, 0u, 0u);

  // SE gate (in_scale) of the gathered chunks: loaded beside the activations, applied when the chunk is stored to
  // LDS (after the current K block's MFMAs), so the loads' latency overlaps the MFMAs instead of stalling the
  // gather -- the gate multiply once made every K block of the deep EfficientNet projections wait for its loads
  // (1.5 us of 3.2 us per block, tools/splitk_bench.py with HISEG_SPLITK sweeps)
  constexpr int GREG = sizeof(T) == 2 ? 2 : 1;   // float4 gate vectors per chunk
  float4 rg[A_CH][GREG];
  bool rgs[A_CH];
  auto gather = [&](int kb) __attribute__((always_inline)) {
    if constexpr (LIN == 2) {
      const unsigned so = __builtin_amdgcn_readfirstlane((unsigned)((kb - kb0) * BK * 2));
      const bool kvalid = ky < d.KH;
      const int tap = ky * KW + kx;
      const unsigned delta = (unsigned)((ky * a.Ws + kx) * d.a_cstride + ci) * 2u;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const bool ok = kvalid && ((voff_g[i] >> tap) & 1u);
        ra[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsA, ok ? voff_a[i] + delta : OOB, 0u, 0));
        rgs[i] = false;
      }
#pragma unroll
      for (int i = 0; i < W_CH; ++i) {
        const int r = (t >> 3) + 32 * i;
        if (W_FULL || r < BCO) rw[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsW, voff_w[i], so, 0));
      }
      return;
    }
    if constexpr (LIN == 1) {
      const unsigned so = __builtin_amdgcn_readfirstlane((unsigned)((kb - kb0) * BK * 2));
      const bool kc = kb * BK + c * KCH < Cin;   // chunks past Cin (the last K block's padding) are zeros
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const unsigned va = kc ? voff_a[i] : OOB;
        ra[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsA, va, so, 0));
        rgs[i] = false;
        if (d.in_scale) {
          rgs[i] = kc && voff_a[i] != OOB;
          const unsigned vg = rgs[i] ? voff_g[i] : OOB;
#pragma unroll
          for (int e = 0; e < GREG; ++e)
            rg[i][e] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsG, vg + 16u * e, 2u * so, 0));
        }
      }
#pragma unroll
      for (int i = 0; i < W_CH; ++i) {
        const int r = (t >> 3) + 32 * i;
        if (W_FULL || r < BCO) rw[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsW, voff_w[i], so, 0));
      }
      return;
    }
    const bool kvalid = ky < d.KH;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      rgs[i] = false;
      if (rn[i] >= 0 && kvalid) {
        const int iy = riy[i] + ky, ix = rix[i] + kx;
        if (iy >= 0 && iy < d.H && ix >= 0 && ix < d.W) {
          if (ci < d.Ca) {
            const int sy = d.a_up == 2 ? (iy >> 1) : iy;
            const int sx = d.a_up == 2 ? (ix >> 1) : ix;
            const long long off = (((long long)rn[i] * a.Hs + sy) * a.Ws + sx) * d.a_cstride + d.a_coff + ci;
            v = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(d.srcA) + off);
            if (d.in_scale) {
              const float* s = d.in_scale + (long long)rn[i] * d.Ca + ci;
              rgs[i] = true;
              if (a.ins_vec) {   // 16-B aligned gate rows: vector loads
#pragma unroll
                for (int e = 0; e < GREG; ++e) rg[i][e] = *reinterpret_cast<const float4*>(s + 4 * e);
              } else {
#pragma unroll
                for (int e = 0; e < GREG; ++e) rg[i][e] = make_float4(s[4 * e], s[4 * e + 1], s[4 * e + 2], s[4 * e + 3]);
              }
            }
          } else {
            const long long off = (((long long)rn[i] * d.H + iy) * d.W + ix) * d.b_cstride + d.b_coff + (ci - d.Ca);
            v = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(d.srcB) + off);
          }
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < W_CH; ++i) {
      const int r = (t >> 3) + 32 * i;
      if (W_FULL || r < BCO) {
        // the last Cout tile may overhang Cout_pad: clamp the row, zero the value
        const int row = co0 + r < d.Cout_pad ? co0 + r : d.Cout_pad - 1;
        const long long off = (long long)row * d.K_pad + (long long)kb * BK + c * KCH;
        const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(d.weight) + off);
        rw[i] = co0 + r < d.Cout_pad ? v : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  };
  auto advance = [&]() __attribute__((always_inline)) {
    ci += BK;
    while (ci >= Cin) {
      ci -= Cin;
      if (++kx == KW) { kx = 0; ++ky; }
    }
  };
  auto stage_store = [&](int s) __attribute__((always_inline)) {
    uint4* sm = smem + s * STAGE;
#pragma unroll
    for (int i = 0; i < W_CH; ++i) {
      const int r = (t >> 3) + 32 * i;
      if (W_FULL || r < BCO) sm[swz(r, c)] = rw[i];
    }
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int r = (t >> 3) + 32 * i;
      uint4 v = ra[i];
      if (d.in_scale && rgs[i]) {   // the loader's rounding: bf16(x * gate) (f32: exact product)
        float f[KCH];
        Chunk<T>::unpack(v, f);
#pragma unroll
        for (int e = 0; e < GREG; ++e) {
          f[4 * e] *= rg[i][e].x; f[4 * e + 1] *= rg[i][e].y; f[4 * e + 2] *= rg[i][e].z; f[4 * e + 3] *= rg[i][e].w;
        }
        v = Chunk<T>::pack(f);
      }
      if (A_FULL || r < BPX) sm[BCO * 8 + swz(r, c)] = v;
    }
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  gather(kb0);
  stage_store(0);
  __syncthreads();

  for (int kb = kb0; kb < kb1; ++kb) {
    const int cur = (kb - kb0) & 1;
    if (kb + 1 < kb1) {
      advance();
      gather(kb + 1);
    }
    const uint4* sW = smem + cur * STAGE;
    const uint4* sX = sW + BCO * 8;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s * 4 + (lane >> 4);
      uint4 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = sW[swz(wco * TM * 16 + i * 16 + (lane & 15), ch)];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = sX[swz(wpx * TN * 16 + j * 16 + (lane & 15), ch)];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (sizeof(T) == 2) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8_t, af[i]), __builtin_bit_cast(bf16x8_t, bfr[j]),
                acc[i][j], 0, 0, 0);
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i].x), __uint_as_float(bfr[j].x), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i].y), __uint_as_float(bfr[j].y), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i].z), __uint_as_float(bfr[j].z), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i].w), __uint_as_float(bfr[j].w), acc[i][j], 0, 0, 0);
          }
        }
      }
    }
    if (kb + 1 < kb1) stage_store(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue ----
  int epx[TN], eco[TM];
#pragma unroll
  for (int j = 0; j < TN; ++j) epx[j] = px0 + wpx * TN * 16 + j * 16 + (lane & 15);
#pragma unroll
  for (int i = 0; i < TM; ++i) eco[i] = co0 + wco * TM * 16 + i * 16 + (lane >> 4) * 4;
  if constexpr (SPLIT) {
    float* ws = a.ws + (long long)blockIdx.z * a.M * d.Cout_pad;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        if (epx[j] < a.M && eco[i] < d.Cout_pad)
          *reinterpret_cast<floatx4*>(ws + (long long)epx[j] * d.Cout_pad + eco[i]) = acc[i][j];
    return;
  }
  if (TileEpi<T, TO, TM, TN>::ok(d)) {
    TileEpi<T, TO, TM, TN> ep;
    ep.prefetch(d, a.M, epx, eco);
    ep.store(d, a.M, epx, eco, acc);
  } else {
#pragma clang loop unroll(full)
    for (int i = 0; i < TM; ++i) {
#pragma clang loop unroll(full)
      for (int j = 0; j < TN; ++j) {
        if (epx[j] < a.M) conv_epilogue<T, TO>(a, epx[j], eco[i], acc[i][j]);
      }
    }
  }
}

// Split-K reduction: one thread per (pixel, 4-column quad); the splits are summed in order 0..S-1, then the
// conv epilogue (scale / shift, residual, activation, mul, dual store) of the unsplit kernel.
template <typename T, typename TO>
__global__ void __launch_bounds__(256) conv_splitk_reduce_kernel(ConvArgs a, int splits) {
  const hiseg_conv2d_desc& d = a.d;
  const int nq = d.Cout_pad >> 2;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)a.M * nq) return;
  const int px = (int)(i / nq), co = (int)(i - (long long)px * nq) * 4;
  const long long plane = (long long)a.M * d.Cout_pad;
  const float* p = a.ws + (long long)px * d.Cout_pad + co;
  floatx4 acc = *reinterpret_cast<const floatx4*>(p);
  for (int z = 1; z < splits; ++z) acc += *reinterpret_cast<const floatx4*>(p + z * plane);
  conv_epilogue<T, TO>(a, px, co, acc);
}

// The LIN gather applies (bf16 checked by the caller): 1x1, pad 0, one un-upsampled source, gate rows 16-B aligned,
// every tensor within one buffer resource.  HISEG_IGEMM_LIN=0 keeps the general gather (A/B timing and the
// equivalence test; read per call).
static int lin_ok(const ConvArgs& a) {
  const hiseg_conv2d_desc& d = a.d;
  const char* e = getenv("HISEG_IGEMM_LIN");
  const int mode = e ? atoi(e) : 2;   // 0: general gather, 1: 1x1 only, 2: 1x1 and the tap form
  if (mode == 0) return 0;
  if (d.Cb != 0 || d.a_up != 1 || d.convT) return 0;
  const long long lim = 0x7fff0000ll;
  if ((long long)d.N * a.Hs * a.Ws * d.a_cstride * 2 >= lim) return 0;
  if ((long long)d.Cout_pad * d.K_pad * 2 >= lim) return 0;
  if (d.KH == 1 && d.KW == 1 && d.pad == 0) {
    if (d.in_scale && !a.ins_vec) return 0;
    if (d.in_scale && (long long)d.N * d.Ca * 4 >= lim) return 0;
    return 1;
  }
  if (mode < 2 || d.in_scale || d.KH * d.KW > 32 || a.Cin % 8) return 0;
  return 2;
}

template <typename T, typename TO, int BCO, int BPX, int WCO, int WPX>
static int launch_cfg(const ConvArgs& a, hipStream_t s, int splits) {
  dim3 grid((a.M + BPX - 1) / BPX, (a.d.Cout_pad + BCO - 1) / BCO, splits > 1 ? splits : 1);
  const size_t lds = 2u * (BCO + BPX) * 8u * 16u;
  if constexpr (sizeof(T) == 2) {
    const int lin = lin_ok(a);
    if (lin) {
      if (splits > 1) {
        if (lin == 1) hipLaunchKernelGGL((conv_igemm_kernel<T, TO, BCO, BPX, WCO, WPX, true, 1>), grid, dim3(256), lds, s, a);
        else hipLaunchKernelGGL((conv_igemm_kernel<T, TO, BCO, BPX, WCO, WPX, true, 2>), grid, dim3(256), lds, s, a);
        const int r = hiseg_check_launch("conv_igemm_splitk");
        if (r) return r;
        const long long n = (long long)a.M * (a.d.Cout_pad >> 2);
        hipLaunchKernelGGL((conv_splitk_reduce_kernel<T, TO>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, splits);
        return hiseg_check_launch("conv_splitk_reduce");
      }
      if (lin == 1) hipLaunchKernelGGL((conv_igemm_kernel<T, TO, BCO, BPX, WCO, WPX, false, 1>), grid, dim3(256), lds, s, a);
      else hipLaunchKernelGGL((conv_igemm_kernel<T, TO, BCO, BPX, WCO, WPX, false, 2>), grid, dim3(256), lds, s, a);
      return hiseg_check_launch("conv_igemm");
    }
  }
  if (splits > 1) {
    hipLaunchKernelGGL((conv_igemm_kernel<T, TO, BCO, BPX, WCO, WPX, true>), grid, dim3(256), lds, s, a);
    const int r = hiseg_check_launch("conv_igemm_splitk");
    if (r) return r;
    const long long n = (long long)a.M * (a.d.Cout_pad >> 2);
    hipLaunchKernelGGL((conv_splitk_reduce_kernel<T, TO>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, splits);
    return hiseg_check_launch("conv_splitk_reduce");
  }
  hipLaunchKernelGGL((conv_igemm_kernel<T, TO, BCO, BPX, WCO, WPX>), grid, dim3(256), lds, s, a);
  return hiseg_check_launch("conv_igemm");
}

// Tile choice: the widest Cout tile whose overhang past Cout_pad adds <= 1/6 to the MFMA work.
static int igemm_bco(int cp) {
  auto fits = [&](int bco) { return ((cp + bco - 1) / bco) * bco * 6 <= cp * 7; };
  auto padded = [&](int bco) { return ((cp + bco - 1) / bco) * bco; };
  if (cp >= 96 && fits(128)) return 128;
  if (cp >= 48 && fits(64)) return 64;
  // >= 48 columns that fit neither: the 64 / 128 tile with the less overhang (tie: 128), not the narrow 32 / 16 x
  // 256 tiles -- one or four MFMAs per wave per k-step ran the B1 EnhancedUNet's 72- and 144-channel 3x3 layers
  // at 53-80 TFLOP/s (tools: bench.py call_profile top_layers, C3)
  if (cp >= 48) return padded(64) < padded(128) ? 64 : 128;
  if (fits(32)) return 32;
  return 16;
}

// split-K tiles: 128 x 128, or 64 x 128 -- never the narrow 32 / 16 x 256 tiles, whose eight gathered chunks per
// thread made a gated split workgroup several times slower (960 -> 160 over 4 x 40 x 40: 57 us)
static int splitk_bco(int cp) { return cp >= 96 && igemm_bco(cp) == 128 ? 128 : 64; }

template <typename T, typename TO>
static int launch_typed(const ConvArgs& a, hipStream_t s, int splits = 1) {
  // SE-gated layers as the split-K ones: the narrow 16 / 32 x 256 tiles gather their gated A chunks through
  // registers (the B7's 480 -> 80 projections over 4 x 80 x 80 at 16 x 256 tiles: 66 us per launch)
  static const bool gated_wide = [] { const char* e = getenv("HISEG_GATED_WIDE"); return !(e && atoi(e) == 0); }();
  if (splits > 1 || (gated_wide && a.d.in_scale != nullptr)) {
    if (splitk_bco(a.d.Cout_pad) == 128) return launch_cfg<T, TO, 128, 128, 2, 2>(a, s, splits);
    return launch_cfg<T, TO, 64, 128, 2, 2>(a, s, splits);
  }
  const char* eb = getenv("HISEG_IGEMM_BCO");   // A/B timing: force the Cout tile (read per call)
  switch (eb ? atoi(eb) : igemm_bco(a.d.Cout_pad)) {
    case 128: return launch_cfg<T, TO, 128, 128, 2, 2>(a, s, splits);
    case 64: return launch_cfg<T, TO, 64, 128, 2, 2>(a, s, splits);
    case 32: return launch_cfg<T, TO, 32, 256, 1, 4>(a, s, splits);
    default: return launch_cfg<T, TO, 16, 256, 1, 4>(a, s, splits);
  }
}

// Split-K plan of the generic kernel for a bf16 1x1 layer with a long K loop over a small image: splits (>= 2) or 1
// (no split).  The plan depends on the layer and the per-image grid only, never on the batch: an output element's
// f32 summation order (K blocks within a split, then the splits in order) is then the same whether its image is
// computed alone or in a batch, which keeps the exported masks batch-invariant bit for bit
// (test_c2_shape_bf16_properties_and_oracle).  Images of <= 1600 pixels (the EfficientNet's stride-16 / 32
// stages at 640 x 640 and 480 x 640), >= 6 K blocks: nK / 4 splits, 2..8.  The workspace it needs: splits x M x
// Cout_pad f32.
static int splitk_plan(const ConvArgs& a) {
  const hiseg_conv2d_desc& d = a.d;
  if (d.dtype != HISEG_BF16 || d.convT || a.nK < 6) return 1;
  // 3x3 layers over images of <= 256 pixels with long K (the B7 EnhancedUNet's 768-channel 3x3 pair over 8 x 16 x 12:
  // the halo kernel gets one 16 x 16 tile per image x 6 Cout tiles = 48 workgroups, 118 TFLOP/s): nK / 4 splits,
  // 2..8, on the generic kernel -- when the caller passes the workspace (the train engine does for <= 8192 pixels in
  // all; a large batch of such images fills the GPU on the halo kernel)
  if (d.KH == 3 && d.KW == 3 && d.stride == 1 && d.a_up == 1 && (long long)d.Ho * d.Wo <= 256 && a.nK >= 24 &&
      d.in_scale == nullptr) {
    int sp = a.nK / 4;
    return sp > 8 ? 8 : sp;
  }
  if (d.KH != 1 || d.KW != 1) return 1;
  // ungated layers take the LDS-DMA ring kernel (conv_fast.hip), which keeps more K blocks in flight: only long
  // K loops split there (the 384 -> 2304 expansion over 4 x 20 x 20 pixels: 17 us unsplit, 31 us split in two)
  if (d.in_scale == nullptr && a.nK < 24) return 1;
  // HISEG_SPLITK=S forces S splits on every layer the split applies to (A/B timing only)
  static const int forced = [] { const char* e = getenv("HISEG_SPLITK"); return e ? atoi(e) : 0; }();
  if (forced > 0) return forced < a.nK ? forced : a.nK;
  if ((long long)d.Ho * d.Wo > 1600) return 1;
  int sp = a.nK / 4;
  if (sp > 8) sp = 8;
  return sp >= 2 ? sp : 2;
}

static long long splitk_bytes(const ConvArgs& a, int splits) {
  return splits > 1 ? (long long)splits * a.M * a.d.Cout_pad * 4 : 0;
}

}  // namespace hiseg

namespace hiseg {
int conv_fast_try(const ConvArgs& a, hipStream_t s, int variant);
int conv_wide_try(const ConvArgs& a, hipStream_t s, int variant);
int conv_hw_try(const ConvArgs& a, hipStream_t s, int variant);
int conv_pw_try(const ConvArgs& a, hipStream_t s, int variant);
int conv_hwr_try(const ConvArgs& a, hipStream_t s, int variant);
int conv_hwt_try(const ConvArgs& a, hipStream_t s, int variant);
int conv_hwc_try(const ConvArgs& a, hipStream_t s, int variant);
int conv_hwc_stats_tiles(const ConvArgs& a);
int conv_small_try(const ConvArgs& a, hipStream_t s, int variant);
int conv_rows_try(const ConvArgs& a, hipStream_t s, int variant);
bool conv_pw_applies(const ConvArgs& a);
int conv_pw_gate_images(const ConvArgs& a);
bool conv_rows_form(const ConvArgs& a);
}

using namespace hiseg;


static int conv2d_impl(const hiseg_conv2d_desc* d, hiseg_stream_t stream, int variant);

extern "C" int hiseg_conv2d_fwd(const hiseg_conv2d_desc* d, hiseg_stream_t stream) {
  return conv2d_impl(d, stream, 0);
}

// The variants a release library accepts: the automatic choice, the generic kernel and every configuration
// tests/test_gpu_parity.py checks bit for bit.  Timing-only, stamp and experimental kernels exist only in a
// -DHISEG_DIAG build (Makefile DIAG=1).
// HISEG_CONV_HWC64=0 (read per call; A/B timing): the 64-Cout layers on conv_hwr (variant 100) instead of conv_hwc 107
static bool hwc64_mode() {
  const char* e = getenv("HISEG_CONV_HWC64");
  return !(e && atoi(e) == 0);
}

// HISEG_CONV_HWC_R3=0 (read per call; A/B timing): the 128-Cout layers on variant 104 (two halo buffers) instead of 108
static bool hwc_r3_mode() {
  const char* e = getenv("HISEG_CONV_HWC_R3");
  return !(e && atoi(e) == 0);
}

// HISEG_CONV_HWC_MTW=0|1 (read per call; A/B timing): the multi-tile conv_hwc forms (109 for 128-multiple Cout, 102 for
// the 64-Cout layers) instead of 108 / 107
#ifndef HISEG_CONV_HWC_MT_DEFAULT
#define HISEG_CONV_HWC_MT_DEFAULT(bco) false
#endif
static bool hwc_mt_mode(int bco) {
  const char* e = getenv("HISEG_CONV_HWC_MTW");
  if (e) return atoi(e) != 0;
  return HISEG_CONV_HWC_MT_DEFAULT(bco);
}

static bool release_variant(int v) {
  return v == -1 || v == 0 || (v >= 1 && v <= 8) || v == 50 || v == 51 || v == 52 || v == 54 || v == 58 ||
         (v >= 60 && v <= 69) || v == 70 || v == 71 || v == 72 || v == 74 || v == 80 || v == 82 || v == 84 || v == 86 ||
         v == 88 || v == 89 || v == 90 || (v >= 92 && v <= 101) || v == 103 || v == 102 || (v >= 104 && v <= 109);
}

// Workspace bytes the automatic choice uses for this layer (split-K generic kernel), 0 when it needs none.
extern "C" long long hiseg_conv2d_workspace_bytes(const hiseg_conv2d_desc* d) {
  if (d == nullptr || d->dtype != HISEG_BF16 || d->convT || d->N <= 0) return 0;
  const long long M = (long long)d->N * d->Ho * d->Wo;
  if (M >= (1ll << 31) || d->K_pad % 64) return 0;
  ConvArgs a;
  a.d = *d;
  a.M = (int)M;
  a.Cin = d->Ca + d->Cb;
  a.nK = d->K_pad / 64;
  a.Hs = d->H / (d->a_up > 0 ? d->a_up : 1);
  a.Ws = d->W / (d->a_up > 0 ? d->a_up : 1);
  if (conv_pw_applies(a)) return 0;
  // an SE-gated 1x1 layer whose gate table exceeds the pointwise kernel's LDS runs in image ranges on that kernel
  // (conv2d_impl), never on the split-K path
  if (d->in_scale && d->KH == 1 && d->KW == 1 && conv_pw_gate_images(a) > 0) return 0;
  return splitk_bytes(a, splitk_plan(a));
}

extern "C" int hiseg_conv2d_stats_tiles(const hiseg_conv2d_desc* d) {
  if (d == nullptr || d->dtype != HISEG_BF16 || d->convT || d->N <= 0) return 0;
  const long long M = (long long)d->N * d->Ho * d->Wo;
  if (M >= (1ll << 31)) return 0;
  ConvArgs a;
  a.d = *d;
  a.M = (int)M;
  a.Cin = d->Ca + d->Cb;
  a.nK = d->K_pad / 64;
  a.Hs = d->H / (d->a_up > 0 ? d->a_up : 1);
  a.Ws = d->W / (d->a_up > 0 ? d->a_up : 1);
  return conv_hwc_stats_tiles(a);
}

extern "C" int hiseg_conv2d_fwd_variant(const hiseg_conv2d_desc* d, int variant, hiseg_stream_t stream) {
#ifndef HISEG_DIAG
  HISEG_REQUIRE(release_variant(variant), HISEG_ERR_BAD_ARG,
                "conv2d: variant %d is not a release variant (diagnostic kernels need a DIAG=1 build)", variant);
#endif
  return conv2d_impl(d, stream, variant);
}

static int conv2d_impl(const hiseg_conv2d_desc* d, hiseg_stream_t stream, int variant) {
  HISEG_REQUIRE(d != nullptr, HISEG_ERR_BAD_ARG, "conv2d: null descriptor");
  HISEG_REQUIRE(d->dtype == HISEG_F32 || d->dtype == HISEG_BF16, HISEG_ERR_BAD_DTYPE, "conv2d: dtype %d", d->dtype);
  HISEG_REQUIRE(d->out_dtype == HISEG_F32 || d->out_dtype == HISEG_BF16, HISEG_ERR_BAD_DTYPE, "conv2d: out_dtype %d", d->out_dtype);
  HISEG_REQUIRE(d->srcA && d->weight && d->scale && d->shift && d->out, HISEG_ERR_BAD_ARG, "conv2d: null pointer");
  HISEG_REQUIRE(d->N > 0 && d->H > 0 && d->W > 0 && d->Ho > 0 && d->Wo > 0, HISEG_ERR_BAD_SHAPE, "conv2d: empty grid");
  HISEG_REQUIRE(d->KH > 0 && d->KW > 0 && d->stride > 0 && d->pad >= 0, HISEG_ERR_BAD_SHAPE, "conv2d: bad window");
  HISEG_REQUIRE(d->a_up == 1 || d->a_up == 2, HISEG_ERR_BAD_SHAPE, "conv2d: a_up must be 1 or 2");
  HISEG_REQUIRE(d->a_up == 1 || (d->H % 2 == 0 && d->W % 2 == 0), HISEG_ERR_BAD_SHAPE, "conv2d: upsampled grid must be even");
  HISEG_REQUIRE(d->Cb == 0 || d->srcB, HISEG_ERR_BAD_ARG, "conv2d: Cb > 0 needs srcB");
  HISEG_REQUIRE(d->Cout > 0 && d->Cout_pad >= d->Cout && d->Cout_pad % 16 == 0, HISEG_ERR_BAD_SHAPE,
                "conv2d: Cout %d Cout_pad %d (must be multiple of 16)", d->Cout, d->Cout_pad);
  const int kch = d->dtype == HISEG_BF16 ? 8 : 4;
  const int bk = 8 * kch;
  const int Cin = d->Ca + d->Cb;
  HISEG_REQUIRE(d->Ca > 0 && d->Ca % kch == 0 && d->Cb % kch == 0 && d->a_cstride % kch == 0 &&
                    d->a_coff % kch == 0 && (d->Cb == 0 || (d->b_cstride % kch == 0 && d->b_coff % kch == 0)),
                HISEG_ERR_BAD_SHAPE, "conv2d: input channels/strides must be multiples of %d", kch);
  HISEG_REQUIRE(d->K_pad % bk == 0 && d->K_pad >= d->KH * d->KW * Cin, HISEG_ERR_BAD_SHAPE,
                "conv2d: K_pad %d must be a multiple of %d and >= %d", d->K_pad, bk, d->KH * d->KW * Cin);
  HISEG_REQUIRE(al16(d->srcA) && al16(d->srcB) && al16(d->weight), HISEG_ERR_BAD_SHAPE, "conv2d: operands must be 16-B aligned");
  HISEG_REQUIRE(!d->convT || (d->KH == 1 && d->KW == 1 && d->stride == 1 && d->pad == 0 && d->Cout % 16 == 0 &&
                              d->Ho == d->H && d->Wo == d->W),
                HISEG_ERR_BAD_SHAPE, "conv2d: convT requires a 1x1 GEMM with Cout = 4*C, C %% 4 == 0");
  // BatchNorm statistics fused into the epilogue: only the halo kernel's fused-statistics form computes them, and no
  // fallback may silently skip them (the caller would finalize garbage)
  if (d->stats_partial || d->bnb_partial) {   // (also the fused BatchNorm-backward reduction of a data gradient)
    HISEG_REQUIRE(variant == 0 || variant == 104 || variant == 107, HISEG_ERR_BAD_ARG,
                  "conv2d: stats_partial / bnb_partial with variant %d", variant);
    HISEG_REQUIRE(al16(d->out) && al16(d->scale) && al16(d->shift), HISEG_ERR_BAD_SHAPE, "conv2d: alignment");
    ConvArgs a;
    a.d = *d;
    a.M = (int)((long long)d->N * d->Ho * d->Wo);
    a.Cin = Cin;
    a.nK = d->K_pad / bk;
    a.Hs = d->H / d->a_up;
    a.Ws = d->W / d->a_up;
    HISEG_REQUIRE(conv_hwc_stats_tiles(a) > 0, HISEG_ERR_BAD_ARG,
                  "conv2d: stats_partial / bnb_partial set but the layer has no fused kernel (hiseg_conv2d_stats_tiles)");
    const int r = conv_hwc_try(a, (hipStream_t)stream, d->Cout % 128 == 0 ? 104 : 107);
    HISEG_REQUIRE(r != 0, HISEG_ERR_BAD_ARG, "conv2d: the fused-statistics kernel declined the layer");
    return r < 0 ? r : HISEG_OK;
  }
  // Operands of >= 2 GiB: the LDS-DMA kernels address through 32-bit buffer offsets, so the launch is split
  // into image ranges whose every operand spans < 2 GiB (NHWC images are contiguous blocks; the conv never
  // mixes images), each range a launch of its own on the same stream.
  {
    const long long ea = d->dtype == HISEG_BF16 ? 2 : 4, eo = d->out_dtype == HISEG_BF16 ? 2 : 4;
    const long long in_px = (long long)(d->H / d->a_up) * (d->W / d->a_up);
    const long long out_px = (long long)d->Ho * d->Wo * (d->convT ? 4 : 1);
    long long per = in_px * d->a_cstride * ea;
    auto upd = [&](long long v) { if (v > per) per = v; };
    if (d->srcB) upd((long long)d->H * d->W * d->b_cstride * ea);
    if (d->residual) upd(out_px * d->r_cstride * ea);
    if (d->mul) upd(out_px * d->m_cstride * ea);
    upd(out_px * d->o_cstride * eo);
    if (d->out2) upd(out_px * d->o2_cstride * ea);
    const long long lim = (1ll << 31) - (1ll << 20);
    int step = 0;
    if (per * d->N > lim) {
      HISEG_REQUIRE(per <= lim, HISEG_ERR_BAD_SHAPE, "conv2d: one image's operand exceeds 2 GiB");
      step = (int)(lim / per);
    }
    if (variant == 0 && d->in_scale && d->dtype == HISEG_BF16 && d->KH == 1 && d->KW == 1) {
      // an SE-gated 1x1 layer the pointwise kernel takes at up to `g` images per launch (its LDS gate table):
      // image ranges of g, whatever the batch (batch-invariant numerics, conv_pw_gate_images)
      ConvArgs ga;
      ga.d = *d;
      ga.M = (int)((long long)d->N * d->Ho * d->Wo < (1ll << 31) ? (long long)d->N * d->Ho * d->Wo : 0);
      ga.Cin = d->Ca + d->Cb;
      ga.nK = d->K_pad / (8 * kch);
      ga.Hs = d->H / d->a_up;
      ga.Ws = d->W / d->a_up;
      const int g = conv_pw_gate_images(ga);
      if (g > 0 && (step == 0 || g < step)) step = g;
    }
    if (step > 0 && step < d->N) {
      for (int n0 = 0; n0 < d->N; n0 += step) {
        hiseg_conv2d_desc c = *d;
        c.N = d->N - n0 < step ? d->N - n0 : step;
        auto at = [&](const void* p, long long bytes_per_image) {
          return p ? (const void*)((const char*)p + bytes_per_image * n0) : p;
        };
        c.srcA = at(d->srcA, in_px * d->a_cstride * ea);
        c.srcB = at(d->srcB, (long long)d->H * d->W * d->b_cstride * ea);
        c.residual = at(d->residual, out_px * d->r_cstride * ea);
        c.mul = at(d->mul, out_px * d->m_cstride * ea);
        c.out = const_cast<void*>(at(d->out, out_px * d->o_cstride * eo));
        c.out2 = const_cast<void*>(at(d->out2, out_px * d->o2_cstride * ea));
        if (d->in_scale) c.in_scale = d->in_scale + (long long)n0 * d->Ca;   // per-image SE gate [N][Ca]
        const int r = conv2d_impl(&c, stream, variant);
        if (r) return r;
      }
      return HISEG_OK;
    }
  }
  const long long M = (long long)d->N * d->Ho * d->Wo;
  HISEG_REQUIRE(M < (1ll << 31), HISEG_ERR_BAD_SHAPE, "conv2d: too many pixels");
  ConvArgs a;
  a.d = *d;
  a.M = (int)M;
  a.Cin = Cin;
  a.nK = d->K_pad / bk;
  a.Hs = d->H / d->a_up;
  a.Ws = d->W / d->a_up;
  hipStream_t s = (hipStream_t)stream;
  // Automatic choice (variant 0) = the fastest measured configuration per layer class
  // (tools/conv_bench.py): LDS-DMA ring kernel, 128x128 tiles for Cout >= 128, 64x128 for 64.
  a.ins_vec = d->in_scale != nullptr && ((uintptr_t)d->in_scale & 15) == 0 && (d->Ca & 3) == 0;
  a.ws = static_cast<float*>(d->workspace);
  a.kper = a.nK;
  if (variant == 99 || variant == 0) {
    // split-K generic kernel for small-grid, long-K 1x1 layers (variant 99 forces it when the plan splits)
    const int sp = splitk_plan(a);
    if (sp > 1 && d->workspace != nullptr && d->workspace_bytes >= splitk_bytes(a, sp) &&
        !(variant == 0 && conv_pw_applies(a))) {
      a.kper = (a.nK + sp - 1) / sp;
      const int spl = (a.nK + a.kper - 1) / a.kper;
      return d->out_dtype == HISEG_BF16 ? launch_typed<bf16_t, bf16_t>(a, s, spl) : launch_typed<bf16_t, float>(a, s, spl);
    }
    HISEG_REQUIRE(variant == 0, HISEG_ERR_BAD_ARG, "conv2d: variant 99 (split-K) does not apply to this layer / workspace");
  }
  if (variant == 98) {
    const int r = conv_rows_try(a, s, variant);
    if (r != 0) return r < 0 ? r : HISEG_OK;
  } else if (variant == 90 || (variant >= 190 && variant < 222)) {
    const int r = conv_pw_try(a, s, variant);
    if (r != 0) return r < 0 ? r : HISEG_OK;
  } else if ((variant >= 92 && variant <= 97) || variant == 100 || variant == 101 || (variant >= 110 && variant < 142)) {
    const int r = conv_hwr_try(a, s, variant);
    if (r != 0) return r < 0 ? r : HISEG_OK;
  } else if (variant == 102 || (variant >= 104 && variant <= 109) || (variant >= 150 && variant < 4300)) {
    const int r = conv_hwc_try(a, s, variant);
    if (r != 0) return r < 0 ? r : HISEG_OK;
  } else if (variant == 103) {
    const int r = conv_hwt_try(a, s, variant);
    if (r != 0) return r < 0 ? r : HISEG_OK;
  } else if (variant >= 80 && variant < 90) {
    const int r = conv_hw_try(a, s, variant);
    if (r != 0) return r < 0 ? r : HISEG_OK;
  } else if (variant >= 70 && variant < 80) {
    const int r = conv_wide_try(a, s, variant);
    if (r != 0) return r < 0 ? r : HISEG_OK;
  } else if (variant >= 60 && variant < 70) {
    const int r = conv_fast_try(a, s, variant);
    if (r != 0) return r < 0 ? r : HISEG_OK;
  } else if (variant >= 50) {
    const int r = conv_small_try(a, s, variant);
    if (r != 0) return r < 0 ? r : HISEG_OK;
  } else if (variant >= 0) {
    int v = variant;
    // 61 = 128x128 ring, 8 waves as 4 (Cout) x 2 (pixel) with 32x64 wave tiles, LDS full-row epilogue;
    // 68 = the same wave grid on 64x128 tiles (tools/conv_bench.py: +1..4 % / +7..9 % over the 4-wave
    // 66 / 67, which had beaten the register epilogue by 4..17 %; all bit-identical)
    // HISEG_CONV_WAVES=4 restores the 4-wave tiles (A/B timing only)
    static const bool four_waves = [] { const char* e = getenv("HISEG_CONV_WAVES"); return e && atoi(e) == 4; }();
    // 256-output-channel 3x3 layers: the wide-tile kernel (conv_wide.hip: 256x256 workgroup tile, 128x128 wave
    // tiles, LDS epilogue; tools/conv_bench.py: 0.99 vs 1.23 ms on the 256->256 3x3 @64x48 x256 ROI class,
    // 0.58 vs 0.66 ms on 128->256, bit-identical).  It declines what it does not cover.
    // 3x3 single-source layers with 128-multiple Cout: the halo-tiled kernel, BCO 128 with B-fragment reuse
    // across ky (conv_hw.hip, variant 86: two workgroups per CU; tools/conv_bench.py: 0.85 vs 1.02 ms (wide
    // kernel) on the 256->256 @64x48 x256 ROI class, 1.01 vs 1.37 ms on 128->128 @128x96, 0.44 vs 0.54 ms on
    // 128->256; channel-major K order, within bf16 rounding); 64-multiple Cout: its BCO-64 configuration (variant
    // 89: 0.104 vs 0.140 ms on the 64->64 residual class, 0.26 vs 0.43 ms on 256->64)
    // HISEG_CONV_HALO=0 keeps the tap-major kernels (A/B timing only)
    static const bool halo = [] { const char* e = getenv("HISEG_CONV_HALO"); return !(e && atoi(e) == 0); }();
    // 1x1 layers and the ConvTranspose GEMM with 256-multiple GEMM columns: the persistent pointwise kernel
    // (conv_pw.hip, variant 90: weights resident in LDS, activations streamed into MFMA registers;
    // tools/conv_bench.py: 0.205 vs 0.308 ms on 256->256 @64x48 x256 ROIs, 0.21 vs 0.34 ms on the 256+8
    // combiner, 0.16 vs 0.24 ms on 128->256; bit-identical)
    if (v == 0 && d->KH == 1 && d->KW == 1) {
      const int r = conv_pw_try(a, s, 90);
      if (r != 0) return r < 0 ? r : HISEG_OK;
    }
    // narrow 3x3 layers (16 / 32 output channels: the full-image UNet's last decoder blocks and head): the
    // row-streaming kernel (conv_rows.hip, variant 98: weights in registers, input rows streamed through an LDS
    // ring; bit-identical to conv_small)
    if (v == 0 && d->KH == 3 && d->KW == 3 && d->Cout_pad <= 32) {
      const int r = conv_rows_try(a, s, 98);
      if (r != 0) return r < 0 ? r : HISEG_OK;
      // (sources far apart in memory: conv_rows takes them through one buffer resource each, VERDICT r3 weak #1.)
      // A layer of its form it still declines (an output alignment it does not store) takes conv_small, whose
      // accumulation order is conv_rows' (bit-identical)
      if (conv_rows_form(a)) {
        const int r2 = conv_small_try(a, s, 0);
        if (r2 != 0) return r2 < 0 ? r2 : HISEG_OK;
      }
    }
    // 3x3 layers with weights also packed in MFMA fragment order (hiseg.ops.frag_pack) and 128-multiple Cout: the
    // register-streamed-weight halo kernel (conv_hwr.hip: one barrier per 32-channel slice) in its B-reuse,
    // MFMA-priority configuration (variant 97; tools/conv_bench.py, profiles/r3_conv_bench_hwr*.json: 0.732 vs
    // 0.793 ms (variant 86) on 256->256 @64x48 x256 ROIs, 0.879 vs 0.930 ms on 128->128 @128x96, 0.364 vs 0.408 ms
    // on 128->256; bit-identical to variant 86)
    // Round 5: the Cout-split form of the same kernel (conv_hwc.hip, variant 104: each wave 32 Cout x all 256 pixels
    // of the tile -- half the weight-fragment loads, each halo row's B fragment reused across the 3 ky taps;
    // tools/conv_bench.py, profiles/r5_conv_hwc.txt: 256->256 @64x48 x256 ROIs 0.736 -> 0.678 ms, 128->128 @128x96
    // 0.875 -> 0.799, 128->256 0.369 -> 0.345; bit-identical to variant 97 / 86)
    // Round 6: variant 108, the same kernel with a ring of three halo buffers (slice sl + 2's halo in flight during
    // slice sl; 72 KiB of LDS, two workgroups per CU): bit-identical, 256->256 @64x48 x256 ROIs 0.709 -> 0.701 ms,
    // 128->128 @128x96 0.829 -> 0.814, 128->256 0.364 -> 0.351 (tools/conv_bench.py, profiles/r6_conv_hwc_r3.txt)
    // Round 6: variants 109 / 102, multi-tile workgroups (conv_hwc_mt_kernel: the next tile's first halo slice lands
    // during the last slice, two-half epilogue; bit-identical; HISEG_CONV_HWC_MTW=0|1 overrides the default)
    if (v == 0 && !four_waves && halo && d->weight_frag != nullptr && d->Cout % 128 == 0 && hwc_mt_mode(128)) {
      const int r = conv_hwc_try(a, s, 109);
      if (r != 0) return r < 0 ? r : HISEG_OK;
    }
    if (v == 0 && !four_waves && halo && d->weight_frag != nullptr && d->Cout % 128 == 0) {
      const int r = conv_hwc_try(a, s, hwc_r3_mode() ? 108 : 104);
      if (r != 0) return r < 0 ? r : HISEG_OK;
    }
    if (v == 0 && !four_waves && halo && d->weight_frag != nullptr && d->Cout % 128 == 0) {
      const int r = conv_hwr_try(a, s, 97);
      if (r != 0) return r < 0 ? r : HISEG_OK;
    }
    // 64-multiple Cout (the EnhancedUNet's 64-channel layers, the smp decoder's 64-channel block): conv_hwc on 64-Cout
    // x 16 x 32-pixel tiles (variant 107, round 5), else conv_hwr's (variant 100)
    if (v == 0 && !four_waves && halo && d->weight_frag != nullptr && d->Cout % 64 == 0 && hwc64_mode() &&
        hwc_mt_mode(64)) {
      const int r = conv_hwc_try(a, s, 102);
      if (r != 0) return r < 0 ? r : HISEG_OK;
    }
    if (v == 0 && !four_waves && halo && d->weight_frag != nullptr && d->Cout % 64 == 0 && hwc64_mode()) {
      const int r = conv_hwc_try(a, s, 107);
      if (r != 0) return r < 0 ? r : HISEG_OK;
    }
    if (v == 0 && !four_waves && halo && d->weight_frag != nullptr && d->Cout % 64 == 0) {
      const int r = conv_hwr_try(a, s, 100);
      if (r != 0) return r < 0 ? r : HISEG_OK;
    }
    if (v == 0 && !four_waves && halo) {
      // (BCO 64 for every Cout that is not a 128 multiple: full 64 tiles plus a partial last tile)
      const int r = conv_hw_try(a, s, d->Cout % 128 ? 89 : 86);
      if (r != 0) return r < 0 ? r : HISEG_OK;
    }
    if (v == 0 && d->Cout % 256 == 0 && d->KH * d->KW > 1 && !four_waves) {
      const int r = conv_wide_try(a, s, 70);
      if (r != 0) return r < 0 ? r : HISEG_OK;
    }
    if (v == 0) v = four_waves ? ((d->Cout_pad % 128 == 0) ? 66 : 67) : ((d->Cout_pad % 128 == 0) ? 61 : 68);
    const int r = conv_fast_try(a, s, v);
    if (r != 0) return r < 0 ? r : HISEG_OK;
    if (variant == 0) {   // narrow / ragged layers: halo-tiled direct kernel
      const int r2 = conv_small_try(a, s, 0);
      if (r2 != 0) return r2 < 0 ? r2 : HISEG_OK;
    }
  }
  if (d->dtype == HISEG_BF16) {
    return d->out_dtype == HISEG_BF16 ? launch_typed<bf16_t, bf16_t>(a, s) : launch_typed<bf16_t, float>(a, s);
  }
  return d->out_dtype == HISEG_BF16 ? launch_typed<float, bf16_t>(a, s) : launch_typed<float, float>(a, s);
}
