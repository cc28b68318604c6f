// 256x256-tile phased implicit-GEMM convolution for wide uniform layers (bf16, gfx950).
//
// The dominant layers of the ROI head are 3x3 / 1x1 convs with 256 output channels over
// 64x48 ROI grids.  One 512-thread workgroup owns a 256(Cout) x 256(pixel)
// output tile; eight waves as 2(Cout) x 4(pixel), each wave a 128 x 64 sub-tile = 8 x 4 MFMA
// 16x16x32 accumulators.  K runs in 64-deep K tiles (one filter tap x 64 input channels; the
// same "uniform layer" conditions as conv_fast.hip).
//
// Schedule (cdna_hip_programming.md §5, the 256² phased template, restated for a conv): each
// K tile is 4 phases; phase q computes one quadrant of the wave's sub-tile (16 MFMAs):
//   q0: A-lo x B-lo   (reads A-lo 8 + B-lo 4 fragments)
//   q1: A-lo x B-hi   (reads B-hi 4)
//   q2: A-hi x B-hi   (reads A-hi 8)
//   q3: A-hi x B-lo   (no reads)
// A K tile's operands are four 16-KiB "half tiles" in LDS: AL/AH = the lo/hi 64 rows of both
// Cout halves, BL/BH = the lo/hi 32 pixels of each wave's 64-pixel column, so every half tile
// is last read early in its K tile and can be restaged two phases later.  One half tile is
// issued per phase by LDS-DMA (2 instructions per thread), K tile s+2 into the buffer of K tile
// s:  AL(s) at phase 4s-6, BL(s) 4s-5, BH(s) 4s-4, AH(s) 4s-3.  Before the first barrier of
// phase P every wave retires (counted vmcnt) what phase P+1 reads; waves 4-7 run one barrier
// behind waves 0-3, so one group's MFMAs overlap the other group's LDS reads and DMA issue.
// Per phase: reads, DMA issue, vmcnt, barrier, lgkmcnt(0), 16 MFMA (setprio 1), barrier.
#include <type_traits>

#include "conv_common.h"

namespace hiseg {

typedef __attribute__((address_space(3))) void lds8_void;

__device__ __forceinline__ void dma16_8ph(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, unsigned voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(lds_addr), "v"(voff), "s"(rsrc) : "memory");
}

__device__ __forceinline__ void bar8() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void vmwait8(int y) {  // y = half tiles allowed in flight (x2 DMAs)
  switch (y) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
  }
}

__device__ __forceinline__ unsigned long long stamp8() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  return t;
}

// STAGGER: waves 4-7 one barrier behind.  PRIO: s_setprio around the MFMA clusters.
// STAMP: diagnostic s_memtime (entry, loop start, loop end, exit) into desc.out2 (u64 x 4 / WG).
template <bool STAGGER, bool PRIO, bool STAMP, bool NOLOAD = false>
__global__ void __launch_bounds__(512) conv_8ph_kernel(ConvArgs a) {
  unsigned long long st0 = 0, st1 = 0, st2 = 0;
  if constexpr (STAMP) st0 = stamp8();
  constexpr int HT = 128 * 8;          // 16-B slots per half tile
  constexpr int RING = 8 * HT;         // 2 K-tile buffers x 4 half tiles = 128 KiB
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  float* s_scale = reinterpret_cast<float*>(smem + RING);   // [256] then shift [256]
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 2, wc = w & 3;

  // ---- XCD-major bijective remap, Cout tiles fastest
  const int nco = d.Cout_pad >> 8;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = orig & 7, loc = orig >> 3;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int co0 = (wg % nco) << 8;
  const int px0 = (wg / nco) << 8;

  // ---- epilogue scale/shift staged in LDS (plain loads, before any DMA is in flight)
  if (t < 128) {
    const int c = (t & 63) * 4;
    const float* src = (t < 64 ? d.scale : d.shift) + co0 + c;
    *reinterpret_cast<float4*>(s_scale + (t < 64 ? 0 : 256) + c) = *reinterpret_cast<const float4*>(src);
  }

  // ---- per-lane DMA state.  Instruction g of half tile k writes half-tile rows
  // hr = 8(w + 8g) + lane/8, 16-B slot lane%8, which holds source chunk lane%8 ^ ((hr>>1)&7).
  const int pch = (lane & 7) ^ ((4 * w + (lane >> 4)) & 7);
  unsigned woff[2][2];                         // [AL/AH][g]
  int piy[2][2], pix[2][2], pidx[2][2];        // [BL/BH][g]
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int hr = 8 * (w + 8 * g) + (lane >> 3);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int co = co0 + (hr >> 6) * 128 + h * 64 + (hr & 63);
      woff[h][g] = ((unsigned)co * (unsigned)d.K_pad + (unsigned)pch * 8u) * 2u;
      const int m = px0 + (hr >> 5) * 64 + h * 32 + (hr & 31);
      if (m < a.M) {
        const int ox = m % d.Wo;
        const int tt = m / d.Wo;
        const int oy = tt % d.Ho;
        const int n = tt / d.Ho;
        piy[h][g] = oy * d.stride - d.pad;
        pix[h][g] = ox * d.stride - d.pad;
        pidx[h][g] = (n * d.H + piy[h][g]) * d.W + pix[h][g];
      } else {
        piy[h][g] = -(1 << 28); pix[h][g] = 0; pidx[h][g] = 0;
      }
    }
  }
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.srcA), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.srcB ? d.srcB : d.srcA), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.weight), (short)0, 0x7fffffff, 0x00020000);
  const unsigned OOB = 0x80000000u;
  const int bpt = a.Cin >> 6;
  const int nK = a.nK;
  const unsigned lds_base = (unsigned)(uintptr_t)(lds8_void*)smem;

  // half tile kind k: 0 AL, 1 AH, 2 BL, 3 BH; K tile s -> buffer s&1
  auto issue = [&](auto kc, int s_) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    const int s = __builtin_amdgcn_readfirstlane(s_);
    const unsigned hbase = lds_base + (unsigned)((((s & 1) * 4 + k) * HT) * 16);
    if constexpr (k < 2) {
      const unsigned kofs = (unsigned)s * 128u;
#pragma unroll
      for (int g = 0; g < 2; ++g)
        dma16_8ph(rW, hbase + (unsigned)(8 * 8 * (w + 8 * g)) * 16u, woff[k][g] + kofs);
    } else {
      const int h = k - 2;
      const int tap = s / bpt;
      const int ci0 = (s - tap * bpt) << 6;
      const int ky = tap / d.KW, kx = tap - ky * d.KW;
      const bool fromA = __builtin_amdgcn_readfirstlane(ci0 < d.Ca ? 1 : 0) != 0;
      const int cs = fromA ? d.a_cstride : d.b_cstride;
      const int cbase = fromA ? d.a_coff + ci0 : d.b_coff + ci0 - d.Ca;
      const int dpix = ky * d.W + kx;
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int iy = piy[h][g] + ky, ix = pix[h][g] + kx;
        const bool ok = (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
        const unsigned off = ok ? ((unsigned)((pidx[h][g] + dpix) * cs + cbase) + (unsigned)pch * 8u) * 2u : OOB;
        if (fromA) dma16_8ph(rA, hbase + (unsigned)(8 * 8 * (w + 8 * g)) * 16u, off);
        else dma16_8ph(rB, hbase + (unsigned)(8 * 8 * (w + 8 * g)) * 16u, off);
      }
    }
  };

  floatx4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  uint4 ar[2][4], bl[2][2], bh[2][2];   // [k-half][fragment]

  // prologue = phases -6..-1 of the issue schedule
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  using K2 = std::integral_constant<int, 2>;
  using K3 = std::integral_constant<int, 3>;
  issue(K0{}, 0); issue(K2{}, 0); issue(K3{}, 0); issue(K1{}, 0);
  if (nK > 1) { issue(K0{}, 1); issue(K2{}, 1); }
  {
    int y = 4 * nK - 2;
    vmwait8(y < 0 ? 0 : (y > 4 ? 4 : y));
  }
  bar8();                              // every wave's share of K tile 0 has landed
  if constexpr (STAMP) st1 = stamp8();
  if (STAGGER && wr == 1) bar8();

  const int nP = 4 * nK;
  auto phase = [&](int kt, auto qc) __attribute__((always_inline)) {
    constexpr int q = decltype(qc)::value;
    const int P = 4 * kt + q;
    const uint4* buf = smem + (kt & 1) * 4 * HT;
    // ---- LDS fragment reads for this phase
    if constexpr (q == 0 || q == 2) {
      const uint4* sA = buf + (q >> 1) * HT;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int hr = wr * 64 + i * 16 + (lane & 15);
          ar[ks][i] = sA[swz(hr, ks * 4 + (lane >> 4))];
        }
    }
    if constexpr (q == 0 || q == 1) {
      const uint4* sB = buf + (2 + q) * HT;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int hr = wc * 32 + j * 16 + (lane & 15);
          if constexpr (q == 0) bl[ks][j] = sB[swz(hr, ks * 4 + (lane >> 4))];
          else bh[ks][j] = sB[swz(hr, ks * 4 + (lane >> 4))];
        }
    }
    // ---- one half tile of DMA: phase X targets K tile (X+6)/4 (kinds BH, AH, AL, BL for q 0..3)
    {
      const int tgt = (P + 6) >> 2;
      if (!NOLOAD && tgt < nK) issue(std::integral_constant<int, (q == 0 ? 3 : q == 1 ? 1 : q == 2 ? 0 : 2)>{}, tgt);
    }
    {
      const int y = nP - 3 - P;   // half tiles younger than the one phase P+1 reads
      if (!NOLOAD) vmwait8(y < 0 ? 0 : (y > 4 ? 4 : y));
    }
    bar8();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
    constexpr int ia0 = (q >= 2) ? 4 : 0;
    constexpr int jb0 = (q == 1 || q == 2) ? 2 : 0;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const uint4 bv = (jb0 == 2) ? bh[ks][j] : bl[ks][j];
          acc[ia0 + i][jb0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8_t, ar[ks][i]), __builtin_bit_cast(bf16x8_t, bv), acc[ia0 + i][jb0 + j], 0, 0, 0);
        }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    bar8();
  };
  for (int kt = 0; kt < nK; ++kt) {
    phase(kt, K0{});
    phase(kt, K1{});
    phase(kt, K2{});
    phase(kt, K3{});
  }
  if (STAGGER && wr == 0) bar8();   // equal barrier counts for both groups
  if constexpr (STAMP) st2 = stamp8();

  // ---- epilogue
  const bool fast_ep = (!d.convT || ((d.Cout >> 2) & 3) == 0) && (d.Cout & 3) == 0 &&
                       ((d.o_cstride | d.o_coff) & 3) == 0 && (!d.out2 || ((d.o2_cstride | d.o2_coff) & 3) == 0) &&
                       (!d.residual || ((d.r_cstride | d.r_coff) & 3) == 0) &&
                       (!d.mul || ((d.m_cstride | d.m_coff) & 3) == 0) &&
                       (((uintptr_t)d.out | (uintptr_t)d.out2 | (uintptr_t)d.residual | (uintptr_t)d.mul) & 7) == 0;
  if (fast_ep) {
    const bool has_res = d.residual != nullptr, has_mul = d.mul != nullptr;
    void* out2 = STAMP ? nullptr : d.out2;
#pragma clang loop unroll(full)
    for (int hh = 0; hh < 2; ++hh) {
      uint2 er[4][4], em[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = co0 + wr * 128 + (hh * 4 + i) * 16 + (lane >> 4) * 4;
          const int cc = co < d.Cout ? co : 0;
          int px = px0 + wc * 64 + j * 16 + (lane & 15);
          px = px < a.M ? px : a.M - 1;
          long long op;
          int oc;
          out_site(d, px, cc, op, oc);
          er[i][j] = make_uint2(0u, 0u);
          em[i][j] = make_uint2(0u, 0u);
          if (has_res)
            er[i][j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(d.residual) + op * d.r_cstride + d.r_coff + oc);
          if (has_mul)
            em[i][j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(d.mul) + op * d.m_cstride + d.m_coff + oc);
        }
#pragma clang loop unroll(full)
      for (int i = 0; i < 4; ++i) {
        const int cl = wr * 128 + (hh * 4 + i) * 16 + (lane >> 4) * 4;
        const int co = co0 + cl;
        const float4 sc = *reinterpret_cast<const float4*>(s_scale + cl);
        const float4 sh = *reinterpret_cast<const float4*>(s_scale + 256 + cl);
#pragma clang loop unroll(full)
        for (int j = 0; j < 4; ++j) {
          const int px = px0 + wc * 64 + j * 16 + (lane & 15);
          if (px >= a.M || co >= d.Cout) continue;
          long long op;
          int oc;
          out_site(d, px, co, op, oc);
          const floatx4 ac = acc[hh * 4 + i][j];
          float v[4] = {ac[0] * sc.x + sh.x, ac[1] * sc.y + sh.y, ac[2] * sc.z + sh.z, ac[3] * sc.w + sh.w};
          if (has_res) {
            const uint2 qv = er[i][j];
            v[0] += __uint_as_float(qv.x << 16); v[1] += __uint_as_float(qv.x & 0xffff0000u);
            v[2] += __uint_as_float(qv.y << 16); v[3] += __uint_as_float(qv.y & 0xffff0000u);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], d.act, d.act_beta);
          if (has_mul) {
            const uint2 qv = em[i][j];
            v[0] *= __uint_as_float(qv.x << 16); v[1] *= __uint_as_float(qv.x & 0xffff0000u);
            v[2] *= __uint_as_float(qv.y << 16); v[3] *= __uint_as_float(qv.y & 0xffff0000u);
          }
          uint2 o;
          o.x = f2bf2(v[0], v[1]);
          o.y = f2bf2(v[2], v[3]);
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(d.out) + op * d.o_cstride + d.o_coff + oc) = o;
          if (out2)
            *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out2) + op * d.o2_cstride + d.o2_coff + oc) = o;
        }
      }
    }
  } else {
    ConvArgs ae = a;
    if constexpr (STAMP) ae.d.out2 = nullptr;
#pragma clang loop unroll(full)
    for (int i = 0; i < 8; ++i)
#pragma clang loop unroll(full)
      for (int j = 0; j < 4; ++j) {
        const int px = px0 + wc * 64 + j * 16 + (lane & 15);
        const int co = co0 + wr * 128 + i * 16 + (lane >> 4) * 4;
        if (px < a.M) conv_epilogue<bf16_t, bf16_t>(ae, px, co, acc[i][j]);
      }
  }
  if constexpr (STAMP) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long st3 = stamp8();
    if (t == 0) {
      unsigned long long* sb = reinterpret_cast<unsigned long long*>(a.d.out2) + 4 * blockIdx.x;
      sb[0] = st0; sb[1] = st1; sb[2] = st2; sb[3] = st3;
    }
  }
}

template <bool STAGGER, bool PRIO, bool STAMP, bool NOLOAD = false>
static int launch_8ph(const ConvArgs& a, hipStream_t s) {
  const int npx = (a.M + 255) / 256;
  const int nco = a.d.Cout_pad / 256;
  const size_t lds = (size_t)8 * 128 * 8 * 16 + 512 * 4;
  auto kern = conv_8ph_kernel<STAGGER, PRIO, STAMP, NOLOAD>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(npx * nco), dim3(512), lds, s, a);
  return hiseg_check_launch("conv_8ph");
}

// Returns 1 if launched, 0 if the layer does not qualify, <0 on error.
// variants: 40 staggered + setprio, 41 = 40 with STAMP, 42 no stagger, 43 no setprio.
int conv_8ph_try(const ConvArgs& a, hipStream_t s, int variant) {
  const hiseg_conv2d_desc& d = a.d;
  if (d.dtype != HISEG_BF16 || d.out_dtype != HISEG_BF16) return 0;
  if (d.a_up != 1 || d.in_scale != nullptr) return 0;
  if (d.Ca % 64 != 0 || d.Cb % 64 != 0) return 0;
  if (d.Cout_pad % 256 != 0) return 0;
  if (d.K_pad != d.KH * d.KW * a.Cin) return 0;
  if (((d.a_cstride | d.a_coff) & 7) || (d.Cb && ((d.b_cstride | d.b_coff) & 7))) return 0;
  if ((((uintptr_t)d.scale | (uintptr_t)d.shift) & 15) != 0) return 0;
  const long long span_a = (long long)d.N * d.H * d.W * d.a_cstride * 2;
  const long long span_b = d.Cb ? (long long)d.N * d.H * d.W * d.b_cstride * 2 : 0;
  const long long span_w = (long long)d.Cout_pad * d.K_pad * 2;
  if (span_a >= 0x7fffffffll || span_b >= 0x7fffffffll || span_w >= 0x7fffffffll) return 0;
  // the STAMP diagnostic writes 4 u64 per workgroup through desc.out2: refuse it without that buffer
  HISEG_REQUIRE(variant != 41 || d.out2 != nullptr, HISEG_ERR_BAD_ARG, "conv_8ph: stamp variant needs desc.out2");
  int r;
  switch (variant) {
    case 0: case 40: r = launch_8ph<true, true, false>(a, s); break;
    case 41: r = launch_8ph<true, true, true>(a, s); break;
    case 42: r = launch_8ph<false, true, false>(a, s); break;
    case 43: r = launch_8ph<true, false, false>(a, s); break;
    // timing-only ceilings (no DMA in the K loop: wrong outputs)
    case 44: r = launch_8ph<true, true, false, true>(a, s); break;
    case 45: r = launch_8ph<false, true, false, true>(a, s); break;
    default: return 0;
  }
  return r < 0 ? r : 1;
}

}  // namespace hiseg
