// Pipelined implicit-GEMM convolution for "uniform" layers (bf16, gfx950).
//
// Applies when every 64-wide K block lies inside ONE filter tap and ONE loader source, i.e.
// both source channel counts are multiples of 64 and src A is not upsampled — all the 3x3 /
// 1x1 convs of the ROI head (256/128/64-channel layers).  The tap, channel
// offset and source of a K block are then wave-uniform scalars and the only per-lane work of
// the activation gather is one bounds test and one offset per 16-B chunk.
//
// Operands reach LDS by LDS-DMA (buffer_load_dwordx4 ... lds): one wave instruction fills 8
// tile rows x 128 B.  Zero padding of the 3x3 halo costs nothing: an out-of-image tap gets a
// voffset beyond the buffer descriptor's range and the DMA writes zeros.  The LDS image is
// lane-linear, so the XOR swizzle (chunk c of row r at slot c ^ ((r>>1)&7), conflict-free for
// the fragment reads) is applied on the SOURCE address (cdna_hip_programming.md §5.4 rule 21).
// STAGES-deep ring, loads for K block kb+STAGES-1 issued right after the barrier of block kb,
// counted `s_waitcnt vmcnt` + raw s_barrier (no vmcnt(0) in the loop).
// Workgroups are remapped XCD-major (bijective), Cout tiles fastest, so the Cout tiles and the
// neighbouring pixel tiles that share a 3x3 halo run on the same XCD's L2.
#include "conv_common.h"

namespace hiseg {

typedef __attribute__((address_space(3))) void lds_void;

// One 16-B-per-lane LDS-DMA (1 KiB per wave instruction) written as inline asm so that hipcc's
// waitcnt pass does not see it: the compiler would otherwise drain vmcnt(0) before the first
// ds_read after every issue (LDS-DMA writes alias the LDS the MFMAs read), which serialises the
// ring.  Completion is tracked by the explicit counted s_waitcnt vmcnt in the K loop
// (cdna_hip_programming.md §5.7 item 1).  M0 is written inside the same statement.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, unsigned voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(lds_addr), "v"(voff), "s"(rsrc) : "memory");
}

// STAMP (diagnostic builds only): wave 0 lane 0 writes s_memtime at kernel entry, loop entry,
// loop exit and kernel exit to the u64 buffer passed in desc.out2 (4 per workgroup) and skips
// the out2 store; outputs are otherwise unchanged.
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  return t;
}

// PRIO: s_setprio 1 around each MFMA cluster (cdna_hip_programming.md T2).  LATE: the next stage's DMA is
// issued after the first K-substep's fragment reads and MFMAs instead of right after the barrier, so the
// DMA issue of one wave overlaps the MFMAs of the other waves on its SIMD.  Same addresses either way.
// EPI: the epilogue goes through LDS -- each lane writes its scaled / shifted / residual-added / activated
// f32 fragments into a [BPX][BCO] tile (16-B chunks XOR-swizzled by row, conflict-free both ways), then the
// workgroup stores whole output rows: consecutive lanes write consecutive channels of one pixel (for a
// ConvTranspose tile: of one scattered output pixel), so every store instruction covers full lines instead
// of 16 pixels x 32 B.  Same arithmetic and rounding as TileEpi::store.
template <int BCO, int BPX, int WCO, int WPX, int STAGES, bool NOLOAD = false, bool STAMP = false, bool PRIO = false,
          bool LATE = false, bool EPI = false>
__global__ void __launch_bounds__(64 * WCO * WPX) conv_fast_kernel(ConvArgs a) {
  unsigned long long st0 = 0, st1 = 0, st2 = 0;
  if constexpr (STAMP) st0 = stamp_now();
  constexpr int NW = WCO * WPX;
  constexpr int TM = BCO / (WCO * 16);
  constexpr int TN = BPX / (WPX * 16);
  constexpr int NA = BPX / (8 * NW);   // act DMA instructions per wave per K block
  constexpr int NB = BCO / (8 * NW);   // weight DMA instructions per wave per K block
  constexpr int NL = NA + NB;
  constexpr int STAGE = (BCO + BPX) * 8;  // 16-B slots
  static_assert(NA >= 1 && NB >= 1 && TM >= 1 && TN >= 1, "tile");
  static_assert(BPX % (8 * NW) == 0 && BCO % (8 * NW) == 0, "rows per DMA instruction");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wco = w / WPX, wpx = w % WPX;

  // ---- XCD-major bijective remap, Cout tiles fastest
  const int nco = d.Cout_pad / BCO;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int q = nwg >> 3, r8 = nwg & 7, xcd = orig & 7, loc = orig >> 3;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + loc;
  const int co0 = (wg % nco) * BCO;
  const int px0 = (wg / nco) * BPX;

  // ---- per-lane gather state (act rows)
  const int lrow = lane >> 3;      // row within an 8-row DMA instruction
  const int slot = lane & 7;       // LDS slot this lane fills
  int pidx[NA], piy[NA], pix[NA], pch[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int r = 8 * (w + NW * i) + lrow;
    const int m = px0 + r;
    pch[i] = slot ^ ((r >> 1) & 7);
    if (m < a.M) {
      const int ox = m % d.Wo;
      const int tt = m / d.Wo;
      const int oy = tt % d.Ho;
      const int n = tt / d.Ho;
      piy[i] = oy * d.stride - d.pad;
      pix[i] = ox * d.stride - d.pad;
      pidx[i] = (n * d.H + piy[i]) * d.W + pix[i];
    } else {
      piy[i] = -(1 << 28); pix[i] = 0; pidx[i] = 0;  // never in bounds
    }
  }
  unsigned woff[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int r = 8 * (w + NW * i) + lrow;
    const int c = slot ^ ((r >> 1) & 7);
    woff[i] = ((unsigned)(co0 + r) * (unsigned)d.K_pad + (unsigned)c * 8u) * 2u;
  }

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.srcA), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.srcB ? d.srcB : d.srcA), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.weight), (short)0, 0x7fffffff, 0x00020000);
  const unsigned OOB = 0x80000000u;  // >= num_records: the DMA returns zeros

  const int Cin = a.Cin;
  const int bpt = (Cin + 63) >> 6;  // K blocks per tap (a 1x1 layer's src-B tail block is partial)
  const int nK = a.nK;
  const unsigned lds_base = (unsigned)(uintptr_t)(lds_void*)smem;

  auto issue = [&](int kb, int s) __attribute__((always_inline)) {
    const int tap = kb / bpt;
    const int ci0 = (kb - tap * bpt) << 6;
    const int ky = tap / d.KW, kx = tap - (tap / d.KW) * d.KW;
    const bool fromA = ci0 < d.Ca;
    const int cs = fromA ? d.a_cstride : d.b_cstride;
    const int cbase = fromA ? d.a_coff + ci0 : d.b_coff + ci0 - d.Ca;
    const int dpix = ky * d.W + kx;
    const unsigned sbase = lds_base + (unsigned)(s * STAGE) * 16u;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int iy = piy[i] + ky, ix = pix[i] + kx;
      const bool ok = (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W &&
                      (fromA || ci0 - d.Ca + pch[i] * 8 < d.Cb);
      const unsigned off = ok ? ((unsigned)((pidx[i] + dpix) * cs + cbase) + (unsigned)pch[i] * 8u) * 2u : OOB;
      const unsigned dst = sbase + (unsigned)(BCO * 8 + 8 * 8 * (w + NW * i)) * 16u;
      dma16(fromA ? rA : rB, dst, off);
    }
    const unsigned kofs = (unsigned)kb * 128u;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const unsigned dst = sbase + (unsigned)(8 * 8 * (w + NW * i)) * 16u;
      dma16(rW, dst, woff[i] + kofs);
    }
  };

  // ---- epilogue operands (scale/shift, residual) are fetched at kernel entry so their latency
  // hides under the K loop; issued as plain loads, they are older than every DMA of the ring,
  // and the loop's counted vmcnt waits stay exact (in-order return).
  int epx[TN], eco[TM];
#pragma unroll
  for (int j = 0; j < TN; ++j) epx[j] = px0 + wpx * TN * 16 + j * 16 + (lane & 15);
#pragma unroll
  for (int i = 0; i < TM; ++i) eco[i] = co0 + wco * TM * 16 + i * 16 + (lane >> 4) * 4;
  const bool fast_ep = TileEpi<bf16_t, bf16_t, TM, TN>::ok(d);
  TileEpi<bf16_t, bf16_t, TM, TN> ep;
  if (fast_ep) ep.prefetch(d, a.M, epx, eco);

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nK) issue(s, s);

  if constexpr (STAMP) st1 = stamp_now();
  for (int kb = 0; kb < nK; ++kb) {
    // loads of block kb are done once at most (STAGES-2) younger stages are outstanding
    if (kb + STAGES - 2 < nK) {
      if constexpr (STAGES == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if constexpr (STAGES == 3) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NL) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * NL) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (!LATE && !NOLOAD && kb + STAGES - 1 < nK) issue(kb + STAGES - 1, (kb + STAGES - 1) % STAGES);

    const uint4* sW = smem + (kb % STAGES) * STAGE;
    const uint4* sX = sW + BCO * 8;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s * 4 + (lane >> 4);
      uint4 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = sW[swz(wco * TM * 16 + i * 16 + (lane & 15), ch)];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = sX[swz(wpx * TN * 16 + j * 16 + (lane & 15), ch)];
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                              __builtin_bit_cast(bf16x8_t, bfr[j]), acc[i][j], 0, 0, 0);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      if constexpr (LATE) {
        if (s == 0 && !NOLOAD && kb + STAGES - 1 < nK) issue(kb + STAGES - 1, (kb + STAGES - 1) % STAGES);
      }
    }
  }

  if constexpr (STAMP) st2 = stamp_now();
  if constexpr (EPI && !STAMP) {
    static_assert(STAGES * (BCO + BPX) * 128 >= BCO * BPX * 4, "LDS epilogue tile exceeds the ring");
    constexpr int NCH = BCO / 4;                          // 16-B chunks per tile row
    if (fast_ep) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __syncthreads();                                      // every wave is done with the ring (no DMA in flight)
      float* st = reinterpret_cast<float*>(smem);
      with_act(d.act, [&](auto ac) __attribute__((always_inline)) {
        constexpr int A = decltype(ac)::value;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int rl = wpx * TN * 16 + j * 16 + (lane & 15);
            const int cl = wco * TM * 16 + i * 16 + (lane >> 4) * 4;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * ep.sc[i][e] + ep.sh[i][e];
            if (d.residual) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] += Quad<bf16_t>::get(ep.res[i][j], e);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = act_c<A>(v[e], d.act, d.act_beta);
            *reinterpret_cast<float4*>(st + rl * BCO + (((cl >> 2) ^ (rl & (NCH - 1))) << 2)) =
                make_float4(v[0], v[1], v[2], v[3]);
          }
      });
      __syncthreads();
      for (int idx = t; idx < BPX * NCH; idx += 64 * NW) {
        const int rl = idx / NCH, k = idx - (idx / NCH) * NCH;
        const int px = px0 + rl, co = co0 + 4 * k;
        if (px >= a.M || co >= d.Cout) continue;
        const float4 q = *reinterpret_cast<const float4*>(st + rl * BCO + ((k ^ (rl & (NCH - 1))) << 2));
        float v[4] = {q.x, q.y, q.z, q.w};
        long long op;
        int oc;
        out_site(d, px, co, op, oc);
        if (d.mul) {
          const typename Quad<bf16_t>::V m = Quad<bf16_t>::load(d.mul, op * d.m_cstride + d.m_coff + oc);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= Quad<bf16_t>::get(m, e);
        }
        Quad<bf16_t>::store(d.out, op * d.o_cstride + d.o_coff + oc, v);
        if (d.out2) Quad<bf16_t>::store(d.out2, op * d.o2_cstride + d.o2_coff + oc, v);
      }
      return;
    }
  }
  if (fast_ep) {
    ep.store(d, a.M, epx, eco, acc, !STAMP);
  } else {
    ConvArgs ae = a;
    if constexpr (STAMP) ae.d.out2 = nullptr;
#pragma clang loop unroll(full)
    for (int i = 0; i < TM; ++i)
#pragma clang loop unroll(full)
      for (int j = 0; j < TN; ++j)
        if (epx[j] < a.M) conv_epilogue<bf16_t, bf16_t>(ae, epx[j], eco[i], acc[i][j]);
  }
  if constexpr (STAMP) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long st3 = stamp_now();
    if (t == 0) {
      unsigned long long* sb = reinterpret_cast<unsigned long long*>(a.d.out2) + 4 * blockIdx.x;
      sb[0] = st0; sb[1] = st1; sb[2] = st2; sb[3] = st3;
    }
  }
}

template <int BCO, int BPX, int WCO, int WPX, int STAGES, bool NOLOAD = false, bool STAMP = false, bool PRIO = false,
          bool LATE = false, bool EPI = false>
static int launch_fast(const ConvArgs& a, hipStream_t s) {
  const int npx = (a.M + BPX - 1) / BPX;
  const int nco = a.d.Cout_pad / BCO;
  const size_t lds = (size_t)STAGES * (BCO + BPX) * 8 * 16;
  auto kern = conv_fast_kernel<BCO, BPX, WCO, WPX, STAGES, NOLOAD, STAMP, PRIO, LATE, EPI>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(npx * nco), dim3(64 * WCO * WPX), lds, s, a);
  return hiseg_check_launch("conv_fast");
}

// Returns 1 if launched, 0 if the layer is not "uniform" (caller falls back to the generic
// kernel), <0 on error.  variant: 0 = auto.
int conv_fast_try(const ConvArgs& a, hipStream_t s, int variant) {
  const hiseg_conv2d_desc& d = a.d;
  if (d.dtype != HISEG_BF16 || d.out_dtype != HISEG_BF16) return 0;
  if (d.a_up != 1 || d.in_scale != nullptr) return 0;
  // K blocks must not straddle a tap or a source: Ca, Cb multiples of 64, or (1x1 only) a src-B tail of
  // 8k channels in one last partial block whose missing chunks the DMA zero-fills (feature_combiner's
  // 256 RGB + 2 logit channels, rgb.py:695)
  const bool tail = d.KH == 1 && d.KW == 1 && d.Cb % 64 != 0 && d.Cb < 64 && d.Cb % 8 == 0;
  if (d.Ca % 64 != 0 || (d.Cb % 64 != 0 && !tail)) return 0;
  if (d.K_pad != d.KH * d.KW * ((a.Cin + 63) / 64) * 64) return 0;
  if (((d.a_cstride | d.a_coff) & 7) || (d.Cb && ((d.b_cstride | d.b_coff) & 7))) return 0;
  // 32-bit byte offsets
  const long long span_a = (long long)d.N * d.H * d.W * d.a_cstride * 2;
  const long long span_b = d.Cb ? (long long)d.N * d.H * d.W * d.b_cstride * 2 : 0;
  const long long span_w = (long long)d.Cout_pad * d.K_pad * 2;
  if (span_a >= 0x7fffffffll || span_b >= 0x7fffffffll || span_w >= 0x7fffffffll) return 0;
  // the STAMP diagnostic writes 4 u64 per workgroup through desc.out2: refuse it without that buffer
  HISEG_REQUIRE(variant != 18 || d.out2 != nullptr, HISEG_ERR_BAD_ARG, "conv_fast: stamp variant needs desc.out2");
  int r;
  if (variant == 0) variant = (d.Cout_pad % 128 == 0) ? 1 : (d.Cout_pad % 64 == 0 ? 3 : -1);
  switch (variant) {
    case 1: if (d.Cout_pad % 128) return 0; r = launch_fast<128, 256, 2, 4, 3>(a, s); break;
    case 2: if (d.Cout_pad % 128) return 0; r = launch_fast<128, 128, 2, 2, 4>(a, s); break;
    case 3: if (d.Cout_pad % 64) return 0; r = launch_fast<64, 256, 1, 4, 4>(a, s); break;
    case 4: if (d.Cout_pad % 128) return 0; r = launch_fast<128, 128, 2, 2, 2>(a, s); break;
    case 5: if (d.Cout_pad % 256) return 0; r = launch_fast<256, 256, 2, 4, 2>(a, s); break;
    case 6: if (d.Cout_pad % 128) return 0; r = launch_fast<128, 256, 2, 4, 2>(a, s); break;
    case 7: if (d.Cout_pad % 256) return 0; r = launch_fast<256, 128, 4, 2, 2>(a, s); break;
    case 8: if (d.Cout_pad % 64) return 0; r = launch_fast<64, 128, 1, 4, 2>(a, s); break;
#ifdef HISEG_DIAG
    // timing-only ceilings (K-loop without global loads: wrong outputs) and the s_memtime stamp variant
    case 9: if (d.Cout_pad % 128) return 0; r = launch_fast<128, 128, 2, 2, 2, true>(a, s); break;
    case 19: if (d.Cout_pad % 256) return 0; r = launch_fast<256, 256, 2, 4, 2, true>(a, s); break;
    case 18: if (d.Cout_pad % 128) return 0; r = launch_fast<128, 128, 2, 2, 2, false, true>(a, s); break;
#endif
    // schedule variants of the production 128x128 configuration (variant 4)
    case 60: if (d.Cout_pad % 128) return 0; r = launch_fast<128, 128, 2, 2, 2, false, false, true, false>(a, s); break;
    // 4 Cout x N pixel wave grids with 32x64 wave tiles: 128x128 (61, 8 waves), 128x64 (62), 128x256 (63, 16 waves),
    // 256x128 (64, 8x2), 64x64 (65), 64x128 (68), 128x128 with s_setprio (69)
    case 61: if (d.Cout_pad % 128) return 0; r = launch_fast<128, 128, 4, 2, 2, false, false, false, false, true>(a, s); break;
    case 62: if (d.Cout_pad % 128) return 0; r = launch_fast<128, 64, 4, 1, 2, false, false, false, false, true>(a, s); break;
    case 68: if (d.Cout_pad % 64) return 0; r = launch_fast<64, 128, 4, 2, 2, false, false, true, false, true>(a, s); break;
    case 69: if (d.Cout_pad % 128) return 0; r = launch_fast<128, 128, 4, 2, 2, false, false, true, false, true>(a, s); break;
    case 63: if (d.Cout_pad % 128) return 0; r = launch_fast<128, 256, 4, 4, 2, false, false, false, false, false>(a, s); break;
    case 64: if (d.Cout_pad % 256) return 0; r = launch_fast<256, 128, 8, 2, 2, false, false, false, false, false>(a, s); break;
    case 65: if (d.Cout_pad % 64) return 0; r = launch_fast<64, 64, 4, 1, 2, false, false, false, false, true>(a, s); break;
    case 66: if (d.Cout_pad % 128) return 0; r = launch_fast<128, 128, 2, 2, 2, false, false, true, false, true>(a, s); break;
    case 67: if (d.Cout_pad % 64) return 0; r = launch_fast<64, 128, 1, 4, 2, false, false, false, false, true>(a, s); break;
    default: return 0;
  }
  return r < 0 ? r : 1;
}

}  // namespace hiseg
