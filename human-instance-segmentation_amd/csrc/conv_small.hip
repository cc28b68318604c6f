// Halo-tiled direct convolution for narrow layers (bf16, gfx950): the full-resolution smp
// decoder / segmentation head and the EfficientNet 1x1 projections, where Cin and/or Cout are
// far below a 64-wide GEMM tile and the layer is bound by HBM, not by MFMA.
//
// One 256-thread workgroup owns TH output rows x 64 output columns of one image.  It stages
//   * the whole packed weight matrix [Cout_pad][K_pad] (rows padded to an odd number of 16-B
//     slots: conflict-free ds_read_b128 of 16 rows at one k offset), and
//   * the input halo (TH+KS-1) x (64+KS-1) pixels x (Ca+Cb) channels, zero outside the image,
//     src A nearest-upsampled on the fly (a_up = 2), the squeeze-excite gate (in_scale) applied
//     and rounded to bf16 exactly as the generic kernel does (pixel stride an odd number of
//     16-B slots),
// then runs v_mfma_f32_16x16x32_bf16 over K in the generic kernel's order (tap-major, 32-deep
// chunks: k = tap*(Ca+Cb) + ci), so results are bit-identical to conv_igemm_kernel.  Each wave
// takes whole 16-pixel groups; each B fragment (16 pixels x 32 k) is read once per group and
// reused for up to 4 Cout blocks per pass.  Every HBM byte is read once per workgroup: the
// 9 taps of a 3x3 reuse the halo in LDS instead of re-gathering from L2.
#include "conv_common.h"

namespace hiseg {

// i / d for 0 <= i < 2^32 / d by one multiply-high (m = ceil(2^32 / d)): the staging loops' run-time divisions by
// the chunk counts were ~40 VALU instructions each, twice per staged 16-B chunk
struct SmallDiv {
  unsigned m;
  int d;
  __device__ explicit SmallDiv(int d_) : m(d_ > 1 ? 0xffffffffu / (unsigned)d_ + 1u : 0u), d(d_) {}
  __device__ __forceinline__ int div(int i) const { return d > 1 ? (int)__umulhi((unsigned)i, m) : i; }
};

__device__ __forceinline__ unsigned long long stamp_small() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  return t;
}

// STAMP (diagnostic): s_memtime at entry, after staging, after compute, at exit -> u64 x 4 per
// workgroup in the buffer passed as desc.out2 (out2 itself is then not written).
// ST: stride (2: the EfficientNet stem, halo of (TH-1)*2+KS rows x 129 columns).  NW: waves per workgroup -- 8
// where the LDS footprint allows one workgroup per CU (wide-K two-source decoder convs: weights + halo > 80 KB),
// so that each SIMD still has two waves to hide the staging loads' and the fragment reads' latency.
template <int KS, int TH, typename TO, int NJ, bool STAMP = false, int ST = 1, int NW = 4>
__global__ void __launch_bounds__(NW * 64) conv_small_kernel(ConvArgs a, int WS, int PS) {
  constexpr int NT = NW * 64;
  unsigned long long st0 = 0, st1 = 0, st2 = 0;
  if constexpr (STAMP) st0 = stamp_small();
  unsigned long long* stamp_buf = STAMP ? reinterpret_cast<unsigned long long*>(a.d.out2) : nullptr;
  constexpr int TW = 64;
  constexpr int HR = (TH - 1) * ST + KS, HC = (TW - 1) * ST + KS;
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int ntx = (d.Wo + TW - 1) / TW;
  const int nty = (d.Ho + TH - 1) / TH;
  const int bx = blockIdx.x % ntx;
  const int by = (blockIdx.x / ntx) % nty;
  const int n = blockIdx.x / (ntx * nty);
  const int x0 = bx * TW, y0 = by * TH;
  const int Cin = a.Cin;
  const int cch = Cin >> 3;            // 16-B chunks per pixel
  const int kch = d.K_pad >> 3;        // 16-B chunks per weight row
  const int pad = KS / 2;
  uint4* sW = smem;
  uint4* sX = smem + d.Cout_pad * WS;

  // ---- stage weights and the halo (zero padding, upsampling, in_scale).  Loads are issued
  // unconditionally in batches of UB per thread (clamped addresses, zero-select after the
  // load) so that UB loads are in flight before the first LDS store.
  constexpr int UB = 16;   // 16 x 16 B per thread in flight: a workgroup stages up to 140 KB, at one CU per workgroup
  const int nw = d.Cout_pad * kch;
  const SmallDiv dkch(kch), dcch(cch);
  for (int i0 = t; i0 < nw; i0 += NT * UB) {
    uint4 v[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      int i = i0 + u * NT;
      i = i < nw ? i : nw - 1;
      const int r = dkch.div(i), c = i - r * kch;
      v[u] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(d.weight) + (long long)r * d.K_pad + c * 8);
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int i = i0 + u * NT;
      if (i < nw) {
        const int r = dkch.div(i), c = i - r * kch;
        sW[r * WS + c] = v[u];
      }
    }
  }
  const int nh = HR * HC * cch;
  const uint16_t* srcA = reinterpret_cast<const uint16_t*>(d.srcA);
  const uint16_t* srcB = reinterpret_cast<const uint16_t*>(d.Cb ? d.srcB : d.srcA);
  for (int i0 = t; i0 < nh; i0 += NT * UB) {
    uint4 v[UB];
    bool ok[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int i = i0 + u * NT;
      const int pix = dcch.div(i), c = i - pix * cch;
      const int prow = pix / HC, pcol = pix - prow * HC;
      const int iy = y0 * ST + prow - pad, ix = x0 * ST + pcol - pad;
      ok[u] = i < nh && iy >= 0 && iy < d.H && ix >= 0 && ix < d.W;
      const int ciy = ok[u] ? iy : 0, cix = ok[u] ? ix : 0;
      const int ci = c * 8;
      const bool fromA = ci < d.Ca;
      const int sy = d.a_up == 2 ? (ciy >> 1) : ciy;
      const int sx = d.a_up == 2 ? (cix >> 1) : cix;
      const long long offA = (((long long)n * a.Hs + sy) * a.Ws + sx) * d.a_cstride + d.a_coff + ci;
      const long long offB = (((long long)n * d.H + ciy) * d.W + cix) * d.b_cstride + d.b_coff + (ci - d.Ca);
      v[u] = *reinterpret_cast<const uint4*>(fromA ? srcA + offA : srcB + offB);
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int i = i0 + u * NT;
      if (i < nh) {
        const int pix = dcch.div(i), c = i - pix * cch;
        sX[pix * PS + c] = ok[u] ? v[u] : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  }
  __syncthreads();
  if (d.in_scale) {   // squeeze-excite gate on the src-A channels, rounded to bf16 in place
    const int cha = d.Ca >> 3;
    for (int i = t; i < HR * HC * cha; i += NT) {
      const int c = i % cha, pix = i / cha;
      uint4* q = &sX[pix * PS + c];
      const float4* sp = reinterpret_cast<const float4*>(d.in_scale + (long long)n * d.Ca + c * 8);
      const float4 s0 = sp[0], s1 = sp[1];
      float f[8];
      Chunk<bf16_t>::unpack(*q, f);
      f[0] *= s0.x; f[1] *= s0.y; f[2] *= s0.z; f[3] *= s0.w;
      f[4] *= s1.x; f[5] *= s1.y; f[6] *= s1.z; f[7] *= s1.w;
      *q = Chunk<bf16_t>::pack(f);
    }
    __syncthreads();
  }

  if constexpr (STAMP) st1 = stamp_small();
  // ---- compute.  Work item = G consecutive 16-pixel groups of one tile row (G = 4 when TH >= 4,
  // so every wave has work); wave w takes items w, w+4, ...  Cout is covered in passes of up to
  // 4 blocks of 16: per 32-deep k chunk a wave reads G B fragments and (<= 4) A fragments and
  // issues G x 4 independent MFMAs.  The (tap, channel) of a lane's 8 k values advances
  // incrementally from chunk to chunk (no division in the loop).
  constexpr int G0 = TH * 4 / NW;
  constexpr int G = G0 >= 4 ? 4 : (G0 >= 2 ? 2 : 1);
  constexpr int NI = TH * 4 / G;          // work items per tile
  const int K = KS * KS * Cin;
  const int nkc = (K + 31) >> 5;          // 32-deep chunks holding real k
  const int nco = d.Cout_pad >> 4;
  const int lg = lane >> 4, lr = lane & 15;
  const bool vec = (d.Cout & 3) == 0 && ((d.o_cstride | d.o_coff) & 3) == 0 &&
                   (!d.out2 || ((d.o2_cstride | d.o2_coff) & 3) == 0) &&
                   (!d.residual || ((d.r_cstride | d.r_coff) & 3) == 0) &&
                   (!d.mul || ((d.m_cstride | d.m_coff) & 3) == 0) &&
                   (((uintptr_t)d.scale | (uintptr_t)d.shift) & 15) == 0 &&
                   (((uintptr_t)d.out | (uintptr_t)d.out2 | (uintptr_t)d.residual | (uintptr_t)d.mul) & 7) == 0;
  const bool lite = vec || (!d.residual && !d.mul && !d.out2 && (((uintptr_t)d.scale | (uintptr_t)d.shift) & 15) == 0);
  // k position of this lane in chunk 0: k = 8*lg  ->  (tap, ci)
  int tap0 = (8 * lg) / Cin, ci0 = 8 * lg - tap0 * Cin;
  for (int p = 0; p < nco; p += NJ) {
    floatx4 sc[NJ], sh[NJ];
    if (lite) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        int co = (p + j) * 16 + lg * 4;
        co = co < d.Cout_pad ? co : 0;
        sc[j] = *reinterpret_cast<const floatx4*>(d.scale + co);
        sh[j] = *reinterpret_cast<const floatx4*>(d.shift + co);
      }
    }
    for (int it = w; it < NI; it += NW) {
      const int r = (it * G) >> 2;
      const int gx0 = ((it * G) & 3) * 16;
      const int oy = y0 + r;
      if (oy >= d.Ho || x0 + gx0 >= d.Wo) continue;
      // epilogue operands of this item, in flight during the MFMAs
      uint2 eres[G][NJ];
      int pxs[G];
#pragma unroll
      for (int q = 0; q < G; ++q) {
        const int ox = x0 + gx0 + q * 16 + lr;
        pxs[q] = (n * d.Ho + oy) * d.Wo + (ox < d.Wo ? ox : d.Wo - 1);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          int co = (p + j) * 16 + lg * 4;
          co = co < d.Cout ? co : 0;
          eres[q][j] = make_uint2(0u, 0u);
          if (vec && d.residual)
            eres[q][j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(d.residual) + (long long)pxs[q] * d.r_cstride + d.r_coff + co);
        }
      }
      floatx4 acc[G][NJ];
#pragma unroll
      for (int q = 0; q < G; ++q)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[q][j] = floatx4{0.f, 0.f, 0.f, 0.f};
      int tap = tap0, ci = ci0;
      const uint4* xrow = sX + (r * ST * HC + (gx0 + lr) * ST) * PS;
      for (int kc = 0; kc < nkc; ++kc) {
        const int dy = tap / KS, dx = tap - dy * KS;
        const bool kok = tap < KS * KS;
        const uint4* xb = xrow + (dy * HC + dx) * PS + (ci >> 3);
        uint4 b[G];
#pragma unroll
        for (int q = 0; q < G; ++q) b[q] = kok ? xb[q * 16 * ST * PS] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          if (p + j < nco) {
            const uint4 av = sW[((p + j) * 16 + lr) * WS + kc * 4 + lg];
#pragma unroll
            for (int q = 0; q < G; ++q)
              acc[q][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, av),
                                                                  __builtin_bit_cast(bf16x8_t, b[q]), acc[q][j], 0, 0, 0);
          }
        }
        ci += 32;
        while (ci >= Cin) { ci -= Cin; ++tap; }
      }
#pragma clang loop unroll(full)
      for (int q = 0; q < G; ++q) {
        const int ox = x0 + gx0 + q * 16 + lr;
        const bool live = ox < d.Wo;
        const int px = pxs[q];
        if (lite) {
#pragma clang loop unroll(full)
          for (int j = 0; j < NJ; ++j) {
            const int co = (p + j) * 16 + lg * 4;
            if (p + j >= nco || !live || co >= d.Cout) continue;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[q][j][e] * sc[j][e] + sh[j][e];
            if (d.residual) {
              v[0] += __uint_as_float(eres[q][j].x << 16); v[1] += __uint_as_float(eres[q][j].x & 0xffff0000u);
              v[2] += __uint_as_float(eres[q][j].y << 16); v[3] += __uint_as_float(eres[q][j].y & 0xffff0000u);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], d.act, d.act_beta);
            if (d.mul) {   // (vec only: lite without vec excludes mul)
              const uint2 m = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(d.mul) + (long long)px * d.m_cstride + d.m_coff + co);
              v[0] *= __uint_as_float(m.x << 16); v[1] *= __uint_as_float(m.x & 0xffff0000u);
              v[2] *= __uint_as_float(m.y << 16); v[3] *= __uint_as_float(m.y & 0xffff0000u);
            }
            const int nv = d.Cout - co < 4 ? d.Cout - co : 4;
            store4<TO>(d.out, (long long)px * d.o_cstride + d.o_coff + co, nv == 4 && vec, nv, v);
            if (!STAMP && d.out2) store4<bf16_t>(d.out2, (long long)px * d.o2_cstride + d.o2_coff + co, nv == 4 && vec, nv, v);
          }
        } else if (live) {
#pragma clang loop unroll(full)
          for (int j = 0; j < NJ; ++j)
            if (p + j < nco) conv_epilogue<bf16_t, TO>(a, px, (p + j) * 16 + lg * 4, acc[q][j]);
        }
      }
    }
  }
  if constexpr (STAMP) {
    st2 = stamp_small();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long st3 = stamp_small();
    if (threadIdx.x == 0) {
      unsigned long long* sb = stamp_buf + 4 * blockIdx.x;
      sb[0] = st0; sb[1] = st1; sb[2] = st2; sb[3] = st3;
    }
  }
}

static int odd_slots(int n) { return (n & 1) ? n : n + 1; }

template <int KS, int TH, typename TO, int NJ, bool STAMP, int ST = 1, int NW = 4>
static int launch_small_nj(const ConvArgs& a, hipStream_t s, int WS, int PS, size_t lds) {
  const hiseg_conv2d_desc& d = a.d;
  const int ntx = (d.Wo + 63) / 64, nty = (d.Ho + TH - 1) / TH;
  auto kern = conv_small_kernel<KS, TH, TO, NJ, STAMP, ST, NW>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(ntx * nty * d.N), dim3(NW * 64), lds, s, a, WS, PS);
  return hiseg_check_launch("conv_small");
}

template <int KS, int TH, typename TO, bool STAMP = false>
static int launch_small(const ConvArgs& a, hipStream_t s, int WS, int PS, size_t lds) {
  const int nco = a.d.Cout_pad / 16;
  if constexpr (!STAMP && KS == 3 && TH >= 2) {
    // HISEG_SMALL_NW8=0 keeps 4-wave workgroups (A/B timing only)
    static const bool nw8 = [] { const char* e = getenv("HISEG_SMALL_NW8"); return !(e && atoi(e) == 0); }();
    if (nw8 && lds > 80 * 1024) {   // one workgroup per CU: 8 waves
      if (nco == 1) return launch_small_nj<KS, TH, TO, 1, STAMP, 1, 8>(a, s, WS, PS, lds);
      if (nco == 2) return launch_small_nj<KS, TH, TO, 2, STAMP, 1, 8>(a, s, WS, PS, lds);
      return launch_small_nj<KS, TH, TO, 4, STAMP, 1, 8>(a, s, WS, PS, lds);
    }
  }
  if (nco == 1) return launch_small_nj<KS, TH, TO, 1, STAMP>(a, s, WS, PS, lds);
  if (nco == 2) return launch_small_nj<KS, TH, TO, 2, STAMP>(a, s, WS, PS, lds);
  return launch_small_nj<KS, TH, TO, 4, STAMP>(a, s, WS, PS, lds);
}

// stride 2 (3x3, bf16 out): 8 output rows when the halo fits two workgroups per CU, else 4.  Returns 1 if
// launched, 0 if the layer does not fit, <0 on error.
static int launch_small_s2(const ConvArgs& a, hipStream_t s, int WS, int PS) {
  const hiseg_conv2d_desc& d = a.d;
  const size_t wbytes = (size_t)d.Cout_pad * WS * 16;
  auto lds_for = [&](int th) { return wbytes + (size_t)((th - 1) * 2 + 3) * (63 * 2 + 3) * PS * 16; };
  const int nco = d.Cout_pad / 16;
  int r;
  if (lds_for(8) <= 80 * 1024) {
    const size_t l = lds_for(8);
    r = nco == 1 ? launch_small_nj<3, 8, bf16_t, 1, false, 2>(a, s, WS, PS, l)
      : nco == 2 ? launch_small_nj<3, 8, bf16_t, 2, false, 2>(a, s, WS, PS, l)
                 : launch_small_nj<3, 8, bf16_t, 4, false, 2>(a, s, WS, PS, l);
  } else if (lds_for(4) <= 160 * 1024) {
    const size_t l = lds_for(4);
    r = nco == 1 ? launch_small_nj<3, 4, bf16_t, 1, false, 2>(a, s, WS, PS, l)
      : nco == 2 ? launch_small_nj<3, 4, bf16_t, 2, false, 2>(a, s, WS, PS, l)
                 : launch_small_nj<3, 4, bf16_t, 4, false, 2>(a, s, WS, PS, l);
  } else {
    return 0;
  }
  return r < 0 ? r : 1;
}

template <int KS, typename TO>
static int pick_th(const ConvArgs& a, hipStream_t s, int WS, int PS, int force_th, bool stamp) {
  const hiseg_conv2d_desc& d = a.d;
  const size_t wbytes = (size_t)d.Cout_pad * WS * 16;
  auto lds_for = [&](int th) { return wbytes + (size_t)(th + KS - 1) * (64 + KS - 1) * PS * 16; };
  int th = force_th;
  if (th == 0) {   // 8 rows at >= 2 workgroups per CU, else the most rows that fit one CU
    if (lds_for(8) <= 80 * 1024 || (d.Ho >= 8 && lds_for(8) <= 160 * 1024)) th = 8;
    else if (lds_for(4) <= 160 * 1024) th = 4;
    else if (lds_for(2) <= 160 * 1024) th = 2;
    else th = 1;
  }
  if (lds_for(th) > 160 * 1024) return 0;
  int r;
#ifdef HISEG_DIAG
  if (stamp) {
    r = th == 8 ? launch_small<KS, 8, TO, true>(a, s, WS, PS, lds_for(8)) : HISEG_ERR_BAD_ARG;
    return r < 0 ? r : 1;
  }
#else
  if (stamp) return HISEG_ERR_BAD_ARG;   // the stamp variant exists only in a DIAG=1 build
#endif
  switch (th) {
    case 8: r = launch_small<KS, 8, TO>(a, s, WS, PS, lds_for(8)); break;
    case 4: r = launch_small<KS, 4, TO>(a, s, WS, PS, lds_for(4)); break;
    case 2: r = launch_small<KS, 2, TO>(a, s, WS, PS, lds_for(2)); break;
    default: r = launch_small<KS, 1, TO>(a, s, WS, PS, lds_for(1)); break;
  }
  return r < 0 ? r : 1;
}

// Returns 1 if launched, 0 if the layer does not qualify, <0 on error.
// variant: 0 auto, 50 auto TH, 51/52/54/58 force TH = 1/2/4/8.
int conv_small_try(const ConvArgs& a, hipStream_t s, int variant) {
  const hiseg_conv2d_desc& d = a.d;
  if (d.dtype != HISEG_BF16 || d.convT || (d.stride != 1 && d.stride != 2)) return 0;
  if (!(d.KH == d.KW && (d.KH == 1 || d.KH == 3) && d.pad == d.KH / 2)) return 0;
  const bool s2 = d.stride == 2;
  if (s2 ? (d.KH != 3 || d.a_up != 1 || d.out_dtype != HISEG_BF16 || d.Ho != (d.H - 1) / 2 + 1 ||
            d.Wo != (d.W - 1) / 2 + 1)
         : (d.Ho != d.H || d.Wo != d.W))
    return 0;
  const int KS = d.KH;
  const int K = KS * KS * a.Cin;
  if (d.K_pad < K || d.K_pad % 64 != 0) return 0;
  if (a.Cin > 256) return 0;
  if (reinterpret_cast<uintptr_t>(d.in_scale) & 15) return 0;
  const int WS = odd_slots(d.K_pad / 8);
  const int PS = odd_slots(a.Cin / 8);
  if ((size_t)d.Cout_pad * WS * 16 > 96 * 1024) return 0;
  int th = 0;
  const bool stamp = variant == 59;   // diagnostic: TH 8 with stamps (see conv_small_kernel)
  HISEG_REQUIRE(!stamp || a.d.out2 != nullptr, HISEG_ERR_BAD_ARG, "conv_small: stamp variant needs desc.out2");
  if (stamp) th = 8;
  if (s2) {
    if (stamp || variant != 0) return 0;
    return launch_small_s2(a, s, WS, PS);
  }
  if (variant >= 51 && variant <= 58) th = variant - 50;
  if (th != 0 && th != 1 && th != 2 && th != 4 && th != 8) return 0;
  int r;
  if (KS == 3) {
    r = d.out_dtype == HISEG_BF16 ? pick_th<3, bf16_t>(a, s, WS, PS, th, stamp) : pick_th<3, float>(a, s, WS, PS, th, stamp);
  } else {
    r = d.out_dtype == HISEG_BF16 ? pick_th<1, bf16_t>(a, s, WS, PS, th, stamp) : pick_th<1, float>(a, s, WS, PS, th, stamp);
  }
  return r;
}

}  // namespace hiseg
