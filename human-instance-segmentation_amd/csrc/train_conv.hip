// Convolution backward on CDNA4 MFMA (gfx950): weight gradient, split reduction into the
// reference parameter layouts, and the per-step weight packing of every layer in one launch.
// (The data gradient reuses the forward implicit-GEMM kernels with packed dgrad weights.)
//
// Weight gradient GEMM (include/hiseg_train.h, hiseg_conv2d_wgrad):
//   D[k][j] = sum_p X[p][k] * dY[p][j]        k: im2col column (tap, ci), j: GEMM output column
// Both operands are pixel-major in HBM (NHWC), but MFMA wants each lane's 8 (bf16) / 4 (f32)
// contraction elements -- here consecutive PIXELS -- in one register chunk.  Each staging task
// therefore loads KCH pixels x one 16-B channel chunk (KCH coalesced 16-B loads, neighbouring
// threads on neighbouring chunks of the same pixel rows), transposes the KCH x KCH block in
// registers and writes KCH 16-B rows ("channel row, pixel chunk") into the same XOR-swizzled
// 128-B-row LDS image the forward kernel uses, so the fragment reads and the MFMA loop are the
// forward kernel's.  Register-staged double buffering, one barrier per pixel block.
// The pixel dimension is split across workgroups (split-K); every split writes its own f32
// partial tile (deterministic, no atomics) and hiseg_conv2d_wgrad_reduce sums them.
// That register-transpose kernel serves f32 (parity) and bf16 two-source layers whose sources are not
// 128-channel multiples; every other bf16 layer (GEMM-bias columns and ConvTranspose included) takes
// conv_wgrad_tr_kernel below (LDS-DMA + ds_read_b64_tr_b16, 4.5x faster on the ROI head's 256-channel 3x3
// layers).
#include <atomic>
#include <cstdlib>

#include "conv_common.h"
#include "hiseg_train.h"
#include "wgrad_common.h"

namespace hiseg {
int wgrad_wide_try(const WgradArgs& a, hipStream_t s);
int wgrad_hwc_try(const WgradArgs& a, hipStream_t s);
bool wgrad_hwc_shape_ok(const hiseg_conv2d_desc* d);
int wgrad_hwc_splits(const hiseg_conv2d_desc* d);
}

namespace hiseg {

// KCH x KCH transpose of 16-B chunks: in[i] = chunk of pixel i (KCH channels), out[e] = chunk of
// channel e (KCH pixels).
template <typename T> struct Tr;
template <> struct Tr<bf16_t> {
  __device__ static __forceinline__ void run(const uint4 (&in)[8], uint4 (&out)[8]) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 a = in[2 * q], b = in[2 * q + 1];
        const uint32_t wa = (e >> 1) == 0 ? a.x : (e >> 1) == 1 ? a.y : (e >> 1) == 2 ? a.z : a.w;
        const uint32_t wb = (e >> 1) == 0 ? b.x : (e >> 1) == 1 ? b.y : (e >> 1) == 2 ? b.z : b.w;
        w[q] = (e & 1) ? ((wa >> 16) | (wb & 0xffff0000u)) : ((wa & 0xffffu) | (wb << 16));
      }
      out[e] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
};
template <> struct Tr<float> {
  __device__ static __forceinline__ void run(const uint4 (&in)[4], uint4 (&out)[4]) {
    out[0] = make_uint4(in[0].x, in[1].x, in[2].x, in[3].x);
    out[1] = make_uint4(in[0].y, in[1].y, in[2].y, in[3].y);
    out[2] = make_uint4(in[0].z, in[1].z, in[2].z, in[3].z);
    out[3] = make_uint4(in[0].w, in[1].w, in[2].w, in[3].w);
  }
};

template <typename T, int BK, int BC, int WK, int WC>
__global__ void __launch_bounds__(256) conv_wgrad_kernel(WgradArgs a) {
  constexpr int KCH = Chunk<T>::N;
  constexpr int PB = 8 * KCH;             // pixels per block (one LDS stage row = 8 chunks)
  constexpr int TM = BK / (WK * 16);
  constexpr int TN = BC / (WC * 16);
  constexpr int NXT = (BK / KCH) * 8;     // X staging tasks (row group x pixel group)
  constexpr int NYT = (BC / KCH) * 8;
  constexpr int NT = NXT + NYT;
  constexpr int TPT = (NT + 255) / 256;   // tasks per thread
  constexpr int STAGE = (BK + BC) * 8;
  static_assert(WK * WC == 4 && TM >= 1 && TN >= 1, "tile");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int wk = wave / WC;
  const int wc = wave % WC;
  const int k0 = blockIdx.x * BK;
  const int j0 = blockIdx.y * BC;
  const int split = blockIdx.z;
  const int pb_begin = split * a.blocks_per_split;
  int pb_end = pb_begin + a.blocks_per_split;
  const int nblocks = (a.M + PB - 1) / PB;
  if (pb_end > nblocks) pb_end = nblocks;

  // static per-task decode (row group, pixel group, operand)
  int tk_row[TPT], tk_pg[TPT], tk_kind[TPT];  // kind: 0 = X, 1 = dY, -1 = none
  int tk_tap_y[TPT], tk_tap_x[TPT], tk_ci[TPT];
#pragma unroll
  for (int i = 0; i < TPT; ++i) {
    const int task = t + 256 * i;
    tk_kind[i] = -1; tk_row[i] = 0; tk_pg[i] = 0; tk_tap_y[i] = 0; tk_tap_x[i] = 0; tk_ci[i] = 0;
    if (task < NXT) {
      tk_kind[i] = 0;
      tk_row[i] = (task >> 3) * KCH;  // local k row
      tk_pg[i] = task & 7;
      const int k = k0 + tk_row[i];
      const int tap = k / a.Cin;
      tk_ci[i] = k - tap * a.Cin;
      tk_tap_y[i] = tap / d.KW;
      tk_tap_x[i] = tap - tk_tap_y[i] * d.KW;
    } else if (task < NT) {
      tk_kind[i] = 1;
      const int tt = task - NXT;
      tk_row[i] = (tt >> 3) * KCH;
      tk_pg[i] = tt & 7;
    }
  }

  uint4 reg[TPT][KCH];
  auto gather = [&](int pb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      if (tk_kind[i] < 0) continue;
      const int p0 = pb * PB + tk_pg[i] * KCH;
      if (tk_kind[i] == 0) {
        const int k = k0 + tk_row[i];
        const bool is_bias = a.want_bias && k == a.Ktot;
        const bool kvalid = k < a.Ktot;
        int ox = p0 % d.Wo, tt = p0 / d.Wo;
        int oy = tt % d.Ho, n = tt / d.Ho;
#pragma unroll
        for (int e = 0; e < KCH; ++e) {
          uint4 v = make_uint4(0u, 0u, 0u, 0u);
          const int p = p0 + e;
          if (p < a.M) {
            if (kvalid) {
              const int iy = oy * d.stride - d.pad + tk_tap_y[i];
              const int ix = ox * d.stride - d.pad + tk_tap_x[i];
              if (iy >= 0 && iy < d.H && ix >= 0 && ix < d.W) {
                const int ci = tk_ci[i];
                if (ci < d.Ca) {
                  const int Hs = d.H / d.a_up, Ws = d.W / d.a_up;
                  const int sy = d.a_up == 2 ? (iy >> 1) : iy, sx = d.a_up == 2 ? (ix >> 1) : ix;
                  const long long off = (((long long)n * Hs + sy) * Ws + sx) * d.a_cstride + d.a_coff + ci;
                  v = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(d.srcA) + off);
                } else {
                  const long long off = (((long long)n * d.H + iy) * d.W + ix) * d.b_cstride + d.b_coff + (ci - d.Ca);
                  v = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(d.srcB) + off);
                }
              }
            } else if (is_bias) {
              v = sizeof(T) == 2 ? make_uint4(0x3f80u, 0u, 0u, 0u) : make_uint4(0x3f800000u, 0u, 0u, 0u);
            }
          }
          reg[i][e] = v;
          if (++ox == d.Wo) { ox = 0; if (++oy == d.Ho) { oy = 0; ++n; } }
        }
      } else {
        const int j = j0 + tk_row[i];
        const bool jvalid = j < d.Cout;
        int q = 0, co = j;
        if (d.convT) { const int Cq = d.Cout >> 2; q = j / Cq; co = j - q * Cq; }
        int ox = p0 % d.Wo, tt = p0 / d.Wo;
        int oy = tt % d.Ho, n = tt / d.Ho;
#pragma unroll
        for (int e = 0; e < KCH; ++e) {
          uint4 v = make_uint4(0u, 0u, 0u, 0u);
          const int p = p0 + e;
          if (p < a.M && jvalid) {
            long long op = p;
            if (d.convT) op = ((long long)n * (2 * d.Ho) + 2 * oy + (q >> 1)) * (2 * d.Wo) + 2 * ox + (q & 1);
            v = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.dy) + op * a.dy_cs + a.dy_coff + co);
          }
          reg[i][e] = v;
          if (++ox == d.Wo) { ox = 0; if (++oy == d.Ho) { oy = 0; ++n; } }
        }
      }
    }
  };
  auto stage_store = [&](int s) __attribute__((always_inline)) {
    uint4* sm = smem + s * STAGE;
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      if (tk_kind[i] < 0) continue;
      uint4 o[KCH];
      Tr<T>::run(reg[i], o);
      uint4* base = tk_kind[i] == 0 ? sm : sm + BK * 8;
#pragma unroll
      for (int e = 0; e < KCH; ++e) base[swz(tk_row[i] + e, tk_pg[i])] = o[e];
    }
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  if (pb_begin < pb_end) {
    gather(pb_begin);
    stage_store(0);
  }
  __syncthreads();
  for (int pb = pb_begin; pb < pb_end; ++pb) {
    const int cur = (pb - pb_begin) & 1;
    if (pb + 1 < pb_end) gather(pb + 1);
    const uint4* sX = smem + cur * STAGE;
    const uint4* sY = sX + BK * 8;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s * 4 + (lane >> 4);
      uint4 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = sX[swz(wk * TM * 16 + i * 16 + (lane & 15), ch)];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = sY[swz(wc * TN * 16 + j * 16 + (lane & 15), ch)];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (sizeof(T) == 2) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8_t, af[i]), __builtin_bit_cast(bf16x8_t, bfr[j]), acc[i][j], 0, 0, 0);
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i].x), __uint_as_float(bfr[j].x), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i].y), __uint_as_float(bfr[j].y), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i].z), __uint_as_float(bfr[j].z), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i].w), __uint_as_float(bfr[j].w), acc[i][j], 0, 0, 0);
          }
        }
      }
    }
    if (pb + 1 < pb_end) stage_store(cur ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds rows k..k+3 (4*(lane>>4)+r) of column j (lane & 15) -> ws[split][j][k..k+3]
  float* ws = a.ws + (long long)split * a.Cg * a.Kg;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int k = k0 + wk * TM * 16 + i * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int jj = j0 + wc * TN * 16 + j * 16 + (lane & 15);
      if (k < a.Kg && jj < a.Cg)
        *reinterpret_cast<floatx4*>(ws + (long long)jj * a.Kg + k) = acc[i][j];
    }
  }
}

// ------------------------------------------------------------------------------------------ wgrad, bf16 fast path
// Same GEMM, no register transposes: both operands go HBM -> LDS by LDS-DMA in their natural NHWC
// orientation (rows = pixels, 128 bf16 = 256 B per row), and the MFMA fragments, which need 8
// consecutive PIXELS per lane, are read with gfx950's transposing LDS read ds_read_b64_tr_b16
// (cdna_hip_programming.md T10): per 16-lane group a 4-pixel x 16-column block arrives column-major,
// two reads give one 16x16x32 operand.  Image layout (T10 (b)): chunk ch of row r at byte
// 256 r + 16 (ch ^ (((r & 3) << 2) | ((r >> 2) & 3))) -- conflict-free for these transposed reads;
// applied on the DMA source side (the DMA writes lane-linear).  Im2col halo and tails cost nothing:
// an out-of-image tap or a pixel past M gets a voffset beyond the buffer range and the DMA writes 0.
// STAGES-deep ring with counted vmcnt + raw s_barrier, as conv_fast.
typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;
typedef __attribute__((address_space(3))) void lds_void_t;
typedef unsigned v4u_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4u_t lds_v4u_t;

__device__ __forceinline__ unsigned trswz(int row, int ch) {
  return 256u * (unsigned)row + 16u * (unsigned)(ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ void wg_dma16(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, unsigned voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(lds_addr), "v"(voff), "s"(rsrc) : "memory");
}

__device__ __forceinline__ v4s_t tr_read(unsigned byte_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(uintptr_t)byte_addr);
}

// INC: stride 1, no upsampled source, no ConvTranspose and Ho x Wo = H x W -- each DMA row's X and dY byte offsets
// advance by PB pixels' stride per stage, kept in registers (wgrad_wide.hip's SHT 2), instead of the per-stage
// (n, y, x) -> offset products
// TOG (STAGES == 2): image-major ring (X of stage s at s IMG, dY at (2 + s) IMG, so the stage is address bit 14) and
// per-lane fragment-read addresses in registers, flipped once per stage (wgrad_wide.hip's TOG)
// XR: two X buffer resources, one per source (x_tile_src 2: the sources lie too far apart for one 2^31-byte
// resource).  A lane's chunk belongs to one source for the whole kernel, so each X DMA runs once under the exec mask
// of source-A lanes and once under source-B lanes: masked-off lanes write nothing to LDS, the lanes of a row still
// fill its 256 B, and the tiles may mix the two sources as in the one-resource mode -- same tiles, same per-element
// accumulation order, so the result does not depend on where the allocator put the two tensors.
template <int BC, int WK, int WC, int STAGES, bool INC = false, bool TOG = false, bool XR = false>
__global__ void __launch_bounds__(256) conv_wgrad_tr_kernel(WgradArgs a) {
  constexpr int BK = 128, PB = 64;
  constexpr int TM = BK / (WK * 16), TN = BC / (WC * 16);
  constexpr int IMG = PB * 256;            // bytes of one operand image
  constexpr int STAGE = 2 * IMG;           // X image, then dY image
  constexpr int NL = 8;                    // DMA instructions per wave per stage (4 X + 4 dY)
  static_assert(WK * WC == 4 && TM >= 1 && TN >= 1, "tile");
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wk = w / WC, wc = w % WC;
  // 1-D grid, XCD-major bijective remap: the hardware deals consecutive workgroups round-robin over the 8 XCDs,
  // so consecutive remapped ids -- the K / Cout tiles of one pixel split, fastest -- run on one XCD at about
  // the same time and share its L2: every tap tile of a split re-reads the same (shifted) activation rows
  // and the same dY rows, which otherwise came from HBM once per tile
  const int nkt = (a.Kg + BK - 1) / BK, nct = (a.Cg + BC - 1) / BC;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = orig & 7, loc = orig >> 3;
  const int wgi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int k0 = (wgi % nkt) * BK, j0 = ((wgi / nkt) % nct) * BC, split = wgi / (nkt * nct);
  const int pb_begin = split * a.blocks_per_split;
  const int nblocks = (a.M + PB - 1) / PB;
  int pb_end = pb_begin + a.blocks_per_split;
  if (pb_end > nblocks) pb_end = nblocks;
  const int nit = pb_end > pb_begin ? pb_end - pb_begin : 0;

  // X source per lane chunk: a 128-column K tile may hold channels of both sources (the EnhancedUNet's 64 + 64
  // decoder concat), so one buffer resource spans both tensors from the lower address (the launcher checks that
  // the two fit in 2^31 bytes of it) and each lane carries its source's byte offset, channel stride and
  // upsampling shift
  const char* const pa = reinterpret_cast<const char*>(d.srcA);
  const char* const pb = d.Cb ? reinterpret_cast<const char*>(d.srcB) : pa;
  const bool tile_a = d.Cb == 0 || k0 % a.Cin < d.Ca;   // (x_tile_src 1: the K tile's one source)
  const char* const xbase = XR ? pa : a.x_tile_src ? (tile_a ? pa : pb) : (pa < pb ? pa : pb);
  const unsigned dA = a.x_tile_src ? 0u : (unsigned)(pa - xbase), dB = a.x_tile_src ? 0u : (unsigned)(pb - xbase);
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(xbase), (short)0, 0x7fffffff,
                                                                       0x00020000);
  const __amdgpu_buffer_rsrc_t rXb = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(pb), (short)0, 0x7fffffff,
                                                                        0x00020000);
  const __amdgpu_buffer_rsrc_t rY = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.dy), (short)0, 0x7fffffff,
                                                                       0x00020000);
  const unsigned OOB = 0x80000000u;

  // per-lane DMA state: instruction i fills rows 4(w + 4i) .. +3; this lane row (lane >> 4), slot lane & 15
  int xo[4], ky[4], kx[4], yo[4];       // X channel offset (or -1 = zero column), tap; dY column offset (or -1)
  int xcs[4], xsh[4];                   // X source's channel stride and upsampling shift (src A of a decoder: 1)
  unsigned xd[4];                       // X source's byte offset from the resource base
  int pn[4], py[4], px[4], pp[4];       // pixel (n, oy, ox) and flat index of the lane's row
  int yq[4];                            // ConvTranspose: the column's sub-pixel q (output pixel 2y + q/2, 2x + q%2)
  unsigned bias_lanes = 0;              // bit i: this lane's chunk of instruction i is the GEMM-bias column's
  unsigned b_lanes = 0;                 // XR, bit i: this lane's chunk of instruction i reads source B
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 4 * (w + 4 * i) + (lane >> 4);
    const int c = (lane & 15) ^ (((r & 3) << 2) | ((r >> 2) & 3));
    const int k = k0 + 8 * c;
    const int tap = k / a.Cin;
    const int ci = k - tap * a.Cin;
    const bool la = d.Cb == 0 || ci < d.Ca;
    xo[i] = k < a.Ktot ? (la ? d.a_coff + ci : d.b_coff + ci - d.Ca) : -1;
    xcs[i] = la ? d.a_cstride : d.b_cstride;
    xsh[i] = (la && d.a_up == 2) ? 1 : 0;
    xd[i] = la ? dA : dB;
    if (!la) b_lanes |= 1u << i;
    if (a.want_bias && k == a.Ktot) bias_lanes |= 1u << i;
    ky[i] = tap / d.KW;
    kx[i] = tap - ky[i] * d.KW;
    const int j = j0 + 8 * c;
    yq[i] = 0;
    if (d.convT) {   // GEMM column j = q * C + co (C % 8 == 0: a chunk never straddles two q)
      const int C = d.Cout >> 2, q = j / C;
      yq[i] = q;
      yo[i] = j < d.Cout ? a.dy_coff + (j - q * C) : -1;
    } else {
      yo[i] = j < d.Cout ? a.dy_coff + j : -1;
    }
    const int p = pb_begin * PB + r;
    pp[i] = p;
    px[i] = p % d.Wo;
    const int tt = p / d.Wo;
    py[i] = tt % d.Ho;
    pn[i] = tt / d.Ho;
  }
  unsigned ob[4], yb[4];   // INC: byte offsets of the row's tap-shifted X pixel (+ channel) and of its dY pixel
  if constexpr (INC) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int toff = (ky[i] - d.pad) * d.W + kx[i] - d.pad;
      ob[i] = xd[i] + 2u * (unsigned)xo[i] + 2u * (unsigned)(pp[i] + toff) * (unsigned)xcs[i];
      yb[i] = 2u * (unsigned)pp[i] * (unsigned)a.dy_cs;
    }
  }
  const unsigned yb_step = 2u * PB * (unsigned)a.dy_cs;
  const int adv_x = PB % d.Wo, adv_y = PB / d.Wo;
  const unsigned lds_base = (unsigned)(uintptr_t)(lds_void_t*)smem;

  static_assert(!TOG || (STAGES == 2 && IMG == 16384), "toggled fragment addressing");
  // LDS byte offsets of stage s's X and dY images
  auto xoff = [&](int s) __attribute__((always_inline)) -> unsigned { return (unsigned)(TOG ? s * IMG : s * STAGE); };
  auto yoff = [&](int s) __attribute__((always_inline)) -> unsigned {
    return (unsigned)(TOG ? (STAGES + s) * IMG : s * STAGE + IMG);
  };
  // the X DMA of instruction i (XR: from the lane's source's resource, under that source's lanes)
  auto dma_x = [&](int i, unsigned lds_addr, unsigned voff) __attribute__((always_inline)) {
    if constexpr (XR) {
      if (b_lanes & (1u << i)) wg_dma16(rXb, lds_addr, voff);
      else wg_dma16(rX, lds_addr, voff);
    } else {
      wg_dma16(rX, lds_addr, voff);
    }
  };
  auto issue = [&](int s) __attribute__((always_inline)) {
    const unsigned sb = lds_base + xoff(s), sby = lds_base + yoff(s);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned row_base = 256u * (unsigned)(4 * (w + 4 * i));
      if constexpr (INC) {
        const int iy = py[i] - d.pad + ky[i];
        const int ix = px[i] - d.pad + kx[i];
        const bool okx = xo[i] >= 0 && pp[i] < a.M && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
        dma_x(i, sb + row_base, okx ? ob[i] : OOB);
        const bool oky = yo[i] >= 0 && pp[i] < a.M;
        wg_dma16(rY, sby + row_base, oky ? yb[i] + 2u * (unsigned)yo[i] : OOB);
        ob[i] += (unsigned)xcs[i] * (2u * PB);
        yb[i] += yb_step;
        pp[i] += PB;
        px[i] += adv_x;
        py[i] += adv_y;
        if (px[i] >= d.Wo) { px[i] -= d.Wo; ++py[i]; }
        while (py[i] >= d.Ho) py[i] -= d.Ho;
        continue;
      }
      const int iy = py[i] * d.stride - d.pad + ky[i];
      const int ix = px[i] * d.stride - d.pad + kx[i];
      const bool okx = xo[i] >= 0 && pp[i] < a.M && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
      const int sh = xsh[i], Hs = d.H >> sh, Ws = d.W >> sh;
      const unsigned offx =
          okx ? xd[i] + (unsigned)((((pn[i] * Hs + (iy >> sh)) * Ws + (ix >> sh)) * xcs[i] + xo[i]) * 2) : OOB;
      dma_x(i, sb + row_base, offx);
      const bool oky = yo[i] >= 0 && pp[i] < a.M;
      int yp = pp[i];
      if (d.convT)   // the dY pixel of sub-pixel q: (n, 2y + q/2, 2x + q%2) of the 2H x 2W output grid
        yp = (pn[i] * (2 * d.Ho) + 2 * py[i] + (yq[i] >> 1)) * (2 * d.Wo) + 2 * px[i] + (yq[i] & 1);
      const unsigned offy = oky ? (unsigned)((yp * a.dy_cs + yo[i]) * 2) : OOB;
      wg_dma16(rY, sby + row_base, offy);
      // advance this row by PB pixels
      pp[i] += PB;
      px[i] += adv_x;
      py[i] += adv_y;
      if (px[i] >= d.Wo) { px[i] -= d.Wo; ++py[i]; }
      while (py[i] >= d.Ho) { py[i] -= d.Ho; ++pn[i]; }
    }
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // fragment read addressing: group g = lane >> 4 takes pixel rows 8g..8g+7 of a 32-pixel k-step;
  // lane 4q+p of the group addresses row q, columns 4p..4p+3 of its 16-column block
  const int g = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;

  // TOG: rows 8g + q (+ 4) of a k-step (k-step 1's rows 32 below), this wave's channel pairs, stage 0
  unsigned oX[TOG ? TM : 1][2], oY[TOG ? TN : 1][2];
  if constexpr (TOG) {
#pragma unroll
    for (int hi = 0; hi < 2; ++hi) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        oX[i][hi] = lds_base + xoff(0) + trswz(8 * g + q + 4 * hi, (wk * TM * 16 + i * 16) / 8 + (pq >> 1)) + 8u * (pq & 1);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        oY[j][hi] = lds_base + yoff(0) + trswz(8 * g + q + 4 * hi, (wc * TN * 16 + j * 16) / 8 + (pq >> 1)) + 8u * (pq & 1);
    }
  }

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nit) issue(s);

  for (int it = 0; it < nit; ++it) {
    if (it + STAGES - 2 < nit) {
      if constexpr (STAGES == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if constexpr (STAGES == 3) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NL) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * NL) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (bias_lanes) {   // the GEMM-bias column: X = 1 in every row (rows past M meet zero dY), written over the
                        // DMA's zeros once this stage landed
      const unsigned sb = lds_base + xoff(it % STAGES);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (bias_lanes & (1u << i))
          *reinterpret_cast<lds_v4u_t*>((uintptr_t)(sb + 256u * (unsigned)(4 * (w + 4 * i)) + 16u * (unsigned)lane)) =
              v4u_t{0x3f80u, 0u, 0u, 0u};
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (it + STAGES - 1 < nit) issue((it + STAGES - 1) % STAGES);

    const unsigned sX = lds_base + xoff(it % STAGES);
    const unsigned sY = lds_base + yoff(it % STAGES);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int r0 = ks * 32 + 8 * g + q;
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int ch = (wk * TM * 16 + i * 16) / 8 + (pq >> 1);
        const unsigned lo_a = TOG ? oX[i][0] + (unsigned)(ks * 32 * 256) : sX + trswz(r0, ch) + 8u * (pq & 1);
        const unsigned hi_a = TOG ? oX[i][1] + (unsigned)(ks * 32 * 256) : sX + trswz(r0 + 4, ch) + 8u * (pq & 1);
        const v4s_t lo = tr_read(lo_a);
        const v4s_t hi = tr_read(hi_a);
        af[i] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int ch = (wc * TN * 16 + j * 16) / 8 + (pq >> 1);
        const unsigned lo_a = TOG ? oY[j][0] + (unsigned)(ks * 32 * 256) : sY + trswz(r0, ch) + 8u * (pq & 1);
        const unsigned hi_a = TOG ? oY[j][1] + (unsigned)(ks * 32 * 256) : sY + trswz(r0 + 4, ch) + 8u * (pq & 1);
        const v4s_t lo = tr_read(lo_a);
        const v4s_t hi = tr_read(hi_a);
        bfr[j] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if constexpr (TOG) {   // the next stage's buffers
#pragma unroll
      for (int hi = 0; hi < 2; ++hi) {
#pragma unroll
        for (int i = 0; i < TM; ++i) oX[i][hi] ^= (unsigned)IMG;
#pragma unroll
        for (int j = 0; j < TN; ++j) oY[j][hi] ^= (unsigned)IMG;
      }
    }
  }

  float* ws = a.ws + (long long)split * a.Cg * a.Kg;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int k = k0 + wk * TM * 16 + i * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int jj = j0 + wc * TN * 16 + j * 16 + (lane & 15);
      if (k < a.Kg && jj < a.Cg)
        *reinterpret_cast<floatx4*>(ws + (long long)jj * a.Kg + k) = acc[i][j];
    }
  }
}

template <int BC, int WK, int WC, int STAGES, bool INC = false, bool TOG = false, bool XR = false>
static int wgrad_tr_launch(const WgradArgs& a, hipStream_t s) {
  const size_t lds = (size_t)STAGES * 2 * 64 * 256;
  auto kern = conv_wgrad_tr_kernel<BC, WK, WC, STAGES, INC, TOG, XR>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  const int nwg = ((a.Kg + 127) / 128) * ((a.Cg + BC - 1) / BC) * a.splits;
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(256), lds, s, a);
  return hiseg_check_launch("conv_wgrad_tr");
}

// developer knob: HISEG_WGRAD_TR=0 forces the register-transpose kernel
static int wgrad_tr_mode() {
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("HISEG_WGRAD_TR");
    mode = e ? atoi(e) : 1;
  }
  return mode;
}

// 1 = launched, 0 = layer not eligible (caller uses the generic kernel)
static int wgrad_tr_try(const WgradArgs& a, hipStream_t s) {
  const hiseg_conv2d_desc& d = a.d;
  if (!wgrad_tr_mode()) return 0;
  if (d.dtype != HISEG_BF16) return 0;
  // 8-channel chunks never straddle the two sources
  if (d.Ca % 8 || a.Cin % 8 || a.dy_cs % 8 || a.dy_coff % 8 || d.a_cstride % 8 || d.a_coff % 8) return 0;
  if (d.Cb && (d.b_cstride % 8 || d.b_coff % 8)) return 0;
  if (d.convT && (d.Cout % 32 || d.a_up != 1)) return 0;   // C = Cout / 4 a multiple of 8
  const long long span_a = (long long)d.N * d.H * d.W * d.a_cstride * 2;
  const long long span_b = d.Cb ? (long long)d.N * d.H * d.W * d.b_cstride * 2 : 0;
  const long long span_y = ((long long)a.M * (d.convT ? 4 : 1) * a.dy_cs + a.dy_coff + a.Cg) * 2;
  if (span_a >= 0x7fffffffll || span_b >= 0x7fffffffll || span_y >= 0x7fffffffll) return 0;
  WgradArgs b = a;
  b.x_tile_src = 0;
  if (d.Cb) {   // both sources within 2^31 bytes of the lower one (one X resource), else one source per K tile
    const long long pa = (long long)(uintptr_t)d.srcA, pb = (long long)(uintptr_t)d.srcB;
    const long long lo = pa < pb ? pa : pb;
    if (pa - lo + span_a >= 0x7fffffffll || pb - lo + span_b >= 0x7fffffffll || hiseg_force_far()) {
      // A ends on a 128-column tile boundary and (with more than one tap) so does each tap: one source per tile;
      // else one resource per source, chosen per lane (XR)
      const bool aligned = d.Ca % 128 == 0 && (d.KH * d.KW == 1 || d.Cb % 128 == 0);
      hiseg_note_placement(aligned ? "wgrad_tr: one source per tile (sources far apart)"
                                   : "wgrad_tr: one resource per source (sources far apart)", &d);
      b.x_tile_src = aligned ? 1 : 2;
    }
  }
  // incremental DMA offsets (INC above; HISEG_WGRAD_INC=0 for A/B timing, read per call)
  const char* e = getenv("HISEG_WGRAD_INC");
  const bool inc = !(e && atoi(e) == 0) && !d.convT && d.stride == 1 && d.a_up == 1 && d.Ho == d.H && d.Wo == d.W;
  const char* et = getenv("HISEG_WGRAD_TOG");   // flipped fragment-read registers (TOG above; 0 for A/B timing)
  const bool tog = !(et && atoi(et) == 0);
  if (b.x_tile_src == 2) {
    const int r = inc && b.Cg >= 128 ? wgrad_tr_launch<128, 2, 2, 2, true, true, true>(b, s)
                : inc && b.Cg >= 64  ? wgrad_tr_launch<64, 4, 1, 2, true, true, true>(b, s)
                : b.Cg >= 128 ? wgrad_tr_launch<128, 2, 2, 2, false, false, true>(b, s)
                : b.Cg >= 64  ? wgrad_tr_launch<64, 4, 1, 2, false, false, true>(b, s)
                : b.Cg >= 32  ? wgrad_tr_launch<32, 4, 1, 2, false, false, true>(b, s)
                              : wgrad_tr_launch<16, 4, 1, 2, false, false, true>(b, s);
    return r < 0 ? r : 1;
  }
  const int r = inc && tog && b.Cg >= 128 ? wgrad_tr_launch<128, 2, 2, 2, true, true>(b, s)
              : inc && tog && b.Cg >= 64  ? wgrad_tr_launch<64, 4, 1, 2, true, true>(b, s)
              : inc && b.Cg >= 128 ? wgrad_tr_launch<128, 2, 2, 2, true>(b, s)
              : inc && b.Cg >= 64  ? wgrad_tr_launch<64, 4, 1, 2, true>(b, s)
              : b.Cg >= 128 ? wgrad_tr_launch<128, 2, 2, 2>(b, s)
              : b.Cg >= 64  ? wgrad_tr_launch<64, 4, 1, 2>(b, s)
              : b.Cg >= 32  ? wgrad_tr_launch<32, 4, 1, 2>(b, s)
                            : wgrad_tr_launch<16, 4, 1, 2>(b, s);
  return r < 0 ? r : 1;
}

template <typename T, int BK, int BC, int WK, int WC>
static int wgrad_launch(const WgradArgs& a, hipStream_t s) {
  constexpr int STAGE = (BK + BC) * 8;
  const size_t lds = 2 * STAGE * sizeof(uint4);
  dim3 grid((a.Kg + BK - 1) / BK, (a.Cg + BC - 1) / BC, a.splits);
  hipLaunchKernelGGL((conv_wgrad_kernel<T, BK, BC, WK, WC>), grid, dim3(256), lds, s, a);
  return hiseg_check_launch("conv_wgrad");
}

template <typename T>
static int wgrad_typed(const WgradArgs& a, hipStream_t s) {
  if (a.Cg >= 128) return wgrad_launch<T, 128, 128, 2, 2>(a, s);
  if (a.Cg >= 64) return wgrad_launch<T, 128, 64, 2, 2>(a, s);
  if (a.Cg >= 32) return wgrad_launch<T, 128, 32, 2, 2>(a, s);
  return wgrad_launch<T, 64, 16, 4, 1>(a, s);
}

// Which kernel took each weight gradient (hiseg_wgrad_path_stats, hiseg_wgrad_last_path): the wide tile, the
// transposed-read tile, the generic register-transpose kernel in bf16 (a fallback: HISEG_LOG_WGRAD=1 names the
// layer), or the f32 kernel (parity mode, by design).
static std::atomic<long long> g_wgrad_paths[5];
static thread_local int g_wgrad_last = -1;

static void wgrad_note_path(int path, const hiseg_conv2d_desc* d, int dy_cs, int dy_coff) {
  g_wgrad_paths[path].fetch_add(1);
  g_wgrad_last = path;
  static const bool log = getenv("HISEG_LOG_WGRAD") != nullptr;
  if (log && path == HISEG_WGRAD_PATH_GENERIC)
    fprintf(stderr,
            "[hiseg wgrad] generic kernel: %d+%d -> %d, %dx%d taps s%d p%d, N %d %dx%d -> %dx%d, convT %d up %d, "
            "A %p cs %d off %d, B %p cs %d off %d, dy cs %d off %d\n",
            d->Ca, d->Cb, d->Cout, d->KH, d->KW, d->stride, d->pad, d->N, d->H, d->W, d->Ho, d->Wo, d->convT, d->a_up,
            d->srcA, d->a_cstride, d->a_coff, d->srcB, d->b_cstride, d->b_coff, dy_cs, dy_coff);
}

static int wgrad_geometry(const hiseg_conv2d_desc* d, int want_bias, int* Cg, int* Kg, int* splits, int* M,
                          int* Cin, int* Ktot, int* bps) {
  HISEG_REQUIRE(d != nullptr, HISEG_ERR_BAD_ARG, "wgrad: null descriptor");
  HISEG_REQUIRE(d->dtype == HISEG_F32 || d->dtype == HISEG_BF16, HISEG_ERR_BAD_DTYPE, "wgrad: dtype %d", d->dtype);
  const int kch = d->dtype == HISEG_BF16 ? 8 : 4;
  *Cin = d->Ca + d->Cb;
  HISEG_REQUIRE(d->Ca > 0 && d->Ca % kch == 0 && d->Cb % kch == 0, HISEG_ERR_BAD_SHAPE, "wgrad: channels");
  HISEG_REQUIRE(d->Cout > 0 && d->Cout % kch == 0 && (!d->convT || (d->Cout / 4) % kch == 0), HISEG_ERR_BAD_SHAPE,
                "wgrad: Cout %d must be a multiple of %d (per sub-pixel for convT)", d->Cout, kch);
  *Ktot = d->KH * d->KW * (*Cin);
  *Kg = (*Ktot + (want_bias ? 1 : 0) + 63) / 64 * 64;
  *Cg = (d->Cout + 15) / 16 * 16;
  const long long Mll = (long long)d->N * d->Ho * d->Wo;
  HISEG_REQUIRE(Mll > 0 && Mll < (1ll << 31), HISEG_ERR_BAD_SHAPE, "wgrad: pixels");
  *M = (int)Mll;
  const int PB = 8 * kch;
  const int nblocks = (*M + PB - 1) / PB;
  // The pixel partition into splits follows the 128-column tiles for every kernel (the wide 256 x 256 tile of
  // wgrad_wide.hip included): an element's f32 accumulation order -- the 64-pixel blocks of its split, then the
  // splits in order -- is then the same whichever kernel runs it, and the kernel choice depends on where the
  // allocator placed two-source operands (one buffer resource must span both), which must never change the result.
  const int BK = *Kg >= 128 ? 128 : 64;
  const int BC = *Cg >= 128 ? 128 : *Cg >= 64 ? 64 : *Cg >= 32 ? 32 : 16;
  const long long tiles = (long long)((*Kg + BK - 1) / BK) * ((*Cg + BC - 1) / BC);
  // about 1024 workgroups but never past it: the wgrad kernels run two workgroups per CU, so 1024 = two full
  // rounds on 256 CUs, and rounding up (36 tiles x 29 splits = 1044) added a third, nearly empty round that cost
  // a third of the layer's time (the wide kernel, one workgroup per CU, gets a quarter of them per round)
  int sp = (int)(1024 / tiles);
  if (wgrad_hwc_shape_ok(d)) sp = wgrad_hwc_splits(d);   // the halo tile's own pixel partition (wgrad_hwc.hip)
  if (sp > nblocks) sp = nblocks;
  if (sp < 1) sp = 1;
  *bps = (nblocks + sp - 1) / sp;
  *splits = (nblocks + *bps - 1) / *bps;
  return HISEG_OK;
}

}  // namespace hiseg

using namespace hiseg;

extern "C" int hiseg_conv2d_wgrad_dims(const hiseg_conv2d_desc* fwd, int want_bias, int* Cg, int* Kg, int* splits) {
  int M, Cin, Ktot, bps;
  return wgrad_geometry(fwd, want_bias, Cg, Kg, splits, &M, &Cin, &Ktot, &bps);
}

extern "C" int hiseg_conv2d_wgrad(const hiseg_conv2d_desc* fwd, const void* dy, int dy_cstride, int dy_coff,
                                  int want_bias, float* ws, int splits, hiseg_stream_t stream) {
  WgradArgs a;
  int sp;
  const int r = wgrad_geometry(fwd, want_bias, &a.Cg, &a.Kg, &sp, &a.M, &a.Cin, &a.Ktot, &a.blocks_per_split);
  if (r) return r;
  HISEG_REQUIRE(splits == sp, HISEG_ERR_BAD_ARG, "wgrad: splits %d != %d from hiseg_conv2d_wgrad_dims", splits, sp);
  HISEG_REQUIRE(dy && ws && fwd->srcA, HISEG_ERR_BAD_ARG, "wgrad: null pointer");
  const int kch = fwd->dtype == HISEG_BF16 ? 8 : 4;
  HISEG_REQUIRE(dy_cstride % kch == 0 && dy_coff % kch == 0, HISEG_ERR_BAD_SHAPE, "wgrad: dy view alignment");
  HISEG_REQUIRE(al16(dy) && al16(fwd->srcA) && al16(fwd->srcB) && al16(ws), HISEG_ERR_BAD_SHAPE, "wgrad: alignment");
  a.d = *fwd;
  a.dy = dy; a.dy_cs = dy_cstride; a.dy_coff = dy_coff;
  a.want_bias = want_bias;
  a.splits = splits;
  a.ws = ws;
  hipStream_t s = (hipStream_t)stream;
  const int rh = wgrad_hwc_try(a, s);
  if (rh != 0) {
    if (rh > 0) wgrad_note_path(HISEG_WGRAD_PATH_HWC, fwd, dy_cstride, dy_coff);
    return rh < 0 ? rh : HISEG_OK;
  }
  const int rw = wgrad_wide_try(a, s);
  if (rw != 0) {
    if (rw > 0) wgrad_note_path(HISEG_WGRAD_PATH_WIDE, fwd, dy_cstride, dy_coff);
    return rw < 0 ? rw : HISEG_OK;
  }
  const int rt = wgrad_tr_try(a, s);
  if (rt != 0) {
    if (rt > 0) wgrad_note_path(HISEG_WGRAD_PATH_TR, fwd, dy_cstride, dy_coff);
    return rt < 0 ? rt : HISEG_OK;
  }
  wgrad_note_path(fwd->dtype == HISEG_BF16 ? HISEG_WGRAD_PATH_GENERIC : HISEG_WGRAD_PATH_F32, fwd, dy_cstride, dy_coff);
  return fwd->dtype == HISEG_BF16 ? wgrad_typed<bf16_t>(a, s) : wgrad_typed<float>(a, s);
}

extern "C" int hiseg_wgrad_path_stats(long long* counts, int reset) {
  for (int i = 0; i < 5; ++i) {
    if (counts) counts[i] = g_wgrad_paths[i].load();
    if (reset) g_wgrad_paths[i] = 0;
  }
  return HISEG_OK;
}

extern "C" int hiseg_wgrad_last_path(void) { return g_wgrad_last; }

// A block = 64 column quads (4 consecutive K columns of one GEMM column j each) x 4 split groups: group g sums splits
// g, g + 4, ... with eight float4 loads in flight, the groups are combined in LDS in a fixed order, then the quad's
// 4 sums go to their reference-layout slots.  (One thread per quad walking every split four loads at a time left
// the 113-split 128-channel layers latency-bound: 144 blocks, ~30 us per launch at ~2.3 TB/s.)
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* ws, int splits, hiseg_wgrad_map m, float* gw,
                                                           float* gb, int acc) {
  __shared__ float4 red[4][64];
  const int ql = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const long long idx = (long long)blockIdx.x * 64 + ql;
  const int Cin = m.ca + m.cb;
  const int Ktot = m.KH * m.KW * Cin;
  const int ncol = Ktot + (m.want_bias ? 1 : 0);
  const int nq4 = (ncol + 3) >> 2;
  const bool live = idx < (long long)m.Cout * nq4;
  const int j = live ? (int)(idx / nq4) : 0;
  const int k0 = live ? 4 * (int)(idx - (long long)j * nq4) : 0;
  const long long plane = (long long)m.Cg * m.Kg;
  const float* src = ws + (long long)j * m.Kg + k0;
  float4 s8[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) s8[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live) {
    for (int sp = sg; sp < splits; sp += 32) {
      float4 a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        a[u] = sp + 4 * u < splits ? *reinterpret_cast<const float4*>(src + (sp + 4 * u) * plane) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 8; ++u) { s8[u].x += a[u].x; s8[u].y += a[u].y; s8[u].z += a[u].z; s8[u].w += a[u].w; }
    }
  }
  auto add4 = [](float4 x, float4 y) { return make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w); };
  red[sg][ql] = add4(add4(add4(s8[0], s8[1]), add4(s8[2], s8[3])), add4(add4(s8[4], s8[5]), add4(s8[6], s8[7])));
  __syncthreads();
  if (sg != 0 || !live) return;
  const float4 t4 = add4(add4(red[0][ql], red[1][ql]), add4(red[2][ql], red[3][ql]));
  const float tot[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = k0 + e;
    if (k >= ncol) break;
    if (k == Ktot) {  // bias column
      if (!gb) continue;
      if (m.convT) {
        const int C = m.Cout / 4;
        if (j >= C) continue;  // the q == 0 thread sums the 4 sub-pixel columns
        float b = 0.f;
        for (int q = 0; q < 4; ++q) {
          const int jj = j + q * C;
          for (int p = 0; p < splits; ++p) b += ws[p * plane + (long long)jj * m.Kg + k];
        }
        gb[j] = acc ? gb[j] + b : b;
      } else {
        gb[j] = acc ? gb[j] + tot[e] : tot[e];
      }
      continue;
    }
    long long dst;
    if (m.convT) {
      const int C = m.Cout / 4;
      const int q = j / C, co = j - q * C;
      if (k >= m.ca_real) continue;
      dst = (((long long)k * C + co) * 2 + (q >> 1)) * 2 + (q & 1);
    } else {
      const int tap = k / Cin, cp = k - tap * Cin;
      int ci;
      if (cp < m.ca) {
        if (cp >= m.ca_real) continue;
        ci = cp;
      } else {
        const int b = cp - m.ca;
        if (b >= m.cb_real) continue;
        ci = m.ca_real + b;
      }
      const int ky = tap / m.KW, kx = tap - ky * m.KW;
      dst = (((long long)j * (m.ca_real + m.cb_real) + ci) * m.KH + ky) * m.KW + kx;
    }
    gw[dst] = acc ? gw[dst] + tot[e] : tot[e];
  }
}

// 3x3 single-source layers: one item = (GEMM column j, 4 consecutive input channels) over all 9 taps, so an item's
// 36 sums are 36 consecutive floats of the reference layout [Cout][Cin][3][3] -- nine 16-B stores -- where the
// quad-of-K kernel above scatters 4-B stores 9 floats apart (the write traffic of the 768-channel 3x3 layers of the
// B7 head: 137 us per reduce).  Sixteen split groups per item, combined in a fixed order.
// NI items x NG split groups per block: 64 x 4, or 16 x 16 for more than 64 splits (round 5: 64 x 4 left the halo
// weight-gradient tile's many-split planes latency-bound -- 64 -> 64 at 256 splits: 42 -> 17 us; with 32 splits the
// 16 x 16 form was 3x slower, its combine left to 16 lanes per block); group g sums splits g, g + NG, ...
template <int NI, int NG>
__global__ void __launch_bounds__(256) wgrad_reduce_taps_kernel(const float* ws, int splits, hiseg_wgrad_map m,
                                                                float* gw, float* gb, int acc) {
  __shared__ float4 red[NG][9][NI];
  __shared__ float redb[NG][NI];
  const int il = threadIdx.x % NI, sg = threadIdx.x / NI;
  const int Cin = m.ca, nc4 = Cin >> 2;
  const long long idx = (long long)blockIdx.x * NI + il;
  const bool live = idx < (long long)m.Cout * nc4;
  const int j = live ? (int)(idx / nc4) : 0;
  const int ci0 = live ? 4 * (int)(idx - (long long)j * nc4) : 0;
  const long long plane = (long long)m.Cg * m.Kg;
  const float* src = ws + (long long)j * m.Kg + ci0;
  const bool bias = m.want_bias && gb && ci0 == 0;
  float4 t9[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) t9[t] = make_float4(0.f, 0.f, 0.f, 0.f);
  float tb = 0.f;
  if (live) {
    for (int sp = sg; sp < splits; sp += NG) {
      float4 a[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) a[t] = *reinterpret_cast<const float4*>(src + sp * plane + t * Cin);
      if (bias) tb += src[sp * plane + 9 * Cin];
#pragma unroll
      for (int t = 0; t < 9; ++t) { t9[t].x += a[t].x; t9[t].y += a[t].y; t9[t].z += a[t].z; t9[t].w += a[t].w; }
    }
  }
#pragma unroll
  for (int t = 0; t < 9; ++t) red[sg][t][il] = t9[t];
  redb[sg][il] = tb;
  __syncthreads();
  if (sg != 0 || !live) return;
  auto add4 = [](float4 x, float4 y) { return make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w); };
  float o[36];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    float4 v = red[0][t][il];
#pragma unroll
    for (int g = 1; g < NG; ++g) v = add4(v, red[g][t][il]);
    o[t] = v.x; o[9 + t] = v.y; o[18 + t] = v.z; o[27 + t] = v.w;   // [channel][tap]
  }
  float4* dst = reinterpret_cast<float4*>(gw + ((long long)j * Cin + ci0) * 9);
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    float4 v = make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    if (acc) v = add4(dst[q], v);
    dst[q] = v;
  }
  if (bias) {   // the GEMM-bias column (k = 9 Cin), the groups in order
    float b = redb[0][il];
#pragma unroll
    for (int g = 1; g < NG; ++g) b += redb[g][il];
    gb[j] = acc ? gb[j] + b : b;
  }
}

extern "C" int hiseg_conv2d_wgrad_reduce(const float* ws, int splits, const hiseg_wgrad_map* map, float* gw, float* gb,
                                         int accumulate, hiseg_stream_t stream) {
  HISEG_REQUIRE(ws && map && gw && splits > 0, HISEG_ERR_BAD_ARG, "wgrad_reduce: null argument");
  const hiseg_wgrad_map m = *map;
  HISEG_REQUIRE(!m.convT || m.Cout % 4 == 0, HISEG_ERR_BAD_SHAPE, "wgrad_reduce: convT Cout");
  HISEG_REQUIRE(m.Kg % 4 == 0 && al16(ws), HISEG_ERR_BAD_SHAPE, "wgrad_reduce: partial rows must be 16-B aligned");
  const char* te = getenv("HISEG_WGRAD_REDUCE_TAPS");   // 0: the quad-of-K kernel (A/B, the equivalence test)
  const bool taps_ok = !(te && atoi(te) == 0);
  if (taps_ok && !m.convT && m.KH == 3 && m.KW == 3 && m.cb == 0 && m.ca == m.ca_real && m.ca % 4 == 0 && al16(gw)) {
    const long long items = (long long)m.Cout * (m.ca / 4);
    if (splits > 64)
      hipLaunchKernelGGL((wgrad_reduce_taps_kernel<16, 16>), dim3((unsigned)((items + 15) / 16)), dim3(256), 0,
                         (hipStream_t)stream, ws, splits, m, gw, gb, accumulate);
    else
      hipLaunchKernelGGL((wgrad_reduce_taps_kernel<64, 4>), dim3((unsigned)((items + 63) / 64)), dim3(256), 0,
                         (hipStream_t)stream, ws, splits, m, gw, gb, accumulate);
    return hiseg_check_launch("wgrad_reduce");
  }
  const long long n = (long long)m.Cout * ((m.KH * m.KW * (m.ca + m.cb) + (m.want_bias ? 1 : 0) + 3) / 4);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, (hipStream_t)stream, ws,
                     splits, m, gw, gb, accumulate);
  return hiseg_check_launch("wgrad_reduce");
}

// ------------------------------------------------------------------------------------------ packing
__device__ __forceinline__ int real_channel(const hiseg_pack_entry& e, int cp) {
  if (cp < e.ca) return cp < e.ca_real ? cp : -1;
  const int b = cp - e.ca;
  return b < e.cb_real ? e.ca_real + b : -1;
}

__global__ void __launch_bounds__(256) pack_weights_kernel(const hiseg_pack_entry* table) {
  const hiseg_pack_entry e = table[blockIdx.y];
  // 32-bit element indices (total is an int; the 64-bit divisions were software routines -- measured no faster:
  // the launch, 0.9 ms of the B7 train step, is bound by the gathered / transposed f32 reads of the dgrad layouts)
  for (int idx = blockIdx.x * 256 + threadIdx.x; idx < e.total; idx += gridDim.x * 256) {
    int row, k;
    const int cinp = e.ca + e.cb;
    const int mode = e.mode & 7;
    if (e.mode & HISEG_PACK_FRAG) {   // fragment order: idx = (((((ct*ncb + cb)*taps + tap)*2 + s)*4 + lg)*16 + r)*8 + el
      const int kc = mode == 0 ? cinp : e.cop;   // K channels per tap
      const int taps = e.KH * e.KW, ncb = kc >> 6;
      int t = idx;
      const int el = t & 7; t >>= 3;
      const int r = t & 15; t >>= 4;
      const int lg = t & 3; t >>= 2;
      const int s = t & 1; t >>= 1;
      const int tap = t % taps; t /= taps;
      const int cb = t % ncb;
      const int ct = t / ncb;
      row = ct * 16 + r;
      k = tap * kc + cb * 64 + s * 32 + lg * 8 + el;
    } else {
      row = idx / e.K_pad;
      k = idx - row * e.K_pad;
    }
    float v = 0.f;
    if (mode == HISEG_PACK_BIAS) {  // bias -> f32 epilogue shift, replicated per ConvTranspose sub-pixel block
      v = e.src[idx % e.Cout];   // (32-bit)
    } else if (mode == 0) {     // conv forward: [co][tap*cinp + cp]
      if (row < e.Cout && k < e.KH * e.KW * cinp) {
        const int tap = k / cinp, ci = real_channel(e, k - tap * cinp);
        if (ci >= 0) v = e.src[((long long)row * e.Cin_real + ci) * e.KH * e.KW + tap];
      }
    } else if (mode == 1) {       // conv dgrad: [cp_in][tap'*cop + co], taps flipped
      const int ci = row < cinp ? real_channel(e, row) : -1;
      if (ci >= 0 && k < e.KH * e.KW * e.cop) {
        const int tap2 = k / e.cop, co = k - tap2 * e.cop;
        if (co < e.Cout) {
          const int ky = e.KH - 1 - tap2 / e.KW, kx = e.KW - 1 - (tap2 % e.KW);
          v = e.src[(((long long)co * e.Cin_real + ci) * e.KH + ky) * e.KW + kx];
        }
      }
    } else if (mode == 2) {       // convT forward: [q*C + co][ci], W [Cin][C][2][2]
      if (row < 4 * e.Cout && k < e.Cin_real) {
        const int q = row / e.Cout, co = row - q * e.Cout;
        v = e.src[((long long)k * e.Cout + co) * 4 + q];
      }
    } else {                      // convT dgrad: 2x2/s2 conv [ci][tap*cop + co]
      if (row < e.Cin_real && k < 4 * e.cop) {
        const int tap = k / e.cop, co = k - tap * e.cop;
        if (co < e.Cout) v = e.src[((long long)row * e.Cout + co) * 4 + tap];
      }
    }
    if (e.dtype == HISEG_BF16) reinterpret_cast<uint16_t*>(e.dst)[idx] = f2bf(v);
    else reinterpret_cast<float*>(e.dst)[idx] = v;
  }
}

extern "C" int hiseg_pack_weights(const hiseg_pack_entry* table_dev, int n, int max_total, hiseg_stream_t stream) {
  HISEG_REQUIRE(table_dev && n > 0 && max_total > 0, HISEG_ERR_BAD_ARG, "pack_weights: empty table");
  int bx = (max_total + 255) / 256;
  if (bx > 512) bx = 512;
  hipLaunchKernelGGL(pack_weights_kernel, dim3(bx, n), dim3(256), 0, (hipStream_t)stream, table_dev);
  return hiseg_check_launch("pack_weights");
}
