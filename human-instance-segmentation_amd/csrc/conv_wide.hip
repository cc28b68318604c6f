// Wide-tile implicit-GEMM convolution for uniform bf16 layers (gfx950): one 256-thread workgroup
// per CU owns a BCO (Cout) x 256 (pixel) output tile, 4 waves as 2 (Cout) x 2 (pixel), each wave a
// (BCO/2) x 128 sub-tile.
//
// Why this shape (tools/conv_bench.py + PMC/stamp measurements, profiles/r2_*): the 128x128 ring
// kernel (conv_fast.hip) spends its K loop at ~44 % MFMA: a 32x64 wave tile needs 0.75 ds_read_b128
// LDS cycles per MFMA cycle on top of the LDS-DMA writes, and a 128x128 tile draws 64 B/clk/CU from
// L2 at full MFMA rate -- both at their limits.  A 128x128 WAVE tile halves the LDS read bytes per
// FLOP twice over (0.25 LDS cycles per MFMA cycle) and the 256-wide workgroup tile halves the L2
// bytes per FLOP (32 B/clk/CU at peak).  The accumulators (256 per lane for BCO = 256) live in the
// AGPR half of the register file, so the file is built without -amdgpu-mfma-vgpr-form and runs one
// wave per SIMD.
//
// K runs in 32-deep stages (one filter tap x 32 input channels).  Operands reach LDS by LDS-DMA
// (buffer_load_dwordx4 ... lds, 16 rows x 64 B per wave instruction) into a STAGES-deep ring;
// out-of-image taps get an out-of-range voffset and the DMA writes zeros.  64-B LDS rows are
// swizzled chunk c of row r -> slot c ^ f(r), f(r) = (-(r >> 2)) & 3: conflict-free for the four
// ds_read_b128 lane groups of a fragment read (MI355X_MICROARCH.md §LDS; rows r..r+15 with 16 | r),
// applied on the SOURCE address because the DMA writes lane-linearly.
// Per stage each wave runs 4 groups of (TM/4) x 8 MFMAs; the fragment reads of group g+1 are issued
// before the MFMAs of group g, the stage hand-over (counted vmcnt + lgkmcnt(0) + raw s_barrier + the
// DMA of stage s+STAGES-1) sits between groups 2 and 3, and the next stage's B fragments are read
// under group 3's MFMAs: one barrier per 1024 MFMA cycles per wave and no exposed fragment read.
// Accumulation order equals conv_fast's (k ascending in 32-deep MFMA steps): bit-identical outputs.
#include <type_traits>

#include "conv_common.h"

namespace hiseg {

#ifdef HISEG_DIAG
constexpr bool HISEG_DIAG_ON = true;
#else
constexpr bool HISEG_DIAG_ON = false;
#endif

typedef __attribute__((address_space(3))) void lds_void_w;

__device__ __forceinline__ void dma16w(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, unsigned voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(__builtin_amdgcn_readfirstlane(lds_addr)), "v"(voff), "s"(rsrc) : "memory");
}

template <int N>
__device__ __forceinline__ void wvm() {
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

// wait until at most k stages of NL DMA instructions each are outstanding
template <int NL>
__device__ __forceinline__ void wvm_stages(int k) {
  if (k <= 0) wvm<0>();
  else if (k == 1) wvm<NL>();
  else if (k == 2) wvm<2 * NL>();
  else wvm<3 * NL>();
}

__device__ __forceinline__ int wswz(int r) { return (-(r >> 2)) & 3; }

__device__ __forceinline__ unsigned long long wstamp() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  return t;
}

// STAMP (diagnostic builds only): wave 0 lane 0 writes s_memtime at kernel entry, K-loop entry, K-loop
// exit and kernel exit to the u64 buffer passed in desc.out2 (4 per workgroup); out2 is not stored.
template <int BCO, int STAGES, int ACT, bool RES, bool STAMP = false, int NOLOAD = 0, bool CM = false>
__global__ void __launch_bounds__(256, 1) conv_wide_kernel(ConvArgs a) {
  unsigned long long st0 = 0, st1 = 0, st2 = 0;
  if constexpr (STAMP) st0 = wstamp();
  constexpr int BPX = 256;
  constexpr int TM = BCO / 32;        // A (Cout) fragments per wave
  constexpr int TN = 8;               // B (pixel) fragments per wave
  constexpr int GA = TM / 4;          // A fragments per MFMA group
  constexpr int NAI = BCO / 64;       // weight DMA instructions per wave per stage
  constexpr int NBI = BPX / 64;       // activation DMA instructions per wave per stage
  constexpr int NL = NAI + NBI;
  constexpr int STAGE_BYTES = (BCO + BPX) * 64;
  static_assert(GA >= 1 && TM % 4 == 0, "tile");
  static_assert(STAGES == 4 || STAGES == 5, "ring depth: STAGES - 2 stages in flight");
  static_assert(NL <= 8, "DMA slots: 2 in group 3, 2 per group 0..2");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  const hiseg_conv2d_desc& d = a.d;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wco = w >> 1, wpx = w & 1;

  // ---- XCD-major bijective remap, Cout tiles fastest (neighbouring pixel tiles share a halo)
  const int nco = d.Cout_pad / BCO;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int q = nwg >> 3, r8 = nwg & 7, xcd = orig & 7, loc = orig >> 3;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + loc;
  const int co0 = (wg % nco) * BCO;
  const int px0 = (wg / nco) * BPX;

  // ---- per-lane DMA state: instruction i of wave w fills rows 16*(w + 4i) + lane/4, slot lane%4
  const int lrow = lane >> 2, slot = lane & 3;
  unsigned woff[NAI];
#pragma unroll
  for (int i = 0; i < NAI; ++i) {
    const int r = 16 * (w + 4 * i) + lrow;
    woff[i] = ((unsigned)(co0 + r) * (unsigned)d.K_pad + (unsigned)((slot ^ wswz(r)) * 8)) * 2u;
  }
  // activation rows: input tap origin (piy, pix), pixel index of tap (0,0) and the lane's swizzled chunk
  int piy[NBI], pix[NBI], pidx[NBI], pch[NBI];
#pragma unroll
  for (int i = 0; i < NBI; ++i) {
    const int r = 16 * (w + 4 * i) + lrow;
    const int m = px0 + r;
    pch[i] = (slot ^ wswz(r)) * 8;
    pidx[i] = 0;
    if (m < a.M) {
      const int ox = m % d.Wo;
      const int tt = m / d.Wo;
      const int oy = tt % d.Ho;
      const int n = tt / d.Ho;
      piy[i] = oy * d.stride - d.pad;
      pix[i] = ox * d.stride - d.pad;
      pidx[i] = (n * d.H + piy[i]) * d.W + pix[i];
    } else {
      piy[i] = -(1 << 28); pix[i] = 0;  // never in bounds
    }
  }
  // every buffer descriptor covers exactly its tensor: an offset past it reads zeros instead of faulting
  const int nrec_w = d.Cout_pad * d.K_pad * 2;
  const int nrec_a = d.N * d.H * d.W * d.a_cstride * 2;
  const int nrec_b = d.Cb ? d.N * d.H * d.W * d.b_cstride * 2 : nrec_a;
  const int nrec_r = RES ? a.M * d.r_cstride * 2 : 0;
  const unsigned OOB = 0x80000000u;  // >= num_records: the DMA returns zeros
  const int nS = d.K_pad >> 5;
  const unsigned lds_base = (unsigned)(uintptr_t)(lds_void_w*)smem;

  // ---- the stage to be issued next (tap-major K order of the packed weights), advanced without division
  int n_ci = 0, n_kx = 0, n_ky = 0;
  // Residual prefetch (PREF, BCO = 256): the epilogue stages the output tile as 256 pixel rows x 512 B, row r
  // in ring buffer (nS + r / 64) % 4 -- so the "stages" past the end (s = nS + q, q = 0..2, whose buffers are
  // free) are quarters q of the residual tile (rows 64q .. 64q + 63, 2 rows x 512 B per wave instruction),
  // loaded under the last K stages; quarter 3 follows the loop into the last stage's buffer.
  constexpr bool PREF = RES && BCO == 256;
  constexpr int EROWB = BCO * 2;                 // epilogue tile row bytes
  const unsigned r_qinc = (unsigned)(64 * d.r_cstride * 2);
  const unsigned m_left = (unsigned)(a.M - px0);
  // residual quarter q of slot k: lane offset (OOB past the last pixel) -- computed where needed (the tail),
  // so nothing of it stays live through the main loop
  auto res_voff = [&](int k, int q) __attribute__((always_inline)) -> unsigned {
    const int row = 2 * (w + 4 * k) + (lane >> 5);
    const int c = lane & 31;
    const unsigned base = (unsigned)(((px0 + row) * d.r_cstride + d.r_coff + co0 + ((c ^ (row & 15)) * 8)) * 2);
    return (unsigned)(row + 64 * q) < m_left ? base + (unsigned)q * r_qinc : OOB;
  };
  // pending stage: per-slot LDS destinations, buffer descriptors (slots < NAI / >= NAI) and lane offsets
  unsigned p_sbase = lds_base, p_voff[NL];
  // buffer bases of the slots < NAI / >= NAI, kept as wave-uniform 64-bit values (a descriptor carried
  // through the loop's control flow may be given vector registers, which buffer_load cannot take)
  unsigned long long p_baseA = (unsigned long long)d.weight, p_baseB = (unsigned long long)d.weight;
  int p_numA = nrec_w, p_numB = nrec_w;
  auto uni = [](const void* ptr) __attribute__((always_inline)) -> unsigned long long {
    const unsigned long long v = (unsigned long long)ptr;
    return ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32)) << 32) |
           (unsigned)__builtin_amdgcn_readfirstlane((unsigned)v);
  };
#pragma unroll
  for (int k = 0; k < NL; ++k) p_voff[k] = OOB;
  // prepare_live: stage s < nS (branch-free, so that its scalar/vector work can interleave with the MFMAs
  // around it); prepare_dead: a stage past the end -- residual quarter s - nS (PREF) or a DMA set that reads
  // nothing (every offset out of range).
  // Slot k of wave w always fills the 1 KiB at p_sbase + 1024 (w + 4k): rows 16 (w + 4k) of the stage's
  // [weights; activations] 64-B row image, or rows 2 (w + 4k) of a 512-B residual row image.
  auto prepare_live = [&](int s) __attribute__((always_inline)) {   // s = stage index of (n_ci, n_kx, n_ky)
    p_sbase = lds_base + (unsigned)((s % STAGES) * STAGE_BYTES);
    const bool fromA = n_ci < d.Ca;
    const void* src = fromA ? d.srcA : d.srcB;
    const int cs = fromA ? d.a_cstride : d.b_cstride;
    const int cbase = fromA ? d.a_coff + n_ci : d.b_coff + n_ci - d.Ca;
    const int dpix = n_ky * d.W + n_kx;
    const unsigned kofs = (unsigned)((n_ky * d.KW + n_kx) * a.Cin + n_ci) * 2u;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      if (k < NAI) {
        p_voff[k] = woff[k < NAI ? k : 0] + kofs;
      } else {
        const int i = k >= NAI ? k - NAI : 0;
        const int iy = piy[i] + n_ky, ix = pix[i] + n_kx;
        const bool ok = (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
        p_voff[k] = ok ? (unsigned)((pidx[i] + dpix) * cs + cbase + pch[i]) * 2u : OOB;
        if constexpr (NOLOAD == 4) p_voff[k] &= 0xffffu;   // diagnostic: every activation read an L2 hit
      }
    }
    p_baseA = uni(d.weight);
    p_baseB = uni(src);
    p_numA = nrec_w;
    p_numB = fromA ? nrec_a : nrec_b;
    if constexpr (CM) {
      // channel-major K order: the taps of one 32-channel slice back to back (their shifted activation windows
      // stay L2-resident); accumulation order differs from the packed weights' tap-major order
      const int kx = n_kx + 1;
      const bool wrap_x = kx == d.KW;
      const int ky = n_ky + (wrap_x ? 1 : 0);
      const bool wrap_y = ky == d.KH;
      n_kx = wrap_x ? 0 : kx;
      n_ky = wrap_y ? 0 : ky;
      n_ci = n_ci + (wrap_y ? 32 : 0);
    } else {
      // advance to the next stage (tap-major K order of the packed weights)
      const int ci = n_ci + 32;
      const bool wrap_c = ci == a.Cin;
      const int kx = n_kx + (wrap_c ? 1 : 0);
      const bool wrap_x = kx == d.KW;
      n_ci = wrap_c ? 0 : ci;
      n_kx = wrap_x ? 0 : kx;
      n_ky = n_ky + (wrap_x ? 1 : 0);
    }
  };
  auto prepare_dead = [&](int s) __attribute__((always_inline)) {
    p_sbase = lds_base + (unsigned)((s % STAGES) * STAGE_BYTES);
    const int qd = s - nS;
#pragma unroll
    for (int k = 0; k < NL; ++k) p_voff[k] = PREF && qd < 4 ? res_voff(k, qd) : OOB;
    if constexpr (PREF) {
      p_baseA = uni(d.residual);
      p_baseB = p_baseA;
      p_numA = p_numB = nrec_r;
    }
  };
  auto prepare = [&](int s) __attribute__((always_inline)) {
    if (s < nS) prepare_live(s);
    else prepare_dead(s);
  };
  auto slot_dma = [&](auto kc) __attribute__((always_inline)) {   // DMA instruction k of the pending stage
    constexpr int k = decltype(kc)::value;
    // NOLOAD (timing diagnostics): 1 = no DMA in the K loop, 2 = no activation DMA, 3 = no weight DMA
    if constexpr (k < NL && NOLOAD != 1 && !(NOLOAD == 2 && k >= NAI) && !(NOLOAD == 3 && k < NAI)) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<void*>(k < NAI ? p_baseA : p_baseB), (short)0, k < NAI ? p_numA : p_numB, 0x00020000);
      dma16w(rs, p_sbase + (unsigned)(1024 * (w + 4 * k)), p_voff[k]);
    }
  };

  // fragment reads: row (16-aligned block base) + lane%16, chunk lane/16 at its swizzled slot
  const int lane_off = (lane & 15) * 64 + (((lane >> 4) ^ wswz(lane & 15)) << 4);
  const char* lds_c = reinterpret_cast<const char*>(smem);
  auto rdA = [&](int s, int i) __attribute__((always_inline)) {
    return *reinterpret_cast<const uint4*>(lds_c + (s % STAGES) * STAGE_BYTES + (wco * TM * 16 + i * 16) * 64 + lane_off);
  };
  auto rdB = [&](int s, int j) __attribute__((always_inline)) {
    return *reinterpret_cast<const uint4*>(lds_c + (s % STAGES) * STAGE_BYTES + (BCO + wpx * TN * 16 + j * 16) * 64 + lane_off);
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: stages 0 .. STAGES-3 issued whole, slots 0..1 of stage STAGES-2 (slots 2..7 go out under
  // the first stage's groups 0..2, as in every later stage); wait for stage 0
#pragma unroll
  for (int s = 0; s < STAGES - 2; ++s) {
    prepare(s);
    slot_dma(std::integral_constant<int, 0>{}); slot_dma(std::integral_constant<int, 1>{});
    slot_dma(std::integral_constant<int, 2>{}); slot_dma(std::integral_constant<int, 3>{});
    slot_dma(std::integral_constant<int, 4>{}); slot_dma(std::integral_constant<int, 5>{});
    slot_dma(std::integral_constant<int, 6>{}); slot_dma(std::integral_constant<int, 7>{});
  }
  prepare(STAGES - 2);
  slot_dma(std::integral_constant<int, 0>{}); slot_dma(std::integral_constant<int, 1>{});
  wvm<(STAGES - 3) * NL + 2>();   // stage 0 landed: the younger stages may stay in flight
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  uint4 af[TM], bf[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bf[j] = rdB(0, j);
#pragma unroll
  for (int i = 0; i < GA; ++i) af[i] = rdA(0, i);

  auto mfma = [&](int i, int j) __attribute__((always_inline)) {
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                         __builtin_bit_cast(bf16x8_t, bf[j]), acc[i][j], 0, 0, 0);
  };

  // One K stage s (uniform: stages past the end are DMA sets that read nothing, and the fragment reads of
  // "stage nS" in the last iteration are never consumed).  Groups 0..2: the next group's A fragments are
  // read ahead and DMA slots 2..7 of stage s+2 go out.  Hand-over: stage s+1 landed (stage s+2 may stay
  // in flight), barrier (every wave is done with stage s-1, whose buffer stage s+3 refills), stage s+3
  // prepared.  Group 3, column-major: B fragment j of stage s+1 is read as soon as column j is done, and
  // DMA slots 0..1 of stage s+3 go out.
  if constexpr (STAMP) st1 = wstamp();
  auto body = [&](int s, auto tailc) __attribute__((always_inline)) {
    constexpr bool TAIL = decltype(tailc)::value;
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int i = 0; i < GA; ++i) mfma(g * GA + i, j);
        if (j == 1) {
#pragma unroll
          for (int i = 0; i < GA; ++i) af[(g + 1) * GA + i] = rdA(s, (g + 1) * GA + i);
        }
      }
      __builtin_amdgcn_s_setprio(0);
      if (g == 0) { slot_dma(std::integral_constant<int, 2>{}); slot_dma(std::integral_constant<int, 3>{}); }
      if (g == 1) { slot_dma(std::integral_constant<int, 4>{}); slot_dma(std::integral_constant<int, 5>{}); }
      if (g == 2) { slot_dma(std::integral_constant<int, 6>{}); slot_dma(std::integral_constant<int, 7>{}); }
    }
    wvm<(STAGES - 3) * NL>();   // stage s+1 landed, stages s+2 .. s+STAGES-2 may stay in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (TAIL) prepare_dead(s + STAGES - 1);
    else prepare_live(s + STAGES - 1);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int i = 0; i < GA; ++i) mfma(3 * GA + i, j);
      bf[j] = rdB(s + 1, j);
      if (j == 1) {
#pragma unroll
        for (int i = 0; i < GA; ++i) af[i] = rdA(s + 1, i);
      }
      if (j == 3) slot_dma(std::integral_constant<int, 0>{});
      if (j == 5) slot_dma(std::integral_constant<int, 1>{});
    }
    __builtin_amdgcn_s_setprio(0);
  };
  // the main loop prepares live stages only; the last three stages (straight-line code, so that the
  // accumulators keep their registers) prepare the stages past the end
  for (int s = 0; s < nS - (STAGES - 1); ++s) body(s, std::false_type{});
#pragma unroll
  for (int q = STAGES - 1; q >= 1; --q) body(nS - q, std::true_type{});
  // the last prepared stage's slots 2..7 (a residual quarter under PREF, else an empty set)
  slot_dma(std::integral_constant<int, 2>{}); slot_dma(std::integral_constant<int, 3>{});
  slot_dma(std::integral_constant<int, 4>{}); slot_dma(std::integral_constant<int, 5>{});
  slot_dma(std::integral_constant<int, 6>{}); slot_dma(std::integral_constant<int, 7>{});
  if constexpr (!PREF) wvm<0>();   // the tail's empty DMA sets have landed (PREF: waited for below)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if constexpr (STAMP) st2 = wstamp();

  // ---- epilogue through LDS.  The output tile is staged as 256 pixel rows x BCO bf16 (EROWB bytes), 16-B
  // chunk c of row r at slot c ^ (r & 15); with PREF row r lives in ring buffer (nS + r / 64) % 4, else rows
  // are contiguous from the LDS base.  The residual tile arrives there by LDS-DMA (whole rows, 16 B per lane;
  // PREF: quarters 0..2 already under the last K stages), each lane turns its accumulator quads into bf16
  // output quads in place (ds_read_b64 / ds_write_b64, conflict-free: the 16 rows of a fragment hit 16
  // distinct slots), and whole rows leave by 16-B stores.  Same arithmetic and rounding as the register
  // epilogue: v = acc*scale + shift (+ residual), act, one f32 -> bf16 rounding.
  constexpr int CPR = BCO / 8;                 // 16-B chunks per row
  constexpr int RPI = 64 / CPR;                // rows per wave instruction
  char* tile = reinterpret_cast<char*>(smem);
  auto row_base = [&](int r) __attribute__((always_inline)) -> int {
    if constexpr (PREF) return ((nS + (r >> 6)) % STAGES) * STAGE_BYTES + (r & 63) * EROWB;
    else return r * EROWB;
  };
  const __amdgpu_buffer_rsrc_t rR = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(RES ? d.residual : d.out), (short)0, RES ? nrec_r : 0, 0x00020000);
  if constexpr (PREF && STAGES == 4) {
    // quarter 3 into the last stage's buffer (every wave is past its reads: the barrier above)
#pragma unroll
    for (int k = 0; k < NL; ++k)
      dma16w(rR, lds_base + (unsigned)(((nS + 3) % STAGES) * STAGE_BYTES + 2 * (w + 4 * k) * EROWB), res_voff(k, 3));
    wvm<NL>();   // quarters 0..2 landed (own DMAs)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  } else if constexpr (PREF) {
    wvm<0>();    // every quarter was issued under the last K stages
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  } else if constexpr (RES) {
    constexpr int NRI = BPX / (RPI * 4);         // residual DMA instructions per wave
    const int c = lane % CPR;
#pragma unroll
    for (int k = 0; k < NRI; ++k) {
      const int r = RPI * (w + 4 * k) + lane / CPR;
      const int px = px0 + r;
      const unsigned off = px < a.M ? (unsigned)((px * d.r_cstride + d.r_coff + co0 + ((c ^ (r & 15)) * 8)) * 2) : OOB;
      dma16w(rR, lds_base + (unsigned)(row_base(RPI * (w + 4 * k))), off);
    }
    wvm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  floatx4 sc[TM], sh[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int cl = wco * TM * 16 + i * 16 + (lane >> 4) * 4;
    const int cc = co0 + cl < d.Cout ? co0 + cl : 0;
    sc[i] = *reinterpret_cast<const floatx4*>(d.scale + cc);
    sh[i] = *reinterpret_cast<const floatx4*>(d.shift + cc);
  }
  auto epi_frag = [&](int i, int j) __attribute__((always_inline)) {
    const int cl = wco * TM * 16 + i * 16 + (lane >> 4) * 4;   // channel within the tile
    const int r = wpx * TN * 16 + j * 16 + (lane & 15);
    char* q = tile + row_base(r) + ((((cl >> 3) ^ (r & 15)) << 4) | ((cl & 4) << 1));
    const floatx4 ac = acc[i][j];
    float v[4];
    uint2 rv = make_uint2(0u, 0u);
    if constexpr (RES) rv = *reinterpret_cast<const uint2*>(q);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = ac[e] * sc[i][e] + sh[i][e];
      if constexpr (RES) v[e] += Quad<bf16_t>::get(rv, e);
      if constexpr (ACT == HISEG_ACT_RELU) v[e] = v[e] > 0.f ? v[e] : 0.f;
    }
    uint2 o;
    o.x = f2bf2(v[0], v[1]);
    o.y = f2bf2(v[2], v[3]);
    *reinterpret_cast<uint2*>(q) = o;
  };
  // rows of quarter 3 (pixel half wpx = 1, fragments j >= 4) wait for the post-loop quarter
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      if (!(PREF && STAGES == 4) || wpx == 0 || j < 4) epi_frag(i, j);
  if constexpr (PREF && STAGES == 4) {
    wvm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (wpx == 1) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 4; j < TN; ++j) epi_frag(i, j);
    }
  }
  __syncthreads();
  constexpr int NST = BPX * CPR / 256;          // 16-B output chunks per thread
#pragma unroll 4
  for (int k = 0; k < NST; ++k) {
    const int idx = t + 256 * k;
    const int r = idx / CPR, c = idx % CPR;
    const int px = px0 + r, co = co0 + 8 * c;
    const uint4 v = *reinterpret_cast<const uint4*>(tile + row_base(r) + ((c ^ (r & 15)) << 4));
    if (px < a.M && co < d.Cout)
      *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(d.out) + (long long)px * d.o_cstride + d.o_coff + co) = v;
  }
  if constexpr (STAMP) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long st3 = wstamp();
    if (t == 0) {
      unsigned long long* sb = reinterpret_cast<unsigned long long*>(a.d.out2) + 4 * blockIdx.x;
      sb[0] = st0; sb[1] = st1; sb[2] = st2; sb[3] = st3;
    }
  }
}

template <int BCO, bool STAMP = false, int NOLOAD = 0, bool CM = false, int STAGES = 4>
static int launch_wide(const ConvArgs& a, hipStream_t s) {
  const int npx = (a.M + 255) / 256;
  const int nco = a.d.Cout_pad / BCO;
  const size_t lds = (size_t)STAGES * (BCO + 256) * 64;
  const bool res = a.d.residual != nullptr;
  const int act = a.d.act;
  auto kern = res ? (act == HISEG_ACT_RELU ? conv_wide_kernel<BCO, STAGES, HISEG_ACT_RELU, true, STAMP, NOLOAD, CM>
                                           : conv_wide_kernel<BCO, STAGES, HISEG_ACT_NONE, true, STAMP, NOLOAD, CM>)
                  : (act == HISEG_ACT_RELU ? conv_wide_kernel<BCO, STAGES, HISEG_ACT_RELU, false, STAMP, NOLOAD, CM>
                                           : conv_wide_kernel<BCO, STAGES, HISEG_ACT_NONE, false, STAMP, NOLOAD, CM>);
  static bool attr_set[2][2] = {};   // once per instantiation (no API call but the launch per layer: capturable)
  bool& done = attr_set[res ? 1 : 0][act == HISEG_ACT_RELU ? 1 : 0];
  if (!done) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    done = true;
  }
  hipLaunchKernelGGL(kern, dim3(npx * nco), dim3(256), lds, s, a);
  return hiseg_check_launch("conv_wide");
}

// Automatic BCO-256 configuration: 70 = tap-major K order (bit-identical to the generic kernel), 74 =
// channel-major K order (the 9 taps of a 32-channel slice back to back: 0.42x the L2 fetch of 70).
#ifndef HISEG_WIDE_AUTO
#define HISEG_WIDE_AUTO 70
#endif

// Returns 1 if launched, 0 if the layer does not qualify (caller falls back), <0 on error.
// variant 0 = automatic (BCO 256 when 256 | Cout_pad, else 128), 70 = BCO 256, 72 = BCO 128.
int conv_wide_try(const ConvArgs& a, hipStream_t s, int variant) {
  const hiseg_conv2d_desc& d = a.d;
  if (d.dtype != HISEG_BF16 || d.out_dtype != HISEG_BF16) return 0;
  if (d.a_up != 1 || d.in_scale != nullptr || d.convT || d.mul != nullptr || (d.out2 != nullptr && !(HISEG_DIAG_ON && variant == 79))) return 0;
  if (d.act != HISEG_ACT_NONE && d.act != HISEG_ACT_RELU) return 0;
  if (d.Ca % 64 != 0 || d.Cb % 64 != 0) return 0;
  if (d.K_pad != d.KH * d.KW * a.Cin || d.K_pad < 128) return 0;   // >= 4 K stages (the pipeline's depth)
  if (((d.a_cstride | d.a_coff) & 7) || (d.Cb && ((d.b_cstride | d.b_coff) & 7))) return 0;
  // LDS epilogue: whole 16-B chunks of whole BCO-channel tiles (Cout a multiple of the tile: the residual
  // DMA reads BCO channels per row), 16-B aligned views and scale/shift
  if ((d.Cout & 127) || ((d.o_cstride | d.o_coff) & 7) || (d.residual && ((d.r_cstride | d.r_coff) & 7))) return 0;
  if ((((uintptr_t)d.scale | (uintptr_t)d.shift | (uintptr_t)d.out | (uintptr_t)d.residual) & 15)) return 0;
  // 32-bit byte offsets for the buffer descriptors
  const long long span_a = (long long)d.N * d.H * d.W * d.a_cstride * 2;
  const long long span_b = d.Cb ? (long long)d.N * d.H * d.W * d.b_cstride * 2 : 0;
  const long long span_w = (long long)d.Cout_pad * d.K_pad * 2;
  const long long span_r = d.residual ? (long long)a.M * d.r_cstride * 2 : 0;
  if (span_a >= 0x7fffffffll || span_b >= 0x7fffffffll || span_w >= 0x7fffffffll || span_r >= 0x7fffffffll) return 0;
  if (variant == 0) variant = (d.Cout % 256 == 0) ? HISEG_WIDE_AUTO : 72;
  int r;
  switch (variant) {
    case 70: if (d.Cout % 256) return 0; r = launch_wide<256>(a, s); break;
    case 72: r = launch_wide<128>(a, s); break;
#ifdef HISEG_DIAG
    // timing-only diagnostics (wrong outputs): 77 no K-loop DMA, 75 no activation DMA, 76 no weight DMA, 73 every
    // activation read an L2 hit; 79 per-workgroup s_memtime stamps into desc.out2
    case 77: if (d.Cout % 256) return 0; r = launch_wide<256, false, 1>(a, s); break;
    case 75: if (d.Cout % 256) return 0; r = launch_wide<256, false, 2>(a, s); break;
    case 76: if (d.Cout % 256) return 0; r = launch_wide<256, false, 3>(a, s); break;
    case 73: if (d.Cout % 256) return 0; r = launch_wide<256, false, 4>(a, s); break;
    case 79:
      HISEG_REQUIRE(d.out2 != nullptr, HISEG_ERR_BAD_ARG, "conv_wide: stamp variant needs desc.out2");
      if (d.Cout % 256) return 0;
      r = launch_wide<256, true>(a, s);
      break;
#endif
    case 74: if (d.Cout % 256) return 0; r = launch_wide<256, false, 0, true>(a, s); break;   // channel-major K
    case 71: if (d.Cout % 256) return 0; r = launch_wide<256, false, 0, false, 5>(a, s); break;   // 5-deep ring
    default: return 0;
  }
  return r < 0 ? r : 1;
}

}  // namespace hiseg
