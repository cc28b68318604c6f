// Row-streaming direct 3x3 convolution for the full-image UNet's narrow decoder layers (bf16 in, gfx950).
//
// The smp decoder's last two blocks and the segmentation head (smp Unet DecoderBlock conv1/conv2 + head,
// unet.py:1770-1774 via smp) run at 1/2 and full image resolution with 16-32 output channels: ~13 GFLOP per
// 32-image step but ~0.4 GB of activations per layer, so they are HBM-bound, not MFMA-bound.  conv_small (the
// halo-tiled kernel) stages the whole weight matrix plus a (TH+2)-row halo per 4-8-row tile and then computes,
// with one workgroup per CU for the wide-K layers -- load and compute never overlap, and the 2 halo rows are
// re-read per tile (profiles/r2_v8_pmc_hbm_unet.txt: 894 GB/s on the 96->32 layer).
//
// Here a workgroup (8 waves) owns a contiguous run of output rows of one or more TW-pixel column strips and
// streams the input down the strip:
//   * weights live in registers for the whole launch, in MFMA A-fragment order: wave w owns Cout block
//     w % NCB and one 16-pixel group, so it needs all NKC k-steps of one 16-row weight block (<= 36 x 4 VGPRs);
//   * input rows (TW+2 pixels x Cin channels) go HBM -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds) into a
//     ring of P+3 rows, streamed P rows ahead of the row being computed: one counted vmcnt + barrier per
//     output row; out-of-image pixels get an out-of-range offset, so the DMA writes zeros;
//   * ring row layout: blocks of 8 pixels of one 16-B channel chunk, slot ((pix / 8) * CH + c) * 8 + pix % 8 --
//     one 64-lane DMA covers 8 pixels x 8 chunks (8 x 128 contiguous bytes in HBM), and a B fragment (lane:
//     pixel lr, chunk lg) meets 16 distinct 4-bank groups in every ds_read_b128 lane group;
//   * each row of the input is read from HBM once per strip (the halo re-read is 2 rows per run of ~48),
//     src A nearest-upsampled x2 on the fly and the skip (src B) concatenated in the K order;
//   * every wave issues exactly NJ DMAs (spares fill a sink slot) and one store (dead lanes and halo steps
//     write a sink buffer) per row, both as inline asm, so the vmcnt count that leaves the next P-1 rows in
//     flight is a constant: (P-1) * (NJ + 1).
// Per output row, a wave issues NKC v_mfma_f32_16x16x32_bf16 over K in conv_small's / the generic kernel's
// order (tap-major, 32-deep chunks: k = tap*Cin + ci), reading one kernel row's B fragments ahead of its
// MFMAs, and applies the same lite epilogue (folded BN, act, store4): results are bit-identical to
// conv_small_kernel.
#include "conv_common.h"

namespace hiseg {

template <int CH, int TW>
struct RowsGeom {
  static constexpr int CIN = CH * 8;
  static constexpr int NKC = (9 * CIN + 31) / 32;
  static constexpr int HP = TW + 2;                            // halo'd row (pixels)
  static constexpr int NSLOT = (HP + 7) / 8 * 8 * CH;          // 16-B slots holding the row
  static constexpr int ROWS = (NSLOT + 63) / 64 * 64;          // slots per ring row (whole DMA instructions)
  static constexpr int NDMA = ROWS / 64;                       // DMA instructions per row
  static constexpr int NJ = (NDMA + 7) / 8;                    // ... per wave (8 waves)
};

__device__ __forceinline__ void rows_dma16(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, unsigned voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(lds_addr), "v"(voff), "s"(rsrc) : "memory");
}

// Two-resource form (sources far apart): the lanes of source A load through rsrc_a, those of source B through
// rsrc_b, into the same LDS slots -- two instructions under complementary exec masks (both non-empty: mixed groups
// only; the caller handles single-source groups), exec restored inside the asm block.
__device__ __forceinline__ void rows_dma16_ab(__amdgpu_buffer_rsrc_t rsrc_a, __amdgpu_buffer_rsrc_t rsrc_b,
                                              unsigned lds_addr, unsigned voff, unsigned long long mask_a,
                                              unsigned long long mask_b) {
  unsigned long long saved;
  asm volatile("s_mov_b32 m0, %[lds]\n\t"
               "s_and_saveexec_b64 %[sv], %[ma]\n\t"
               "s_nop 0\n\t"
               "buffer_load_dwordx4 %[off], %[ra], 0 offen lds\n\t"
               "s_mov_b64 exec, %[sv]\n\t"
               "s_and_b64 exec, exec, %[mb]\n\t"
               "s_nop 0\n\t"
               "buffer_load_dwordx4 %[off], %[rb], 0 offen lds\n\t"
               "s_mov_b64 exec, %[sv]"
               : [sv] "=&s"(saved)
               : [lds] "s"(lds_addr), [off] "v"(voff), [ra] "s"(rsrc_a), [rb] "s"(rsrc_b), [ma] "s"(mask_a),
                 [mb] "s"(mask_b)
               : "memory", "scc");
}

__device__ uint4 g_conv_rows_sink[64];            // the stores of dead lanes / halo steps (never read)

template <typename TO>
__device__ __forceinline__ void rows_store(void* p, const float (&v)[4], bool vec4) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  if constexpr (sizeof(TO) == 2) {
    const u32x2 q = {f2bf2(v[0], v[1]), f2bf2(v[2], v[3])};
    asm volatile("global_store_dwordx2 %0, %1, off" :: "v"(p), "v"(q) : "memory");
  } else if (vec4) {
    const floatx4 q = {v[0], v[1], v[2], v[3]};
    asm volatile("global_store_dwordx4 %0, %1, off" :: "v"(p), "v"(q) : "memory");
  } else {
    asm volatile("global_store_dword %0, %1, off" :: "v"(p), "v"(v[0]) : "memory");
  }
}

// CH: input channels / 8.  NCB: 16-channel output blocks (1 or 2; TW = 128 / NCB pixels per strip).
// P (even): rows in flight ahead of the computed pair.  OCC: workgroups per CU the launch bounds allow.
// Output forms: bf16 with Cout % 4 == 0, f32 with Cout % 4 == 0 (vec4) or Cout == 1 (the head).
// TWO: the concat's two sources through one buffer resource each (their allocations lie too far apart for one
// 32-bit offset range): every DMA group becomes two counted instructions (same slots, same arithmetic after).
template <int CH, int NCB, typename TO, int P, int OCC, int ACT, bool TWO>
__global__ void __launch_bounds__(512, 2 * OCC) conv_rows_kernel(ConvArgs a, int nstrip, long long ntask, int nwg,
                                                                 unsigned dA, unsigned dB) {
  constexpr int TW = 128 / NCB;
  using G = RowsGeom<CH, TW>;
  constexpr int CIN = G::CIN, NKC = G::NKC, HP = G::HP, ROWS = G::ROWS, NDMA = G::NDMA, NJ = G::NJ;
  constexpr int RB = P + 4;
  constexpr int WAIT = (P / 2 - 1) * 2 * ((TWO ? 2 : 1) * NJ + 1);
  static_assert(P % 2 == 0 && WAIT <= 63, "P even; vmcnt field");
  extern __shared__ __attribute__((aligned(16))) uint4 ring[];   // RB rows, then a 64-slot DMA sink
  // descriptor fields as scalars (a reference into the kernel arguments inside the lambdas below would be
  // read through a flat pointer: a per-lane load and vmcnt(0) per use)
  const int H = a.d.H, W = a.d.W, Hs = a.Hs, Ws = a.Ws;
  const int Ca = a.d.Ca, acs = a.d.a_cstride, aco = a.d.a_coff, bcs = a.d.b_cstride, bco = a.d.b_coff;
  const int Cout = a.d.Cout, ocs = a.d.o_cstride, oco = a.d.o_coff;
  char* const out = reinterpret_cast<char*>(a.d.out);
  const int t = threadIdx.x;
  const int lane = t & 63, lr = lane & 15, lg = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int cb = w % NCB, pg = w / NCB;

  // this workgroup's output rows: tasks [t0, t1) of (image, strip, row), row fastest
  const long long t0 = ntask * blockIdx.x / nwg, t1 = ntask * (blockIdx.x + 1) / nwg;
  if (t1 <= t0) return;
  const long long q0 = t0 / H;                 // first strip (image * nstrip + strip)
  const int y0 = (int)(t0 - q0 * H);
  const int L0 = (int)((t1 - t0 < H - y0) ? t1 - t0 : H - y0) + 2;   // stream rows of the first segment
  const long long rest = (t1 - t0) - (L0 - 2);
  const int nfull = (int)(rest / H), rem = (int)(rest - (long long)nfull * H);
  const int S = L0 + nfull * (H + 2) + (rem ? rem + 2 : 0);          // stream length (input rows)
  // Stream cursor (wave-uniform, advanced one position per step: no divisions in the loop): strip (n, sx),
  // input row r, first output row ys and last input row rlast of the current segment, segment index si.
  struct Cursor {
    int n, sx, r, ys, rlast, si;
  };
  auto cursor_at0 = [&]() {
    Cursor c;
    c.n = (int)(q0 / nstrip);
    c.sx = (int)(q0 - (long long)c.n * nstrip);
    c.r = y0 - 1; c.ys = y0; c.rlast = y0 + L0 - 2; c.si = 0;
    return c;
  };
  auto advance = [&](Cursor& c) {
    if (c.r < c.rlast) { ++c.r; return; }
    ++c.si;
    if (++c.sx == nstrip) { c.sx = 0; ++c.n; }
    c.r = -1; c.ys = 0;
    c.rlast = c.si <= nfull ? H : rem;
  };

  // weights -> registers (A fragments: row co = cb*16 + lr, k = 32*kc + 8*lg .. +8)
  uint4 wr[NKC];
  {
    const uint16_t* wp = reinterpret_cast<const uint16_t*>(a.d.weight) + (long long)(cb * 16 + lr) * a.d.K_pad + lg * 8;
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) wr[kc] = *reinterpret_cast<const uint4*>(wp + kc * 32);
  }
  const int co4 = cb * 16 + lg * 4;
  const floatx4 sc = *reinterpret_cast<const floatx4*>(a.d.scale + co4);
  const floatx4 sh = *reinterpret_cast<const floatx4*>(a.d.shift + co4);
  // consume the weights and the affine here, so the compiler's waits for their loads sit before the loop (the
  // loop's own memory traffic is inline asm the compiler does not count)
#pragma unroll
  for (int kc = 0; kc < NKC; ++kc) asm volatile("" :: "v"(wr[kc].x));
  asm volatile("" :: "v"(sc[0]), "v"(sh[0]));
  const int esz = sizeof(TO);
  const bool vec4 = sizeof(TO) == 2 || Cout != 1;
  char* const sink = reinterpret_cast<char*>(g_conv_rows_sink) + 16 * lane;

  // DMA: instruction j = w + 8 i of a row fills slots 64 j .. 64 j + 63; this lane's slot 64 j + lane holds
  // chunk c of pixel pix (or nothing: past the row -> an out-of-range offset, the DMA writes zeros).  Every wave
  // issues NJ per row; j >= NDMA goes to the sink slots.
  const char* const base = TWO ? reinterpret_cast<const char*>(a.d.srcA)
                               : reinterpret_cast<const char*>(a.d.Cb && a.d.srcB < a.d.srcA ? a.d.srcB : a.d.srcA);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0,
                                                                        0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsrc_b = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(TWO ? a.d.srcB : a.d.srcA), (short)0, 0x7fffffff, 0x00020000);
  const unsigned OOB = 0x80000000u;
  const int up = a.d.a_up == 2 ? 1 : 0;
  int jpix[NJ], jcoff[NJ];
  bool jA[NJ];
  unsigned jcol[NJ];                           // per strip: byte offset of this lane's chunk within its row
  bool jok[NJ];                                // per strip: the lane's pixel lies in the image
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    const int slot = 64 * (w + 8 * i) + lane;
    const int blk = slot >> 3, c = blk % CH;
    const int pix = (blk / CH) * 8 + (slot & 7);
    const int ci = c * 8;
    jA[i] = ci < Ca;
    jcoff[i] = jA[i] ? aco + ci : bco + (ci - Ca);
    jpix[i] = (slot < G::NSLOT && pix < HP && w + 8 * i < NDMA) ? pix : -(1 << 20);
  }
  // TWO: per DMA group, the lanes reading source A / B (wave-uniform masks)
  unsigned long long mA[NJ], mB[NJ];
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    mA[i] = TWO ? __builtin_amdgcn_ballot_w64(jA[i]) : ~0ull;
    mB[i] = TWO ? ~mA[i] : 0ull;
  }
  const unsigned lds_base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)ring;
  const unsigned lds_sink = lds_base + 16u * (unsigned)(RB * ROWS);
  int col_sx = -1;                             // the strip jcol / jok were computed for
  auto set_strip = [&](int sx) {
    col_sx = sx;
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
      const int ix = sx * TW - 1 + jpix[i];
      jok[i] = ix >= 0 && ix < W;
      jcol[i] = jA[i] ? dA + 2u * (unsigned)((ix >> up) * acs + jcoff[i]) : dB + 2u * (unsigned)(ix * bcs + jcoff[i]);
    }
  };
  auto issue_row = [&](const Cursor& c, bool live, int slot) {   // DMA of one input row (sink-only if !live)
    if (c.sx != col_sx) set_strip(c.sx);       // (wave-uniform; once per segment)
    const bool rok = live && c.r >= 0 && c.r < H;
    const unsigned rowA = 2u * (unsigned)(((c.n * Hs + (c.r >> up)) * Ws) * acs);
    const unsigned rowB = 2u * (unsigned)(((c.n * H + c.r) * W) * bcs);
    const unsigned slotb = lds_base + 16u * (unsigned)(slot * ROWS);
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
      const unsigned off = rok && jok[i] ? jcol[i] + (jA[i] ? rowA : rowB) : OOB;
      const bool real = live && w + 8 * i < NDMA;  // (wave-uniform)
      const unsigned dst = real ? slotb + 1024u * (unsigned)(w + 8 * i) : lds_sink;
      if constexpr (TWO) {                     // exactly two counted instructions per group, whatever its sources
        if (mB[i] == 0ull) {
          rows_dma16(rsrc, dst, off);
          rows_dma16(rsrc, lds_sink, OOB);
        } else if (mA[i] == 0ull) {
          rows_dma16(rsrc_b, dst, off);
          rows_dma16(rsrc, lds_sink, OOB);
        } else {
          rows_dma16_ab(rsrc, rsrc_b, dst, off, mA[i], mB[i]);
        }
      } else {
        rows_dma16(rsrc, dst, off);
      }
    }
  };

  // B fragment slot offsets of this lane: pixel pg*16 + lr + dx, chunk lg (CIN % 32 == 0; the k-step's chunk
  // base is added per instruction) or lg & 1 (CIN == 16)
  int bofs[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    const int pix = pg * 16 + lr + dx;
    const int c = CIN % 32 == 0 ? lg : (lg & 1);
    bofs[dx] = (((pix >> 3) * CH + c) << 3) + (pix & 7);
  }

  // Each step computes the output rows of two stream positions p, p+1 (input rows p-2 .. p+1): four kernel-row
  // fragment groups, the middle two shared by both rows, two independent MFMA chains -- each in its own kc order,
  // so bit-identical to the one-row-at-a-time order.  The pair is stored one step later (before that step's
  // DMA): two stores per wave per step.
  float resA[4] = {0.f, 0.f, 0.f, 0.f}, resB[4] = {0.f, 0.f, 0.f, 0.f};
  char* dstA = sink;
  char* dstB = sink;
  auto store2 = [&]() { rows_store<TO>(dstA, resA, vec4); rows_store<TO>(dstB, resB, vec4); };

  // prologue: positions 0 .. P-1, two per pseudo-step after two (sink) stores, as in every step
  Cursor cd = cursor_at0();                    // the DMA cursor runs P positions ahead of the compute cursor
  Cursor cc = cd;
  int sd = 0;                                  // ring row of the DMA cursor's position
  auto issue_next = [&](int pos) {
    issue_row(cd, pos < S, sd);
    if (pos + 1 < S) advance(cd);
    sd = sd + 1 == RB ? 0 : sd + 1;
  };
#pragma unroll
  for (int p = 0; p < P; p += 2) { store2(); issue_next(p); issue_next(p + 1); }
  int s0 = RB - 2, s1 = RB - 1, s2 = 0, s3 = 1; // ring rows of positions p-2, p-1, p, p+1
  for (int p = 0; p < S; p += 2) {
    // positions p, p+1 landed (the rows issued in the P/2 - 1 later steps, with their stores, may stay in
    // flight), every wave done with step p-2's fragment reads
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "n"(WAIT) : "memory");
    store2();                                  // the previous pair
    issue_next(p + P);                         // over the ring rows of positions p-4, p-3
    issue_next(p + P + 1);
    Cursor cb2 = cc;
    if (p + 1 < S) advance(cb2);
    const int yA = cc.r - 1, yB = cb2.r - 1;  // position p holds input row yA+1
    const bool vA = yA >= cc.ys, vB = p + 1 < S && yB >= cb2.ys;   // else: halo rows of a segment / past the end
    dstA = sink;
    dstB = sink;
    if (vA || vB) {
      const int rowb[4] = {s0 * ROWS, s1 * ROWS, s2 * ROWS, s3 * ROWS};
      floatx4 accA = floatx4{0.f, 0.f, 0.f, 0.f}, accB = accA;
      auto mf = [&](floatx4& acc, int kc, const uint4& b) {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wr[kc]),
                                                      __builtin_bit_cast(bf16x8_t, b), acc, 0, 0, 0);
      };
      if constexpr (CIN % 32 == 0) {           // one tap per 32-deep chunk; fragments one kernel row ahead
        constexpr int CPT = CIN / 32, NG = 3 * CPT;
        uint4 g0[NG], g1[NG];
        auto load = [&](uint4 (&g)[NG], int rb) {
#pragma unroll
          for (int kx = 0; kx < 3; ++kx)
#pragma unroll
            for (int c = 0; c < CPT; ++c) g[kx * CPT + c] = ring[rb + bofs[kx] + c * 32];
        };
        load(g0, rowb[0]);
        load(g1, rowb[1]);
#pragma unroll
        for (int j = 0; j < NG; ++j) mf(accA, j, g0[j]);                       // A ky0
        load(g0, rowb[2]);
#pragma unroll
        for (int j = 0; j < NG; ++j) { mf(accA, NG + j, g1[j]); mf(accB, j, g1[j]); }   // A ky1, B ky0
        load(g1, rowb[3]);
#pragma unroll
        for (int j = 0; j < NG; ++j) { mf(accA, 2 * NG + j, g0[j]); mf(accB, NG + j, g0[j]); }   // A ky2, B ky1
#pragma unroll
        for (int j = 0; j < NG; ++j) mf(accB, 2 * NG + j, g1[j]);              // B ky2
      } else {                                 // CIN == 16: lanes 0-31 tap 2kc, lanes 32-63 tap 2kc+1
        const int h = lg >> 1;
        uint4 bA[NKC], bB[NKC];
#pragma unroll
        for (int kc = 0; kc < NKC; ++kc) {
          const int ta = 2 * kc, tb = 2 * kc + 1;
          const int offa = bofs[ta % 3], offb = tb < 9 ? bofs[tb % 3] : offa;
          const int ra = ta / 3, rbb = tb < 9 ? tb / 3 : ra;
          bA[kc] = ring[h ? rowb[rbb] + offb : rowb[ra] + offa];
          bB[kc] = ring[h ? rowb[rbb + 1] + offb : rowb[ra + 1] + offa];
          if (tb >= 9 && h) { bA[kc] = make_uint4(0u, 0u, 0u, 0u); bB[kc] = bA[kc]; }
        }
#pragma unroll
        for (int kc = 0; kc < NKC; ++kc) { mf(accA, kc, bA[kc]); mf(accB, kc, bB[kc]); }
      }
      const int oxA = cc.sx * TW + pg * 16 + lr, oxB = cb2.sx * TW + pg * 16 + lr;
#pragma unroll
      for (int e2 = 0; e2 < 4; ++e2) {
        resA[e2] = apply_act(accA[e2] * sc[e2] + sh[e2], ACT);
        resB[e2] = apply_act(accB[e2] * sc[e2] + sh[e2], ACT);
      }
      if (vA && oxA < W && co4 < Cout)
        dstA = out + ((long long)((cc.n * H + yA) * W + oxA) * ocs + oco + co4) * esz;
      if (vB && oxB < W && co4 < Cout)
        dstB = out + ((long long)((cb2.n * H + yB) * W + oxB) * ocs + oco + co4) * esz;
    }
    if (p + 2 < S) { cc = cb2; advance(cc); }
    s0 = s2; s1 = s3;
    s2 = s3 + 1 == RB ? 0 : s3 + 1;
    s3 = s2 + 1 == RB ? 0 : s2 + 1;
  }
  store2();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int CH, int NCB, typename TO, int P, int OCC, int ACT, bool TWO>
static int launch_rows_act(const ConvArgs& a, hipStream_t s, int rows_per_wg, unsigned dA, unsigned dB) {
  const hiseg_conv2d_desc& d = a.d;
  constexpr int TW = 128 / NCB;
  constexpr int LDS = ((P + 4) * RowsGeom<CH, TW>::ROWS + 64) * 16;
  static_assert(LDS <= (OCC == 1 ? 160 : 80) * 1024, "ring exceeds LDS");
  const size_t lds = LDS;
  const int nstrip = (d.W + TW - 1) / TW;
  const long long ntask = (long long)d.N * nstrip * d.H;
  // whole rounds of workgroup slots (CUs x OCC) of at most ~160 rows each: a partial last round cost up to a
  // quarter of the layer (tools/conv_bench.py, HISEG_ROWS_PER_WG sweep); small layers: >= 16 rows per workgroup
  long long nwg;
  if (rows_per_wg > 0) {
    nwg = (ntask + rows_per_wg - 1) / rows_per_wg;
  } else {
    static const int ncu = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
      return n;
    }();
    const long long slots = (long long)ncu * OCC;
    const long long rounds = (ntask + slots * 160 - 1) / (slots * 160);
    nwg = slots * rounds;
    const long long cap = (ntask + 15) / 16;
    if (nwg > cap) nwg = cap;
  }
  if (nwg > (1ll << 30)) nwg = 1ll << 30;
  auto kern = conv_rows_kernel<CH, NCB, TO, P, OCC, ACT, TWO>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(512), lds, s, a, nstrip, ntask, (int)nwg, dA, dB);
  const int r = hiseg_check_launch("conv_rows");
  return r < 0 ? r : 1;
}

template <int CH, int NCB, typename TO, int P, int OCC>
static int launch_rows(const ConvArgs& a, hipStream_t s, int rows_per_wg, unsigned dA, unsigned dB, bool two) {
  if (two)
    return a.d.act == HISEG_ACT_RELU ? launch_rows_act<CH, NCB, TO, P, OCC, HISEG_ACT_RELU, true>(a, s, rows_per_wg, dA, dB)
                                     : launch_rows_act<CH, NCB, TO, P, OCC, HISEG_ACT_NONE, true>(a, s, rows_per_wg, dA, dB);
  return a.d.act == HISEG_ACT_RELU ? launch_rows_act<CH, NCB, TO, P, OCC, HISEG_ACT_RELU, false>(a, s, rows_per_wg, dA, dB)
                                   : launch_rows_act<CH, NCB, TO, P, OCC, HISEG_ACT_NONE, false>(a, s, rows_per_wg, dA, dB);
}

template <typename TO>
static int dispatch_rows(const ConvArgs& a, hipStream_t s, int ch, int ncb, int rpw, unsigned dA, unsigned dB,
                         bool two) {
  if (ncb == 2) {
    switch (ch) {
      case 4: return launch_rows<4, 2, TO, 8, 2>(a, s, rpw, dA, dB, two);
      case 12: return launch_rows<12, 2, TO, 6, 1>(a, s, rpw, dA, dB, two);
      case 16: return launch_rows<16, 2, TO, 4, 1>(a, s, rpw, dA, dB, two);
      default: return 0;
    }
  }
  switch (ch) {
    case 2: return launch_rows<2, 1, TO, 8, 2>(a, s, rpw, dA, dB, two);
    case 4: return launch_rows<4, 1, TO, 4, 2>(a, s, rpw, dA, dB, two);
    default: return 0;
  }
}

// Returns 1 if launched, 0 if the layer does not qualify, <0 on error.  variant: 0 / 98 (the same kernel).
// The layer forms conv_rows computes, address constraints aside (conv2d_impl sends such a layer to conv_small when
// conv_rows declines it for its sources' placement only).
bool conv_rows_form(const ConvArgs& a) {
  const hiseg_conv2d_desc& d = a.d;
  if (d.dtype != HISEG_BF16 || d.convT || d.stride != 1 || d.KH != 3 || d.KW != 3 || d.pad != 1) return false;
  if (d.Ho != d.H || d.Wo != d.W) return false;
  if (d.residual || d.mul || d.out2 || d.in_scale) return false;
  if (d.act != HISEG_ACT_NONE && d.act != HISEG_ACT_RELU) return false;
  const int ncb = d.Cout_pad / 16;
  return (ncb == 1 || ncb == 2) && a.Cin % 8 == 0 && d.Ca % 8 == 0;
}

int conv_rows_try(const ConvArgs& a, hipStream_t s, int variant) {
  const hiseg_conv2d_desc& d = a.d;
  (void)variant;
  if (d.dtype != HISEG_BF16 || d.convT || d.stride != 1 || d.KH != 3 || d.KW != 3 || d.pad != 1) return 0;
  if (d.Ho != d.H || d.Wo != d.W) return 0;
  if (d.residual || d.mul || d.out2 || d.in_scale) return 0;
  if (d.act != HISEG_ACT_NONE && d.act != HISEG_ACT_RELU) return 0;   // (the decoder's ReLU, the head, train z)
  if ((((uintptr_t)d.scale | (uintptr_t)d.shift) & 15) != 0) return 0;
  // one store instruction per lane and row: 4 bf16 / 4 f32 output channels (8- / 16-B aligned), or the single
  // f32 channel of the segmentation head
  if (d.out_dtype == HISEG_BF16 ? (d.Cout % 4 || (d.o_cstride | d.o_coff) % 4 || ((uintptr_t)d.out & 7))
                                : (d.Cout != 1 && (d.Cout % 4 || (d.o_cstride | d.o_coff) % 4 || ((uintptr_t)d.out & 15))))
    return 0;
  if (d.out_dtype == HISEG_F32 && d.Cout == 1 && ((uintptr_t)d.out & 3)) return 0;
  const int Cin = a.Cin;
  if (Cin % 8 != 0 || d.Ca % 8 != 0) return 0;
  const int ncb = d.Cout_pad / 16;
  if (ncb != 1 && ncb != 2) return 0;
  const int ch = Cin / 8;
  const int nkc = (9 * Cin + 31) / 32;
  if (d.K_pad < nkc * 32) return 0;
  // the DMA moves 16-B chunks: every source's channel stride / offset in 8-channel units
  if ((d.a_cstride | d.a_coff) % 8 != 0 || (d.Cb && ((d.b_cstride | d.b_coff) % 8 != 0))) return 0;
  // one buffer resource from the lower source when both sources lie within 2^31 bytes of it; otherwise one
  // resource per source (the TWO form: two DMA instructions per group) -- the same kernel and arithmetic either
  // way, so the layer's speed and bits do not depend on where the allocator placed its sources
  const long long span_a = (long long)d.N * a.Hs * a.Ws * d.a_cstride * 2;
  const long long span_b = d.Cb ? (long long)d.N * d.H * d.W * d.b_cstride * 2 : 0;
  if (span_a >= 0x7fffffffll || span_b >= 0x7fffffffll) return 0;   // (conv2d_impl's image ranges prevent it)
  const long long pa = (long long)(uintptr_t)d.srcA, pb = d.Cb ? (long long)(uintptr_t)d.srcB : pa;
  const long long lo = pa < pb ? pa : pb;
  const bool two = d.Cb && (pa - lo + span_a >= 0x7fffffffll || pb - lo + span_b >= 0x7fffffffll || hiseg_force_far());
  if (two) hiseg_note_placement("conv_rows: sources far apart, one buffer resource each", &d);
  const unsigned dA = two ? 0u : (unsigned)(pa - lo), dB = two ? 0u : (unsigned)(pb - lo);
  // HISEG_ROWS_PER_WG=n: fixed rows per workgroup instead of whole rounds (A/B timing only)
  static const int rpw = [] { const char* e = getenv("HISEG_ROWS_PER_WG"); const int v = e ? atoi(e) : 0; return v > 0 ? v : 0; }();
  return d.out_dtype == HISEG_BF16 ? dispatch_rows<bf16_t>(a, s, ch, ncb, rpw, dA, dB, two)
                                   : dispatch_rows<float>(a, s, ch, ncb, rpw, dA, dB, two);
}

}  // namespace hiseg
