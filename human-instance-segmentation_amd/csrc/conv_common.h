// Shared pieces of the implicit-GEMM conv kernels (GEMM view, epilogue).
#pragma once
#include "common.h"

namespace hiseg {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

struct ConvArgs {
  hiseg_conv2d_desc d;
  int M;       // GEMM rows
  int Cin;     // Ca + Cb
  int nK;      // K blocks
  int Hs, Ws;  // src-A grid
  int kper;    // split-K: K blocks per split (grid.z = splits); nK when unsplit
  int ins_vec; // in_scale rows 16-B aligned (vector gate loads)
  float* ws;   // split-K workspace [splits][M][Cout_pad] f32
  int abl = 0; // DIAG builds only: ablation bits of a timing variant (parts of a kernel switched off)
};

template <typename T>
__device__ __forceinline__ void load4(const void* base, long long idx, bool vec, int nvalid,
                                      float* v) {
  if (vec) {
    if constexpr (sizeof(T) == 4) {
      float4 q = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(base) + idx);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
      uint2 q = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(base) + idx);
      v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
      v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (e < nvalid) ? Elem<T>::load(base, idx + e) : 0.f;
  }
}

template <typename T>
__device__ __forceinline__ void store4(void* base, long long idx, bool vec, int nvalid,
                                       const float* v) {
  if (vec) {
    if constexpr (sizeof(T) == 4) {
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(base) + idx) =
          make_float4(v[0], v[1], v[2], v[3]);
    } else {
      uint2 q;
      q.x = f2bf2(v[0], v[1]);
      q.y = f2bf2(v[2], v[3]);
      *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(base) + idx) = q;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (e < nvalid) Elem<T>::store(base, idx + e, v[e]);
  }
}

__device__ __forceinline__ int swz(int row, int c) { return row * 8 + (c ^ ((row >> 1) & 7)); }

// Output site of GEMM element (px, co): (op, oc) = (px, co), or for a ConvTranspose 2x2/s2 GEMM
// (columns q*Cout/4 + oc, q = 2*dy + dx) the scattered full-resolution pixel.
__device__ __forceinline__ void out_site(const hiseg_conv2d_desc& d, int px, int co, long long& op, int& oc) {
  if (d.convT) {
    const int Cq = d.Cout >> 2;
    const int q = co / Cq;
    oc = co - q * Cq;
    const int x = px % d.Wo;
    const int t = px / d.Wo;
    const int y = t % d.Ho;
    const int n = t / d.Ho;
    op = ((long long)n * (2 * d.Ho) + 2 * y + (q >> 1)) * (2 * d.Wo) + 2 * x + (q & 1);
  } else {
    op = px;
    oc = co;
  }
}

template <typename T, typename TO>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, int px, int co, floatx4 acc) {
  const hiseg_conv2d_desc& d = a.d;
  float v[4] = {acc[0], acc[1], acc[2], acc[3]};
  const int ncol = d.Cout - co;
  if (ncol <= 0) return;
  const int nv = ncol < 4 ? ncol : 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (e < nv) v[e] = v[e] * d.scale[co + e] + d.shift[co + e];
  }
  long long op;  // output pixel index
  int oc;        // output channel
  out_site(d, px, co, op, oc);
  if (d.residual) {
    float r[4];
    const bool vec = (nv == 4) && ((d.r_cstride | d.r_coff | oc) & 3) == 0;
    load4<T>(d.residual, op * d.r_cstride + d.r_coff + oc, vec, nv, r);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] += r[e];
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], d.act, d.act_beta);
  if (d.mul) {
    float m[4];
    const bool vec = (nv == 4) && ((d.m_cstride | d.m_coff | oc) & 3) == 0;
    load4<T>(d.mul, op * d.m_cstride + d.m_coff + oc, vec, nv, m);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] *= m[e];
  }
  {
    const bool vec = (nv == 4) && ((d.o_cstride | d.o_coff | oc) & 3) == 0;
    store4<TO>(d.out, op * d.o_cstride + d.o_coff + oc, vec, nv, v);
  }
  if (d.out2) {
    const bool vec = (nv == 4) && ((d.o2_cstride | d.o2_coff | oc) & 3) == 0;
    store4<T>(d.out2, op * d.o2_cstride + d.o2_coff + oc, vec, nv, v);
  }
}

// 4 consecutive elements of T as one vector load / store.
template <typename T> struct Quad;
template <> struct Quad<bf16_t> {
  typedef uint2 V;
  __device__ static __forceinline__ V load(const void* p, long long i) {
    return *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(p) + i);
  }
  __device__ static __forceinline__ float get(const V& v, int e) {
    const uint32_t w = e < 2 ? v.x : v.y;
    return (e & 1) ? __uint_as_float(w & 0xffff0000u) : __uint_as_float(w << 16);
  }
  __device__ static __forceinline__ V zero() { return make_uint2(0u, 0u); }
  __device__ static __forceinline__ void store(void* p, long long i, const float* f) {
    uint2 o;
    o.x = f2bf2(f[0], f[1]);
    o.y = f2bf2(f[2], f[3]);
    *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p) + i) = o;
  }
};
template <> struct Quad<float> {
  typedef float4 V;
  __device__ static __forceinline__ V load(const void* p, long long i) {
    return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + i);
  }
  __device__ static __forceinline__ float get(const V& v, int e) {
    return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
  }
  __device__ static __forceinline__ V zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ static __forceinline__ void store(void* p, long long i, const float* f) {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(p) + i) = make_float4(f[0], f[1], f[2], f[3]);
  }
};

// Epilogue of a TM x TN block of 16x16 accumulators whose lane owns 4 consecutive output channels
// co[i] of pixel px[j].  prefetch() issues every scale / shift / residual load before the first
// store, so the loads are not serialised behind the stores (out and residual may alias as far as
// the compiler knows); call it early (e.g. before the K loop) to hide their latency.  Applies
// when ok(): 4-aligned channel views and 4 | Cout (4 | Cout/4 for ConvTranspose); otherwise
// use conv_epilogue per fragment.
template <typename T, typename TO, int TM, int TN>
struct TileEpi {
  floatx4 sc[TM], sh[TM];
  typename Quad<T>::V res[TM][TN];

  __device__ static __forceinline__ bool ok(const hiseg_conv2d_desc& d) {
    constexpr uintptr_t va = sizeof(T) == 2 ? 7 : 15, vo = sizeof(TO) == 2 ? 7 : 15;
    return (!d.convT || ((d.Cout >> 2) & 3) == 0) && (d.Cout & 3) == 0 &&
           ((d.o_cstride | d.o_coff) & 3) == 0 && (!d.out2 || ((d.o2_cstride | d.o2_coff) & 3) == 0) &&
           (!d.residual || ((d.r_cstride | d.r_coff) & 3) == 0) &&
           (!d.mul || ((d.m_cstride | d.m_coff) & 3) == 0) &&
           (((uintptr_t)d.scale | (uintptr_t)d.shift) & 15) == 0 && ((uintptr_t)d.out & vo) == 0 &&
           (((uintptr_t)d.out2 | (uintptr_t)d.residual | (uintptr_t)d.mul) & va) == 0;
  }

  __device__ __forceinline__ void prefetch(const hiseg_conv2d_desc& d, int M, const int (&px)[TN], const int (&co)[TM]) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int cc = co[i] < d.Cout ? co[i] : 0;
      sc[i] = *reinterpret_cast<const floatx4*>(d.scale + cc);
      sh[i] = *reinterpret_cast<const floatx4*>(d.shift + cc);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        res[i][j] = Quad<T>::zero();
        if (d.residual) {
          long long op;
          int oc;
          out_site(d, px[j] < M ? px[j] : M - 1, cc, op, oc);
          res[i][j] = Quad<T>::load(d.residual, op * d.r_cstride + d.r_coff + oc);
        }
      }
    }
  }

  __device__ __forceinline__ void store(const hiseg_conv2d_desc& d, int M, const int (&px)[TN], const int (&co)[TM],
                                        const floatx4 (&acc)[TM][TN], bool write_out2 = true) {
    with_act(d.act, [&](auto ac) __attribute__((always_inline)) {
      constexpr int A = decltype(ac)::value;
#pragma clang loop unroll(full)
      for (int i = 0; i < TM; ++i)
#pragma clang loop unroll(full)
        for (int j = 0; j < TN; ++j) {
          if (px[j] >= M || co[i] >= d.Cout) continue;
          long long op;
          int oc;
          out_site(d, px[j], co[i], op, oc);
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * sc[i][e] + sh[i][e];
          if (d.residual) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += Quad<T>::get(res[i][j], e);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = act_c<A>(v[e], d.act, d.act_beta);
          if (d.mul) {
            const typename Quad<T>::V m = Quad<T>::load(d.mul, op * d.m_cstride + d.m_coff + oc);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] *= Quad<T>::get(m, e);
          }
          Quad<TO>::store(d.out, op * d.o_cstride + d.o_coff + oc, v);
          if (write_out2 && d.out2) Quad<T>::store(d.out2, op * d.o2_cstride + d.o2_coff + oc, v);
        }
    });
  }
};

}  // namespace hiseg
