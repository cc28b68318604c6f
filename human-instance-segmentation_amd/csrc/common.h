// Shared device helpers for libhiseg (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "hiseg.h"

namespace hiseg {

// bf16 is carried as raw 16-bit storage; arithmetic is always f32.
struct bf16_t { uint16_t x; };

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// Round-to-nearest-even by the gfx950 conversion instruction v_cvt_pk_bf16_f32 (a plain cast at -O3), NaN kept
// a NaN (MI355X_MICROARCH.md "Correctness boundaries"); one instruction per PAIR with f2bf2 -- the integer
// rounding sequence it replaces cost ~5 VALU instructions per value, which bound the narrow-input 1x1 layers'
// epilogues.
typedef __bf16 hiseg_bf16x2_t __attribute__((ext_vector_type(2)));
typedef float hiseg_f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ uint32_t f2bf2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((hiseg_f32x2_t){lo, hi}, hiseg_bf16x2_t));
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  static constexpr int kChunk = 4;  // elements per 16-B chunk
  __device__ static __forceinline__ float load(const void* p, long long i) {
    return reinterpret_cast<const float*>(p)[i];
  }
  __device__ static __forceinline__ void store(void* p, long long i, float v) {
    reinterpret_cast<float*>(p)[i] = v;
  }
};
template <> struct Elem<bf16_t> {
  static constexpr int kChunk = 8;
  __device__ static __forceinline__ float load(const void* p, long long i) {
    return bf2f(reinterpret_cast<const uint16_t*>(p)[i]);
  }
  __device__ static __forceinline__ void store(void* p, long long i, float v) {
    reinterpret_cast<uint16_t*>(p)[i] = f2bf(v);
  }
};

// 1 / (1 + e^-x) with the hardware reciprocal (v_rcp_f32, 1 ulp) instead of the correctly rounded division's
// 11-instruction sequence: sigmoid / SiLU epilogues are VALU-bound on the wide EfficientNet expansions
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// nn.GELU() (approximate='none'): x * Phi(x) with the exact erf.  Out of line, as its derivative below: the runtime
// activation switch is inlined per output element into unrolled epilogues, and the erf body was most of their code
// (conv_igemm's 128x128 kernels 132 -> 93 KB) -- instruction fetch, not arithmetic, bounds the short launches
// (tools/icache_probe.hip: ~0.6 us per KB of straight-line code run once per wave, profiles/r6_icache_probe.txt)
__device__ __noinline__ float gelu_(float v) { return 0.5f * v * (1.f + erff(v * 0.70710678118654752f)); }
__device__ __noinline__ float gelu_grad_(float v) {
  return 0.5f * (1.f + erff(v * 0.70710678118654752f)) + v * 0.39894228040143268f * __expf(-0.5f * v * v);
}

// Activation of the pre-activation v (advanced/activation_utils.py:71-101); beta is Swish's.  The sigmoid family
// shares one exp / rcp sequence (a switch inlined per output element into the unrolled epilogues carried three of
// them; same arithmetic per activation, so the same bits).
__device__ __forceinline__ float apply_act(float v, int act, float beta = 1.f) {
  if (act == HISEG_ACT_NONE) return v;
  if (act == HISEG_ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == HISEG_ACT_GELU) return gelu_(v);
  if (act != HISEG_ACT_SIGMOID && act != HISEG_ACT_SILU && act != HISEG_ACT_SWISH) return v;
  const float s = sigmoidf_(act == HISEG_ACT_SWISH ? beta * v : v);
  return act == HISEG_ACT_SIGMOID ? s : v * s;
}

// d act / d v at the pre-activation v.
__device__ __forceinline__ float act_grad_pre(float v, int act, float beta = 1.f) {
  if (act == HISEG_ACT_NONE) return 1.f;
  if (act == HISEG_ACT_RELU) return v > 0.f ? 1.f : 0.f;
  if (act == HISEG_ACT_GELU) return gelu_grad_(v);
  if (act != HISEG_ACT_SIGMOID && act != HISEG_ACT_SILU && act != HISEG_ACT_SWISH) return 1.f;
  const float b = act == HISEG_ACT_SWISH ? beta : 1.f;
  const float s = sigmoidf_(act == HISEG_ACT_SWISH ? beta * v : v);
  return act == HISEG_ACT_SIGMOID ? s * (1.f - s) : s * (1.f + b * v * (1.f - s));
}

// Run `f` with the activation as a compile-time constant when it is identity / ReLU / SiLU (kActRt: the run-time switch
// for the others): an unrolled epilogue then holds one compact branch-free body per form instead of the activation
// switch once per output element -- less code to fetch cold on short launches (tools/icache_probe.hip), same bits.
constexpr int kActRt = -1;
template <typename F>
__device__ __forceinline__ void with_act(int act, F&& f) {
  if (act == HISEG_ACT_NONE) f(std::integral_constant<int, HISEG_ACT_NONE>{});
  else if (act == HISEG_ACT_RELU) f(std::integral_constant<int, HISEG_ACT_RELU>{});
  else if (act == HISEG_ACT_SILU) f(std::integral_constant<int, HISEG_ACT_SILU>{});
  else f(std::integral_constant<int, kActRt>{});
}
template <int A>
__device__ __forceinline__ float act_c(float v, int act, float beta) {
  return A == kActRt ? apply_act(v, act, beta) : apply_act(v, A);
}

// Activations whose derivative needs the pre-activation (not recoverable from the output).
__host__ __device__ __forceinline__ bool act_smooth(int act) {
  return act == HISEG_ACT_SILU || act == HISEG_ACT_GELU || act == HISEG_ACT_SWISH;
}

// Unpack a 16-B chunk into f32 values / pack back.
template <typename T> struct Chunk;
template <> struct Chunk<float> {
  static constexpr int N = 4;
  __device__ static __forceinline__ void unpack(const uint4& c, float* v) {
    v[0] = __uint_as_float(c.x); v[1] = __uint_as_float(c.y);
    v[2] = __uint_as_float(c.z); v[3] = __uint_as_float(c.w);
  }
  __device__ static __forceinline__ uint4 pack(const float* v) {
    return make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                      __float_as_uint(v[3]));
  }
};
template <> struct Chunk<bf16_t> {
  static constexpr int N = 8;
  __device__ static __forceinline__ void unpack(const uint4& c, float* v) {
    const uint32_t w[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ static __forceinline__ uint4 pack(const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = f2bf2(v[2 * i], v[2 * i + 1]);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
};

}  // namespace hiseg

// Host-side error plumbing (defined in capi.cpp).
void hiseg_set_error(const char* fmt, ...);
int hiseg_check_launch(const char* what);
struct hiseg_conv2d_desc;
void hiseg_note_placement(const char* what, const hiseg_conv2d_desc* d);
bool hiseg_force_far();

static inline bool al16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

#define HISEG_REQUIRE(cond, code, ...)  \
  do {                                  \
    if (!(cond)) {                      \
      hiseg_set_error(__VA_ARGS__);     \
      return (code);                    \
    }                                   \
  } while (0)
