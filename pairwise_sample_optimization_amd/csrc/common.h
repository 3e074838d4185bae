// Shared device/host helpers for the PSO MI355X library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/pso_amd.h"
#ifdef PSO_BENCH_KNOBS
#include "../../include/pso_amd_knobs.h"
#endif

typedef uint16_t bf16_t;  // raw bf16 storage
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;

__device__ __forceinline__ float bf2f(bf16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32, RNE, NaN-preserving
  return __builtin_bit_cast(bf16_t, b);
}
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  // one v_cvt_pk_bf16_f32 (RNE, NaN-preserving) for both halves
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{lo, hi}), bf16x2_t));
}
// raw v_exp_f32 (2^x; results below 2^-126 flush to 0 -- fine for softmax weights, saves the denormal range fix-up)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// erf GELU and its derivative: diffusers GEGLU -> F.gelu(approximate="none").  erf(x) for x = |g|/sqrt(2) by
// Abramowitz & Stegun 7.1.26, 1 - t(a1 + t(a2 + ...)) exp(-x^2) with t = 1/(1 + p x), |error| <= 1.5e-7 (far below the
// bf16 rounding of every output; relative error of GELU(g) <= 5e-5 for g >= -3, values below that are < 4e-3 in
// magnitude with absolute error <= 2e-7): branch-free, one v_exp_f32 + one v_rcp_f32 + 8 FMAs, where the library erff is a
// branchy piecewise polynomial (these GELUs run in GEMM epilogues, 2-3 per output element).  exp(-x^2) = exp(-g^2/2)
// is also the derivative's Gaussian density, so the pair shares it.
__device__ __forceinline__ void gelu_erf_parts(float g, float& cdf, float& e) {
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * 0.70710678118654752f * fabsf(g));
  e = __builtin_amdgcn_exp2f(-0.72134752044448170f * g * g);  // exp(-g^2 / 2)
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float tail = 0.5f * poly * e;  // Phi(-|g|) = erfc(|g| / sqrt 2) / 2, formed without cancellation
  cdf = g >= 0.f ? 1.f - tail : tail;   // Phi(g) = (1 + erf(g / sqrt 2)) / 2
}
__device__ __forceinline__ float gelu_erf(float g) {
  float cdf, e;
  gelu_erf_parts(g, cdf, e);
  return g * cdf;
}
__device__ __forceinline__ float gelu_erf_grad(float g) {
  float cdf, e;
  gelu_erf_parts(g, cdf, e);
  return cdf + 0.39894228040143268f * g * e;
}
__device__ __forceinline__ float bf_round(float x) { return bf2f(f2bf(x)); }

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double warp_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- launch bookkeeping (host): the demangled name of the last GEMM-family kernel launched on this thread, as
// rocprofv3 prints it, so HIP-event timings can be attributed per kernel (bench.py roofline) ----
void pso_note_kernel(const char* fmt, ...);

// ---- error plumbing (host) ----
void pso_set_error(const char* fmt, ...);
int pso_check_launch(const char* what);

#define PSO_ARG_CHECK(cond, ...)            \
  do {                                      \
    if (!(cond)) {                          \
      pso_set_error(__VA_ARGS__);           \
      return PSO_ERR_ARG;                   \
    }                                       \
  } while (0)

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
