// Row-wise fp8 (OCP e4m3) quantisation for the fp8 forward GEMMs (pso_amd.h, pso_gemm_fp8; BASELINE config 5).
//
//   e[m] = smallest integer with rowmax|x[m][:]| * 2^-e <= 448 (0 for an all-zero row), q[m][k] = e4m3(x[m][k] 2^-e[m])
//
// One wave per row: 16-B bf16 loads, a wave max, v_cvt_pk_fp8_f32 (round to nearest even) on the scaled values,
// 8-B fp8 stores.  The exponent goes out as an E8M0 byte (127 + e), the operand form of v_mfma_scale_f32_*_f8f6f4.
// HBM-bound: 2 bytes read + 1 byte written per element (x is read twice; the second read hits L2 for rows <= 16 KB).
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void quant_rows_fp8_kernel(int M, int K, const bf16_t* __restrict__ x, long ldx,
                                                             uint8_t* __restrict__ q, long ldq,
                                                             uint8_t* __restrict__ e8m0) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const bf16_t* xr = x + (long)row * ldx;
  float amax = 0.f;
  for (int k = lane * 8; k < K; k += 512) {
    const uint4 v = *reinterpret_cast<const uint4*>(xr + k);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      amax = fmaxf(amax, fmaxf(fabsf(bf2f(w[e] & 0xffff)), fabsf(bf2f(w[e] >> 16))));
  }
  amax = warp_max(amax);
  int ex = 0;
  if (amax > 0.f) {
    int p;
    const float m = frexpf(amax * (1.f / 448.f), &p);  // amax / 448 = m 2^p, m in [0.5, 1)
    ex = (m == 0.5f) ? p - 1 : p;                      // ceil(log2(amax / 448))
    ex = max(-126, min(127, ex));
  }
  const float inv = ldexpf(1.f, -ex);
  uint8_t* qr = q + (long)row * ldq;
  for (int k = lane * 8; k < K; k += 512) {
    const uint4 v = *reinterpret_cast<const uint4*>(xr + k);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    int lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(bf2f(w[0] & 0xffff) * inv, -448.f), 448.f),
                                         fminf(fmaxf(bf2f(w[0] >> 16) * inv, -448.f), 448.f), lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(bf2f(w[1] & 0xffff) * inv, -448.f), 448.f),
                                         fminf(fmaxf(bf2f(w[1] >> 16) * inv, -448.f), 448.f), lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(bf2f(w[2] & 0xffff) * inv, -448.f), 448.f),
                                         fminf(fmaxf(bf2f(w[2] >> 16) * inv, -448.f), 448.f), hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(bf2f(w[3] & 0xffff) * inv, -448.f), 448.f),
                                         fminf(fmaxf(bf2f(w[3] >> 16) * inv, -448.f), 448.f), hi, true);
    *reinterpret_cast<uint2*>(qr + k) = make_uint2((uint32_t)lo, (uint32_t)hi);
  }
  if (lane == 0) e8m0[row] = (uint8_t)(127 + ex);
}

}  // namespace

extern "C" int pso_quant_rows_fp8(int M, int K, const void* x, long ldx, void* q, long ldq, void* e8m0, void* stream) {
  PSO_ARG_CHECK(M > 0 && K > 0 && (K % 8) == 0, "pso_quant_rows_fp8: need K %% 8 == 0 (K=%d)", K);
  PSO_ARG_CHECK(x && q && e8m0, "pso_quant_rows_fp8: null operand");
  PSO_ARG_CHECK(((uintptr_t)x & 15) == 0 && (ldx % 8) == 0 && ((uintptr_t)q & 7) == 0 && (ldq % 8) == 0,
                "pso_quant_rows_fp8: x needs 16-B aligned rows, q 8-B aligned rows");
  pso_note_kernel("quant_rows_fp8_kernel");
  quant_rows_fp8_kernel<<<(M + 3) / 4, 256, 0, (hipStream_t)stream>>>(M, K, (const bf16_t*)x, ldx, (uint8_t*)q, ldq,
                                                                      (uint8_t*)e8m0);
  return pso_check_launch("pso_quant_rows_fp8");
}
