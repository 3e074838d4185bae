// Skinny-N GEMM for gfx950: out[M][N] (+)= alpha * A[M][K] . W[N][K]^T with N <= 128.
//
// The LoRA products of the SDXL UNet: u = x A^T (N = r = 32, 3r = 96 for the fused q/k/v adapters, 2r = 64 for the
// cross-attention k/v pair) and v = dy (sB) in the backward (N = r), at M = B*tokens (4096 .. 65536 rows) and
// K = 320 .. 2048.  Replaces peft's lora_A / lora_B nn.Linear calls (`T:338-345`).
//
// These are HBM-streaming products (2 FLOP per byte of A at N = 32), far from the MFMA roofline: the tiled kernel
// (64x64 tiles, 64 blocks at M = 4096) was latency-bound at ~13 TFLOP/s.  Here every 4-wave workgroup owns 16 rows
// and ALL N columns; the four waves split the K range (contiguous 4-chunk runs of 32), stream A straight into MFMA
// fragments (no LDS round trip: each A element is used by exactly one wave) with 4 chunks of loads in flight, read the
// small W (L2-resident, shared by every workgroup) the same way, and reduce their four partial 16xN tiles through
// LDS.  M = 4096 gives 256 workgroups (one per CU), M = 16384 gives 1024.
#include "common.h"

__device__ __attribute__((aligned(16))) uint4 g_skinny_zero[4];  // source of every masked (K tail / N pad) load

namespace {

constexpr int SK_U = 4;  // K chunks (of 32) per wave per iteration

template <int NJ, int KW>
__global__ __launch_bounds__(64 * KW) void gemm_skinny_nt_kernel(int M, int N, int K, const bf16_t* __restrict__ A,
                                                                 long lda, const bf16_t* __restrict__ W, long ldw,
                                                                 float alpha, void* __restrict__ out, long ldo,
                                                                 int out_f32, int accumulate) {
  __shared__ f32x4 red[KW][NJ][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int r0 = blockIdx.x * 16;
  const int row = min(r0 + fr, M - 1);  // clamped: rows >= M are computed but never stored
  const bf16_t* arow = A + (long)row * lda;
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_skinny_zero);
  const int nc = (K + 31) / 32;
  f32x4 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c0 = wave * SK_U; c0 < nc; c0 += KW * SK_U) {
    bf16x8 af[SK_U], bfr[SK_U][NJ];
#pragma unroll
    for (int u = 0; u < SK_U; ++u) {
      const int k = (c0 + u) * 32 + fk * 8;
      const bool ok = k < K;  // also covers c0 + u >= nc
      af[u] = *reinterpret_cast<const bf16x8*>(ok ? arow + k : zero);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = j * 16 + fr;
        bfr[u][j] = *reinterpret_cast<const bf16x8*>((ok && n < N) ? W + (long)n * ldw + k : zero);
      }
    }
#pragma unroll
    for (int u = 0; u < SK_U; ++u)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[u][j], af[u], acc[j], 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) red[wave][j][lane] = acc[j];
  __syncthreads();
  // fragment position (j, l) holds out[r0 + (l & 15)][j*16 + (l >> 4)*4 .. +3]
  for (int idx = threadIdx.x; idx < NJ * 64; idx += 64 * KW) {
    const int j = idx >> 6, l = idx & 63;
    f32x4 s = red[0][j][l];
#pragma unroll
    for (int w = 1; w < KW; ++w) s += red[w][j][l];
    const int m = r0 + (l & 15);
    const int n = j * 16 + (l >> 4) * 4;
    if (m >= M || n >= N) continue;
    float v0 = s[0] * alpha, v1 = s[1] * alpha, v2 = s[2] * alpha, v3 = s[3] * alpha;
    if (out_f32) {
      float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + (long)m * ldo + n);
      if (accumulate) {
        const float4 old = *o;
        v0 += old.x; v1 += old.y; v2 += old.z; v3 += old.w;
      }
      *o = make_float4(v0, v1, v2, v3);
    } else {
      *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(out) + (long)m * ldo + n) =
          make_uint2(pack2bf(v0, v1), pack2bf(v2, v3));
    }
  }
}

template <int NJ>
int launch_skinny(int M, int N, int K, const bf16_t* a, long lda, const bf16_t* w, long ldw, float alpha, void* out,
                  long ldo, int out_f32, int accumulate, hipStream_t st) {
  // waves per block: enough K-split that every wave has at most one 4-chunk run in flight (all loads issued at once)
  const int runs = ((K + 31) / 32 + SK_U - 1) / SK_U;
  const dim3 grid((M + 15) / 16);
  if (runs > 8 && NJ <= 6)
    gemm_skinny_nt_kernel<NJ, 16><<<grid, 1024, 0, st>>>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate);
  else if (runs > 4)
    gemm_skinny_nt_kernel<NJ, 8><<<grid, 512, 0, st>>>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate);
  else
    gemm_skinny_nt_kernel<NJ, 4><<<grid, 256, 0, st>>>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate);
  return pso_check_launch("pso_gemm(skinny)");
}

}  // namespace

// host entry used by run_gemm (gemm.hip); preconditions checked there: N <= 128, N % 4 == 0, K % 8 == 0,
// 16-B aligned A/W rows, 8/16-B aligned output rows.
int pso_gemm_skinny_nt(int M, int N, int K, const void* A, long lda, const void* W, long ldw, float alpha, void* out,
                       long ldo, int out_f32, int accumulate, hipStream_t st) {
  const int nj = (N + 15) / 16;
  auto a = (const bf16_t*)A;
  auto w = (const bf16_t*)W;
  switch (nj) {
    case 1: return launch_skinny<1>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate, st);
    case 2: return launch_skinny<2>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate, st);
    case 3: return launch_skinny<3>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate, st);
    case 4: return launch_skinny<4>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate, st);
    case 5: case 6: return launch_skinny<6>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate, st);
    default: return launch_skinny<8>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate, st);
  }
}
