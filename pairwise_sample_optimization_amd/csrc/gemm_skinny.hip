// Skinny-N GEMM for gfx950: out[M][N] (+)= alpha * A[M][K] . W[N][K]^T with N <= 128.
//
// The LoRA products of the SDXL UNet: u = x A^T (N = r = 32, 3r = 96 for the fused q/k/v adapters, 2r = 64 for the
// cross-attention k/v pair) and v = dy (sB) in the backward (N = r), at M = B*tokens (616 .. 131072 rows) and
// K = 320 .. 2048.  Replaces peft's lora_A / lora_B nn.Linear calls (`T:338-345`).
//
// These are HBM streams of A (2 FLOP per byte at N = 32).  Every 8-wave workgroup owns 64 rows (four 16-row MFMA
// tiles per wave, so each W fragment feeds four MFMAs) and ALL N columns; the eight waves take the 32-deep K steps
// round-robin, stream A and the small L2-resident W straight into MFMA fragments (no LDS round trip: every A
// element is used by exactly one wave) with up to four K steps of loads in flight, and reduce their eight partial
// 64 x N tiles through LDS.  Grouped form (gridDim.y = groups > 1, the fused q/k/v adapters of the backward):
// group j multiplies A columns [j*K, (j+1)*K) with W columns [j*K, (j+1)*K) into out columns [j*N, (j+1)*N).
#include "common.h"

#include <cstdlib>

__device__ __attribute__((aligned(16))) uint4 g_skinny_zero[4];  // source of every masked (K tail / N pad) load

namespace {

constexpr int SK_W = 8;   // waves per workgroup (K split)

// SK_MT 16-row MFMA tiles per wave (16*SK_MT rows per workgroup): 4 when M gives >= 256 workgroups, else 2
template <int NJ, int SK_MT, int SK_U_ = 0>
__global__ __launch_bounds__(64 * SK_W) void gemm_skinny_nt_kernel(int M, int N, int K, const bf16_t* __restrict__ A,
                                                                   long lda, const bf16_t* __restrict__ W, long ldw,
                                                                   float alpha, void* __restrict__ out, long ldo,
                                                                   int out_f32, int accumulate) {
  // K steps of loads in flight per wave (register budget: 2 waves / SIMD)
  constexpr int SK_U = SK_U_ > 0 ? SK_U_ : ((NJ <= 2 && SK_MT <= 2) ? 4 : 2);
  __shared__ f32x4 red[SK_W][NJ][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int r0 = blockIdx.x * (16 * SK_MT);
  const int grp = blockIdx.y;
  A += (long)grp * K;
  W += (long)grp * K;
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_skinny_zero);
  const bf16_t* arow[SK_MT];
#pragma unroll
  for (int t = 0; t < SK_MT; ++t) arow[t] = A + (long)min(r0 + t * 16 + fr, M - 1) * lda;  // clamped rows: not stored
  const bf16_t* wrow[NJ];
  bool wok[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    wok[j] = j * 16 + fr < N;
    wrow[j] = W + (long)min(j * 16 + fr, N - 1) * ldw;
  }
  const int nc = (K + 31) / 32;
  f32x4 acc[SK_MT][NJ];
#pragma unroll
  for (int t = 0; t < SK_MT; ++t)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c0 = wave; c0 < nc; c0 += SK_W * SK_U) {
    bf16x8 af[SK_U][SK_MT], bfr[SK_U][NJ];
#pragma unroll
    for (int u = 0; u < SK_U; ++u) {
      const int k = (c0 + u * SK_W) * 32 + fk * 8;
      const bool ok = k < K;  // also covers steps past nc
#pragma unroll
      for (int t = 0; t < SK_MT; ++t) af[u][t] = *reinterpret_cast<const bf16x8*>(ok ? arow[t] + k : zero);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bfr[u][j] = *reinterpret_cast<const bf16x8*>((ok && wok[j]) ? wrow[j] + k : zero);
    }
    // all SK_U steps' loads issued before the first MFMA: left alone, the scheduler interleaves them with the MFMAs
    // under vmcnt(0) waits (two or three loads in flight per wave, one HBM round trip per K step)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < SK_U; ++u)
#pragma unroll
      for (int t = 0; t < SK_MT; ++t)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[u][j], af[u][t], acc[t][j], 0, 0, 0);
  }
  // reduce the eight K-partials through LDS, one 16-row tile at a time
  // fragment position (j, l) of tile t holds out[r0 + 16t + (l & 15)][j*16 + (l >> 4)*4 .. +3]
#pragma unroll
  for (int t = 0; t < SK_MT; ++t) {
    if (t > 0) __syncthreads();
#pragma unroll
    for (int j = 0; j < NJ; ++j) red[wave][j][lane] = acc[t][j];
    __syncthreads();
    for (int idx = threadIdx.x; idx < NJ * 64; idx += 64 * SK_W) {
      const int l = idx & 63, j = idx >> 6;
      f32x4 s = red[0][j][l];
#pragma unroll
      for (int w = 1; w < SK_W; ++w) s += red[w][j][l];
      const int m = r0 + t * 16 + (l & 15);
      const int n = j * 16 + (l >> 4) * 4;
      if (m >= M || n >= N) continue;
      float v0 = s[0] * alpha, v1 = s[1] * alpha, v2 = s[2] * alpha, v3 = s[3] * alpha;
      const long o = (long)m * ldo + (long)grp * N + n;
      if (out_f32) {
        float4* po = reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + o);
        if (accumulate) {
          const float4 old = *po;
          v0 += old.x; v1 += old.y; v2 += old.z; v3 += old.w;
        }
        *po = make_float4(v0, v1, v2, v3);
      } else {
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(out) + o) = make_uint2(pack2bf(v0, v1), pack2bf(v2, v3));
      }
    }
  }
}

// benchmark knob (PSO_SKINNY_VARIANT, tools build only): 1 = 16-row tiles x 8 K steps in flight, 2 = 32-row x 8,
// 3 = 16-row x 4, 4 = never 5 steps (the K = 1280 single-round form off)
#ifdef PSO_BENCH_KNOBS
static int skinny_variant() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PSO_SKINNY_VARIANT");
    v = e ? atoi(e) : 0;
  }
  return v;
}
#else
static constexpr int skinny_variant() { return 0; }
#endif

template <int NJ>
int launch_skinny(int M, int N, int K, const bf16_t* a, long lda, const bf16_t* w, long ldw, float alpha, void* out,
                  long ldo, int out_f32, int accumulate, int groups, hipStream_t st) {
  const int var = NJ <= 2 ? skinny_variant() : 0;
#ifdef PSO_BENCH_KNOBS
  if (var == 1 || var == 3) {
    const dim3 grid((M + 15) / 16, groups);
    if (var == 1) {
      pso_note_kernel("gemm_skinny_nt_kernel<%d, %d, %d>", NJ, 1, 8);
      gemm_skinny_nt_kernel<NJ, 1, 8><<<grid, 64 * SK_W, 0, st>>>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32,
                                                                    accumulate);
    } else {
      pso_note_kernel("gemm_skinny_nt_kernel<%d, %d, %d>", NJ, 1, 4);
      gemm_skinny_nt_kernel<NJ, 1, 4><<<grid, 64 * SK_W, 0, st>>>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32,
                                                                    accumulate);
    }
    return pso_check_launch("pso_gemm(skinny)");
  }
  if (var == 2) {
    const dim3 grid((M + 31) / 32, groups);
    pso_note_kernel("gemm_skinny_nt_kernel<%d, %d, %d>", NJ, 2, 8);
    gemm_skinny_nt_kernel<NJ, 2, 8><<<grid, 64 * SK_W, 0, st>>>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32,
                                                                accumulate);
    return pso_check_launch("pso_gemm(skinny)");
  }
#endif
  // K = 1280 is 40 steps of 32: with 4 steps in flight per wave that is two dependent load rounds (the second one
  // step deep); 5 steps per wave take it in one (same per-wave step order, so the same bits).  var 4 keeps the 4.
  // Up to 96 outputs (the fused q/k/v LoRA-down) for 16- and 32-row tiles, up to 32 for 64-row tiles (wider forms
  // spill); forms that never take it name a form they already instantiate.
  const bool k40 = var != 4 && (K + 31) / 32 > SK_W * 4 && (K + 31) / 32 <= SK_W * 5;
  const bool five = NJ <= 6 && k40, five4 = NJ <= 2 && k40;
  constexpr int U5 = NJ <= 6 ? 5 : 4, U5m = NJ <= 6 ? 5 : 0, U5d = NJ <= 2 ? 5 : 0;
  if ((long)((M + 31) / 32) * groups < 128) {
    // small M (the bs = 1 / GPU pass: 2048-row products are 64 workgroups of 32 rows): 16-row tiles, twice the
    // workgroups (bs = 1 step 23.29 vs 22.93 imgs/s same box)
    const dim3 grid((M + 15) / 16, groups);
    if (five) {
      pso_note_kernel("gemm_skinny_nt_kernel<%d, %d, %d>", NJ, 1, U5);
      gemm_skinny_nt_kernel<NJ, 1, U5><<<grid, 64 * SK_W, 0, st>>>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32,
                                                                    accumulate);
    } else {
      pso_note_kernel("gemm_skinny_nt_kernel<%d, %d, %d>", NJ, 1, 4);
      gemm_skinny_nt_kernel<NJ, 1, 4><<<grid, 64 * SK_W, 0, st>>>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32,
                                                                    accumulate);
    }
  } else if ((long)((M + 63) / 64) * groups >= 256) {
    const dim3 grid((M + 63) / 64, groups);
    if (five4) {
      pso_note_kernel("gemm_skinny_nt_kernel<%d, %d, %d>", NJ, 4, U5d);
      gemm_skinny_nt_kernel<NJ, 4, U5d><<<grid, 64 * SK_W, 0, st>>>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32,
                                                                    accumulate);
    } else {
      pso_note_kernel("gemm_skinny_nt_kernel<%d, %d, 0>", NJ, 4);
      gemm_skinny_nt_kernel<NJ, 4><<<grid, 64 * SK_W, 0, st>>>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32,
                                                               accumulate);
    }
  } else {
    const dim3 grid((M + 31) / 32, groups);
    if (five) {
      pso_note_kernel("gemm_skinny_nt_kernel<%d, %d, %d>", NJ, 2, U5m);
      gemm_skinny_nt_kernel<NJ, 2, U5m><<<grid, 64 * SK_W, 0, st>>>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32,
                                                                    accumulate);
    } else {
      pso_note_kernel("gemm_skinny_nt_kernel<%d, %d, 0>", NJ, 2);
      gemm_skinny_nt_kernel<NJ, 2><<<grid, 64 * SK_W, 0, st>>>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32,
                                                               accumulate);
    }
  }
  return pso_check_launch("pso_gemm(skinny)");
}

}  // namespace

// host entry used by run_gemm / pso_gemm_skinny_grouped (gemm.hip); preconditions checked there: N <= 128,
// N % 4 == 0, K % 8 == 0, 16-B aligned A/W rows, 8/16-B aligned output rows.  groups > 1: block-diagonal form.
int pso_gemm_skinny_nt(int M, int N, int K, const void* A, long lda, const void* W, long ldw, float alpha, void* out,
                       long ldo, int out_f32, int accumulate, int groups, hipStream_t st) {
  const int nj = (N + 15) / 16;
  auto a = (const bf16_t*)A;
  auto w = (const bf16_t*)W;
  switch (nj) {
    case 1: return launch_skinny<1>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate, groups, st);
    case 2: return launch_skinny<2>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate, groups, st);
    case 3: case 4: return launch_skinny<4>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate, groups, st);
    case 5: case 6: return launch_skinny<6>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate, groups, st);
    default: return launch_skinny<8>(M, N, K, a, lda, w, ldw, alpha, out, ldo, out_f32, accumulate, groups, st);
  }
}
