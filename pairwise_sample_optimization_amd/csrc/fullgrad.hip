// Weight-gradient helpers for full-UNet training (BASELINE config C3/C4, SURVEY §8a a6 "full dW in C3").
//
// The reference trains LoRA only; C3 asks the build for gradients of every UNet parameter (App. A #4).  The dW GEMMs
// themselves run on the TN GEMM (gemm.hip pso_gemm_tn); these kernels supply what they need around it:
//   pso_colsum_acc         out[g][n] += sum of x[m][n] over the rows m of group g (bias gradients: one group; the
//                          per-image time-embedding row-bias gradients of the resnets: one group per image)
//   pso_layer_norm_dparam  dgamma[c] += sum_m dy[m][c] * (x[m][c] - mean_m) * rstd_m,  dbeta[c] += sum_m dy[m][c]
//   (the *_ws forms: the same sums reduced in a fixed order through a caller-owned workspace -- no float atomics;
//   the product path uses them, so the full-UNet backward is bit-reproducible)
//   pso_im2col_conv        the 3x3 patch matrix [B*Ho*Wo][9*(C1+C2)] (tap-major, channel-minor: the NHWC weight
//                          layout [Cout][kh][kw][Cin]) of a NORMAL (stride 1/2) or UP2 (nearest 2x upsample) conv over
//                          one or two concatenated NHWC sources, so dW = dY^T . cols is one TN GEMM.
#include "common.h"

namespace {

constexpr int CS_ROWS = 256;  // rows per colsum / dparam workgroup

// 256 threads = 4 row slices x 64 column quads; each block covers 256 rows x 256 columns
__global__ __launch_bounds__(256) void colsum_kernel(long M, int N, const bf16_t* __restrict__ x, long ldx, long rpg,
                                                     float* __restrict__ out, long ldo) {
  const int t = threadIdx.x;
  const int n = (blockIdx.x * 64 + (t & 63)) * 4;
  const long r0 = (long)blockIdx.y * CS_ROWS;
  const long r1 = min(M, r0 + CS_ROWS);
  if (n >= N) return;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  long cur = r0 / rpg;
  for (long m = r0 + (t >> 6); m < r1; m += 4) {
    const long gm = m / rpg;
    if (gm != cur) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (n + r < N) atomicAdd(out + cur * ldo + n + r, s[r]);
      s[0] = s[1] = s[2] = s[3] = 0.f;
      cur = gm;
    }
    if (n + 4 <= N) {
      const uint2 v = *reinterpret_cast<const uint2*>(x + m * ldx + n);
      s[0] += bf2f(v.x & 0xffff); s[1] += bf2f(v.x >> 16); s[2] += bf2f(v.y & 0xffff); s[3] += bf2f(v.y >> 16);
    } else {
      for (int r = 0; r < 4 && n + r < N; ++r) s[r] += bf2f(x[m * ldx + n + r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (n + r < N) atomicAdd(out + cur * ldo + n + r, s[r]);
}

__global__ __launch_bounds__(256) void ln_dparam_kernel(int M, int C, const bf16_t* __restrict__ x, long ldx,
                                                        const bf16_t* __restrict__ dy, long lddy,
                                                        const float* __restrict__ stats, float* __restrict__ dgamma,
                                                        float* __restrict__ dbeta) {
  const int t = threadIdx.x;
  const int c = (blockIdx.x * 64 + (t & 63)) * 4;
  const int r0 = blockIdx.y * CS_ROWS;
  const int r1 = min(M, r0 + CS_ROWS);
  if (c >= C) return;
  float g[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
  for (int m = r0 + (t >> 6); m < r1; m += 4) {
    const float mean = stats[2 * m], rstd = stats[2 * m + 1];
    const uint2 xv = *reinterpret_cast<const uint2*>(x + (long)m * ldx + c);
    const uint2 dv = *reinterpret_cast<const uint2*>(dy + (long)m * lddy + c);
    const float xs[4] = {bf2f(xv.x & 0xffff), bf2f(xv.x >> 16), bf2f(xv.y & 0xffff), bf2f(xv.y >> 16)};
    const float ds[4] = {bf2f(dv.x & 0xffff), bf2f(dv.x >> 16), bf2f(dv.y & 0xffff), bf2f(dv.y >> 16)};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      g[r] += ds[r] * (xs[r] - mean) * rstd;
      b[r] += ds[r];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    atomicAdd(dgamma + c + r, g[r]);
    atomicAdd(dbeta + c + r, b[r]);
  }
}

// Vector forms (N % 8 == 0, 16-B aligned rows): 256 threads = 4 row slices x 64 chunks of 8 columns (16-B loads), a
// block = CS2_ROWS rows x 512 columns, so even the smallest weight (6144 x 1280 rows x columns of one image group) has
// ~300 blocks in flight; the 4 slices are summed in LDS and one atomic per column leaves the block (a block that
// straddles a row group -- per-image sums -- flushes per thread instead).
constexpr int CS2_ROWS = 64;

__device__ __forceinline__ void unpack8f(const uint4 v, float (&f)[8]) {
  f[0] = bf2f(v.x & 0xffff); f[1] = bf2f(v.x >> 16); f[2] = bf2f(v.y & 0xffff); f[3] = bf2f(v.y >> 16);
  f[4] = bf2f(v.z & 0xffff); f[5] = bf2f(v.z >> 16); f[6] = bf2f(v.w & 0xffff); f[7] = bf2f(v.w >> 16);
}

// NS sums per column (colsum: 1, LN dparam: 2) of the block's slices -> LDS -> one atomic each per column, the
// block's 512 columns 2 per thread in column order (each wave-instruction adds 64 consecutive floats: 4 atomic
// requests of 64 B; a lane-per-8-columns order would scatter every lane into its own 64-B request)
template <int NS>
__device__ __forceinline__ void cs2_flush(float (&acc)[NS][8], float* __restrict__ o0, float* __restrict__ o1, int nb,
                                          int N, float (*red)[4][64][8]) {
  const int t = threadIdx.x, tx = t & 63, ty = t >> 6;
#pragma unroll
  for (int k = 0; k < NS; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) red[k][ty][tx][e] = acc[k][e];
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = h * 256 + t, n = nb + c;  // column c of the block
    if (n >= N) continue;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const float v = red[k][0][c >> 3][c & 7] + red[k][1][c >> 3][c & 7] + red[k][2][c >> 3][c & 7] +
                      red[k][3][c >> 3][c & 7];
      atomicAdd((k ? o1 : o0) + n, v);
    }
  }
}

__global__ __launch_bounds__(256) void colsum8_kernel(long M, int N, const bf16_t* __restrict__ x, long ldx, long rpg,
                                                      float* __restrict__ out, long ldo) {
  __shared__ float red[1][4][64][8];
  const int t = threadIdx.x, tx = t & 63, ty = t >> 6;
  const int n = (blockIdx.x * 64 + tx) * 8;
  const long r0 = (long)blockIdx.y * CS2_ROWS, r1 = min(M, r0 + CS2_ROWS);
  const bool straddle = r0 / rpg != (r1 - 1) / rpg;  // block-uniform
  float acc[1][8] = {{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}};
  long cur = r0 / rpg;
  if (n < N) {
    for (long m = r0 + ty; m < r1; m += 4) {
      if (straddle && m / rpg != cur) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { atomicAdd(out + cur * ldo + n + e, acc[0][e]); acc[0][e] = 0.f; }
        cur = m / rpg;
      }
      float f[8];
      unpack8f(*reinterpret_cast<const uint4*>(x + m * ldx + n), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[0][e] += f[e];
    }
  }
  if (straddle) {
    if (n < N)
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(out + cur * ldo + n + e, acc[0][e]);
    return;
  }
  cs2_flush<1>(acc, out + cur * ldo, nullptr, blockIdx.x * 512, N, red);
}

__global__ __launch_bounds__(256) void ln_dparam8_kernel(int M, int C, const bf16_t* __restrict__ x, long ldx,
                                                         const bf16_t* __restrict__ dy, long lddy,
                                                         const float* __restrict__ stats, float* __restrict__ dgamma,
                                                         float* __restrict__ dbeta) {
  __shared__ float red[2][4][64][8];
  const int t = threadIdx.x, tx = t & 63, ty = t >> 6;
  const int c = (blockIdx.x * 64 + tx) * 8;
  const int r0 = blockIdx.y * CS2_ROWS, r1 = min(M, r0 + CS2_ROWS);
  float acc[2][8] = {{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}};
  if (c < C) {
    for (int m = r0 + ty; m < r1; m += 4) {
      const float2 st = *reinterpret_cast<const float2*>(stats + 2 * m);
      float xs[8], ds[8];
      unpack8f(*reinterpret_cast<const uint4*>(x + (long)m * ldx + c), xs);
      unpack8f(*reinterpret_cast<const uint4*>(dy + (long)m * lddy + c), ds);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        acc[0][e] += ds[e] * (xs[e] - st.x) * st.y;
        acc[1][e] += ds[e];
      }
    }
  }
  cs2_flush<2>(acc, dgamma, dbeta, blockIdx.x * 512, C, red);
}

// Ordered (deterministic) forms -- no float atomics: stage 1 stores every row block's column partials, stage 2 adds
// them in row-block order (the full-UNet backward then gives the same bits run to run and in any stream schedule).
// colsum: row block j of group g covers rows [g*rpg + j*CS2_ROWS, min(+CS2_ROWS, (g+1)*rpg)) (blocks never straddle a
// group); part[(g*nbg + j)][N].  LN dparam: part[j][2][C] (dgamma, dbeta).  256 threads = 4 row slices x 64 chunks of 8
// columns; the slices are folded in LDS in slice order.
template <int NS>
__device__ __forceinline__ void cs2_store(float (&acc)[NS][8], float* __restrict__ p0, float* __restrict__ p1, int nb,
                                          int N, float (*red)[4][64][8]) {
  const int t = threadIdx.x, tx = t & 63, ty = t >> 6;
#pragma unroll
  for (int k = 0; k < NS; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) red[k][ty][tx][e] = acc[k][e];
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = h * 256 + t, n = nb + c;
    if (n >= N) continue;
#pragma unroll
    for (int k = 0; k < NS; ++k)
      (k ? p1 : p0)[n] = red[k][0][c >> 3][c & 7] + red[k][1][c >> 3][c & 7] + red[k][2][c >> 3][c & 7] +
                         red[k][3][c >> 3][c & 7];
  }
}

__device__ __forceinline__ void load8_tail(const bf16_t* __restrict__ p, int n, int N, float (&f)[8], bool vec) {
  if (vec && n + 8 <= N) {
    unpack8f(*reinterpret_cast<const uint4*>(p), f);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = n + e < N ? bf2f(p[e]) : 0.f;
  }
}

__global__ __launch_bounds__(256) void colsum_part_kernel(long M, int N, const bf16_t* __restrict__ x, long ldx,
                                                          long rpg, int nbg, int vec, float* __restrict__ part) {
  __shared__ float red[1][4][64][8];
  const int t = threadIdx.x, tx = t & 63, ty = t >> 6;
  const int n = (blockIdx.x * 64 + tx) * 8;
  const long g = blockIdx.y / nbg, j = blockIdx.y - g * nbg;
  const long r0 = g * rpg + j * CS2_ROWS, r1 = min(min(M, (g + 1) * rpg), r0 + CS2_ROWS);
  float acc[1][8] = {{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}};
  if (n < N) {
    for (long m = r0 + ty; m < r1; m += 4) {
      float f[8];
      load8_tail(x + m * ldx + n, n, N, f, vec != 0);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[0][e] += f[e];
    }
  }
  cs2_store<1>(acc, part + (size_t)blockIdx.y * N, nullptr, blockIdx.x * 512, N, red);
}

// Ordered two-level reduction of row-block partials (colsum: part[g][R][N]; LN dparam: part[1][R][2C]):
//   level 1: split s of S adds rows [s*ch, (s+1)*ch) of its group in row order -> p2[g][s][N]  (ch rows in flight
//            8 at a time: a single pass over R = 1,536 partials per column was a 1,536-long dependent load chain)
//   level 2: out[g][n] += sum over s of p2[g][s][n], s in order
// The grouping (R, S, ch) is a function of the shape only, so the sums are bit-reproducible.
__global__ __launch_bounds__(256) void ordered_reduce_l1_kernel(int R, int N, int S, int ch,
                                                                const float* __restrict__ part,
                                                                float* __restrict__ p2) {
  const int n = blockIdx.x * 256 + threadIdx.x, sp = blockIdx.y, g = blockIdx.z;
  if (n >= N) return;
  const int j0 = sp * ch, j1 = min(R, j0 + ch);
  const float* p = part + ((size_t)g * R) * N + n;
  float acc = 0.f;
  for (int j = j0; j < j1; j += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = j + u < j1 ? p[(size_t)(j + u) * N] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];  // row order (the trailing zeros add exactly)
  }
  p2[((size_t)g * S + sp) * N + n] = acc;
}

// level 2.  LN dparam (split2 = C): columns [0, C) -> dgamma, [C, 2C) -> dbeta; colsum (split2 = 0): out[g*ldo + n]
__global__ void ordered_reduce_l2_kernel(int G, int N, int S, const float* __restrict__ p2, float* __restrict__ out,
                                         long ldo, float* __restrict__ out2, int split2) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)G * N) return;
  const int g = (int)(i / N), n = (int)(i - (long)g * N);
  float acc = 0.f;
  for (int sp = 0; sp < S; ++sp) acc += p2[((size_t)g * S + sp) * N + n];
  if (split2 > 0) {
    if (n < split2) out[n] += acc;
    else out2[n - split2] += acc;
  } else {
    out[(long)g * ldo + n] += acc;
  }
}

// split count of the level-1 pass: ~32 partial rows per split, at most 64 splits; R <= 48 partial rows take level 2
// alone (S = R, ch = 1: the level-1 pass would copy them)
static void ordered_reduce_plan(int R, int& S, int& ch) {
  if (R <= 48) {
    S = R;
    ch = 1;
    return;
  }
  S = (R + 31) / 32;
  if (S > 64) S = 64;
  if (S < 1) S = 1;
  ch = (R + S - 1) / S;
  S = (R + ch - 1) / ch;
}

__global__ __launch_bounds__(256) void ln_dparam_part_kernel(int M, int C, const bf16_t* __restrict__ x, long ldx,
                                                             const bf16_t* __restrict__ dy, long lddy,
                                                             const float* __restrict__ stats, int vec,
                                                             float* __restrict__ part) {
  __shared__ float red[2][4][64][8];
  const int t = threadIdx.x, tx = t & 63, ty = t >> 6;
  const int c = (blockIdx.x * 64 + tx) * 8;
  const int r0 = blockIdx.y * CS2_ROWS, r1 = min(M, r0 + CS2_ROWS);
  float acc[2][8] = {{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}};
  if (c < C) {
    for (int m = r0 + ty; m < r1; m += 4) {
      const float mean = stats[2 * m], rstd = stats[2 * m + 1];
      float xs[8], ds[8];
      load8_tail(x + (long)m * ldx + c, c, C, xs, vec != 0);
      load8_tail(dy + (long)m * lddy + c, c, C, ds, vec != 0);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        acc[0][e] += ds[e] * (xs[e] - mean) * rstd;
        acc[1][e] += ds[e];
      }
    }
  }
  float* p = part + (size_t)blockIdx.y * 2 * C;
  cs2_store<2>(acc, p, p + C, blockIdx.x * 512, C, red);
}

// one thread per (output pixel, tap, 8-channel chunk)
__global__ __launch_bounds__(256) void im2col_conv_kernel(int mode, int B, const bf16_t* __restrict__ s1, int C1,
                                                          const bf16_t* __restrict__ s2, int C2, int H, int W, int Ho,
                                                          int Wo, int stride, int pad, bf16_t* __restrict__ out,
                                                          long ldo) {
  const int Ct = C1 + C2, nch = Ct / 8;
  const long idx = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long total = (long)B * Ho * Wo * 9 * nch;
  if (idx >= total) return;
  const int ch = (int)(idx % nch);
  const long rest = idx / nch;
  const int tap = (int)(rest % 9);
  const long p = rest / 9;
  const int ox = (int)(p % Wo);
  const int oy = (int)((p / Wo) % Ho);
  const int b = (int)(p / ((long)Wo * Ho));
  const int ky = tap / 3, kx = tap - 3 * (tap / 3);
  int iy, ix;
  bool ok;
  if (mode == PSO_CONV_UP2) {
    const int uy = oy + ky - pad, ux = ox + kx - pad;
    ok = (unsigned)uy < (unsigned)(2 * H) && (unsigned)ux < (unsigned)(2 * W);
    iy = uy >> 1;
    ix = ux >> 1;
  } else {
    iy = oy * stride + ky - pad;
    ix = ox * stride + kx - pad;
    ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
  }
  const int c = ch * 8;
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (ok) {
    const long pix = ((long)b * H + iy) * W + ix;
    v = c < C1 ? *reinterpret_cast<const uint4*>(s1 + pix * C1 + c)
               : *reinterpret_cast<const uint4*>(s2 + pix * C2 + (c - C1));
  }
  *reinterpret_cast<uint4*>(out + p * ldo + (long)tap * Ct + c) = v;
}

}  // namespace

extern "C" {

int pso_colsum_acc(long M, int N, const void* x, long ldx, long rows_per_group, float* out, long ldo, void* stream) {
  PSO_ARG_CHECK(M >= 0 && N > 0 && x && out && rows_per_group > 0, "pso_colsum_acc: bad arguments");
  PSO_ARG_CHECK((((uintptr_t)x) & 7) == 0 && (ldx % 4) == 0, "pso_colsum_acc: 8-B aligned rows");
  if (M == 0) return PSO_OK;
  if ((N % 8) == 0 && (((uintptr_t)x) & 15) == 0 && (ldx % 8) == 0) {
    const dim3 grid((N + 511) / 512, (unsigned)((M + CS2_ROWS - 1) / CS2_ROWS));
    colsum8_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(M, N, (const bf16_t*)x, ldx, rows_per_group, out, ldo);
    return pso_check_launch("pso_colsum_acc");
  }
  const dim3 grid((N + 255) / 256, (unsigned)((M + CS_ROWS - 1) / CS_ROWS));
  colsum_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(M, N, (const bf16_t*)x, ldx, rows_per_group, out, ldo);
  return pso_check_launch("pso_colsum_acc");
}

int pso_layer_norm_dparam(int M, int C, const void* x, long ldx, const void* dy, long lddy, const float* stats,
                          float* dgamma, float* dbeta, void* stream) {
  PSO_ARG_CHECK(M >= 0 && C > 0 && (C % 4) == 0 && x && dy && stats && dgamma && dbeta,
                "pso_layer_norm_dparam: bad arguments (C % 4 == 0)");
  PSO_ARG_CHECK((((uintptr_t)x) & 7) == 0 && (((uintptr_t)dy) & 7) == 0 && (ldx % 4) == 0 && (lddy % 4) == 0,
                "pso_layer_norm_dparam: 8-B aligned rows");
  if (M == 0) return PSO_OK;
  if ((C % 8) == 0 && ((((uintptr_t)x) | ((uintptr_t)dy)) & 15) == 0 && (ldx % 8) == 0 && (lddy % 8) == 0 &&
      (((uintptr_t)stats) & 7) == 0) {
    const dim3 grid((C + 511) / 512, (M + CS2_ROWS - 1) / CS2_ROWS);
    ln_dparam8_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(M, C, (const bf16_t*)x, ldx, (const bf16_t*)dy, lddy,
                                                            stats, dgamma, dbeta);
    return pso_check_launch("pso_layer_norm_dparam");
  }
  const dim3 grid((C + 255) / 256, (M + CS_ROWS - 1) / CS_ROWS);
  ln_dparam_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(M, C, (const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, stats,
                                                         dgamma, dbeta);
  return pso_check_launch("pso_layer_norm_dparam");
}

static int colsum_nbg(long M, long rpg) { return (int)(((M < rpg ? M : rpg) + CS2_ROWS - 1) / CS2_ROWS); }

size_t pso_colsum_acc_ws_bytes(long M, int N, long rows_per_group) {
  if (M <= 0 || N <= 0 || rows_per_group <= 0) return 0;
  const long G = (M + rows_per_group - 1) / rows_per_group;
  int S, ch;
  ordered_reduce_plan(colsum_nbg(M, rows_per_group), S, ch);
  return (size_t)G * (colsum_nbg(M, rows_per_group) + S) * N * sizeof(float);
}

int pso_colsum_acc_ws(long M, int N, const void* x, long ldx, long rows_per_group, float* out, long ldo, void* ws,
                      size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(M >= 0 && N > 0 && x && out && rows_per_group > 0, "pso_colsum_acc_ws: bad arguments");
  if (M == 0) return PSO_OK;
  PSO_ARG_CHECK(ws && ws_bytes >= pso_colsum_acc_ws_bytes(M, N, rows_per_group), "pso_colsum_acc_ws: workspace");
  const long G = (M + rows_per_group - 1) / rows_per_group;
  const int nbg = colsum_nbg(M, rows_per_group);
  PSO_ARG_CHECK(G * nbg < 65536L * 1024, "pso_colsum_acc_ws: too many row blocks");
  const int vec = (N % 8) == 0 && (((uintptr_t)x) & 15) == 0 && (ldx % 8) == 0;
  const hipStream_t st = (hipStream_t)stream;
  colsum_part_kernel<<<dim3((N + 511) / 512, (unsigned)(G * nbg)), 256, 0, st>>>(M, N, (const bf16_t*)x, ldx,
                                                                                rows_per_group, nbg, vec, (float*)ws);
  int S, ch;
  ordered_reduce_plan(nbg, S, ch);
  float* p2 = (float*)ws + (size_t)G * nbg * N;
  if (ch == 1) p2 = (float*)ws;  // level 2 straight over the partials ([g][R][N] = [g][S][N])
  else ordered_reduce_l1_kernel<<<dim3((N + 255) / 256, S, (unsigned)G), 256, 0, st>>>(nbg, N, S, ch, (const float*)ws, p2);
  ordered_reduce_l2_kernel<<<(unsigned)((G * N + 255) / 256), 256, 0, st>>>((int)G, N, S, p2, out, ldo, nullptr, 0);
  return pso_check_launch("pso_colsum_acc_ws");
}

size_t pso_layer_norm_dparam_ws_bytes(int M, int C) {
  if (M <= 0 || C <= 0) return 0;
  const int nb = (M + CS2_ROWS - 1) / CS2_ROWS;
  int S, ch;
  ordered_reduce_plan(nb, S, ch);
  return (size_t)(nb + S) * 2 * C * sizeof(float);
}

int pso_layer_norm_dparam_ws(int M, int C, const void* x, long ldx, const void* dy, long lddy, const float* stats,
                             float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(M >= 0 && C > 0 && x && dy && stats && dgamma && dbeta, "pso_layer_norm_dparam_ws: bad arguments");
  if (M == 0) return PSO_OK;
  PSO_ARG_CHECK(ws && ws_bytes >= pso_layer_norm_dparam_ws_bytes(M, C), "pso_layer_norm_dparam_ws: workspace");
  const int nb = (M + CS2_ROWS - 1) / CS2_ROWS;
  const int vec = (C % 8) == 0 && ((((uintptr_t)x) | ((uintptr_t)dy)) & 15) == 0 && (ldx % 8) == 0 && (lddy % 8) == 0;
  const hipStream_t st = (hipStream_t)stream;
  ln_dparam_part_kernel<<<dim3((C + 511) / 512, nb), 256, 0, st>>>(M, C, (const bf16_t*)x, ldx, (const bf16_t*)dy,
                                                                  lddy, stats, vec, (float*)ws);
  int S, ch;
  ordered_reduce_plan(nb, S, ch);
  float* p2 = (float*)ws + (size_t)nb * 2 * C;
  if (ch == 1) p2 = (float*)ws;
  else ordered_reduce_l1_kernel<<<dim3((2 * C + 255) / 256, S, 1), 256, 0, st>>>(nb, 2 * C, S, ch, (const float*)ws, p2);
  ordered_reduce_l2_kernel<<<(2 * C + 255) / 256, 256, 0, st>>>(1, 2 * C, S, p2, dgamma, 0, dbeta, C);
  return pso_check_launch("pso_layer_norm_dparam_ws");
}

int pso_im2col_conv(int mode, int B, const void* src1, int C1, const void* src2, int C2, int H, int W, int Ho, int Wo,
                    int stride, int pad, void* out, long ldo, void* stream) {
  PSO_ARG_CHECK(B > 0 && src1 && out && C1 > 0 && (C1 % 8) == 0 && (C2 % 8) == 0 && (!C2 || src2) &&
                    (mode == PSO_CONV_NORMAL || mode == PSO_CONV_UP2) && ldo >= 9L * (C1 + C2) && (ldo % 8) == 0,
                "pso_im2col_conv: bad arguments (C1, C2 % 8 == 0; NORMAL or UP2; ldo >= 9 (C1 + C2))");
  PSO_ARG_CHECK((((uintptr_t)src1) & 15) == 0 && (!src2 || (((uintptr_t)src2) & 15) == 0) &&
                    (((uintptr_t)out) & 15) == 0,
                "pso_im2col_conv: 16-B aligned buffers");
  const long total = (long)B * Ho * Wo * 9 * ((C1 + C2) / 8);
  const unsigned blocks = (unsigned)((total + 255) / 256);
  im2col_conv_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(mode, B, (const bf16_t*)src1, C1, (const bf16_t*)src2,
                                                              C2, H, W, Ho, Wo, stride, pad, (bf16_t*)out, ldo);
  return pso_check_launch("pso_im2col_conv");
}

}  // extern "C"
