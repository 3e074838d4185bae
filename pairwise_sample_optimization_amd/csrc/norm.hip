// GroupNorm(+SiLU) and LayerNorm, forward and backward, on channels-last bf16 activations (fp32 statistics).
//
// Replaces the implicit norm kernels of the diffusers SDXL UNet/VAE (SURVEY §2 "GroupNorm(32) + SiLU", "LayerNorm"):
//   ResnetBlock2D.norm1/norm2 + SiLU, Transformer2DModel.norm (eps 1e-6), conv_norm_out + SiLU, VAE GroupNorms,
//   BasicTransformerBlock.norm1/2/3 (LayerNorm eps 1e-5).
//
// GroupNorm on NHWC: a group is Cg = C/G channels of every pixel of one image.  Each pass streams whole pixel rows
// (C contiguous channels -> 16-B coalesced loads; a group-major walk would read 20-B fragments at C=320):
//   partial  : block = (pixel chunk, image); thread (slot, 8-channel chunk) accumulates per-channel sums
//              fwd: (sum x, sum x^2)      bwd: (sum dz, sum dz*xhat)   -> ws [B][chunks][C][2] (fp32)
//   finalize : one thread per (image, group), fixed-order fp64 combine -> (mean, rstd) | (mean dxhat, mean dxhat*xhat)
//   apply    : element-wise, 8 channels per thread: y = silu?((x-mean)*rstd*gamma + beta)
//              dx = rstd*(dz*gamma - a - xhat*b) (+ residual gradient), dz = dy*silu'(z) when SiLU is fused.
// Backward also emits per-channel dgamma/dbeta partial sums (full-UNet gradients, config 3) when asked.
#include "common.h"

#define GN_ROWS 64  // pixels per partial / apply block
// Pixels per block of the forward passes above 256 blocks of GN_ROWS per image (HW > 16384: only the VAE's 256^2 -
// 1024^2 levels; every UNet GroupNorm has HW <= 128^2 and keeps GN_ROWS and its bits): 8x fewer partial rows for the
// finalize pass's serial combine, and 8x longer blocks (16 pixel rows per thread at C = 128 instead of 2); VAE decode
// 127.7 -> 113.0 ms per 8 images at 512 (256: 114.1-114.8, 1024: 113.3-113.7; profiles/r06_vae_groupnorm_ab.log)
#define GN_ROWS_BIG 512
static int gn_rows_fwd(int HW) { return (HW + GN_ROWS - 1) / GN_ROWS > 256 ? GN_ROWS_BIG : GN_ROWS; }

__device__ __forceinline__ void unpack8(uint4 v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bf2f(w[i] & 0xffff);
    f[2 * i + 1] = bf2f(w[i] >> 16);
  }
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

// ---------------------------------------------------------------------------------------------------------------
// partial sums.  BWD=false: (x) -> per group sum x, sum x^2.
//                BWD=true:  (x, dy, stats, gamma, beta) -> per group sum dz*gamma, sum dz*gamma*xhat
//                           (+ optional per-channel sum dz, sum dz*xhat for dbeta / dgamma)
// ws layout: [B][chunks][G][2] (+ per-channel [B][chunks][C][2] after it when DPARAM)
// ---------------------------------------------------------------------------------------------------------------
template <bool BWD, bool SILU>
__global__ void gn_partial_kernel(int HW, int rows, int C, int G, const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                  const float* __restrict__ stats, const bf16_t* __restrict__ gamma,
                                  const bf16_t* __restrict__ beta, float* __restrict__ ws, float* __restrict__ ws_ch) {
  extern __shared__ float red[];  // [RS][C][2]
  const int TPR = C / 8;
  const int RS = blockDim.x / TPR;
  const int slot = threadIdx.x / TPR, cc = threadIdx.x - slot * TPR;
  const int b = blockIdx.y, chunk = blockIdx.x, nchunks = gridDim.x;
  const int r0 = chunk * rows, r1 = min(HW, r0 + rows);
  const int Cg = C / G;
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  float mean[8], rstd[8], gm[8], bt[8];
  if (BWD && slot < RS) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = cc * 8 + j, g = c / Cg;
      mean[j] = stats[(b * G + g) * 2];
      rstd[j] = stats[(b * G + g) * 2 + 1];
      gm[j] = gamma ? bf2f(gamma[c]) : 1.f;
      bt[j] = beta ? bf2f(beta[c]) : 0.f;
    }
  }
  if (slot < RS) {
    for (int r = r0 + slot; r < r1; r += RS) {
      const size_t off = ((size_t)b * HW + r) * C + cc * 8;
      float xv[8];
      unpack8(*reinterpret_cast<const uint4*>(x + off), xv);
      if (!BWD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s1[j] += xv[j];
          s2[j] += xv[j] * xv[j];
        }
      } else {
        float dv[8];
        unpack8(*reinterpret_cast<const uint4*>(dy + off), dv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (xv[j] - mean[j]) * rstd[j];
          float dz = dv[j];
          if (SILU) {
            const float z = xh * gm[j] + bt[j];
            const float sg = sigmoidf_(z);
            dz *= sg * (1.f + z * (1.f - sg));
          }
          s1[j] += dz;
          s2[j] += dz * xh;
        }
      }
    }
  }
  if (slot < RS) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(slot * C + cc * 8 + j) * 2] = s1[j];
      red[(slot * C + cc * 8 + j) * 2 + 1] = s2[j];
    }
  }
  __syncthreads();
  // fold the row slots: per-channel sums back into slot 0
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f, q = 0.f;
    for (int s = 0; s < RS; ++s) {
      a += red[(s * C + c) * 2];
      q += red[(s * C + c) * 2 + 1];
    }
    if (ws_ch) {
      float* o = ws_ch + (((size_t)b * nchunks + chunk) * C + c) * 2;
      o[0] = a;
      o[1] = q;
    }
    if (BWD && gamma) {  // the group coefficients need gamma-weighted sums
      const float gmc = bf2f(gamma[c]);
      a *= gmc;
      q *= gmc;
    }
    red[c * 2] = a;
    red[c * 2 + 1] = q;
  }
  __syncthreads();
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    float a = 0.f, q = 0.f;
    for (int c = g * Cg; c < (g + 1) * Cg; ++c) {
      a += red[c * 2];
      q += red[c * 2 + 1];
    }
    float* o = ws + (((size_t)b * nchunks + chunk) * G + g) * 2;
    o[0] = a;
    o[1] = q;
  }
}

// one wave per (image, group): fixed-order fp64 combine over the chunks.
// FWD: stats = (mean, rstd).  BWD: coef = (mean(dz*gamma), mean(dz*gamma*xhat)).
template <bool BWD>
__global__ void gn_finalize_kernel(int B, int HW, int C, int G, int nchunks, float eps, const float* __restrict__ ws,
                                   float* __restrict__ out) {
  const int id = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (id >= B * G) return;
  const int b = id / G, g = id - b * G;
  const int Cg = C / G;
  double a = 0.0, q = 0.0;
  for (int k = lane; k < nchunks; k += 64) {
    const float* p = ws + (((size_t)b * nchunks + k) * G + g) * 2;
    a += p[0];
    q += p[1];
  }
  a = warp_sum_d(a);
  q = warp_sum_d(q);
  if (lane != 0) return;
  const double n = (double)HW * Cg;
  if (!BWD) {
    const double mean = a / n;
    double var = q / n - mean * mean;
    if (var < 0) var = 0;
    out[id * 2] = (float)mean;
    out[id * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
  } else {
    out[id * 2] = (float)(a / n);
    out[id * 2 + 1] = (float)(q / n);
  }
}

// per-channel dgamma/dbeta from the per-channel bwd partials (sum over images and chunks)
__global__ void gn_dparam_kernel(int B, int C, int nchunks, const float* __restrict__ ws, float* __restrict__ dgamma,
                                 float* __restrict__ dbeta, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double a = 0.0, q = 0.0;
  for (int b = 0; b < B; ++b)
    for (int k = 0; k < nchunks; ++k) {
      const float* p = ws + (((size_t)b * nchunks + k) * C + c) * 2;
      a += p[0];
      q += p[1];
    }
  if (dbeta) dbeta[c] = (accumulate ? dbeta[c] : 0.f) + (float)a;
  if (dgamma) dgamma[c] = (accumulate ? dgamma[c] : 0.f) + (float)q;
}

// The same sums spread over the chip: block (64 channels, split s of S) adds the (image, chunk) entries s, s + S, ...
// in 4 slices (fp64, summed in LDS) into part2[s][c][2] (doubles); gn_dparam_final_kernel adds the S partials per
// channel in fixed order.  (The one-pass form above runs C / 128 workgroups -- 3 for 320 channels -- each walking every
// entry: ~130 us per call in the full-UNet backward.)
__global__ __launch_bounds__(256) void gn_dparam_split_kernel(int BK, int C, int S, const float* __restrict__ ws,
                                                              double* __restrict__ part2) {
  __shared__ double red[4][64][2];
  const int t = threadIdx.x, tx = t & 63, ty = t >> 6;
  const int c = blockIdx.x * 64 + tx, sp = blockIdx.y;
  double a = 0.0, q = 0.0;
  if (c < C)
    for (int e = sp + S * ty; e < BK; e += 4 * S) {
      const float2 v = *reinterpret_cast<const float2*>(ws + ((size_t)e * C + c) * 2);
      a += v.x;
      q += v.y;
    }
  red[ty][tx][0] = a;
  red[ty][tx][1] = q;
  __syncthreads();
  if (ty == 0 && c < C) {
    part2[((size_t)sp * C + c) * 2] = red[0][tx][0] + red[1][tx][0] + red[2][tx][0] + red[3][tx][0];
    part2[((size_t)sp * C + c) * 2 + 1] = red[0][tx][1] + red[1][tx][1] + red[2][tx][1] + red[3][tx][1];
  }
}

__global__ void gn_dparam_final_kernel(int C, int S, const double* __restrict__ part2, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double a = 0.0, q = 0.0;
  for (int sp = 0; sp < S; ++sp) {
    a += part2[((size_t)sp * C + c) * 2];
    q += part2[((size_t)sp * C + c) * 2 + 1];
  }
  if (dbeta) dbeta[c] = (accumulate ? dbeta[c] : 0.f) + (float)a;
  if (dgamma) dgamma[c] = (accumulate ? dgamma[c] : 0.f) + (float)q;
}

// Apply passes: block = (pixel chunk of GN_ROWS, image) like the partial pass; thread (row slot, 8-channel chunk) folds
// mean / rstd / gamma / beta of its 8 channels into per-channel (scale, shift) once and streams its pixel rows with
// one FMA (+ SiLU) per element -- no per-element divisions or scalar parameter loads.
template <bool SILU>
__global__ void gn_apply_fwd_kernel(int HW, int rows, int C, int G, const bf16_t* __restrict__ x, const float* __restrict__ stats,
                                    const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta,
                                    bf16_t* __restrict__ y) {
  const int TPR = C / 8;
  const int RS = blockDim.x / TPR;
  const int slot = threadIdx.x / TPR, cc = threadIdx.x - slot * TPR;
  if (slot >= RS) return;
  const int b = blockIdx.y;
  const int r0 = blockIdx.x * rows, r1 = min(HW, r0 + rows);
  const int Cg = C / G;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cc * 8 + j, g = c / Cg;
    const float mean = stats[(b * G + g) * 2], rstd = stats[(b * G + g) * 2 + 1];
    const float gm = gamma ? bf2f(gamma[c]) : 1.f, bt = beta ? bf2f(beta[c]) : 0.f;
    sc[j] = rstd * gm;
    sh[j] = bt - mean * rstd * gm;
  }
  for (int r = r0 + slot; r < r1; r += RS) {
    const size_t off = ((size_t)b * HW + r) * C + cc * 8;
    float xv[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(x + off), xv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float z = fmaf(xv[j], sc[j], sh[j]);
      o[j] = SILU ? z * sigmoidf_(z) : z;
    }
    *reinterpret_cast<uint4*>(y + off) = pack8(o);
  }
}

// dx = rstd*(dz*gamma - ca - xhat*cb) (+ dadd), dz = dy * silu'(z) when SiLU is fused; per channel
// xhat = x*rstd - mean*rstd, z = x*(rstd*gamma) + (beta - mean*rstd*gamma), dx = P*dz + Q + R*xhat.
template <bool SILU>
__global__ void gn_apply_bwd_kernel(int HW, int C, int G, const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                    const float* __restrict__ stats, const float* __restrict__ coef,
                                    const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta,
                                    const bf16_t* __restrict__ dadd, bf16_t* __restrict__ dx) {
  const int TPR = C / 8;
  const int RS = blockDim.x / TPR;
  const int slot = threadIdx.x / TPR, cc = threadIdx.x - slot * TPR;
  if (slot >= RS) return;
  const int b = blockIdx.y;
  const int r0 = blockIdx.x * GN_ROWS, r1 = min(HW, r0 + GN_ROWS);
  const int Cg = C / G;
  float xs[8], xo[8], zs[8], zo[8], P[8], Q[8], R[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cc * 8 + j, g = c / Cg;
    const float mean = stats[(b * G + g) * 2], rstd = stats[(b * G + g) * 2 + 1];
    const float ca = coef[(b * G + g) * 2], cb = coef[(b * G + g) * 2 + 1];
    const float gm = gamma ? bf2f(gamma[c]) : 1.f, bt = beta ? bf2f(beta[c]) : 0.f;
    xs[j] = rstd;
    xo[j] = -mean * rstd;
    zs[j] = rstd * gm;
    zo[j] = bt - mean * rstd * gm;
    P[j] = rstd * gm;
    Q[j] = -rstd * ca;
    R[j] = -rstd * cb;
  }
  for (int r = r0 + slot; r < r1; r += RS) {
    const size_t off = ((size_t)b * HW + r) * C + cc * 8;
    float xv[8], dv[8], o[8], av[8];
    unpack8(*reinterpret_cast<const uint4*>(x + off), xv);
    unpack8(*reinterpret_cast<const uint4*>(dy + off), dv);
    if (dadd) unpack8(*reinterpret_cast<const uint4*>(dadd + off), av);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xh = fmaf(xv[j], xs[j], xo[j]);
      float dz = dv[j];
      if (SILU) {
        const float z = fmaf(xv[j], zs[j], zo[j]);
        const float sg = sigmoidf_(z);
        dz *= sg * (1.f + z * (1.f - sg));
      }
      o[j] = fmaf(P[j], dz, fmaf(R[j], xh, Q[j])) + (dadd ? av[j] : 0.f);
    }
    *reinterpret_cast<uint4*>(dx + off) = pack8(o);
  }
}

static int gn_block(int C) {
  const int TPR = C / 8;
  int rs = 1;
  while (TPR * rs * 2 <= 512) rs *= 2;
  return TPR * rs;
}


// ---------------------------------------------------------------------------------------------------------------
// LayerNorm over the last dim (one wave per row).  MAXV = 16-B chunks per lane (C <= 64*8*MAXV).
// ---------------------------------------------------------------------------------------------------------------
template <int MAXV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int M, int C, float eps, const bf16_t* __restrict__ x, long ldx,
                                                     const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta,
                                                     bf16_t* __restrict__ y, long ldy, float* __restrict__ stats) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const int C8 = C / 8;
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int ch = lane + 64 * i;
    if (ch < C8) {
      unpack8(*reinterpret_cast<const uint4*>(x + row * ldx + ch * 8), v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
  }
  const float mean = warp_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int ch = lane + 64 * i;
    if (ch < C8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(warp_sum(q) / C + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int ch = lane + 64 * i;
    if (ch < C8) {
      const uint4 gv = *reinterpret_cast<const uint4*>(gamma + ch * 8);
      const uint4 bv = *reinterpret_cast<const uint4*>(beta + ch * 8);
      float gf[8], bf[8], o[8];
      unpack8(gv, gf);
      unpack8(bv, bf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * gf[j] + bf[j];
      *reinterpret_cast<uint4*>(y + row * ldy + ch * 8) = pack8(o);
    }
  }
  if (stats && lane == 0) {
    stats[row * 2] = mean;
    stats[row * 2 + 1] = rstd;
  }
}

template <int MAXV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int M, int C, const bf16_t* __restrict__ x, long ldx,
                                                     const bf16_t* __restrict__ dy, long lddy,
                                                     const float* __restrict__ stats, const bf16_t* __restrict__ gamma,
                                                     const bf16_t* __restrict__ dadd, long ldadd,
                                                     bf16_t* __restrict__ dx, long lddx) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const int C8 = C / 8;
  const float mean = stats[row * 2], rstd = stats[row * 2 + 1];
  float xh[MAXV][8], g[MAXV][8];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int ch = lane + 64 * i;
    if (ch < C8) {
      float xv[8], dv[8], gf[8];
      unpack8(*reinterpret_cast<const uint4*>(x + row * ldx + ch * 8), xv);
      unpack8(*reinterpret_cast<const uint4*>(dy + row * lddy + ch * 8), dv);
      unpack8(*reinterpret_cast<const uint4*>(gamma + ch * 8), gf);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xh[i][j] = (xv[j] - mean) * rstd;
        g[i][j] = dv[j] * gf[j];
        s1 += g[i][j];
        s2 += g[i][j] * xh[i][j];
      }
    }
  }
  const float a = warp_sum(s1) / C, b = warp_sum(s2) / C;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int ch = lane + 64 * i;
    if (ch < C8) {
      float o[8], av[8];
      if (dadd) unpack8(*reinterpret_cast<const uint4*>(dadd + row * ldadd + ch * 8), av);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = rstd * (g[i][j] - a - xh[i][j] * b) + (dadd ? av[j] : 0.f);
      *reinterpret_cast<uint4*>(dx + row * lddx + ch * 8) = pack8(o);
    }
  }
}

extern "C" {

size_t pso_group_norm_ws_bytes(int B, int HW, int C) {
  // group partials (G <= C) + per-channel partials (dgamma/dbeta) + group coefficients
  return (size_t)B * cdiv(HW, GN_ROWS) * C * 2 * sizeof(float) * 2 + (size_t)B * C * 2 * sizeof(float);
}

int pso_group_norm_fwd(int B, int HW, int C, int G, float eps, const void* x, const void* gamma, const void* beta,
                       int silu, void* y, float* stats, void* ws, size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(B > 0 && HW > 0 && C > 0 && G > 0 && C % G == 0 && C % 8 == 0 && C <= 4096,
                "pso_group_norm_fwd: bad shape B=%d HW=%d C=%d G=%d", B, HW, C, G);
  PSO_ARG_CHECK(x && y && stats && ws, "pso_group_norm_fwd: null pointer");
  PSO_ARG_CHECK(ws_bytes >= pso_group_norm_ws_bytes(B, HW, C), "pso_group_norm_fwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int rows = gn_rows_fwd(HW);
  const int nchunks = cdiv(HW, rows);
  const int threads = gn_block(C);
  const size_t shm = (size_t)(threads / (C / 8)) * C * 2 * sizeof(float);
  gn_partial_kernel<false, false><<<dim3(nchunks, B), threads, shm, st>>>(HW, rows, C, G, (const bf16_t*)x, nullptr,
                                                                          nullptr, nullptr, nullptr, (float*)ws,
                                                                          nullptr);
  gn_finalize_kernel<false><<<cdiv(B * G, 4), 256, 0, st>>>(B, HW, C, G, nchunks, eps, (const float*)ws, stats);
  if (silu)
    gn_apply_fwd_kernel<true><<<dim3(nchunks, B), threads, 0, st>>>(HW, rows, C, G, (const bf16_t*)x, stats,
                                                                    (const bf16_t*)gamma, (const bf16_t*)beta,
                                                                    (bf16_t*)y);
  else
    gn_apply_fwd_kernel<false><<<dim3(nchunks, B), threads, 0, st>>>(HW, rows, C, G, (const bf16_t*)x, stats,
                                                                     (const bf16_t*)gamma, (const bf16_t*)beta,
                                                                     (bf16_t*)y);
  return pso_check_launch("pso_group_norm_fwd");
}

int pso_group_norm_bwd(int B, int HW, int C, int G, const void* x, const void* dy, const float* stats,
                       const void* gamma, const void* beta, int silu, const void* dadd, void* dx, float* dgamma,
                       float* dbeta, int accumulate_dparams, void* ws, size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(B > 0 && HW > 0 && C > 0 && G > 0 && C % G == 0 && C % 8 == 0 && C <= 4096,
                "pso_group_norm_bwd: bad shape");
  PSO_ARG_CHECK(x && dy && stats && dx && ws, "pso_group_norm_bwd: null pointer");
  PSO_ARG_CHECK(ws_bytes >= pso_group_norm_ws_bytes(B, HW, C), "pso_group_norm_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int nchunks = cdiv(HW, GN_ROWS);
  const int threads = gn_block(C);
  const size_t shm = (size_t)(threads / (C / 8)) * C * 2 * sizeof(float);
  const size_t half = (size_t)B * nchunks * C * 2;
  float* part = (float*)ws;                       // [B][chunks][G][2]
  float* part_ch = (dgamma || dbeta) ? part + half : nullptr;  // [B][chunks][C][2]
  float* coef = part + 2 * half;                  // [B][G][2]
  const bf16_t *xp = (const bf16_t*)x, *dyp = (const bf16_t*)dy, *gp = (const bf16_t*)gamma,
               *bp = (const bf16_t*)beta;
  if (silu)
    gn_partial_kernel<true, true><<<dim3(nchunks, B), threads, shm, st>>>(HW, GN_ROWS, C, G, xp, dyp, stats, gp, bp,
                                                                          part, part_ch);
  else
    gn_partial_kernel<true, false><<<dim3(nchunks, B), threads, shm, st>>>(HW, GN_ROWS, C, G, xp, dyp, stats, gp, bp,
                                                                           part, part_ch);
  gn_finalize_kernel<true><<<cdiv(B * G, 4), 256, 0, st>>>(B, HW, C, G, nchunks, 0.f, part, coef);
  if (dgamma || dbeta) {
    // the group partials (part) are consumed by gn_finalize above: their space takes the split sums (S <= B*chunks/2
    // doubles per channel pair fit in B*chunks*C*2 floats)
    const int BK = B * nchunks, S = BK >= 64 ? 32 : BK / 2;
    if (S >= 2) {
      gn_dparam_split_kernel<<<dim3(cdiv(C, 64), S), 256, 0, st>>>(BK, C, S, part_ch, (double*)part);
      gn_dparam_final_kernel<<<cdiv(C, 128), 128, 0, st>>>(C, S, (const double*)part, dgamma, dbeta,
                                                           accumulate_dparams);
    } else {
      gn_dparam_kernel<<<cdiv(C, 128), 128, 0, st>>>(B, C, nchunks, part_ch, dgamma, dbeta, accumulate_dparams);
    }
  }
  if (silu)
    gn_apply_bwd_kernel<true><<<dim3(nchunks, B), threads, 0, st>>>(HW, C, G, xp, dyp, stats, coef, gp, bp,
                                                                    (const bf16_t*)dadd, (bf16_t*)dx);
  else
    gn_apply_bwd_kernel<false><<<dim3(nchunks, B), threads, 0, st>>>(HW, C, G, xp, dyp, stats, coef, gp, bp,
                                                                     (const bf16_t*)dadd, (bf16_t*)dx);
  return pso_check_launch("pso_group_norm_bwd");
}

int pso_layer_norm_fwd(int M, int C, float eps, const void* x, long ldx, const void* gamma, const void* beta, void* y,
                       long ldy, float* stats, void* stream) {
  PSO_ARG_CHECK(M >= 0 && C > 0 && C % 8 == 0 && C <= 64 * 8 * 4, "pso_layer_norm_fwd: C=%d unsupported", C);
  PSO_ARG_CHECK(x && y && gamma && beta, "pso_layer_norm_fwd: null pointer");
  if (M == 0) return PSO_OK;
  hipStream_t st = (hipStream_t)stream;
  const int C8 = C / 8;
  const int grid = cdiv(M, 4);
  if (C8 <= 64)
    ln_fwd_kernel<1><<<grid, 256, 0, st>>>(M, C, eps, (const bf16_t*)x, ldx, (const bf16_t*)gamma,
                                          (const bf16_t*)beta, (bf16_t*)y, ldy, stats);
  else if (C8 <= 128)
    ln_fwd_kernel<2><<<grid, 256, 0, st>>>(M, C, eps, (const bf16_t*)x, ldx, (const bf16_t*)gamma,
                                          (const bf16_t*)beta, (bf16_t*)y, ldy, stats);
  else
    ln_fwd_kernel<4><<<grid, 256, 0, st>>>(M, C, eps, (const bf16_t*)x, ldx, (const bf16_t*)gamma,
                                          (const bf16_t*)beta, (bf16_t*)y, ldy, stats);
  return pso_check_launch("pso_layer_norm_fwd");
}

int pso_layer_norm_bwd(int M, int C, const void* x, long ldx, const void* dy, long lddy, const float* stats,
                       const void* gamma, const void* dadd, long ldadd, void* dx, long lddx, void* stream) {
  PSO_ARG_CHECK(M >= 0 && C > 0 && C % 8 == 0 && C <= 64 * 8 * 4, "pso_layer_norm_bwd: C=%d unsupported", C);
  PSO_ARG_CHECK(x && dy && stats && gamma && dx, "pso_layer_norm_bwd: null pointer");
  if (M == 0) return PSO_OK;
  hipStream_t st = (hipStream_t)stream;
  const int C8 = C / 8;
  const int grid = cdiv(M, 4);
  if (C8 <= 64)
    ln_bwd_kernel<1><<<grid, 256, 0, st>>>(M, C, (const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, stats,
                                          (const bf16_t*)gamma, (const bf16_t*)dadd, ldadd, (bf16_t*)dx, lddx);
  else if (C8 <= 128)
    ln_bwd_kernel<2><<<grid, 256, 0, st>>>(M, C, (const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, stats,
                                          (const bf16_t*)gamma, (const bf16_t*)dadd, ldadd, (bf16_t*)dx, lddx);
  else
    ln_bwd_kernel<4><<<grid, 256, 0, st>>>(M, C, (const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, stats,
                                          (const bf16_t*)gamma, (const bf16_t*)dadd, ldadd, (bf16_t*)dx, lddx);
  return pso_check_launch("pso_layer_norm_bwd");
}

}  // extern "C"
