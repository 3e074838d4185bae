// Element-wise and data-movement kernels of the UNet / VAE hot path (bf16, 16-B vector access).
//
//   GEGLU fwd/bwd         diffusers GEGLU (FeedForward.net[0]): h, gate = proj(x).chunk(2); h * gelu(gate) (erf gelu)
//   SiLU                  nonlinearity applied to the time embedding before every time_emb_proj (ResnetBlock2D)
//   timestep embedding    diffusers Timesteps(flip_sin_to_cos=True, downscale_freq_shift=0) for time_proj and
//                         add_time_proj (UNet2DConditionModel.forward, SDXL "text_time" added condition)
//   transpose             [R][C] -> [C][R] bf16 (operands of the reduction-over-tokens GEMMs in backward)
//   im2col (small C)      conv_in (C=4) and the input-gradient of conv_out (C=4) as plain GEMMs
//   sum-pool 2x2          input-gradient of the nearest-2x upsample of Upsample2D
//   add / scale / cast    gradient merges, fp32 -> bf16 casts
#include "common.h"

__device__ __forceinline__ void unpack8e(uint4 v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bf2f(w[i] & 0xffff);
    f[2 * i + 1] = bf2f(w[i] >> 16);
  }
}
__device__ __forceinline__ uint4 pack8e(const float* f) {
  return make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
}

static int grid_for(long n, int per_thread = 1) {
  long g = (n / per_thread + 255) / 256;
  if (g > 8192) g = 8192;
  return (int)(g < 1 ? 1 : g);
}

#define GRID_STRIDE(i, n) for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (n); i += (long)gridDim.x * blockDim.x)


// in [M][ld_in] holding [h | gate] (F each); out [M][F] = h * gelu(gate)
__global__ void geglu_fwd_kernel(long M, int F, const bf16_t* __restrict__ in, long ldi, bf16_t* __restrict__ out,
                                 long ldo) {
  const int F8 = F / 8;
  GRID_STRIDE(v, M * F8) {
    const long m = v / F8;
    const int c = (int)(v - m * F8) * 8;
    float h[8], g[8], o[8];
    unpack8e(*reinterpret_cast<const uint4*>(in + m * ldi + c), h);
    unpack8e(*reinterpret_cast<const uint4*>(in + m * ldi + F + c), g);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = h[j] * gelu_erf(g[j]);
    *reinterpret_cast<uint4*>(out + m * ldo + c) = pack8e(o);
  }
}

// dout [M][F] -> din [M][2F] = [dout*gelu(g) | dout*h*gelu'(g)]
__global__ void geglu_bwd_kernel(long M, int F, const bf16_t* __restrict__ in, long ldi,
                                 const bf16_t* __restrict__ dout, long lddo, bf16_t* __restrict__ din, long lddi) {
  const int F8 = F / 8;
  GRID_STRIDE(v, M * F8) {
    const long m = v / F8;
    const int c = (int)(v - m * F8) * 8;
    float h[8], g[8], d[8], dh[8], dg[8];
    unpack8e(*reinterpret_cast<const uint4*>(in + m * ldi + c), h);
    unpack8e(*reinterpret_cast<const uint4*>(in + m * ldi + F + c), g);
    unpack8e(*reinterpret_cast<const uint4*>(dout + m * lddo + c), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float c, e;
      gelu_erf_parts(g[j], c, e);
      dh[j] = d[j] * g[j] * c;
      dg[j] = d[j] * h[j] * (c + 0.39894228040143268f * g[j] * e);
    }
    *reinterpret_cast<uint4*>(din + m * lddi + c) = pack8e(dh);
    *reinterpret_cast<uint4*>(din + m * lddi + F + c) = pack8e(dg);
  }
}

__global__ void silu_kernel(long n8, const bf16_t* __restrict__ x, bf16_t* __restrict__ y) {
  GRID_STRIDE(v, n8) {
    float a[8];
    unpack8e(*reinterpret_cast<const uint4*>(x + v * 8), a);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = a[j] / (1.f + __expf(-a[j]));
    *reinterpret_cast<uint4*>(y + v * 8) = pack8e(a);
  }
}

// t [n] (fp32) -> out [n][dim] (bf16 at column offset out_col, row stride ldo): [cos(t*f) | sin(t*f)],
// f_i = exp(-ln(10000) * i / half)   (flip_sin_to_cos=True, downscale_freq_shift=0, scale=1)
__global__ void timestep_embed_kernel(int n, int dim, const float* __restrict__ t, bf16_t* __restrict__ out, long ldo,
                                      int out_col) {
  const int half = dim / 2;
  GRID_STRIDE(i, (long)n * half) {
    const int r = (int)(i / half), k = (int)(i - (long)r * half);
    const float expo = -9.210340371976184f * (float)k / (float)half;  // -ln(10000)*k/half
    const float arg = t[r] * expf(expo);
    out[(long)r * ldo + out_col + k] = f2bf(cosf(arg));
    out[(long)r * ldo + out_col + half + k] = f2bf(sinf(arg));
  }
}

// 64x64 tiled transpose, bf16: in [R][C] (ldi) -> out [C][Rp] (ldo); rows R..Rp-1 of the input read as zero
// one 64 x 64 tile of out [C][Rp] = in [R][C]^T (rows >= R zero): rows read as 16-B chunks where the view allows (C,
// ldi multiples of 8, 16-B base), written back as 64 consecutive 2-B elements per output row
__device__ __forceinline__ void transpose_tile(int R, int Rp, int C, const bf16_t* __restrict__ in, long ldi,
                                               bf16_t* __restrict__ out, long ldo, int r0, int c0,
                                               bf16_t (*tile)[72]) {
  const int t = threadIdx.x;
  const bool vec = (C % 8) == 0 && (ldi % 8) == 0 && (reinterpret_cast<uintptr_t>(in) & 15) == 0;
  for (int q = t; q < 64 * 8; q += 256) {
    const int i = q >> 3, c = (q & 7) * 8, r = r0 + i;
    const bf16_t* src = in + (long)r * ldi + c0 + c;
    if (vec && r < R && c0 + c + 8 <= C) {
      *reinterpret_cast<uint4*>(&tile[i][c]) = *reinterpret_cast<const uint4*>(src);
    } else {
      for (int e = 0; e < 8; ++e) tile[i][c + e] = (r < R && c0 + c + e < C) ? src[e] : (bf16_t)0;
    }
  }
  __syncthreads();
  const int tx = t & 63, ty = t >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (c < C && r < Rp) out[(long)c * ldo + r] = tile[tx][i];
  }
}

__global__ __launch_bounds__(256) void transpose_kernel(int R, int Rp, int C, const bf16_t* __restrict__ in, long ldi,
                                                        bf16_t* __restrict__ out, long ldo) {
  __shared__ bf16_t tile[64][72];
  transpose_tile(R, Rp, C, in, ldi, out, ldo, blockIdx.y * 64, blockIdx.x * 64, tile);
}

// many transposes of different shapes in ONE launch (the full-UNet step rebuilds ~460 transposed weights after every
// optimizer step): a flat grid over all their 64 x 64 tiles; each workgroup finds its matrix by a binary search over
// the tile offsets (uniform across the workgroup: scalar loads)
struct TransposeMultiDesc {
  const bf16_t* src;
  bf16_t* dst;
  long ldi, ldo;
  int R, C, tiles_c, tile0;
};
static_assert(sizeof(TransposeMultiDesc) == 48, "descriptor layout shared with kernels.py");

__global__ __launch_bounds__(256) void transpose_multi_kernel(int n, const TransposeMultiDesc* __restrict__ d) {
  __shared__ bf16_t tile[64][72];
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].tile0 <= b) lo = mid;
    else hi = mid - 1;
  }
  const TransposeMultiDesc t = d[lo];
  const int k = b - t.tile0, tr = k / t.tiles_c, tc = k - tr * t.tiles_c;
  transpose_tile(t.R, t.R, t.C, t.src, t.ldi, t.dst, t.ldo, tr * 64, tc * 64, tile);
}

// NHWC small-channel im2col for 3x3/pad 1/stride 1: in [B][H][W][C] -> out [B*H*W][Kp] (Kp >= 9C, zero padded),
// column order (kh, kw, c) to match [Cout][kh][kw][C] weights.
__global__ void im2col3_kernel(int B, int H, int W, int C, const bf16_t* __restrict__ in, int flip,
                               bf16_t* __restrict__ out, int Kp) {
  GRID_STRIDE(i, (long)B * H * W * Kp) {
    const long pix = i / Kp;
    const int k = (int)(i - pix * Kp);
    bf16_t v = 0;
    if (k < 9 * C) {
      const int tap = k / C, c = k - tap * C;
      const int kh = tap / 3, kw = tap - kh * 3;
      const int b = (int)(pix / ((long)H * W));
      const int rem = (int)(pix - (long)b * H * W);
      const int y = rem / W, x = rem - y * W;
      const int iy = y + kh - 1, ix = x + kw - 1;
      if (iy >= 0 && iy < H && ix >= 0 && ix < W) v = in[(((long)b * H + iy) * W + ix) * C + c];
    }
    out[i] = v;
  }
}

// upsample-2x input gradient: in [B][2H][2W][C] -> out [B][H][W][C] = sum of the 2x2 block (+ dadd)
__global__ void sumpool2_kernel(int B, int H, int W, int C, const bf16_t* __restrict__ in,
                                const bf16_t* __restrict__ dadd, bf16_t* __restrict__ out) {
  const int C8 = C / 8;
  GRID_STRIDE(v, (long)B * H * W * C8) {
    const long pix = v / C8;
    const int c = (int)(v - pix * C8) * 8;
    const int b = (int)(pix / ((long)H * W));
    const int rem = (int)(pix - (long)b * H * W);
    const int y = rem / W, x = rem - y * W;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        float a[8];
        unpack8e(*reinterpret_cast<const uint4*>(in + (((long)b * 2 * H + 2 * y + dy) * 2 * W + 2 * x + dx) * C + c), a);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += a[j];
      }
    if (dadd) {
      float a[8];
      unpack8e(*reinterpret_cast<const uint4*>(dadd + pix * C + c), a);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += a[j];
    }
    *reinterpret_cast<uint4*>(out + pix * C + c) = pack8e(acc);
  }
}

// y = a*x + b*z (bf16 in, bf16 out); z may be null
__global__ void axpby_kernel(long n8, float a, const bf16_t* __restrict__ x, float b, const bf16_t* __restrict__ z,
                             bf16_t* __restrict__ y) {
  GRID_STRIDE(v, n8) {
    float p[8], q[8];
    unpack8e(*reinterpret_cast<const uint4*>(x + v * 8), p);
    if (z) unpack8e(*reinterpret_cast<const uint4*>(z + v * 8), q);
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = a * p[j] + (z ? b * q[j] : 0.f);
    *reinterpret_cast<uint4*>(y + v * 8) = pack8e(p);
  }
}

// casts: 8 elements per thread (32-B / 16-B accesses) where both buffers are 16-B aligned, scalar otherwise and for
// the ragged tail
__global__ void cast_f32_bf16_kernel(long n, const float* __restrict__ x, float scale, bf16_t* __restrict__ y) {
  long done = 0;
  if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0) {
    done = n & ~7L;
    GRID_STRIDE(v, n >> 3) {
      const float4 a = reinterpret_cast<const float4*>(x)[2 * v], b = reinterpret_cast<const float4*>(x)[2 * v + 1];
      reinterpret_cast<uint4*>(y)[v] = make_uint4(pack2bf(a.x * scale, a.y * scale), pack2bf(a.z * scale, a.w * scale),
                                                  pack2bf(b.x * scale, b.y * scale), pack2bf(b.z * scale, b.w * scale));
    }
  }
  GRID_STRIDE(i, n - done) y[done + i] = f2bf(x[done + i] * scale);
}
__global__ void cast_bf16_f32_kernel(long n, const bf16_t* __restrict__ x, float* __restrict__ y) {
  long done = 0;
  if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0) {
    done = n & ~7L;
    GRID_STRIDE(v, n >> 3) {
      const uint4 u = reinterpret_cast<const uint4*>(x)[v];
      reinterpret_cast<float4*>(y)[2 * v] = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                                        __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
      reinterpret_cast<float4*>(y)[2 * v + 1] = make_float4(__uint_as_float(u.z << 16), __uint_as_float(u.z & 0xffff0000u),
                                                            __uint_as_float(u.w << 16), __uint_as_float(u.w & 0xffff0000u));
    }
  }
  GRID_STRIDE(i, n - done) y[done + i] = bf2f(x[done + i]);
}

// conv weight [Co][kh][kw][Ci] -> input-gradient weight [Ci][kh'][kw'][Co]; flip=1: kh'=ks-1-kh (stride-1 bwd).
// Per tap this is a [Co][Ci] -> [Ci][Co] transpose of a strided view: 64 x 64 tiles through LDS, one tap per
// blockIdx.z, 16-B reads along Ci and 2-B writes along Co by 64 consecutive lanes (was one scattered 2-B store per
// element, Co elements apart).
__global__ __launch_bounds__(256) void conv_weight_t_kernel(int Co, int ks, int Ci, int flip,
                                                            const bf16_t* __restrict__ w, bf16_t* __restrict__ wt) {
  __shared__ bf16_t tile[64][72];  // [co][ci], 144-B pitch
  const int tap = blockIdx.z, kh = tap / ks, kw = tap - kh * ks;
  const int tap2 = flip ? (ks - 1 - kh) * ks + (ks - 1 - kw) : tap;
  const int ci0 = blockIdx.x * 64, co0 = blockIdx.y * 64, t = threadIdx.x;
  const long ldw = (long)ks * ks * Ci;
  const bool vec = (Ci % 8) == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0;
  for (int q = t; q < 64 * 8; q += 256) {  // 64 rows (co) x 8 chunks of 8 ci
    const int r = q >> 3, c = (q & 7) * 8, co = co0 + r, ci = ci0 + c;
    const bf16_t* src = w + co * ldw + (long)tap * Ci + ci;
    if (vec && co < Co && ci + 8 <= Ci) {
      *reinterpret_cast<uint4*>(&tile[r][c]) = *reinterpret_cast<const uint4*>(src);
    } else {
      for (int e = 0; e < 8; ++e) tile[r][c + e] = (co < Co && ci + e < Ci) ? src[e] : (bf16_t)0;
    }
  }
  __syncthreads();
  const int lx = t & 63, ly = t >> 6;
  for (int i = ly; i < 64; i += 4) {  // output row ci0 + i, 64 consecutive co
    const int ci = ci0 + i, co = co0 + lx;
    if (ci < Ci && co < Co) wt[((long)ci * ks * ks + tap2) * Co + co] = tile[lx][i];
  }
}

// out [npix][C1+C2] = [x1 | x2]  (torch.cat(dim=1) of NCHW == channel concat of NHWC rows)
__global__ void concat_kernel(long npix, int C1, const bf16_t* __restrict__ x1, int C2, const bf16_t* __restrict__ x2,
                              bf16_t* __restrict__ out) {
  const int C8 = (C1 + C2) / 8, c18 = C1 / 8;
  GRID_STRIDE(v, npix * C8) {
    const long p = v / C8;
    const int ch = (int)(v - p * C8);
    const uint4 val = ch < c18 ? *reinterpret_cast<const uint4*>(x1 + p * C1 + ch * 8)
                               : *reinterpret_cast<const uint4*>(x2 + p * C2 + (ch - c18) * 8);
    *reinterpret_cast<uint4*>(out + v * 8) = val;
  }
}

// inverse of concat, with optional accumulation of the second part into an existing gradient (d_skip += ...)
__global__ void split_kernel(long npix, int C1, int C2, const bf16_t* __restrict__ in, bf16_t* __restrict__ y1,
                             bf16_t* __restrict__ y2, const bf16_t* __restrict__ add2) {
  const int C8 = (C1 + C2) / 8, c18 = C1 / 8;
  GRID_STRIDE(v, npix * C8) {
    const long p = v / C8;
    const int ch = (int)(v - p * C8);
    const uint4 val = *reinterpret_cast<const uint4*>(in + v * 8);
    if (ch < c18) {
      *reinterpret_cast<uint4*>(y1 + p * C1 + ch * 8) = val;
    } else {
      bf16_t* o = y2 + p * C2 + (ch - c18) * 8;
      if (add2) {
        float a[8], b[8];
        unpack8e(val, a);
        unpack8e(*reinterpret_cast<const uint4*>(add2 + p * C2 + (ch - c18) * 8), b);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] += b[j];
        *reinterpret_cast<uint4*>(o) = pack8e(a);
      } else {
        *reinterpret_cast<uint4*>(o) = val;
      }
    }
  }
}

// NCHW (fp32 or bf16) -> NHWC bf16, and back (fp32 or bf16 out).  Small tensors (latents): plain element mapping.
__global__ void nchw_to_nhwc_kernel(int B, int C, int Cp, long HW, const void* __restrict__ src, int src_f32,
                                    float scale, bf16_t* __restrict__ dst) {
  GRID_STRIDE(i, (long)B * Cp * HW) {
    const int c = (int)(i % Cp);
    const long p = (i / Cp) % HW;
    const int b = (int)(i / (Cp * HW));
    const long s = ((long)b * C + c) * HW + p;
    float v = 0.f;
    if (c < C) v = src_f32 ? reinterpret_cast<const float*>(src)[s] : bf2f(reinterpret_cast<const bf16_t*>(src)[s]);
    dst[i] = f2bf(v * scale);
  }
}
__global__ void nhwc_to_nchw_kernel(int B, int C, long HW, const bf16_t* __restrict__ src, void* __restrict__ dst,
                                    int dst_f32) {
  GRID_STRIDE(i, (long)B * C * HW) {
    const long p = i % HW;
    const int c = (int)((i / HW) % C);
    const int b = (int)(i / (C * HW));
    const bf16_t v = src[((long)b * HW + p) * C + c];
    if (dst_f32) reinterpret_cast<float*>(dst)[i] = bf2f(v);
    else reinterpret_cast<bf16_t*>(dst)[i] = v;
  }
}

// many small transposes in one launch: grid (64x64 tiles of the largest matrix, n matrices)
struct TransposeDesc {
  const bf16_t* src;
  bf16_t* dst;
  int R, C;
  long ldi, ldo;
};
__global__ void transpose_batched_kernel(const TransposeDesc* __restrict__ d) {
  __shared__ bf16_t tile[64][66];
  const TransposeDesc t = d[blockIdx.z];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  if (r0 >= t.R || c0 >= t.C) return;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < t.R && c < t.C) ? t.src[(long)r * t.ldi + c] : (bf16_t)0;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (c < t.C && r < t.R) t.dst[(long)c * t.ldo + r] = tile[tx][i];
  }
}

// dst[i] = src[idx[i]] for rows of `units` elements of type U (16-B units when the row size allows, else 4-B)
template <typename U>
__global__ void gather_rows_kernel(long n, long units, const U* __restrict__ src, const int64_t* __restrict__ idx,
                                   U* __restrict__ dst) {
  GRID_STRIDE(i, n * units) {
    const long r = i / units, c = i - r * units;
    dst[i] = src[idx[r] * units + c];
  }
}

// in-place row softmax of bf16 scores (fp32 math): one 256-thread block per row, 3 passes over the (L2-resident) row
__global__ __launch_bounds__(256) void softmax_rows_kernel(int N, bf16_t* __restrict__ x, long ld) {
  __shared__ float red[4];
  bf16_t* row = x + blockIdx.x * ld;
  float mx = -INFINITY;
  for (int c = threadIdx.x * 8; c < N; c += 256 * 8) {
    float a[8];
    unpack8e(*reinterpret_cast<const uint4*>(row + c), a);
#pragma unroll
    for (int j = 0; j < 8; ++j) mx = fmaxf(mx, a[j]);
  }
  mx = warp_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int c = threadIdx.x * 8; c < N; c += 256 * 8) {
    float a[8];
    unpack8e(*reinterpret_cast<const uint4*>(row + c), a);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(a[j] - mx);
  }
  s = warp_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const float inv = 1.f / (red[0] + red[1] + red[2] + red[3]);
  for (int c = threadIdx.x * 8; c < N; c += 256 * 8) {
    float a[8];
    unpack8e(*reinterpret_cast<const uint4*>(row + c), a);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = __expf(a[j] - mx) * inv;
    *reinterpret_cast<uint4*>(row + c) = pack8e(a);
  }
}

extern "C" {

int pso_softmax_rows(int M, int N, void* x, long ld, void* stream) {
  PSO_ARG_CHECK(N % 8 == 0 && ld % 8 == 0 && x, "pso_softmax_rows: N, ld multiples of 8");
  softmax_rows_kernel<<<M, 256, 0, (hipStream_t)stream>>>(N, (bf16_t*)x, ld);
  return pso_check_launch("pso_softmax_rows");
}

int pso_transpose_batched(int n, const void* descs, int max_r, int max_c, void* stream) {
  PSO_ARG_CHECK(n > 0 && descs, "pso_transpose_batched: bad args");
  dim3 grid(cdiv(max_c, 64), cdiv(max_r, 64), n);
  transpose_batched_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((const TransposeDesc*)descs);
  return pso_check_launch("pso_transpose_batched");
}

int pso_gather_rows(long n, long row_bytes, const void* src, const int64_t* idx, void* dst, void* stream) {
  PSO_ARG_CHECK(row_bytes % 4 == 0 && src && idx && dst, "pso_gather_rows: row_bytes %% 4");
  if (row_bytes % 16 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0)
    gather_rows_kernel<uint4><<<grid_for(n * (row_bytes / 16)), 256, 0, (hipStream_t)stream>>>(
        n, row_bytes / 16, (const uint4*)src, idx, (uint4*)dst);
  else
    gather_rows_kernel<uint32_t><<<grid_for(n * (row_bytes / 4)), 256, 0, (hipStream_t)stream>>>(
        n, row_bytes / 4, (const uint32_t*)src, idx, (uint32_t*)dst);
  return pso_check_launch("pso_gather_rows");
}

int pso_nchw_to_nhwc(int B, int C, int Cp, long HW, const void* src, int src_dtype, float scale, void* dst,
                     void* stream) {
  PSO_ARG_CHECK(src && dst && Cp >= C && (src_dtype == PSO_F32 || src_dtype == PSO_BF16), "pso_nchw_to_nhwc: bad args");
  nchw_to_nhwc_kernel<<<grid_for((long)B * Cp * HW), 256, 0, (hipStream_t)stream>>>(
      B, C, Cp, HW, src, src_dtype == PSO_F32, scale, (bf16_t*)dst);
  return pso_check_launch("pso_nchw_to_nhwc");
}

int pso_nhwc_to_nchw(int B, int C, long HW, const void* src, void* dst, int dst_dtype, void* stream) {
  PSO_ARG_CHECK(src && dst && (dst_dtype == PSO_F32 || dst_dtype == PSO_BF16), "pso_nhwc_to_nchw: bad args");
  nhwc_to_nchw_kernel<<<grid_for((long)B * C * HW), 256, 0, (hipStream_t)stream>>>(B, C, HW, (const bf16_t*)src,
                                                                                  dst, dst_dtype == PSO_F32);
  return pso_check_launch("pso_nhwc_to_nchw");
}

int pso_concat_channels(long npix, int C1, const void* x1, int C2, const void* x2, void* out, void* stream) {
  PSO_ARG_CHECK(C1 % 8 == 0 && C2 % 8 == 0 && x1 && x2 && out, "pso_concat_channels: C %% 8");
  concat_kernel<<<grid_for(npix * (C1 + C2) / 8), 256, 0, (hipStream_t)stream>>>(
      npix, C1, (const bf16_t*)x1, C2, (const bf16_t*)x2, (bf16_t*)out);
  return pso_check_launch("pso_concat_channels");
}

int pso_split_channels(long npix, int C1, int C2, const void* in, void* y1, void* y2, const void* add2,
                       void* stream) {
  PSO_ARG_CHECK(C1 % 8 == 0 && C2 % 8 == 0 && in && y1 && y2, "pso_split_channels: C %% 8");
  split_kernel<<<grid_for(npix * (C1 + C2) / 8), 256, 0, (hipStream_t)stream>>>(
      npix, C1, C2, (const bf16_t*)in, (bf16_t*)y1, (bf16_t*)y2, (const bf16_t*)add2);
  return pso_check_launch("pso_split_channels");
}

int pso_geglu_fwd(long M, int F, const void* in, long ldi, void* out, long ldo, void* stream) {
  PSO_ARG_CHECK(F % 8 == 0 && ldi % 8 == 0 && ldo % 8 == 0 && in && out, "pso_geglu_fwd: bad args");
  geglu_fwd_kernel<<<grid_for(M * (F / 8)), 256, 0, (hipStream_t)stream>>>(M, F, (const bf16_t*)in, ldi,
                                                                          (bf16_t*)out, ldo);
  return pso_check_launch("pso_geglu_fwd");
}

int pso_geglu_bwd(long M, int F, const void* in, long ldi, const void* dout, long lddo, void* din, long lddi,
                  void* stream) {
  PSO_ARG_CHECK(F % 8 == 0 && ldi % 8 == 0 && lddo % 8 == 0 && lddi % 8 == 0 && in && dout && din,
                "pso_geglu_bwd: bad args");
  geglu_bwd_kernel<<<grid_for(M * (F / 8)), 256, 0, (hipStream_t)stream>>>(M, F, (const bf16_t*)in, ldi,
                                                                          (const bf16_t*)dout, lddo, (bf16_t*)din,
                                                                          lddi);
  return pso_check_launch("pso_geglu_bwd");
}

int pso_silu(long n, const void* x, void* y, void* stream) {
  PSO_ARG_CHECK(n % 8 == 0 && x && y, "pso_silu: n must be a multiple of 8");
  silu_kernel<<<grid_for(n / 8), 256, 0, (hipStream_t)stream>>>(n / 8, (const bf16_t*)x, (bf16_t*)y);
  return pso_check_launch("pso_silu");
}

int pso_timestep_embedding(int n, int dim, const float* t, void* out, long ldo, int out_col, void* stream) {
  PSO_ARG_CHECK(dim % 2 == 0 && t && out, "pso_timestep_embedding: bad args");
  timestep_embed_kernel<<<grid_for((long)n * dim / 2), 256, 0, (hipStream_t)stream>>>(n, dim, t, (bf16_t*)out, ldo,
                                                                                      out_col);
  return pso_check_launch("pso_timestep_embedding");
}

int pso_transpose_multi(int n, const void* descs, int total_tiles, void* stream) {
  PSO_ARG_CHECK(n > 0 && descs && total_tiles > 0, "pso_transpose_multi: bad args");
  transpose_multi_kernel<<<total_tiles, 256, 0, (hipStream_t)stream>>>(n, (const TransposeMultiDesc*)descs);
  return pso_check_launch("pso_transpose_multi");
}

int pso_transpose(int R, int Rp, int C, const void* in, long ldi, void* out, long ldo, void* stream) {
  PSO_ARG_CHECK(in && out && Rp >= R, "pso_transpose: bad args");
  dim3 grid(cdiv(C, 64), cdiv(Rp, 64));
  transpose_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(R, Rp, C, (const bf16_t*)in, ldi, (bf16_t*)out, ldo);
  return pso_check_launch("pso_transpose");
}

int pso_im2col3(int B, int H, int W, int C, const void* in, void* out, int Kp, void* stream) {
  PSO_ARG_CHECK(Kp >= 9 * C && in && out, "pso_im2col3: Kp < 9C");
  im2col3_kernel<<<grid_for((long)B * H * W * Kp), 256, 0, (hipStream_t)stream>>>(B, H, W, C, (const bf16_t*)in, 0,
                                                                                  (bf16_t*)out, Kp);
  return pso_check_launch("pso_im2col3");
}

int pso_sumpool2(int B, int H, int W, int C, const void* in, const void* dadd, void* out, void* stream) {
  PSO_ARG_CHECK(C % 8 == 0 && in && out, "pso_sumpool2: C %% 8");
  sumpool2_kernel<<<grid_for((long)B * H * W * C / 8), 256, 0, (hipStream_t)stream>>>(
      B, H, W, C, (const bf16_t*)in, (const bf16_t*)dadd, (bf16_t*)out);
  return pso_check_launch("pso_sumpool2");
}

int pso_axpby(long n, float a, const void* x, float b, const void* z, void* y, void* stream) {
  PSO_ARG_CHECK(n % 8 == 0 && x && y, "pso_axpby: n %% 8");
  axpby_kernel<<<grid_for(n / 8), 256, 0, (hipStream_t)stream>>>(n / 8, a, (const bf16_t*)x, b, (const bf16_t*)z,
                                                                 (bf16_t*)y);
  return pso_check_launch("pso_axpby");
}

int pso_cast_f32_bf16(long n, const float* x, float scale, void* y, void* stream) {
  cast_f32_bf16_kernel<<<grid_for(n, 8), 256, 0, (hipStream_t)stream>>>(n, x, scale, (bf16_t*)y);
  return pso_check_launch("pso_cast_f32_bf16");
}

int pso_cast_bf16_f32(long n, const void* x, float* y, void* stream) {
  cast_bf16_f32_kernel<<<grid_for(n, 8), 256, 0, (hipStream_t)stream>>>(n, (const bf16_t*)x, y);
  return pso_check_launch("pso_cast_bf16_f32");
}

int pso_conv_weight_t(int Co, int ks, int Ci, int flip, const void* w, void* wt, void* stream) {
  conv_weight_t_kernel<<<dim3(cdiv(Ci, 64), cdiv(Co, 64), ks * ks), 256, 0, (hipStream_t)stream>>>(
      Co, ks, Ci, flip, (const bf16_t*)w, (bf16_t*)wt);
  return pso_check_launch("pso_conv_weight_t");
}

}  // extern "C"
