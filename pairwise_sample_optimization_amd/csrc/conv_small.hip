// Direct 3x3 convolution for a tiny output width (Cout <= 3): the VAE decoder's conv_out (128 channels -> RGB at
// 1024^2; DP/sdxl_turbo_with_logprob.py:154-155).  As an implicit GEMM it is an N = 3 product padded
// to 64-column MFMA tiles -- 61 of every 64 MACs wasted (1.34 ms per 4-image chunk, 22 TF/s useful); as a direct
// convolution it is a VALU stream of v_dot2c_f32_bf16 over an LDS image of the input tile.
//
// Block = 256 threads = a 16 x 16 tile of output pixels of one image (one pixel per thread).  Per 64-channel chunk the
// block stages its 18 x 18-pixel input window (zeros outside the image) into LDS with a 144-B pixel pitch: the 16 lanes
// of a ds_read_b128 group read 16 consecutive pixels 36 dwords apart, i.e. 16 disjoint 4-bank slots (conflict-free).
// The thread then walks the 9 taps x 32 channel pairs; the weights ([Cout][3][3][Cin] bf16, the prepared NHWC
// filter) are wave-uniform, read through the scalar cache (loads only).  fp32 accumulation, bias, bf16 out.
#include "common.h"

#define CS_T 16          // output tile side
#define CS_CH 64         // channels per chunk
#define CS_PITCH 72      // bf16 per staged pixel (64 + 8: 144-B pitch)

typedef __attribute__((ext_vector_type(2))) __bf16 cs_bf16x2;

// CIN > 0: the channel count as a constant (the weight offsets become scalar-load immediates: no per-load SGPR
// address arithmetic); 0: read from the argument
template <int COUT, int CIN>
__global__ __launch_bounds__(256) void conv3x3_smallc_kernel(int H, int W, int cin_arg, const bf16_t* __restrict__ x,
                                                             const bf16_t* __restrict__ w,
                                                             const bf16_t* __restrict__ bias, bf16_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) bf16_t img[(CS_T + 2) * (CS_T + 2) * CS_PITCH];
  const int Cin = CIN > 0 ? CIN : cin_arg;
  const int tid = threadIdx.x;
  const int tx = tid & (CS_T - 1), ty = tid >> 4;
  const int x0 = blockIdx.x * CS_T, y0 = blockIdx.y * CS_T, b = blockIdx.z;
  const bf16_t* xb = x + (long)b * H * W * Cin;
  float acc[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) acc[c] = 0.f;
  const uint32_t* w32 = reinterpret_cast<const uint32_t*>(w);  // bf16 pairs
  const int wrow = 9 * Cin / 2;                                  // pairs per output channel
  for (int c0 = 0; c0 < Cin; c0 += CS_CH) {
    __syncthreads();  // the previous chunk's reads are done
    // stage 18 x 18 pixels x 64 channels: 8 pieces of 16 B per pixel
    for (int q = tid; q < (CS_T + 2) * (CS_T + 2) * 8; q += 256) {
      const int p = q >> 3, piece = q & 7;
      const int py = p / (CS_T + 2), px = p - py * (CS_T + 2);
      const int gy = y0 + py - 1, gx = x0 + px - 1;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (gy >= 0 && gy < H && gx >= 0 && gx < W)
        v = *reinterpret_cast<const uint4*>(xb + ((long)gy * W + gx) * Cin + c0 + piece * 8);
      *reinterpret_cast<uint4*>(img + p * CS_PITCH + piece * 8) = v;
    }
    __syncthreads();
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3, dx = tap - dy * 3;
      const bf16_t* src = img + ((ty + dy) * (CS_T + 2) + tx + dx) * CS_PITCH;
#pragma unroll
      for (int piece = 0; piece < 8; ++piece) {
        const uint4 v = *reinterpret_cast<const uint4*>(src + piece * 8);
        const uint32_t xv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int c = 0; c < COUT; ++c) {
          const uint32_t* wp = w32 + c * wrow + (tap * Cin + c0 + piece * 8) / 2;  // wave-uniform
#pragma unroll
          for (int k = 0; k < 4; ++k)
            acc[c] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(cs_bf16x2, xv[k]),
                                                     __builtin_bit_cast(cs_bf16x2, wp[k]), acc[c], false);
        }
      }
    }
  }
  const int oy = y0 + ty, ox = x0 + tx;
  bf16_t* o = out + (((long)b * H + oy) * W + ox) * COUT;
#pragma unroll
  for (int c = 0; c < COUT; ++c) o[c] = f2bf(acc[c] + (bias ? bf2f(bias[c]) : 0.f));
}

// Entry from pso_conv2d (gemm.hip) when the shape qualifies; returns PSO_OK, or -1 when it does not (caller runs the
// implicit GEMM).  Requires H, W multiples of 16, Cin a multiple of 64, 1 <= Cout <= 3, bf16 NHWC in / out (dense rows).
int pso_conv3x3_smallc_run(int B, int H, int W, int Cin, int Cout, const void* x, const void* w, const void* bias,
                           void* out, hipStream_t st) {
  if (Cout < 1 || Cout > 3 || (H % CS_T) != 0 || (W % CS_T) != 0 || (Cin % CS_CH) != 0 || B < 1 || B > 65535 ||
      (long)B * H * W * Cin >= (1L << 31))
    return -1;
  const dim3 grid(W / CS_T, H / CS_T, B);
  const bf16_t *xp = (const bf16_t*)x, *wp = (const bf16_t*)w, *bp = (const bf16_t*)bias;
  bf16_t* op = (bf16_t*)out;
  pso_note_kernel("conv3x3_smallc_kernel<%d, %d>", Cout, Cin == 128 ? 128 : 0);
  if (Cout == 3 && Cin == 128) conv3x3_smallc_kernel<3, 128><<<grid, 256, 0, st>>>(H, W, Cin, xp, wp, bp, op);
  else if (Cout == 1) conv3x3_smallc_kernel<1, 0><<<grid, 256, 0, st>>>(H, W, Cin, xp, wp, bp, op);
  else if (Cout == 2) conv3x3_smallc_kernel<2, 0><<<grid, 256, 0, st>>>(H, W, Cin, xp, wp, bp, op);
  else conv3x3_smallc_kernel<3, 0><<<grid, 256, 0, st>>>(H, W, Cin, xp, wp, bp, op);
  return pso_check_launch("pso_conv2d (direct small-Cout 3x3)");
}
