// Optimizer step, gradient-norm clipping and preference labels of the PSO train loop (all on device, no host sync).
//
//   grad norm + clip   accelerator.clip_grad_norm_(params, max_grad_norm)  T:858-859  (torch clip_grad_norm_:
//                      coef = min(1, max_norm / (||g||_2 + 1e-6)))
//   AdamW              torch.optim.AdamW step T:860 (the reference default is bitsandbytes AdamW8bit,
//                      config_sdxl_turbo_dpo.py:86, which has no ROCm build here), decoupled weight
//                      decay, bias-corrected moments; the clip coefficient and the 1/world DDP mean are folded into
//                      the gradient read, so clip + step is one pass over (param, grad, m, v).
//   preference         sample_compare T:401-416 (random reward index, ties -> member 0 loses) and
//                      compare D:420-434 (strict Pareto dominance, ties -> (0, 0)).
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <vector>

#define OPT_THREADS 256

// partial sums of g^2 (fp64) per block -> one final block computes the clip coefficient.  16-B loads where the
// gradient is 16-B aligned (the flat buckets are), the ragged tail by the scalar loop.
__global__ void sqnorm_partial_kernel(long n, const float* __restrict__ g, double* __restrict__ part) {
  __shared__ double red[OPT_THREADS / 64];
  double acc = 0.0;
  const long tid = blockIdx.x * (long)blockDim.x + threadIdx.x, nth = (long)gridDim.x * blockDim.x;
  long tail = 0;
  if ((reinterpret_cast<uintptr_t>(g) & 15) == 0) {
    const long n4 = n >> 2;
    for (long i = tid; i < n4; i += nth) {
      const float4 v = reinterpret_cast<const float4*>(g)[i];
      acc += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
    tail = n4 << 2;
  }
  for (long i = tail + tid; i < n; i += nth) {
    const double v = g[i];
    acc += v * v;
  }
  acc = warp_sum_d(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < OPT_THREADS / 64; ++w) s += red[w];
    part[blockIdx.x] = s;
  }
}

// out[0] = ||g * scale||_2, out[1] = clip coefficient (1 if max_norm <= 0)
__global__ void clip_coef_kernel(int nparts, const double* __restrict__ part, float scale, float max_norm,
                                 float* __restrict__ out) {
  // one workgroup sums the per-block partials (fixed order: strided per thread, then wave and workgroup trees)
  __shared__ double red[OPT_THREADS / 64];
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += part[i];
  acc = warp_sum_d(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < OPT_THREADS / 64; ++w) s += red[w];
    const float norm = (float)sqrt(s) * scale;
    out[0] = norm;
    float c = 1.0f;
    if (max_norm > 0.f) {
      c = max_norm / (norm + 1e-6f);
      if (c > 1.0f) c = 1.0f;
    }
    out[1] = c;
  }
}

__global__ void adamw_kernel(long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, float lr, float b1, float b2, float eps, float wd, float bc1,
                             float bc2_sqrt, float gscale, const float* __restrict__ clip) {
  const float s = gscale * (clip ? clip[1] : 1.0f);
  const float step = lr / bc1;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float gi = g[i] * s;
    float pi = p[i] * (1.0f - lr * wd);
    const float mi = b1 * m[i] + (1.0f - b1) * gi;
    const float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi -= step * (mi / denom);
    p[i] = pi;
  }
}

// ---- blockwise 8-bit AdamW (bitsandbytes AdamW8bit: the reference default, config_sdxl_turbo_dpo.py:86, T:427-435)
// m and v live as uint8 codes into two 256-entry dynamic quantisation maps (signed for m, unsigned for v) with one
// fp32 absmax per 2048-element block; each step dequantises with the previous absmax, updates, and requantises
// (nearest code) against the block's new absmax.  One 256-thread workgroup per block, 8 consecutive elements per
// thread (32-B / 8-B vector loads and stores); the maps travel in the kernel arguments and sit in LDS.  Arithmetic in the order of bitsandbytes'
// kOptimizerStatic8bit2StateBlockwise ADAM branch (restated in oracle/adam8bit.py, parity unpinned: no bitsandbytes
// here), contraction off so the fp32 rounding matches the restatement step for step.
#define ADAM8_BLOCK 2048
#define ADAM8_LAYOUT_DEFAULT 1  // element-to-thread mapping of the 8-bit AdamW (adamw8bit_kernel<LAY>)
struct Adam8Maps {
  float s[256], u[256];
};

// nearest code of x in a sorted 256-entry map (ties -> the lower index): lo = the count of the first 255 entries
// below x (equal to lower_bound except that it stops at 255, which the clamp below maps to the same index), then the
// nearer neighbour.  The count descends a breadth-first (Eytzinger) copy of those 255 entries, tree[1..255]: step d
// reads one of the 2^d consecutive nodes of level d, so the 64 lanes' reads of a level hit distinct LDS banks (the
// sorted-order bisection probed entries 2h apart at step h -- one bank for every lane -- and serialised up to 4-way).
// The searches of a thread's values run in lockstep, so every level issues NV independent LDS reads.
template <int NV>
__device__ __forceinline__ void adam8_nearest(const float* __restrict__ code, const float* __restrict__ tree,
                                              const float (&x)[NV], int (&idx)[NV]) {
  // the descent tracks the node's byte offset (4 * node): compare, select, shift-add per level (no separate index to
  // address shift)
  const char* tb = reinterpret_cast<const char*>(tree);
  unsigned a[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) a[k] = 4u;
#pragma unroll
  for (int d = 0; d < 8; ++d)
#pragma unroll
    for (int k = 0; k < NV; ++k) a[k] = (a[k] << 1) + (*reinterpret_cast<const float*>(tb + a[k]) < x[k] ? 4u : 0u);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int lo = (int)(a[k] >> 2) - 256;
    const int i = lo < 1 ? 1 : lo;
    const float a = code[i - 1], b = code[i];
    idx[k] = fabsf(x[k] - a) <= fabsf(b - x[k]) ? i - 1 : i;
  }
}

// node of the breadth-first tree over sorted entries 0..254 that holds sorted entry i: height h = ctz(i + 1) above
// the leaves, position (i + 1) >> (h + 1) within its level
__device__ __forceinline__ int adam8_node(int i) {
  const int h = __builtin_ctz(i + 1);
  return (1 << (7 - h)) + ((i + 1) >> (h + 1));
}

// Block table (desc, optional): block b covers elements [desc[4b], desc[4b] + desc[4b+1]) of the flat buffers -- the
// blocks restart at every tensor, as bitsandbytes quantises each parameter tensor on its own -- and desc[4b+2] >= 0
// marks a block of a tensor under min_8bit_size (4096 elements) that keeps 32-bit state: m / v fp32 at
// m32 / v32 + desc[4b+2] + (i - start).  desc == nullptr: uniform 2048-element blocks over [0, n), all 8-bit.
// Non-finite gradient elements leave the parameter, m and v unchanged (bitsandbytes skips the parameter update for
// them; its state update for such an element is not pinned here).
// LAY = element-to-thread mapping inside a block.  0: thread t owns the 8 consecutive elements 8t .. 8t + 7 (each
// 16-B access instruction of a wave spans 2 KB with 16-B gaps); 1: thread t owns 4t .. 4t + 3 and 1024 + 4t .. +3, so
// every access instruction of a wave covers one contiguous range.  Per-block results are the same bits either way.
template <int LAY>
__global__ __launch_bounds__(256) void adamw8bit_kernel(
    long n, float* __restrict__ p, float* g, uint8_t* __restrict__ qm, uint8_t* __restrict__ qv,
    float* __restrict__ am, float* __restrict__ av, float b1, float omb1, float b2, float omb2, float eps_c2,
    float step_size, float decay, float gscale, const float* __restrict__ clip, bf16_t* __restrict__ pw,
    const long* __restrict__ desc, float* __restrict__ m32, float* __restrict__ v32, int zero_grad, Adam8Maps maps) {
#pragma clang fp contract(off)
  __shared__ float cs[256], cu[256], ts[256], tu[256];
  __shared__ float red[2][4];
  const int t = threadIdx.x;
  const long blk = blockIdx.x;
  long base = blk * ADAM8_BLOCK, end = min(n, base + ADAM8_BLOCK), soff = -1;
  if (desc) {
    base = desc[4 * blk];
    end = base + desc[4 * blk + 1];
    soff = desc[4 * blk + 2];
  }
  const bool st32 = soff >= 0;  // uniform over the workgroup
  if (!st32) {
    cs[t] = maps.s[t];
    cu[t] = maps.u[t];
    if (t < 255) {
      ts[adam8_node(t)] = maps.s[t];
      tu[adam8_node(t)] = maps.u[t];
    }
  }
  // the thread's two 4-element chunks: elements e < 4 at o0 + e, e >= 4 at o1 + e - 4
  const long o0 = LAY ? base + 4L * t : base + 8L * t;
  const long o1 = LAY ? o0 + ADAM8_BLOCK / 2 : o0 + 4;
  auto at = [&](int e) { return (e < 4 ? o0 : o1) + (e & 3); };
  // 16-B / 4-B vector accesses wherever both chunks are whole and aligned
  const bool full = o0 + 4 <= end && o1 + 4 <= end && (base & 3) == 0 && (!st32 || (soff & 3) == 0);
  const float s = gscale * (clip ? clip[1] : 1.0f);
  float gv[8], pv[8];
  if (full) {
    const float4 g0 = *reinterpret_cast<const float4*>(g + o0), g1 = *reinterpret_cast<const float4*>(g + o1);
    const float4 p0 = *reinterpret_cast<const float4*>(p + o0), p1 = *reinterpret_cast<const float4*>(p + o1);
    gv[0] = g0.x; gv[1] = g0.y; gv[2] = g0.z; gv[3] = g0.w; gv[4] = g1.x; gv[5] = g1.y; gv[6] = g1.z; gv[7] = g1.w;
    pv[0] = p0.x; pv[1] = p0.y; pv[2] = p0.z; pv[3] = p0.w; pv[4] = p1.x; pv[5] = p1.y; pv[6] = p1.z; pv[7] = p1.w;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const long i = at(e);
      gv[e] = i < end ? g[i] : 0.f;
      pv[e] = i < end ? p[i] : 0.f;
    }
  }
  if (st32) {  // bitsandbytes 32-bit state (kOptimizer32bit2State ADAM): same arithmetic, no quantisation
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const long i = at(e);
      if (i >= end) continue;
      const float gi = gv[e] * s;
      if (isfinite(gi)) {
        float* ms = m32 + soff + (i - base);
        float* vs = v32 + soff + (i - base);
        float m = *ms, v = *vs;
        m = (m * b1) + (omb1 * gi);
        v = (v * b2) + ((omb2 * gi) * gi);
        *ms = m;
        *vs = v;
        pv[e] = pv[e] + (step_size * (m / (sqrtf(v) + eps_c2)));
        pv[e] = pv[e] * decay;
      }
      p[i] = pv[e];
      if (pw) pw[i] = f2bf(pv[e]);
      if (zero_grad) g[i] = 0.f;
    }
    return;
  }
  const float am0 = am[blk], av0 = av[blk];
  uint32_t cm[2], cv[2];
  if (full) {
    cm[0] = *reinterpret_cast<const uint32_t*>(qm + o0);
    cm[1] = *reinterpret_cast<const uint32_t*>(qm + o1);
    cv[0] = *reinterpret_cast<const uint32_t*>(qv + o0);
    cv[1] = *reinterpret_cast<const uint32_t*>(qv + o1);
  } else {
    cm[0] = cm[1] = cv[0] = cv[1] = 0u;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const long i = at(e);
      if (i < end) {
        cm[e >> 2] |= (uint32_t)qm[i] << (8 * (e & 3));
        cv[e >> 2] |= (uint32_t)qv[i] << (8 * (e & 3));
      }
    }
  }
  __syncthreads();
  float m[8], v[8];
  float mx_m = 0.f, mx_v = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if (full || at(e) < end) {
      const float gi = gv[e] * s;
      m[e] = cs[(cm[e >> 2] >> (8 * (e & 3))) & 255u] * am0;
      v[e] = cu[(cv[e >> 2] >> (8 * (e & 3))) & 255u] * av0;
      // branch-free: a non-finite gradient element keeps p, m and v (the update is computed and discarded)
      const bool fin = isfinite(gi);
      const float m1 = (m[e] * b1) + (omb1 * gi);
      const float v1 = (v[e] * b2) + ((omb2 * gi) * gi);
      const float p1 = (pv[e] + (step_size * (m1 / (sqrtf(v1) + eps_c2)))) * decay;
      m[e] = fin ? m1 : m[e];
      v[e] = fin ? v1 : v[e];
      pv[e] = fin ? p1 : pv[e];
      mx_m = fmaxf(mx_m, fabsf(m[e]));
      mx_v = fmaxf(mx_v, fabsf(v[e]));
    } else {
      m[e] = v[e] = pv[e] = 0.f;
    }
  }
  // block maxima: wave (64 lanes) then the 4 waves
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx_m = fmaxf(mx_m, __shfl_xor(mx_m, o, 64));
    mx_v = fmaxf(mx_v, __shfl_xor(mx_v, o, 64));
  }
  if ((t & 63) == 0) { red[0][t >> 6] = mx_m; red[1][t >> 6] = mx_v; }
  __syncthreads();
  const float nm = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
  const float nv = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
  float xm[8], xv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    xm[e] = nm > 0.f ? m[e] / nm : 0.f;
    xv[e] = nv > 0.f ? v[e] / nv : 0.f;
  }
  int im[8], iv[8];
  adam8_nearest(cs, ts, xm, im);
  adam8_nearest(cu, tu, xv, iv);
  if (full) {
    *reinterpret_cast<float4*>(p + o0) = make_float4(pv[0], pv[1], pv[2], pv[3]);
    *reinterpret_cast<float4*>(p + o1) = make_float4(pv[4], pv[5], pv[6], pv[7]);
    if (pw) {  // the bf16 working copy of the parameters (round to nearest even)
      *reinterpret_cast<uint2*>(pw + o0) = make_uint2(pack2bf(pv[0], pv[1]), pack2bf(pv[2], pv[3]));
      *reinterpret_cast<uint2*>(pw + o1) = make_uint2(pack2bf(pv[4], pv[5]), pack2bf(pv[6], pv[7]));
    }
    *reinterpret_cast<uint32_t*>(qm + o0) =
        (uint32_t)im[0] | (uint32_t)im[1] << 8 | (uint32_t)im[2] << 16 | (uint32_t)im[3] << 24;
    *reinterpret_cast<uint32_t*>(qm + o1) =
        (uint32_t)im[4] | (uint32_t)im[5] << 8 | (uint32_t)im[6] << 16 | (uint32_t)im[7] << 24;
    *reinterpret_cast<uint32_t*>(qv + o0) =
        (uint32_t)iv[0] | (uint32_t)iv[1] << 8 | (uint32_t)iv[2] << 16 | (uint32_t)iv[3] << 24;
    *reinterpret_cast<uint32_t*>(qv + o1) =
        (uint32_t)iv[4] | (uint32_t)iv[5] << 8 | (uint32_t)iv[6] << 16 | (uint32_t)iv[7] << 24;
    if (zero_grad) {  // optimizer.zero_grad folded into the step: the gradient was read above
      *reinterpret_cast<float4*>(g + o0) = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(g + o1) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const long i = at(e);
      if (i >= end) continue;
      p[i] = pv[e];
      if (pw) pw[i] = f2bf(pv[e]);
      qm[i] = (uint8_t)im[e];
      qv[i] = (uint8_t)iv[e];
      if (zero_grad) g[i] = 0.f;
    }
  }
  if (t == 0) { am[blk] = nm; av[blk] = nv; }
}

// bitsandbytes.functional.create_dynamic_map(signed, max_exponent_bits = 7, total_bits = 8), float32 like the
// torch original (numpy-style linspace in double, cast to float32)
static void adam8_dynamic_map(bool sgn, float* out) {
  std::vector<float> d;
  const int max_exp = 7, non_sign = 7;
  for (int i = 0; i < max_exp; ++i) {
    const int nitems = sgn ? (1 << (i + non_sign - max_exp)) + 1 : (1 << (i + non_sign - max_exp + 1)) + 1;
    std::vector<float> b(nitems);
    const double step = (1.0 - 0.1) / (nitems - 1);
    for (int k = 0; k < nitems; ++k) b[k] = (float)(k == nitems - 1 ? 1.0 : 0.1 + k * step);
    const float sc = (float)std::pow(10.0, (double)(-(max_exp - 1) + i));
    for (int k = 0; k + 1 < nitems; ++k) {
      const float mean = (b[k] + b[k + 1]) / 2.0f;
      d.push_back(sc * mean);
      if (sgn) d.push_back(-sc * mean);
    }
  }
  d.push_back(0.f);
  d.push_back(1.f);
  while (d.size() < 256) d.push_back(0.f);
  std::sort(d.begin(), d.end());
  for (int k = 0; k < 256; ++k) out[k] = d[k];
}

__global__ void zero_kernel(long n, float* __restrict__ x) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) x[i] = 0.f;
}

// rewards [P][2][m]; mode 0 (turbo): column idx[p] (or 0), a<=b -> (-1,+1), b<a -> (+1,-1);
// mode 1 (dmd): strict Pareto over all m columns, ties -> (0,0).
__global__ void preference_kernel(int P, int m, const float* __restrict__ rewards, const int64_t* __restrict__ idx,
                                  int mode, float* __restrict__ pref) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const float* a = rewards + (long)p * 2 * m;
  const float* b = a + m;
  float c0 = 0.f, c1 = 0.f;
  if (mode == 0) {
    const int k = idx ? (int)idx[p] : 0;
    if (a[k] <= b[k]) { c0 = -1.f; c1 = 1.f; }
    else if (b[k] < a[k]) { c0 = 1.f; c1 = -1.f; }
  } else {
    bool a_le = true, a_lt = false, b_le = true, b_lt = false;
    for (int j = 0; j < m; ++j) {
      a_le &= a[j] <= b[j];
      a_lt |= a[j] < b[j];
      b_le &= b[j] <= a[j];
      b_lt |= b[j] < a[j];
    }
    if (a_le && a_lt) { c0 = -1.f; c1 = 1.f; }
    if (b_le && b_lt) { c0 = 1.f; c1 = -1.f; }
  }
  pref[2 * p] = c0;
  pref[2 * p + 1] = c1;
}

static int nblocks(long n) {
  long b = (n + OPT_THREADS - 1) / OPT_THREADS;
  return (int)(b > 2048 ? 2048 : (b < 1 ? 1 : b));
}

extern "C" {

size_t pso_grad_clip_ws_bytes(long n) { return 2048 * sizeof(double); }

int pso_grad_clip_coef(long n, const float* grad, float grad_scale, float max_norm, float* out_norm_coef, void* ws,
                       size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(grad && out_norm_coef && ws && ws_bytes >= pso_grad_clip_ws_bytes(n), "pso_grad_clip_coef: bad args");
  hipStream_t st = (hipStream_t)stream;
  const int nb = nblocks(n);
  sqnorm_partial_kernel<<<nb, OPT_THREADS, 0, st>>>(n, grad, (double*)ws);
  clip_coef_kernel<<<1, OPT_THREADS, 0, st>>>(nb, (const double*)ws, grad_scale, max_norm, out_norm_coef);
  return pso_check_launch("pso_grad_clip_coef");
}

int pso_adamw_step(long n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, float lr, float beta1,
                   float beta2, float eps, float weight_decay, int step, float grad_scale, const float* clip_coef,
                   void* stream) {
  PSO_ARG_CHECK(param && grad && exp_avg && exp_avg_sq && step >= 1, "pso_adamw_step: bad args");
  const float bc1 = 1.0f - powf(beta1, (float)step);
  const float bc2 = 1.0f - powf(beta2, (float)step);
  adamw_kernel<<<nblocks(n), OPT_THREADS, 0, (hipStream_t)stream>>>(n, param, grad, exp_avg, exp_avg_sq, lr, beta1,
                                                                    beta2, eps, weight_decay, bc1, sqrtf(bc2),
                                                                    grad_scale, clip_coef);
  return pso_check_launch("pso_adamw_step");
}

size_t pso_adamw8bit_blocks(long n) { return (size_t)((n + ADAM8_BLOCK - 1) / ADAM8_BLOCK); }

void pso_adamw8bit_maps(float* signed_map, float* unsigned_map) {
  adam8_dynamic_map(true, signed_map);
  adam8_dynamic_map(false, unsigned_map);
}

static int adam8_launch(long n, int nblk, float* param, void* param_bf16, float* grad, int zero_grad, uint8_t* exp_avg_q,
                        uint8_t* exp_avg_sq_q, float* absmax_m, float* absmax_v, const long* desc, float* m32,
                        float* v32, float lr, float beta1, float beta2, float eps, float weight_decay, int step,
                        float grad_scale, const float* clip_coef, void* stream) {
  static Adam8Maps maps = [] {
    Adam8Maps m;
    adam8_dynamic_map(true, m.s);
    adam8_dynamic_map(false, m.u);
    return m;
  }();
  const double b1 = beta1, b2 = beta2;
  const float c1 = (float)(1.0 - std::pow(b1, step));
  const float c2 = (float)std::sqrt(1.0 - std::pow(b2, step));
  const float step_size = (-lr) * c2 / c1;
  const float decay = (float)(1.0 - (double)lr * weight_decay);
  if (nblk <= 0) return PSO_OK;
  // element layout inside a block: PSO_ADAM8_LAYOUT (0 / 1) for the benchmark (tools build only)
#ifdef PSO_BENCH_KNOBS
  static const int lay = [] {
    const char* e = getenv("PSO_ADAM8_LAYOUT");
    return e ? (atoi(e) != 0) : ADAM8_LAYOUT_DEFAULT;
  }();
#else
  constexpr int lay = ADAM8_LAYOUT_DEFAULT;
#endif
  const hipStream_t st = (hipStream_t)stream;
  const float omb1 = (float)(1.0 - b1), omb2 = (float)(1.0 - b2);
#define PSO_ADAM8_ARGS                                                                                                   \
  n, param, grad, exp_avg_q, exp_avg_sq_q, absmax_m, absmax_v, beta1, omb1, beta2, omb2, c2 * eps, step_size, decay,     \
      grad_scale, clip_coef, (bf16_t*)param_bf16, desc, m32, v32, zero_grad, maps
#ifdef PSO_BENCH_KNOBS
  if (lay)
    adamw8bit_kernel<1><<<nblk, 256, 0, st>>>(PSO_ADAM8_ARGS);
  else
    adamw8bit_kernel<0><<<nblk, 256, 0, st>>>(PSO_ADAM8_ARGS);
#else
  (void)lay;
  adamw8bit_kernel<ADAM8_LAYOUT_DEFAULT><<<nblk, 256, 0, st>>>(PSO_ADAM8_ARGS);
#endif
#undef PSO_ADAM8_ARGS
  return pso_check_launch("pso_adamw8bit_step");
}

int pso_adamw8bit_step_bf16(long n, float* param, void* param_bf16, const float* grad, uint8_t* exp_avg_q, uint8_t* exp_avg_sq_q,
                       float* absmax_m, float* absmax_v, float lr, float beta1, float beta2, float eps,
                       float weight_decay, int step, float grad_scale, const float* clip_coef, void* stream) {
  PSO_ARG_CHECK(param && grad && exp_avg_q && exp_avg_sq_q && absmax_m && absmax_v && step >= 1 && n > 0,
                "pso_adamw8bit_step_bf16: bad args");
  PSO_ARG_CHECK((((uintptr_t)param | (uintptr_t)grad | (uintptr_t)param_bf16) & 15) == 0 && (((uintptr_t)exp_avg_q | (uintptr_t)exp_avg_sq_q) & 7) == 0,
                "pso_adamw8bit_step_bf16: param / grad / param_bf16 need 16-B, the code arrays 8-B alignment");
  return adam8_launch(n, (int)pso_adamw8bit_blocks(n), param, param_bf16, const_cast<float*>(grad), 0, exp_avg_q, exp_avg_sq_q, absmax_m,
                      absmax_v, nullptr, nullptr, nullptr, lr, beta1, beta2, eps, weight_decay, step, grad_scale,
                      clip_coef, stream);
}

static int adam8_blocks(const char* who, long n, int nblk, const long* desc, float* param, void* param_bf16,
                        float* grad, int zero_grad, uint8_t* exp_avg_q, uint8_t* exp_avg_sq_q, float* absmax_m,
                        float* absmax_v, float* exp_avg_32, float* exp_avg_sq_32, float lr, float beta1, float beta2,
                        float eps, float weight_decay, int step, float grad_scale, const float* clip_coef,
                        void* stream) {
  PSO_ARG_CHECK(param && grad && exp_avg_q && exp_avg_sq_q && absmax_m && absmax_v && step >= 1 && n > 0 &&
                    nblk >= 0 && (nblk == 0 || desc),
                "%s: bad args", who);
  PSO_ARG_CHECK((((uintptr_t)param | (uintptr_t)grad | (uintptr_t)param_bf16 | (uintptr_t)exp_avg_32 |
                  (uintptr_t)exp_avg_sq_32) & 15) == 0 && (((uintptr_t)exp_avg_q | (uintptr_t)exp_avg_sq_q) & 7) == 0,
                "%s: param / grad / param_bf16 / 32-bit state need 16-B, the code arrays 8-B alignment", who);
  return adam8_launch(n, nblk, param, param_bf16, grad, zero_grad, exp_avg_q, exp_avg_sq_q, absmax_m, absmax_v, desc,
                      exp_avg_32, exp_avg_sq_32, lr, beta1, beta2, eps, weight_decay, step, grad_scale, clip_coef,
                      stream);
}

int pso_adamw8bit_step_blocks(long n, int nblk, const long* desc, float* param, void* param_bf16, const float* grad,
                              uint8_t* exp_avg_q, uint8_t* exp_avg_sq_q, float* absmax_m, float* absmax_v,
                              float* exp_avg_32, float* exp_avg_sq_32, float lr, float beta1, float beta2, float eps,
                              float weight_decay, int step, float grad_scale, const float* clip_coef, void* stream) {
  return adam8_blocks("pso_adamw8bit_step_blocks", n, nblk, desc, param, param_bf16, const_cast<float*>(grad), 0,
                      exp_avg_q, exp_avg_sq_q, absmax_m, absmax_v, exp_avg_32, exp_avg_sq_32, lr, beta1, beta2, eps,
                      weight_decay, step, grad_scale, clip_coef, stream);
}

int pso_adamw8bit_step_blocks_zero_grad(long n, int nblk, const long* desc, float* param, void* param_bf16,
                                        float* grad, uint8_t* exp_avg_q, uint8_t* exp_avg_sq_q, float* absmax_m,
                                        float* absmax_v, float* exp_avg_32, float* exp_avg_sq_32, float lr,
                                        float beta1, float beta2, float eps, float weight_decay, int step,
                                        float grad_scale, const float* clip_coef, void* stream) {
  return adam8_blocks("pso_adamw8bit_step_blocks_zero_grad", n, nblk, desc, param, param_bf16, grad, 1, exp_avg_q,
                      exp_avg_sq_q, absmax_m, absmax_v, exp_avg_32, exp_avg_sq_32, lr, beta1, beta2, eps,
                      weight_decay, step, grad_scale, clip_coef, stream);
}

int pso_adamw8bit_step(long n, float* param, const float* grad, uint8_t* exp_avg_q, uint8_t* exp_avg_sq_q,
                       float* absmax_m, float* absmax_v, float lr, float beta1, float beta2, float eps,
                       float weight_decay, int step, float grad_scale, const float* clip_coef, void* stream) {
  return pso_adamw8bit_step_bf16(n, param, nullptr, grad, exp_avg_q, exp_avg_sq_q, absmax_m, absmax_v, lr, beta1,
                                 beta2, eps, weight_decay, step, grad_scale, clip_coef, stream);
}

int pso_zero_f32(long n, float* x, void* stream) {
  zero_kernel<<<nblocks(n), OPT_THREADS, 0, (hipStream_t)stream>>>(n, x);
  return pso_check_launch("pso_zero_f32");
}

int pso_preference(int P, int m, const float* rewards, const int64_t* reward_idx, int mode, float* pref,
                   void* stream) {
  PSO_ARG_CHECK(P > 0 && m > 0 && rewards && pref && (mode == 0 || mode == 1), "pso_preference: bad args");
  preference_kernel<<<cdiv(P, 64), 64, 0, (hipStream_t)stream>>>(P, m, rewards, reward_idx, mode, pref);
  return pso_check_launch("pso_preference");
}

}  // extern "C"
