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

#define OPT_THREADS 256

// partial sums of g^2 (fp64) per block -> one final block computes the clip coefficient
__global__ void sqnorm_partial_kernel(long n, const float* __restrict__ g, double* __restrict__ part) {
  __shared__ double red[OPT_THREADS / 64];
  double acc = 0.0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
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
