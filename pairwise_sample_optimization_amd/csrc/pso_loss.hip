// Fused PSO step log-prob + pairwise clipped log-ratio loss (forward and backward to eps_theta).
//
// Reference arithmetic (restated, never copied):
//   turbo step   DP/turbo_inference_with_logprob.py:69-114  (x0 = x - s*e; d = (x - x0)/s; mu = x + d*dt)
//   DMD2 step    DP/distilled_inference_with_logprob.py:36-42,84-135 (x0 = (x - sb*e)/sa; mu = sa_prev*x0)
//   log-prob     mean over C,H,W of -(x'-mu)^2/(2 std^2) - log std - log sqrt(2 pi)
//   loss         T:844-850 / D:848-854: -log sigmoid(beta*log clip(e^{dlp0})*pref0 + beta*log clip(e^{dlp1})*pref1)
//
// Design: a launch-bound elementwise+reduce path.  Kernel 1 streams x, x', eps (fp32/bf16, 16-B vector loads) and
// writes per-chunk fp64 partial sums (fixed order => bitwise deterministic).  Kernel 2 re-derives every per-pair
// scalar from the partials inside each block (no extra launch, no atomics) and streams d loss / d eps_theta.
#include "common.h"

// Element-wise op order must mirror the reference (no FMA contraction) for 1e-6 parity.
#pragma clang fp contract(off)

// DMD2 replay modes (PSO_MODE_DMD_F16 / _BF16): every intermediate of the reference's latent-dtype arithmetic is
// rounded to that dtype (torch's CPU/GPU fp16 and bf16 element-wise ops compute in fp32 and round the result).
template <int MODE>
__device__ __forceinline__ float rl(float x) {
  if constexpr (MODE == PSO_MODE_DMD_F16) return (float)(_Float16)x;
  else if constexpr (MODE == PSO_MODE_DMD_BF16) return bf_round(x);
  else return x;
}
// An opaque copy: the compiler cannot fuse an operation across it.  Every product / quotient of the step arithmetic
// goes through one, so the expressions are evaluated exactly as the reference's separate torch element-wise ops (each
// IEEE-rounded) no matter which contraction mode a translation unit is built with (an FMA of `x - c*e` once flipped a
// bf16 rounding tie of the DMD2 replay x0 against DP/distilled_inference_with_logprob.py).
__device__ __forceinline__ float rnd(float x) {
  asm("" : "+v"(x));
  return x;
}
__device__ __forceinline__ float rl_rt(int mode, float x) {
  return mode == PSO_MODE_DMD_F16 ? rl<PSO_MODE_DMD_F16>(x) : mode == PSO_MODE_DMD_BF16 ? rl<PSO_MODE_DMD_BF16>(x) : x;
}

#define LP_CHUNK 8192
#define LP_THREADS 256

struct Coef {
  float c[PSO_COEF_STRIDE];
};

__device__ __forceinline__ Coef load_coef(const float* coef, int img) {
  Coef k;
#pragma unroll
  for (int i = 0; i < PSO_COEF_STRIDE; ++i) k.c[i] = coef[img * PSO_COEF_STRIDE + i];
  return k;
}

template <int MODE>
__device__ __forceinline__ float step_mean(float x, float e, const Coef& k) {
  if (MODE == PSO_MODE_TURBO) {
    const float s = k.c[0];
    const float pred = x - rnd(s * e);
    const float deriv = rnd((x - pred) / s);
    return x + rnd(deriv * k.c[2]);
  } else {  // DP/distilled_inference_with_logprob.py:84-86 (x0 cast to the latent dtype), :112
    const float x0 = rl<MODE>(rnd(x - rnd(k.c[1] * e)) / k.c[0]);
    return rl<MODE>(rnd(k.c[2] * x0));
  }
}
// one element of the Gaussian log-density, DP/turbo_inference_with_logprob.py:108-112 / DP/distilled_...:129-133
template <int MODE>
__device__ __forceinline__ float lp_term(float pv, float mu, float denom, float lstd, float lc) {
  const float d = rl<MODE>(pv - mu);
  const float q = rl<MODE>(rnd(-rl<MODE>(rnd(d * d)) / denom));
  return rl<MODE>(rl<MODE>(q - lstd) - lc);
}
template <int MODE>
__device__ __forceinline__ float step_std(const Coef& k) { return MODE == PSO_MODE_TURBO ? k.c[1] : k.c[3]; }
template <int MODE>
__device__ __forceinline__ float step_denom(const Coef& k) { return MODE == PSO_MODE_TURBO ? k.c[3] : k.c[4]; }
template <int MODE>
__device__ __forceinline__ float step_logstd(const Coef& k) { return MODE == PSO_MODE_TURBO ? k.c[4] : k.c[5]; }
template <int MODE>
__device__ __forceinline__ float step_logc(const Coef& k) { return MODE == PSO_MODE_TURBO ? k.c[5] : k.c[6]; }
template <int MODE>
__device__ __forceinline__ float step_dmu_deps(const Coef& k) {
  return MODE == PSO_MODE_TURBO ? k.c[2] : -(k.c[2] * k.c[1] / k.c[0]);
}

__device__ __forceinline__ void load4_eps(const void* eps, int dtype, size_t i, float* e) {
  if (dtype == PSO_BF16) {
    const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(eps) + i);
    e[0] = bf2f(v.x & 0xffff); e[1] = bf2f(v.x >> 16); e[2] = bf2f(v.y & 0xffff); e[3] = bf2f(v.y >> 16);
  } else {
    const float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(eps) + i);
    e[0] = v.x; e[1] = v.y; e[2] = v.z; e[3] = v.w;
  }
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  v = warp_sum_d(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    for (int i = 0; i < LP_THREADS / 64; ++i) s += red[i];
  }
  return s;  // valid in thread 0
}

// grid: (nchunks, ncombo).  combo -> (image, eps source).  PAIR=true: combo = 2*img + which (0 pol, 1 ref).
template <int MODE, bool PAIR>
__global__ __launch_bounds__(LP_THREADS) void lp_partial_kernel(
    int n, const float* __restrict__ x, const float* __restrict__ prev_in, const void* eps_a, const void* eps_b,
    int eps_dtype, const float* __restrict__ noise, int noise_shared, const float* __restrict__ coef,
    float* __restrict__ prev_out, double* __restrict__ partial) {
  __shared__ double red[LP_THREADS / 64];
  const int combo = blockIdx.y;
  const int img = PAIR ? combo >> 1 : combo;
  const void* eps = (PAIR && (combo & 1)) ? eps_b : eps_a;
  const Coef k = load_coef(coef, img);
  const float std = step_std<MODE>(k), denom = step_denom<MODE>(k), lstd = step_logstd<MODE>(k),
              lc = step_logc<MODE>(k);
  const size_t base = (size_t)img * n;
  const int c0 = blockIdx.x * LP_CHUNK;
  const int c1 = min(n, c0 + LP_CHUNK);
  double acc = 0.0;
  for (int i = c0 + threadIdx.x * 4; i < c1; i += LP_THREADS * 4) {
    const float4 xv = *reinterpret_cast<const float4*>(x + base + i);
    float e[4];
    load4_eps(eps, eps_dtype, base + i, e);
    const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
    float pv[4];
    float mu[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) mu[j] = step_mean<MODE>(xs[j], e[j], k);
    if (prev_in) {
      const float4 p = *reinterpret_cast<const float4*>(prev_in + base + i);
      pv[0] = p.x; pv[1] = p.y; pv[2] = p.z; pv[3] = p.w;
    } else {
      const size_t nb = noise_shared ? (size_t)i : base + i;
      const float4 z = *reinterpret_cast<const float4*>(noise + nb);
      const float zs[4] = {z.x, z.y, z.z, z.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        pv[j] = MODE == PSO_MODE_TURBO ? mu[j] + rnd(zs[j] * std) : rl<MODE>(mu[j] + rl<MODE>(rnd(std * zs[j])));
      *reinterpret_cast<float4*>(prev_out + base + i) = make_float4(pv[0], pv[1], pv[2], pv[3]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc += (double)lp_term<MODE>(pv[j], mu[j], denom, lstd, lc);
  }
  const double s = block_sum_d(acc, red);
  if (threadIdx.x == 0) partial[(size_t)combo * gridDim.x + blockIdx.x] = s;
}

// the mean over C,H,W (the latent-dtype result of .mean() in the replay modes)
__device__ __forceinline__ float lp_from_partials(int mode, const double* partial, int combo, int nchunks, int n) {
  double s = 0.0;
  for (int c = 0; c < nchunks; ++c) s += partial[(size_t)combo * nchunks + c];
  return rl_rt(mode, (float)(s / (double)n));
}

__global__ void lp_finalize_kernel(int mode, int B, int n, int nchunks, const double* __restrict__ partial,
                                   float* __restrict__ log_prob) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) log_prob[b] = lp_from_partials(mode, partial, b, nchunks, n);
}

struct PairScalars {
  float lp[2][2];  // [member][pol/ref]
  float g[2];      // dL/d lp_pol[member], already * grad_scale
  float loss;      // -log sigmoid(z) of this pair
};

// T:844-850 on the four log-probs of pair p.  Replay modes round Δ, exp(Δ), the clamped ratio, its log and beta*log
// to the latent dtype (the reference's log-probs are latent-dtype tensors there); pref is fp32, so z and the rest stay
// fp32.  torch.clamp's backward passes the gradient where lo <= r <= hi (bounds included).
__device__ __forceinline__ PairScalars pair_scalars_lp(int mode, const float (&lp)[2][2], float p0, float p1, int P,
                                                       float beta, float clip_eps, float grad_scale) {
  PairScalars s;
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    s.lp[m][0] = lp[m][0];
    s.lp[m][1] = lp[m][1];
  }
  const float lo = 1.0f - clip_eps, hi = 1.0f + clip_eps;
  float lr[2];
  bool inside[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const float r = rl_rt(mode, expf(rl_rt(mode, lp[m][0] - lp[m][1])));
    inside[m] = (r >= lo) && (r <= hi);
    lr[m] = rl_rt(mode, beta * rl_rt(mode, logf(rl_rt(mode, fminf(fmaxf(r, lo), hi)))));
  }
  const float z = lr[0] * p0 + lr[1] * p1;
  const float sig = 1.0f / (1.0f + expf(-z));
  s.loss = -logf(sig);
  const float common = -(1.0f - sig) * beta / (float)P * grad_scale;
  s.g[0] = inside[0] ? common * p0 : 0.0f;
  s.g[1] = inside[1] ? common * p1 : 0.0f;
  return s;
}

__device__ __forceinline__ PairScalars pair_scalars(int mode, const double* partial, int p, int P, int nchunks, int n,
                                                    const float* pref, float beta, float clip_eps,
                                                    float grad_scale) {
  float lp[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int w = 0; w < 2; ++w) lp[m][w] = lp_from_partials(mode, partial, 2 * (2 * p + m) + w, nchunks, n);
  return pair_scalars_lp(mode, lp, pref[2 * p], pref[2 * p + 1], P, beta, clip_eps, grad_scale);
}

// Forward finalize: one thread per pair writes lp_out and the per-pair loss; thread 0 then averages (fixed order).
__global__ void pair_loss_finalize_kernel(int mode, int P, int n, int nchunks, const float* __restrict__ pref,
                                          float beta, float clip_eps, const double* __restrict__ partial,
                                          float* __restrict__ lp_out, float* __restrict__ loss_out) {
  __shared__ float pair_loss_sh[1024];
  for (int q = threadIdx.x; q < P; q += blockDim.x) {
    const PairScalars s = pair_scalars(mode, partial, q, P, nchunks, n, pref, beta, clip_eps, 1.0f);
    pair_loss_sh[q & 1023] = s.loss;
    for (int mm = 0; mm < 2; ++mm) {
      lp_out[(2 * q + mm) * 2 + 0] = s.lp[mm][0];
      lp_out[(2 * q + mm) * 2 + 1] = s.lp[mm][1];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double L = 0.0;
    for (int q = 0; q < P; ++q) L += (double)pair_loss_sh[q];
    loss_out[0] = (float)(L / (double)P);
  }
}

// Backward: grid (nchunks, 2P) -- one row per policy image; every block re-derives its pair's dL/d lp_theta from
// the forward's partials (bit-identical across blocks), times the upstream gradient read on device.
template <int MODE>
__global__ __launch_bounds__(LP_THREADS) void pair_grad_kernel(
    int P, int n, int nchunks, const float* __restrict__ x, const float* __restrict__ prev,
    const void* eps_pol, int eps_dtype, const float* __restrict__ coef, const float* __restrict__ pref, float beta,
    float clip_eps, const float* __restrict__ grad_out, float grad_scale, const double* __restrict__ partial,
    void* deps, int deps_dtype) {
  const int img = blockIdx.y;
  const int p = img >> 1, m = img & 1;
  __shared__ float g_sh;
  if (threadIdx.x == 0) {
    const float up = grad_out ? grad_out[0] * grad_scale : grad_scale;
    g_sh = pair_scalars(MODE, partial, p, P, nchunks, n, pref, beta, clip_eps, up).g[m];
  }
  __syncthreads();
  const Coef k = load_coef(coef, img);
  // dL/de = g * (1/n) * (2 d / denom) * dmu/deps
  const float scale = g_sh / (float)n * 2.0f / step_denom<MODE>(k) * step_dmu_deps<MODE>(k);
  const size_t base = (size_t)img * n;
  const int c0 = blockIdx.x * LP_CHUNK;
  const int c1 = min(n, c0 + LP_CHUNK);
  for (int i = c0 + threadIdx.x * 4; i < c1; i += LP_THREADS * 4) {
    const float4 xv = *reinterpret_cast<const float4*>(x + base + i);
    const float4 pv = *reinterpret_cast<const float4*>(prev + base + i);
    float e[4];
    load4_eps(eps_pol, eps_dtype, base + i, e);
    const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, ps[4] = {pv.x, pv.y, pv.z, pv.w};
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = scale * (ps[j] - step_mean<MODE>(xs[j], e[j], k));
    if (deps_dtype == PSO_BF16) {
      *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(deps) + base + i) =
          make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
    } else {
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(deps) + base + i) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

__global__ void pair_loss_lp_kernel(int mode, int P, const float* __restrict__ lp_pol, const float* __restrict__ lp_ref,
                                    const float* __restrict__ pref, float beta, float clip_eps,
                                    float* __restrict__ loss_out, float* __restrict__ dlp_out) {
  __shared__ float pair_loss_sh[1024];
  for (int q = threadIdx.x; q < P; q += blockDim.x) {
    const float lp[2][2] = {{lp_pol[2 * q], lp_ref[2 * q]}, {lp_pol[2 * q + 1], lp_ref[2 * q + 1]}};
    const PairScalars s = pair_scalars_lp(mode, lp, pref[2 * q], pref[2 * q + 1], P, beta, clip_eps, 1.0f);
    pair_loss_sh[q] = s.loss;
    if (dlp_out) {
      dlp_out[2 * q] = s.g[0];
      dlp_out[2 * q + 1] = s.g[1];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double L = 0.0;
    for (int q = 0; q < P; ++q) L += (double)pair_loss_sh[q];
    loss_out[0] = (float)(L / (double)P);
  }
}

#define PSO_MODE_OK(m) ((m) == PSO_MODE_TURBO || (m) == PSO_MODE_DMD || (m) == PSO_MODE_DMD_F16 || (m) == PSO_MODE_DMD_BF16)
// mode -> template instantiation
#define PSO_MODE_DISPATCH(mode, KERNEL_CALL)                       \
  switch (mode) {                                                  \
    case PSO_MODE_TURBO: { constexpr int M_ = PSO_MODE_TURBO; KERNEL_CALL; } break; \
    case PSO_MODE_DMD: { constexpr int M_ = PSO_MODE_DMD; KERNEL_CALL; } break;     \
    case PSO_MODE_DMD_F16: { constexpr int M_ = PSO_MODE_DMD_F16; KERNEL_CALL; } break; \
    default: { constexpr int M_ = PSO_MODE_DMD_BF16; KERNEL_CALL; } break;           \
  }

extern "C" {

size_t pso_step_logprob_ws_bytes(int B, int n) { return (size_t)B * cdiv(n, LP_CHUNK) * sizeof(double); }
size_t pso_pair_loss_ws_bytes(int P, int n) { return (size_t)4 * P * cdiv(n, LP_CHUNK) * sizeof(double); }

int pso_step_logprob(int mode, int B, int n, const float* sample, const void* eps, int eps_dtype,
                     const float* prev_in, const float* noise, int noise_shared, const float* coef,
                     float* prev_out, float* log_prob, void* ws, size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(PSO_MODE_OK(mode), "pso_step_logprob: bad mode %d", mode);
  PSO_ARG_CHECK(B > 0 && n > 0 && (n % 4) == 0, "pso_step_logprob: need B>0, n>0, n%%4==0 (B=%d n=%d)", B, n);
  PSO_ARG_CHECK(sample && eps && coef && log_prob, "pso_step_logprob: null pointer");
  PSO_ARG_CHECK(prev_in || (noise && prev_out), "pso_step_logprob: need prev_in, or noise and prev_out");
  PSO_ARG_CHECK(eps_dtype == PSO_F32 || eps_dtype == PSO_BF16, "pso_step_logprob: bad eps dtype");
  PSO_ARG_CHECK(ws && ws_bytes >= pso_step_logprob_ws_bytes(B, n), "pso_step_logprob: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int nchunks = cdiv(n, LP_CHUNK);
  double* partial = (double*)ws;
  dim3 grid(nchunks, B);
  PSO_MODE_DISPATCH(mode, (lp_partial_kernel<M_, false><<<grid, LP_THREADS, 0, st>>>(
                              n, sample, prev_in, eps, nullptr, eps_dtype, noise, noise_shared, coef, prev_out,
                              partial)))
  lp_finalize_kernel<<<cdiv(B, 64), 64, 0, st>>>(mode, B, n, nchunks, partial, log_prob);
  return pso_check_launch("pso_step_logprob");
}

int pso_pair_loss_fwd(int mode, int P, int n, const float* x, const float* x_prev, const void* eps_pol,
                      const void* eps_ref, int eps_dtype, const float* coef, const float* pref, float beta,
                      float clip_eps, float* lp_out, float* loss_out, void* ws, size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(PSO_MODE_OK(mode), "pso_pair_loss_fwd: bad mode %d", mode);
  PSO_ARG_CHECK(P > 0 && P <= 1024 && n > 0 && (n % 4) == 0,
                "pso_pair_loss_fwd: need 0<P<=1024, n>0, n%%4==0 (P=%d n=%d)", P, n);
  PSO_ARG_CHECK(x && x_prev && eps_pol && eps_ref && coef && pref && lp_out && loss_out,
                "pso_pair_loss_fwd: null pointer");
  PSO_ARG_CHECK(eps_dtype == PSO_F32 || eps_dtype == PSO_BF16, "pso_pair_loss_fwd: bad eps dtype");
  PSO_ARG_CHECK(ws && ws_bytes >= pso_pair_loss_ws_bytes(P, n), "pso_pair_loss_fwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int nchunks = cdiv(n, LP_CHUNK);
  double* partial = (double*)ws;
  dim3 g1(nchunks, 4 * P);
  PSO_MODE_DISPATCH(mode, (lp_partial_kernel<M_, true><<<g1, LP_THREADS, 0, st>>>(
                              n, x, x_prev, eps_pol, eps_ref, eps_dtype, nullptr, 0, coef, nullptr, partial)))
  pair_loss_finalize_kernel<<<1, 256, 0, st>>>(mode, P, n, nchunks, pref, beta, clip_eps, partial, lp_out, loss_out);
  return pso_check_launch("pso_pair_loss_fwd");
}

int pso_pair_loss_bwd(int mode, int P, int n, const float* x, const float* x_prev, const void* eps_pol,
                      int eps_dtype, const float* coef, const float* pref, float beta, float clip_eps,
                      const float* grad_out, float grad_scale, void* deps_pol, int deps_dtype, const void* ws,
                      size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(PSO_MODE_OK(mode), "pso_pair_loss_bwd: bad mode %d", mode);
  PSO_ARG_CHECK(P > 0 && n > 0 && (n % 4) == 0, "pso_pair_loss_bwd: need P>0, n>0, n%%4==0");
  PSO_ARG_CHECK(x && x_prev && eps_pol && coef && pref && deps_pol, "pso_pair_loss_bwd: null pointer");
  PSO_ARG_CHECK(eps_dtype == PSO_F32 || eps_dtype == PSO_BF16, "pso_pair_loss_bwd: bad eps dtype");
  PSO_ARG_CHECK(deps_dtype == PSO_F32 || deps_dtype == PSO_BF16, "pso_pair_loss_bwd: bad deps dtype");
  PSO_ARG_CHECK(ws && ws_bytes >= pso_pair_loss_ws_bytes(P, n), "pso_pair_loss_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int nchunks = cdiv(n, LP_CHUNK);
  const double* partial = (const double*)ws;
  dim3 g2(nchunks, 2 * P);
  PSO_MODE_DISPATCH(mode, (pair_grad_kernel<M_><<<g2, LP_THREADS, 0, st>>>(
                              P, n, nchunks, x, x_prev, eps_pol, eps_dtype, coef, pref, beta, clip_eps, grad_out,
                              grad_scale, partial, deps_pol, deps_dtype)))
  return pso_check_launch("pso_pair_loss_bwd");
}

int pso_pair_loss_from_lp(int mode, int P, const float* lp_pol, const float* lp_ref, const float* pref, float beta,
                          float clip_eps, float* loss_out, float* dlp_out, void* stream) {
  PSO_ARG_CHECK(PSO_MODE_OK(mode), "pso_pair_loss_from_lp: bad mode %d", mode);
  PSO_ARG_CHECK(P > 0 && P <= 1024, "pso_pair_loss_from_lp: need 0 < P <= 1024 (P=%d)", P);
  PSO_ARG_CHECK(lp_pol && lp_ref && pref && loss_out, "pso_pair_loss_from_lp: null pointer");
  pair_loss_lp_kernel<<<1, 256, 0, (hipStream_t)stream>>>(mode, P, lp_pol, lp_ref, pref, beta, clip_eps, loss_out,
                                                          dlp_out);
  return pso_check_launch("pso_pair_loss_from_lp");
}

}  // extern "C"
