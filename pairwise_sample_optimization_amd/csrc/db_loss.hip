// DreamBooth PSO loss (C5), forward and backward to the UNet's eps prediction.
//
// Reference arithmetic (personalization/train_pso_sdxl_turbo_dreambooth.py = DB; restated, never copied), EDM-style
// epsilon training with an Euler scheduler (the recipe's --do_edm_style_training, scripts/pso_dog.sh:35):
//   x0_pred_i = eps_i * (-sigma_i) + noisy_i                                DB:1854-1855
//   l_i       = mean_{C,H,W}( sigma_i^-2 * (x0_pred_i - x0_i)^2 )           DB:1864-1865, 1885-1890
//   (w_b, l_b) = images b and B + b (instance first, negatives second)       DB:1731, 1891
//   model_diff_b = l_w - nd * l_l                                           DB:1892
//   "pso":    logits = ref_diff - model_diff (ref: adapters disabled)        DB:1894-1920
//             loss   = mean_b -log sigmoid(beta * logits)                   DB:1924-1925
//   "pso_db": logits = -model_diff ; loss = mean_b relu(1 - beta * logits)  DB:1921-1927
//   + prior_w * mean_b l_l                                                  DB:1932-1935
// The reference forms x0_pred in the autocast dtype and the MSE in fp32 (DB:1886 .float()); here both are fp32 from
// the bf16 eps.
//
// Same three-kernel shape as pso_loss.hip: per-(image, chunk) fp64 partials of the weighted squared error (fixed
// order => deterministic), a one-block finalize (per-image losses, logits, loss), and a gradient pass in which every
// block re-derives its image's dL/dl_i from the partials and streams dL/deps = g_i * 2/(n sigma_i^2) * (-sigma_i) *
// (x0_pred - x0).
#include "common.h"

#define DB_CHUNK 8192
#define DB_THREADS 256

__device__ __forceinline__ void db_load4(const void* p, int dtype, size_t i, float* e) {
  if (dtype == PSO_BF16) {
    const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(p) + i);
    e[0] = bf2f(v.x & 0xffff); e[1] = bf2f(v.x >> 16); e[2] = bf2f(v.y & 0xffff); e[3] = bf2f(v.y >> 16);
  } else {
    const float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + i);
    e[0] = v.x; e[1] = v.y; e[2] = v.z; e[3] = v.w;
  }
}

// grid (nchunks, nsrc * 2B): combo = src * 2B + img (src 0: policy eps, 1: reference eps)
__global__ __launch_bounds__(DB_THREADS) void db_partial_kernel(int n2b, int n, const void* eps_pol,
                                                                const void* eps_ref, int eps_dtype,
                                                                const float* __restrict__ noisy,
                                                                const float* __restrict__ x0,
                                                                const float* __restrict__ sigma,
                                                                double* __restrict__ partial) {
  __shared__ double red[DB_THREADS / 64];
  const int combo = blockIdx.y;
  const int src = combo / n2b, img = combo - src * n2b;
  const void* eps = src ? eps_ref : eps_pol;
  const float s = sigma[img];
  const float w = 1.0f / (s * s);
  const size_t base = (size_t)img * n;
  const int c0 = blockIdx.x * DB_CHUNK, c1 = min(n, c0 + DB_CHUNK);
  double acc = 0.0;
  for (int i = c0 + threadIdx.x * 4; i < c1; i += DB_THREADS * 4) {
    float e[4];
    db_load4(eps, eps_dtype, base + i, e);
    const float4 nv = *reinterpret_cast<const float4*>(noisy + base + i);
    const float4 tv = *reinterpret_cast<const float4*>(x0 + base + i);
    const float ns[4] = {nv.x, nv.y, nv.z, nv.w}, ts[4] = {tv.x, tv.y, tv.z, tv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d = (e[j] * -s + ns[j]) - ts[j];
      acc += (double)(w * (d * d));
    }
  }
  acc = warp_sum_d(acc);
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[wv] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < DB_THREADS / 64; ++k) t += red[k];
    partial[(size_t)combo * gridDim.x + blockIdx.x] = t;
  }
}

__device__ __forceinline__ float db_image_loss(const double* partial, int combo, int nchunks, int n) {
  double s = 0.0;
  for (int c = 0; c < nchunks; ++c) s += partial[(size_t)combo * nchunks + c];
  return (float)(s / (double)n);
}

struct DbPair {
  float lw, ll, logit, loss, gw, gl;  // gw / gl: dL/d l_w, dL/d l_l (times the upstream gradient)
};

__device__ __forceinline__ DbPair db_pair(const double* partial, int b, int B, int nchunks, int n, int loss_type,
                                          float beta, float nd, float prior_w, float up) {
  DbPair r;
  r.lw = db_image_loss(partial, b, nchunks, n);
  r.ll = db_image_loss(partial, B + b, nchunks, n);
  const float model_diff = r.lw - nd * r.ll;
  float logit = -model_diff;
  if (loss_type == PSO_DB_SIGMOID) {
    const float rw = db_image_loss(partial, 2 * B + b, nchunks, n), rl = db_image_loss(partial, 3 * B + b, nchunks, n);
    logit = (rw - nd * rl) - model_diff;
  }
  r.logit = logit;
  const float z = beta * logit;
  float dlogit;
  if (loss_type == PSO_DB_SIGMOID) {  // -log sigmoid(z) = softplus(-z)
    r.loss = z > 0.f ? log1pf(expf(-z)) : -z + log1pf(expf(z));
    dlogit = -beta / (1.0f + expf(z));
  } else {  // relu(1 - z); torch.relu passes no gradient at 0
    r.loss = fmaxf(1.0f - z, 0.0f);
    dlogit = (1.0f - z > 0.0f) ? -beta : 0.0f;
  }
  dlogit = dlogit / (float)B * up;
  // logits = c - lw + nd * ll  =>  dlogit/dlw = -1, dlogit/dll = +nd ;  the prior term adds prior_w / B to dL/dll
  r.gw = -dlogit;
  r.gl = nd * dlogit + prior_w / (float)B * up;
  return r;
}

// one block: per-image losses (policy, then reference), logits [B], loss scalar (fixed-order means)
__global__ void db_finalize_kernel(int B, int n, int nchunks, int loss_type, float beta, float nd, float prior_w,
                                   const double* __restrict__ partial, float* __restrict__ losses_out,
                                   float* __restrict__ logits_out, float* __restrict__ loss_out) {
  __shared__ float sh_loss[1024], sh_ll[1024];
  const int nsrc = loss_type == PSO_DB_SIGMOID ? 2 : 1;
  for (int c = threadIdx.x; c < nsrc * 2 * B; c += blockDim.x)
    if (losses_out) losses_out[c] = db_image_loss(partial, c, nchunks, n);
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const DbPair r = db_pair(partial, b, B, nchunks, n, loss_type, beta, nd, prior_w, 1.0f);
    sh_loss[b] = r.loss;
    sh_ll[b] = r.ll;
    if (logits_out) logits_out[b] = r.logit;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double L = 0.0, P = 0.0;
    for (int b = 0; b < B; ++b) {
      L += (double)sh_loss[b];
      P += (double)sh_ll[b];
    }
    loss_out[0] = (float)(L / (double)B + (double)prior_w * (P / (double)B));
  }
}

// grid (nchunks, 2B): dL/d eps_i = g_i * (2 / (n sigma_i^2)) * (-sigma_i) * (x0_pred_i - x0_i)
__global__ __launch_bounds__(DB_THREADS) void db_grad_kernel(int B, int n, int nchunks, int loss_type, float beta,
                                                             float nd, float prior_w,
                                                             const float* __restrict__ grad_out, float grad_scale,
                                                             const void* eps, int eps_dtype,
                                                             const float* __restrict__ noisy,
                                                             const float* __restrict__ x0,
                                                             const float* __restrict__ sigma,
                                                             const double* __restrict__ partial, void* deps,
                                                             int deps_dtype) {
  const int img = blockIdx.y;
  const int b = img < B ? img : img - B;
  __shared__ float g_sh;
  if (threadIdx.x == 0) {
    const float up = grad_out ? grad_out[0] * grad_scale : grad_scale;
    const DbPair r = db_pair(partial, b, B, nchunks, n, loss_type, beta, nd, prior_w, up);
    g_sh = img < B ? r.gw : r.gl;
  }
  __syncthreads();
  const float s = sigma[img];
  const float scale = g_sh * 2.0f / ((float)n * s * s) * -s;
  const size_t base = (size_t)img * n;
  const int c0 = blockIdx.x * DB_CHUNK, c1 = min(n, c0 + DB_CHUNK);
  for (int i = c0 + threadIdx.x * 4; i < c1; i += DB_THREADS * 4) {
    float e[4];
    db_load4(eps, eps_dtype, base + i, e);
    const float4 nv = *reinterpret_cast<const float4*>(noisy + base + i);
    const float4 tv = *reinterpret_cast<const float4*>(x0 + base + i);
    const float ns[4] = {nv.x, nv.y, nv.z, nv.w}, ts[4] = {tv.x, tv.y, tv.z, tv.w};
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = scale * ((e[j] * -s + ns[j]) - ts[j]);
    if (deps_dtype == PSO_BF16)
      *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(deps) + base + i) =
          make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
    else
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(deps) + base + i) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

extern "C" {

size_t pso_db_loss_ws_bytes(int B, int n) { return (size_t)4 * B * cdiv(n, DB_CHUNK) * sizeof(double); }

int pso_db_loss_fwd(int loss_type, int B, int n, const void* eps, const void* eps_ref, int eps_dtype,
                    const float* noisy, const float* x0, const float* sigma, float beta, float neg_defactor,
                    float prior_w, float* losses_out, float* logits_out, float* loss_out, void* ws, size_t ws_bytes,
                    void* stream) {
  PSO_ARG_CHECK(loss_type == PSO_DB_SIGMOID || loss_type == PSO_DB_HINGE, "pso_db_loss_fwd: bad loss type %d",
                loss_type);
  PSO_ARG_CHECK(B > 0 && B <= 1024 && n > 0 && (n % 4) == 0, "pso_db_loss_fwd: need 0<B<=1024, n%%4==0");
  PSO_ARG_CHECK(eps && noisy && x0 && sigma && loss_out, "pso_db_loss_fwd: null pointer");
  PSO_ARG_CHECK(loss_type == PSO_DB_HINGE || eps_ref, "pso_db_loss_fwd: loss 'pso' needs the reference eps");
  PSO_ARG_CHECK(eps_dtype == PSO_F32 || eps_dtype == PSO_BF16, "pso_db_loss_fwd: bad eps dtype");
  PSO_ARG_CHECK(ws && ws_bytes >= pso_db_loss_ws_bytes(B, n), "pso_db_loss_fwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int nchunks = cdiv(n, DB_CHUNK);
  const int nsrc = (loss_type == PSO_DB_SIGMOID) ? 2 : 1;
  double* partial = (double*)ws;
  db_partial_kernel<<<dim3(nchunks, nsrc * 2 * B), DB_THREADS, 0, st>>>(2 * B, n, eps, eps_ref, eps_dtype, noisy, x0,
                                                                       sigma, partial);
  db_finalize_kernel<<<1, 256, 0, st>>>(B, n, nchunks, loss_type, beta, neg_defactor, prior_w, partial, losses_out,
                                        logits_out, loss_out);
  return pso_check_launch("pso_db_loss_fwd");
}

int pso_db_loss_bwd(int loss_type, int B, int n, const void* eps, int eps_dtype, const float* noisy, const float* x0,
                    const float* sigma, float beta, float neg_defactor, float prior_w, const float* grad_out,
                    float grad_scale, void* deps, int deps_dtype, const void* ws, size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(loss_type == PSO_DB_SIGMOID || loss_type == PSO_DB_HINGE, "pso_db_loss_bwd: bad loss type");
  PSO_ARG_CHECK(B > 0 && B <= 1024 && n > 0 && (n % 4) == 0, "pso_db_loss_bwd: need 0<B<=1024, n%%4==0");
  PSO_ARG_CHECK(eps && noisy && x0 && sigma && deps, "pso_db_loss_bwd: null pointer");
  PSO_ARG_CHECK(eps_dtype == PSO_F32 || eps_dtype == PSO_BF16, "pso_db_loss_bwd: bad eps dtype");
  PSO_ARG_CHECK(deps_dtype == PSO_F32 || deps_dtype == PSO_BF16, "pso_db_loss_bwd: bad deps dtype");
  PSO_ARG_CHECK(ws && ws_bytes >= pso_db_loss_ws_bytes(B, n), "pso_db_loss_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int nchunks = cdiv(n, DB_CHUNK);
  db_grad_kernel<<<dim3(nchunks, 2 * B), DB_THREADS, 0, st>>>(B, n, nchunks, loss_type, beta, neg_defactor, prior_w,
                                                             grad_out, grad_scale, eps, eps_dtype, noisy, x0, sigma,
                                                             (const double*)ws, deps, deps_dtype);
  return pso_check_launch("pso_db_loss_bwd");
}

}  // extern "C"
