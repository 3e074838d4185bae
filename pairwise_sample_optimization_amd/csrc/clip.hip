// CLIP towers and the reward-image path for gfx950: the prompt encoders of the SDXL trainers (CLIP ViT-L/14 text +
// OpenCLIP ViT-bigG/14 text, `encode_prompt` T:81-118) and the PickScore reward model (CLIP ViT-H/14 vision + text,
// pso_pytorch/pickscore_utils.py:12-62) with its image preprocessing (T:632-640: uint8 quantisation, then the
// CLIPImageProcessor's PIL bicubic resize / centre crop / rescale / normalise), plus the synthetic light_reward
// (pso_pytorch/rewards.py:5-9).  The projections / MLPs of these towers run on the MFMA GEMM (gemm.hip) and
// LayerNorm (norm.hip); this file holds what is specific to them:
//   * attn_small_kernel  - softmax attention over short sequences (77 text / 257 vision tokens), head dim <= 128,
//                          optional causal mask (CLIP text), fp32 online softmax; K/V chunks staged in LDS as fp32
//   * act_kernel         - GELU (erf) / quick-GELU (x * sigmoid(1.702 x)) in place
//   * embed kernels      - token + position embeddings (text), class token + patch + position embeddings (vision)
//   * rowdot_kernel      - cosine similarity of matched rows (PickScore's diag(text_n @ image_n^T))
//   * row_mean_kernel    - per-image mean (light_reward)
//   * clip_preprocess    - [-1,1] image -> uint8 (the trainer's quantisation, in the image dtype) -> PIL bicubic
//                          (antialiased, 8-bit fixed point, horizontal then vertical pass) -> crop -> /255 ->
//                          (x - mean) / std -> 14x14 patch rows for the patch-embedding GEMM
#include <math.h>
#include <map>
#include <mutex>
#include <vector>

#include "common.h"

namespace {

constexpr int AS_ROWS = 4;     // query rows per wave
constexpr int AS_WAVES = 4;    // waves per workgroup -> 16 query rows
constexpr int AS_KC = 64;      // keys per LDS chunk
constexpr int AS_DMAX = 128;

// One workgroup = 16 queries of one (batch, head).  Lane j owns key j of the current chunk for the scores and output
// dims d = lane, lane + 64 for the P.V product.  K is staged transposed (Kt[d][j]) so the score loop reads one
// conflict-free dword per lane per d; q rows and the chunk's probabilities are broadcast from LDS.
__global__ __launch_bounds__(256) void attn_small_kernel(int S, int D, int H, const bf16_t* __restrict__ q, long ldq,
                                                         long sqb, const bf16_t* __restrict__ k, long ldk, long skb,
                                                         const bf16_t* __restrict__ v, long ldv, long svb, int causal,
                                                         float scale, bf16_t* __restrict__ o, long ldo, long sob) {
  __shared__ float kt[AS_DMAX][AS_KC + 1];
  __shared__ float vs[AS_KC][AS_DMAX + 1];
  __shared__ float qs[AS_WAVES * AS_ROWS][AS_DMAX];
  __shared__ float ps[AS_WAVES][AS_ROWS][AS_KC];
  const int b = blockIdx.z, h = blockIdx.y;
  const int q0 = blockIdx.x * AS_WAVES * AS_ROWS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16_t* qb = q + b * sqb + h * D;
  const bf16_t* kb = k + b * skb + h * D;
  const bf16_t* vb = v + b * svb + h * D;
  for (int i = tid; i < AS_WAVES * AS_ROWS * D; i += 256) {
    const int r = i / D, d = i - r * D;
    qs[r][d] = (q0 + r < S) ? bf2f(qb[(long)(q0 + r) * ldq + d]) * scale : 0.f;
  }
  float m[AS_ROWS], l[AS_ROWS], acc[AS_ROWS][2];
#pragma unroll
  for (int r = 0; r < AS_ROWS; ++r) {
    m[r] = -INFINITY;
    l[r] = 0.f;
    acc[r][0] = acc[r][1] = 0.f;
  }
  const int last_q = min(S, q0 + AS_WAVES * AS_ROWS) - 1;
  const int kend = causal ? last_q + 1 : S;
  for (int c0 = 0; c0 < kend; c0 += AS_KC) {
    __syncthreads();  // previous chunk fully consumed (and q staged on the first pass)
    for (int i = tid; i < AS_KC * D; i += 256) {
      const int j = i / D, d = i - j * D;
      const bool in = c0 + j < S;
      kt[d][j] = in ? bf2f(kb[(long)(c0 + j) * ldk + d]) : 0.f;
      vs[j][d] = in ? bf2f(vb[(long)(c0 + j) * ldv + d]) : 0.f;
    }
    __syncthreads();
    const int key = c0 + lane;
    float s[AS_ROWS];
#pragma unroll
    for (int r = 0; r < AS_ROWS; ++r) s[r] = 0.f;
    for (int d = 0; d < D; ++d) {
      const float kv = kt[d][lane];
#pragma unroll
      for (int r = 0; r < AS_ROWS; ++r) s[r] = fmaf(qs[wave * AS_ROWS + r][d], kv, s[r]);
    }
#pragma unroll
    for (int r = 0; r < AS_ROWS; ++r) {
      const int qi = q0 + wave * AS_ROWS + r;
      const bool ok = key < S && !(causal && key > qi);
      const float sv = ok ? s[r] : -INFINITY;
      const float mc = warp_max(sv);
      const float mn = fmaxf(m[r], mc);
      const float p = ok ? __expf(sv - mn) : 0.f;
      const float corr = m[r] == -INFINITY ? 0.f : __expf(m[r] - mn);
      l[r] = l[r] * corr + warp_sum(p);
      acc[r][0] *= corr;
      acc[r][1] *= corr;
      m[r] = mn == -INFINITY ? m[r] : mn;
      ps[wave][r][lane] = p;
    }
    __builtin_amdgcn_s_barrier();  // ps written by this wave only; a wave-level fence suffices, the barrier is cheap
    const int nj = min(AS_KC, kend - c0);
    for (int j = 0; j < nj; ++j) {
      const float v0 = lane < D ? vs[j][lane] : 0.f;
      const float v1 = lane + 64 < D ? vs[j][lane + 64] : 0.f;
#pragma unroll
      for (int r = 0; r < AS_ROWS; ++r) {
        const float p = ps[wave][r][j];
        acc[r][0] = fmaf(p, v0, acc[r][0]);
        acc[r][1] = fmaf(p, v1, acc[r][1]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < AS_ROWS; ++r) {
    const int qi = q0 + wave * AS_ROWS + r;
    if (qi >= S) continue;
    const float inv = l[r] > 0.f ? 1.f / l[r] : 0.f;
    bf16_t* orow = o + b * sob + (long)qi * ldo + h * D;
    if (lane < D) orow[lane] = f2bf(acc[r][0] * inv);
    if (lane + 64 < D) orow[lane + 64] = f2bf(acc[r][1] * inv);
  }
}

__global__ void act_kernel(long n, bf16_t* __restrict__ x, int mode) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float a = bf2f(x[i]);
    float y;
    if (mode == PSO_ACT_QUICK_GELU) y = a / (1.f + __expf(-1.702f * a));
    else y = 0.5f * a * (1.f + erff(a * 0.70710678118654752f));
    x[i] = f2bf(y);
  }
}

// out[b*S + t] = tok[ids[b*S + t]] + pos[t]   (fp32 add, one rounding)
__global__ void embed_tokens_kernel(int S, int C, const int64_t* __restrict__ ids, const bf16_t* __restrict__ tok,
                                    const bf16_t* __restrict__ pos, bf16_t* __restrict__ out) {
  const long row = blockIdx.x;
  const int t = (int)(row % S);
  const bf16_t* tr = tok + ids[row] * (long)C;
  const bf16_t* pr = pos + (long)t * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) out[row * C + c] = f2bf(bf2f(tr[c]) + bf2f(pr[c]));
}

// vision embeddings: row 0 of image b = class + pos[0]; row 1 + p = patch[b][p] + pos[1 + p]
__global__ void embed_vision_kernel(int P, int C, const bf16_t* __restrict__ patch, const bf16_t* __restrict__ cls,
                                    const bf16_t* __restrict__ pos, bf16_t* __restrict__ out) {
  const long row = blockIdx.x;  // over B * (P + 1)
  const int t = (int)(row % (P + 1));
  const long b = row / (P + 1);
  const bf16_t* src = t == 0 ? cls : patch + (b * P + t - 1) * (long)C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) out[row * C + c] = f2bf(bf2f(src[c]) + bf2f(pos[(long)t * C + c]));
}

// out[i] = <a_i, b_i> / (|a_i| |b_i|)  (fp32 rows; one wave per row, fp64 sums)
__global__ void rowdot_kernel(int n, int C, const float* __restrict__ a, long lda, const float* __restrict__ b,
                              long ldb, float* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= n) return;
  double ab = 0, aa = 0, bb = 0;
  for (int c = lane; c < C; c += 64) {
    const double x = a[(long)row * lda + c], y = b[(long)row * ldb + c];
    ab += x * y;
    aa += x * x;
    bb += y * y;
  }
  ab = warp_sum_d(ab);
  aa = warp_sum_d(aa);
  bb = warp_sum_d(bb);
  if (lane == 0) out[row] = (float)((ab / sqrt(aa)) / sqrt(bb));
}

// out[r] = mean of the n bf16 values of row r (fp64 accumulation)
__global__ __launch_bounds__(256) void row_mean_kernel(long n, const bf16_t* __restrict__ x, float* __restrict__ out) {
  __shared__ double red[4];
  const bf16_t* row = x + blockIdx.x * n;
  double s = 0;
  const long n8 = n / 8;
  for (long i = threadIdx.x; i < n8; i += 256) {
    const uint4 u = reinterpret_cast<const uint4*>(row)[i];
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
    float f = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) f += bf2f(w[e] & 0xffff) + bf2f(w[e] >> 16);
    s += f;
  }
  for (long i = n8 * 8 + threadIdx.x; i < n; i += 256) s += bf2f(row[i]);
  s = warp_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (float)((red[0] + red[1] + red[2] + red[3]) / (double)n);
}

// patch rows of an already processed NCHW fp32 image: out[(b * np + py) * np + px][c * P * P + ky * P + kx] (bf16)
__global__ void patchify_kernel(int C, int S, int P, int kpad, const float* __restrict__ x, bf16_t* __restrict__ out) {
  const int b = blockIdx.y;
  const int np = S / P;
  const long per_img = (long)np * np * kpad;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < per_img; i += (long)gridDim.x * blockDim.x) {
    const int kk = (int)(i % kpad);
    const long patch = i / kpad;
    float v = 0.f;
    if (kk < C * P * P) {
      const int c = kk / (P * P), ky = (kk / P) % P, kx = kk % P;
      const int py = (int)(patch / np), px = (int)(patch % np);
      v = x[(((long)b * C + c) * S + py * P + ky) * S + px * P + kx];
    }
    out[(long)b * per_img + i] = f2bf(v);
  }
}

// ---- image preprocessing -------------------------------------------------------------------------------------------
// PIL ImagingResample for 8-bit images (libImaging/Resample.c): per output index a window [xmin, xmin + xmax) of
// fixed-point (22 fractional bits) coefficients; horizontal pass into a uint8 intermediate, then the vertical pass.
constexpr int PIL_PREC = 22;

__device__ __forceinline__ uint8_t clip8(long v) {
  v >>= PIL_PREC;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// trainer quantisation ((img + 1) * 127.5).clamp(0, 255).to(uint8) in the image dtype (bf16: every op rounds), then
// the horizontal resample of image rows [y0, y0 + rows): tmp[b][y][ox][c]
__global__ void resample_h_kernel(int H, int W, int OW, int y0, int rows, const void* __restrict__ img, int img_dtype,
                                  const int* __restrict__ bounds, const int* __restrict__ coef, int ksize,
                                  uint8_t* __restrict__ tmp) {
  const int b = blockIdx.y;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (long)rows * OW * 3; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % 3);
    const int ox = (int)((i / 3) % OW);
    const int y = (int)(i / (3L * OW));
    const int xmin = bounds[2 * ox], xn = bounds[2 * ox + 1];
    const long base = (((long)b * H + y0 + y) * W) * 3 + c;
    long ss = 1L << (PIL_PREC - 1);
    for (int x = 0; x < xn; ++x) {
      const long e = base + (long)(xmin + x) * 3;
      int u;
      if (img_dtype == PSO_U8) {
        u = reinterpret_cast<const uint8_t*>(img)[e];
      } else {
        float t;
        if (img_dtype == PSO_BF16) t = bf_round(bf_round(bf2f(reinterpret_cast<const bf16_t*>(img)[e]) + 1.0f) * 127.5f);
        else t = (reinterpret_cast<const float*>(img)[e] + 1.0f) * 127.5f;
        u = (int)fminf(fmaxf(t, 0.f), 255.f);  // clamp, then .to(torch.uint8) truncates
      }
      ss += (long)u * coef[ox * ksize + x];
    }
    tmp[(((long)b * rows + y) * OW + ox) * 3 + c] = clip8(ss);
  }
}

// vertical resample + centre crop + rescale + normalise + patchify:
//   out[(b * PP + py * np + px)][c * P * P + ky * P + kx] (K padded to kpad with zeros), bf16
__global__ void resample_v_patch_kernel(int rows, int OW, int OH, int crop, int top, int left, int P, int kpad,
                                        const uint8_t* __restrict__ tmp, const int* __restrict__ bounds,
                                        const int* __restrict__ coef, int ksize, float m0, float m1, float m2,
                                        float s0, float s1, float s2, bf16_t* __restrict__ out) {
  const int b = blockIdx.y;
  const int np = crop / P;
  const long per_img = (long)np * np * kpad;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < per_img; i += (long)gridDim.x * blockDim.x) {
    const int kk = (int)(i % kpad);
    const long patch = i / kpad;
    float val = 0.f;
    if (kk < 3 * P * P) {
      const int c = kk / (P * P), ky = (kk / P) % P, kx = kk % P;
      const int py = (int)(patch / np), px = (int)(patch % np);
      const int oy = top + py * P + ky, ox = left + px * P + kx;
      const int ymin = bounds[2 * oy], yn = bounds[2 * oy + 1];
      long ss = 1L << (PIL_PREC - 1);
      for (int y = 0; y < yn; ++y) ss += (long)tmp[(((long)b * rows + ymin + y) * OW + ox) * 3 + c] * coef[oy * ksize + y];
      const uint8_t u = clip8(ss);
      // transformers rescale (float64 * 1/255 -> float32) then (x - mean) / std in float32
      const float r = (float)((double)u * (1.0 / 255.0));
      const float mean = c == 0 ? m0 : (c == 1 ? m1 : m2);
      const float sd = c == 0 ? s0 : (c == 1 ? s1 : s2);
      val = (r - mean) / sd;
    }
    out[(long)b * per_img + i] = f2bf(val);
  }
}

// Host: PIL precompute_coeffs + normalize_coeffs_8bpc (double arithmetic as in Resample.c), cached per (in, out) size
struct ResampleTable {
  int ksize = 0;
  int* d_bounds = nullptr;
  int* d_coef = nullptr;
  std::vector<int> bounds;
};

double bicubic_filter(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

int build_table(int in_size, int out_size, ResampleTable& t) {
  const double support0 = 2.0;  // bicubic
  double scale = (double)in_size / out_size, filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = support0 * filterscale;
  const int ksize = (int)ceil(support) * 2 + 1;
  std::vector<double> kk((size_t)out_size * ksize);
  std::vector<int> bounds(2 * (size_t)out_size), coef((size_t)out_size * ksize);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double* k = &kk[(size_t)xx * ksize];
    int x = 0;
    for (; x < xmax; ++x) {
      const double w = bicubic_filter((x + xmin - center + 0.5) * ss);
      k[x] = w;
      ww += w;
    }
    for (x = 0; x < xmax; ++x)
      if (ww != 0.0) k[x] /= ww;
    for (; x < ksize; ++x) k[x] = 0;
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  for (size_t i = 0; i < kk.size(); ++i)
    coef[i] = kk[i] < 0 ? (int)(-0.5 + kk[i] * (1 << PIL_PREC)) : (int)(0.5 + kk[i] * (1 << PIL_PREC));
  t.ksize = ksize;
  t.bounds = bounds;
  if (hipMalloc(&t.d_bounds, bounds.size() * sizeof(int)) != hipSuccess ||
      hipMalloc(&t.d_coef, coef.size() * sizeof(int)) != hipSuccess)
    return PSO_ERR_HIP;
  if (hipMemcpy(t.d_bounds, bounds.data(), bounds.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(t.d_coef, coef.data(), coef.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
    return PSO_ERR_HIP;
  return PSO_OK;
}

std::mutex g_tab_mu;
std::map<std::pair<int, int>, ResampleTable> g_tabs;  // immutable once built (metadata, not hot-path allocations)

int get_table(int in_size, int out_size, const ResampleTable** t) {
  std::lock_guard<std::mutex> lk(g_tab_mu);
  auto key = std::make_pair(in_size, out_size);
  auto it = g_tabs.find(key);
  if (it == g_tabs.end()) {
    ResampleTable nt;
    const int rc = build_table(in_size, out_size, nt);
    if (rc != PSO_OK) {
      pso_set_error("pso_clip_preprocess: resample table upload failed");
      return rc;
    }
    it = g_tabs.emplace(key, nt).first;
  }
  *t = &it->second;
  return PSO_OK;
}

}  // namespace

extern "C" {

int pso_attention_small(int B, int H, int S, int D, const void* q, long ldq, long sq_b, const void* k, long ldk,
                        long sk_b, const void* v, long ldv, long sv_b, int causal, float scale, void* o, long ldo,
                        long so_b, void* stream) {
  PSO_ARG_CHECK(B > 0 && H > 0 && S > 0 && D > 0 && D <= AS_DMAX, "pso_attention_small: bad shape (D <= 128)");
  PSO_ARG_CHECK(q && k && v && o, "pso_attention_small: null operand");
  dim3 grid(cdiv(S, AS_WAVES * AS_ROWS), H, B);
  attn_small_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(S, D, H, (const bf16_t*)q, ldq, sq_b, (const bf16_t*)k, ldk,
                                                          sk_b, (const bf16_t*)v, ldv, sv_b, causal, scale,
                                                          (bf16_t*)o, ldo, so_b);
  return pso_check_launch("pso_attention_small");
}

int pso_activation(long n, void* x, int mode, void* stream) {
  PSO_ARG_CHECK(x && (mode == PSO_ACT_GELU || mode == PSO_ACT_QUICK_GELU), "pso_activation: bad args");
  if (n <= 0) return PSO_OK;
  const int grid = (int)(n / 256 + 1 > 8192 ? 8192 : n / 256 + 1);
  act_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(n, (bf16_t*)x, mode);
  return pso_check_launch("pso_activation");
}

int pso_embed_tokens(int B, int S, int C, const int64_t* ids, const void* tok, const void* pos, void* out,
                     void* stream) {
  PSO_ARG_CHECK(B > 0 && S > 0 && C > 0 && ids && tok && pos && out, "pso_embed_tokens: bad args");
  embed_tokens_kernel<<<B * S, 256, 0, (hipStream_t)stream>>>(S, C, ids, (const bf16_t*)tok, (const bf16_t*)pos,
                                                              (bf16_t*)out);
  return pso_check_launch("pso_embed_tokens");
}

int pso_embed_vision(int B, int P, int C, const void* patch, const void* cls, const void* pos, void* out,
                     void* stream) {
  PSO_ARG_CHECK(B > 0 && P > 0 && C > 0 && patch && cls && pos && out, "pso_embed_vision: bad args");
  embed_vision_kernel<<<B * (P + 1), 256, 0, (hipStream_t)stream>>>(P, C, (const bf16_t*)patch, (const bf16_t*)cls,
                                                                    (const bf16_t*)pos, (bf16_t*)out);
  return pso_check_launch("pso_embed_vision");
}

int pso_cosine_rows(int n, int C, const float* a, long lda, const float* b, long ldb, float* out, void* stream) {
  PSO_ARG_CHECK(n > 0 && C > 0 && a && b && out, "pso_cosine_rows: bad args");
  rowdot_kernel<<<cdiv(n, 4), 256, 0, (hipStream_t)stream>>>(n, C, a, lda, b, ldb, out);
  return pso_check_launch("pso_cosine_rows");
}

int pso_row_mean(int rows, long n, const void* x, float* out, void* stream) {
  PSO_ARG_CHECK(rows > 0 && n > 0 && x && out && (((uintptr_t)x) & 15) == 0 && (n % 8) == 0,
                "pso_row_mean: bad args (16-B aligned rows of n %% 8 == 0 values)");
  row_mean_kernel<<<rows, 256, 0, (hipStream_t)stream>>>(n, (const bf16_t*)x, out);
  return pso_check_launch("pso_row_mean");
}

int pso_patchify(int B, int C, int S, int P, int kpad, const float* x, void* out, void* stream) {
  PSO_ARG_CHECK(B > 0 && C > 0 && P > 0 && S % P == 0 && kpad >= C * P * P && x && out, "pso_patchify: bad args");
  const long per = (long)(S / P) * (S / P) * kpad;
  patchify_kernel<<<dim3(cdiv(per, 256) > 4096 ? 4096 : cdiv(per, 256), B), 256, 0, (hipStream_t)stream>>>(
      C, S, P, kpad, x, (bf16_t*)out);
  return pso_check_launch("pso_patchify");
}

size_t pso_clip_preprocess_ws_bytes(int B, int H, int W, int size) {
  // horizontal-pass intermediate: every source row x the resized width, 3 uint8 channels
  const int ow = H <= W ? (int)((long)size * W / H) : size;
  return (size_t)B * H * ow * 3;
}

int pso_clip_preprocess(int B, int H, int W, const void* img, int img_dtype, int size, int patch, int kpad,
                        const float* mean, const float* stdv, void* out, void* ws, size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(B > 0 && H > 0 && W > 0 && img && out && ws && mean && stdv, "pso_clip_preprocess: null / bad shape");
  PSO_ARG_CHECK(img_dtype == PSO_BF16 || img_dtype == PSO_F32 || img_dtype == PSO_U8,
                "pso_clip_preprocess: the image must be bf16 / f32 in [-1, 1] or uint8, NHWC [B,H,W,3]");
  PSO_ARG_CHECK(patch > 0 && size % patch == 0 && kpad >= 3 * patch * patch && kpad % 8 == 0,
                "pso_clip_preprocess: size must be a multiple of patch, kpad >= 3 * patch^2 (multiple of 8)");
  PSO_ARG_CHECK(ws_bytes >= pso_clip_preprocess_ws_bytes(B, H, W, size), "pso_clip_preprocess: workspace too small");
  // transformers CLIPImageProcessor: shortest edge -> size (long edge int(size * long / short)), centre crop size
  int oh, ow;
  if (H <= W) { oh = size; ow = (int)((long)size * W / H); }
  else { ow = size; oh = (int)((long)size * H / W); }
  const int top = (oh - size) / 2, left = (ow - size) / 2;
  const ResampleTable *th, *tv;
  int rc = get_table(W, ow, &th);
  if (rc != PSO_OK) return rc;
  rc = get_table(H, oh, &tv);
  if (rc != PSO_OK) return rc;
  hipStream_t st = (hipStream_t)stream;
  uint8_t* tmp = (uint8_t*)ws;
  const long htot = (long)H * ow * 3;
  resample_h_kernel<<<dim3(cdiv(htot, 256) > 4096 ? 4096 : cdiv(htot, 256), B), 256, 0, st>>>(
      H, W, ow, 0, H, img, img_dtype, th->d_bounds, th->d_coef, th->ksize, tmp);
  rc = pso_check_launch("pso_clip_preprocess(h)");
  if (rc != PSO_OK) return rc;
  const long np = size / patch;
  const long vtot = np * np * kpad;
  resample_v_patch_kernel<<<dim3(cdiv(vtot, 256) > 4096 ? 4096 : cdiv(vtot, 256), B), 256, 0, st>>>(
      H, ow, oh, size, top, left, patch, kpad, tmp, tv->d_bounds, tv->d_coef, tv->ksize, mean[0], mean[1], mean[2],
      stdv[0], stdv[1], stdv[2], (bf16_t*)out);
  return pso_check_launch("pso_clip_preprocess(v)");
}

}  // extern "C"
