// Flash attention (head dim 64) forward and backward for gfx950, bf16 I/O, fp32 softmax state.
//
// Replaces the SDPA kernels of the 140 diffusers Attention modules of the SDXL UNet (attn1 self-attention over
// 4096/1024 tokens, attn2 cross-attention over the 77 text tokens; SURVEY §2 "SDPA", Appendix B).  Q/K/V/O are the
// projection GEMM outputs in their natural [B][S][heads*64] layout (head h = columns h*64..h*64+63, any row stride),
// so no head transposes are ever materialised.
//
// Forward: one workgroup = 4 waves = 128 query rows of one (batch, head); each wave owns 32 rows (2 x 16).  Scores are
// computed transposed, S^T = K . Q^T (v_mfma_f32_16x16x32_bf16 with the K fragment as the A operand), so every lane
// holds 16 of a query's 64 scores per key tile: row max / row sum need 2 cross-lane steps, and the exponentiated
// tile, converted to bf16 in place, IS the B operand of O^T = V^T . P^T (the key order inside the 32-deep MFMA step
// is permuted to match the accumulator layout; the V^T fragment with the same permutation comes from two
// ds_read_b64_tr_b16 per MFMA).  K/V tiles of 64 keys are double-buffered in LDS (register-staged, one barrier per
// tile); K uses the chunk^(row&7) swizzle for conflict-free ds_read_b128, V a chunk^(2*((row>>1)&3)) swizzle for
// conflict-free transposed reads.  Outputs O (bf16) and the log-sum-exp (fp32, natural log) for the backward.
//
// Backward (FlashAttention-2 split without atomics): a dK/dV kernel (key-block parallel, keys on the MFMA lane axis so
// P and dS are lane-local B operands) and a dQ kernel (query-block parallel, same structure as the forward), both
// recomputing P from Q, K and the saved LSE; delta = rowsum(dO * O) comes from a small pre-pass.
#include "common.h"

#define ATT_D 64
#define ATT_KT 64  // keys per tile
#define ATT_THREADS 256

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int swz_row(int r, int c) { return r * ATT_D + ((c ^ (r & 7)) << 3); }
__device__ __forceinline__ int swz_tr(int r, int c) { return r * ATT_D + ((c ^ (((r >> 1) & 3) << 1)) << 3); }

// 4 rows (r0..r0+3) x 16 columns (col0..col0+15) transposed read from a [row][64] bf16 image with swz_tr layout.
// Lane i of each 16-lane group receives column col0+i of the 4 rows.  Caller passes r0/col0 per 16-lane group.
__device__ __forceinline__ s16x4 tr_read(const bf16_t* img, int r0, int col0, int lane) {
  const int li = lane & 15;
  const int q = li >> 2, p = li & 3;
  const int row = r0 + q;
  const int col = col0 + 4 * p;
  const int off = swz_tr(row, col >> 3) + (col & 7);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + off));
}

__device__ __forceinline__ bf16x8 cat_frag(s16x4 a, s16x4 b) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 pack_p(const f32x4& a, const f32x4& b) {
  typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
  u32x4 v = {pack2bf(a[0], a[1]), pack2bf(a[2], a[3]), pack2bf(b[0], b[1]), pack2bf(b[2], b[3])};
  return __builtin_bit_cast(bf16x8, v);
}

struct AttnArgs {
  const bf16_t *q, *k, *v;
  long ldq, ldk, ldv;          // row strides (elements)
  long sq_b, sk_b, sv_b;       // batch strides (elements)
  bf16_t* o; long ldo; long so_b;
  float* lse;                  // [B][H][Sq]
  int Sq, Sk, H;
  float scale_log2;            // softmax scale * log2(e)
  // backward
  const bf16_t* dO; long lddo; long sdo_b;
  float* delta;                // [B][H][Sq]
  bf16_t *dq, *dk, *dv; long lddq, lddk, lddv; long sdq_b, sdk_b, sdv_b;
  float *dk_acc, *dv_acc;      // fp32 [B][Sk][H*64] when q is split (cross-attention)
  int q_split;
};

// stage a [64 rows][64 d] bf16 tile (rows r0.. of a [S][ld] matrix, zero beyond nrows) into registers: 2 chunks/thread
__device__ __forceinline__ void stage_load(uint4 (&r)[2], const bf16_t* base, long ld, int r0, int nrows, int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = tid + ATT_THREADS * i;
    const int row = q >> 3, ch = q & 7;
    r[i] = (r0 + row < nrows) ? *reinterpret_cast<const uint4*>(base + (long)(r0 + row) * ld + ch * 8)
                              : make_uint4(0, 0, 0, 0);
  }
}
template <bool TR>
__device__ __forceinline__ void stage_store(const uint4 (&r)[2], bf16_t* img, int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = tid + ATT_THREADS * i;
    const int row = q >> 3, ch = q & 7;
    *reinterpret_cast<uint4*>(img + (TR ? swz_tr(row, ch) : swz_row(row, ch))) = r[i];
  }
}

// ================================================================================================================
// forward
// ================================================================================================================
__global__ __launch_bounds__(ATT_THREADS, 2) void attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t sK[2][ATT_KT * ATT_D];
  __shared__ __attribute__((aligned(16))) bf16_t sV[2][ATT_KT * ATT_D];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int b = blockIdx.z, h = blockIdx.y;
  const int q0 = blockIdx.x * 128 + wave * 32;

  const bf16_t* Q = a.q + b * a.sq_b + h * ATT_D;
  const bf16_t* K = a.k + b * a.sk_b + h * ATT_D;
  const bf16_t* V = a.v + b * a.sv_b + h * ATT_D;

  // Q fragments (B operand of S^T = K.Q^T): lane holds Q[q0 + qi*16 + c][ds*32 + 8g .. +8]
  bf16x8 qf[2][2];
#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    const int qr = q0 + qi * 16 + c;
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (qr < a.Sq) v = *reinterpret_cast<const uint4*>(Q + (long)qr * a.ldq + ds * 32 + 8 * g);
      qf[qi][ds] = __builtin_bit_cast(bf16x8, v);
    }
  }

  f32x4 o[2][4];
#pragma unroll
  for (int qi = 0; qi < 2; ++qi)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qi][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};

  const int nkt = (a.Sk + ATT_KT - 1) / ATT_KT;
  uint4 rk[2], rv[2];
  stage_load(rk, K, a.ldk, 0, a.Sk, tid);
  stage_load(rv, V, a.ldv, 0, a.Sk, tid);
  stage_store<false>(rk, sK[0], tid);
  stage_store<true>(rv, sV[0], tid);
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) {
      stage_load(rk, K, a.ldk, (kt + 1) * ATT_KT, a.Sk, tid);
      stage_load(rv, V, a.ldv, (kt + 1) * ATT_KT, a.Sk, tid);
    }
    const bf16_t* k_img = sK[cur];
    const bf16_t* v_img = sV[cur];
    // ---- S^T tiles: s[qi][kj] holds S[q = qi*16 + c][key = kj*16 + 4g + r] ----
    f32x4 s[2][4];
#pragma unroll
    for (int kj = 0; kj < 4; ++kj) {
      bf16x8 kf[2];
#pragma unroll
      for (int ds = 0; ds < 2; ++ds)
        kf[ds] = *reinterpret_cast<const bf16x8*>(k_img + swz_row(kj * 16 + c, ds * 4 + g));
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[0], qf[qi][0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[1], qf[qi][1], acc, 0, 0, 0);
        s[qi][kj] = acc;
      }
    }
    // ---- online softmax (base 2) ----
    const int kbase = kt * ATT_KT;
#pragma unroll
    for (int qi = 0; qi < 2; ++qi) {
      float mx = -INFINITY;
#pragma unroll
      for (int kj = 0; kj < 4; ++kj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kbase + kj * 16 + 4 * g + r;
          float x = s[qi][kj][r] * a.scale_log2;
          if (key >= a.Sk) x = -INFINITY;
          s[qi][kj][r] = x;
          mx = fmaxf(mx, x);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run[qi], mx);
      const float alpha = exp2f(m_run[qi] - m_new);
      float sum = 0.f;
#pragma unroll
      for (int kj = 0; kj < 4; ++kj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2f(s[qi][kj][r] - m_new);
          s[qi][kj][r] = p;
          sum += p;
        }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      l_run[qi] = l_run[qi] * alpha + sum;
      m_run[qi] = m_new;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[qi][dt] *= alpha;
    }
    // ---- O^T += V^T . P^T ----
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pf[2];
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) pf[qi] = pack_p(s[qi][2 * ks], s[qi][2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const s16x4 v0 = tr_read(v_img, (2 * ks) * 16 + 4 * g, dt * 16, lane);
        const s16x4 v1 = tr_read(v_img, (2 * ks + 1) * 16 + 4 * g, dt * 16, lane);
        const bf16x8 vf = cat_frag(v0, v1);
#pragma unroll
        for (int qi = 0; qi < 2; ++qi) o[qi][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qi], o[qi][dt], 0, 0, 0);
      }
    }
    if (kt + 1 < nkt) {
      stage_store<false>(rk, sK[cur ^ 1], tid);
      stage_store<true>(rv, sV[cur ^ 1], tid);
    }
    __syncthreads();
  }

  // ---- epilogue: lane holds O[q = qi*16 + c][d = dt*16 + 4g + r] ----
  bf16_t* O = a.o + b * a.so_b + h * ATT_D;
#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    const int qr = q0 + qi * 16 + c;
    if (qr >= a.Sq) continue;
    const float inv = 1.f / l_run[qi];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const f32x4 v = o[qi][dt];
      *reinterpret_cast<uint2*>(O + (long)qr * a.ldo + dt * 16 + 4 * g) =
          make_uint2(pack2bf(v[0] * inv, v[1] * inv), pack2bf(v[2] * inv, v[3] * inv));
    }
    if (a.lse && g == 0) a.lse[((long)b * a.H + h) * a.Sq + qr] = (m_run[qi] + log2f(l_run[qi])) * 0.69314718055994531f;
  }
}

// ================================================================================================================
// backward pre-pass: delta[b][h][q] = sum_d dO * O
// ================================================================================================================
__global__ void attn_delta_kernel(AttnArgs a, int B) {
  const long idx = blockIdx.x * (long)(blockDim.x / 64) + (threadIdx.x >> 6);  // one wave per (b, q), all heads
  const int lane = threadIdx.x & 63;
  if (idx >= (long)B * a.Sq) return;
  const int b = (int)(idx / a.Sq), q = (int)(idx - (long)b * a.Sq);
  const bf16_t* O = a.o + b * a.so_b + (long)q * a.ldo;
  const bf16_t* D = a.dO + b * a.sdo_b + (long)q * a.lddo;
  // each head = 64 d = 8 chunks; lane handles chunk (lane & 7) of heads (lane >> 3) + 8k
  for (int h0 = 0; h0 < a.H; h0 += 8) {
    const int h = h0 + (lane >> 3);
    float s = 0.f;
    if (h < a.H) {
      const int off = h * ATT_D + (lane & 7) * 8;
      const uint4 ov = *reinterpret_cast<const uint4*>(O + off);
      const uint4 dv = *reinterpret_cast<const uint4*>(D + off);
      const uint32_t ow[4] = {ov.x, ov.y, ov.z, ov.w}, dw[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        s += bf2f(ow[j] & 0xffff) * bf2f(dw[j] & 0xffff) + bf2f(ow[j] >> 16) * bf2f(dw[j] >> 16);
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if (h < a.H && (lane & 7) == 0) a.delta[((long)b * a.H + h) * a.Sq + q] = s;
  }
}

// ================================================================================================================
// backward dK/dV: one workgroup = 128 keys of one (b, h) (32 per wave, keys on the MFMA lane axis); loops over the
// query tiles [qa, qb).  Scores S[q][k] = Q.K^T with Q fragments as the A operand -> lane holds S[q=4g+r][k=c].
// ================================================================================================================
__global__ __launch_bounds__(ATT_THREADS, 2) void attn_bwd_dkv_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t sQr[ATT_KT * ATT_D];   // row image of the Q tile
  __shared__ __attribute__((aligned(16))) bf16_t sQt[ATT_KT * ATT_D];   // transposed-read image
  __shared__ __attribute__((aligned(16))) bf16_t sOr[ATT_KT * ATT_D];   // dO row image
  __shared__ __attribute__((aligned(16))) bf16_t sOt[ATT_KT * ATT_D];   // dO transposed-read image
  __shared__ float sL[ATT_KT], sD[ATT_KT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int nkb = (a.Sk + 127) / 128;
  const int kb = blockIdx.x % nkb, split = blockIdx.x / nkb;
  const int b = blockIdx.z, h = blockIdx.y;
  const int k0 = kb * 128 + wave * 32;

  const bf16_t* Q = a.q + b * a.sq_b + h * ATT_D;
  const bf16_t* K = a.k + b * a.sk_b + h * ATT_D;
  const bf16_t* V = a.v + b * a.sv_b + h * ATT_D;
  const bf16_t* DO = a.dO + b * a.sdo_b + h * ATT_D;
  const float* LSE = a.lse + ((long)b * a.H + h) * a.Sq;
  const float* DEL = a.delta + ((long)b * a.H + h) * a.Sq;

  // K and V fragments of this wave's 32 keys (B operands): lane holds K[k0 + kj*16 + c][ds*32 + 8g ..]
  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int kj = 0; kj < 2; ++kj) {
    const int kr = k0 + kj * 16 + c;
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) {
      uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
      if (kr < a.Sk) {
        kv = *reinterpret_cast<const uint4*>(K + (long)kr * a.ldk + ds * 32 + 8 * g);
        vv = *reinterpret_cast<const uint4*>(V + (long)kr * a.ldv + ds * 32 + 8 * g);
      }
      kf[kj][ds] = __builtin_bit_cast(bf16x8, kv);
      vf[kj][ds] = __builtin_bit_cast(bf16x8, vv);
    }
  }
  f32x4 dk[2][4], dv[2][4];  // [kj][dt]: lane holds d?[k = kj*16 + c][d = dt*16 + 4g + r]
#pragma unroll
  for (int kj = 0; kj < 2; ++kj)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dk[kj][dt] = dv[kj][dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nqt = (a.Sq + ATT_KT - 1) / ATT_KT;
  const int per = (nqt + a.q_split - 1) / a.q_split;
  const int qa = split * per, qb = min(nqt, qa + per);
  const float ln2inv = 1.4426950408889634f;

  for (int qt = qa; qt < qb; ++qt) {
    const int qbase = qt * ATT_KT;
    uint4 rq[2], ro[2];
    stage_load(rq, Q, a.ldq, qbase, a.Sq, tid);
    stage_load(ro, DO, a.lddo, qbase, a.Sq, tid);
    __syncthreads();  // previous tile fully consumed
    stage_store<false>(rq, sQr, tid);
    stage_store<true>(rq, sQt, tid);
    stage_store<false>(ro, sOr, tid);
    stage_store<true>(ro, sOt, tid);
    if (tid < ATT_KT) {
      const int q = qbase + tid;
      sL[tid] = q < a.Sq ? LSE[q] * ln2inv : INFINITY;  // base-2 LSE; padded rows give p = 0
      sD[tid] = q < a.Sq ? DEL[q] : 0.f;
    }
    __syncthreads();
    // S and dP for 4 q-subtiles x 2 key subtiles: lane holds X[q = qs*16 + 4g + r][k = kj*16 + c]
    f32x4 p[4][2], ds_[4][2];
#pragma unroll
    for (int qs = 0; qs < 4; ++qs) {
      bf16x8 qa_[2], oa_[2];
#pragma unroll
      for (int d2 = 0; d2 < 2; ++d2) {
        qa_[d2] = *reinterpret_cast<const bf16x8*>(sQr + swz_row(qs * 16 + c, d2 * 4 + g));
        oa_[d2] = *reinterpret_cast<const bf16x8*>(sOr + swz_row(qs * 16 + c, d2 * 4 + g));
      }
      float lq[4], dq_[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        lq[r] = sL[qs * 16 + 4 * g + r];
        dq_[r] = sD[qs * 16 + 4 * g + r];
      }
#pragma unroll
      for (int kj = 0; kj < 2; ++kj) {
        f32x4 sacc = {0.f, 0.f, 0.f, 0.f}, pacc = {0.f, 0.f, 0.f, 0.f};
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa_[0], kf[kj][0], sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa_[1], kf[kj][1], sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa_[0], vf[kj][0], pacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa_[1], vf[kj][1], pacc, 0, 0, 0);
        const bool kvalid = (k0 + kj * 16 + c) < a.Sk;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pr = kvalid ? exp2f(sacc[r] * a.scale_log2 - lq[r]) : 0.f;
          p[qs][kj][r] = pr;
          ds_[qs][kj][r] = pr * (pacc[r] - dq_[r]);
        }
      }
    }
    // dV^T[d][k] += dO^T . P ;  dK^T[d][k] += Q^T . dS   (q permuted within 32-deep steps, lane-local B operands)
#pragma unroll
    for (int qk = 0; qk < 2; ++qk) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 of = cat_frag(tr_read(sOt, (2 * qk) * 16 + 4 * g, dt * 16, lane),
                                   tr_read(sOt, (2 * qk + 1) * 16 + 4 * g, dt * 16, lane));
        const bf16x8 qf = cat_frag(tr_read(sQt, (2 * qk) * 16 + 4 * g, dt * 16, lane),
                                   tr_read(sQt, (2 * qk + 1) * 16 + 4 * g, dt * 16, lane));
#pragma unroll
        for (int kj = 0; kj < 2; ++kj) {
          dv[kj][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(of, pack_p(p[2 * qk][kj], p[2 * qk + 1][kj]),
                                                              dv[kj][dt], 0, 0, 0);
          dk[kj][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf, pack_p(ds_[2 * qk][kj], ds_[2 * qk + 1][kj]),
                                                              dk[kj][dt], 0, 0, 0);
        }
      }
    }
  }
  // ---- epilogue: lane holds d?[k = k0 + kj*16 + c][d = dt*16 + 4g + r]; dK carries the softmax scale ----
  const float sc = a.scale_log2 * 0.69314718055994531f;
#pragma unroll
  for (int kj = 0; kj < 2; ++kj) {
    const int kr = k0 + kj * 16 + c;
    if (kr >= a.Sk) continue;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int d = h * ATT_D + dt * 16 + 4 * g;
      if (a.q_split > 1) {
        float* pk = a.dk_acc + ((long)b * a.Sk + kr) * (a.H * ATT_D) + d;
        float* pv = a.dv_acc + ((long)b * a.Sk + kr) * (a.H * ATT_D) + d;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          atomicAdd(pk + r, dk[kj][dt][r] * sc);
          atomicAdd(pv + r, dv[kj][dt][r]);
        }
      } else {
        *reinterpret_cast<uint2*>(a.dk + b * a.sdk_b + (long)kr * a.lddk + d) =
            make_uint2(pack2bf(dk[kj][dt][0] * sc, dk[kj][dt][1] * sc), pack2bf(dk[kj][dt][2] * sc, dk[kj][dt][3] * sc));
        *reinterpret_cast<uint2*>(a.dv + b * a.sdv_b + (long)kr * a.lddv + d) =
            make_uint2(pack2bf(dv[kj][dt][0], dv[kj][dt][1]), pack2bf(dv[kj][dt][2], dv[kj][dt][3]));
      }
    }
  }
}

// ================================================================================================================
// backward dQ: forward structure (128 queries per workgroup, S^T = K.Q^T lane-local per query), K/V tiles through LDS
//   dP^T = V . dO^T ; dS^T = P^T * (dP^T - delta) ; dQ^T[d][q] += K^T . dS^T  (K^T via transposed reads)
// ================================================================================================================
__global__ __launch_bounds__(ATT_THREADS, 2) void attn_bwd_dq_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t sKr[ATT_KT * ATT_D];
  __shared__ __attribute__((aligned(16))) bf16_t sKt[ATT_KT * ATT_D];
  __shared__ __attribute__((aligned(16))) bf16_t sVr[ATT_KT * ATT_D];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int b = blockIdx.z, h = blockIdx.y;
  const int q0 = blockIdx.x * 128 + wave * 32;
  const bf16_t* Q = a.q + b * a.sq_b + h * ATT_D;
  const bf16_t* K = a.k + b * a.sk_b + h * ATT_D;
  const bf16_t* V = a.v + b * a.sv_b + h * ATT_D;
  const bf16_t* DO = a.dO + b * a.sdo_b + h * ATT_D;
  const float ln2inv = 1.4426950408889634f;

  bf16x8 qf[2][2], of[2][2];
  float lq[2], dl[2];
#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    const int qr = q0 + qi * 16 + c;
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) {
      uint4 v = make_uint4(0, 0, 0, 0), w = make_uint4(0, 0, 0, 0);
      if (qr < a.Sq) {
        v = *reinterpret_cast<const uint4*>(Q + (long)qr * a.ldq + ds * 32 + 8 * g);
        w = *reinterpret_cast<const uint4*>(DO + (long)qr * a.lddo + ds * 32 + 8 * g);
      }
      qf[qi][ds] = __builtin_bit_cast(bf16x8, v);
      of[qi][ds] = __builtin_bit_cast(bf16x8, w);
    }
    lq[qi] = qr < a.Sq ? a.lse[((long)b * a.H + h) * a.Sq + qr] * ln2inv : INFINITY;
    dl[qi] = qr < a.Sq ? a.delta[((long)b * a.H + h) * a.Sq + qr] : 0.f;
  }
  f32x4 dq[2][4];
#pragma unroll
  for (int qi = 0; qi < 2; ++qi)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[qi][dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (a.Sk + ATT_KT - 1) / ATT_KT;
  for (int kt = 0; kt < nkt; ++kt) {
    const int kbase = kt * ATT_KT;
    uint4 rk[2], rv[2];
    stage_load(rk, K, a.ldk, kbase, a.Sk, tid);
    stage_load(rv, V, a.ldv, kbase, a.Sk, tid);
    __syncthreads();
    stage_store<false>(rk, sKr, tid);
    stage_store<true>(rk, sKt, tid);
    stage_store<false>(rv, sVr, tid);
    __syncthreads();
    f32x4 dsT[2][4];  // lane holds dS[q = qi*16 + c][key = kj*16 + 4g + r]
#pragma unroll
    for (int kj = 0; kj < 4; ++kj) {
      bf16x8 kf[2], vf[2];
#pragma unroll
      for (int ds = 0; ds < 2; ++ds) {
        kf[ds] = *reinterpret_cast<const bf16x8*>(sKr + swz_row(kj * 16 + c, ds * 4 + g));
        vf[ds] = *reinterpret_cast<const bf16x8*>(sVr + swz_row(kj * 16 + c, ds * 4 + g));
      }
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) {
        f32x4 sacc = {0.f, 0.f, 0.f, 0.f}, pacc = {0.f, 0.f, 0.f, 0.f};
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[0], qf[qi][0], sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[1], qf[qi][1], sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[0], of[qi][0], pacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[1], of[qi][1], pacc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kbase + kj * 16 + 4 * g + r;
          const float p = key < a.Sk ? exp2f(sacc[r] * a.scale_log2 - lq[qi]) : 0.f;
          dsT[qi][kj][r] = p * (pacc[r] - dl[qi]);
        }
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pf[2];
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) pf[qi] = pack_p(dsT[qi][2 * ks], dsT[qi][2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 kf = cat_frag(tr_read(sKt, (2 * ks) * 16 + 4 * g, dt * 16, lane),
                                   tr_read(sKt, (2 * ks + 1) * 16 + 4 * g, dt * 16, lane));
#pragma unroll
        for (int qi = 0; qi < 2; ++qi) dq[qi][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, pf[qi], dq[qi][dt], 0, 0, 0);
      }
    }
  }
  const float sc = a.scale_log2 * 0.69314718055994531f;
  bf16_t* DQ = a.dq + b * a.sdq_b + h * ATT_D;
#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    const int qr = q0 + qi * 16 + c;
    if (qr >= a.Sq) continue;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const f32x4 v = dq[qi][dt];
      *reinterpret_cast<uint2*>(DQ + (long)qr * a.lddq + dt * 16 + 4 * g) =
          make_uint2(pack2bf(v[0] * sc, v[1] * sc), pack2bf(v[2] * sc, v[3] * sc));
    }
  }
}

__global__ void f32_to_bf16_strided_kernel(long rows, int cols, const float* __restrict__ src, bf16_t* __restrict__ dst,
                                           long ldd) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < rows * cols; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cols;
    const int cc = (int)(i - r * cols);
    dst[r * ldd + cc] = f2bf(src[i]);
  }
}

static bool a16(const void* p, long ld) { return (((uintptr_t)p) & 15) == 0 && (ld % 8) == 0; }

extern "C" {

int pso_attention_fwd(int B, int H, int Sq, int Sk, const void* q, long ldq, long sq_b, const void* k, long ldk,
                      long sk_b, const void* v, long ldv, long sv_b, float scale, void* o, long ldo, long so_b,
                      float* lse, void* stream) {
  PSO_ARG_CHECK(B > 0 && H > 0 && Sq > 0 && Sk > 0, "pso_attention_fwd: bad shape");
  PSO_ARG_CHECK(q && k && v && o, "pso_attention_fwd: null");
  PSO_ARG_CHECK(a16(q, ldq) && a16(k, ldk) && a16(v, ldv) && (((uintptr_t)o) & 7) == 0 && (ldo % 4) == 0,
                "pso_attention_fwd: operands need 16-B aligned rows");
  AttnArgs a{};
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v;
  a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.sq_b = sq_b; a.sk_b = sk_b; a.sv_b = sv_b;
  a.o = (bf16_t*)o; a.ldo = ldo; a.so_b = so_b; a.lse = lse;
  a.Sq = Sq; a.Sk = Sk; a.H = H; a.scale_log2 = scale * 1.4426950408889634f;
  dim3 grid(cdiv(Sq, 128), H, B);
  attn_fwd_kernel<<<grid, ATT_THREADS, 0, (hipStream_t)stream>>>(a);
  return pso_check_launch("pso_attention_fwd");
}

size_t pso_attention_bwd_ws_bytes(int B, int H, int Sq, int Sk) {
  size_t d = (size_t)B * H * Sq * sizeof(float);
  size_t acc = (Sk <= 256) ? 2 * (size_t)B * Sk * H * ATT_D * sizeof(float) : 0;
  return ((d + 255) / 256) * 256 + acc;
}

int pso_attention_bwd(int B, int H, int Sq, int Sk, const void* q, long ldq, long sq_b, const void* k, long ldk,
                      long sk_b, const void* v, long ldv, long sv_b, const void* o, long ldo, long so_b,
                      const float* lse, const void* dO, long lddo, long sdo_b, float scale, void* dq, long lddq,
                      long sdq_b, void* dk, long lddk, long sdk_b, void* dv, long lddv, long sdv_b, void* ws,
                      size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(B > 0 && H > 0 && Sq > 0 && Sk > 0, "pso_attention_bwd: bad shape");
  PSO_ARG_CHECK(q && k && v && o && lse && dO && dq && dk && dv && ws, "pso_attention_bwd: null");
  PSO_ARG_CHECK(ws_bytes >= pso_attention_bwd_ws_bytes(B, H, Sq, Sk), "pso_attention_bwd: workspace too small");
  PSO_ARG_CHECK(a16(q, ldq) && a16(k, ldk) && a16(v, ldv) && a16(o, ldo) && a16(dO, lddo),
                "pso_attention_bwd: operands need 16-B aligned rows");
  hipStream_t st = (hipStream_t)stream;
  AttnArgs a{};
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v;
  a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.sq_b = sq_b; a.sk_b = sk_b; a.sv_b = sv_b;
  a.o = (bf16_t*)o; a.ldo = ldo; a.so_b = so_b; a.lse = (float*)lse;
  a.Sq = Sq; a.Sk = Sk; a.H = H; a.scale_log2 = scale * 1.4426950408889634f;
  a.dO = (const bf16_t*)dO; a.lddo = lddo; a.sdo_b = sdo_b;
  float* delta = (float*)ws;
  a.delta = delta;
  a.dq = (bf16_t*)dq; a.dk = (bf16_t*)dk; a.dv = (bf16_t*)dv;
  a.lddq = lddq; a.lddk = lddk; a.lddv = lddv; a.sdq_b = sdq_b; a.sdk_b = sdk_b; a.sdv_b = sdv_b;
  const size_t doff = (((size_t)B * H * Sq * sizeof(float) + 255) / 256) * 256;
  const int nkb = cdiv(Sk, 128);
  int qsplit = 1;
  if (Sk <= 256) {  // few key blocks (cross-attention over 77 text tokens): split the query sweep, fp32 atomics
    const int nqt = cdiv(Sq, ATT_KT);
    qsplit = nqt < 16 ? nqt : 16;
    a.dk_acc = (float*)((char*)ws + doff);
    a.dv_acc = a.dk_acc + (size_t)B * Sk * H * ATT_D;
    hipMemsetAsync(a.dk_acc, 0, 2 * (size_t)B * Sk * H * ATT_D * sizeof(float), st);
  }
  a.q_split = qsplit;
  attn_delta_kernel<<<cdiv((long)B * Sq, 4), 256, 0, st>>>(a, B);
  attn_bwd_dkv_kernel<<<dim3(nkb * qsplit, H, B), ATT_THREADS, 0, st>>>(a);
  attn_bwd_dq_kernel<<<dim3(cdiv(Sq, 128), H, B), ATT_THREADS, 0, st>>>(a);
  if (qsplit > 1) {
    const long rows = (long)B * Sk;
    const int cols = H * ATT_D;
    // dk/dv outputs are [B][Sk] rows of H*64 with row stride lddk (batch stride must be Sk*lddk)
    f32_to_bf16_strided_kernel<<<cdiv(rows * cols, 256) > 4096 ? 4096 : cdiv(rows * cols, 256), 256, 0, st>>>(
        rows, cols, a.dk_acc, (bf16_t*)dk, lddk);
    f32_to_bf16_strided_kernel<<<cdiv(rows * cols, 256) > 4096 ? 4096 : cdiv(rows * cols, 256), 256, 0, st>>>(
        rows, cols, a.dv_acc, (bf16_t*)dv, lddv);
  }
  return pso_check_launch("pso_attention_bwd");
}

}  // extern "C"
