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

#include <type_traits>

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

// The same read as inline asm, for kernels whose LDS ring is filled by LDS-DMA: hipcc cannot tell the builtin's LDS
// read from the pending DMA writes and drains the ring (vmcnt(0)) before it.  The caller waits lgkmcnt itself.
__device__ __forceinline__ s16x4 tr_read_asm(const bf16_t* img, int r0, int col0, int lane) {
  const int li = lane & 15;
  const int q = li >> 2, p = li & 3;
  const int col = col0 + 4 * p;
  const unsigned addr = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)(img + swz_tr(r0 + q, col >> 3) + (col & 7));
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
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
  float* delta;                // [B][H][Sq]: -rowsum(dO * O), written by the dQ kernel for the dK/dV kernel
  float* lse2;                 // [B][H][Sq]: the LSE in log2 units, likewise (no per-tile rescale / negation there)
  bf16_t *dq, *dk, *dv; long lddq, lddk, lddv; long sdq_b, sdk_b, sdv_b;
  float *dk_acc, *dv_acc;      // fp32 [B][Sk][H*64] when q is split (cross-attention)
  int q_split;
  int nbatch;                  // B (split-slice stride)
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
// Cross-lane max over the 4 lanes {c, c+16, c+32, c+48} that hold one query row (v_permlane16/32_swap: VALU, no LDS).
__device__ __forceinline__ float rowmax4(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float rowsum4(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

typedef __attribute__((address_space(3))) void att_lds_void;

// XCD-aware flat block order: the hardware deals blocks round-robin over the 8 XCDs; give each XCD a contiguous run of
// logical blocks so the query blocks of one (batch, head) share one L2 copy of its K/V.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  if (nblk < 8) return bid;
  const int q = nblk / 8, r = nblk % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// One workgroup = 4 waves x (16*QI) query rows of one (batch, head).  K/V tiles of 64 keys go global -> LDS directly
// (global_load_lds_dwordx4, 2 K + 2 V pieces of 8 rows x 128 B per wave per tile) through a 3-stage ring, two tiles in
// flight behind a counted vmcnt and ONE s_barrier per tile.  The LDS swizzles are applied on the source side (lane i of
// a piece lands at byte 16*i): K row-image chunk p ^ (row & 7), V transposed-read chunk p ^ 2*((row >> 1) & 3).
// Softmax: raw-score running max (exp2(s*c - m*c) = one FMA + one exp per score), row sums accumulated by one extra
// MFMA per PV step against an all-ones operand (no per-score VALU add, no cross-lane reduction), the O/l rescale
// skipped when no row max moved (wave-uniform), key masking on the last tile only.
template <int QI, bool MSUM = true>
__global__ __launch_bounds__(ATT_THREADS, 2) void attn_fwd_kernel(AttnArgs a, int nqb) {
  constexpr int STG = 3;
  constexpr int PIECES = 4;  // glds per wave per tile
  __shared__ __attribute__((aligned(16))) bf16_t sKV[STG][2][ATT_KT * ATT_D];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = bid % nqb, bh = bid / nqb;
  const int h = bh % a.H, b = bh / a.H;
  const int q0 = qb * (64 * QI) + wave * (16 * QI);

  const bf16_t* Q = a.q + b * a.sq_b + h * ATT_D;
  const bf16_t* K = a.k + b * a.sk_b + h * ATT_D;
  const bf16_t* V = a.v + b * a.sv_b + h * ATT_D;
  const float c2 = a.scale_log2;

  // this lane's staging source rows/chunks: piece pw (0/1) of wave w covers tile rows (2w + pw)*8 .. +8
  const int prow = lane >> 3, pch = lane & 7;
  const int lcK = pch ^ prow;
  const int lcV = pch ^ (2 * ((prow >> 1) & 3));
  const int nkt = (a.Sk + ATT_KT - 1) / ATT_KT;
  auto issue = [&](int kt, int buf) {
#pragma unroll
    for (int pw = 0; pw < 2; ++pw) {
      const int piece = wave * 2 + pw;
      const int key = min(kt * ATT_KT + piece * 8 + prow, a.Sk - 1);  // clamped rows are masked (p = 0)
      __builtin_amdgcn_global_load_lds(static_cast<const void*>(K + (long)key * a.ldk + lcK * 8),
                                       (att_lds_void*)(sKV[buf][0] + piece * 8 * ATT_D), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(static_cast<const void*>(V + (long)key * a.ldv + lcV * 8),
                                       (att_lds_void*)(sKV[buf][1] + piece * 8 * ATT_D), 16, 0, 0);
    }
  };

  // Q fragments (B operand of S^T = K.Q^T): lane holds Q[q0 + qi*16 + c][ds*32 + 8g .. +8]
  bf16x8 qf[QI][2];
#pragma unroll
  for (int qi = 0; qi < QI; ++qi) {
    const int qr = min(q0 + qi * 16 + c, a.Sq - 1);
#pragma unroll
    for (int ds = 0; ds < 2; ++ds)
      qf[qi][ds] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(Q + (long)qr * a.ldq + ds * 32 + 8 * g));
  }
  issue(0, 0);
  if (nkt > 1) issue(1, 1);

  f32x4 o[QI][4];
  // row sums on the matrix cores: lsum[qi] += 1^T . P^T (an all-ones A operand), so every lane gets the full row sum
  // of its query without a VALU add per score or a cross-lane reduction; it sums the bf16 P the PV product uses
  f32x4 lsum[QI];
  float m_run[QI];
  const bf16x8 ones = __builtin_bit_cast(bf16x8, make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u));
#pragma unroll
  for (int qi = 0; qi < QI; ++qi) {
    m_run[qi] = -INFINITY;
    lsum[qi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qi][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  for (int kt = 0; kt < nkt; ++kt) {
    // tile kt landed (this wave's pieces: all but the PIECES youngest), then every wave's (barrier); the barrier also
    // orders every wave's reads of tile kt-1 before the re-staging of its buffer below
    if (kt + 1 < nkt) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(PIECES) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + 2 < nkt) issue(kt + 2, (kt + 2) % STG);
    const bf16_t* k_img = sKV[kt % STG][0];
    const bf16_t* v_img = sKV[kt % STG][1];
    // ---- S^T tiles: s[qi][kj] holds S[q = qi*16 + c][key = kj*16 + 4g + r] (raw scores) ----
    f32x4 s[QI][4];
#pragma unroll
    for (int kj = 0; kj < 4; ++kj) {
      bf16x8 kf[2];
#pragma unroll
      for (int ds = 0; ds < 2; ++ds)
        kf[ds] = *reinterpret_cast<const bf16x8*>(k_img + swz_row(kj * 16 + c, ds * 4 + g));
#pragma unroll
      for (int qi = 0; qi < QI; ++qi) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[0], qf[qi][0], acc, 0, 0, 0);
        s[qi][kj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[1], qf[qi][1], acc, 0, 0, 0);
      }
    }
    const int kbase = kt * ATT_KT;
    if (kbase + ATT_KT > a.Sk) {  // partial last tile (wave-uniform)
#pragma unroll
      for (int qi = 0; qi < QI; ++qi)
#pragma unroll
        for (int kj = 0; kj < 4; ++kj)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kbase + kj * 16 + 4 * g + r >= a.Sk) s[qi][kj][r] = -INFINITY;
    }
    // ---- online softmax (base 2, raw-score max) ----
#pragma unroll
    for (int qi = 0; qi < QI; ++qi) {
      float mx = fmaxf(fmaxf(s[qi][0][0], s[qi][0][1]), fmaxf(s[qi][0][2], s[qi][0][3]));
#pragma unroll
      for (int kj = 1; kj < 4; ++kj)
        mx = fmaxf(mx, fmaxf(fmaxf(s[qi][kj][0], s[qi][kj][1]), fmaxf(s[qi][kj][2], s[qi][kj][3])));
      mx = rowmax4(mx);
      const float m_new = fmaxf(m_run[qi], mx);
      if (__any(m_new > m_run[qi])) {
        const float alpha = fast_exp2((m_run[qi] - m_new) * c2);  // first tile: exp2(-inf) = 0
        lsum[qi] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qi][dt] *= alpha;
        m_run[qi] = m_new;
      }
      const float mc = m_run[qi] * c2;
      float sum = 0.f;
#pragma unroll
      for (int kj = 0; kj < 4; ++kj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[qi][kj][r] = fast_exp2(fmaf(s[qi][kj][r], c2, -mc));
          if (!MSUM) sum += s[qi][kj][r];
        }
      if (!MSUM) lsum[qi][0] += sum;  // VALU form (A/B knob): this lane's keys; the 4 lanes summed at the end
    }
    // ---- O^T += V^T . P^T ----
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pf[QI];
#pragma unroll
      for (int qi = 0; qi < QI; ++qi) {
        pf[qi] = pack_p(s[qi][2 * ks], s[qi][2 * ks + 1]);
        if (MSUM) lsum[qi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[qi], lsum[qi], 0, 0, 0);
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const s16x4 v0 = tr_read(v_img, (2 * ks) * 16 + 4 * g, dt * 16, lane);
        const s16x4 v1 = tr_read(v_img, (2 * ks + 1) * 16 + 4 * g, dt * 16, lane);
        const bf16x8 vf = cat_frag(v0, v1);
#pragma unroll
        for (int qi = 0; qi < QI; ++qi) o[qi][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qi], o[qi][dt], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: lane holds O[q = qi*16 + c][d = dt*16 + 4g + r] ----
  bf16_t* O = a.o + b * a.so_b + h * ATT_D;
#pragma unroll
  for (int qi = 0; qi < QI; ++qi) {
    const float l = MSUM ? lsum[qi][0] : rowsum4(lsum[qi][0]);  // MSUM: every element holds the query's row sum
    const int qr = q0 + qi * 16 + c;
    if (qr >= a.Sq) continue;
    const float inv = 1.f / l;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const f32x4 v = o[qi][dt];
      *reinterpret_cast<uint2*>(O + (long)qr * a.ldo + dt * 16 + 4 * g) =
          make_uint2(pack2bf(v[0] * inv, v[1] * inv), pack2bf(v[2] * inv, v[3] * inv));
    }
    if (a.lse && g == 0)
      a.lse[((long)b * a.H + h) * a.Sq + qr] = (m_run[qi] * c2 + log2f(l)) * 0.69314718055994531f;
  }
}

// ================================================================================================================
// forward v2: the same tiling with the per-tile vector work cut to what the math needs (the loop above issues ~390
// non-MFMA vector instructions per wave and tile, measured SQ_INSTS_VALU; the vector issue, not the matrix pipe, bounds
// it at two waves per SIMD):
//  * the tile loop is unrolled by the ring depth, so every LDS address is a lane base + an immediate (no per-tile
//    ring-slot arithmetic);
//  * row maxima by v_max3_f32 in inline asm (fmaxf on MFMA results makes hipcc canonicalise each operand first:
//    3 instructions per 2 scores instead of 1);
//  * deferred rescale: the running max moves only when some row of the wave grew by more than RESCALE_LOG2 (in
//    log2 units), so P <= 2^RESCALE_LOG2 (exact in fp32, rounded to bf16 like every P) and the O / l rescale (and its
//    branch) is skipped on almost every tile after the first few; one wave-uniform decision covers all QI row groups.
// Output and LSE are the same function of the inputs: l and O carry the same scale, and LSE = m*c + log2(l).
// ================================================================================================================
#define ATT_RESCALE_LOG2 8.0f

__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float vmax2(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float rowmax4_asm(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = vmax2(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return vmax2(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

template <int V> struct ic { static constexpr int value = V; };

// s_waitcnt + s_barrier that leaves the n (<= 3) youngest ring tiles of P LDS-DMA pieces each in flight (n is
// wave-uniform: the branch is scalar; vmcnt needs an immediate)
template <int P>
__device__ __forceinline__ void att_wait_barrier(int n) {
  static_assert(3 * P <= 63, "vmcnt field");
  if (n >= 3) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(3 * P) : "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(2 * P) : "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(P) : "memory");
  else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// 8 transposed V reads (inline asm, see tr_read_asm) and the wait that makes their registers available: the wait takes
// the fragments as in/out operands, so no consumer can be scheduled above it
__device__ __forceinline__ void lds_wait8(s16x4 (&v)[8]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]));
}

// transposed read at a lane base + a compile-time byte offset (ring slot and row block fold into the immediate, so a
// handful of base registers serve every read of the loop)
template <int OFF>
__device__ __forceinline__ s16x4 tr_read_imm(unsigned base) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset range");
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(base), "n"(OFF));
  return v;
}

// LG (lane-local growth test, the round-2 variant ea590ae): the rescale test runs on each lane's own 16 scores (m_run
// is the same on a row's 4 lanes, so "some lane grew" == "the row grew") and the cross-lane row max is formed only
// inside the (rare) rescale branch.  Same decisions, same arithmetic: outputs bit-identical to LG = false.
template <int QI, bool LG = false>
__global__ __launch_bounds__(ATT_THREADS, 2) void attn_fwd2_kernel(AttnArgs a, int nqb) {
  constexpr int STG = 3;
  constexpr int PIECES = 4;
  __shared__ __attribute__((aligned(16))) bf16_t sKV[STG][2][ATT_KT * ATT_D];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: LDS-DMA destinations (M0) are scalar
  const int g = lane >> 4, c = lane & 15;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = bid % nqb, bh = bid / nqb;
  const int h = bh % a.H, b = bh / a.H;
  const int q0 = qb * (64 * QI) + wave * (16 * QI);

  const bf16_t* Q = a.q + b * a.sq_b + h * ATT_D;
  const bf16_t* K = a.k + b * a.sk_b + h * ATT_D;
  const bf16_t* V = a.v + b * a.sv_b + h * ATT_D;
  const float c2 = a.scale_log2;
  const float thr = ATT_RESCALE_LOG2 / c2;  // raw-score growth that triggers a rescale

  // K/V staging by buffer_load ... lds against per-(batch, head) SGPR resources whose range ends at key row Sk - 1:
  // rows past the end read as zeros (masked on the last tile), so the per-lane part of every staging address is one
  // loop-invariant 32-bit offset and the tile advance is the scalar soffset
  const int prow = lane >> 3, pch = lane & 7;
  const int lcK = pch ^ prow;
  const int lcV = pch ^ (2 * ((prow >> 1) & 3));
  const int nkt = (a.Sk + ATT_KT - 1) / ATT_KT;
  const __amdgpu_buffer_rsrc_t rK =
      __builtin_amdgcn_make_buffer_rsrc((void*)K, (short)0, (int)(((long)(a.Sk - 1) * a.ldk + ATT_D) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rV =
      __builtin_amdgcn_make_buffer_rsrc((void*)V, (short)0, (int)(((long)(a.Sk - 1) * a.ldv + ATT_D) * 2), 0x00020000);
  unsigned kvo[2], vvo[2];
#pragma unroll
  for (int pw = 0; pw < 2; ++pw) {
    const int row = (wave * 2 + pw) * 8 + prow;
    kvo[pw] = (unsigned)(row * (int)a.ldk + lcK * 8) * 2u;
    vvo[pw] = (unsigned)(row * (int)a.ldv + lcV * 8) * 2u;
  }
  const int kstep = ATT_KT * (int)a.ldk * 2, vstep = ATT_KT * (int)a.ldv * 2;  // bytes per key tile
  // lane bases of the transposed V reads, one per 16-column block dt (rows 4g.. of slot 0's V image; the ring slot and
  // the 16-row block are immediates)
  unsigned vbase[4];
  {
    const unsigned lds0 = (unsigned)(uintptr_t)(const att_lds_void*)&sKV[0][0][0];
    const int li = lane & 15, q = li >> 2, p = li & 3;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = dt * 16 + 4 * p;
      vbase[dt] = lds0 + 2u * (unsigned)(swz_tr(4 * g + q, col >> 3) + (col & 7));
    }
  }
  auto issue = [&](int kt, int buf) {
#pragma unroll
    for (int pw = 0; pw < 2; ++pw) {
      const int piece = wave * 2 + pw;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rK, (att_lds_void*)(sKV[buf][0] + piece * 8 * ATT_D), 16, kvo[pw],
                                               kt * kstep, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rV, (att_lds_void*)(sKV[buf][1] + piece * 8 * ATT_D), 16, vvo[pw],
                                               kt * vstep, 0, 0);
    }
  };

  bf16x8 qf[QI][2];
#pragma unroll
  for (int qi = 0; qi < QI; ++qi) {
    const int qr = min(q0 + qi * 16 + c, a.Sq - 1);
#pragma unroll
    for (int ds = 0; ds < 2; ++ds)
      qf[qi][ds] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(Q + (long)qr * a.ldq + ds * 32 + 8 * g));
  }
  issue(0, 0);
  if (nkt > 1) issue(1, 1);

  f32x4 o[QI][4];
  f32x4 lsum[QI];
  float m_run[QI];
  const bf16x8 ones = __builtin_bit_cast(bf16x8, make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u));
#pragma unroll
  for (int qi = 0; qi < QI; ++qi) {
    m_run[qi] = -INFINITY;
    lsum[qi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qi][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  auto tile = [&](auto bufc, int kt) {
    constexpr int buf = decltype(bufc)::value;
    if (kt + 1 < nkt) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(PIECES) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + 2 < nkt) issue(kt + 2, (buf + 2) % STG);
    const bf16_t* k_img = sKV[buf][0];
    f32x4 s[QI][4];
#pragma unroll
    for (int kj = 0; kj < 4; ++kj) {
      bf16x8 kf[2];
#pragma unroll
      for (int ds = 0; ds < 2; ++ds)
        kf[ds] = *reinterpret_cast<const bf16x8*>(k_img + swz_row(kj * 16 + c, ds * 4 + g));
#pragma unroll
      for (int qi = 0; qi < QI; ++qi) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[0], qf[qi][0], acc, 0, 0, 0);
        s[qi][kj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[1], qf[qi][1], acc, 0, 0, 0);
      }
    }
    // V fragments of the first 32 keys: in flight during the softmax
    constexpr int VOFF = (buf * 2 + 1) * ATT_KT * ATT_D * 2;  // byte offset of this slot's V image
    s16x4 vr0[8];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      vr0[2 * dt] = tr_read_imm<VOFF + 0 * 2048>(vbase[dt]);
      vr0[2 * dt + 1] = tr_read_imm<VOFF + 1 * 2048>(vbase[dt]);
    }
    const int kbase = kt * ATT_KT;
    if (kbase + ATT_KT > a.Sk) {
#pragma unroll
      for (int qi = 0; qi < QI; ++qi)
#pragma unroll
        for (int kj = 0; kj < 4; ++kj)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kbase + kj * 16 + 4 * g + r >= a.Sk) s[qi][kj][r] = -INFINITY;
    }
    float mx[QI];
    bool grow = false;
#pragma unroll
    for (int qi = 0; qi < QI; ++qi) {
      float m = vmax3(s[qi][0][0], s[qi][0][1], s[qi][0][2]);
      m = vmax3(m, s[qi][0][3], s[qi][1][0]);
      m = vmax3(m, s[qi][1][1], s[qi][1][2]);
      m = vmax3(m, s[qi][1][3], s[qi][2][0]);
      m = vmax3(m, s[qi][2][1], s[qi][2][2]);
      m = vmax3(m, s[qi][2][3], s[qi][3][0]);
      m = vmax3(m, s[qi][3][1], s[qi][3][2]);
      m = vmax2(m, s[qi][3][3]);
      mx[qi] = LG ? m : rowmax4_asm(m);
      grow |= mx[qi] > m_run[qi] + thr;
    }
    if (__any(grow)) {  // wave-uniform; every tile while m_run = -inf, rarely afterwards
#pragma unroll
      for (int qi = 0; qi < QI; ++qi) {
        const float m_new = fmaxf(m_run[qi], LG ? rowmax4_asm(mx[qi]) : mx[qi]);
        const float alpha = fast_exp2((m_run[qi] - m_new) * c2);  // first tile: exp2(-inf) = 0
        lsum[qi] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qi][dt] *= alpha;
        m_run[qi] = m_new;
      }
    }
#pragma unroll
    for (int qi = 0; qi < QI; ++qi) {
      const float mc = m_run[qi] * c2;
#pragma unroll
      for (int kj = 0; kj < 4; ++kj)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[qi][kj][r] = fast_exp2(fmaf(s[qi][kj][r], c2, -mc));
    }
    lds_wait8(vr0);
    s16x4 vr1[8];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      vr1[2 * dt] = tr_read_imm<VOFF + 2 * 2048>(vbase[dt]);
      vr1[2 * dt + 1] = tr_read_imm<VOFF + 3 * 2048>(vbase[dt]);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks == 1) lds_wait8(vr1);
      bf16x8 pf[QI];
#pragma unroll
      for (int qi = 0; qi < QI; ++qi) {
        pf[qi] = pack_p(s[qi][2 * ks], s[qi][2 * ks + 1]);
        lsum[qi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[qi], lsum[qi], 0, 0, 0);
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 vf = ks == 0 ? cat_frag(vr0[2 * dt], vr0[2 * dt + 1]) : cat_frag(vr1[2 * dt], vr1[2 * dt + 1]);
#pragma unroll
        for (int qi = 0; qi < QI; ++qi) o[qi][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qi], o[qi][dt], 0, 0, 0);
      }
    }
  };
  for (int kt = 0; kt < nkt; kt += STG) {
    tile(ic<0>{}, kt);
    if (kt + 1 < nkt) tile(ic<1>{}, kt + 1);
    if (kt + 2 < nkt) tile(ic<2>{}, kt + 2);
  }

  bf16_t* O = a.o + b * a.so_b + h * ATT_D;
#pragma unroll
  for (int qi = 0; qi < QI; ++qi) {
    const float l = lsum[qi][0];
    const int qr = q0 + qi * 16 + c;
    if (qr >= a.Sq) continue;
    const float inv = 1.f / l;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const f32x4 v = o[qi][dt];
      *reinterpret_cast<uint2*>(O + (long)qr * a.ldo + dt * 16 + 4 * g) =
          make_uint2(pack2bf(v[0] * inv, v[1] * inv), pack2bf(v[2] * inv, v[3] * inv));
    }
    if (a.lse && g == 0)
      a.lse[((long)b * a.H + h) * a.Sq + qr] = (m_run[qi] * c2 + log2f(l)) * 0.69314718055994531f;
  }
}

// ================================================================================================================
// backward dK/dV: one workgroup = 4 waves x (16*KJ) keys of one (b, h) (keys on the MFMA lane axis); query tiles of
// 64 stream through a STG-stage LDS ring filled directly from global memory: per tile the Q row image, the Q
// transposed-read image, the dO row image, the dO transposed-read image (8 pieces of 8 rows x 128 B each, 8 per wave)
// and the 64 LSE / delta values (one 256-B dword piece each, waves 0 / 1).  Scores S[q][k] = Q.K^T with Q fragments
// as the A operand -> lane holds S[q = 4g + r][k = c]; P and dS then feed dV^T += dO^T P and dK^T += Q^T dS as
// lane-local B operands (query order permuted inside each 32-deep step, matching the transposed dO / Q reads).
// ================================================================================================================
// PF: the tile's 64 LSE / -delta values are read into registers once, right after the tile's barrier (8 ds_read_b128
// behind one lgkmcnt wait), instead of one read + wait + scheduling barrier per 16-query subtile -- so nothing pins the
// S / dP MFMAs of one subtile behind the exp / dS vector work of the previous one
// ONE: one LDS image per operand (Q, dO) in the transposed-read layout (swz_tr), which the row fragment reads
// (ds_read_b128, 16 rows x 16 B per lane group) also hit conflict-free: half the LDS bytes and DMA traffic per tile,
// so a deeper ring fits at two workgroups per CU
template <int KJ, int STG, bool PF = false, bool ONE = false>
__global__ __launch_bounds__(ATT_THREADS, KJ == 2 ? 2 : 1) void attn_bwd_dkv_kernel(AttnArgs a, int nkb) {
  constexpr int IMG = ATT_KT * ATT_D;  // elements of one 64 x 64 image
  constexpr int NIMG = ONE ? 2 : 4;    // images per ring stage
  constexpr int PIECES = 2 * NIMG;     // 16-B glds per wave per tile (+1 dword piece on waves 0 and 1)
  extern __shared__ __attribute__((aligned(16))) bf16_t att_dyn[];
  bf16_t* const sbase = att_dyn;  // [STG][NIMG][IMG]: Qr, Qt, Or, Ot (ONE: Qt, Ot)
  float* const sLD = reinterpret_cast<float*>(att_dyn + STG * NIMG * IMG);  // [STG][2][64]: LSE, delta
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: LDS-DMA destinations (M0) and the LSE / delta resource are scalar
  const int g = lane >> 4, c = lane & 15;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int per_bh = nkb * a.q_split;
  const int bh = bid / per_bh, rem = bid - bh * per_bh;
  const int split = rem / nkb, kb = rem - split * nkb;
  const int h = bh % a.H, b = bh / a.H;
  const int k0 = kb * (64 * KJ) + wave * (16 * KJ);

  const bf16_t* Q = a.q + b * a.sq_b + h * ATT_D;
  const bf16_t* K = a.k + b * a.sk_b + h * ATT_D;
  const bf16_t* V = a.v + b * a.sv_b + h * ATT_D;
  const bf16_t* DO = a.dO + b * a.sdo_b + h * ATT_D;
  const float* LSE = a.lse2 + ((long)b * a.H + h) * a.Sq;  // log2 units
  const float* DEL = a.delta + ((long)b * a.H + h) * a.Sq;  // -delta
  const float c2 = a.scale_log2;

  const int nqt = (a.Sq + ATT_KT - 1) / ATT_KT;
  const int per = (nqt + a.q_split - 1) / a.q_split;
  const int qa = split * per, qb = min(nqt, qa + per);
  const int n = qb > qa ? qb - qa : 0;

  // staging: wave w fills rows (2w + pw)*8 .. +8 of each of the four images
  const int prow = lane >> 3, pch = lane & 7;
  const int lcR = pch ^ prow;                       // row-image source chunk
  const int lcT = pch ^ (2 * ((prow >> 1) & 3));    // transposed-image source chunk
  // buffer_load ... lds against per-(batch, head) SGPR resources ending at query row Sq - 1 (rows past it read as
  // zeros; padded queries are masked through the LSE): loop-invariant 32-bit lane offsets, the tile advance is the
  // scalar soffset
  const __amdgpu_buffer_rsrc_t rQ =
      __builtin_amdgcn_make_buffer_rsrc((void*)Q, (short)0, (int)(((long)(a.Sq - 1) * a.ldq + ATT_D) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rO =
      __builtin_amdgcn_make_buffer_rsrc((void*)DO, (short)0, (int)(((long)(a.Sq - 1) * a.lddo + ATT_D) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rL =
      __builtin_amdgcn_make_buffer_rsrc((void*)(wave == 0 ? LSE : DEL), (short)0, a.Sq * 4, 0x00020000);
  unsigned qro[2], qto[2], oro[2], oto[2];
#pragma unroll
  for (int pw = 0; pw < 2; ++pw) {
    const int row = (wave * 2 + pw) * 8 + prow;
    qro[pw] = (unsigned)(row * (int)a.ldq + lcR * 8) * 2u;
    qto[pw] = (unsigned)(row * (int)a.ldq + lcT * 8) * 2u;
    oro[pw] = (unsigned)(row * (int)a.lddo + lcR * 8) * 2u;
    oto[pw] = (unsigned)(row * (int)a.lddo + lcT * 8) * 2u;
  }
  const int qstep = ATT_KT * (int)a.ldq * 2, ostep = ATT_KT * (int)a.lddo * 2;  // bytes per query tile
  auto issue = [&](int qt, int buf) {
    bf16_t* img = sbase + buf * NIMG * IMG;
    if (wave < 2)  // LSE (wave 0) / delta (wave 1): one dword per lane, issued first so it retires first
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rL, (att_lds_void*)(sLD + (buf * 2 + wave) * 64), 4, lane * 4,
                                               qt * ATT_KT * 4, 0, 0);
#pragma unroll
    for (int pw = 0; pw < 2; ++pw) {
      const int piece = wave * 2 + pw;
      if constexpr (ONE) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rQ, (att_lds_void*)(img + piece * 8 * ATT_D), 16, qto[pw], qt * qstep,
                                                 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rO, (att_lds_void*)(img + IMG + piece * 8 * ATT_D), 16, oto[pw],
                                                 qt * ostep, 0, 0);
        continue;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rQ, (att_lds_void*)(img + piece * 8 * ATT_D), 16, qro[pw], qt * qstep, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rQ, (att_lds_void*)(img + IMG + piece * 8 * ATT_D), 16, qto[pw], qt * qstep,
                                               0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rO, (att_lds_void*)(img + 2 * IMG + piece * 8 * ATT_D), 16, oro[pw],
                                               qt * ostep, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rO, (att_lds_void*)(img + 3 * IMG + piece * 8 * ATT_D), 16, oto[pw],
                                               qt * ostep, 0, 0);
    }
  };

  // K and V fragments of this wave's 16*KJ keys (B operands): lane holds K[k0 + kj*16 + c][ds*32 + 8g ..]
  bf16x8 kf[KJ][2], vf[KJ][2];
#pragma unroll
  for (int kj = 0; kj < KJ; ++kj) {
    const int kr = min(k0 + kj * 16 + c, a.Sk - 1);  // clamped keys: computed, never stored
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) {
      kf[kj][ds] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(K + (long)kr * a.ldk + ds * 32 + 8 * g));
      vf[kj][ds] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(V + (long)kr * a.ldv + ds * 32 + 8 * g));
    }
  }
  // PF: byte offset (inside a 64 x 64 transposed-read image) of this lane's ds_read_b64_tr_b16 for d-block dt at query
  // rows 0..15; the query row block (32 qk + 16 h) adds (32 qk + 16 h) * 128 B and the dO image sits 16 KB after the Q
  // image, so one base register per dt serves all 32 transposed reads of a tile through the instruction's offset field
  unsigned troff[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int li = lane & 15;
    const int col = dt * 16 + 4 * (li & 3);
    troff[dt] = 2u * (unsigned)(swz_tr(4 * g + (li >> 2), col >> 3) + (col & 7));
  }
  f32x4 dk[KJ][4], dv[KJ][4];  // [kj][dt]: lane holds d?[k = kj*16 + c][d = dt*16 + 4g + r]
#pragma unroll
  for (int kj = 0; kj < KJ; ++kj)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dk[kj][dt] = dv[kj][dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  static_assert(STG >= 2 && STG <= 5, "att_wait_barrier covers rings of up to 5 stages");
  for (int t = 0; t < STG - 1 && t < n; ++t) issue(qa + t, t);
  for (int i = 0; i < n; ++i) {
    // tile i landed (this wave's pieces: all but those of the min(STG - 2, n - 1 - i) younger tiles), then every
    // wave's; the barrier also orders every wave's reads of tile i - 1 before its slot is re-staged below
    att_wait_barrier<PIECES>(min(STG - 2, n - 1 - i));
    if (i + STG - 1 < n) issue(qa + i + STG - 1, (i + STG - 1) % STG);
    const int buf = i % STG;
    const bf16_t* sQt = sbase + buf * NIMG * IMG + (ONE ? 0 : IMG);
    const bf16_t* sOt = sbase + buf * NIMG * IMG + (ONE ? IMG : 3 * IMG);
    const bf16_t* sQr = ONE ? sQt : sbase + buf * NIMG * IMG;
    const bf16_t* sOr = ONE ? sOt : sbase + buf * NIMG * IMG + 2 * IMG;
    const float* sL = sLD + buf * 2 * 64;
    const float* sD = sL + 64;
    const int qbase = (qa + i) * ATT_KT;
    const bool qpart = qbase + ATT_KT > a.Sq;
    float4 lpf[4], dpf[4];
    if constexpr (PF) {
      const unsigned lb = (unsigned)(uintptr_t)(const att_lds_void*)(sL + 4 * g);  // sD = sL + 64 floats (256 B)
      asm volatile("ds_read_b128 %0, %1" : "=v"(lpf[0]) : "v"(lb));
      asm volatile("ds_read_b128 %0, %1 offset:64" : "=v"(lpf[1]) : "v"(lb));
      asm volatile("ds_read_b128 %0, %1 offset:128" : "=v"(lpf[2]) : "v"(lb));
      asm volatile("ds_read_b128 %0, %1 offset:192" : "=v"(lpf[3]) : "v"(lb));
      asm volatile("ds_read_b128 %0, %1 offset:256" : "=v"(dpf[0]) : "v"(lb));
      asm volatile("ds_read_b128 %0, %1 offset:320" : "=v"(dpf[1]) : "v"(lb));
      asm volatile("ds_read_b128 %0, %1 offset:384" : "=v"(dpf[2]) : "v"(lb));
      asm volatile("ds_read_b128 %0, %1 offset:448" : "=v"(dpf[3]) : "v"(lb));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int qk = 0; qk < 2; ++qk) {
      // P and dS for 32 queries (2 subtiles) x this wave's keys: lane holds X[q = qs*16 + 4g + r][k = kj*16 + c]
      f32x4 p[2][KJ], dsv[2][KJ];
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) {
        const int qs = 2 * qk + qh;
        bf16x8 qa_[2], oa_[2];
#pragma unroll
        for (int d2 = 0; d2 < 2; ++d2) {
          const int ro = ONE ? swz_tr(qs * 16 + c, d2 * 4 + g) : swz_row(qs * 16 + c, d2 * 4 + g);
          qa_[d2] = *reinterpret_cast<const bf16x8*>(sQr + ro);
          oa_[d2] = *reinterpret_cast<const bf16x8*>(sOr + ro);
        }
        // LSE / delta through inline-asm LDS reads: as plain loads hipcc cannot tell them from the ring's pending
        // LDS-DMA writes and drains the whole ring (vmcnt(0)), prefetch of the next query tile included
        float4 l4, d4;
        if constexpr (PF) {
          l4 = lpf[qs];
          d4 = dpf[qs];
        } else {
          asm volatile("ds_read_b128 %0, %1" : "=v"(l4) : "v"((unsigned)(uintptr_t)(const att_lds_void*)(sL + qs * 16 + 4 * g)));
          asm volatile("ds_read_b128 %0, %1" : "=v"(d4) : "v"((unsigned)(uintptr_t)(const att_lds_void*)(sD + qs * 16 + 4 * g)));
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);  // nothing reads l4 / d4 (or moves above) before the wait
        }
        float lq[4] = {l4.x, l4.y, l4.z, l4.w};  // LSE * log2(e), from the dQ kernel
        const f32x4 ndel = {d4.x, d4.y, d4.z, d4.w};  // -delta, from the dQ kernel
        // PF: no mask -- query rows past Sq read as zeros (Q, dO and the LSE / delta resources end at row Sq - 1), so a
        // padded row has S = 0, p = 1, dP = 0 and dS = 0, and its zero Q / dO rows add nothing to dK / dV
        if (!PF && qpart) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (qbase + qs * 16 + 4 * g + r >= a.Sq) lq[r] = INFINITY;  // padded query rows: p = 0
        }
#pragma unroll
        for (int kj = 0; kj < KJ; ++kj) {
          // dP accumulates onto -delta (register r = query 4g + r), so dS = P * acc: one VALU op per score less
          f32x4 sacc = {0.f, 0.f, 0.f, 0.f}, pacc = ndel;
          sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa_[0], kf[kj][0], sacc, 0, 0, 0);
          sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa_[1], kf[kj][1], sacc, 0, 0, 0);
          pacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa_[0], vf[kj][0], pacc, 0, 0, 0);
          pacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa_[1], vf[kj][1], pacc, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float pr = fast_exp2(fmaf(sacc[r], c2, -lq[r]));
            p[qh][kj][r] = pr;
            dsv[qh][kj][r] = pr * pacc[r];
          }
        }
      }
      // dV^T[d][k] += dO^T . P ;  dK^T[d][k] += Q^T . dS
      bf16x8 of[4], qf[4];
      if constexpr (PF) {
        // the wait is tied to the 16 read registers (no scheduling barrier): only the dV / dK MFMAs wait for it, so
        // the compiler may interleave them with the next subtile's independent work
        s16x4 otr[8], qtr[8];
        const unsigned qtb = (unsigned)(uintptr_t)(const att_lds_void*)sQt;  // sOt = sQt + 16 KB (ONE: 8 KB)
        auto trd = [&](auto QK_) {
          constexpr int o = decltype(QK_)::value * 4096;  // query rows 32 qk ..
          constexpr int OT = ONE ? 8192 : 16384;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            const unsigned ab = qtb + troff[dt];
            qtr[2 * dt] = tr_read_imm<o>(ab);
            qtr[2 * dt + 1] = tr_read_imm<o + 2048>(ab);
            otr[2 * dt] = tr_read_imm<OT + o>(ab);
            otr[2 * dt + 1] = tr_read_imm<OT + o + 2048>(ab);
          }
        };
        if (qk == 0) trd(ic<0>{});
        else trd(ic<1>{});
        lds_wait8(otr);
        lds_wait8(qtr);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          of[dt] = cat_frag(otr[2 * dt], otr[2 * dt + 1]);
          qf[dt] = cat_frag(qtr[2 * dt], qtr[2 * dt + 1]);
        }
      } else {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          of[dt] = cat_frag(tr_read_asm(sOt, (2 * qk) * 16 + 4 * g, dt * 16, lane),
                            tr_read_asm(sOt, (2 * qk + 1) * 16 + 4 * g, dt * 16, lane));
          qf[dt] = cat_frag(tr_read_asm(sQt, (2 * qk) * 16 + 4 * g, dt * 16, lane),
                            tr_read_asm(sQt, (2 * qk + 1) * 16 + 4 * g, dt * 16, lane));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
        for (int kj = 0; kj < KJ; ++kj) {
          dv[kj][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(of[dt], pack_p(p[0][kj], p[1][kj]), dv[kj][dt], 0, 0, 0);
          dk[kj][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[dt], pack_p(dsv[0][kj], dsv[1][kj]), dk[kj][dt], 0, 0, 0);
        }
      }
    }
  }
  // ---- epilogue: lane holds d?[k = k0 + kj*16 + c][d = dt*16 + 4g + r]; dK carries the softmax scale ----
  const float sc = a.scale_log2 * 0.69314718055994531f;
#pragma unroll
  for (int kj = 0; kj < KJ; ++kj) {
    const int kr = k0 + kj * 16 + c;
    if (kr >= a.Sk) continue;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int d = h * ATT_D + dt * 16 + 4 * g;
      if (a.q_split > 1) {  // this query split's partial sums -> its own fp32 slice (reduced by reduce_splits_kernel)
        const long slice = (long)split * (a.nbatch * (long)a.Sk) * (a.H * ATT_D);
        float* pk = a.dk_acc + slice + ((long)b * a.Sk + kr) * (a.H * ATT_D) + d;
        float* pv = a.dv_acc + slice + ((long)b * a.Sk + kr) * (a.H * ATT_D) + d;
        *reinterpret_cast<float4*>(pk) = make_float4(dk[kj][dt][0] * sc, dk[kj][dt][1] * sc, dk[kj][dt][2] * sc,
                                                     dk[kj][dt][3] * sc);
        *reinterpret_cast<float4*>(pv) = make_float4(dv[kj][dt][0], dv[kj][dt][1], dv[kj][dt][2], dv[kj][dt][3]);
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
// backward for short key sequences (cross-attention over the 77 text tokens, Sk <= XK_KP = 96): ONE pass over the
// query tiles makes dQ, dK and dV.  attn_bwd_dkv_kernel's structure (4 waves x 32 keys on the MFMA lane axis, so all
// keys of the (batch, head) sit in one workgroup; query tiles of 64 through a 2-stage LDS-DMA ring, query splits
// reduced by reduce_splits_kernel), plus:
//   * the output O as a third ring image: -delta = -rowsum(dO * O) of the tile's 64 queries is formed in the kernel
//     (the dQ kernel's lane pattern and summation order), so neither a dQ launch nor a delta pre-pass runs;
//   * dQ of the tile: dS is written to LDS transposed ([key][query], 4 consecutive queries per lane: ds_write_b64), and
//     wave w forms dQ^T for queries 16w .. 16w+15 against an LDS image of K (staged once; rows past Sk zero):
//     dQ^T[d][q] = sum_k K^T[d][k] dS^T[k][q], both fragments by transposed reads, 4 consecutive d per lane on store.
// Versus the dQ + dK/dV + reduce launches it skips the dQ kernel's second S / dP / exp sweep over the same queries.
// ================================================================================================================
#define XK_KP 96  // key rows of the K / dS^T images (multiple of 32: whole 32-deep MFMA steps)
__global__ __launch_bounds__(ATT_THREADS, 2) void attn_bwd_x_kernel(AttnArgs a) {
  constexpr int KJ = 2, STG = 2;
  constexpr int IMG = ATT_KT * ATT_D;  // one 64 x 64 image
  constexpr int NIMG = 3;              // Q^T, dO^T, O^T (swz_tr layout: row and transposed reads)
  constexpr int PIECES = 2 * NIMG;     // 16-B glds per wave per tile (+1 LSE dword piece on wave 0)
  __shared__ __attribute__((aligned(16))) bf16_t sRing[STG][NIMG][IMG];
  __shared__ __attribute__((aligned(16))) float sLD[STG][2][64];  // LSE (natural, by DMA), -delta (formed here)
  __shared__ __attribute__((aligned(16))) bf16_t sK[XK_KP * ATT_D];    // K rows 0 .. XK_KP-1 (swz_tr), zero past Sk
  __shared__ __attribute__((aligned(16))) bf16_t sDS[XK_KP * ATT_D];   // dS^T [key][query of the tile] (swz_tr)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c = lane & 15;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / a.q_split, split = bid - bh * a.q_split;
  const int h = bh % a.H, b = bh / a.H;
  const int k0 = wave * (16 * KJ);

  const bf16_t* Q = a.q + b * a.sq_b + h * ATT_D;
  const bf16_t* K = a.k + b * a.sk_b + h * ATT_D;
  const bf16_t* V = a.v + b * a.sv_b + h * ATT_D;
  const bf16_t* DO = a.dO + b * a.sdo_b + h * ATT_D;
  const bf16_t* Y = a.o + b * a.so_b + h * ATT_D;
  const float* LSE = a.lse + ((long)b * a.H + h) * a.Sq;
  const float c2 = a.scale_log2;
  const float ln2inv = 1.4426950408889634f;

  const int nqt = (a.Sq + ATT_KT - 1) / ATT_KT;
  const int per = (nqt + a.q_split - 1) / a.q_split;
  const int qa = split * per, qb = min(nqt, qa + per);
  const int n = qb > qa ? qb - qa : 0;

  const int prow = lane >> 3, pch = lane & 7;
  const int lcT = pch ^ (2 * ((prow >> 1) & 3));
  const __amdgpu_buffer_rsrc_t rQ =
      __builtin_amdgcn_make_buffer_rsrc((void*)Q, (short)0, (int)(((long)(a.Sq - 1) * a.ldq + ATT_D) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rD =
      __builtin_amdgcn_make_buffer_rsrc((void*)DO, (short)0, (int)(((long)(a.Sq - 1) * a.lddo + ATT_D) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rY =
      __builtin_amdgcn_make_buffer_rsrc((void*)Y, (short)0, (int)(((long)(a.Sq - 1) * a.ldo + ATT_D) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rL = __builtin_amdgcn_make_buffer_rsrc((void*)LSE, (short)0, a.Sq * 4, 0x00020000);
  unsigned qto[2], dto[2], yto[2];
#pragma unroll
  for (int pw = 0; pw < 2; ++pw) {
    const int row = (wave * 2 + pw) * 8 + prow;
    qto[pw] = (unsigned)(row * (int)a.ldq + lcT * 8) * 2u;
    dto[pw] = (unsigned)(row * (int)a.lddo + lcT * 8) * 2u;
    yto[pw] = (unsigned)(row * (int)a.ldo + lcT * 8) * 2u;
  }
  const int qstep = ATT_KT * (int)a.ldq * 2, dstep = ATT_KT * (int)a.lddo * 2, ystep = ATT_KT * (int)a.ldo * 2;
  auto issue = [&](int qt, int buf) {
    if (wave == 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rL, (att_lds_void*)(&sLD[buf][0][0]), 4, lane * 4, qt * ATT_KT * 4, 0, 0);
#pragma unroll
    for (int pw = 0; pw < 2; ++pw) {
      const int piece = wave * 2 + pw;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rQ, (att_lds_void*)(sRing[buf][0] + piece * 8 * ATT_D), 16, qto[pw],
                                               qt * qstep, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rD, (att_lds_void*)(sRing[buf][1] + piece * 8 * ATT_D), 16, dto[pw],
                                               qt * dstep, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rY, (att_lds_void*)(sRing[buf][2] + piece * 8 * ATT_D), 16, yto[pw],
                                               qt * ystep, 0, 0);
    }
  };

  // K / V fragments of this wave's 32 keys (B operands; keys past Sk clamped: computed, never stored, their dS is
  // dropped before it reaches dQ); the K image for dQ (rows past Sk zero)
  bf16x8 kf[KJ][2], vf[KJ][2];
#pragma unroll
  for (int kj = 0; kj < KJ; ++kj) {
    const int kr = min(k0 + kj * 16 + c, a.Sk - 1);
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) {
      kf[kj][ds] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(K + (long)kr * a.ldk + ds * 32 + 8 * g));
      vf[kj][ds] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(V + (long)kr * a.ldv + ds * 32 + 8 * g));
    }
  }
  for (int e = tid; e < XK_KP * 8; e += ATT_THREADS) {
    const int row = e >> 3, ch = e & 7;
    const uint4 v = row < a.Sk ? *reinterpret_cast<const uint4*>(K + (long)row * a.ldk + ch * 8) : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(sK + swz_tr(row, ch)) = v;
  }
  unsigned troff[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int li = lane & 15;
    const int col = dt * 16 + 4 * (li & 3);
    troff[dt] = 2u * (unsigned)(swz_tr(4 * g + (li >> 2), col >> 3) + (col & 7));
  }
  f32x4 dk[KJ][4], dv[KJ][4];
#pragma unroll
  for (int kj = 0; kj < KJ; ++kj)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dk[kj][dt] = dv[kj][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float sc = a.scale_log2 * 0.69314718055994531f;  // the softmax scale (dQ and dK carry it)
  const int nks = (min(a.Sk, XK_KP) + 31) >> 5;           // 32-key steps of dQ that hold a key

  // -delta of a landed tile's 64 queries into sLD[buf][1]: wave w, lane (g, c) -> query 16w + c, d chunks 4 ds + g
  // (the dQ kernel's lanes and summation order)
  auto form_delta = [&](int buf) {
    const int qr = wave * 16 + c;
    float part = 0.f;
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) {
      const uint4 w = *reinterpret_cast<const uint4*>(sRing[buf][1] + swz_tr(qr, ds * 4 + g));
      const uint4 u = *reinterpret_cast<const uint4*>(sRing[buf][2] + swz_tr(qr, ds * 4 + g));
      const uint32_t ow[4] = {u.x, u.y, u.z, u.w}, dw[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        part += bf2f(ow[j] & 0xffff) * bf2f(dw[j] & 0xffff) + bf2f(ow[j] >> 16) * bf2f(dw[j] >> 16);
    }
    part += __shfl_xor(part, 16, 64);
    part += __shfl_xor(part, 32, 64);
    if (g == 0) sLD[buf][1][qr] = -part;
  };
  // Per tile two barriers: (A) at the top -- tile i landed, its -delta formed (during tile i - 1's dQ phase), every
  // read of the previous tile's sDS done; (B) after the dS^T writes -- tile i + 1 landed too, so its -delta is formed
  // beside tile i's dQ MFMAs.
  if (n > 0) {
    issue(qa, 0);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    form_delta(0);
  }
  for (int i = 0; i < n; ++i) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // (A): no vmcnt -- the last dQ stores stay in flight
    if (i + 1 < n) issue(qa + i + 1, (i + 1) % STG);
    const int buf = i % STG;
    const bf16_t* sQt = sRing[buf][0];
    const bf16_t* sOt = sRing[buf][1];
    float4 lpf[4], dpf[4];
#pragma unroll
    for (int qs = 0; qs < 4; ++qs) {
      lpf[qs] = *reinterpret_cast<const float4*>(&sLD[buf][0][qs * 16 + 4 * g]);
      dpf[qs] = *reinterpret_cast<const float4*>(&sLD[buf][1][qs * 16 + 4 * g]);
    }
#pragma unroll
    for (int qk = 0; qk < 2; ++qk) {
      f32x4 p[2][KJ], dsv[2][KJ];
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) {
        const int qs = 2 * qk + qh;
        bf16x8 qa_[2], oa_[2];
#pragma unroll
        for (int d2 = 0; d2 < 2; ++d2) {
          const int ro = swz_tr(qs * 16 + c, d2 * 4 + g);
          qa_[d2] = *reinterpret_cast<const bf16x8*>(sQt + ro);
          oa_[d2] = *reinterpret_cast<const bf16x8*>(sOt + ro);
        }
        // rows past Sq read as zeros (Q, dO, O and the LSE resources end at row Sq - 1): S = 0, p = 1, dP = 0,
        // delta = 0, dS = 0 -- they add nothing to dK / dV and their dQ rows are not stored
        const float lq[4] = {lpf[qs].x * ln2inv, lpf[qs].y * ln2inv, lpf[qs].z * ln2inv, lpf[qs].w * ln2inv};
        const f32x4 ndel = {dpf[qs].x, dpf[qs].y, dpf[qs].z, dpf[qs].w};
#pragma unroll
        for (int kj = 0; kj < KJ; ++kj) {
          f32x4 sacc = {0.f, 0.f, 0.f, 0.f}, pacc = ndel;
          sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa_[0], kf[kj][0], sacc, 0, 0, 0);
          sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa_[1], kf[kj][1], sacc, 0, 0, 0);
          pacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa_[0], vf[kj][0], pacc, 0, 0, 0);
          pacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa_[1], vf[kj][1], pacc, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float pr = fast_exp2(fmaf(sacc[r], c2, -lq[r]));
            p[qh][kj][r] = pr;
            dsv[qh][kj][r] = pr * pacc[r];
          }
          // dS^T for dQ: key row k, queries qs*16 + 4g .. +3 (8 B); keys past Sk (clamped duplicates) are zero
          const int kr = k0 + kj * 16 + c;
          if (kr < XK_KP) {
            const bool live = kr < a.Sk;
            const uint2 wv = live ? make_uint2(pack2bf(dsv[qh][kj][0], dsv[qh][kj][1]), pack2bf(dsv[qh][kj][2], dsv[qh][kj][3]))
                                  : make_uint2(0u, 0u);
            const int col = qs * 16 + 4 * g;
            *reinterpret_cast<uint2*>(sDS + swz_tr(kr, col >> 3) + (col & 7)) = wv;
          }
        }
      }
      bf16x8 of[4], qf[4];
      {
        s16x4 otr[8], qtr[8];
        const unsigned qtb = (unsigned)(uintptr_t)(const att_lds_void*)sQt;
        const unsigned otb = (unsigned)(uintptr_t)(const att_lds_void*)sOt;
        auto trd = [&](auto QK_) {
          constexpr int o = decltype(QK_)::value * 4096;  // query rows 32 qk ..
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            qtr[2 * dt] = tr_read_imm<o>(qtb + troff[dt]);
            qtr[2 * dt + 1] = tr_read_imm<o + 2048>(qtb + troff[dt]);
            otr[2 * dt] = tr_read_imm<o>(otb + troff[dt]);
            otr[2 * dt + 1] = tr_read_imm<o + 2048>(otb + troff[dt]);
          }
        };
        if (qk == 0) trd(ic<0>{});
        else trd(ic<1>{});
        lds_wait8(otr);
        lds_wait8(qtr);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          of[dt] = cat_frag(otr[2 * dt], otr[2 * dt + 1]);
          qf[dt] = cat_frag(qtr[2 * dt], qtr[2 * dt + 1]);
        }
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
        for (int kj = 0; kj < KJ; ++kj) {
          dv[kj][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(of[dt], pack_p(p[0][kj], p[1][kj]), dv[kj][dt], 0, 0, 0);
          dk[kj][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[dt], pack_p(dsv[0][kj], dsv[1][kj]), dk[kj][dt], 0, 0, 0);
        }
      }
    }
    // dQ^T of queries 16 wave .. +15 of the tile: A = K^T (16 d x 32 keys), B = dS^T (32 keys x 16 queries), both by
    // transposed reads in natural key order (rows 8g .. 8g+7 of each 32-key step)
    att_wait_barrier<PIECES>(0);  // (B): every wave's dS^T written, tile i + 1 landed
    if (i + 1 < n) form_delta((i + 1) % STG);
    {
      f32x4 dq[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int st = 0; st < nks; ++st) {
        const int r0 = st * 32 + 8 * g;
        const bf16x8 bfr = cat_frag(tr_read(sDS, r0, wave * 16, lane), tr_read(sDS, r0 + 4, wave * 16, lane));
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const bf16x8 kfr = cat_frag(tr_read(sK, r0, dt * 16, lane), tr_read(sK, r0 + 4, dt * 16, lane));
          dq[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kfr, bfr, dq[dt], 0, 0, 0);
        }
      }
      const int qr = (qa + i) * ATT_KT + wave * 16 + c;
      if (qr < a.Sq) {
        bf16_t* dQ = a.dq + b * a.sdq_b + (long)qr * a.lddq + h * ATT_D;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          *reinterpret_cast<uint2*>(dQ + dt * 16 + 4 * g) =
              make_uint2(pack2bf(dq[dt][0] * sc, dq[dt][1] * sc), pack2bf(dq[dt][2] * sc, dq[dt][3] * sc));
      }
    }
  }
  // dK / dV epilogue (lane holds d?[k = k0 + kj*16 + c][d = dt*16 + 4g + r]), as attn_bwd_dkv_kernel
#pragma unroll
  for (int kj = 0; kj < KJ; ++kj) {
    const int kr = k0 + kj * 16 + c;
    if (kr >= a.Sk) continue;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int d = h * ATT_D + dt * 16 + 4 * g;
      if (a.q_split > 1) {
        const long slice = (long)split * (a.nbatch * (long)a.Sk) * (a.H * ATT_D);
        float* pk = a.dk_acc + slice + ((long)b * a.Sk + kr) * (a.H * ATT_D) + d;
        float* pv = a.dv_acc + slice + ((long)b * a.Sk + kr) * (a.H * ATT_D) + d;
        *reinterpret_cast<float4*>(pk) = make_float4(dk[kj][dt][0] * sc, dk[kj][dt][1] * sc, dk[kj][dt][2] * sc,
                                                     dk[kj][dt][3] * sc);
        *reinterpret_cast<float4*>(pv) = make_float4(dv[kj][dt][0], dv[kj][dt][1], dv[kj][dt][2], dv[kj][dt][3]);
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
// backward dK/dV, ping-pong form: one workgroup = 8 waves = 256 keys of one (b, h), 32 per wave as in the form above
// (same arithmetic, same accumulation order: bit-identical dK / dV).  Waves w and w + 4 share a SIMD; the two groups
// (waves 0-3 / 4-7) share one Q / dO query-tile ring and run one segment apart, every query tile being two segments
// separated by s_barrier:
//     A_t (matrix): dV += dO^T P, dK += Q^T dS of tile t - 1 (transposed reads), then S = Q K^T and dP = dO V^T - delta
//                   of tile t (row reads)                                  -- 64 MFMAs, the LDS reads
//     B_t (vector): P = exp2(S c - LSE), dS = P dP, packed to bf16        -- 32 exp + ~96 VALU, no MFMA
// Group 1 takes one extra barrier before its loop and group 0 one after it, so while one wave of a SIMD runs its A
// segment the other runs its B segment: the exp / dS vector work issues beside the partner's MFMAs instead of in
// series with its own.  Ring: STG slots of [Q 64 x 64 | dO 64 x 64] (the swz_tr layout serves the row and the
// transposed reads) + [LSE 64 | -delta 64]; every wave stages one 8-row piece of Q and of dO and the LSE (even waves)
// or -delta (odd waves) of each tile.  The slot of tile t is last read in group 1's A_{t+1} (global segment 2t + 3),
// so tile t + STG is issued at global segment 2t + 4 (group 0: at A_{t+2}; group 1: at B_{t+1}) and has 2 STG - 4
// segments to land before group 0 reads it; each group waits for a tile right before the barrier that opens the
// segment where it (group 0) or its partner group first reads it.
// ================================================================================================================
template <int OFF>
__device__ __forceinline__ bf16x8 lds_b128(unsigned addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset range");
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ f32x4 lds_f32x4(unsigned addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset range");
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
// An empty volatile asm that takes a segment's results as in/out operands: they must be computed before it, and it
// cannot move across the segment's closing s_barrier (volatile asm keeps its order), so the compiler cannot sink a
// segment's MFMA or VALU work into the next segment (machine sinking otherwise moves the exp / dS block, whose only
// users are the next segment's MFMAs, behind the barrier, and the two groups' segments stop being complementary)
template <int A, int B>
__device__ __forceinline__ void pin_segment(f32x4 (&x)[A][B], f32x4 (&y)[A][B]) {
  static_assert(A * B == 8 || A * B == 4, "operand count");
  if constexpr (A * B == 8)
    asm volatile("" : "+v"(x[0][0]), "+v"(x[0][1]), "+v"(x[0][2]), "+v"(x[0][3]), "+v"(x[1][0]), "+v"(x[1][1]),
                 "+v"(x[1][2]), "+v"(x[1][3]), "+v"(y[0][0]), "+v"(y[0][1]), "+v"(y[0][2]), "+v"(y[0][3]),
                 "+v"(y[1][0]), "+v"(y[1][1]), "+v"(y[1][2]), "+v"(y[1][3]));
}
template <>
__device__ __forceinline__ void pin_segment<4, 2>(f32x4 (&x)[4][2], f32x4 (&y)[4][2]) {
  asm volatile("" : "+v"(x[0][0]), "+v"(x[0][1]), "+v"(x[1][0]), "+v"(x[1][1]), "+v"(x[2][0]), "+v"(x[2][1]),
               "+v"(x[3][0]), "+v"(x[3][1]), "+v"(y[0][0]), "+v"(y[0][1]), "+v"(y[1][0]), "+v"(y[1][1]),
               "+v"(y[2][0]), "+v"(y[2][1]), "+v"(y[3][0]), "+v"(y[3][1]));
}
__device__ __forceinline__ void pp_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// PRIO: the A segment at s_setprio 1.  TR (diagnostic): workgroup 0's waves 0 and 4 record the shader clock before
// and after every barrier in g_pp_trace (tools/pp_trace.py).  Measured, not the default: compiled
// into the tools build only (-DPSO_BENCH_KNOBS).
#ifdef PSO_BENCH_KNOBS
__device__ unsigned long long g_pp_trace[2][520];
template <int STG, bool PRIO = false, bool TR = false>
__global__ __launch_bounds__(512, 1) void attn_bwd_dkv_pp_kernel(AttnArgs a, int nkb) {
  static_assert(STG == 3 || STG == 4, "ring depth: the counted waits encode at most 3 younger tiles");
  constexpr int IMG = ATT_KT * ATT_D;
  constexpr int P = 3;                      // LDS-DMA loads per wave per tile
  constexpr unsigned SLOT = 2 * IMG * 2;    // bytes of one slot's Q + dO images
  constexpr unsigned OIMG = IMG * 2;        // byte offset of the dO image in a slot
  extern __shared__ __attribute__((aligned(16))) bf16_t att_dyn[];
  float* const sLD = reinterpret_cast<float*>(att_dyn + STG * 2 * IMG);  // [STG][LSE 64 | -delta 64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;  // (a wave & 1 map, same-phase partners on a SIMD: 1.43 vs 1.18 ms, measured)
  const int g = lane >> 4, c = lane & 15;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / nkb, kb = bid - bh * nkb;
  const int h = bh % a.H, b = bh / a.H;
  const int k0 = kb * 256 + wave * 32;

  const bf16_t* Q = a.q + b * a.sq_b + h * ATT_D;
  const bf16_t* K = a.k + b * a.sk_b + h * ATT_D;
  const bf16_t* V = a.v + b * a.sv_b + h * ATT_D;
  const bf16_t* DO = a.dO + b * a.sdo_b + h * ATT_D;
  const float* LSE = a.lse2 + ((long)b * a.H + h) * a.Sq;  // log2 units
  const float* DEL = a.delta + ((long)b * a.H + h) * a.Sq;  // -delta
  const float c2 = a.scale_log2;
  const int n = (a.Sq + ATT_KT - 1) / ATT_KT;

  // staging (rows past Sq read as zeros through the resources: a padded query has S = 0, p = 1, dP = 0, dS = 0 and
  // zero Q / dO rows, so it adds nothing -- no mask)
  const int prow = lane >> 3, pch = lane & 7;
  const int lcT = pch ^ (2 * ((prow >> 1) & 3));
  const __amdgpu_buffer_rsrc_t rQ =
      __builtin_amdgcn_make_buffer_rsrc((void*)Q, (short)0, (int)(((long)(a.Sq - 1) * a.ldq + ATT_D) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rO =
      __builtin_amdgcn_make_buffer_rsrc((void*)DO, (short)0, (int)(((long)(a.Sq - 1) * a.lddo + ATT_D) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rL =
      __builtin_amdgcn_make_buffer_rsrc((void*)((wave & 1) ? DEL : LSE), (short)0, a.Sq * 4, 0x00020000);
  const unsigned qo = (unsigned)((wave * 8 + prow) * (int)a.ldq + lcT * 8) * 2u;
  const unsigned oo = (unsigned)((wave * 8 + prow) * (int)a.lddo + lcT * 8) * 2u;
  const int qstep = ATT_KT * (int)a.ldq * 2, ostep = ATT_KT * (int)a.lddo * 2;
  auto issue = [&](int qt) {
    const int sl = qt % STG;
    bf16_t* img = att_dyn + sl * 2 * IMG;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rL, (att_lds_void*)(sLD + sl * 128 + (wave & 1) * 64), 4, lane * 4,
                                             qt * ATT_KT * 4, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rQ, (att_lds_void*)(img + wave * 8 * ATT_D), 16, qo, qt * qstep, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rO, (att_lds_void*)(img + IMG + wave * 8 * ATT_D), 16, oo, qt * ostep, 0,
                                             0);
  };

  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int kj = 0; kj < 2; ++kj) {
    const int kr = min(k0 + kj * 16 + c, a.Sk - 1);  // clamped keys: computed, never stored
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) {
      kf[kj][ds] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(K + (long)kr * a.ldk + ds * 32 + 8 * g));
      vf[kj][ds] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(V + (long)kr * a.ldv + ds * 32 + 8 * g));
    }
  }
  const unsigned lds0 = (unsigned)(uintptr_t)(const att_lds_void*)att_dyn;
  const unsigned ldl = lds0 + STG * SLOT + 16u * g;  // this lane's LSE quad (queries 4g ..) of slot 0
  // transposed reads (as the form above): one lane offset per 16-column block dt, rows / image / slot are offsets
  unsigned troff[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int li = lane & 15;
    const int col = dt * 16 + 4 * (li & 3);
    troff[dt] = 2u * (unsigned)(swz_tr(4 * g + (li >> 2), col >> 3) + (col & 7));
  }
  // row reads: Q[qs * 16 + c][d2 * 32 + 8 g ..] -- the swz_tr XOR of row qs * 16 + c does not depend on qs
  const unsigned rb0 = 2u * (unsigned)swz_tr(c, g), rb1 = 2u * (unsigned)swz_tr(c, 4 + g);

  f32x4 dk[2][4], dv[2][4];
#pragma unroll
  for (int kj = 0; kj < 2; ++kj)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dk[kj][dt] = dv[kj][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 S[4][2], DP[4][2];   // [qs][kj]: lane holds X[q = qs*16 + 4g + r][k = kj*16 + c]
  bf16x8 pP[2][2], pS[2][2];  // [qk][kj]: P / dS of the query pairs (qs = 2 qk, 2 qk + 1), packed

  // transposed Q / dO fragments of the tile whose dV / dK the next A segment forms: read at the end of the B segment
  // (whose wave then waits at the barrier for its partner's longer A segment anyway), so A opens on loaded registers
  s16x4 qtr[2][8], otr[2][8];
  auto t_issue_q = [&](int sl, auto QK_) {
    constexpr int qk = decltype(QK_)::value;
    const unsigned sb = lds0 + (unsigned)sl * SLOT;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const unsigned ab = sb + troff[dt];
      qtr[qk][2 * dt] = tr_read_imm<qk * 4096>(ab);
      qtr[qk][2 * dt + 1] = tr_read_imm<qk * 4096 + 2048>(ab);
      otr[qk][2 * dt] = tr_read_imm<OIMG + qk * 4096>(ab);
      otr[qk][2 * dt + 1] = tr_read_imm<OIMG + qk * 4096 + 2048>(ab);
    }
  };
  auto t_issue = [&](int sl) {
    t_issue_q(sl, ic<0>{});
    t_issue_q(sl, ic<1>{});
  };
  // A: dV / dK of the query pair qk of the previous tile (its fragments landed before the opening barrier)
  auto m2q = [&](int qk) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8 of = cat_frag(otr[qk][2 * dt], otr[qk][2 * dt + 1]);
      const bf16x8 qf = cat_frag(qtr[qk][2 * dt], qtr[qk][2 * dt + 1]);
#pragma unroll
      for (int kj = 0; kj < 2; ++kj) {
        dv[kj][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(of, pP[qk][kj], dv[kj][dt], 0, 0, 0);
        dk[kj][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf, pS[qk][kj], dk[kj][dt], 0, 0, 0);
      }
    }
  };
  // A: S and dP (onto -delta) of the tile in slot sl (reads of query pair qs + 1 in flight during qs's MFMAs)
  f32x4 nd[4];
  bf16x8 fr[2][4];  // [qs parity][qa0 qa1 oa0 oa1]
  auto m1 = [&](int sl) {
    const unsigned sb = lds0 + (unsigned)sl * SLOT;
    const unsigned r0 = sb + rb0, r1 = sb + rb1;
    const unsigned db = ldl + (unsigned)sl * 512u;  // + 256: -delta
    nd[0] = lds_f32x4<256>(db);
    nd[1] = lds_f32x4<256 + 64>(db);
    nd[2] = lds_f32x4<256 + 128>(db);
    nd[3] = lds_f32x4<256 + 192>(db);
    auto rd = [&](auto QS_) {
      constexpr int qs = decltype(QS_)::value;
      fr[qs & 1][0] = lds_b128<qs * 2048>(r0);
      fr[qs & 1][1] = lds_b128<qs * 2048>(r1);
      fr[qs & 1][2] = lds_b128<OIMG + qs * 2048>(r0);
      fr[qs & 1][3] = lds_b128<OIMG + qs * 2048>(r1);
    };
    auto mm = [&](auto QS_) {
      constexpr int qs = decltype(QS_)::value;
      bf16x8(&f)[4] = fr[qs & 1];
      if (qs == 0)  // the 4 delta reads and qs 0's 4 fragments; qs 1's 4 stay in flight
        asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(nd[0]), "+v"(nd[1]),
                     "+v"(nd[2]), "+v"(nd[3]));
      else if (qs < 3)
        asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
      else
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
#pragma unroll
      for (int kj = 0; kj < 2; ++kj) {
        f32x4 sacc = {0.f, 0.f, 0.f, 0.f}, pacc = nd[qs];
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[0], kf[kj][0], sacc, 0, 0, 0);
        S[qs][kj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[1], kf[kj][1], sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[2], vf[kj][0], pacc, 0, 0, 0);
        DP[qs][kj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[3], vf[kj][1], pacc, 0, 0, 0);
      }
    };
    rd(ic<0>{});
    rd(ic<1>{});
    mm(ic<0>{});
    rd(ic<2>{});
    mm(ic<1>{});
    rd(ic<3>{});
    mm(ic<2>{});
    mm(ic<3>{});
    pin_segment(S, DP);
  };
  // B: P and dS of the tile in slot sl, packed
  auto vseg = [&](int sl) {
    const unsigned lb = ldl + (unsigned)sl * 512u;
    f32x4 lq[4];
    lq[0] = lds_f32x4<0>(lb);
    lq[1] = lds_f32x4<64>(lb);
    lq[2] = lds_f32x4<128>(lb);
    lq[3] = lds_f32x4<192>(lb);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lq[0]), "+v"(lq[1]), "+v"(lq[2]), "+v"(lq[3]));
#pragma unroll
    for (int qk = 0; qk < 2; ++qk)
#pragma unroll
      for (int kj = 0; kj < 2; ++kj) {
        f32x4 pv[2], dsv[2];
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          const int qs = 2 * qk + qh;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float pr = fast_exp2(fmaf(S[qs][kj][r], c2, -lq[qs][r]));
            pv[qh][r] = pr;
            dsv[qh][r] = pr * DP[qs][kj][r];
          }
        }
        pP[qk][kj] = pack_p(pv[0], pv[1]);
        pS[qk][kj] = pack_p(dsv[0], dsv[1]);
      }
    asm volatile("" : "+v"(pP[0][0]), "+v"(pP[0][1]), "+v"(pP[1][0]), "+v"(pP[1][1]), "+v"(pS[0][0]), "+v"(pS[0][1]),
                 "+v"(pS[1][0]), "+v"(pS[1][1]));
  };

  const bool trw = TR && blockIdx.x == 0 && (wave & 3) == 0 && lane == 0;
  int trn = 0;
  auto trace = [&]() {
    if (TR) {
      const unsigned long long tc = __builtin_amdgcn_s_memtime();
      if (trw && trn < 520) g_pp_trace[grp][trn] = tc;
      ++trn;
    }
  };
  for (int t = 0; t < STG && t < n; ++t) issue(t);
  if (grp) att_wait_barrier<P>(min(n - 1, STG - 1));  // group 1's extra barrier: it runs one segment behind
  for (int t = 0;; ++t) {
    trace();  // (TR: end of the previous segment's work, before its barrier wait)
    // barrier opening A_t: group 0 first reads tile t in it
    if (!grp && t < n) att_wait_barrier<P>(min(n - 1, max(STG - 1, t + STG - 3)) - t);
    else pp_bar();
    trace();
    if (!grp && t >= 2 && t + STG - 2 < n) issue(t + STG - 2);
    if (PRIO) __builtin_amdgcn_s_setprio(1);
    if (t > 0) {
      m2q(0);
      m2q(1);
      pin_segment(dv, dk);
    }
    if (t == n) break;
    m1(t % STG);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    // barrier opening B_t: group 1's partner (group 0) reads tile t + 1 right after it
    trace();
    if (grp) att_wait_barrier<P>(t + 1 < n ? min(n - 1, max(STG - 1, t + STG - 2)) - (t + 1) : 0);
    else pp_bar();
    trace();
    if (grp && t >= 1 && t + STG - 1 < n) issue(t + STG - 1);
    vseg(t % STG);
    t_issue(t % STG);
  }
  if (!grp) pp_bar();  // group 0's extra barrier: every wave takes 2 n + 2

  const float sc = a.scale_log2 * 0.69314718055994531f;
#pragma unroll
  for (int kj = 0; kj < 2; ++kj) {
    const int kr = k0 + kj * 16 + c;
    if (kr >= a.Sk) continue;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int d = h * ATT_D + dt * 16 + 4 * g;
      *reinterpret_cast<uint2*>(a.dk + b * a.sdk_b + (long)kr * a.lddk + d) =
          make_uint2(pack2bf(dk[kj][dt][0] * sc, dk[kj][dt][1] * sc), pack2bf(dk[kj][dt][2] * sc, dk[kj][dt][3] * sc));
      *reinterpret_cast<uint2*>(a.dv + b * a.sdv_b + (long)kr * a.lddv + d) =
          make_uint2(pack2bf(dv[kj][dt][0], dv[kj][dt][1]), pack2bf(dv[kj][dt][2], dv[kj][dt][3]));
    }
  }
}
#endif  // PSO_BENCH_KNOBS (the ping-pong dK/dV form)

// ================================================================================================================
// backward dQ: forward structure (128 queries per workgroup, S^T = K.Q^T lane-local per query), K/V tiles through LDS;
// also forms delta[b][h][q] = sum_d dO * O for its queries (stored for the dK/dV kernel launched after it)
//   dP^T = V . dO^T ; dS^T = P^T * (dP^T - delta) ; dQ^T[d][q] += K^T . dS^T  (K^T via transposed reads)
// ================================================================================================================
// ONE: the K row reads come from the transposed-read image (swz_tr serves both reads conflict-free), so a stage holds
// two images instead of three
template <int STG = 3, bool ONE = false>
__global__ __launch_bounds__(ATT_THREADS, 2) void attn_bwd_dq_kernel(AttnArgs a) {
  // K/V tiles arrive by LDS-DMA through a STG-stage ring (STG - 1 tiles in flight behind a counted vmcnt, one barrier
  // per tile) as three images per stage: K row image, K transposed-read image, V row image (source-side swizzles).
  static_assert(STG == 3 || STG == 4, "ring depth");
  constexpr int NIMG = ONE ? 2 : 3;
  constexpr int PIECES = 2 * NIMG;  // glds per wave per tile: 2 pieces per image
  constexpr int IMG = ATT_KT * ATT_D;
  __shared__ __attribute__((aligned(16))) bf16_t sRing[STG][NIMG][IMG];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: LDS-DMA destinations (M0) are scalar
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
  const bf16_t* O = a.o + b * a.so_b + h * ATT_D;
#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    const int qr = q0 + qi * 16 + c;
    float part = 0.f;  // delta = sum_d dO * O of this query: lanes c, c+16, c+32, c+48 hold its 64 d (2 x 8 each)
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) {
      uint4 v = make_uint4(0, 0, 0, 0), w = make_uint4(0, 0, 0, 0), u = make_uint4(0, 0, 0, 0);
      if (qr < a.Sq) {
        v = *reinterpret_cast<const uint4*>(Q + (long)qr * a.ldq + ds * 32 + 8 * g);
        w = *reinterpret_cast<const uint4*>(DO + (long)qr * a.lddo + ds * 32 + 8 * g);
        u = *reinterpret_cast<const uint4*>(O + (long)qr * a.ldo + ds * 32 + 8 * g);
      }
      qf[qi][ds] = __builtin_bit_cast(bf16x8, v);
      of[qi][ds] = __builtin_bit_cast(bf16x8, w);
      const uint32_t ow[4] = {u.x, u.y, u.z, u.w}, dw[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        part += bf2f(ow[j] & 0xffff) * bf2f(dw[j] & 0xffff) + bf2f(ow[j] >> 16) * bf2f(dw[j] >> 16);
    }
    part += __shfl_xor(part, 16, 64);
    part += __shfl_xor(part, 32, 64);
    dl[qi] = part;
    lq[qi] = qr < a.Sq ? a.lse[((long)b * a.H + h) * a.Sq + qr] * ln2inv : INFINITY;
    // published for the dK/dV kernel, which runs after this one on the stream: -delta and the LSE in log2 units, the
    // forms its tile loop consumes as they stand
    if (qr < a.Sq && g == 0) {
      a.delta[((long)b * a.H + h) * a.Sq + qr] = -part;
      a.lse2[((long)b * a.H + h) * a.Sq + qr] = lq[qi];
    }
  }
  f32x4 dq[2][4];
#pragma unroll
  for (int qi = 0; qi < 2; ++qi)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[qi][dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (a.Sk + ATT_KT - 1) / ATT_KT;
  const int prow = lane >> 3, pch = lane & 7;
  const int lcR = pch ^ prow;                     // row-image source chunk (swz_row)
  const int lcT = pch ^ (2 * ((prow >> 1) & 3));  // transposed-read image source chunk (swz_tr)
  // buffer_load ... lds against per-(batch, head) SGPR resources ending at key row Sk - 1 (rows past it read as zeros
  // and are masked on the last tile): the per-lane part of every staging address is a loop-invariant 32-bit offset and
  // the tile advance the scalar soffset (per-lane 64-bit row pointers cost ~50 VALU instructions per tile)
  const __amdgpu_buffer_rsrc_t rK =
      __builtin_amdgcn_make_buffer_rsrc((void*)K, (short)0, (int)(((long)(a.Sk - 1) * a.ldk + ATT_D) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rV =
      __builtin_amdgcn_make_buffer_rsrc((void*)V, (short)0, (int)(((long)(a.Sk - 1) * a.ldv + ATT_D) * 2), 0x00020000);
  unsigned kro[2], kto[2], vro[2];
#pragma unroll
  for (int pw = 0; pw < 2; ++pw) {
    const int row = (wave * 2 + pw) * 8 + prow;
    kro[pw] = (unsigned)(row * (int)a.ldk + lcR * 8) * 2u;
    kto[pw] = (unsigned)(row * (int)a.ldk + lcT * 8) * 2u;
    vro[pw] = (unsigned)(row * (int)a.ldv + lcR * 8) * 2u;
  }
  const int kstep = ATT_KT * (int)a.ldk * 2, vstep = ATT_KT * (int)a.ldv * 2;  // bytes per key tile
  auto issue = [&](int kt, int buf) {
#pragma unroll
    for (int pw = 0; pw < 2; ++pw) {
      const int piece = wave * 2 + pw;
      if constexpr (!ONE)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rK, (att_lds_void*)(sRing[buf][0] + piece * 8 * ATT_D), 16, kro[pw],
                                                 kt * kstep, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rK, (att_lds_void*)(sRing[buf][NIMG - 2] + piece * 8 * ATT_D), 16,
                                               kto[pw], kt * kstep, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rV, (att_lds_void*)(sRing[buf][NIMG - 1] + piece * 8 * ATT_D), 16,
                                               vro[pw], kt * vstep, 0, 0);
    }
  };
  for (int t = 0; t < STG - 1 && t < nkt; ++t) issue(t, t);
  // the tile loop unrolled by the ring depth: every LDS fragment address is a lane base + an immediate
  auto tile = [&](auto BUF_, int kt) {
    constexpr int buf = decltype(BUF_)::value;
    // tile kt landed (all but this wave's PIECES youngest), then every wave's; the barrier also orders every wave's
    // reads of tile kt-1 before its buffer is re-staged below
    att_wait_barrier<PIECES>(min(STG - 2, nkt - 1 - kt));
    if (kt + STG - 1 < nkt) issue(kt + STG - 1, (buf + STG - 1) % STG);
    const bf16_t* sKt = sRing[buf][NIMG - 2];
    const bf16_t* sKr = ONE ? sKt : sRing[buf][0];
    const bf16_t* sVr = sRing[buf][NIMG - 1];
    const int kbase = kt * ATT_KT;
    // the tile body in two straight-line forms: the key mask of a partial last tile is decided once per tile, not
    // per (key block, query block) -- a branch there splits the body into 16 blocks the scheduler cannot interleave
    auto body = [&](auto KPART_) {
    constexpr bool kpart = decltype(KPART_)::value;
    f32x4 dsT[2][4];  // lane holds dS[q = qi*16 + c][key = kj*16 + 4g + r]
#pragma unroll
    for (int kj = 0; kj < 4; ++kj) {
      bf16x8 kf[2], vf[2];
#pragma unroll
      for (int ds = 0; ds < 2; ++ds) {
        kf[ds] = *reinterpret_cast<const bf16x8*>(sKr + (ONE ? swz_tr(kj * 16 + c, ds * 4 + g) : swz_row(kj * 16 + c, ds * 4 + g)));
        vf[ds] = *reinterpret_cast<const bf16x8*>(sVr + swz_row(kj * 16 + c, ds * 4 + g));
      }
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) {
        // dP^T accumulates onto -delta of this lane's query (one VALU op per score less)
        f32x4 sacc = {0.f, 0.f, 0.f, 0.f}, pacc = {-dl[qi], -dl[qi], -dl[qi], -dl[qi]};
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[0], qf[qi][0], sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[1], qf[qi][1], sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[0], of[qi][0], pacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[1], of[qi][1], pacc, 0, 0, 0);
        if constexpr (kpart) {  // last, partial key tile only: padded keys get p = 0
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kbase + kj * 16 + 4 * g + r;
            const float p = key < a.Sk ? fast_exp2(fmaf(sacc[r], a.scale_log2, -lq[qi])) : 0.f;
            dsT[qi][kj][r] = p * pacc[r];
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) dsT[qi][kj][r] = fast_exp2(fmaf(sacc[r], a.scale_log2, -lq[qi])) * pacc[r];
        }
      }
    }
    // K^T fragments by inline-asm transposed reads: the builtin form makes hipcc drain the LDS-DMA ring (vmcnt(0),
    // the next two key tiles included) before them on every tile
    s16x4 kr[2][8];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        kr[ks][2 * dt] = tr_read_asm(sKt, (2 * ks) * 16 + 4 * g, dt * 16, lane);
        kr[ks][2 * dt + 1] = tr_read_asm(sKt, (2 * ks + 1) * 16 + 4 * g, dt * 16, lane);
      }
    bf16x8 pf[2][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) pf[ks][qi] = pack_p(dsT[qi][2 * ks], dsT[qi][2 * ks + 1]);
    lds_wait8(kr[0]);
    lds_wait8(kr[1]);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 kf = cat_frag(kr[ks][2 * dt], kr[ks][2 * dt + 1]);
#pragma unroll
        for (int qi = 0; qi < 2; ++qi)
          dq[qi][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, pf[ks][qi], dq[qi][dt], 0, 0, 0);
      }
    }
    };
    if (kbase + ATT_KT > a.Sk) body(std::true_type{});  // wave-uniform
    else body(std::false_type{});
  };
  for (int kt = 0; kt < nkt; kt += STG) {
    tile(ic<0>{}, kt);
    if (kt + 1 < nkt) tile(ic<1>{}, kt + 1);
    if (kt + 2 < nkt) tile(ic<2>{}, kt + 2);
    if constexpr (STG > 3)
      if (kt + 3 < nkt) tile(ic<3>{}, kt + 3);
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

// dst[r][c] = bf16( sum_s src[s][r][c] ) : the query-split partials of the cross-attention dK (blockIdx.y = 0) and
// dV (blockIdx.y = 1) in one launch
__global__ void reduce_splits_kernel(long rows, int cols, int nsplit, const float* __restrict__ src_k,
                                     const float* __restrict__ src_v, long split_stride, bf16_t* __restrict__ dst_k,
                                     long ldd_k, bf16_t* __restrict__ dst_v, long ldd_v) {
  const float* __restrict__ src = blockIdx.y ? src_v : src_k;
  bf16_t* __restrict__ dst = blockIdx.y ? dst_v : dst_k;
  const long ldd = blockIdx.y ? ldd_v : ldd_k;
  const int c4 = cols / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < rows * c4; i += (long)gridDim.x * blockDim.x) {
    const long r = i / c4;
    const int cc = (int)(i - r * c4) * 4;
    float4 acc = *reinterpret_cast<const float4*>(src + r * cols + cc);
    for (int sp = 1; sp < nsplit; ++sp) {
      const float4 v = *reinterpret_cast<const float4*>(src + sp * split_stride + r * cols + cc);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    *reinterpret_cast<uint2*>(dst + r * ldd + cc) = make_uint2(pack2bf(acc.x, acc.y), pack2bf(acc.z, acc.w));
  }
}

// benchmark knobs (tools build only; compile-time zeros in the product library, whose dispatch is the default forms)
#ifdef PSO_BENCH_KNOBS
static int g_attn_fwd_variant = 0;
static bool g_attn_vsum = false;
static int g_attn_bwd_variant = 0;  // benchmark knob (the tens digit of pso_attention_set_variant): see pso_attention_bwd
static bool g_attn_pp_trace = false;  // the ping-pong dK/dV form records segment clocks (diagnostic)
static int g_attn_xqs = 0;  // query splits of the short-KV backward (0 = automatic)
#else
static constexpr int g_attn_fwd_variant = 0, g_attn_bwd_variant = 0, g_attn_xqs = 0;
#endif

// Query splits of the dK/dV sweep when there are few key blocks (cross-attention over the 77 text tokens): enough
// workgroups for ~2 per CU; each split writes its own fp32 partial slice (no atomics).
static int cross_qsplit(int B, int H, int Sq, int Sk) {
  if (Sk > 256) return 1;
  if (Sk <= XK_KP && g_attn_bwd_variant != 7) {  // attn_bwd_x_kernel: at most one round of its 512 co-resident slots
    int qs = g_attn_xqs > 0 ? g_attn_xqs : 512 / (H * B);
    const int nqt = cdiv(Sq, ATT_KT);
    if (qs > nqt) qs = nqt;
    return qs < 1 ? 1 : qs;
  }
  const int nqt = cdiv(Sq, ATT_KT);
  int qs = cdiv(512, (long)cdiv(Sk, 128) * H * B);
  if (qs > nqt) qs = nqt;
  return qs < 1 ? 1 : qs;
}


static bool a16(const void* p, long ld) { return (((uintptr_t)p) & 15) == 0 && (ld % 8) == 0; }

extern "C" {

#ifdef PSO_BENCH_KNOBS
// diagnostic: the segment-start clocks of the last traced ping-pong dK/dV launch (2 x 520, group-major)
int pso_attn_pp_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pp_trace), sizeof(g_pp_trace)) == hipSuccess ? 0 : 1;
}

void pso_attention_set_variant(int v) {
  g_attn_fwd_variant = v % 10;
  g_attn_bwd_variant = (v / 10) % 10;
  g_attn_vsum = (v / 100) % 10 == 1;  // 100+: row sums on the VALU (A/B knob)
  g_attn_pp_trace = (v / 1000) % 10 == 1;
  g_attn_xqs = (v / 10000) % 100;  // 10000 * qs: the short-KV backward's query splits
}
#endif

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
  // 256 queries per workgroup (4 x 64-row waves) when that still gives >= 2 rounds of the 512 co-resident
  // workgroups, else 128 (4 x 32): fewer K/V LDS bytes per MFMA vs. a fuller grid
  const int nq4 = cdiv(Sq, 256), nq2 = cdiv(Sq, 128);
  // cross-attention (77 keys: two key tiles) keeps 128: its per-workgroup set-up outweighs the K/V reuse (-10 %)
  // fwd variant knob (benchmarks / tests): 0 auto, 1 auto with the lane-local growth test (LG), 2 / 4 force 32 / 64
  // rows per wave, +5 (5, 7, 9) the first-round loop
  const int fv = g_attn_fwd_variant;
  const int qsel = fv >= 5 ? fv - 5 : fv;
  const bool big = qsel == 4 || ((qsel == 0 || qsel == 1) && (long)nq4 * H * B >= 1024 && Sk > 128);
  hipStream_t st = (hipStream_t)stream;
#ifdef PSO_BENCH_KNOBS
  if (g_attn_vsum) {
    if (big) attn_fwd_kernel<4, false><<<nq4 * H * B, ATT_THREADS, 0, st>>>(a, nq4);
    else attn_fwd_kernel<2, false><<<nq2 * H * B, ATT_THREADS, 0, st>>>(a, nq2);
    return pso_check_launch("pso_attention_fwd");
  } else if (fv >= 5) {
    if (big) attn_fwd_kernel<4><<<nq4 * H * B, ATT_THREADS, 0, st>>>(a, nq4);
    else attn_fwd_kernel<2><<<nq2 * H * B, ATT_THREADS, 0, st>>>(a, nq2);
    return pso_check_launch("pso_attention_fwd");
  } else if (fv == 1) {  // lane-local growth test (LG)
    if (big) attn_fwd2_kernel<4, true><<<nq4 * H * B, ATT_THREADS, 0, st>>>(a, nq4);
    else attn_fwd2_kernel<2, true><<<nq2 * H * B, ATT_THREADS, 0, st>>>(a, nq2);
    return pso_check_launch("pso_attention_fwd");
  }
#endif
  if (big) {
    attn_fwd2_kernel<4><<<nq4 * H * B, ATT_THREADS, 0, st>>>(a, nq4);
  } else {
    attn_fwd2_kernel<2><<<nq2 * H * B, ATT_THREADS, 0, st>>>(a, nq2);
  }
  return pso_check_launch("pso_attention_fwd");
}

size_t pso_attention_bwd_ws_bytes(int B, int H, int Sq, int Sk) {
  size_t d = (size_t)B * H * Sq * sizeof(float);
  const int qs = cross_qsplit(B, H, Sq, Sk);
  size_t acc = qs > 1 ? 2 * (size_t)qs * B * Sk * H * ATT_D * sizeof(float) : 0;
  return 2 * (((d + 255) / 256) * 256) + acc;  // -delta, LSE * log2(e), split partials
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
  const size_t dsz = (((size_t)B * H * Sq * sizeof(float) + 255) / 256) * 256;
  float* delta = (float*)ws;
  a.delta = delta;
  a.lse2 = (float*)((char*)ws + dsz);
  a.dq = (bf16_t*)dq; a.dk = (bf16_t*)dk; a.dv = (bf16_t*)dv;
  a.lddq = lddq; a.lddk = lddk; a.lddv = lddv; a.sdq_b = sdq_b; a.sdk_b = sdk_b; a.sdv_b = sdv_b;
  const size_t doff = 2 * dsz;
  const int nkb = cdiv(Sk, 128);
  const int qsplit = cross_qsplit(B, H, Sq, Sk);
  const long part = (long)B * Sk * H * ATT_D;  // elements of one split slice
  if (qsplit > 1) {
    a.dk_acc = (float*)((char*)ws + doff);
    a.dv_acc = a.dk_acc + qsplit * part;
  }
  a.q_split = qsplit;
  a.nbatch = B;
  // dQ first: it forms delta = rowsum(dO * O) for its own queries and stores it for the dK/dV sweep (no separate
  // delta pre-pass launch)
  // one LDS image per operand (ONE) by default: bit-identical to the two-image form (bwd variant 3, A/B knob) and
  // 3-5 % faster on the self-attention shapes (L1 1.113 vs 1.157 ms, L2 0.168 vs 0.177 ms, medians of 4 alternated
  // runs, profiles/r05_attn_bwd_ab.log); 5 / 6 = ONE with rings of 3 / 4 (no faster)
  const dim3 gq(cdiv(Sq, 128), H, B);
  const bool xpath = Sk <= XK_KP && g_attn_bwd_variant != 7;  // 7: the dQ + dK/dV launches (A/B knob)
  if (xpath) {  // short key sequences (cross-attention): dQ, dK and dV in one pass over the query tiles
    attn_bwd_x_kernel<<<dim3(qsplit * H * B), ATT_THREADS, 0, st>>>(a);
  } else {
#ifdef PSO_BENCH_KNOBS
  const int bv = g_attn_bwd_variant;
  if (bv == 3 || bv == 1) attn_bwd_dq_kernel<3, false><<<gq, ATT_THREADS, 0, st>>>(a);
  else if (bv == 6) attn_bwd_dq_kernel<4, true><<<gq, ATT_THREADS, 0, st>>>(a);
  else attn_bwd_dq_kernel<3, true><<<gq, ATT_THREADS, 0, st>>>(a);
  // keys per wave: 32 (2 x 16, 128 keys per workgroup, 2 workgroups per CU); 64 on request (benchmark knob)
  const int nkb4 = cdiv(Sk, 256);
  const bool kj4 = g_attn_bwd_variant == 4;  // measured slower on every UNet shape (1 wave/SIMD, AGPR spills)
  if (kj4) {
    const size_t shm = 3 * (4 * ATT_KT * ATT_D * sizeof(bf16_t) + 2 * 64 * sizeof(float));
    static bool attr4 = false;
    if (!attr4) {
      (void)hipFuncSetAttribute((const void*)attn_bwd_dkv_kernel<4, 3>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)shm);
      attr4 = true;
    }
    attn_bwd_dkv_kernel<4, 3><<<nkb4 * qsplit * H * B, ATT_THREADS, shm, st>>>(a, nkb4);
  } else if ((bv == 8 || bv == 9) && qsplit == 1) {
    // ping-pong form (A/B knob, bit-identical; measured no faster: DESIGN §9): 8 waves, 256 keys per workgroup;
    // 9: A segments at raised priority; the 1000s digit of the variant traces segment clocks
    constexpr int PST = 4;
    const size_t shm = PST * (2 * ATT_KT * ATT_D * sizeof(bf16_t) + 2 * 64 * sizeof(float));
    static bool attr8 = false;
    if (!attr8) {
      (void)hipFuncSetAttribute((const void*)attn_bwd_dkv_pp_kernel<PST>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)shm);
      (void)hipFuncSetAttribute((const void*)attn_bwd_dkv_pp_kernel<PST, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
      (void)hipFuncSetAttribute((const void*)attn_bwd_dkv_pp_kernel<PST, false, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
      attr8 = true;
    }
    const dim3 gk(nkb4 * H * B);
    if (g_attn_pp_trace) attn_bwd_dkv_pp_kernel<PST, false, true><<<gk, 512, shm, st>>>(a, nkb4);
    else if (bv == 9) attn_bwd_dkv_pp_kernel<PST, true><<<gk, 512, shm, st>>>(a, nkb4);
    else attn_bwd_dkv_pp_kernel<PST><<<gk, 512, shm, st>>>(a, nkb4);
  } else if (bv != 1 && bv != 3) {  // ONE: Q / dO once per stage (swz_tr image for row and transposed reads)
    const int stg = bv == 5 ? 3 : (bv == 6 ? 4 : 2);
    const size_t shm = stg * (2 * ATT_KT * ATT_D * sizeof(bf16_t) + 2 * 64 * sizeof(float));
    static bool attr1 = false;
    if (!attr1) {
      (void)hipFuncSetAttribute((const void*)attn_bwd_dkv_kernel<2, 3, true, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)(3 * shm / stg));
      (void)hipFuncSetAttribute((const void*)attn_bwd_dkv_kernel<2, 4, true, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)(4 * shm / stg));
      attr1 = true;
    }
    const dim3 gk(nkb * qsplit * H * B);
    if (stg == 3) attn_bwd_dkv_kernel<2, 3, true, true><<<gk, ATT_THREADS, shm, st>>>(a, nkb);
    else if (stg == 4) attn_bwd_dkv_kernel<2, 4, true, true><<<gk, ATT_THREADS, shm, st>>>(a, nkb);
    else attn_bwd_dkv_kernel<2, 2, true, true><<<gk, ATT_THREADS, shm, st>>>(a, nkb);
  } else if (g_attn_bwd_variant == 1) {  // per-subtile LSE / delta reads (the round-3 form, A/B knob)
    const size_t shm = 2 * (4 * ATT_KT * ATT_D * sizeof(bf16_t) + 2 * 64 * sizeof(float));
    attn_bwd_dkv_kernel<2, 2><<<nkb * qsplit * H * B, ATT_THREADS, shm, st>>>(a, nkb);
  } else {  // two images per operand (variant 3): tile-level LSE / delta prefetch
    const size_t shm = 2 * (4 * ATT_KT * ATT_D * sizeof(bf16_t) + 2 * 64 * sizeof(float));
    attn_bwd_dkv_kernel<2, 2, true><<<nkb * qsplit * H * B, ATT_THREADS, shm, st>>>(a, nkb);
  }
#else
  attn_bwd_dq_kernel<3, true><<<gq, ATT_THREADS, 0, st>>>(a);
  {  // ONE: Q / dO once per stage (swz_tr image for row and transposed reads), 2-stage ring
    const size_t shm = 2 * (2 * ATT_KT * ATT_D * sizeof(bf16_t) + 2 * 64 * sizeof(float));
    attn_bwd_dkv_kernel<2, 2, true, true><<<dim3(nkb * qsplit * H * B), ATT_THREADS, shm, st>>>(a, nkb);
  }
#endif
  }
  if (qsplit > 1) {
    // dk/dv outputs are [B][Sk] rows of H*64 with row stride lddk (batch stride must be Sk*lddk)
    const long rows = (long)B * Sk;
    const int cols = H * ATT_D;
    const int nb = cdiv(rows * cols / 4, 256) > 2048 ? 2048 : cdiv(rows * cols / 4, 256);
    reduce_splits_kernel<<<dim3(nb, 2), 256, 0, st>>>(rows, cols, qsplit, a.dk_acc, a.dv_acc, part, (bf16_t*)dk, lddk,
                                                      (bf16_t*)dv, lddv);
  }
  return pso_check_launch("pso_attention_bwd");
}

}  // extern "C"
