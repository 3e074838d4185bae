// Rank-r TN GEMM for gfx950: the LoRA weight gradients of the SDXL UNet.
//
//   D[c][j] = alpha * sum_m X[m][c] * U[m][j]      X: [M][C] (C >= 128, the activation / output gradient stream)
//                                                  U: [M][R] (R = 16*NJT = 16 / 32 / 64 / 96, the rank-r projection)
// accumulated into out[c][j] (dB = s dY^T u) or out[j][c] (dA = v^T x): either with f32 atomics (pso_gemm_tn_rank_batch)
// or -- the training path -- deterministically: every workgroup stores its 128 x R partial into a caller-owned
// workspace and a second kernel adds the partials of each column block in row-range order (pso_gemm_tn_rank_batch_ws),
// so two runs (and a hipGraph replay) give the same bits, as cuBLAS's fixed-order dW GEMMs do in the reference.  Replaces the reduction over the
// B*S tokens inside peft's lora_A / lora_B weight gradients (`T:857` backward through `T:338-345`).
//
// The product is an HBM stream of X (2 FLOP per byte at R = 32).  Every 4-wave workgroup owns 128 columns of X and a
// contiguous range of rows; 64-row steps of X (two 64 x 64 transposed-read images) and U (one or two images) go
// global -> LDS directly (global_load_lds_dwordx4, source-side swizzle chunk ^ 2*((row >> 1) & 3)) through a 3-stage
// ring with two steps in flight behind a counted vmcnt and one s_barrier per step.  Both MFMA operands are read
// with ds_read_b64_tr_b16 (rows permuted identically inside each 32-deep step).  Rows past M load from a zero page.
// `group_c` > 0: the U columns used by X column c start at (c / group_c) * R (the fused q/k/v adapters: dqkv columns
// [jC, (j+1)C) pair with u_qkv columns [j r, (j+1) r)).
#include "common.h"

namespace {

typedef __attribute__((address_space(3))) void tnr_lds_void;
typedef __attribute__((address_space(3))) s16x4 tnr_lds_s16x4;
__device__ __attribute__((aligned(16))) uint4 g_tnr_zero[4];

constexpr int TNR_IMG = 64 * 64;  // one 64-row x 64-column bf16 image

__device__ __forceinline__ int tnr_swz(int r, int c) { return r * 64 + ((c ^ (((r >> 1) & 3) << 1)) << 3); }

// lane i of each 16-lane group: column col0 + i of rows r0 .. r0+3 (r0 per group)
__device__ __forceinline__ s16x4 tnr_tr(const bf16_t* img, int r0, int col0, int lane) {
  const int li = lane & 15;
  const int q = li >> 2, p = li & 3;
  const int col = col0 + 4 * p;
  // inline asm: the builtin form is an LDS read the waitcnt pass cannot separate from the ring's pending LDS-DMA
  // writes, so hipcc drains the whole ring (vmcnt(0)) before it.  The caller waits lgkmcnt itself.
  const unsigned addr = (unsigned)(uintptr_t)(const tnr_lds_void*)(img + tnr_swz(r0 + q, col >> 3) + (col & 7));
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ bf16x8 tnr_frag(const bf16_t* img, int m0, int col0, int lane) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  const int g = lane >> 4;
  const s16x4 a = tnr_tr(img, m0 + 4 * g, col0, lane), b = tnr_tr(img, m0 + 16 + 4 * g, col0, lane);
  s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Batched form: one launch runs many independent products (the LoRA dA / dB of every adapter of a gradient unit,
// deferred until the unit's backward is done).  The problem table travels in the kernel arguments; workgroup b runs
// problem p with blk0[p] <= b < blk0[p + 1] (a scalar scan over <= TNR_MAXP entries read straight from the kernarg
// segment), so a small product no longer pays a launch, a ramp and a tail of its own.
constexpr int TNR_MAXP = 32;
struct TnrProb {
  const bf16_t* x; long ldx;
  const bf16_t* u; long ldu;
  float* out; long ldo;
  int M, C, group_c, spb;
  float alpha; int blk0;
  int rblk0;  // first block of this problem in the ordered-reduction launch (workspace form)
};
struct TnrBatch {
  int count, nblk, nrblk;
  TnrProb p[TNR_MAXP];
};

template <int NJT, bool OUT_JC, bool WS>
__global__ __launch_bounds__(256, NJT == 6 ? 1 : 2) void gemm_tn_rank_kernel(TnrBatch bt, float4* __restrict__ ws) {
  int pi = 0;
  for (int q = 1; q < bt.count; ++q)
    if ((int)blockIdx.x >= bt.p[q].blk0) pi = q;
  const TnrProb& pr_ = bt.p[pi];
  const int M = pr_.M, C = pr_.C, group_c = pr_.group_c, steps_per_block = pr_.spb;
  const bf16_t* __restrict__ X = pr_.x;
  const bf16_t* __restrict__ U = pr_.u;
  float* __restrict__ out = pr_.out;
  const long ldx = pr_.ldx, ldu = pr_.ldu, ldo = pr_.ldo;
  const float alpha = pr_.alpha;
  const int lblk = (int)blockIdx.x - pr_.blk0;
  constexpr int R = 16 * NJT;
  constexpr int UIMG = (R + 63) / 64;
  constexpr int STG = 3;
  constexpr int STAGE = (2 + UIMG) * TNR_IMG;
  constexpr int PIECES = 2 * 2 + (UIMG * 8 + 3) / 4;  // X: 16 pieces / 4 waves; U: 8 per image
  __shared__ __attribute__((aligned(16))) bf16_t lds[STG * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, cl = lane & 15;
  const int ncb = C / 128;
  const int cb = lblk % ncb, mb = lblk / ncb;
  const int c0 = cb * 128;
  const int u_off = group_c > 0 ? (c0 / group_c) * R : 0;
  const int nsteps_all = (M + 63) / 64;
  const int s_beg = mb * steps_per_block;
  const int s_end = min(nsteps_all, s_beg + steps_per_block);
  const int n = s_end > s_beg ? s_end - s_beg : 0;

  const int prow = lane >> 3, pch = lane & 7;
  const int lc = pch ^ (2 * ((prow >> 1) & 3));  // logical source chunk of this lane's physical chunk
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_tnr_zero);
  // Per-lane constant parts of the sources.  U padding columns (col >= R) read the zero chunk at row stride 0, so
  // a full 64-row step issues its pieces with no per-lane predicate: exec-masked loads would make hipcc wrap every
  // glds in a branch and drain the ring with vmcnt(0) before the LDS reads.  Only the ragged last step (M % 64)
  // takes the predicated path.
  static_assert((UIMG * 8) % 4 == 0, "U pieces split evenly over the 4 waves");
  const bf16_t* xsrc[4];
  int xdst[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;
    const int xi = piece >> 3, pr = piece & 7;
    xsrc[i] = X + (long)(pr * 8 + prow) * ldx + c0 + xi * 64 + lc * 8;
    xdst[i] = xi * TNR_IMG + pr * 8 * 64;
  }
  constexpr int UP = UIMG * 8 / 4;
  const bf16_t* usrc[UP];
  long ustr[UP];
  int udst[UP], urow[UP];
#pragma unroll
  for (int i = 0; i < UP; ++i) {
    const int piece = wave + 4 * i;
    const int ui = piece >> 3, pr = piece & 7;
    const int col = ui * 64 + lc * 8;
    const bool ok = col < R;
    urow[i] = pr * 8 + prow;
    usrc[i] = ok ? U + (long)urow[i] * ldu + u_off + col : zero;
    ustr[i] = ok ? ldu : 0;
    udst[i] = (2 + ui) * TNR_IMG + pr * 8 * 64;
  }
  auto issue = [&](int st, int buf) {
    bf16_t* base = lds + buf * STAGE;
    const long m0 = (long)st * 64;
    if (m0 + 64 <= M) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(xsrc[i] + m0 * ldx), (tnr_lds_void*)(base + xdst[i]),
                                         16, 0, 0);
#pragma unroll
      for (int i = 0; i < UP; ++i)
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(usrc[i] + m0 * ustr[i]),
                                         (tnr_lds_void*)(base + udst[i]), 16, 0, 0);
    } else {  // ragged last step: rows past M read the zero chunk
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int piece = wave * 4 + i;
        const bool ok = m0 + (piece & 7) * 8 + prow < M;
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(ok ? xsrc[i] + m0 * ldx : zero),
                                         (tnr_lds_void*)(base + xdst[i]), 16, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < UP; ++i) {
        const bool ok = m0 + urow[i] < M;
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(ok ? usrc[i] + m0 * ustr[i] : zero),
                                         (tnr_lds_void*)(base + udst[i]), 16, 0, 0);
      }
    }
  };

  f32x4 acc[2][NJT];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int j = 0; j < NJT; ++j) acc[ci][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (n > 0) issue(s_beg, 0);
  if (n > 1) issue(s_beg + 1, 1);
  for (int i = 0; i < n; ++i) {
    // every wave issues the same number of pieces per step (padding pieces included), so vmcnt counts match
    if (i + 1 < n) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(PIECES) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (i + 2 < n) issue(s_beg + i + 2, (i + 2) % STG);
    const bf16_t* base = lds + (i % STG) * STAGE;
    // wave w owns X columns c0 + 32w .. +32 = image (w >> 1), columns (w & 1) * 32 ..
    const bf16_t* ximg = base + (wave >> 1) * TNR_IMG;
    const int xcol = (wave & 1) * 32;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 xf[2], uf[NJT];
#pragma unroll
      for (int ci = 0; ci < 2; ++ci) xf[ci] = tnr_frag(ximg, ks * 32, xcol + ci * 16, lane);
#pragma unroll
      for (int j = 0; j < NJT; ++j) uf[j] = tnr_frag(base + (2 + (j >> 2)) * TNR_IMG, ks * 32, (j & 3) * 16, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs behind the wait (hipcc moves register-only ops past asm)
#pragma unroll
      for (int ci = 0; ci < 2; ++ci)
#pragma unroll
        for (int j = 0; j < NJT; ++j) {
          if (OUT_JC)  // lane holds D^T[j = 16j' + 4g + r][c = 16ci + cl]: consecutive lanes -> consecutive c
            acc[ci][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(uf[j], xf[ci], acc[ci][j], 0, 0, 0);
          else  // lane holds D[c = 16ci + 4g + r][j = 16j' + cl]
            acc[ci][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[ci], uf[j], acc[ci][j], 0, 0, 0);
        }
    }
  }
  if constexpr (WS) {
    // partial of this workgroup: 2*NJT float4 slots per thread, slot-major so every store is one coalesced 4 KB row
    float4* dst = ws + (size_t)blockIdx.x * (2 * NJT * 256) + tid;
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
      for (int j = 0; j < NJT; ++j)
        dst[(ci * NJT + j) * 256] = make_float4(acc[ci][j][0], acc[ci][j][1], acc[ci][j][2], acc[ci][j][3]);
    return;
  }
  if (n == 0) return;
  const int cw = c0 + wave * 32;
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int j = 0; j < NJT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (OUT_JC) atomicAdd(out + (long)(j * 16 + 4 * g + r) * ldo + cw + ci * 16 + cl, acc[ci][j][r] * alpha);
        else atomicAdd(out + (long)(cw + ci * 16 + 4 * g + r) * ldo + j * 16 + cl, acc[ci][j][r] * alpha);
      }
}

// Ordered reduction of the workspace partials: thread t of column block cb of problem p owns float4 slot s of the
// partial tile (the same (slot, thread) position every workgroup of that column block stored) and adds the partials
// of the row ranges mb = 0, 1, ... in that order, then out += alpha * sum at the positions the atomic epilogue would
// have used.  One thread per float4 slot: 2*NJT*256 threads per column block.
template <int NJT, bool OUT_JC>
__global__ __launch_bounds__(256) void tn_rank_reduce_kernel(TnrBatch bt, const float4* __restrict__ ws) {
  constexpr int SLOTS = 2 * NJT;
  const int gblk = blockIdx.x;  // one 256-thread block per (problem, column block, slot)
  int pi = 0;
  for (int q = 1; q < bt.count; ++q)
    if (gblk >= bt.p[q].rblk0) pi = q;
  const TnrProb& pr = bt.p[pi];
  const int ncb = pr.C / 128;
  const int l = gblk - pr.rblk0;
  const int cb = l / SLOTS, slot = l - cb * SLOTS;
  const int ci = slot / NJT, j = slot - ci * NJT;
  const int nmb = (((pr.M + 63) / 64) + pr.spb - 1) / pr.spb;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, cl = lane & 15;
  const float4* src = ws + (size_t)(pr.blk0 + cb) * (SLOTS * 256) + slot * 256 + tid;
  float4 s = src[0];
  for (int mb = 1; mb < nmb; ++mb) {
    const float4 v = src[(size_t)mb * ncb * (SLOTS * 256)];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const float a[4] = {s.x, s.y, s.z, s.w};
  const int cw = cb * 128 + wave * 32;
  float* out = pr.out;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float* o = OUT_JC ? out + (long)(j * 16 + 4 * g + r) * pr.ldo + cw + ci * 16 + cl
                      : out + (long)(cw + ci * 16 + 4 * g + r) * pr.ldo + j * 16 + cl;
    *o += a[r] * pr.alpha;
  }
}

template <int NJT>
int launch_tnr_batch(TnrBatch& bt, bool out_jc, hipStream_t st, float4* ws = nullptr) {
  if (bt.count == 0) return PSO_OK;
  if (ws) {
    if (out_jc) {
      pso_note_kernel("gemm_tn_rank_kernel<%d, true, true>", NJT);
      gemm_tn_rank_kernel<NJT, true, true><<<bt.nblk, 256, 0, st>>>(bt, ws);
      tn_rank_reduce_kernel<NJT, true><<<bt.nrblk, 256, 0, st>>>(bt, ws);
    } else {
      pso_note_kernel("gemm_tn_rank_kernel<%d, false, true>", NJT);
      gemm_tn_rank_kernel<NJT, false, true><<<bt.nblk, 256, 0, st>>>(bt, ws);
      tn_rank_reduce_kernel<NJT, false><<<bt.nrblk, 256, 0, st>>>(bt, ws);
    }
    return pso_check_launch("pso_gemm_tn_rank_batch_ws");
  }
  if (out_jc) {
    pso_note_kernel("gemm_tn_rank_kernel<%d, true, false>", NJT);
    gemm_tn_rank_kernel<NJT, true, false><<<bt.nblk, 256, 0, st>>>(bt, nullptr);
  } else {
    pso_note_kernel("gemm_tn_rank_kernel<%d, false, false>", NJT);
    gemm_tn_rank_kernel<NJT, false, false><<<bt.nblk, 256, 0, st>>>(bt, nullptr);
  }
  return pso_check_launch("pso_gemm_tn(rank)");
}

// Row-steps per workgroup.  Each workgroup adds its 128 x R partial into the f32 output with atomics
// (128 * R * 4 bytes at the chip's ~1.3 TB/s atomic rate, MI355X_MICROARCH.md "Global float atomics") after
// streaming spb * 64 rows of X (spb * 16 KB at ~6 TB/s): spb >= R / 4 keeps the atomics near a tenth of the stream.
// Alone (one product per launch) the split is finer -- ~2 workgroups per CU -- and at least 3 steps (two in flight
// behind the one being multiplied).
static int tnr_spb(int M, int C, int R, bool batched) {
  const int ncb = C / 128, nsteps = (M + 63) / 64;
  int spb;
  if (batched) {
    spb = R / 4;
  } else {
    const int nmb = (512 + ncb - 1) / ncb;
    spb = (nsteps + nmb - 1) / nmb;
  }
  if (spb < 3) spb = 3;
  if (spb > nsteps) spb = nsteps;
  return spb < 1 ? 1 : spb;
}

template <int NJT>
int launch_tnr(int M, int C, const bf16_t* X, long ldx, const bf16_t* U, long ldu, int group_c, float alpha, float* out,
               long ldo, bool out_jc, hipStream_t st) {
  TnrBatch bt{};
  const int spb = tnr_spb(M, C, 16 * NJT, false);
  bt.count = 1;
  bt.p[0] = TnrProb{X, ldx, U, ldu, out, ldo, M, C, group_c, spb, alpha, 0, 0};
  bt.nblk = (C / 128) * ((((M + 63) / 64) + spb - 1) / spb);
  return launch_tnr_batch<NJT>(bt, out_jc, st);
}

}  // namespace

// host entry used by pso_gemm_tn (gemm.hip) when one side is a rank-r projection: C % 128 == 0, R in {32, 64, 96},
// 16-B aligned rows (checked there).
int pso_gemm_tn_rank(int M, int C, const void* X, long ldx, const void* U, long ldu, int R, int group_c, float alpha,
                     float* out, long ldo, int out_jc, hipStream_t st) {
  auto x = (const bf16_t*)X;
  auto u = (const bf16_t*)U;
  switch (R) {
    case 16: return launch_tnr<1>(M, C, x, ldx, u, ldu, group_c, alpha, out, ldo, out_jc, st);
    case 32: return launch_tnr<2>(M, C, x, ldx, u, ldu, group_c, alpha, out, ldo, out_jc, st);
    case 64: return launch_tnr<4>(M, C, x, ldx, u, ldu, group_c, alpha, out, ldo, out_jc, st);
    case 96: return launch_tnr<6>(M, C, x, ldx, u, ldu, group_c, alpha, out, ldo, out_jc, st);
    default: pso_set_error("pso_gemm_tn(rank): R must be 16, 32, 64 or 96"); return PSO_ERR_ARG;
  }
}

// Batched entries (pso_amd.h pso_gemm_tn_rank_batch / _ws): count products of one rank R and one orientation, in
// chunks of TNR_MAXP per launch.  A chunk never holds two products whose outputs overlap (the ordered reduction
// writes out with plain read-modify-writes), and its workspace need is nblk * 128 * R floats.
namespace {
bool tnr_overlap(const PsoTnRankProblem& a, const PsoTnRankProblem& b, int R, int out_jc) {
  auto span = [&](const PsoTnRankProblem& q, uintptr_t& lo, uintptr_t& hi) {
    const long rows = out_jc ? R : q.C, cols = out_jc ? q.C : R;
    lo = (uintptr_t)q.out;
    hi = (uintptr_t)(q.out + (rows - 1) * q.ldo + cols);
  };
  uintptr_t a0, a1, b0, b1;
  span(a, a0, a1);
  span(b, b0, b1);
  return a0 < b1 && b0 < a1;
}

// Fill the next chunk starting at probs[i]; returns the index after it.
int tnr_chunk(TnrBatch& bt, int R, int out_jc, int count, const PsoTnRankProblem* probs, int i) {
  bt = TnrBatch{};
  int nblk = 0, nrblk = 0;
  const int first = i;
  for (; i < count && bt.count < TNR_MAXP; ++i) {
    const PsoTnRankProblem& q = probs[i];
    if (q.M == 0) continue;
    bool clash = false;
    for (int k = first; k < i && !clash; ++k)
      clash = probs[k].M != 0 && tnr_overlap(probs[k], q, R, out_jc);
    if (clash) break;
    const int spb = tnr_spb(q.M, q.C, R, true);
    const int nb = (q.C / 128) * ((((q.M + 63) / 64) + spb - 1) / spb);
    bt.p[bt.count++] = TnrProb{(const bf16_t*)q.x, q.ldx, (const bf16_t*)q.u, q.ldu, q.out, q.ldo, q.M, q.C,
                               q.group_c, spb, q.alpha, nblk, nrblk};
    nblk += nb;
    nrblk += (q.C / 128) * 2 * (R / 16);
  }
  bt.nblk = nblk;
  bt.nrblk = nrblk;
  return i;
}

int tnr_check(int R, int count, const PsoTnRankProblem* probs, const char* fn) {
  PSO_ARG_CHECK(R == 16 || R == 32 || R == 64 || R == 96, "%s: R must be 16, 32, 64 or 96 (R=%d)", fn, R);
  PSO_ARG_CHECK(count >= 0 && (count == 0 || probs), "%s: bad problem list", fn);
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  for (int i = 0; i < count; ++i) {
    const PsoTnRankProblem& q = probs[i];
    PSO_ARG_CHECK(q.x && q.u && q.out && q.M >= 0 && q.C > 0 && (q.C % 128) == 0,
                  "%s: problem %d: need C %% 128 == 0 and non-null operands", fn, i);
    PSO_ARG_CHECK(al16(q.x) && al16(q.u) && (q.ldx % 8) == 0 && (q.ldu % 8) == 0,
                  "%s: problem %d: X / U need 16-B aligned rows", fn, i);
    PSO_ARG_CHECK(q.group_c == 0 || ((q.group_c % 128) == 0 && (q.C % q.group_c) == 0),
                  "%s: problem %d: group_c must divide C in multiples of 128", fn, i);
  }
  return PSO_OK;
}

int tnr_run(int R, int out_jc, TnrBatch& bt, hipStream_t st, float4* ws) {
  switch (R) {
    case 16: return launch_tnr_batch<1>(bt, out_jc != 0, st, ws);
    case 32: return launch_tnr_batch<2>(bt, out_jc != 0, st, ws);
    case 64: return launch_tnr_batch<4>(bt, out_jc != 0, st, ws);
    default: return launch_tnr_batch<6>(bt, out_jc != 0, st, ws);
  }
}
}  // namespace

extern "C" int pso_gemm_tn_rank_batch(int R, int out_jc, int count, const PsoTnRankProblem* probs, void* stream) {
  int rc = tnr_check(R, count, probs, "pso_gemm_tn_rank_batch");
  if (rc != PSO_OK) return rc;
  const hipStream_t st = (hipStream_t)stream;
  int i = 0;
  while (i < count) {
    TnrBatch bt;
    i = tnr_chunk(bt, R, out_jc, count, probs, i);
    if ((rc = tnr_run(R, out_jc, bt, st, nullptr)) != PSO_OK) return rc;
  }
  return PSO_OK;
}

extern "C" size_t pso_gemm_tn_rank_batch_ws_bytes(int R, int out_jc, int count, const PsoTnRankProblem* probs) {
  if (tnr_check(R, count, probs, "pso_gemm_tn_rank_batch_ws_bytes") != PSO_OK) return 0;
  size_t need = 0;
  int i = 0;
  while (i < count) {
    TnrBatch bt;
    i = tnr_chunk(bt, R, out_jc, count, probs, i);
    const size_t b = (size_t)bt.nblk * 128 * R * sizeof(float);
    if (b > need) need = b;
  }
  return need;
}

extern "C" int pso_gemm_tn_rank_batch_ws(int R, int out_jc, int count, const PsoTnRankProblem* probs, void* ws,
                                         size_t ws_bytes, void* stream) {
  int rc = tnr_check(R, count, probs, "pso_gemm_tn_rank_batch_ws");
  if (rc != PSO_OK) return rc;
  PSO_ARG_CHECK(count == 0 || (ws && ((uintptr_t)ws & 15) == 0), "pso_gemm_tn_rank_batch_ws: need a 16-B aligned ws");
  const hipStream_t st = (hipStream_t)stream;
  int i = 0;
  while (i < count) {  // chunks run in stream order and reuse the one workspace
    TnrBatch bt;
    i = tnr_chunk(bt, R, out_jc, count, probs, i);
    PSO_ARG_CHECK((size_t)bt.nblk * 128 * R * sizeof(float) <= ws_bytes,
                  "pso_gemm_tn_rank_batch_ws: workspace of %zu bytes is too small (need %zu)", ws_bytes,
                  (size_t)bt.nblk * 128 * R * sizeof(float));
    if ((rc = tnr_run(R, out_jc, bt, st, (float4*)ws)) != PSO_OK) return rc;
  }
  return PSO_OK;
}
