// bf16 MFMA GEMM / implicit-GEMM convolution for gfx950 (CDNA4), fp32 accumulate.
//
//   out[M][N] = epilogue( alpha * ( A1[M][K1] . B1[N][K1]^T  +  A2[M][K2] . B2[N][K2]^T ) )
//   epilogue  = + bias[N] + rowbias[m / rows_per_group][N] + resid[M][N]   -> bf16 | f32 | f32 accumulate
//
// Replaces the implicit cuBLAS GEMMs (every nn.Linear of the SDXL UNet / VAE and the peft LoRA product, SURVEY §2
// "cuBLAS GEMM") and the cuDNN conv2d (SURVEY §2 "cuDNN conv2d"): the conv is an implicit GEMM whose A operand is
// gathered on the fly from an NHWC image (M = B*Ho*Wo pixels, K = kh*kw*Cin), with three gather modes:
//   NORMAL  iy = oy*S + kh - P        (conv 3x3/1x1, stride 1 or 2)
//   UP2     iy = (oy + kh - P) >> 1   (nearest 2x upsample fused into the following conv, diffusers Upsample2D)
//   T2      iy = (oy + P - kh) / 2    (transposed stride-2 conv: input-gradient of the Downsample2D conv)
// and an optional second channel source (torch.cat([h, skip], dim=1) of the up blocks, fused into the gather).
// The second (A2, B2) operand pair is the LoRA up-projection fused as a K-tail: y = x W^T + (x A^T)(s B)^T.
//
// Tiling: 256 threads = 4 waves (2 x 2), block tile BM x BN x 64, wave tile (BM/2) x (BN/2) built from
// v_mfma_f32_16x16x32_bf16.  Operands are staged global -> VGPR -> LDS (double buffered, one barrier per K-tile) with
// an XOR swizzle (chunk ^ (row & 7)) that makes both the ds_write_b128 and the ds_read_b128 fragment reads
// conflict-free on 128-B rows.  The MFMA is issued with the B (weight) fragment first so that every lane ends up
// holding 4 consecutive output columns of one row -> 8-B / 16-B vector epilogue stores.
#include "common.h"

#include <cstdlib>

#define GEMM_THREADS 256
#define BK 64

struct ConvGeom {
  int mode;      // 0 = dense A, else PSO_CONV_* gather
  const bf16_t* src2;  // second channel source (concat) or null
  int C1, C2;    // channels of src1 (A1) and src2
  int H, W;      // input spatial size (source grid)
  int Ho, Wo;    // output spatial size
  int ks, stride, pad;
};

struct GemmArgs {
  const bf16_t* a1; long lda1; int K1;
  const bf16_t* b1; long ldb1;
  const bf16_t* a2; long lda2; int K2;
  const bf16_t* b2; long ldb2;
  int tail_group_n;  // >0: the A2 tail of output columns [j*G, (j+1)*G) starts at A2 column j*K2
  int tail_m;        // rows >= tail_m get no A2 tail (policy + reference images in one pass: LoRA on the first rows)
  int M, N;
  ConvGeom conv;
  float alpha;
  const bf16_t* bias;
  const bf16_t* rowbias; long ld_rowbias; int rows_per_group;
  const bf16_t* resid; long ldr;
  void* out; long ldo; int out_dtype; int accumulate;
  int vec_ok;  // 4-wide epilogue vectors are aligned
  int stage_epi;  // bf16 EPI_NONE epilogue staged through LDS: 16-B coalesced residual loads / output stores
  int group_m;  // tile rows per raster group (>= 1)
  // GEGLU epilogues (diffusers GEGLU: [h | gate] = x W^T + b, out = h * gelu(gate)), weight rows interleaved per 64
  // columns as [h 32 | gate 32]:  EPI_GEGLU writes out = h*gelu(gate) (N/2 columns) and, if out2, the interleaved
  // pre-activation;  EPI_GEGLU_BWD takes the GEMM result as dout (N columns), aux = interleaved pre-activation, and
  // writes the interleaved input gradient [dout*gelu(g) | dout*h*gelu'(g)] to out (2N columns).
  void* out2; long ldo2;
  const bf16_t* aux; long ldaux;
  // batched form (gridDim.z = batch, dense A only): operand z starts batch strides further on (elements)
  long bat_a, bat_b, bat_o;
  int batch;
  // deterministic split-K (gridDim.y > 1 with ws): every split STORES its raw partial acc into ws[split][M][N]
  // (fp32, row pitch N); gemm_splitk_reduce_kernel adds the splits in order and applies the epilogue
  float* ws;
};

#define EPI_NONE 0
#define EPI_GEGLU 1
#define EPI_GEGLU_BWD 2

__device__ __forceinline__ int swz(int r, int c) { return r * BK + ((c ^ (r & 7)) << 3); }

template <int BM, int BN, int WAVES>
struct Tile {
  // 8-row x 128-B glds pieces per K-tile (A_P, B_P) and per wave (A_CH, B_CH).  When WAVES does not divide a count
  // (BN = 160 over 8 waves: 20 pieces), wave w takes pieces w, w + WAVES, ... and the waves left short repeat the last
  // piece (same source, same bytes, same LDS slot), so every wave issues the same number of loads: counted vmcnt waits
  // stay uniform.
  static constexpr int A_P = BM / 8, B_P = BN / 8;
  static constexpr int A_CH = (A_P + WAVES - 1) / WAVES;
  static constexpr int B_CH = (B_P + WAVES - 1) / WAVES;
  static constexpr bool A_EVEN = A_P % WAVES == 0, B_EVEN = B_P % WAVES == 0;
};

// ---- per-row conv coordinates (precomputed once per thread) ----
struct RowCoord {
  int b, oy, ox;
  bool valid;
};

__device__ __forceinline__ uint4 load_chunk_dense(const bf16_t* p, long ld, int row, int nrows, int k, int K) {
  if (row < nrows && k < K) return *reinterpret_cast<const uint4*>(p + (long)row * ld + k);
  return make_uint4(0, 0, 0, 0);
}

// per-K-tile conv gather state (uniform over the tile: BK divides every channel source, so one tap / source)
struct TapInfo {
  int kh, kw;
  int c0;            // channel offset inside the selected source
  int Cs;            // channel count (row pitch) of the selected source
  const bf16_t* src;
  bool valid;
};

__device__ __forceinline__ TapInfo tap_info(const GemmArgs& g, int k0) {
  const ConvGeom& cv = g.conv;
  const int Ct = cv.C1 + cv.C2;
  TapInfo t;
  t.valid = k0 < g.K1;
  const int tap = k0 / Ct;
  const int c = k0 - tap * Ct;
  t.kh = tap / cv.ks;
  t.kw = tap - t.kh * cv.ks;
  if (c < cv.C1) { t.src = g.a1; t.c0 = c; t.Cs = cv.C1; }
  else { t.src = cv.src2; t.c0 = c - cv.C1; t.Cs = cv.C2; }
  return t;
}

template <int MODE>
__device__ __forceinline__ uint4 load_chunk_conv(const ConvGeom& cv, const TapInfo& t, const RowCoord& rc, int kc) {
  if (!rc.valid || !t.valid) return make_uint4(0, 0, 0, 0);
  int iy, ix;
  if (MODE == PSO_CONV_NORMAL) {
    iy = rc.oy * cv.stride + t.kh - cv.pad;
    ix = rc.ox * cv.stride + t.kw - cv.pad;
    if ((unsigned)iy >= (unsigned)cv.H || (unsigned)ix >= (unsigned)cv.W) return make_uint4(0, 0, 0, 0);
  } else if (MODE == PSO_CONV_UP2) {
    const int uy = rc.oy + t.kh - cv.pad, ux = rc.ox + t.kw - cv.pad;
    if ((unsigned)uy >= (unsigned)(2 * cv.H) || (unsigned)ux >= (unsigned)(2 * cv.W)) return make_uint4(0, 0, 0, 0);
    iy = uy >> 1;
    ix = ux >> 1;
  } else {  // T2
    const int ty = rc.oy + cv.pad - t.kh, tx = rc.ox + cv.pad - t.kw;
    if (ty < 0 || tx < 0 || (ty & 1) || (tx & 1)) return make_uint4(0, 0, 0, 0);
    iy = ty >> 1;
    ix = tx >> 1;
    if (iy >= cv.H || ix >= cv.W) return make_uint4(0, 0, 0, 0);
  }
  const long pix = ((long)rc.b * cv.H + iy) * cv.W + ix;
  return *reinterpret_cast<const uint4*>(t.src + pix * t.Cs + t.c0 + kc);
}

__device__ __attribute__((aligned(16))) uint4 g_zero16[4];  // source of every zero-filled (padding / tail) chunk

typedef __attribute__((address_space(3))) void lds_void;

// s_waitcnt the compiler's waitcnt pass can see (inline asm is opaque to it).  The builtin exists only in the device
// compilation; the host pass must not see it or the kernel stubs are silently dropped.
#if defined(__HIP_DEVICE_COMPILE__)
#define PSO_S_WAITCNT(imm) __builtin_amdgcn_s_waitcnt(imm)
#else
#define PSO_S_WAITCNT(imm) ((void)0)
#endif

// Wait until at most n K-tiles' worth of this wave's direct-to-LDS loads (P pieces each) are still in flight (n is
// wave-uniform, 0..3: the STAGES <= 5 rings), then the block barrier; LGKM also retires this wave's LDS reads first.
template <int P, bool LGKM>
__device__ __forceinline__ void vm_wait_barrier(int n) {
  static_assert(3 * P <= 63, "vmcnt field");
  if (n >= 3) {
    if (LGKM) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(3 * P) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(3 * P) : "memory");
  } else if (n == 2) {
    if (LGKM) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(2 * P) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * P) : "memory");
  } else if (n == 1) {
    if (LGKM) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(P) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(P) : "memory");
  } else {
    if (LGKM) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
}

// Direct-to-LDS staging (global_load_lds_dwordx4): wave w fills 8-row x 128-B pieces; lane i of a piece lands at
// byte 16*i of it (row i/8, physical chunk i%8), so the XOR swizzle is applied to the SOURCE chunk: physical chunk p of
// row R holds logical chunk p ^ (R & 7) -- the same involution swz() applies on the read side.
// WM x WN waves, each owning a (BM/WM) x (BN/WN) accumulator tile; STAGES-deep LDS ring with STAGES-1 K-tiles of
// direct-to-LDS loads in flight behind a counted vmcnt and a raw s_barrier (a __syncthreads() would drain them).
template <int BM, int BN, int CONV, int WM, int WN, int STAGES, bool PIPE = false, int EPI = EPI_NONE>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_bf16_kernel(GemmArgs g) {
  constexpr int WAVES = WM * WN;
  using T = Tile<BM, BN, WAVES>;
  constexpr int MI = BM / WM / 16;  // 16-row subtiles per wave
  constexpr int NJ = BN / WN / 16;  // 16-col subtiles per wave
  constexpr int PIECES = T::A_CH + T::B_CH;  // glds per wave per K-tile
  static_assert(BM % 8 == 0 && BN % 8 == 0, "tile / wave split");
  extern __shared__ __attribute__((aligned(16))) bf16_t lds_dyn[];
  bf16_t* lds_base = lds_dyn;
  auto stage_ptr = [&](int s) { return lds_base + s * (BM + BN) * BK; };

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  auto pa = [&](int i) { return T::A_EVEN ? wave * T::A_CH + i : min(wave + WAVES * i, T::A_P - 1); };
  auto pb = [&](int i) { return T::B_EVEN ? wave * T::B_CH + i : min(wave + WAVES * i, T::B_P - 1); };

  // XCD-aware block order: blocks b, b+8, b+16 ... share an XCD; give each XCD a contiguous run of tiles.
  const int nbn = (g.N + BN - 1) / BN, nbm = (g.M + BM - 1) / BM;
  const int nblk = nbn * nbm;
  int bid = blockIdx.x;
  {
    const int q = nblk / 8, r = nblk % 8, x = bid % 8;
    if (nblk >= 8) bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  // grouped raster: runs of g.group_m tile rows are walked column by column, so the tiles an XCD's CUs hold at once
  // share A row-panels and B column-panels in its L2 (group_m = 1: plain row-major)
  int bm, bn;
  {
    const int gm = g.group_m;
    const int per_group = gm * nbn;
    const int grp = bid / per_group, first_m = grp * gm;
    const int gsz = min(nbm - first_m, gm);
    const int in = bid - grp * per_group;
    bm = first_m + in % gsz;
    bn = in / gsz;
  }
  const int m0 = bm * BM, n0 = bn * BN;

  const int nt1 = (g.K1 + BK - 1) / BK;
  // tiles made only of rows >= tail_m (the reference half of a paired pass) skip the LoRA K-tail: it is zero there
  const int nt2 = (g.a2 && m0 < g.tail_m) ? (g.K2 + BK - 1) / BK : 0;
  const int nt_all = nt1 + nt2;
  // split-K (gridDim.y > 1): this block owns K-tiles [t_beg, t_end); partials are added atomically (f32 out)
  const int per = (nt_all + gridDim.y - 1) / gridDim.y;
  const int t_beg = blockIdx.y * per;
  const int t_end = min(nt_all, t_beg + per);
  const int nt = t_end > t_beg ? t_end - t_beg : 0;
  const long a2_off = g.tail_group_n > 0 ? (long)(n0 / g.tail_group_n) * g.K2 : 0;

  // This lane's staging rows: piece i of wave w covers rows (w*A_CH + i)*8 .. +8 (B likewise).  Rows past M / N are
  // clamped onto the last valid row (their results are never stored), so the hot loop needs no row predicates and
  // every per-tile address is (per-lane constant offset) + k0: no branches, no kernel-argument reloads.
  const int prow = lane >> 3;
  const int pch = lane & 7;
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_zero16);
  const long zb = blockIdx.z;
  const bf16_t* const a1 = g.a1 + zb * g.bat_a;
  const bf16_t* const b1 = g.b1 + zb * g.bat_b;
  void* const outp = reinterpret_cast<char*>(g.out) + zb * g.bat_o * (g.out_dtype == PSO_F32 ? 4 : 2);
  const int K1 = g.K1;
  int lcA[T::A_CH], offA[T::A_CH];  // logical chunk (source-side swizzle) and element offset of this lane's rows
  int lcB[T::B_CH], offB[T::B_CH];
  RowCoord rc[T::A_CH];
#pragma unroll
  for (int i = 0; i < T::A_CH; ++i) {
    const int R = pa(i) * 8 + prow;
    const int m = min(m0 + R, g.M - 1);
    lcA[i] = pch ^ (R & 7);
    offA[i] = CONV ? 0 : (int)((long)m * g.lda1) + lcA[i] * 8;
    if (CONV) {
      const int hw = g.conv.Ho * g.conv.Wo;
      rc[i].valid = true;
      rc[i].b = m / hw;
      const int rem = m - rc[i].b * hw;
      rc[i].oy = rem / g.conv.Wo;
      rc[i].ox = rem - rc[i].oy * g.conv.Wo;
    }
  }
#pragma unroll
  for (int i = 0; i < T::B_CH; ++i) {
    const int R = pb(i) * 8 + prow;
    const int n = min(n0 + R, g.N - 1);
    lcB[i] = pch ^ (R & 7);
    offB[i] = (int)((long)n * g.ldb1) + lcB[i] * 8;
  }
  // conv geometry in registers once
  const int cvH = g.conv.H, cvW = g.conv.W, cvS = g.conv.stride, cvP = g.conv.pad;

  auto issue_tile = [&](int tt, int buf) {
    const int t = tt + t_beg;
    bf16_t* la = stage_ptr(buf);
    bf16_t* lb = stage_ptr(buf) + BM * BK;
    if (t < nt1) {
      const int k0 = t * BK;
      const bool full = k0 + BK <= K1;  // uniform: partial last K-tile needs per-chunk predicates
      if (CONV) {
        const TapInfo ti = tap_info(g, k0);
#pragma unroll
        for (int i = 0; i < T::A_CH; ++i) {
          const int piece = pa(i);
          int iy, ix;
          bool ok;
          if (CONV == PSO_CONV_NORMAL) {
            iy = rc[i].oy * cvS + ti.kh - cvP;
            ix = rc[i].ox * cvS + ti.kw - cvP;
            ok = (unsigned)iy < (unsigned)cvH && (unsigned)ix < (unsigned)cvW;
          } else if (CONV == PSO_CONV_UP2) {
            const int uy = rc[i].oy + ti.kh - cvP, ux = rc[i].ox + ti.kw - cvP;
            ok = (unsigned)uy < (unsigned)(2 * cvH) && (unsigned)ux < (unsigned)(2 * cvW);
            iy = uy >> 1;
            ix = ux >> 1;
          } else {
            const int ty = rc[i].oy + cvP - ti.kh, tx = rc[i].ox + cvP - ti.kw;
            iy = ty >> 1;
            ix = tx >> 1;
            ok = ty >= 0 && tx >= 0 && !(ty & 1) && !(tx & 1) && iy < cvH && ix < cvW;
          }
          const bf16_t* src = ti.src + ((long)((rc[i].b * cvH + iy) * cvW + ix)) * ti.Cs + ti.c0 + lcA[i] * 8;
          __builtin_amdgcn_global_load_lds(static_cast<const void*>(ok ? src : zero), (lds_void*)(la + piece * 8 * BK), 16, 0, 0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < T::A_CH; ++i) {
          const int piece = pa(i);
          const bool ok = full || k0 + lcA[i] * 8 < K1;
          __builtin_amdgcn_global_load_lds(static_cast<const void*>(ok ? a1 + offA[i] + k0 : zero), (lds_void*)(la + piece * 8 * BK), 16, 0, 0);
        }
      }
#pragma unroll
      for (int i = 0; i < T::B_CH; ++i) {
        const int piece = pb(i);
        const bool ok = full || k0 + lcB[i] * 8 < K1;
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(ok ? b1 + offB[i] + k0 : zero), (lds_void*)(lb + piece * 8 * BK), 16, 0, 0);
      }
    } else {  // LoRA / second-operand K-tail (rare: one or two tiles per launch)
      const int k0 = (t - nt1) * BK;
#pragma unroll
      for (int i = 0; i < T::A_CH; ++i) {
        const int piece = pa(i);
        const int R = piece * 8 + prow;
        const int mr = m0 + R;
        const int m = min(mr, g.tail_m - 1);
        const int k = k0 + lcA[i] * 8;
        const bf16_t* src = g.a2 + a2_off + (long)m * g.lda2 + k;
        __builtin_amdgcn_global_load_lds(static_cast<const void*>((k < g.K2 && mr < g.tail_m) ? src : zero),
                                         (lds_void*)(la + piece * 8 * BK), 16, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < T::B_CH; ++i) {
        const int piece = pb(i);
        const int R = piece * 8 + prow;
        const int n = min(n0 + R, g.N - 1);
        const int k = k0 + lcB[i] * 8;
        const bf16_t* src = g.b2 + (long)n * g.ldb2 + k;
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(k < g.K2 ? src : zero), (lds_void*)(lb + piece * 8 * BK), 16, 0, 0);
      }
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fk = lane >> 4;
  // Epilogue operands (bias, and the residual or the per-row-group bias) for the dense bf16/f32 store path, loaded into
  // registers while the last K-tile computes instead of one dependent load per output subtile afterwards.
  const bool epi_fast = EPI == EPI_NONE && MI * NJ <= 20 && gridDim.y == 1 && g.vec_ok && n0 + BN <= g.N && !(g.resid && g.rowbias);
  uint2 ebias[NJ], eadd[MI][NJ];
  auto epi_prefetch = [&]() {
    if (!epi_fast) return;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wn * (BN / WN) + j * 16 + fk * 4;
      ebias[j] = g.bias ? *reinterpret_cast<const uint2*>(g.bias + n) : make_uint2(0u, 0u);
    }
    const bf16_t* ap = g.resid ? g.resid : g.rowbias;
    if (!ap) return;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = min(m0 + wm * (BM / WM) + i * 16 + fr, g.M - 1);
      const long row = g.resid ? (long)m * g.ldr : (long)(m / g.rows_per_group) * g.ld_rowbias;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        eadd[i][j] = *reinterpret_cast<const uint2*>(ap + row + n0 + wn * (BN / WN) + j * 16 + fk * 4);
    }
  };
  if constexpr (PIPE) {
    // Register-pipelined schedule (2 LDS buffers + fragments of the next K-half in registers):
    //   iteration t:  ds_read kk=1 of tile t | MFMA kk=0 of t | lgkmcnt(0), vmcnt(0) [tile t+1 landed], s_barrier |
    //                 glds tile t+2 -> buffer of t | ds_read kk=0 of t+1 | MFMA kk=1 of t
    // so LDS reads always overlap MFMAs and the barrier is the only cross-wave sync per K-tile.  WAR: buffer t is
    // re-staged only after every wave retired its reads of it (lgkmcnt(0) before the barrier).  RAW: tile t+1 is
    // read only after every wave's glds of it retired (vmcnt(0) before the same barrier).
    static_assert(STAGES == 2, "pipelined schedule uses two LDS buffers");
    bf16x8 fa0[MI], fb0[NJ], fa1[MI], fb1[NJ];
    auto read_frags = [&](int buf, int kk, bf16x8* fa, bf16x8* fb) {
      const bf16_t* la = stage_ptr(buf);
      const bf16_t* lb = stage_ptr(buf) + BM * BK;
#pragma unroll
      for (int i = 0; i < MI; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(la + swz(wm * (BM / WM) + i * 16 + fr, kk * 4 + fk));
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(lb + swz(wn * (BN / WN) + j * 16 + fr, kk * 4 + fk));
    };
    auto mfma_all = [&](const bf16x8* fa, const bf16x8* fb) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    if (nt > 0) issue_tile(0, 0);
    if (nt > 1) issue_tile(1, 1);
    if (nt > 1) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(PIECES) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (nt > 0) read_frags(0, 0, fa0, fb0);
    PSO_S_WAITCNT(0xC07F);  // same state on both loop-header edges (see the end of the loop body)
    for (int t = 0; t < nt; ++t) {
      const int cur = t & 1;
      read_frags(cur, 1, fa1, fb1);
      mfma_all(fa0, fb0);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (t + 2 < nt) issue_tile(t + 2, cur);
      read_frags(cur ^ 1, 0, fa0, fb0);  // unconditional (past the last tile it reads a dead buffer, never used)
      // kk=1 fragments landed; the MI+NJ kk=0 reads just issued stay in flight behind these MFMAs
      static_assert(MI + NJ <= 15, "lgkmcnt field");
      PSO_S_WAITCNT(0xC07F | ((MI + NJ) << 8));
      mfma_all(fa1, fb1);
      // retire the kk=0 fragment reads HERE (behind the MFMAs) with a waitcnt the compiler can see, so the next
      // iteration's MFMAs on them do not wait for the kk=1 reads issued just before (LDS returns in order, but the
      // waitcnt pass merges the loop back-edge conservatively).  0xC07F = vmcnt(63) expcnt(7) lgkmcnt(0).
      PSO_S_WAITCNT(0xC07F);
    }
  } else {
  // prologue: K-tiles 0 .. STAGES-2 in flight; wait for tile 0
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nt) issue_tile(s, s);
  // tile 0 landed; tiles 1 .. STAGES-2 may stay in flight
  static_assert(STAGES <= 5, "vm_wait_barrier covers rings of up to 5 stages");
  vm_wait_barrier<PIECES, false>(min(STAGES - 2, nt - 1));

  int cur = 0;
  auto mfma_half = [&](const bf16_t* la, const bf16_t* lb, int kk) {
    bf16x8 af[MI], bfr[NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
      af[i] = *reinterpret_cast<const bf16x8*>(la + swz(wm * (BM / WM) + i * 16 + fr, kk * 4 + fk));
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8*>(lb + swz(wn * (BN / WN) + j * 16 + fr, kk * 4 + fk));
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // a LoRA K-tail of rank <= 32 fills only the first 32-deep half of its (last) K-tile, the rest being zero padding:
  // that tile is peeled off the loop and multiplies its first half only
  const bool half_last = nt > 0 && nt2 == 1 && g.K2 <= 32 && t_end == nt_all;
  const int nt_loop = nt - (half_last ? 1 : 0);
  for (int t = 0; t < nt_loop; ++t) {
    const bool ahead = t + STAGES - 1 < nt;
    if (ahead) issue_tile(t + STAGES - 1, (cur + STAGES - 1) % STAGES);
    const bf16_t* la = stage_ptr(cur);
    const bf16_t* lb = stage_ptr(cur) + BM * BK;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) mfma_half(la, lb, kk);
    // K-tile t+1 must have landed (every wave's pieces) before anyone reads it; tiles t+2 .. stay in flight
    vm_wait_barrier<PIECES, true>(min(STAGES - 2, nt - t - 2));
    cur = (cur + 1 == STAGES) ? 0 : cur + 1;
  }
  if (half_last) {  // landed: the last loop iteration waited for it (vmcnt(0): nothing was issued beyond it)
    mfma_half(stage_ptr(cur), stage_ptr(cur) + BM * BK, 0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  }  // !PIPE

  // ---- epilogue: lane holds out[m][n0..n0+3] for each (i, j) ----
  if constexpr (EPI == EPI_NONE && !PIPE) {
    if (g.ws) {  // deterministic split-K: this split's partial product (every split stores, empty ones zeros)
      float* part = g.ws + (long)blockIdx.y * g.M * g.N;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = m0 + wm * (BM / WM) + i * 16 + fr;
        if (m >= g.M) continue;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int n = n0 + wn * (BN / WN) + j * 16 + fk * 4;
          if (n < g.N)
            *reinterpret_cast<float4*>(part + (long)m * g.N + n) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2],
                                                                              acc[i][j][3]);
        }
      }
      return;
    }
  }
  if constexpr (EPI == EPI_GEGLU) {
    // this wave's 64 columns = one interleaved group: subtiles j = 0,1 hold h, j = 2,3 the matching gate columns.
    // h and gate are rounded to bf16 first (the unfused path stores them in bf16 before the GEGLU).
    static_assert(NJ == 4, "GEGLU epilogue needs 64-column wave tiles");
    const int ng = n0 + wn * 64;
    // the bias of this lane's 2 x 4 h / gate columns, loaded once up front (the stores below may alias it for the
    // compiler, which would otherwise reload it per row subtile behind each store)
    float bhv[2][4], bgv[2][4];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int nh = ng + jj * 16 + fk * 4;
      const uint2 bh = *reinterpret_cast<const uint2*>(g.bias + nh);
      const uint2 bg = *reinterpret_cast<const uint2*>(g.bias + nh + 32);
      bhv[jj][0] = bf2f(bh.x & 0xffff); bhv[jj][1] = bf2f(bh.x >> 16); bhv[jj][2] = bf2f(bh.y & 0xffff); bhv[jj][3] = bf2f(bh.y >> 16);
      bgv[jj][0] = bf2f(bg.x & 0xffff); bgv[jj][1] = bf2f(bg.x >> 16); bgv[jj][2] = bf2f(bg.y & 0xffff); bgv[jj][3] = bf2f(bg.y >> 16);
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * (BM / WM) + i * 16 + fr;
      if (m >= g.M) continue;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int nh = ng + jj * 16 + fk * 4;
        float vh[4], vg[4], o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          vh[r] = bf_round(acc[i][jj][r] * g.alpha + bhv[jj][r]);
          vg[r] = bf_round(acc[i][jj + 2][r] * g.alpha + bgv[jj][r]);
          o[r] = vh[r] * gelu_erf(vg[r]);
        }
        if (g.out2 && m < g.tail_m) {  // pre-activation rows kept for the backward (policy rows of a paired pass)
          bf16_t* p = reinterpret_cast<bf16_t*>(g.out2) + (long)m * g.ldo2 + nh;
          *reinterpret_cast<uint2*>(p) = make_uint2(pack2bf(vh[0], vh[1]), pack2bf(vh[2], vh[3]));
          *reinterpret_cast<uint2*>(p + 32) = make_uint2(pack2bf(vg[0], vg[1]), pack2bf(vg[2], vg[3]));
        }
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(outp) + (long)m * g.ldo + ng / 2 + jj * 16 + fk * 4) =
            make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
      }
    }
    return;
  }
  if constexpr (EPI == EPI_GEGLU_BWD) {
    // GEGLU backward epilogue, staged through LDS so every global access is a coalesced 16-B chunk: dout is rounded to
    // bf16 into LDS (exactly what the unfused path stores), then the workgroup walks it in 8-column chunks, reading
    // the interleaved pre-activation and writing the interleaved input gradient.
    constexpr int TP = (BM * (BN + 8) * 2 <= STAGES * (BM + BN) * BK * 2) ? BN + 8 : BN;  // tile pitch (elements)
    constexpr int NT = 64 * WM * WN;
    __syncthreads();  // every wave is done with the operand ring
    bf16_t* tl = lds_base;
    const float bscale = g.alpha;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int ml = wm * (BM / WM) + i * 16 + fr;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int nl = wn * (BN / WN) + j * 16 + fk * 4;
        float v[4] = {acc[i][j][0] * bscale, acc[i][j][1] * bscale, acc[i][j][2] * bscale, acc[i][j][3] * bscale};
        *reinterpret_cast<uint2*>(tl + ml * TP + nl) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
      }
    }
    __syncthreads();
    {
      // dout chunk (row ml, columns c .. c+7 of the F-wide gradient) -> interleaved positions ph .. ph+7 (gate +32)
      constexpr int CC = BN / 8;
      constexpr int ITERS = (BM * CC + NT - 1) / NT;
      // every pre-activation load of this thread in flight at once (the output stores may alias them for the
      // compiler, which would otherwise serialise one HBM round trip per chunk)
      uint4 hvv[ITERS], gvv[ITERS];
#pragma unroll
      for (int it = 0; it < ITERS; ++it) {
        const int q = threadIdx.x + it * NT;
        const int ml = q / CC, cl = (q - (q / CC) * CC) * 8;
        const int m = min(m0 + ml, g.M - 1), n = min(n0 + cl, g.N - 8);
        const int ph = (n >> 5) * 64 + (n & 31);
        if (q < BM * CC) {
          hvv[it] = *reinterpret_cast<const uint4*>(g.aux + (long)m * g.ldaux + ph);
          gvv[it] = *reinterpret_cast<const uint4*>(g.aux + (long)m * g.ldaux + ph + 32);
        }
      }
#pragma unroll
      for (int it = 0; it < ITERS; ++it) {
        const int q = threadIdx.x + it * NT;
        const int ml = q / CC, cl = (q - (q / CC) * CC) * 8;
        const int m = m0 + ml, n = n0 + cl;
        if (q >= BM * CC || m >= g.M || n >= g.N) continue;
        const int ph = (n >> 5) * 64 + (n & 31);
        const uint4 dv = *reinterpret_cast<const uint4*>(tl + ml * TP + cl);
        const uint4 hv = hvv[it], gv = gvv[it];
        const uint32_t dw[4] = {dv.x, dv.y, dv.z, dv.w}, hw[4] = {hv.x, hv.y, hv.z, hv.w}, gw[4] = {gv.x, gv.y, gv.z, gv.w};
        uint32_t oh[4], og[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d0 = bf2f(dw[e] & 0xffff), d1 = bf2f(dw[e] >> 16);
          const float h0 = bf2f(hw[e] & 0xffff), h1 = bf2f(hw[e] >> 16);
          const float g0 = bf2f(gw[e] & 0xffff), g1 = bf2f(gw[e] >> 16);
          float c0, e0, c1, e1;
          gelu_erf_parts(g0, c0, e0);
          gelu_erf_parts(g1, c1, e1);
          oh[e] = pack2bf(d0 * g0 * c0, d1 * g1 * c1);
          og[e] = pack2bf(d0 * h0 * (c0 + 0.39894228040143268f * g0 * e0), d1 * h1 * (c1 + 0.39894228040143268f * g1 * e1));
        }
        bf16_t* p = reinterpret_cast<bf16_t*>(outp) + (long)m * g.ldo + ph;
        *reinterpret_cast<uint4*>(p) = make_uint4(oh[0], oh[1], oh[2], oh[3]);
        *reinterpret_cast<uint4*>(p + 32) = make_uint4(og[0], og[1], og[2], og[3]);
      }
    }
    return;
  }
  if constexpr (EPI == EPI_NONE && !PIPE && BM * (BN + 8) * 2 <= STAGES * (BM + BN) * BK * 2) {
    if (g.stage_epi && epi_fast && g.out_dtype == PSO_BF16 && !g.accumulate && nt > 0) {
      // Staged epilogue: y = bf16(acc * alpha + bias [+ rowbias]) goes to LDS in the MFMA layout, then the workgroup
      // walks the tile in 16-B chunks: residual loaded and output stored as whole 16-B vectors (half the store
      // instructions of the 8-B per-lane layout).  The residual is added to the bf16-rounded projection, as the
      // unfused Linear + add does.
      constexpr int TP = BN + 8;
      constexpr int NT = 64 * WM * WN;
      constexpr int CC = BN / 8;
      constexpr int ITERS = (BM * CC + NT - 1) / NT;
      const bool rowb = g.rowbias != nullptr;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wn * (BN / WN) + j * 16 + fk * 4;
        ebias[j] = g.bias ? *reinterpret_cast<const uint2*>(g.bias + n) : make_uint2(0u, 0u);
      }
      if (rowb) {
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int m = min(m0 + wm * (BM / WM) + i * 16 + fr, g.M - 1);
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            eadd[i][j] = *reinterpret_cast<const uint2*>(g.rowbias + (long)(m / g.rows_per_group) * g.ld_rowbias + n0 +
                                                         wn * (BN / WN) + j * 16 + fk * 4);
        }
      }
      __syncthreads();  // every wave is done with the operand ring
      bf16_t* tl = lds_base;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int ml = wm * (BM / WM) + i * 16 + fr;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int nl = wn * (BN / WN) + j * 16 + fk * 4;
          float v[4] = {acc[i][j][0] * g.alpha + bf2f(ebias[j].x & 0xffff), acc[i][j][1] * g.alpha + bf2f(ebias[j].x >> 16),
                        acc[i][j][2] * g.alpha + bf2f(ebias[j].y & 0xffff), acc[i][j][3] * g.alpha + bf2f(ebias[j].y >> 16)};
          if (rowb) {
            v[0] += bf2f(eadd[i][j].x & 0xffff); v[1] += bf2f(eadd[i][j].x >> 16);
            v[2] += bf2f(eadd[i][j].y & 0xffff); v[3] += bf2f(eadd[i][j].y >> 16);
          }
          *reinterpret_cast<uint2*>(tl + ml * TP + nl) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
        }
      }
      // residual chunks: every load in flight at once (the accumulators are dead now)
      uint4 rr[ITERS];
      if (g.resid) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
          const int q = threadIdx.x + it * NT;
          const int ml = q / CC, cl = (q - (q / CC) * CC) * 8;
          const int m = min(m0 + ml, g.M - 1);
          if (q < BM * CC) rr[it] = *reinterpret_cast<const uint4*>(g.resid + (long)m * g.ldr + n0 + cl);
        }
      }
      __syncthreads();
#pragma unroll
      for (int it = 0; it < ITERS; ++it) {
        const int q = threadIdx.x + it * NT;
        const int ml = q / CC, cl = (q - (q / CC) * CC) * 8;
        const int m = m0 + ml;
        if (q >= BM * CC || m >= g.M) continue;
        uint4 y = *reinterpret_cast<const uint4*>(tl + ml * TP + cl);
        if (g.resid) {
          const uint32_t yw[4] = {y.x, y.y, y.z, y.w}, rw[4] = {rr[it].x, rr[it].y, rr[it].z, rr[it].w};
          uint32_t o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            o[e] = pack2bf(bf2f(yw[e] & 0xffff) + bf2f(rw[e] & 0xffff), bf2f(yw[e] >> 16) + bf2f(rw[e] >> 16));
          y = make_uint4(o[0], o[1], o[2], o[3]);
        }
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(outp) + (long)m * g.ldo + n0 + cl) = y;
      }
      return;
    }
  }
  if (!PIPE && epi_fast && nt > 0) {
    epi_prefetch();  // every epilogue load in flight at once, then the arithmetic and the stores
    const bool has_add = g.resid || g.rowbias;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * (BM / WM) + i * 16 + fr;
      if (m >= g.M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wn * (BN / WN) + j * 16 + fk * 4;
        // same association as the generic path below: ((acc*alpha + bias) + rowbias | resid)
        float v[4] = {acc[i][j][0] * g.alpha + bf2f(ebias[j].x & 0xffff), acc[i][j][1] * g.alpha + bf2f(ebias[j].x >> 16),
                      acc[i][j][2] * g.alpha + bf2f(ebias[j].y & 0xffff), acc[i][j][3] * g.alpha + bf2f(ebias[j].y >> 16)};
        if (has_add) {
          v[0] += bf2f(eadd[i][j].x & 0xffff); v[1] += bf2f(eadd[i][j].x >> 16);
          v[2] += bf2f(eadd[i][j].y & 0xffff); v[3] += bf2f(eadd[i][j].y >> 16);
        }
        if (g.out_dtype == PSO_BF16) {
          *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(outp) + (long)m * g.ldo + n) =
              make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
        } else {
          float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(outp) + (long)m * g.ldo + n);
          if (g.accumulate) {
            const float4 old = *o;
            v[0] += old.x; v[1] += old.y; v[2] += old.z; v[3] += old.w;
          }
          *o = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = m0 + wm * (BM / WM) + i * 16 + fr;
    if (m >= g.M) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wn * (BN / WN) + j * 16 + fk * 4;
      if (n >= g.N) continue;
      float v[4] = {acc[i][j][0] * g.alpha, acc[i][j][1] * g.alpha, acc[i][j][2] * g.alpha,
                    acc[i][j][3] * g.alpha};
      if (gridDim.y > 1) {  // split-K partial: f32 accumulate output, no bias / residual (host-checked)
        float* o = reinterpret_cast<float*>(outp) + (long)m * g.ldo + n;
        for (int r = 0; r < 4 && n + r < g.N; ++r) atomicAdd(o + r, v[r]);
        continue;
      }
      const bool full = g.vec_ok && (n + 4 <= g.N);
      if (full) {
        if (g.bias) {
          const uint2 bv = *reinterpret_cast<const uint2*>(g.bias + n);
          v[0] += bf2f(bv.x & 0xffff); v[1] += bf2f(bv.x >> 16); v[2] += bf2f(bv.y & 0xffff); v[3] += bf2f(bv.y >> 16);
        }
        if (g.rowbias) {
          const uint2 bv = *reinterpret_cast<const uint2*>(g.rowbias + (long)(m / g.rows_per_group) * g.ld_rowbias + n);
          v[0] += bf2f(bv.x & 0xffff); v[1] += bf2f(bv.x >> 16); v[2] += bf2f(bv.y & 0xffff); v[3] += bf2f(bv.y >> 16);
        }
        if (g.resid) {
          const uint2 rv = *reinterpret_cast<const uint2*>(g.resid + (long)m * g.ldr + n);
          v[0] += bf2f(rv.x & 0xffff); v[1] += bf2f(rv.x >> 16); v[2] += bf2f(rv.y & 0xffff); v[3] += bf2f(rv.y >> 16);
        }
        if (g.out_dtype == PSO_BF16) {
          *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(outp) + (long)m * g.ldo + n) =
              make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
        } else {
          float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(outp) + (long)m * g.ldo + n);
          if (g.accumulate) {
            const float4 old = *o;
            v[0] += old.x; v[1] += old.y; v[2] += old.z; v[3] += old.w;
          }
          *o = make_float4(v[0], v[1], v[2], v[3]);
        }
      } else {
        for (int r = 0; r < 4 && n + r < g.N; ++r) {
          float x = v[r];
          if (g.bias) x += bf2f(g.bias[n + r]);
          if (g.rowbias) x += bf2f(g.rowbias[(long)(m / g.rows_per_group) * g.ld_rowbias + n + r]);
          if (g.resid) x += bf2f(g.resid[(long)m * g.ldr + n + r]);
          if (g.out_dtype == PSO_BF16) {
            reinterpret_cast<bf16_t*>(outp)[(long)m * g.ldo + n + r] = f2bf(x);
          } else {
            float* o = reinterpret_cast<float*>(outp) + (long)m * g.ldo + n + r;
            *o = g.accumulate ? *o + x : x;
          }
        }
      }
    }
  }
}

template <int BM, int BN, int WM = 2, int WN = 2, int STAGES = 2, bool PIPE = false, int EPI = EPI_NONE>
static int launch(const GemmArgs& g, hipStream_t st, int ksplit = 1) {
  const int nblk = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  dim3 grid(nblk, ksplit, g.batch > 1 ? g.batch : 1);
  const int threads = 64 * WM * WN;
  const size_t shm = (size_t)STAGES * (BM + BN) * BK * sizeof(bf16_t);
  pso_note_kernel("gemm_bf16_kernel<%d, %d, %d, %d, %d, %d, %s, %d>", BM, BN, EPI != EPI_NONE ? 0 : g.conv.mode, WM, WN,
                  STAGES, PIPE ? "true" : "false", EPI);
  static bool attr_done = false;  // >64 KiB dynamic LDS needs the attribute once per instantiation
  if constexpr (EPI != EPI_NONE) {  // fused-activation epilogues: dense operands only
    if (!attr_done) {
      (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<BM, BN, 0, WM, WN, STAGES, PIPE, EPI>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
      attr_done = true;
    }
    gemm_bf16_kernel<BM, BN, 0, WM, WN, STAGES, PIPE, EPI><<<grid, threads, shm, st>>>(g);
    return pso_check_launch("pso_gemm(geglu)");
  }
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<BM, BN, 0, WM, WN, STAGES, PIPE, EPI>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<BM, BN, PSO_CONV_NORMAL, WM, WN, STAGES, PIPE, EPI>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<BM, BN, PSO_CONV_UP2, WM, WN, STAGES, PIPE, EPI>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<BM, BN, PSO_CONV_T2, WM, WN, STAGES, PIPE, EPI>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    attr_done = true;
  }
  switch (g.conv.mode) {
    case PSO_CONV_NORMAL:
      gemm_bf16_kernel<BM, BN, PSO_CONV_NORMAL, WM, WN, STAGES, PIPE, EPI><<<grid, threads, shm, st>>>(g);
      break;
    case PSO_CONV_UP2: gemm_bf16_kernel<BM, BN, PSO_CONV_UP2, WM, WN, STAGES, PIPE, EPI><<<grid, threads, shm, st>>>(g); break;
    case PSO_CONV_T2: gemm_bf16_kernel<BM, BN, PSO_CONV_T2, WM, WN, STAGES, PIPE, EPI><<<grid, threads, shm, st>>>(g); break;
    default: gemm_bf16_kernel<BM, BN, 0, WM, WN, STAGES, PIPE, EPI><<<grid, threads, shm, st>>>(g);
  }
  return pso_check_launch("pso_gemm");
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
static bool al8(const void* p) { return ((uintptr_t)p & 7) == 0; }

int pso_gemm_skinny_nt(int M, int N, int K, const void* A, long lda, const void* W, long ldw, float alpha, void* out,
                       long ldo, int out_f32, int accumulate, int groups, hipStream_t st);
int pso_gemm_tn_rank(int M, int C, const void* X, long ldx, const void* U, long ldu, int R, int group_c, float alpha,
                     float* out, long ldo, int out_jc, hipStream_t st);

// 8-phase 256x256 kernel (gemm8p.hip): epi 0 dense (+ LoRA K-tail, bias, alpha, residual), 1 GEGLU, 2 GEGLU backward
int pso_gemm8p_run(int epi, int M, int N, int K, const void* a, long lda, const void* w, long ldw, const void* a2,
                   long lda2, int K2, const void* w2, long ldw2, int tail_m, int tail_group_n, float alpha,
                   const void* bias, const void* resid, long ldr, void* out, long ldo, void* out2, long ldo2,
                   int pre_rows, const void* aux, long ldaux, int group_m, hipStream_t st);
int pso_gemm8p160_run(int M, int N, int K, const void* a, long lda, const void* w, long ldw, const void* a2, long lda2,
                      int K2, const void* w2, long ldw2, int tail_m, int tail_group_n, float alpha, const void* bias,
                      const void* resid, long ldr, void* out, long ldo, int group_m, hipStream_t st);
int pso_gemm8p320_run(int M, int N, int K, const void* a, long lda, const void* w, long ldw, const void* a2, long lda2,
                      int K2, const void* w2, long ldw2, int tail_m, int tail_group_n, float alpha, const void* bias,
                      const void* resid, long ldr, void* out, long ldo, int group_m, hipStream_t st);
int pso_gemm8p320_conv_run(int B, int H, int W, int C, const void* x, const void* w, int Cout, float alpha,
                           const void* bias, const void* rowbias, long ld_rowbias, const void* resid, long ldr,
                           void* out, long ldo, int group_m, hipStream_t st);
int pso_gemm8p320_geglu_bwd_run(int M, int N, int K, const void* a, long lda, const void* w, long ldw, const void* aux,
                                long ldaux, void* out, long ldo, int group_m, hipStream_t st);
int pso_gemm8p320_geglu_run(int M, int N, int K, const void* a, long lda, const void* w, long ldw, const void* bias,
                            void* out, long ldo, void* out2, long ldo2, int pre_rows, int group_m, hipStream_t st);
static bool fits30(long rows, long ld) { return rows * ld < (1L << 30); }
int pso_conv3x3_smallc_run(int B, int H, int W, int Cin, int Cout, const void* x, const void* w, const void* bias,
                           void* out, hipStream_t st);  // conv_small.hip

// Ordered reduction of the split-K partials + the plain epilogue (4 consecutive columns per thread, N % 4 == 0):
//   y = alpha * sum_s ws[s][m][n] + bias[n] + rowbias[m / rows_per_group][n]
//   bf16 out: out = bf16(bf16(y) + resid) (the staged epilogue's rounding: the residual is added to the rounded
//             projection, as the unfused Linear + add does), f32 out: out (+)= y + resid
__global__ void gemm_splitk_reduce_kernel(GemmArgs g, int ks) {
  const long q = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int nq = g.N / 4;
  if (q >= (long)g.M * nq) return;
  const int m = (int)(q / nq), n = (int)(q - (long)m * nq) * 4;
  const float* src = g.ws + (long)m * g.N + n;
  float4 acc = *reinterpret_cast<const float4*>(src);
  for (int s = 1; s < ks; ++s) {
    const float4 v = *reinterpret_cast<const float4*>(src + (long)s * g.M * g.N);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  float v[4] = {acc.x * g.alpha, acc.y * g.alpha, acc.z * g.alpha, acc.w * g.alpha};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (g.bias) v[r] += bf2f(g.bias[n + r]);
    if (g.rowbias) v[r] += bf2f(g.rowbias[(long)(m / g.rows_per_group) * g.ld_rowbias + n + r]);
  }
  if (g.out_dtype == PSO_BF16) {
    if (g.resid) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = bf2f(f2bf(v[r])) + bf2f(g.resid[(long)m * g.ldr + n + r]);
    }
    bf16_t* o = reinterpret_cast<bf16_t*>(g.out) + (long)m * g.ldo + n;
    *reinterpret_cast<uint2*>(o) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
  } else {
    float* o = reinterpret_cast<float*>(g.out) + (long)m * g.ldo + n;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (g.resid) v[r] += bf2f(g.resid[(long)m * g.ldr + n + r]);
      o[r] = g.accumulate ? o[r] + v[r] : v[r];
    }
  }
}

// Split-K plan of a dense GEMM whose output tiles leave CUs idle while its reduction is long (the bs = 1 / GPU
// backward at M = 2048: 2048 x 1280 x 10240 makes 128 tiles of 128 x 160 -- half a 256-CU round at one workgroup
// each; and one-round shapes with K >= 4096): ks K-splits of >= 16 K-tiles each, towards 512 workgroups (two per
// CU), reduced in split order through a
// caller-owned fp32 workspace (deterministic).  The partials cost 8 M N bytes per split against 2 M N K / ks flop,
// so only K >= 2048 qualifies.  Returns ks (0: no split) and the tile.
struct SplitPlan { int ks, bm, bn; };
// Benchmark knobs (A/B variants, forced tiles, raster groups): only the tools build (-DPSO_BENCH_KNOBS ->
// libpso_amd_knobs.so, include/pso_amd_knobs.h) has them as mutable state; the product library's are compile-time
// zeros, so every knob branch folds away and the measured-not-kept forms are not compiled into it.
#ifdef PSO_BENCH_KNOBS
static int g_gemm_variant = 0;
#else
static constexpr int g_gemm_variant = 0;
#endif
static SplitPlan gemm_split_plan(int M, int N, int K1, int K2, bool has_tail, bool dense) {
  SplitPlan p{0, 0, 0};
  if (!dense || M <= 0 || N <= 0 || (N % 4) != 0) return p;
  const int bm = 128, bn = (N % 160) == 0 ? 160 : 128;
  const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  const int nt_all = (K1 + 63) / 64 + (has_tail ? (K2 + 63) / 64 : 0);
  // variant 51: splits of >= 8 K-tiles (the short-K M = 2048 products: 2048 x 1280 x 1280 + LoRA in two)
  const int min_kt = g_gemm_variant == 51 ? 8 : 16;
  // one full round of tiles (<= 256: the 4096-row products and 3x3 convs of the bs = 1 / GPU pass, K >= 4096) splits
  // in two as well: bs = 1 step 81.56 -> 80.25 ms, C3 237.2 -> 236.5, C2 untouched (tools/bs1_variant_ab.py, one box;
  // K >= 2560 measured the same, up to 384 tiles cost C3 1.5 %).  Variant 55 keeps the half-round rule.
  const bool round2 = g_gemm_variant != 55 && tiles <= 256 && nt_all >= 64;
  if ((tiles > 128 && !round2) || nt_all < 2 * min_kt) return p;
  int ks = (int)((512 + tiles - 1) / tiles);
  if (ks > nt_all / min_kt) ks = nt_all / min_kt;
  if (ks < 2) return p;
  p.ks = ks; p.bm = bm; p.bn = bn;
  return p;
}

#ifdef PSO_BENCH_KNOBS
static int g_tn_split = 0;  // 0 = auto (benchmark knob)  // 0 auto, 1 force 256x128x3, 2 force 128x128x3, 3 force 128x128x2 (benchmarks)
static int g_gemm_group = 0;  // benchmark knob: raster group rows (0 = automatic)
#else
static constexpr int g_tn_split = 0;
static constexpr int g_gemm_group = 0;
#endif
int pso_gemm_group_knob() { return g_gemm_group; }  // gemm8p.hip: a forced group is used as given
// raster group rows: C2-step sweep (tools/_var_ab.sh, same box) 2 / 3 / 4 / 5 / 6 / 8 / 16 -> 240.4 / 239.7 / 239.1 /
// 239.2 / 238.9 / 240.5 / 241.9 ms
#define PSO_GEMM_GROUP_M 4

// the variants 37-58 keep the automatic dispatch and flip one of its rules (41 = per-lane epilogue; 37 / 38 = the
// 256 x 160 8-phase tiles off / forced; 56 = the 256 x 256 TN tiles off; ...); any other non-zero variant forces one tile shape
static int gemm_auto_variant(int gv_raw) { return (gv_raw >= 37 && gv_raw <= 58) ? 0 : gv_raw; }
// the workspace split-K forms (pso_gemm_ws / pso_conv2d_ws) under the benchmark knobs: off where a variant forces a
// tile (38 / 39 / 44: the 8-phase 256 x 160 / 256 x 320 / conv tiles, the tests that pin them), where a raster group
// is forced, and under variant 52 (the conv split off)
static bool gemm_ws_allowed() {
  const int v = g_gemm_variant;
  return g_gemm_group == 0 && gemm_auto_variant(v) == 0 && v != 38 && v != 39 && v != 44 && v != 52;
}

static int run_gemm(GemmArgs& g, hipStream_t st) {
  const int gv_raw = g_gemm_variant;
  const int gv = gemm_auto_variant(gv_raw);
  if (g.M <= 0 || g.N <= 0) return PSO_OK;
  g.group_m = g_gemm_group > 0 ? g_gemm_group : PSO_GEMM_GROUP_M;
  if (g.tail_group_n > 0 && (g.tail_group_n % 64) != 0) {
    pso_set_error("pso_gemm: tail_group_n must be a multiple of 64");
    return PSO_ERR_ARG;
  }
  // staged 16-B epilogue for bf16 outputs with 16-B aligned rows (5-10 % on the K = 640 / 1280 projections with
  // bias + residual, tools/epi_bench.py); variant 41 keeps the per-lane 8-B epilogue (A/B knob)
  g.stage_epi = gv_raw != 41 && g.out_dtype == PSO_BF16 && al16(g.out) && (g.ldo % 8) == 0 &&
                (!g.resid || (al16(g.resid) && (g.ldr % 8) == 0));
  g.vec_ok = (g.ldo % 4) == 0 && (g.out_dtype == PSO_F32 ? al16(g.out) : al8(g.out)) &&
             (!g.resid || ((g.ldr % 4) == 0 && al8(g.resid))) && (!g.bias || al8(g.bias)) &&
             (!g.rowbias || (al8(g.rowbias) && (g.ld_rowbias % 4) == 0));
  const bool bn64_only = g.tail_group_n > 0 && (g.tail_group_n % 128) != 0;  // grouped tail needs BN | group
  const bool bn256_ok = g.tail_group_n == 0 || (g.tail_group_n % 256) == 0;
  const long Ktot = (long)g.K1 + (g.a2 ? g.K2 : 0);
  if (g.batch > 1) {  // batched dense product (the VAE's single-head mid attention): the 2-phase tiles only
    auto tl = [&](int bm, int bn) { return (long)((g.M + bm - 1) / bm) * ((g.N + bn - 1) / bn) * g.batch; };
    if ((g.N % 160) == 0 && tl(128, 160) >= 256) return launch<128, 160, 2, 2, 2>(g, st);
    if (tl(128, 128) >= 256) return launch<128, 128, 2, 4, 2>(g, st);
    return launch<64, 64>(g, st);
  }
  // deterministic split-K through the caller's workspace (pso_gemm_ws): small M x N, long K
  if (g.ws) {
    const SplitPlan sp = gemm_split_plan(g.M, g.N, g.K1, g.K2, g.a2 != nullptr, true);  // entries checked the form
    if (sp.ks >= 2) {
      if (sp.bn == 160) launch<128, 160, 2, 2, 2>(g, st, sp.ks);
      else launch<128, 128, 2, 4, 2>(g, st, sp.ks);
      const long n4 = (long)g.M * (g.N / 4);
      gemm_splitk_reduce_kernel<<<(unsigned)((n4 + 255) / 256), 256, 0, st>>>(g, sp.ks);
      return pso_check_launch("pso_gemm_ws");
    }
    g.ws = nullptr;
  }
  // Skinny N (the LoRA rank-r products): one 16-row x all-N tile per 4-wave block, K split over the waves.
  if (gv == 0 && !g.conv.mode && !g.a2 && !g.bias && !g.rowbias && !g.resid && g.N <= 128 &&
      (g.N % 4) == 0 && g.vec_ok && g.M >= 256)
    return pso_gemm_skinny_nt(g.M, g.N, g.K1, g.a1, g.lda1, g.b1, g.ldb1, g.alpha, g.out, g.ldo,
                              g.out_dtype == PSO_F32, g.accumulate, 1, st);
  // Small outputs with a long reduction: split K over blocks, f32 atomics in the epilogue.
  const bool can_split = g.out_dtype == PSO_F32 && g.accumulate && !g.bias && !g.rowbias && !g.resid &&
                         !g.conv.mode && g.tail_group_n == 0;
  if (can_split && (g.M <= 128 || g.N <= 128) && Ktot >= 2048) {
    const long tiles = (long)((g.M + 63) / 64) * ((g.N + 63) / 64);
    const long ktiles = (Ktot + BK - 1) / BK;
    long ks = (512 + tiles - 1) / tiles;
    if (ks > ktiles / 2) ks = ktiles / 2;
    if (ks < 1) ks = 1;
    return launch<64, 64>(g, st, (int)ks);
  }
  // 3x3 / stride 1 / pad 1 convolutions (the ResNet convs and their input gradients) on the 8-phase 256 x 320 tiles
  // (gemm8p.hip CONV form) wherever they fill a round of CUs; variant 43 keeps them on the 2-phase kernel, 44 forces it
  {
    const ConvGeom& cv = g.conv;
    const long hw = (long)cv.Ho * cv.Wo;
    const bool conv8 = cv.mode == PSO_CONV_NORMAL && cv.ks == 3 && cv.stride == 1 && cv.pad == 1 && cv.H == cv.Ho &&
                       cv.W == cv.Wo && cv.C2 == 0 && (cv.C1 % 64) == 0 && cv.C1 <= 4096 && (hw % 256) == 0 &&
                       (cv.H & (cv.H - 1)) == 0 && (cv.W & (cv.W - 1)) == 0 && cv.W >= 8 &&
                       (g.N % 320) == 0 && !g.a2 && g.out_dtype == PSO_BF16 && !g.accumulate && al16(g.out) &&
                       (g.ldo % 8) == 0 && (!g.resid || (al16(g.resid) && (g.ldr % 8) == 0)) &&
                       (!g.bias || al8(g.bias)) && (!g.rowbias || (al8(g.rowbias) && g.rows_per_group == hw)) &&
                       fits30((long)g.M + 2L * (cv.W + 1), cv.C1) && fits30(g.N, g.ldb1) && al16(g.a1) && al16(g.b1);
    const long t320c = (long)(g.M / 256) * (g.N / 320);
    const long min320c = (gv_raw == 46 || gv_raw == 47) ? 256 : 192;
    if (conv8 && gv_raw != 43 && (gv_raw == 44 || (gv == 0 && t320c >= min320c)))
      return pso_gemm8p320_conv_run(g.M / (int)hw, cv.H, cv.W, cv.C1, g.a1, g.b1, g.N, g.alpha, g.bias, g.rowbias,
                                    g.ld_rowbias, g.resid, g.ldr, g.out, g.ldo, g.group_m, st);
  }
  // 8-phase 256x256 (gemm8p.hip, wave groups staggered) for dense bf16 GEMMs with N % 256 == 0: LDS-staged 16-B
  // epilogue, LoRA K-tail, bias / alpha / residual.  Default for N >= 2560 with >= 256 tiles (tools/gemm8_ab.py, one
  // box: q/k/v 16384 x 3840 x 1280 1071 vs 937 TF/s, ff.out dX 8192 x 5120 x 1280 991 vs 945); N = 1280 keeps 128x160
  // (1.25 rounds of 256x256 tiles at M = 16384: 805 vs 928).  Variant 30 forces it, 31 keeps it off everywhere.
  const bool base8 = !g.conv.mode && !g.rowbias && g.out_dtype == PSO_BF16 && !g.accumulate && (g.K1 % 64) == 0 &&
                     al16(g.a1) && al16(g.b1) && (g.lda1 % 8) == 0 && (g.ldb1 % 8) == 0 && al16(g.out) &&
                     (g.ldo % 8) == 0 && (!g.resid || (al16(g.resid) && (g.ldr % 8) == 0)) &&
                     (!g.bias || al8(g.bias)) && fits30(g.M, g.lda1) && fits30(g.N, g.ldb1) &&
                     (!g.a2 || (fits30(g.tail_m, g.lda2) && fits30(g.N, g.ldb2)));
  const bool ok8 = base8 && (g.N % 256) == 0 && (!g.a2 || g.tail_group_n == 0 || (g.tail_group_n % 256) == 0);
  const long t256 = (long)((g.M + 255) / 256) * (g.N / 256);
  // wide N (>= 2560) whose 256 x 256 tiles leave a partial round while the 256 x 320 ones make whole rounds (C3's
  // 6144 x 10240 x 1280: 960 vs 768 tiles, 979 vs 1079 TF/s; 24576 x 5120 x 640: 802 vs 832) take the 320 form below;
  // variant 46 keeps the round-2 rules
  const bool ok320w = base8 && (g.N % 320) == 0 && g.lda1 == g.ldb1 && (!g.a2 || g.K2 <= 64) &&
                      (!g.a2 || g.tail_group_n == 0 || (g.tail_group_n % 320) == 0);
  const long t320w = (long)((g.M + 255) / 256) * (g.N / 320);
  const bool wide320 = gv == 0 && gv_raw != 46 && ok320w && g.N >= 2560 && (t256 % 256) != 0 && t320w >= 256 &&
                       (t320w % 256) == 0;
  // three quarters of a round of 256 x 256 tiles where the 256 x 320 ones leave more CUs idle (C4's 12288 x 1280:
  // 240 vs 192 tiles, 1056 vs 877-919 TF/s; bs = 1's q/k/v 4096 x 3840: 240 tiles, 938 vs 798 on the 2-phase
  // tiles; tools/small_m_bench.py); variant 50 keeps the full-round rule
  const long t320r = (g.N % 320) == 0 ? (long)((g.M + 255) / 256) * (g.N / 320) : 0;
  const bool part256 = gv == 0 && gv_raw != 50 && t256 >= 192 && t256 < 256 && t256 > t320r;
  if (ok8 && !wide320 && (gv == 30 || part256 || ((gv == 32 || (gv == 0 && g.N >= 2560)) && t256 >= 256)))
    return pso_gemm8p_run(0, g.M, g.N, g.K1, g.a1, g.lda1, g.b1, g.ldb1, g.a2, g.lda2, g.K2, g.b2, g.ldb2, g.tail_m,
                          g.tail_group_n, g.alpha, g.bias, g.resid, g.ldr, g.out, g.ldo, nullptr, 0, 0, nullptr, 0,
                          g.group_m, st);
  // 8-phase 256 x 160 (gemm8p.hip) for the N % 160 == 0 widths with at least one round of tiles and a long reduction
  // (K >= 2560: ff.out 16384 x 1280 x 5120 972 vs 942 TF/s, 32768 x 640 x 5120 1039 vs 910, 65536 x 640 x 2560 823
  // vs 770); at K = 640 / 1280 the 2-phase 128 x 160 with two co-resident blocks per CU (one block's epilogue beside
  // the other's main loop) stays ahead (16384 x 1280 x 1280 827 vs 724, tools/shape_prof.py one box).  Variant 37
  // keeps the 2-phase 128 x 160, 38 forces the 8-phase form wherever it applies.
  // 8-phase 256 x 320 (gemm8p.hip): every SDXL width is a multiple of 320, and at the UNet's M (256 * 2^k rows) the
  // tile count is a whole number of 256-CU rounds (N = 1280 at M = 16384: 256 tiles; N = 640 at M = 65536: 512).
  // Default where it fills at least one round and the reduction is short (K < 2560: the 256 x 160 persistent form
  // keeps the long ones); at half a round (M = 8192, N = 1280: 128 tiles) the 2-phase 128 x 160 stays ahead
  // (tools/shape_prof.py, one box: 16384 x 1280 x 1280 + LoRA 922 vs 816 TF/s, 65536 x 640 x 640 + LoRA 700 vs 652,
  // 65536 x 1920 x 640 + LoRA 849 vs 783; 8192 x 1280 x 1280 + LoRA 574 vs 776).  Variant 39 forces it, 40 keeps it
  // off.
  const bool ok320 = base8 && (g.N % 320) == 0 && g.lda1 == g.ldb1 && (!g.a2 || g.K2 <= 64) &&
                     (!g.a2 || g.tail_group_n == 0 || (g.tail_group_n % 320) == 0);
  const long t320 = (long)((g.M + 255) / 256) * (g.N / 320);
  // three quarters of a round already beats the 2-phase tiles (C4's 12288 x 1280 x 5120: 1072 vs 811 TF/s, x 1280:
  // 875 vs 830; C3's 24576 x 640 x 2560: 1034 vs 725, x 640: 685 vs 612 -- 192 tiles each); half a round does not
  // (8192 x 1280 x 1280: 574 vs 776).  Variant 46 / 47 keep the full-round rule.
  const long min320 = (gv_raw == 46 || gv_raw == 47) ? 256 : 192;
  if (ok320 && gv_raw != 40 && gv_raw != 38 &&
      (gv_raw == 39 || wide320 ||
       (gv == 0 && t320 >= min320 && g.N < 2560 && (gv_raw != 42 || Ktot < 2560))))
    return pso_gemm8p320_run(g.M, g.N, g.K1, g.a1, g.lda1, g.b1, g.ldb1, g.a2, g.lda2, g.K2, g.b2, g.ldb2, g.tail_m,
                             g.tail_group_n, g.alpha, g.bias, g.resid, g.ldr, g.out, g.ldo, g.group_m, st);
  const bool ok160 = base8 && (g.N % 160) == 0 && (!g.a2 || g.tail_group_n == 0 || (g.tail_group_n % 160) == 0);
  const long t160 = (long)((g.M + 255) / 256) * (g.N / 160);
  if (ok160 && gv_raw != 37 && (gv_raw == 38 || (gv == 0 && t160 >= 256 && Ktot >= 2560)))
    return pso_gemm8p160_run(g.M, g.N, g.K1, g.a1, g.lda1, g.b1, g.ldb1, g.a2, g.lda2, g.K2, g.b2, g.ldb2, g.tail_m,
                             g.tail_group_n, g.alpha, g.bias, g.resid, g.ldr, g.out, g.ldo, g.group_m, st);
  const bool n160 = (g.N % 160) == 0 && (g.tail_group_n == 0 || (g.tail_group_n % 160) == 0);
#ifdef PSO_BENCH_KNOBS  // forced tile shapes (A/B and tests of the knobs build)
  if (gv == 4 && bn256_ok) return launch<256, 256, 2, 4, 2>(g, st);
  if (gv == 5 && !bn64_only) return launch<256, 128, 2, 4, 2>(g, st);
  if (gv == 1 && !bn64_only) return launch<256, 128, 4, 2, 3>(g, st);
  if (gv == 2 && !bn64_only) return launch<128, 128, 2, 2, 3>(g, st);
  if (gv == 3 && !bn64_only) return launch<128, 128>(g, st);
  if (gv == 6 && !bn64_only) return launch<64, 128>(g, st);
  if (gv == 7 && bn256_ok) return launch<128, 256, 2, 4, 2>(g, st);
  if (gv == 8 && !bn64_only) return launch<128, 128, 2, 4, 2>(g, st);
  if (gv == 10 && bn256_ok) return launch<256, 256, 2, 4, 2, true>(g, st);
  if (gv == 11 && !bn64_only) return launch<128, 128, 2, 4, 2, true>(g, st);
  const bool n320 = (g.N % 320) == 0 && (g.tail_group_n == 0 || (g.tail_group_n % 320) == 0);
  if (gv == 12 && n160) return launch<128, 160, 2, 2, 2>(g, st);
  if (gv == 14 && n160) return launch<256, 160, 2, 2, 2>(g, st);
  if (gv == 16 && n160) return launch<256, 160, 2, 2, 2, true>(g, st);
  if (gv == 17 && n320) return launch<128, 320, 2, 4, 2>(g, st);
  if (gv == 18 && n320) return launch<256, 320, 2, 4, 2>(g, st);
  if (gv == 19 && n160) return launch<128, 160, 2, 2, 2, true>(g, st);
  // small-M tiles (the bs = 1 backward at M = 2048: N = 1280 makes exactly one 256-CU round of 64 x 160 / 128 x 80)
  if (gv == 20 && n160) return launch<64, 160, 2, 2, 2>(g, st);
  if (gv == 21 && (g.N % 80) == 0 && (g.tail_group_n % 80) == 0) return launch<128, 80, 4, 1, 2>(g, st);
  if (gv == 22 && n160) return launch<64, 160, 2, 2, 3>(g, st);
  // deeper direct-to-LDS rings for the latency-bound short-K small-M products (4 / 5 stages: 3 / 4 K-tiles in flight)
  if (gv == 23 && n160) return launch<64, 160, 2, 2, 4>(g, st);
  if (gv == 24 && n160) return launch<64, 160, 2, 2, 5>(g, st);
  if (gv == 25 && !bn64_only) return launch<64, 64, 2, 2, 4>(g, st);
  if (gv == 26 && n160) return launch<128, 160, 2, 2, 4>(g, st);
  if (gv == 27 && !bn64_only) return launch<64, 128, 2, 2, 4>(g, st);
  if (gv == 28 && !bn64_only) return launch<128, 128, 2, 4, 4>(g, st);
  if (gv == 29 && !bn64_only) return launch<64, 64, 2, 2, 5>(g, st);
#endif
  // Tile choice by occupancy (~2 co-resident 4-wave blocks per CU, 256 CUs): large grids keep 128x128 (best operand
  // reuse); grids that would leave CUs idle drop to 64x128 / 128x64 / 64x64 (e.g. the L2 projections, M=4096 N=1280,
  // and the skinny LoRA projections N = r..3r).
  auto tiles = [&](int bm, int bn) { return (long)((g.M + bm - 1) / bm) * ((g.N + bn - 1) / bn); };
  if (g.N <= 64) return launch<64, 64>(g, st);
  if (bn64_only) return tiles(128, 64) >= 512 ? launch<128, 64>(g, st) : launch<64, 64>(g, st);
  if (g.M <= 64) return launch<64, 128>(g, st);
  // 256x256 block tile, 8 waves x (128x64): twice the MFMAs per LDS fragment read; wins once the grid covers the 256
  // CUs (one 128 KiB-LDS block per CU) and N has no partial 256-column tile; implicit-GEMM convs (long K) already
  // at half a wave of blocks.  Otherwise 128x128 with 8 waves (64x32 each).  Measured on the UNet shapes at 8 images
  // (tools/gemm_bench.py): e.g. L2 qkv 8192x3840x1280 713 vs 645 TF/s; L2 proj 8192x1280x1280 531 vs 474.
  // Very large grids (>= 4 rounds of 256x256 tiles: L1/L2 ff.proj, the 128^2 upsample conv) keep 256x256.  Otherwise
  // N % 160 == 0 (every SDXL width: 320 | N) takes 128x160 with 4 waves of 64x80: fewer LDS bytes per MFMA than the
  // 8-wave 128x128 (64x32 wave tiles) and tile counts that divide the 512 co-resident slots (M=8192, N=1280 -> 512
  // tiles).  tools/gemm_bench.py at 8 images: L2 ff.out 8192x1280x5120 797 -> 1097 TF/s, L2 proj 636 -> 816,
  // L0/L1/L2 3x3 convs 733/887/795 -> 921/994/1005.
  if (bn256_ok && (g.N % 256) == 0 && tiles(256, 256) >= 1024) return launch<256, 256, 2, 4, 2>(g, st);
  // 128 x 160 tiles that leave a quarter of the 512 co-resident slots empty while 128 x 128 ones nearly fill them
  // (C3's 6144-row L2 products, N = 1280: 384 vs 480 tiles; proj 678 -> 753 TF/s, ff.out 860 -> 971, GEGLU dX
  // 940 -> 1023, 3x3 conv 802 -> 864): the 8-wave 128 x 128 kernel.  At half the slots (4096 x 1280, the bs=1 LoRA
  // pass: 256 vs 320 tiles) 128 x 160 stays ahead (step 90.5 vs 93.2 ms).  Variant 46 keeps the 128 x 160 choice.
  if (gv_raw != 46 && !bn64_only && n160 && tiles(128, 160) >= 384 && tiles(128, 160) < 512 &&
      tiles(128, 128) <= 512)
    return launch<128, 128, 2, 4, 2>(g, st);
  // 128 x 160 tiles that make at most one workgroup per CU while 64 x 160 ones make 1.5-2 (the bs = 1 / GPU pass:
  // 4096 x 1280 and 8192 x 640 rows; tools/small_m_bench.py, one box: 4096 x 1280 x 5120 837 vs 755 TF/s, x 1280 + LoRA
  // 649 vs 540, 8192 x 640 x 5120 843 vs 759, x 1920 + LoRA 718 vs 637); variant 48 keeps 128 x 160 there
  if (gv_raw != 48 && n160 && tiles(128, 160) <= 256 && tiles(64, 160) >= 384) return launch<64, 160, 2, 2, 2>(g, st);
  // smaller still (M = 2048, N = 1280: 256 tiles of 64 x 160, 640 of 64 x 64), short K (the long ones split K through
  // a workspace, pso_gemm_ws): variant 49 takes the register-pipelined 8-wave 128 x 128 tiles. They win in isolation
  // (tools/small_m_bench.py: 2048 x 1280 x 1280 + LoRA 404 vs 319 TF/s) but lose inside the bs = 1 step
  // (tools/shape_prof.py, one box: 252-256 vs 277 TF/s), so 64 x 64 stays the default there
#ifdef PSO_BENCH_KNOBS
  if (gv_raw == 49 && !g.conv.mode && !bn64_only && (g.N % 128) == 0 && tiles(64, 160) <= 256 &&
      tiles(128, 128) >= 128 && tiles(128, 160) < 256)
    return launch<128, 128, 2, 4, 2, true>(g, st);
#endif
  if (n160 && tiles(128, 160) >= 256) return launch<128, 160, 2, 2, 2>(g, st);
  if (bn256_ok && (g.N % 256) == 0 && tiles(256, 256) >= (g.conv.mode ? 128 : 256))
    return launch<256, 256, 2, 4, 2>(g, st);
  if (tiles(128, 128) >= 256) return launch<128, 128, 2, 4, 2>(g, st);
  if (tiles(64, 128) >= 512) return (g.N % 128 == 0) ? launch<64, 128>(g, st) : launch<128, 64>(g, st);
  return launch<64, 64>(g, st);
}

// =====================================================================================================================
// TN GEMM: out[I][J] (+)= alpha * sum_m A[m][I] * B[m][J]   (both operands "token-major": the reduction index is the
// row index).  This is the shape of every LoRA weight gradient (dA = v^T x, dB = s dy^T u, reduction over the
// B*S tokens); it replaces two explicit transposes per product.  Tiles of 64 (m) rows x 64 columns are staged
// row-major in LDS with the chunk ^ (2*((row>>1)&3)) swizzle and read as MFMA fragments with ds_read_b64_tr_b16
// (lane i of a 16-lane group receives column i of 4 consecutive rows = 4 consecutive k of one output row).
// Split-K over gridDim.y with f32 atomics in the epilogue (output is always an f32 accumulator).
// =====================================================================================================================
typedef __attribute__((address_space(3))) s16x4 lds_s16x4_g;
typedef __attribute__((address_space(3))) void tnr_lds_void_g;
__device__ __forceinline__ int swz_tr64(int r, int c) { return r * 64 + ((c ^ (((r >> 1) & 3) << 1)) << 3); }

__device__ __forceinline__ s16x4 tr_read64(const bf16_t* img, int r0, int col0, int lane) {
  const int li = lane & 15;
  const int q = li >> 2, p = li & 3;
  const int col = col0 + 4 * p;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_g*)(img + swz_tr64(r0 + q, col >> 3) + (col & 7)));
}

__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(int M, int I, int J, const bf16_t* __restrict__ A, long lda,
                                                         const bf16_t* __restrict__ B, long ldb, float alpha,
                                                         float* __restrict__ out, long ldo,
                                                         float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) bf16_t sA[2][64 * 64];
  __shared__ __attribute__((aligned(16))) bf16_t sB[2][64 * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave >> 1, wj = wave & 1;
  const int nbj = (J + 63) / 64;
  const int bi = blockIdx.x / nbj, bj = blockIdx.x - bi * nbj;
  const int i0 = bi * 64, j0 = bj * 64;
  const int nkt = (M + 63) / 64;
  const int per = (nkt + gridDim.y - 1) / gridDim.y;
  const int t_beg = blockIdx.y * per, t_end = min(nkt, t_beg + per);
  uint4 ra[2], rb[2];
  auto load = [&](int t) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q = tid + 256 * h;
      const int row = q >> 3, ch = q & 7;
      const int m = t * 64 + row;
      const int ci = i0 + ch * 8, cj = j0 + ch * 8;
      ra[h] = (m < M && ci < I) ? *reinterpret_cast<const uint4*>(A + (long)m * lda + ci) : make_uint4(0, 0, 0, 0);
      rb[h] = (m < M && cj < J) ? *reinterpret_cast<const uint4*>(B + (long)m * ldb + cj) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q = tid + 256 * h;
      const int row = q >> 3, ch = q & 7;
      *reinterpret_cast<uint4*>(sA[buf] + swz_tr64(row, ch)) = ra[h];
      *reinterpret_cast<uint4*>(sB[buf] + swz_tr64(row, ch)) = rb[h];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, c = lane & 15;
  if (t_beg < t_end) {
    load(t_beg);
    store(0);
  }
  __syncthreads();
  for (int t = t_beg; t < t_end; ++t) {
    const int cur = (t - t_beg) & 1;
    if (t + 1 < t_end) load(t + 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int col = wi * 32 + a * 16;
        typedef __attribute__((ext_vector_type(8))) short s16x8;
        const s16x4 x0 = tr_read64(sA[cur], ks * 32 + 8 * g, col, lane);
        const s16x4 x1 = tr_read64(sA[cur], ks * 32 + 8 * g + 4, col, lane);
        s16x8 v = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
        af[a] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int col = wj * 32 + b * 16;
        typedef __attribute__((ext_vector_type(8))) short s16x8;
        const s16x4 y0 = tr_read64(sB[cur], ks * 32 + 8 * g, col, lane);
        const s16x4 y1 = tr_read64(sB[cur], ks * 32 + 8 * g + 4, col, lane);
        s16x8 v = {y0[0], y0[1], y0[2], y0[3], y1[0], y1[1], y1[2], y1[3]};
        bfr[b] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[b], af[a], acc[a][b], 0, 0, 0);
    }
    if (t + 1 < t_end) store(cur ^ 1);
    __syncthreads();
  }
  // lane holds out[i = i0 + wi*32 + a*16 + c][j = j0 + wj*32 + b*16 + 4g + r]
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int i = i0 + wi * 32 + a * 16 + c;
    if (i >= I) continue;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int j = j0 + wj * 32 + b * 16 + 4 * g;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (j + r < J) {
          float* o = out + (long)i * ldo + j + r;
          if (part) part[((long)blockIdx.y * I + i) * J + j + r] = acc[a][b][r] * alpha;  // ordered-reduction slice
          else if (gridDim.y > 1) atomicAdd(o, acc[a][b][r] * alpha);
          else *o += acc[a][b][r] * alpha;
        }
    }
  }
}

// 128 x 128 TN tile for the full-weight gradients (C3 / C4: dW = X^T dY over the B*H*W tokens, I, J >= 128):
// 4 waves of 64 x 64 (4 x 4 MFMA tiles, every operand fragment feeds four MFMAs), 64-token K-steps staged by
// buffer_load ... lds (each wave one 64 x 64 image: A cols i0.. / i0+64.., B cols j0.. / j0+64..; source-side
// swizzle for the transposed reads; rows past M read as zeros) through a 2-stage ring, fragments by inline-asm
// ds_read_b64_tr_b16 (the builtin makes hipcc drain the LDS-DMA ring).  Split-K over gridDim.y with f32 atomics.
__device__ __forceinline__ s16x4 tn_tr_asm(unsigned img_base, int r0, int col0, int lane) {
  const int li = lane & 15;
  const int q = li >> 2, p = li & 3;
  const int col = col0 + 4 * p;
  const unsigned addr = img_base + 2u * (unsigned)(swz_tr64(r0 + q, col >> 3) + (col & 7));
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

__global__ __launch_bounds__(256, 2) void gemm_tn128_kernel(int M, int I, int J, const bf16_t* __restrict__ A,
                                                            long lda, const bf16_t* __restrict__ B, long ldb,
                                                            float alpha, float* __restrict__ out, long ldo,
                                                            int steps, float* __restrict__ part, int geglu_f = 0) {
  __shared__ __attribute__((aligned(16))) bf16_t sT[2][4][64 * 64];  // [stage][A0 A1 B0 B1], 64 KB
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave >> 1, wj = wave & 1;
  const int g = lane >> 4, c = lane & 15;
  const int nbj = (J + 127) / 128;
  const int bi = blockIdx.x / nbj, bj = blockIdx.x - bi * nbj;
  const int i0 = bi * 128, j0 = bj * 128;
  const int nkt = (M + 63) / 64;
  const int t_beg = blockIdx.y * steps, t_end = min(nkt, t_beg + steps);
  // wave w stages image w: A (w < 2) or B, 64 columns from col0, all 8 pieces of 8 rows x 128 B
  const bool isA = wave < 2;
  const long ld = isA ? lda : ldb;
  const int col0 = (isA ? i0 : j0) + (wave & 1) * 64;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(isA ? A : B), (short)0, (int)(((long)(M - 1) * ld + (isA ? I : J)) * 2), 0x00020000);
  const int prow = lane >> 3, pch = lane & 7;
  const int sc = pch ^ (((prow >> 1) & 3) << 1);  // source chunk landing at LDS chunk pch (swz_tr64)
  // columns past I / J are clamped to the last 8 (their products land in unstored outputs)
  const int cw = min(col0 + sc * 8, (isA ? I : J) - 8);
  const unsigned voff = (unsigned)((long)prow * ld + cw) * 2u;
  const int kstep = (int)(64 * ld * 2);
  auto issue = [&](int t, int stg) {
#pragma unroll
    for (int p = 0; p < 8; ++p)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (tnr_lds_void_g*)(sT[stg][wave] + p * 8 * 64), 16,
                                               voff + (unsigned)(p * 8 * ld * 2), t * kstep, 0, 0);
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned lbase = (unsigned)(uintptr_t)(const tnr_lds_void_g*)&sT[0][0][0];
  if (t_beg < t_end) issue(t_beg, 0);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  for (int t = t_beg; t < t_end; ++t) {
    const int cur = (t - t_beg) & 1;
    if (t + 1 < t_end) issue(t + 1, cur ^ 1);
    const unsigned ia = lbase + (unsigned)((cur * 4 + wi) * 64 * 64 * 2);
    const unsigned ib = lbase + (unsigned)((cur * 4 + 2 + wj) * 64 * 64 * 2);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      s16x4 ra[8], rb[8];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        ra[2 * a] = tn_tr_asm(ia, ks * 32 + 8 * g, a * 16, lane);
        ra[2 * a + 1] = tn_tr_asm(ia, ks * 32 + 8 * g + 4, a * 16, lane);
        rb[2 * a] = tn_tr_asm(ib, ks * 32 + 8 * g, a * 16, lane);
        rb[2 * a + 1] = tn_tr_asm(ib, ks * 32 + 8 * g + 4, a * 16, lane);
      }
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(ra[0]), "+v"(ra[1]), "+v"(ra[2]), "+v"(ra[3]), "+v"(ra[4]), "+v"(ra[5]), "+v"(ra[6]),
                     "+v"(ra[7]), "+v"(rb[0]), "+v"(rb[1]), "+v"(rb[2]), "+v"(rb[3]), "+v"(rb[4]), "+v"(rb[5]),
                     "+v"(rb[6]), "+v"(rb[7]));
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        typedef __attribute__((ext_vector_type(8))) short s16x8;
        s16x8 va = {ra[2 * a][0], ra[2 * a][1], ra[2 * a][2], ra[2 * a][3],
                    ra[2 * a + 1][0], ra[2 * a + 1][1], ra[2 * a + 1][2], ra[2 * a + 1][3]};
        s16x8 vb = {rb[2 * a][0], rb[2 * a][1], rb[2 * a][2], rb[2 * a][3],
                    rb[2 * a + 1][0], rb[2 * a + 1][1], rb[2 * a + 1][2], rb[2 * a + 1][3]};
        af[a] = __builtin_bit_cast(bf16x8, va);
        bfr[a] = __builtin_bit_cast(bf16x8, vb);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[b], af[a], acc[a][b], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    // the next stage landed (every wave's pieces), and every wave's reads of this stage retired before it is restaged
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // lane holds out[i = i0 + wi*64 + a*16 + c][j = j0 + wj*64 + b*16 + 4g + r]
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int i = i0 + wi * 64 + a * 16 + c;
    if (i >= I) continue;
    // geglu_f > 0: A's columns are the GEGLU interleave (per 32 outputs [h 32 | gate 32]); row i of the product goes
    // to row (i / 64) * 32 + i % 32 of the natural [h | gate] order, plus geglu_f for the gate half
    const int io = geglu_f > 0 ? ((i >> 6) << 5) + (i & 31) + ((i & 32) ? geglu_f : 0) : i;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int j = j0 + wj * 64 + b * 16 + 4 * g;
      if (j >= J) continue;  // J % 8 == 0: a lane's 4 columns are all in or all out
      float* o = out + (long)io * ldo + j;
      if (part) {  // this slice's partial product, stored (added into out by tn_reduce_slices_kernel)
        *reinterpret_cast<float4*>(part + ((long)blockIdx.y * I + i) * J + j) =
            make_float4(acc[a][b][0] * alpha, acc[a][b][1] * alpha, acc[a][b][2] * alpha, acc[a][b][3] * alpha);
      } else if (gridDim.y > 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) atomicAdd(o + r, acc[a][b][r] * alpha);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] += acc[a][b][r] * alpha;
      }
    }
  }
}

// out[i][j] += sum over the ks slices of part[s][i][j], in slice order (4 consecutive j per thread)
__global__ void tn_reduce_slices_kernel(int I, int J, int ks, const float* __restrict__ part, float* __restrict__ out,
                                        long ldo) {
  const long q = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long n4 = (long)I * J / 4;
  if (q >= n4) return;
  const long e = q * 4;
  const int i = (int)(e / J), j = (int)(e - (long)i * J);
  float4 sacc = *reinterpret_cast<const float4*>(part + e);
  for (int sl = 1; sl < ks; ++sl) {
    const float4 v = *reinterpret_cast<const float4*>(part + (long)sl * I * J + e);
    sacc.x += v.x; sacc.y += v.y; sacc.z += v.z; sacc.w += v.w;
  }
  float* o = out + (long)i * ldo + j;
  o[0] += sacc.x; o[1] += sacc.y; o[2] += sacc.z; o[3] += sacc.w;
}

// 256 x 256 TN tile for the large full-weight gradients: 8 waves of 64 x 128 (4 x 8 MFMA tiles; each A fragment
// feeds 8 MFMAs, each B fragment 4), the same per-wave 64 x 64 images and transposed reads as gemm_tn128_kernel.  A
// 128 x 128 tile moves 32 KB of operands per 2.1 MFLOP (one 64-token step) -- ~38 TB/s of L2 reads at the MFMA peak
// over 256 CUs, more than the L2s deliver; the 256 x 256 tile halves the bytes per flop.  One workgroup per CU
// (128 KB LDS: 2 stages x 8 images).  part != nullptr: this slice's partial product into the workspace (ordered
// reduction by tn_reduce_slices_kernel); else out += directly (the caller launches one slice).
__global__ __launch_bounds__(512, 1) void gemm_tn256_kernel(int M, int I, int J, const bf16_t* __restrict__ A,
                                                            long lda, const bf16_t* __restrict__ B, long ldb,
                                                            float alpha, float* __restrict__ out, long ldo,
                                                            int steps, float* __restrict__ part, int geglu_f) {
  extern __shared__ __attribute__((aligned(16))) bf16_t t256s[];  // [stage][A0 A1 A2 A3 B0 B1 B2 B3][64 x 64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave >> 1, wj = wave & 1;
  const int g = lane >> 4, c = lane & 15;
  const int nbj = (J + 255) / 256;
  const int bi = blockIdx.x / nbj, bj = blockIdx.x - bi * nbj;
  const int i0 = bi * 256, j0 = bj * 256;
  const int nkt = (M + 63) / 64;
  const int t_beg = blockIdx.y * steps, t_end = min(nkt, t_beg + steps);
  // wave w stages image w: A columns i0 + 64 w (w < 4) or B columns j0 + 64 (w - 4), 8 pieces of 8 rows x 128 B
  const bool isA = wave < 4;
  const long ld = isA ? lda : ldb;
  const int col0 = (isA ? i0 : j0) + (wave & 3) * 64;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(isA ? A : B), (short)0, (int)(((long)(M - 1) * ld + (isA ? I : J)) * 2), 0x00020000);
  const int prow = lane >> 3, pch = lane & 7;
  const int sc = pch ^ (((prow >> 1) & 3) << 1);
  const int cw = min(col0 + sc * 8, (isA ? I : J) - 8);
  const unsigned voff = (unsigned)((long)prow * ld + cw) * 2u;
  const int kstep = (int)(64 * ld * 2);
  auto issue = [&](int t, int stg) {
#pragma unroll
    for (int p = 0; p < 8; ++p)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (tnr_lds_void_g*)(t256s + (stg * 8 + wave) * 4096 + p * 8 * 64), 16,
                                               voff + (unsigned)(p * 8 * ld * 2), t * kstep, 0, 0);
  };
  f32x4 acc[4][8];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned lbase = (unsigned)(uintptr_t)(const tnr_lds_void_g*)t256s;
  if (t_beg < t_end) issue(t_beg, 0);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  for (int t = t_beg; t < t_end; ++t) {
    const int cur = (t - t_beg) & 1;
    if (t + 1 < t_end) issue(t + 1, cur ^ 1);
    const unsigned ia = lbase + (unsigned)((cur * 8 + wi) * 4096 * 2);
    const unsigned ib = lbase + (unsigned)((cur * 8 + 4 + 2 * wj) * 4096 * 2);  // images 4 + 2 wj, 5 + 2 wj
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      s16x4 ra[8], rb[16];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        ra[2 * a] = tn_tr_asm(ia, ks * 32 + 8 * g, a * 16, lane);
        ra[2 * a + 1] = tn_tr_asm(ia, ks * 32 + 8 * g + 4, a * 16, lane);
      }
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const unsigned im = ib + (unsigned)((b >> 2) * 4096 * 2);
        rb[2 * b] = tn_tr_asm(im, ks * 32 + 8 * g, (b & 3) * 16, lane);
        rb[2 * b + 1] = tn_tr_asm(im, ks * 32 + 8 * g + 4, (b & 3) * 16, lane);
      }
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(ra[0]), "+v"(ra[1]), "+v"(ra[2]), "+v"(ra[3]), "+v"(ra[4]), "+v"(ra[5]), "+v"(ra[6]),
                     "+v"(ra[7]), "+v"(rb[0]), "+v"(rb[1]), "+v"(rb[2]), "+v"(rb[3]));
      asm volatile(""
                   : "+v"(rb[4]), "+v"(rb[5]), "+v"(rb[6]), "+v"(rb[7]), "+v"(rb[8]), "+v"(rb[9]), "+v"(rb[10]),
                     "+v"(rb[11]), "+v"(rb[12]), "+v"(rb[13]), "+v"(rb[14]), "+v"(rb[15]));
      typedef __attribute__((ext_vector_type(8))) short s16x8;
      bf16x8 af[4], bfr[8];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        s16x8 va = {ra[2 * a][0], ra[2 * a][1], ra[2 * a][2], ra[2 * a][3],
                    ra[2 * a + 1][0], ra[2 * a + 1][1], ra[2 * a + 1][2], ra[2 * a + 1][3]};
        af[a] = __builtin_bit_cast(bf16x8, va);
      }
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        s16x8 vb = {rb[2 * b][0], rb[2 * b][1], rb[2 * b][2], rb[2 * b][3],
                    rb[2 * b + 1][0], rb[2 * b + 1][1], rb[2 * b + 1][2], rb[2 * b + 1][3]};
        bfr[b] = __builtin_bit_cast(bf16x8, vb);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[b], af[a], acc[a][b], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // lane holds out[i = i0 + wi*64 + a*16 + c][j = j0 + wj*128 + b*16 + 4g + r]
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int i = i0 + wi * 64 + a * 16 + c;
    if (i >= I) continue;
    const int io = geglu_f > 0 ? ((i >> 6) << 5) + (i & 31) + ((i & 32) ? geglu_f : 0) : i;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int j = j0 + wj * 128 + b * 16 + 4 * g;
      if (j >= J) continue;
      if (part) {
        *reinterpret_cast<float4*>(part + ((long)blockIdx.y * I + i) * J + j) =
            make_float4(acc[a][b][0] * alpha, acc[a][b][1] * alpha, acc[a][b][2] * alpha, acc[a][b][3] * alpha);
      } else {
        float* o = out + (long)io * ldo + j;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] += acc[a][b][r] * alpha;
      }
    }
  }
}

// the 256 x 256 TN tiles (variant 56 keeps the 128 x 128 ones): both sides multiples of 256 and the operands within
// 32-bit buffer offsets.  Returns the slice count: 1 where the tiles alone cover >= 3/4 of the CUs (out += directly);
// one round of workspace slices of >= 8 K-steps each where the 128 x 128 tiles would run one pass of 256-383
// workgroups (< 3/4 of the two-per-CU slots, and too many for tn_ws_slices); else 0 = not this kernel.
// tools/tn_full_bench.py, TF/s 256 vs 128 tiles: 6144 x 1280 x 11520 (225 tiles) 948 / 929 vs 835 / 836, 24576 x 1280
// x 11520 990 vs 823, the GEGLU 6144 x 10240 x 1280 (200 tiles) 720 / 736 vs 658 / 725, 6144 x 3840 x 1280 (75 tiles x
// 3 slices) 675 / 683 vs 607 / 616; slices where the 128 x 128 tiles already fill the slots lose (6144 x 1280 x 5120,
// 100 tiles x 2: 670 vs 752; 6144 x 1280 x 1280, 25 x 10: 411 vs 471): the partials' round trip through HBM.
static int tn256_slices(int M, int I, int J, long lda, long ldb) {
  if (g_gemm_variant == 56 || I % 256 || J % 256 || (long)M * lda >= (1L << 30) || (long)M * ldb >= (1L << 30))
    return 0;
  const int t256 = (I / 256) * (J / 256);
  if (t256 >= 192) return 1;
  const int t128 = (I / 128) * (J / 128);
  if (t128 < 256 || t128 >= 384) return 0;
  const int nkt = (M + 63) / 64;
  int ks = 256 / t256;
  if (ks > nkt / 8) ks = nkt / 8;
  if (ks < 2) return 0;
  const int steps = (nkt + ks - 1) / ks;
  return (nkt + steps - 1) / steps;
}

static void tn256_launch(int M, int I, int J, const void* A, long lda, const void* B, long ldb, float alpha, float* out,
                         long ldo, int ks, float* part, int geglu_f, hipStream_t st) {
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)gemm_tn256_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    return true;
  }();
  (void)attr;
  const int nkt = (M + 63) / 64;
  const int steps = (nkt + ks - 1) / ks;
  pso_note_kernel("gemm_tn256_kernel");
  gemm_tn256_kernel<<<dim3((I / 256) * (J / 256), ks), 512, 131072, st>>>(M, I, J, (const bf16_t*)A, lda,
                                                                          (const bf16_t*)B, ldb, alpha, out, ldo,
                                                                          steps, part, geglu_f);
}

// split of the full-weight TN product into ks slices of the reduction rows for the workspace form: enough slices for
// ~1.5 rounds of 128 x 128 tiles over the 256 CUs, each slice >= 8 K-steps (512 rows)
static int tn_ws_slices(int M, int I, int J) {
  if (I < 128 || J < 128) return 0;
  const int t128 = ((I + 127) / 128) * ((J + 127) / 128);
  if (t128 >= 256) return 0;
  const int nkt = (M + 63) / 64;
  int ks = (384 + t128 - 1) / t128;
  if (ks > nkt / 8) ks = nkt / 8;
  return ks >= 2 ? ks : 0;
}

// Deterministic plan of a TN product with a caller-owned workspace (pso_gemm_tn_ws): every split of the reduction
// rows stores its partial product and the partials are added in split order -- no f32 atomics anywhere.
//   TNP_RANK:  one side a rank-16/32/64/96 projection -> the rank-r streaming kernel's workspace form
//   TNP_128:   both sides >= 128 wide -> 128 x 128 tiles, ks slices (the small-weight split of tn_ws_slices, else the
//              split the atomic form would take)
//   TNP_64:    the rest -> 64 x 64 tiles, ks slices
//   TNP_PLAIN: no split: out += directly (deterministic as it stands)
//   TNP_256:   both sides multiples of 256 with too few tiles for the CUs -> 256 x 256 tiles, one round of slices
enum { TNP_PLAIN = 0, TNP_RANK = 1, TNP_128 = 2, TNP_64 = 3, TNP_256 = 4 };
struct TnPlan { int kind, ks, steps; size_t bytes; };
static bool tn_rank_ok(int r) { return r == 16 || r == 32 || r == 64 || r == 96; }
static TnPlan tn_plan(int M, int I, int J, long lda, long ldb) {
  TnPlan p{TNP_PLAIN, 1, 0, 0};
  if (M <= 0) return p;
  if ((I % 128 == 0 && tn_rank_ok(J)) || (J % 128 == 0 && tn_rank_ok(I))) {
    const bool x_is_a = I % 128 == 0 && tn_rank_ok(J);
    PsoTnRankProblem q{};
    q.x = (const void*)16; q.u = (const void*)16; q.out = (float*)16; q.ldx = 8; q.ldu = 8;
    q.ldo = x_is_a ? J : I; q.M = M; q.C = x_is_a ? I : J; q.group_c = 0; q.alpha = 1.f;
    p.kind = TNP_RANK;
    p.bytes = pso_gemm_tn_rank_batch_ws_bytes(x_is_a ? J : I, x_is_a ? 0 : 1, 1, &q);
    return p;
  }
  const int nkt = (M + 63) / 64;
  const int ks256 = tn256_slices(M, I, J, lda, ldb);
  if (ks256 == 1) return p;  // the direct 256 x 256 form (pso_gemm_tn_grouped)
  if (ks256 >= 2) {
    p.kind = TNP_256;
    p.ks = ks256;
    p.steps = (nkt + ks256 - 1) / ks256;
    p.bytes = (size_t)ks256 * I * J * sizeof(float);
    return p;
  }
  if (I >= 128 && J >= 128 && (long)M * lda < (1L << 30) && (long)M * ldb < (1L << 30)) {
    int ks = tn_ws_slices(M, I, J);
    if (!ks) {  // the split the atomic form takes (pso_gemm_tn_grouped): ks <= M / 16384 where it yields >= 128 blocks
      const int t128 = ((I + 127) / 128) * ((J + 127) / 128);
      ks = (512 + t128 - 1) / t128;
      if (ks > M / 16384) ks = M / 16384;
      if (ks < 1) ks = 1;
      const int st0 = (nkt + ks - 1) / ks;
      ks = (nkt + st0 - 1) / st0;
      if (t128 * ks < 128) ks = 0;  // the 64 x 64 kernel's domain
    }
    if (ks >= 2) {
      p.kind = TNP_128;
      p.steps = (nkt + ks - 1) / ks;
      p.ks = (nkt + p.steps - 1) / p.steps;
      p.bytes = (size_t)p.ks * I * J * sizeof(float);
      return p;
    }
    if (ks == 1) return p;
  }
  const int tiles = ((I + 63) / 64) * ((J + 63) / 64);
  int ks = (160 + tiles - 1) / tiles;
  if (ks > nkt) ks = nkt;
  if (ks >= 2) {
    p.kind = TNP_64;
    p.ks = ks;
    p.bytes = (size_t)ks * I * J * sizeof(float);
  }
  return p;
}

extern "C" {

size_t pso_gemm_tn_ws_bytes(int M, int I, int J) { return tn_plan(M, I, J, I, J).bytes; }

int pso_gemm_tn_ws(int M, int I, int J, const void* A, long lda, const void* B, long ldb, float alpha, float* out,
                   long ldo, void* ws, size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(M >= 0 && I > 0 && J > 0 && A && B && out, "pso_gemm_tn_ws: bad args");
  PSO_ARG_CHECK(((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0 && (lda % 8) == 0 && (ldb % 8) == 0 &&
                    (I % 8) == 0 && (J % 8) == 0,
                "pso_gemm_tn_ws: operands need 16-B aligned rows and I, J multiples of 8");
  if (M == 0) return PSO_OK;
  const hipStream_t st = (hipStream_t)stream;
  const TnPlan p = tn_plan(M, I, J, lda, ldb);
  const bool ws_ok = ws && p.bytes && ws_bytes >= p.bytes && (((uintptr_t)ws) & 15) == 0 && g_tn_split == 0;
  if (p.kind == TNP_RANK && ws_ok) {
    const bool x_is_a = I % 128 == 0 && tn_rank_ok(J);
    PsoTnRankProblem q{};
    q.x = x_is_a ? A : B; q.ldx = x_is_a ? lda : ldb;
    q.u = x_is_a ? B : A; q.ldu = x_is_a ? ldb : lda;
    q.out = out; q.ldo = ldo; q.M = M; q.C = x_is_a ? I : J; q.group_c = 0; q.alpha = alpha;
    return pso_gemm_tn_rank_batch_ws(x_is_a ? J : I, x_is_a ? 0 : 1, 1, &q, ws, ws_bytes, stream);
  }
  if ((p.kind == TNP_128 || p.kind == TNP_64 || p.kind == TNP_256) && ws_ok) {
    const long n4 = (long)I * J / 4;
    if (p.kind == TNP_256) {
      tn256_launch(M, I, J, A, lda, B, ldb, alpha, out, ldo, p.ks, (float*)ws, 0, st);
    } else if (p.kind == TNP_128) {
      const int t128 = ((I + 127) / 128) * ((J + 127) / 128);
      pso_note_kernel("gemm_tn128_kernel");
      gemm_tn128_kernel<<<dim3(t128, p.ks), 256, 0, st>>>(M, I, J, (const bf16_t*)A, lda, (const bf16_t*)B, ldb, alpha,
                                                          out, ldo, p.steps, (float*)ws);
    } else {
      const int tiles = ((I + 63) / 64) * ((J + 63) / 64);
      pso_note_kernel("gemm_tn_kernel");
      gemm_tn_kernel<<<dim3(tiles, p.ks), 256, 0, st>>>(M, I, J, (const bf16_t*)A, lda, (const bf16_t*)B, ldb, alpha,
                                                        out, ldo, (float*)ws);
    }
    tn_reduce_slices_kernel<<<(unsigned)((n4 + 255) / 256), 256, 0, st>>>(I, J, p.ks, (const float*)ws, out, ldo);
    return pso_check_launch("pso_gemm_tn_ws");
  }
  return pso_gemm_tn_grouped(M, I, J, A, lda, B, ldb, alpha, out, ldo, 0, stream);
}

int pso_gemm(int M, int N, const void* a1, long lda1, int K1, const void* b1, long ldb1, const void* a2, long lda2,
             int K2, const void* b2, long ldb2, float alpha, const void* bias, const void* rowbias, long ld_rowbias,
             int rows_per_group, const void* resid, long ldr, void* out, long ldo, int out_dtype, int accumulate,
             int tail_group_n, int tail_rows, void* stream) {
  PSO_ARG_CHECK(M >= 0 && N >= 0 && K1 >= 0 && (K1 % 8) == 0, "pso_gemm: need K1 %% 8 == 0 (K1=%d)", K1);
  PSO_ARG_CHECK(a1 && b1 && out, "pso_gemm: null operand");
  PSO_ARG_CHECK(al16(a1) && al16(b1) && (lda1 % 8) == 0 && (ldb1 % 8) == 0, "pso_gemm: A1/B1 must be 16-B aligned rows");
  PSO_ARG_CHECK(!a2 || (b2 && (K2 % 8) == 0 && al16(a2) && al16(b2) && (lda2 % 8) == 0 && (ldb2 % 8) == 0),
                "pso_gemm: bad second operand");
  PSO_ARG_CHECK(out_dtype == PSO_BF16 || out_dtype == PSO_F32, "pso_gemm: bad out dtype");
  PSO_ARG_CHECK((long)M * lda1 < 0x7fffffffL && (long)N * ldb1 < 0x7fffffffL,
                "pso_gemm: operand spans more than 2^31 elements");
  PSO_ARG_CHECK(!accumulate || out_dtype == PSO_F32, "pso_gemm: accumulate needs f32 output");
  PSO_ARG_CHECK(!rowbias || rows_per_group > 0, "pso_gemm: rowbias needs rows_per_group > 0");
  GemmArgs g{};
  g.a1 = (const bf16_t*)a1; g.lda1 = lda1; g.K1 = K1;
  g.b1 = (const bf16_t*)b1; g.ldb1 = ldb1;
  g.a2 = (const bf16_t*)a2; g.lda2 = lda2; g.K2 = a2 ? K2 : 0;
  g.b2 = (const bf16_t*)b2; g.ldb2 = ldb2;
  g.tail_group_n = a2 ? tail_group_n : 0;
  g.tail_m = (tail_rows > 0 && tail_rows < M) ? tail_rows : M;
  g.M = M; g.N = N;
  g.alpha = alpha;
  g.bias = (const bf16_t*)bias;
  g.rowbias = (const bf16_t*)rowbias; g.ld_rowbias = ld_rowbias; g.rows_per_group = rows_per_group > 0 ? rows_per_group : 1;
  g.resid = (const bf16_t*)resid; g.ldr = ldr;
  g.out = out; g.ldo = ldo; g.out_dtype = out_dtype; g.accumulate = accumulate;
  return run_gemm(g, (hipStream_t)stream);
}

size_t pso_gemm_ws_bytes(int M, int N, int K1, int K2) {
  const SplitPlan sp = gemm_split_plan(M, N, K1, K2, K2 > 0, true);
  return sp.ks >= 2 ? (size_t)sp.ks * M * N * sizeof(float) : 0;
}

int pso_gemm_ws(int M, int N, const void* a1, long lda1, int K1, const void* b1, long ldb1, const void* a2, long lda2,
                int K2, const void* b2, long ldb2, float alpha, const void* bias, const void* rowbias, long ld_rowbias,
                int rows_per_group, const void* resid, long ldr, void* out, long ldo, int out_dtype, int accumulate,
                int tail_group_n, int tail_rows, void* ws, size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(M >= 0 && N >= 0 && K1 >= 0 && (K1 % 8) == 0, "pso_gemm_ws: need K1 %% 8 == 0 (K1=%d)", K1);
  PSO_ARG_CHECK(a1 && b1 && out, "pso_gemm_ws: null operand");
  PSO_ARG_CHECK(al16(a1) && al16(b1) && (lda1 % 8) == 0 && (ldb1 % 8) == 0, "pso_gemm_ws: A1/B1 must be 16-B aligned rows");
  PSO_ARG_CHECK(!a2 || (b2 && (K2 % 8) == 0 && al16(a2) && al16(b2) && (lda2 % 8) == 0 && (ldb2 % 8) == 0),
                "pso_gemm_ws: bad second operand");
  PSO_ARG_CHECK(out_dtype == PSO_BF16 || out_dtype == PSO_F32, "pso_gemm_ws: bad out dtype");
  PSO_ARG_CHECK((long)M * lda1 < 0x7fffffffL && (long)N * ldb1 < 0x7fffffffL,
                "pso_gemm_ws: operand spans more than 2^31 elements");
  PSO_ARG_CHECK(!accumulate || out_dtype == PSO_F32, "pso_gemm_ws: accumulate needs f32 output");
  PSO_ARG_CHECK(!rowbias || rows_per_group > 0, "pso_gemm_ws: rowbias needs rows_per_group > 0");
  GemmArgs g{};
  g.a1 = (const bf16_t*)a1; g.lda1 = lda1; g.K1 = K1;
  g.b1 = (const bf16_t*)b1; g.ldb1 = ldb1;
  g.a2 = (const bf16_t*)a2; g.lda2 = lda2; g.K2 = a2 ? K2 : 0;
  g.b2 = (const bf16_t*)b2; g.ldb2 = ldb2;
  g.tail_group_n = a2 ? tail_group_n : 0;
  g.tail_m = (tail_rows > 0 && tail_rows < M) ? tail_rows : M;
  g.M = M; g.N = N;
  g.alpha = alpha;
  g.bias = (const bf16_t*)bias;
  g.rowbias = (const bf16_t*)rowbias; g.ld_rowbias = ld_rowbias; g.rows_per_group = rows_per_group > 0 ? rows_per_group : 1;
  g.resid = (const bf16_t*)resid; g.ldr = ldr;
  g.out = out; g.ldo = ldo; g.out_dtype = out_dtype; g.accumulate = accumulate;
  // the workspace form applies when the plan splits and the caller's workspace holds every split; else pso_gemm
  const SplitPlan sp = gemm_split_plan(M, N, K1, a2 ? K2 : 0, a2 != nullptr, true);
  const bool ok = ws && (((uintptr_t)ws) & 15) == 0 && sp.ks >= 2 && ws_bytes >= (size_t)sp.ks * M * N * sizeof(float) &&
                  (ldo % 4) == 0 && (out_dtype == PSO_F32 ? al16(out) : al8(out)) && (g.tail_group_n % sp.bn) == 0 &&
                  gemm_ws_allowed();
  g.ws = ok ? (float*)ws : nullptr;
  return run_gemm(g, (hipStream_t)stream);
}

int pso_gemm_batched(int batch, int M, int N, int K, const void* a, long lda, long stride_a, const void* b, long ldb,
                     long stride_b, float alpha, void* out, long ldo, long stride_o, int out_dtype, void* stream) {
  PSO_ARG_CHECK(batch >= 1 && M >= 0 && N >= 0 && K >= 0 && (K % 8) == 0, "pso_gemm_batched: bad shape (K %% 8 == 0)");
  PSO_ARG_CHECK(a && b && out, "pso_gemm_batched: null operand");
  PSO_ARG_CHECK(al16(a) && al16(b) && (lda % 8) == 0 && (ldb % 8) == 0 && (stride_a % 8) == 0 && (stride_b % 8) == 0,
                "pso_gemm_batched: A/B need 16-B aligned rows and batch strides");
  PSO_ARG_CHECK(out_dtype == PSO_BF16 || out_dtype == PSO_F32, "pso_gemm_batched: bad out dtype");
  PSO_ARG_CHECK((long)M * lda < 0x7fffffffL && (long)N * ldb < 0x7fffffffL,
                "pso_gemm_batched: one operand spans more than 2^31 elements");
  GemmArgs g{};
  g.a1 = (const bf16_t*)a; g.lda1 = lda; g.K1 = K;
  g.b1 = (const bf16_t*)b; g.ldb1 = ldb;
  g.M = M; g.N = N; g.tail_m = M;
  g.alpha = alpha; g.rows_per_group = 1;
  g.out = out; g.ldo = ldo; g.out_dtype = out_dtype;
  g.bat_a = stride_a; g.bat_b = stride_b; g.bat_o = stride_o; g.batch = batch;
  return run_gemm(g, (hipStream_t)stream);
}

int pso_conv2d(int mode, int B, const void* src1, int C1, const void* src2, int C2, int H, int W, int Ho, int Wo,
               int ks, int stride, int pad, const void* weight, int Cout, const void* a2, long lda2, int K2,
               const void* b2, long ldb2, float alpha, const void* bias, const void* rowbias, long ld_rowbias,
               const void* resid, long ldr, void* out, long ldo, int out_dtype, int accumulate, void* stream) {
  PSO_ARG_CHECK(mode == PSO_CONV_NORMAL || mode == PSO_CONV_UP2 || mode == PSO_CONV_T2, "pso_conv2d: bad mode");
  PSO_ARG_CHECK(src1 && weight && out, "pso_conv2d: null operand");
  PSO_ARG_CHECK((C1 % 64) == 0 && (C2 % 64) == 0 && (C2 == 0 || src2),
                "pso_conv2d: channel sources must be multiples of 64 (C1=%d C2=%d); use im2col for small C", C1, C2);
  PSO_ARG_CHECK(al16(src1) && (!src2 || al16(src2)) && al16(weight), "pso_conv2d: alignment");
  PSO_ARG_CHECK(ks == 1 || ks == 3, "pso_conv2d: ks must be 1 or 3");
  PSO_ARG_CHECK(mode != PSO_CONV_UP2 || (Ho == 2 * H && Wo == 2 * W && stride == 1), "pso_conv2d: UP2 geometry");
  PSO_ARG_CHECK(!a2 || ((K2 % 8) == 0 && b2 && al16(a2) && al16(b2)), "pso_conv2d: bad second operand");
  PSO_ARG_CHECK(!accumulate || out_dtype == PSO_F32, "pso_conv2d: accumulate needs f32 output");
  // Cout <= 3 (the VAE decoder's conv_out to RGB): a direct convolution instead of an N = 3 GEMM padded to 64-column
  // MFMA tiles (conv_small.hip; 1024^2: 1.34 ms -> see DESIGN §4 / profiles/r06_vae_conv_out_ab.log)
  if (mode == PSO_CONV_NORMAL && ks == 3 && stride == 1 && pad == 1 && Ho == H && Wo == W && C2 == 0 && !a2 &&
      !rowbias && !resid && alpha == 1.f && out_dtype == PSO_BF16 && !accumulate && ldo == Cout && Cout <= 3 &&
      pso_conv3x3_smallc_run(B, H, W, C1, Cout, src1, weight, bias, out, (hipStream_t)stream) == PSO_OK)
    return PSO_OK;
  GemmArgs g{};
  const int Ct = C1 + C2;
  g.a1 = (const bf16_t*)src1; g.lda1 = 0; g.K1 = ks * ks * Ct;
  g.b1 = (const bf16_t*)weight; g.ldb1 = g.K1;
  g.a2 = (const bf16_t*)a2; g.lda2 = lda2; g.K2 = a2 ? K2 : 0;
  g.b2 = (const bf16_t*)b2; g.ldb2 = ldb2;
  g.M = B * Ho * Wo; g.N = Cout;
  g.tail_m = g.M;
  g.conv.mode = mode; g.conv.src2 = (const bf16_t*)src2; g.conv.C1 = C1; g.conv.C2 = C2;
  g.conv.H = H; g.conv.W = W; g.conv.Ho = Ho; g.conv.Wo = Wo; g.conv.ks = ks; g.conv.stride = stride; g.conv.pad = pad;
  g.alpha = alpha;
  g.bias = (const bf16_t*)bias;
  g.rowbias = (const bf16_t*)rowbias; g.ld_rowbias = ld_rowbias; g.rows_per_group = Ho * Wo;
  g.resid = (const bf16_t*)resid; g.ldr = ldr;
  g.out = out; g.ldo = ldo; g.out_dtype = out_dtype; g.accumulate = accumulate;
  return run_gemm(g, (hipStream_t)stream);
}

size_t pso_conv2d_ws_bytes(int B, int Ho, int Wo, int Cout, int K1, int K2) {
  const long M = (long)B * Ho * Wo;
  if (M <= 0 || M > 0x7fffffffL) return 0;
  const SplitPlan sp = gemm_split_plan((int)M, Cout, K1, K2, K2 > 0, true);
  return sp.ks >= 2 ? (size_t)sp.ks * M * Cout * sizeof(float) : 0;
}

int pso_conv2d_ws(int mode, int B, const void* src1, int C1, const void* src2, int C2, int H, int W, int Ho, int Wo,
                  int ks, int stride, int pad, const void* weight, int Cout, const void* a2, long lda2, int K2,
                  const void* b2, long ldb2, float alpha, const void* bias, const void* rowbias, long ld_rowbias,
                  const void* resid, long ldr, void* out, long ldo, int out_dtype, int accumulate, void* ws,
                  size_t ws_bytes, void* stream) {
  PSO_ARG_CHECK(mode == PSO_CONV_NORMAL || mode == PSO_CONV_UP2 || mode == PSO_CONV_T2, "pso_conv2d_ws: bad mode");
  PSO_ARG_CHECK(src1 && weight && out, "pso_conv2d_ws: null operand");
  PSO_ARG_CHECK((C1 % 64) == 0 && (C2 % 64) == 0 && (C2 == 0 || src2),
                "pso_conv2d_ws: channel sources must be multiples of 64 (C1=%d C2=%d)", C1, C2);
  PSO_ARG_CHECK(al16(src1) && (!src2 || al16(src2)) && al16(weight), "pso_conv2d_ws: alignment");
  PSO_ARG_CHECK(ks == 1 || ks == 3, "pso_conv2d_ws: ks must be 1 or 3");
  PSO_ARG_CHECK(mode != PSO_CONV_UP2 || (Ho == 2 * H && Wo == 2 * W && stride == 1), "pso_conv2d_ws: UP2 geometry");
  PSO_ARG_CHECK(!a2 || ((K2 % 8) == 0 && b2 && al16(a2) && al16(b2)), "pso_conv2d_ws: bad second operand");
  PSO_ARG_CHECK(!accumulate || out_dtype == PSO_F32, "pso_conv2d_ws: accumulate needs f32 output");
  GemmArgs g{};
  const int Ct = C1 + C2;
  g.a1 = (const bf16_t*)src1; g.lda1 = 0; g.K1 = ks * ks * Ct;
  g.b1 = (const bf16_t*)weight; g.ldb1 = g.K1;
  g.a2 = (const bf16_t*)a2; g.lda2 = lda2; g.K2 = a2 ? K2 : 0;
  g.b2 = (const bf16_t*)b2; g.ldb2 = ldb2;
  g.M = B * Ho * Wo; g.N = Cout;
  g.tail_m = g.M;
  g.conv.mode = mode; g.conv.src2 = (const bf16_t*)src2; g.conv.C1 = C1; g.conv.C2 = C2;
  g.conv.H = H; g.conv.W = W; g.conv.Ho = Ho; g.conv.Wo = Wo; g.conv.ks = ks; g.conv.stride = stride; g.conv.pad = pad;
  g.alpha = alpha;
  g.bias = (const bf16_t*)bias;
  g.rowbias = (const bf16_t*)rowbias; g.ld_rowbias = ld_rowbias; g.rows_per_group = Ho * Wo;
  g.resid = (const bf16_t*)resid; g.ldr = ldr;
  g.out = out; g.ldo = ldo; g.out_dtype = out_dtype; g.accumulate = accumulate;
  // the workspace form applies when the plan splits and the workspace holds every split; else the plain conv
  const SplitPlan sp = gemm_split_plan(g.M, g.N, g.K1, g.K2, g.a2 != nullptr, true);
  const bool ok = ws && (((uintptr_t)ws) & 15) == 0 && sp.ks >= 2 && ws_bytes >= (size_t)sp.ks * g.M * g.N * sizeof(float) &&
                  (ldo % 4) == 0 && (out_dtype == PSO_F32 ? al16(out) : al8(out)) && (g.N % 4) == 0 &&
                  (!resid || ((ldr % 4) == 0 && al8(resid))) && (!rowbias || (ld_rowbias % 4) == 0) &&
                  gemm_ws_allowed();
  g.ws = ok ? (float*)ws : nullptr;
  return run_gemm(g, (hipStream_t)stream);
}

int pso_gemm_geglu(int M, int N, const void* a, long lda, int K, const void* w, long ldw, const void* bias, void* out,
                   long ldo, void* out_pre, long ld_pre, int pre_rows, void* stream) {
  PSO_ARG_CHECK(M > 0 && N > 0 && (N % 256) == 0 && K > 0 && (K % 8) == 0 && a && w && bias && out,
                "pso_gemm_geglu: need N %% 256 == 0, K %% 8 == 0, bias");
  PSO_ARG_CHECK(al16(a) && al16(w) && (lda % 8) == 0 && (ldw % 8) == 0 && al16(out) && (ldo % 8) == 0 && al8(bias) &&
                    (!out_pre || (al16(out_pre) && (ld_pre % 8) == 0)),
                "pso_gemm_geglu: alignment (16-B rows)");
  PSO_ARG_CHECK((long)M * lda < 0x7fffffffL && (long)N * ldw < 0x7fffffffL, "pso_gemm_geglu: operand too large");
  GemmArgs g{};
  g.a1 = (const bf16_t*)a; g.lda1 = lda; g.K1 = K;
  g.b1 = (const bf16_t*)w; g.ldb1 = ldw;
  g.M = M; g.N = N; g.alpha = 1.f;
  g.bias = (const bf16_t*)bias;
  g.out = out; g.ldo = ldo; g.out_dtype = PSO_BF16;
  g.out2 = out_pre; g.ldo2 = ld_pre;
  g.tail_m = (pre_rows > 0 && pre_rows < M) ? pre_rows : M;
  g.vec_ok = 1; g.rows_per_group = 1;
  g.group_m = g_gemm_group > 0 ? g_gemm_group : PSO_GEMM_GROUP_M;
  // the 8-phase kernel with the LDS-staged epilogue (gemm8p.hip): 16384 x 10240 x 1280 1023 vs 801 TF/s,
  // 65536 x 5120 x 640 814 vs 640 (tools/gemm_bench.py, one box), inside the C2 step 1006 vs 922 / 801 vs 706
  // (tools/shape_prof.py); variant 31 keeps the 2-phase 256x256 kernel
  // 256 x 320 tiles where they cost fewer tile-rounds than 256 x 256 (rounds x tile width: bs = 1's 4096 x 10240:
  // 2 x 320 < 3 x 256; C3's 6144 x 10240: 3 x 320 < 4 x 256; C5's 2048 x 10240: 1 x 320 < 2 x 256; equal at C2's
  // whole-round shapes, which keep 256 x 256); same bits either way.  Variant 57 keeps 256 x 256.
  if (g_gemm_variant != 31 && g_gemm_variant != 57 && (K % 64) == 0 && (N % 320) == 0 && lda == ldw &&
      fits30(M, lda) && fits30(N, ldw)) {
    const long r256 = ((long)((M + 255) / 256) * (N / 256) + 255) / 256, r320 = ((long)((M + 255) / 256) * (N / 320) + 255) / 256;
    // variant 58 (knob): 256 x 320 at equal rounds too (C2's shapes)
    if (r320 * 320 < r256 * 256 || (g_gemm_variant == 58 && r320 * 320 == r256 * 256))
      return pso_gemm8p320_geglu_run(M, N, K, a, lda, w, ldw, bias, out, ldo, out_pre, ld_pre, g.tail_m, g.group_m,
                                     (hipStream_t)stream);
  }
  if (g_gemm_variant != 31 && (K % 64) == 0 && fits30(M, lda) && fits30(N, ldw))
    return pso_gemm8p_run(1, M, N, K, a, lda, w, ldw, nullptr, 0, 0, nullptr, 0, 0, 0, 1.f, bias, nullptr, 0, out, ldo,
                          out_pre, ld_pre, g.tail_m, nullptr, 0, g.group_m, (hipStream_t)stream);
#ifdef PSO_BENCH_KNOBS  // tile A/B knobs (64-column wave tiles are what the interleaved epilogue needs)
  if (g_gemm_variant == 33) return launch<128, 128, 2, 2, 2, false, EPI_GEGLU>(g, (hipStream_t)stream);
  if (g_gemm_variant == 34) return launch<128, 256, 2, 4, 2, false, EPI_GEGLU>(g, (hipStream_t)stream);
  if (g_gemm_variant == 35) return launch<256, 128, 4, 2, 2, false, EPI_GEGLU>(g, (hipStream_t)stream);
  if (g_gemm_variant == 36) return launch<128, 128, 2, 2, 3, false, EPI_GEGLU>(g, (hipStream_t)stream);
#endif
  return launch<256, 256, 2, 4, 2, false, EPI_GEGLU>(g, (hipStream_t)stream);
}

int pso_gemm_geglu_bwd(int M, int N, const void* a, long lda, int K, const void* w, long ldw, const void* pre,
                       long ld_pre, void* out, long ldo, void* stream) {
  PSO_ARG_CHECK(M > 0 && N > 0 && (N % 32) == 0 && K > 0 && (K % 8) == 0 && a && w && pre && out,
                "pso_gemm_geglu_bwd: need N %% 32 == 0, K %% 8 == 0");
  PSO_ARG_CHECK(al16(a) && al16(w) && (lda % 8) == 0 && (ldw % 8) == 0 && al16(out) && (ldo % 8) == 0 && al16(pre) &&
                    (ld_pre % 8) == 0,
                "pso_gemm_geglu_bwd: alignment (16-B rows)");
  PSO_ARG_CHECK((long)M * lda < 0x7fffffffL && (long)N * ldw < 0x7fffffffL, "pso_gemm_geglu_bwd: operand too large");
  GemmArgs g{};
  g.a1 = (const bf16_t*)a; g.lda1 = lda; g.K1 = K;
  g.b1 = (const bf16_t*)w; g.ldb1 = ldw;
  g.M = M; g.N = N; g.alpha = 1.f;
  g.out = out; g.ldo = ldo; g.out_dtype = PSO_BF16;
  g.aux = (const bf16_t*)pre; g.ldaux = ld_pre;
  g.vec_ok = 1; g.rows_per_group = 1;
  g.group_m = g_gemm_group > 0 ? g_gemm_group : PSO_GEMM_GROUP_M;
  const hipStream_t st = (hipStream_t)stream;
  // 256 x 320 tiles where they make whole rounds the 256 x 256 ones do not (8192 x 5120: 512 tiles = 2 rounds vs 640 =
  // 2.5; 32768 x 2560: 1024 = 4 vs 1280 = 5); variant 45 keeps the 256 x 256 form
  if (g_gemm_variant != 45 && g_gemm_variant != 31 && (N % 320) == 0 && (K % 64) == 0 && lda == ldw && fits30(M, lda) &&
      fits30(N, ldw) && ((long)((M + 255) / 256) * (N / 320)) % 256 == 0)
    return pso_gemm8p320_geglu_bwd_run(M, N, K, a, lda, w, ldw, pre, ld_pre, out, ldo, g.group_m, st);
  // 8-phase form (staggered wave groups) by default: 716 vs 658 TF/s for the 2-phase 128x160 kernel at
  // 16384 x 5120 x 1280, 489 vs 472 at 65536 x 2560 x 640 (tools/gemm_bench.py, one box); variant 31 keeps 128x160
  // (from two rounds of tiles: below that the 2-phase 128 x 160 tiles with two workgroups per CU win -- bs = 1's
  // 2048 x 5120 x 1280 620 vs 493-522 TF/s, C3's 6144 x 5120 x 1280 719 vs 680; tools/small_m_bench.py GEGLU_BWD=1)
  if (g_gemm_variant != 31 && (N % 256) == 0 && (K % 64) == 0 && fits30(M, lda) &&
      fits30(N, ldw) && (long)((M + 255) / 256) * (N / 256) >= 512)
    return pso_gemm8p_run(2, M, N, K, a, lda, w, ldw, nullptr, 0, 0, nullptr, 0, 0, 0, 1.f, nullptr, nullptr, 0, out,
                          ldo, nullptr, 0, 0, pre, ld_pre, g.group_m, st);
  const long t160 = (long)((M + 127) / 128) * ((N + 159) / 160);
  if ((N % 160) == 0 && t160 >= 256) return launch<128, 160, 2, 2, 2, false, EPI_GEGLU_BWD>(g, st);
  return launch<64, 64, 2, 2, 2, false, EPI_GEGLU_BWD>(g, st);
}

#ifdef PSO_BENCH_KNOBS
void pso_gemm_set_variant(int v) {
  g_gemm_variant = v % 100;
  g_gemm_group = v / 100;
}
#endif

int pso_gemm_skinny_grouped(int M, int N, int K, const void* A, long lda, const void* W, long ldw, float alpha,
                            void* out, long ldo, int groups, void* stream) {
  PSO_ARG_CHECK(M > 0 && N > 0 && N <= 128 && (N % 4) == 0 && K > 0 && (K % 8) == 0 && groups >= 1 && A && W && out,
                "pso_gemm_skinny_grouped: need 0 < N <= 128, N %% 4 == 0, K %% 8 == 0");
  PSO_ARG_CHECK(al16(A) && al16(W) && (lda % 8) == 0 && (ldw % 8) == 0 && al8(out) && (ldo % 4) == 0,
                "pso_gemm_skinny_grouped: alignment");
  return pso_gemm_skinny_nt(M, N, K, A, lda, W, ldw, alpha, out, ldo, 0, 0, groups, (hipStream_t)stream);
}

int pso_gemm_tn(int M, int I, int J, const void* A, long lda, const void* B, long ldb, float alpha, float* out,
                long ldo, void* stream) {
  return pso_gemm_tn_grouped(M, I, J, A, lda, B, ldb, alpha, out, ldo, 0, stream);
}
#ifdef PSO_BENCH_KNOBS
void pso_gemm_tn_set_split(int ks) { g_tn_split = ks; }
#endif

int pso_gemm_tn_grouped(int M, int I, int J, const void* A, long lda, const void* B, long ldb, float alpha, float* out,
                        long ldo, int group, void* stream) {
  PSO_ARG_CHECK(M >= 0 && I > 0 && J > 0 && A && B && out, "pso_gemm_tn: bad args");
  PSO_ARG_CHECK(al16(A) && al16(B) && (lda % 8) == 0 && (ldb % 8) == 0 && (I % 8) == 0 && (J % 8) == 0,
                "pso_gemm_tn: operands need 16-B aligned rows and I, J multiples of 8");
  if (M == 0) return PSO_OK;
  // One side a rank-r projection (LoRA): the streaming rank kernel.  group > 0 (block-diagonal fused q/k/v): the big
  // side's column c pairs with the small side's columns [(c / group) * r, +r) where r = small width / (big / group).
  auto rk = [](int r) { return r == 16 || r == 32 || r == 64 || r == 96; };
  if (g_tn_split == 0) {
    if (I % 128 == 0 && (group == 0 ? rk(J) : (group % 128 == 0 && I % group == 0 && rk(J / (I / group)))))
      return pso_gemm_tn_rank(M, I, A, lda, B, ldb, group ? J / (I / group) : J, group, alpha, out, ldo, 0,
                              (hipStream_t)stream);
    if (J % 128 == 0 && group == 0 && rk(I))
      return pso_gemm_tn_rank(M, J, B, ldb, A, lda, I, 0, alpha, out, ldo, 1, (hipStream_t)stream);
  }
  PSO_ARG_CHECK(group == 0, "pso_gemm_tn: grouped form needs a rank-32/64/96 side and 128 | group");
  const int nkt = (M + 63) / 64;
  if (g_tn_split == 0 && tn256_slices(M, I, J, lda, ldb) == 1) {
    tn256_launch(M, I, J, A, lda, B, ldb, alpha, out, ldo, 1, nullptr, 0, (hipStream_t)stream);
    return pso_check_launch("pso_gemm_tn");
  }
  // full-weight gradients (both sides >= 128 wide): 128 x 128 tiles; split over M only as far as needed to cover ~2
  // rounds of co-resident blocks (each split adds its tile of f32 atomics)
#ifdef PSO_BENCH_KNOBS
  static const int tn128 = [] {
    const char* e = getenv("PSO_TN128");  // benchmark knob: 0 keeps the 64 x 64 kernel everywhere
    return e ? atoi(e) : 1;
  }();
#else
  constexpr int tn128 = 1;
#endif
  const int t128 = ((I + 127) / 128) * ((J + 127) / 128);
  if (tn128 && g_tn_split == 0 && I >= 128 && J >= 128 && (long)M * lda < (1L << 30) && (long)M * ldb < (1L << 30)) {
    // split over M only while its f32 atomics stay small next to the product: each split adds I*J*4 bytes at the
    // ~1.3 TB/s atomic rate against 2*M*I*J flop, so ks <= M / 16384 keeps them under ~10 %
    int ks = (512 + t128 - 1) / t128;
    if (ks > M / 16384) ks = M / 16384;
    if (ks < 1) ks = 1;
    const int steps = (nkt + ks - 1) / ks;
    ks = (nkt + steps - 1) / steps;
  // fewer than 128 blocks (e.g. 640 x 640 weights: 25 tiles) leave most CUs idle: the 64 x 64 kernel's 4x the tiles
  // win there (C3 step shape_prof: 24576 x 640 x 640 122 vs 59 TF/s, 6144 x 1280 x 1280 234 vs 213; the 128 x 128
  // tiles elsewhere: 6144 x 10240 x 1280 697 vs 417, 98304 x 320 x 2880 485 vs 141, 6144 x 1280 x 11520 815 vs 431)
  if (t128 * ks >= 128) {
    pso_note_kernel("gemm_tn128_kernel");
    gemm_tn128_kernel<<<dim3(t128, ks), 256, 0, (hipStream_t)stream>>>(M, I, J, (const bf16_t*)A, lda,
                                                                        (const bf16_t*)B, ldb, alpha, out, ldo, steps,
                                                                        nullptr);
    return pso_check_launch("pso_gemm_tn");
  }
  }
  const int tiles = ((I + 63) / 64) * ((J + 63) / 64);
  // ~160 blocks: fewer leaves the M-range latency-bound, more multiplies the f32 atomics (measured optimum on the
  // LoRA dW shapes, M = 4096 / 16384, I x J = 1280x32 .. 640x32)
  int ks = g_tn_split > 0 ? g_tn_split : (160 + tiles - 1) / tiles;
  if (ks > nkt) ks = nkt;
  if (ks < 1) ks = 1;
  pso_note_kernel("gemm_tn_kernel");
  gemm_tn_kernel<<<dim3(tiles, ks), 256, 0, (hipStream_t)stream>>>(M, I, J, (const bf16_t*)A, lda, (const bf16_t*)B,
                                                                   ldb, alpha, out, ldo, nullptr);
  return pso_check_launch("pso_gemm_tn");
}

int pso_gemm_tn_geglu(int M, int F2, int J, const void* A, long lda, const void* B, long ldb, float alpha, float* out,
                      long ldo, void* stream) {
  PSO_ARG_CHECK(M >= 0 && F2 > 0 && (F2 % 128) == 0 && J >= 128 && (J % 8) == 0 && A && B && out,
                "pso_gemm_tn_geglu: need 128 | F2 (F2=%d), J >= 128, 8 | J (J=%d)", F2, J);
  PSO_ARG_CHECK(al16(A) && al16(B) && (lda % 8) == 0 && (ldb % 8) == 0, "pso_gemm_tn_geglu: 16-B aligned rows");
  PSO_ARG_CHECK((long)M * lda < (1L << 30) && (long)M * ldb < (1L << 30), "pso_gemm_tn_geglu: operand too large");
  if (M == 0) return PSO_OK;
  // one pass over the reduction rows (no split: += straight into the natural-order gradient, deterministic)
  if (tn256_slices(M, F2, J, lda, ldb) == 1) {
    tn256_launch(M, F2, J, A, lda, B, ldb, alpha, out, ldo, 1, nullptr, F2 / 2, (hipStream_t)stream);
    return pso_check_launch("pso_gemm_tn_geglu");
  }
  const int t128 = (F2 / 128) * ((J + 127) / 128);
  pso_note_kernel("gemm_tn128_kernel");
  gemm_tn128_kernel<<<dim3(t128, 1), 256, 0, (hipStream_t)stream>>>(M, F2, J, (const bf16_t*)A, lda, (const bf16_t*)B,
                                                                     ldb, alpha, out, ldo, (M + 63) / 64, nullptr,
                                                                     F2 / 2);
  return pso_check_launch("pso_gemm_tn_geglu");
}

}  // extern "C"
