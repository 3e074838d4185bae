// 256 x 256 bf16 MFMA GEMM with an 8-phase software pipeline for gfx950, fp32 accumulate.
//
//   out = EPI(A[M][K] . W[N][K]^T + bias)      EPI_NONE: bf16 out[M][N];  EPI_GEGLU: out[M][N/2] = h * gelu(gate)
//   (+ optional interleaved pre-activation rows, see gemm.hip GemmArgs) -- dense operands, no K-tail.
//
// Serves the widest GEMMs of the UNet step: the GEGLU projection ff.net.0.proj (16384 x 10240 x 1280 and
// 65536 x 5120 x 640 in the paired pass; replaces diffusers GEGLU's nn.Linear + gelu).
//
// Structure (one workgroup = 8 waves = a 256 x 256 output tile, 1 per CU):
//   * The K-tile (BK = 64) is split into four half-tile images A0 A1 (rows 0-127 / 128-255) and B0 B1 (columns),
//     16 KB each, and there are two K-tile buffers E (even K-tiles) and O (odd) -> 128 KB of LDS.
//   * A K-tile is consumed in 4 phases, one 128 x 128 C-quadrant each, in the order (A0,B0) (A1,B0) (A1,B1) (A0,B1):
//     inside a quadrant the waves sit 4 (M) x 2 (N), so every wave owns 32 rows x 64 columns = 8 MFMA tiles x K = 64
//     = 16 MFMAs per phase, and its 64 columns are one interleaved [h 32 | gate 32] GEGLU group.  Fragment reads per
//     phase: A 4 + B 8 / A 4 / B 8 / A 4 ds_read_b128 (the other operand stays in registers).
//   * Every phase stages exactly one half-tile (2 glds per thread) into the image whose last read retired a phase
//     earlier (the reads are waited for before the previous phase's MFMAs, which precede its closing barrier):
//         phase:   1      2      3      4      5      6      7      8
//         stage:  O.A0  E'.B0  E'.A1  E'.B1  E'.A0  O'.B0  O'.A1  O'.B1      (E' / O' = the next even / odd K-tile)
//     so three half-tiles stay in flight behind a counted s_waitcnt vmcnt(6) at phases 4 and 8 -- never vmcnt(0) in
//     steady state.  Phase 4's wait retires the odd K-tile (read in phases 5-8), phase 8's the next even one.
//   * Each phase: fragment reads, stage, [vmcnt], s_barrier, 16 MFMAs at raised priority, s_barrier.
// XCD-aware block order and grouped raster as in gemm.hip.
#include "common.h"

#define EPI8_NONE 0
#define EPI8_GEGLU 1

typedef __attribute__((address_space(3))) void lds8_void;

struct Gemm8Args {
  const bf16_t* a; long lda;
  const bf16_t* w; long ldw;
  int M, N, K;
  const bf16_t* bias;
  void* out; long ldo;
  void* out2; long ldo2; int pre_rows;  // EPI_GEGLU: interleaved pre-activation of rows < pre_rows (optional)
  int group_m;
};

namespace {

constexpr int HT = 128 * 64;  // elements of one half-tile image [128 rows][64 k]

__device__ __forceinline__ int swz8(int r, int c) { return r * 64 + ((c ^ (r & 7)) << 3); }

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm8p_kernel(Gemm8Args g) {
  extern __shared__ __attribute__((aligned(16))) bf16_t l8[];  // [2 bufs][A0 A1 B0 B1][HT]
  const int tid = threadIdx.x, lane = tid & 63;
  // wave index in an SGPR: the LDS-DMA destinations (M0) are then scalar arithmetic, not 8 spilled VGPR addresses
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;  // 4 (M) x 2 (N) inside a quadrant
  const int fr = lane & 15, fk = lane >> 4;

  const int nbn = g.N / 256, nbm = (g.M + 255) / 256;
  const int nblk = nbn * nbm;
  int bid = blockIdx.x;
  {
    const int q = nblk / 8, r = nblk % 8, x = bid % 8;
    if (nblk >= 8) bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
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
  const int m0 = bm * 256, n0 = bn * 256;
  const int nt = g.K / 64;  // even (host-checked)

  // staging: wave w fills pieces 2w, 2w+1 (8 rows x 128 B each) of every half-tile image; the XOR swizzle is applied
  // on the source chunk (lane i lands at byte 16 i of its piece).  Rows past M are clamped (never stored).  The loads
  // are buffer_load ... lds against SGPR resources, so the per-lane part of every staging address is one 32-bit byte
  // offset (64-bit per-lane pointers for the 8 source rows spill at this register budget, and a spill reload's
  // vmcnt(0) would drain the whole ring).
  const int prow = lane >> 3, pch = lane & 7;
  unsigned aoff[2][2], woff[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int R = (wave * 2 + i) * 8 + prow;
      const int lc = pch ^ (R & 7);
      aoff[h][i] = (unsigned)(min(m0 + h * 128 + R, g.M - 1) * (int)g.lda + lc * 8) * 2u;
      woff[h][i] = (unsigned)((n0 + h * 128 + R) * (int)g.ldw + lc * 8) * 2u;
    }
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)g.a, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)g.w, (short)0, 0x7fffffff, 0x00020000);
  // image index = buf * 4 + {A0 0, A1 1, B0 2, B1 3}
  auto stage = [&](int kt, int img) {
    const int half = img & 3;
    bf16_t* dst = l8 + img * HT + wave * 2 * 8 * 64;
    const unsigned k0 = (unsigned)kt * 128u;  // bytes
    if (half < 2) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds8_void*)dst, 16, aoff[half][0] + k0, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds8_void*)(dst + 8 * 64), 16, aoff[half][1] + k0, 0, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds8_void*)dst, 16, woff[half - 2][0] + k0, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds8_void*)(dst + 8 * 64), 16, woff[half - 2][1] + k0, 0, 0, 0);
    }
  };

  f32x4 acc[2][2][2][4];  // [A half][B half][row subtile][col subtile]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[2][2], bfr[4][2];  // [row subtile][kk], [col subtile][kk]
  // Fragment addresses: the swizzle term depends only on fr & 7, so within an image a lane needs one byte offset per
  // kk (subtiles are +2048-B immediates).  The image base is added per read by a volatile v_add: left to itself the
  // compiler hoists 8 images x 4 addresses out of the loop and spills at this register budget.
  typedef __attribute__((address_space(3))) const bf16x8 lds_frag;
  const unsigned l8base = (unsigned)(uintptr_t)(lds8_void*)l8;
  unsigned la[2], lb[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    la[kk] = (unsigned)swz8(wr * 32 + fr, kk * 4 + fk) * 2u;
    lb[kk] = (unsigned)swz8(wc * 64 + fr, kk * 4 + fk) * 2u;
  }
  auto read_a = [&](int img) {
    const unsigned ib = l8base + (unsigned)(img * HT * 2);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      unsigned ad;
      asm volatile("v_add_u32 %0, %1, %2" : "=v"(ad) : "s"(ib), "v"(la[kk]));
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i][kk] = *(lds_frag*)(uintptr_t)(ad + i * 2048);
    }
  };
  auto read_b = [&](int img) {
    const unsigned ib = l8base + (unsigned)(img * HT * 2);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      unsigned ad;
      asm volatile("v_add_u32 %0, %1, %2" : "=v"(ad) : "s"(ib), "v"(lb[kk]));
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j][kk] = *(lds_frag*)(uintptr_t)(ad + j * 2048);
    }
  };
  auto mfma_q = [&](int ha, int hb) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[ha][hb][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][kk], af[i][kk], acc[ha][hb][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // one phase: reads (RA / RB: which operand image to (re)load), the stage (if its K-tile exists), the optional
  // counted wait (VM: -1 none, else vmcnt(VM)), barrier, MFMAs of quadrant (HA, HB), barrier.
#define PHASE(BUF, HA, HB, RA, RB, STAGE_KT, STAGE_IMG, VM)                                   \
  {                                                                                           \
    if (RB) read_b((BUF) * 4 + 2 + (HB));                                                     \
    if (RA) read_a((BUF) * 4 + (HA));                                                         \
    if ((STAGE_KT) < nt) stage((STAGE_KT), (STAGE_IMG));                                      \
    if ((VM) == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");                           \
    else if ((VM) == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                      \
    __builtin_amdgcn_s_barrier();                                                             \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    mfma_q((HA), (HB));                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    __builtin_amdgcn_s_barrier();                                                             \
  }

  // prologue: K-tile 0 -> E (in the steady-state staging order), K-tile 1 -> O.B0 O.A1 O.B1; wait for K-tile 0
  stage(0, 2); stage(0, 1); stage(0, 3); stage(0, 0);
  if (nt > 1) { stage(1, 6); stage(1, 5); stage(1, 7); }
  if (nt > 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  for (int j = 0; j < nt; j += 2) {
    const bool last = j + 2 >= nt;
    // even K-tile j in E
    PHASE(0, 0, 0, 1, 1, j + 1, 4, -1)                 // stage O.A0 of K-tile j+1
    PHASE(0, 1, 0, 1, 0, j + 2, 2, -1)                 // E'.B0
    PHASE(0, 1, 1, 0, 1, j + 2, 1, -1)                 // E'.A1
    if (last) { PHASE(0, 0, 1, 1, 0, j + 2, 3, 0) }    // E'.B1 (none past the end); O complete
    else { PHASE(0, 0, 1, 1, 0, j + 2, 3, 6) }
    // odd K-tile j+1 in O
    PHASE(1, 0, 0, 1, 1, j + 2, 0, -1)                 // E'.A0
    PHASE(1, 1, 0, 1, 0, j + 3, 6, -1)                 // O'.B0
    PHASE(1, 1, 1, 0, 1, j + 3, 5, -1)                 // O'.A1
    if (!last) { PHASE(1, 0, 1, 1, 0, j + 3, 7, 6) }   // O'.B1; E' complete
    else { PHASE(1, 0, 1, 1, 0, j + 3, 7, -1) }
  }
#undef PHASE

  // ---- epilogue: lane holds out[m = m0 + 128 ha + 32 wr + 16 i + fr][n = n0 + 128 hb + 64 wc + 16 j + 4 fk + r] ----
  if constexpr (EPI == EPI8_GEGLU) {
    // columns 64 wc .. +64 of each B half = one interleaved group: j = 0,1 hold h, j = 2,3 the matching gate.
    // B half outermost: only its 16 bias values are live beside the accumulators.
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      const int ng = n0 + hb * 128 + wc * 64;
      float bh[2][4], bg[2][4];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int nh = ng + jj * 16 + fk * 4;
        const uint2 vh = *reinterpret_cast<const uint2*>(g.bias + nh);
        const uint2 vg = *reinterpret_cast<const uint2*>(g.bias + nh + 32);
        bh[jj][0] = bf2f(vh.x & 0xffff); bh[jj][1] = bf2f(vh.x >> 16);
        bh[jj][2] = bf2f(vh.y & 0xffff); bh[jj][3] = bf2f(vh.y >> 16);
        bg[jj][0] = bf2f(vg.x & 0xffff); bg[jj][1] = bf2f(vg.x >> 16);
        bg[jj][2] = bf2f(vg.y & 0xffff); bg[jj][3] = bf2f(vg.y >> 16);
      }
#pragma unroll
      for (int ha = 0; ha < 2; ++ha)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int m = m0 + ha * 128 + wr * 32 + i * 16 + fr;
          if (m >= g.M) continue;
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int nh = ng + jj * 16 + fk * 4;
            float vh[4], vg[4], o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              // h and gate rounded to bf16 first (the unfused path stores them in bf16 before the GEGLU)
              vh[r] = bf_round(acc[ha][hb][i][jj][r] + bh[jj][r]);
              vg[r] = bf_round(acc[ha][hb][i][jj + 2][r] + bg[jj][r]);
              o[r] = vh[r] * gelu_erf(vg[r]);
            }
            if (g.out2 && m < g.pre_rows) {
              bf16_t* p = reinterpret_cast<bf16_t*>(g.out2) + (long)m * g.ldo2 + nh;
              *reinterpret_cast<uint2*>(p) = make_uint2(pack2bf(vh[0], vh[1]), pack2bf(vh[2], vh[3]));
              *reinterpret_cast<uint2*>(p + 32) = make_uint2(pack2bf(vg[0], vg[1]), pack2bf(vg[2], vg[3]));
            }
            *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(g.out) + (long)m * g.ldo + ng / 2 + jj * 16 + fk * 4) =
                make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
          }
        }
    }
  } else {
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      float bv[4][4];
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        const int n = n0 + hb * 128 + wc * 64 + jt * 16 + fk * 4;
        const uint2 v = g.bias ? *reinterpret_cast<const uint2*>(g.bias + n) : make_uint2(0u, 0u);
        bv[jt][0] = bf2f(v.x & 0xffff); bv[jt][1] = bf2f(v.x >> 16);
        bv[jt][2] = bf2f(v.y & 0xffff); bv[jt][3] = bf2f(v.y >> 16);
      }
#pragma unroll
      for (int ha = 0; ha < 2; ++ha)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int m = m0 + ha * 128 + wr * 32 + i * 16 + fr;
          if (m >= g.M) continue;
#pragma unroll
          for (int jt = 0; jt < 4; ++jt) {
            const int n = n0 + hb * 128 + wc * 64 + jt * 16 + fk * 4;
            const f32x4 a = acc[ha][hb][i][jt];
            *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(g.out) + (long)m * g.ldo + n) =
                make_uint2(pack2bf(a[0] + bv[jt][0], a[1] + bv[jt][1]), pack2bf(a[2] + bv[jt][2], a[3] + bv[jt][3]));
          }
        }
    }
  }
}

template <int EPI>
int launch8(const Gemm8Args& g, hipStream_t st) {
  const int nblk = ((g.M + 255) / 256) * (g.N / 256);
  const size_t shm = 8 * HT * sizeof(bf16_t);  // 128 KiB
  static bool attr_done = false;
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)gemm8p_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    attr_done = true;
  }
  gemm8p_kernel<EPI><<<nblk, 512, shm, st>>>(g);
  return pso_check_launch("pso_gemm(8-phase)");
}

}  // namespace

// Host entries used by gemm.hip (preconditions checked there): N % 256 == 0, K % 128 == 0, 16-B aligned rows,
// M * lda and N * ldw below 2^30 (byte offsets of the buffer loads).
int pso_gemm8p(int M, int N, int K, const void* a, long lda, const void* w, long ldw, const void* bias, void* out,
               long ldo, int group_m, hipStream_t st) {
  Gemm8Args g{};
  g.a = (const bf16_t*)a; g.lda = lda; g.w = (const bf16_t*)w; g.ldw = ldw;
  g.M = M; g.N = N; g.K = K; g.bias = (const bf16_t*)bias; g.out = out; g.ldo = ldo; g.group_m = group_m;
  return launch8<EPI8_NONE>(g, st);
}

int pso_gemm8p_geglu(int M, int N, int K, const void* a, long lda, const void* w, long ldw, const void* bias,
                     void* out, long ldo, void* out_pre, long ld_pre, int pre_rows, int group_m, hipStream_t st) {
  Gemm8Args g{};
  g.a = (const bf16_t*)a; g.lda = lda; g.w = (const bf16_t*)w; g.ldw = ldw;
  g.M = M; g.N = N; g.K = K; g.bias = (const bf16_t*)bias; g.out = out; g.ldo = ldo;
  g.out2 = out_pre; g.ldo2 = ld_pre; g.pre_rows = pre_rows; g.group_m = group_m;
  return launch8<EPI8_GEGLU>(g, st);
}
