// 256 x 256 bf16 MFMA GEMM with an 8-phase software pipeline for gfx950, fp32 accumulate.
//
//   acc = A[M][K1] . W[N][K1]^T (+ A2[M][K2] . W2[N][K2]^T, the LoRA up-projection as a K-tail on rows < tail_m)
//   EPI_NONE:      out[M][N]   = bf16(alpha * acc + bias) (+ resid, added to the rounded projection)
//   EPI_GEGLU:     out[M][N/2] = h * gelu(gate) of the interleaved [h 32 | gate 32] columns (+ pre-activation rows)
//   EPI_GEGLU_BWD: acc = dout [M][N]; out[M][2N] = interleaved [dout * gelu(g) | dout * h * gelu'(g)] from aux = pre
//
// Serves the widest GEMMs of the UNet step (N % 256 == 0): the GEGLU projection ff.net.0.proj (16384 x 10240 x 1280
// and 65536 x 5120 x 640 in the paired pass; diffusers GEGLU's nn.Linear + gelu), its backward through
// ff.net.2 (GEGLU_BWD) and the fused self-attention q/k/v projection with its LoRA tail (N = 3C = 3840).
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
//
// FP8 form (the fp8 UNet forward of BASELINE config 5): A / W / A2 / W2 are OCP e4m3 bytes with one power-of-two
// scale per row of A (and A2) and per output column (row of W, W2), stored as E8M0 bytes (127 + exponent).  A K-tile is
// 128 deep (the same 128-B rows, so staging and LDS images are byte-for-byte those of the bf16 form); each lane's
// fragment is 32 consecutive k (two ds_read_b128) and one v_mfma_scale_f32_16x16x128_f8f6f4 per 16 x 16 subtile
// applies the row and column scales in the MFMA (per-lane scale bytes, op_sel picks the subtile's byte), so the
// accumulator is in true units and the epilogues are the bf16 form's.
#include "common.h"

#include <cstdlib>

#define EPI8_NONE 0
#define EPI8_GEGLU 1
#define EPI8_GEGLU_BWD 2

typedef __attribute__((address_space(3))) void lds8_void;

struct Gemm8Args {
  const bf16_t* a; long lda;
  const bf16_t* w; long ldw;
  int M, N, K;
  const bf16_t* a2; long lda2; int K2;  // LoRA K-tail (a2 null: none); a2 has tail_m rows
  const bf16_t* w2; long ldw2;
  int tail_m, tail_group_n;              // tail_group_n > 0: column group j takes a2 columns [j*K2, (j+1)*K2)
  float alpha;
  const bf16_t* bias;
  const bf16_t* resid; long ldr;
  void* out; long ldo;
  void* out2; long ldo2; int pre_rows;  // EPI_GEGLU: interleaved pre-activation of rows < pre_rows (optional)
  const bf16_t* aux; long ldaux;        // EPI_GEGLU_BWD: interleaved pre-activation [M][2N]
  int group_m;
  int skip_epi;  // benchmark knob: accumulators kept live, nothing stored (main-loop time alone)
  // FP8 form: E8M0 scale bytes of the rows of A (M), of W (N), of A2 (tail_m) and of W2 (N)
  const uint8_t* sa; const uint8_t* sw; const uint8_t* sa2; const uint8_t* sw2;
  // CONV form (3x3, stride 1, pad 1, NHWC, A = the [B*H*W][C] image with lda = C): image height / width, K-tiles per
  // tap (C / 64) and its 2^20-scaled reciprocal; per-image row bias rowbias[m / (H*W)][N] (the time embedding)
  int cv_H, cv_W, cv_lh, cv_lw, cv_ct, cv_recip;  // H, W powers of two (lh / lw their logs), W >= 8
  const bf16_t* rowbias; long ld_rowbias;
};

int pso_gemm_group_knob();  // gemm.hip: the raster-group benchmark knob (0 = automatic)

namespace {

constexpr int HT = 128 * 64;  // elements of one half-tile image [128 rows][64 k]

__device__ __forceinline__ int swz8(int r, int c) { return r * 64 + ((c ^ (r & 7)) << 3); }

typedef __attribute__((ext_vector_type(8))) int i32x8;
template <int V> struct ic8 { static constexpr int value = V; };
// scaled fp8 MFMA: src0 = W fragment (column scale byte OB of sb), src1 = A fragment (row scale byte OA of sa)
// As inline asm with the accumulator tied in place: the builtin form needs ~20 more VGPRs at this tile size and
// spills the accumulators.  op_sel[k] / op_sel_hi[k] = bits 0 / 1 of the scale byte index of scale operand k (0: the
// src0 = W scale, 1: the src1 = A scale).  Hazards: the scale / fragment registers are written long before (or by LDS
// reads the compiler waits for), dependent accumulations interlock in hardware, and the epilogue's first VALU read
// of an accumulator comes after the closing barrier plus an explicit s_nop pad (see the end of the main loop).
template <int OA, int OB>
__device__ __forceinline__ void mfma8s(i32x8 w, i32x8 x, f32x4& c, int sb, int sa) {
  asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[%5,%6,0] op_sel_hi:[%7,%8,0]"
               : "+v"(c)
               : "v"(w), "v"(x), "v"(sb), "v"(sa), "n"(OB & 1), "n"(OA & 1), "n"(OB >> 1), "n"(OA >> 1));
}

// STAG: the two wave groups (waves 0-3 / 4-7, one of each per SIMD) run half a phase apart -- waves 4-7 take one
// extra s_barrier before the main loop, waves 0-3 one after it -- so on every SIMD one wave's MFMA segment runs beside
// its partner's fragment-read / staging segment (ping-pong).  Every phase then retires its own fragment reads
// (lgkmcnt(0)) before its first barrier: with the lag, a partner may restage an image one barrier after that point.
// SPRIO: waves 4-7 hold s_setprio 1 for the whole main loop instead of every wave raising it around its MFMAs.
//
// BN = 160 (256 x 160 tiles, every SDXL width N % 160 == 0 -- N = 1280 at M = 16384 is 512 tiles = 2 whole rounds where
// 256 x 256 leaves 1.25): the B tile splits into a 96-row and a 64-row image (12 / 8 glds pieces, staged by waves 0-5 /
// 0-3; the counted waits of the other waves count only what they staged), so the quadrants are 128 x 96 and 128 x 64
// with the waves 4 (M) x 2 (N) as in the 256 x 256 form (32 x 48 = 6 and 32 x 32 = 4 MFMA tiles per wave): per K-tile
// 10 / 4 / 4 / 4 fragment reads against 12 / 12 / 8 / 8 MFMAs per phase.  The epilogue tile sits in LDS with a 336-B
// row pitch.  Plain epilogue only, bf16 only.
//
// CONV (256 x 320 only): the 3x3 / stride 1 / pad 1 convolution as an implicit GEMM over the NHWC image (M = B*H*W
// pixels, K = 9 C ordered [tap][c], C % 64 == 0, H*W % 256 == 0).  A K-tile lies inside one tap (dy, dx), and with
// stride 1 the source pixel of output row m is m + dy*W + dx: the tap is a wave-uniform shift of the dense form's
// scalar row base, so the per-lane staging offset stays the one register vA.  A row whose tap falls off its image
// (oy + dy or ox + dx outside) stages from past the buffer range (zeros).  With W a power of two >= 8 a staged piece
// (8 rows) never wraps an image row, so oy and the first ox are wave-uniform: a tap off the top / bottom edge drops the
// whole piece and one off the left / right edge only the piece's first / last row -- two scalar bounds on vA (whose
// value orders the lane's row inside the piece), no per-lane state.  The A resource starts W + 1 pixels before the
// image so every source offset is non-negative.
template <int EPI, bool STAG, bool SPRIO, bool FP8 = false, int BN = 256, bool CONV = false>
__global__ __launch_bounds__(512, 1) void gemm8p_kernel(Gemm8Args g) {
  static_assert(BN == 256 || ((BN == 160 || BN == 320) && !FP8 && (EPI == EPI8_NONE ||
                                                                     (BN == 320 && EPI != EPI8_NONE && !CONV))),
                "256 x 160 / 256 x 320 tiles: bf16, plain epilogue (320: also the GEGLU forward and backward)");
  static_assert(!CONV || BN == 320, "implicit-GEMM conv: 256 x 320 tiles only");
  constexpr int ES = FP8 ? 1 : 2;         // bytes per operand element
  constexpr int KT = FP8 ? 128 : 64;      // K elements per K-tile (always 128 B per row)
  constexpr int BH0 = BN == 256 ? 128 : (BN == 320 ? 160 : 96), BH1 = BN - BH0;  // rows of the two B images
  constexpr int MI = 2;                                       // row subtiles per wave (32 rows of a 128-row half)
  constexpr int CW0 = BH0 / 2, CW1 = BH1 / 2;                 // columns per wave in the B0 / B1 quadrants
  constexpr int NJ0 = CW0 / 16, NJ1 = CW1 / 16, NJ = NJ0;     // column subtiles per wave
  constexpr int BUFE = 2 * HT + BN * 64;                      // elements of one K-tile buffer [A0 A1 B0 B1]
  constexpr int BW0 = BH0 / 16, BW1 = BH1 / 16;               // waves staging B0 / B1 (2 pieces each; 320: XP)
  // 256 x 320: a 160-row B image is 20 pieces -- pieces 2w, 2w+1 for every wave plus piece 16 + w for waves 0-3
  constexpr bool XP = BN == 320;
  extern __shared__ __attribute__((aligned(16))) bf16_t l8[];  // [2 bufs][A0 A1 B0 B1]
  const int tid = threadIdx.x, lane = tid & 63;
  // wave index in an SGPR: the LDS-DMA destinations (M0) are then scalar arithmetic, not 8 spilled VGPR addresses
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;  // 4 (M) x 2 (N) inside a quadrant
  const int fr = lane & 15, fk = lane >> 4;
  // element offset of image img = buf * 4 + {A0 0, A1 1, B0 2, B1 3}
  auto img_off = [](int img) {
    const int p = img & 3;
    return (img >> 2) * BUFE + (p < 2 ? p * HT : 2 * HT + (p - 2) * BH0 * 64);
  };

  const int nbn = g.N / BN, nbm = (g.M + 255) / 256;
  const int nblk = nbn * nbm;
  // persistent: gridDim.x <= 256 workgroups (one per CU) walk the tiles; a tile's epilogue stores drain while the
  // next tile's first K-tiles are in flight (a fresh workgroup per tile paid both latencies in series)
  // (BN = 160 only: the 256 x 256 form spills ~30 VGPRs around a tile loop and runs its body once)
  for (int tile = blockIdx.x; tile < nblk; tile += gridDim.x) {
  int bid = tile;
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
  const int m0 = bm * 256, n0 = bn * BN;
  const int nt1 = g.K / KT;  // K % KT == 0 (host-checked)
  // the LoRA K-tail: tiles made only of rows >= tail_m (the reference half of a paired pass) skip it (zero there).
  // RT (256 x 320): the tail is NOT staged through the ring -- it runs after the main loop from register operands
  // (register budget: the tail's per-lane staging addresses inside the 8-phase loop spill the 160 accumulators)
  constexpr bool RT = BN == 320;
  const bool has_tail = g.a2 && m0 < g.tail_m;  // (CONV: a2 is null; a compile-time false here made hipcc spill)
  const int nt2 = (!RT && has_tail) ? (g.K2 + KT - 1) / KT : 0;
  const int nt = (nt1 + nt2 + 1) & ~1;  // the 8-phase loop consumes K-tiles in pairs: an odd count gets a zero tile

  // staging: wave w fills pieces 2w, 2w+1 (8 rows x 128 B each) of every half-tile image; the XOR swizzle is applied
  // on the source chunk (lane i lands at byte 16 i of its piece).  Rows past M are clamped (never stored).  The loads
  // are buffer_load ... lds against SGPR resources, so the per-lane part of every staging address is one 32-bit byte
  // offset (64-bit per-lane pointers for the 8 source rows spill at this register budget, and a spill reload's
  // vmcnt(0) would drain the whole ring).
  const int prow = lane >> 3, pch = lane & 7;
  // Every piece is 8 rows x 128 B, so a lane's row inside its piece is prow and its swizzled source chunk pch ^ prow
  // for every piece: the per-lane part of a staging offset is ONE register per operand (vA / vW); the piece's row
  // base, the half and the K-tile advance are wave-uniform and go in the scalar soffset.  Rows past M read as zeros
  // through rA's range (they are never stored), so no per-lane clamp is needed.
  const unsigned vA = (unsigned)(prow * (int)g.lda * ES + (pch ^ prow) * 16);
  // CONV: edge bits of the 4 staged pieces (A half h, piece i: pixels p .. p + 7 of one image row, p = m0 + 128 h + 16 w
  // + 8 i mod H*W) in nibble 2 h + i: top (oy == 0), bottom (oy == H - 1), left (ox == 0), right (ox + 7 == W - 1) --
  // wave-uniform (W is a power of two >= 8, so a piece never wraps an image row); and the byte step of one image row
  unsigned cv_edges = 0;
  int cv_rowb = 0;
  if constexpr (CONV) {
    const int hwm = (1 << (g.cv_lh + g.cv_lw)) - 1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = (m0 + (r >> 1) * 128 + wave * 16 + (r & 1) * 8) & hwm;
      const int oy = p >> g.cv_lw, ox0 = p & (g.cv_W - 1);
      cv_edges |= ((oy == 0 ? 1u : 0u) | (oy == g.cv_H - 1 ? 2u : 0u) | (ox0 == 0 ? 4u : 0u) |
                   (ox0 == g.cv_W - 8 ? 8u : 0u)) << (4 * r);
    }
    cv_rowb = g.cv_W * (int)g.lda * ES;
  }
  // (256 x 320: the host guarantees lda == ldw, and A's register serves both operands)
  // (CONV: ldw = 9 lda and 128 | lda * ES, so vW = 9 vA - 8 chunk = vA + 8 (vA & ~127) is formed from vA per staging,
  // in asm so it is not hoisted into a register of its own: see stage)
  const unsigned vW = BN == 320 ? vA : (unsigned)(prow * (int)g.ldw * ES + (pch ^ prow) * 16);
  // row (inside its image) of this lane in B piece i of this wave (LoRA tail path)
  auto bpiece_row = [&](int i) { return (i < 2 ? wave * 2 + i : 16 + wave) * 8 + prow; };
  // (CONV: the resource starts W + 1 pixels before the image -- offsets of in-image taps are then non-negative -- and
  // ends W + 1 pixels after it)
  const long cv_pre = CONV ? (long)(g.cv_W + 1) * g.lda * ES : 0;
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)g.a - cv_pre), (short)0, (int)((long)g.M * g.lda * ES + 2 * cv_pre), 0x00020000);
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)g.w, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rA2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(g.a2 ? g.a2 : g.a), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rW2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(g.w2 ? g.w2 : g.w), (short)0, 0x7fffffff, 0x00020000);
  // a byte offset past the buffer range: the raw buffer load returns zeros (padding of the K-tail / zero tile)
  constexpr unsigned OOB = 0x80000000u;
  const long a2_col = g.tail_group_n > 0 ? (long)(n0 / g.tail_group_n) * g.K2 : 0;
  // image index = buf * 4 + {A0 0, A1 1, B0 2, B1 3}
  auto stage = [&](int kt, int img) {
    const int half = img & 3;
    bf16_t* dst = l8 + img_off(img) + wave * 2 * 8 * 64;
    if (BN == 160 && half >= 2 && wave >= (half == 2 ? BW0 : BW1)) return;  // 96 / 64-row B images: waves 0-5 / 0-3
    // the extra (third) B piece in the 256 x 320 form: piece 16 + w of the image for waves 0-3; waves 4-7 issue the
    // same load with a source past the buffer range (zeros, no memory traffic) into a dummy 1-KB slot behind the
    // ring, so every wave issues 3 pieces per B image: no per-wave branch, one vmcnt count for all waves
    bf16_t* dst_x = wave < 4 ? l8 + img_off(img) + (16 + wave) * 8 * 64 : l8 + 4 * HT + 4 * (BN / 2) * 64 + (wave - 4) * 512;
    const bool xp = XP && half >= 2;
    const int xsrc_oob = wave < 4 ? 0 : (int)OOB;  // in the scalar soffset: no extra lane register
    if (kt < nt1) {
      const int k0 = kt * 128;  // bytes
      if (half < 2) {
        if constexpr (CONV) {
          // K-tile kt = tap * ct + channel block; tap = 3 dy + dx (dy, dx in 0..2 = offsets -1..1)
          const int tap = (kt * g.cv_recip) >> 20;
          const int cb = (kt - tap * g.cv_ct) * 128;  // bytes into the pixel's channels
          const int dy = (tap * 11) >> 5, dx = tap - 3 * dy;
          // the tap's edge mask (bit 0: dy = -1 top, 1: dy = +1 bottom, 2: dx = -1 left, 3: dx = +1 right), one nibble
          // per tap: 5 1 9 / 4 0 8 / 6 2 10
          const unsigned tm = (unsigned)(0xA26804915ull >> (4 * tap)) & 15u;
          // piece 2w, row 0 of the shifted source, in the resource's coordinates (which start at pixel -(W + 1))
          const int sa = (m0 + (half & 1) * 128 + wave * 16) * (int)g.lda * ES + dy * cv_rowb + dx * (int)g.lda * ES + cb;
          const unsigned rowb = (unsigned)g.lda * ES;  // vA = prow * rowb + chunk: prow == 0 <=> vA < rowb
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            // the piece's edge bits against the tap: top / bottom drop the whole piece, left / right its lane row 0 / 7;
            // valid <=> lo <= vA <= hm; off = valid ? vA : 0xC0800000 (the inline constant -4.0: past the range, zeros)
            // -- in asm with the output as the only register (no temporaries: the main loop has none to spare)
            const unsigned hit = (cv_edges >> (4 * (2 * (half & 1) + i))) & tm;
            const unsigned lo = (hit & 3u) ? 0x80000000u : ((hit & 4u) ? rowb : 0u);
            const unsigned hm = (hit & 8u) ? 7u * rowb - 1u : 0x7fffffffu;
            unsigned off;
            asm volatile("v_cmp_le_u32 vcc, %1, %3\n\t"
                         "v_cndmask_b32 %0, -4.0, %3, vcc\n\t"
                         "v_cmp_ge_u32 vcc, %2, %3\n\t"
                         "v_cndmask_b32 %0, -4.0, %0, vcc"
                         : "=&v"(off) : "s"(lo), "s"(hm), "v"(vA) : "vcc");
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds8_void*)(dst + i * 8 * 64), 16, off,
                                                     sa + i * 8 * (int)g.lda * ES, 0, 0);
          }
        } else {
          const int sa = (m0 + (half & 1) * 128 + wave * 16) * (int)g.lda * ES + k0;  // piece 2w, row 0
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds8_void*)dst, 16, vA, sa, 0, 0);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds8_void*)(dst + 8 * 64), 16, vA, sa + 8 * (int)g.lda * ES, 0,
                                                   0);
        }
      } else {
        const int sw = (n0 + (half & 1) * BH0 + wave * 16) * (int)g.ldw * ES + k0;
        unsigned vw = vW;
        if constexpr (CONV) asm volatile("v_and_b32 %0, 0xffffff80, %1\n\tv_lshl_add_u32 %0, %0, 3, %1" : "=&v"(vw) : "v"(vA));
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds8_void*)dst, 16, vw, sw, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds8_void*)(dst + 8 * 64), 16, vw, sw + 8 * (int)g.ldw * ES, 0,
                                                 0);
        if constexpr (XP)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rW, (lds8_void*)dst_x, 16, vw, ((n0 + (half & 1) * BH0 + (16 + wave) * 8) * (int)g.ldw * ES + k0) | xsrc_oob,
              0, 0);
      }
    } else if constexpr (RT) {  // the zero pad tile of an odd K-tile count: every load past the buffer range
      // (the offset materialised in asm at the load: a hoisted constant would hold a register through the main loop)
      unsigned oob;
      asm volatile("v_mov_b32 %0, 0x80000000" : "=v"(oob));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds8_void*)dst, 16, oob, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds8_void*)(dst + 8 * 64), 16, oob, 0, 0, 0);
      if (xp) __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds8_void*)dst_x, 16, oob, 0, 0, 0);
    } else {  // LoRA K-tail (one or two K-tiles per output tile) or the zero pad tile
      const int kc = (kt - nt1) * KT + (pch ^ prow) * (16 / ES);  // this lane's 16-B chunk of the tail
      const bool kin = kt < nt1 + nt2 && kc < g.K2;
#pragma unroll
      for (int i = 0; i < (XP ? 3 : 2); ++i) {
        if (i == 2 && !xp) break;
        unsigned off;
        if (half < 2) {
          if (i == 2) break;
          const int R = (half & 1) * 128 + (wave * 2 + i) * 8 + prow;
          const int m = m0 + R;
          off = (kin && m < g.tail_m) ? (unsigned)(((long)m * g.lda2 + a2_col + kc) * ES) : OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rA2, (lds8_void*)(dst + i * 8 * 64), 16, off, 0, 0, 0);
        } else {
          const int R = (half & 1) * BH0 + bpiece_row(i);
          off = kin ? (unsigned)(((long)(n0 + R) * g.ldw2 + kc) * ES) : OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rW2, (lds8_void*)(i == 2 ? dst_x : dst + i * 8 * 64), 16, off, 0,
                                                   0, 0);
        }
      }
    }
  };

  f32x4 acc[2][2][MI][NJ];  // [A half][B half][row subtile][col subtile]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[MI][2], bfr[NJ][2];  // [row subtile][kk], [col subtile][kk]  (bf16 form)
  i32x8 af8[2], bf8[4];         // FP8 form: [row subtile], [col subtile], 32 fp8 k per lane (two 16-B reads)
  // Fragment addresses: the swizzle term depends only on fr & 7, so within an image a lane needs one byte offset per
  // kk (subtiles are +2048-B immediates).  The image base is added per read by a volatile v_add: left to itself the
  // compiler hoists 8 images x 4 addresses out of the loop and spills at this register budget.
  typedef __attribute__((address_space(3))) const bf16x8 lds_frag;
  typedef __attribute__((ext_vector_type(4))) int i32x4_t;
  typedef __attribute__((address_space(3))) const i32x4_t lds_frag4;
  const unsigned l8base = (unsigned)(uintptr_t)(lds8_void*)l8;
  // ONE lane register serves every fragment read: bf16 chunk kk*4 + fk (k = 32 kk + 8 fk ..), fp8 chunks 2 fk + kk
  // (the lane's 32 consecutive k), so kk = 1 is the kk = 0 offset with byte bit 6 (bf16) / bit 4 (fp8) flipped; the
  // A images' row offset wr * 32 keeps the swizzle (a multiple of 8 rows) and is wave-uniform, like the B images'
  // column offset wc * CW rows
  const unsigned lb0 = (unsigned)swz8(fr, FP8 ? 2 * fk : fk) * 2u;
  constexpr unsigned KKX = FP8 ? 16u : 64u;
  i32x4_t ta[2], tb[4];
  auto read_a = [&](int img) {
    const unsigned ib = l8base + (unsigned)(img_off(img) * 2) + (unsigned)(wr * 32 * 128);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      unsigned ad;
      if (kk == 0) asm volatile("v_add_u32 %0, %1, %2" : "=v"(ad) : "s"(ib), "v"(lb0));
      else asm volatile("v_xor_b32 %0, %1, %2\n\tv_add_u32 %0, %3, %0" : "=&v"(ad) : "v"(lb0), "n"(KKX), "s"(ib));
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if constexpr (FP8) {
          if (kk == 0) ta[i] = *(lds_frag4*)(uintptr_t)(ad + i * 2048);
          else af8[i] = __builtin_shufflevector(ta[i], *(lds_frag4*)(uintptr_t)(ad + i * 2048), 0, 1, 2, 3, 4, 5, 6, 7);
        } else {
          af[i][kk] = *(lds_frag*)(uintptr_t)(ad + i * 2048);
        }
      }
    }
  };
  auto read_b = [&](auto HB_, int buf) {
    constexpr int hb = decltype(HB_)::value;
    const unsigned ib = l8base + (unsigned)(img_off(buf * 4 + 2 + hb) * 2) + (unsigned)(wc * (hb ? CW1 : CW0) * 128);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      unsigned ad;
      if (kk == 0) asm volatile("v_add_u32 %0, %1, %2" : "=v"(ad) : "s"(ib), "v"(lb0));
      else asm volatile("v_xor_b32 %0, %1, %2\n\tv_add_u32 %0, %3, %0" : "=&v"(ad) : "v"(lb0), "n"(KKX), "s"(ib));
#pragma unroll
      for (int j = 0; j < (hb ? NJ1 : NJ0); ++j) {
        if constexpr (FP8) {
          if (kk == 0) tb[j] = *(lds_frag4*)(uintptr_t)(ad + j * 2048);
          else bf8[j] = __builtin_shufflevector(tb[j], *(lds_frag4*)(uintptr_t)(ad + j * 2048), 0, 1, 2, 3, 4, 5, 6, 7);
        } else {
          bfr[j][kk] = *(lds_frag*)(uintptr_t)(ad + j * 2048);
        }
      }
    }
  };
  // FP8: scale bytes of this lane's rows (byte 2 ha + i) and columns (byte j of word hb), main and tail operands
  int sra = 0, srb[2] = {0, 0}, sra2 = 0, srb2[2] = {0, 0};
  if constexpr (FP8) {
#pragma unroll
    for (int ha = 0; ha < 2; ++ha)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int m = m0 + ha * 128 + wr * 32 + i * 16 + fr;
        sra |= (int)g.sa[min(m, g.M - 1)] << (8 * (2 * ha + i));
        if (g.a2) sra2 |= (int)g.sa2[min(m, g.tail_m - 1)] << (8 * (2 * ha + i));
      }
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + hb * 128 + wc * 64 + j * 16 + fr;
        srb[hb] |= (int)g.sw[n] << (8 * j);
        if (g.a2) srb2[hb] |= (int)g.sw2[n] << (8 * j);
      }
  }
  auto mfma_q = [&](auto HA_, auto HB_, bool tail_start) {
    constexpr int ha = decltype(HA_)::value, hb = decltype(HB_)::value;
    if constexpr (FP8) {
      // first quadrant of the first LoRA K-tail tile: from here on the tail operands' scales (in asm, with the wait
      // states an MFMA scale operand needs after a VALU write -- the asm MFMAs are invisible to the hazard recognizer)
      if (ha == 0 && hb == 0 && tail_start)
        asm volatile("v_mov_b32 %0, %3\n\tv_mov_b32 %1, %4\n\tv_mov_b32 %2, %5\n\ts_nop 7"
                     : "=v"(sra), "=v"(srb[0]), "=v"(srb[1])
                     : "v"(sra2), "v"(srb2[0]), "v"(srb2[1]));
    }
    if (!SPRIO) __builtin_amdgcn_s_setprio(1);
    if constexpr (FP8) {
      auto q8 = [&](int sa, int sb) {
        mfma8s<2 * ha, 0>(bf8[0], af8[0], acc[ha][hb][0][0], sb, sa);
        mfma8s<2 * ha, 1>(bf8[1], af8[0], acc[ha][hb][0][1], sb, sa);
        mfma8s<2 * ha, 2>(bf8[2], af8[0], acc[ha][hb][0][2], sb, sa);
        mfma8s<2 * ha, 3>(bf8[3], af8[0], acc[ha][hb][0][3], sb, sa);
        mfma8s<2 * ha + 1, 0>(bf8[0], af8[1], acc[ha][hb][1][0], sb, sa);
        mfma8s<2 * ha + 1, 1>(bf8[1], af8[1], acc[ha][hb][1][1], sb, sa);
        mfma8s<2 * ha + 1, 2>(bf8[2], af8[1], acc[ha][hb][1][2], sb, sa);
        mfma8s<2 * ha + 1, 3>(bf8[3], af8[1], acc[ha][hb][1][3], sb, sa);
      };
      q8(sra, srb[hb]);
      // The hazard recognizer cannot see into the asm: a register copy of an accumulator placed right behind it (the
      // allocator's loop-carried copies) would read the MFMA's destination before it is written.  Route the
      // quadrant's accumulators through one more asm holding the VALU-read wait states, so every later use follows it.
      asm volatile("s_nop 11"
                   : "+v"(acc[ha][hb][0][0]), "+v"(acc[ha][hb][0][1]), "+v"(acc[ha][hb][0][2]), "+v"(acc[ha][hb][0][3]),
                     "+v"(acc[ha][hb][1][0]), "+v"(acc[ha][hb][1][1]), "+v"(acc[ha][hb][1][2]), "+v"(acc[ha][hb][1][3]));
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < (hb ? NJ1 : NJ0); ++j) {
            if constexpr (BN == 320)  // accumulator tied in place (the builtin form double-buffers and spills here)
              asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[ha][hb][i][j]) : "v"(bfr[j][kk]),
                           "v"(af[i][kk]));
            else
              acc[ha][hb][i][j] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][kk], af[i][kk], acc[ha][hb][i][j], 0, 0, 0);
          }
      if constexpr (BN == 320)  // the asm MFMAs are invisible to the hazard recognizer: see the FP8 form's note
        asm volatile("s_nop 7"
                     : "+v"(acc[ha][hb][0][0]), "+v"(acc[ha][hb][0][1]), "+v"(acc[ha][hb][0][2]),
                       "+v"(acc[ha][hb][0][3]), "+v"(acc[ha][hb][0][4]), "+v"(acc[ha][hb][1][0]),
                       "+v"(acc[ha][hb][1][1]), "+v"(acc[ha][hb][1][2]), "+v"(acc[ha][hb][1][3]),
                       "+v"(acc[ha][hb][1][4]));
    }
    if (!SPRIO) __builtin_amdgcn_s_setprio(0);
  };
  // the counted wait that retires all but the last three stagings (B0, A1, B1): 6 loads per wave, fewer for the waves
  // that stage no B1 (4) or no B pieces at all (2) in the 256 x 160 form
  auto vm_wait6 = [&]() {
    if constexpr (BN == 320) {  // every wave stages 3 pieces per B image (see stage): 3 + 2 + 3 in flight
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      if (BN == 256 || wave < BW1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if (wave < BW0) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
  };
  // one phase: reads (RA / RB: which operand image to (re)load), the stage (if its K-tile exists), the optional
  // counted wait (VM: -1 none, else vmcnt(VM)), barrier, MFMAs of quadrant (HA, HB), barrier.
#define PHASE(BUF, HA, HB, RA, RB, STAGE_KT, STAGE_IMG, VM)                                   \
  {                                                                                           \
    if (RB) read_b(ic8<(HB)>{}, (BUF));                                                       \
    if (RA) read_a((BUF) * 4 + (HA));                                                         \
    if ((STAGE_KT) < nt) stage((STAGE_KT), (STAGE_IMG));                                      \
    if (STAG) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                              \
    if ((VM) == 6) vm_wait6();                                                                \
    else if ((VM) == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                      \
    __builtin_amdgcn_s_barrier();                                                             \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    mfma_q(ic8<(HA)>{}, ic8<(HB)>{}, FP8 && nt2 > 0 && j + (BUF) == nt1);                     \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    __builtin_amdgcn_s_barrier();                                                             \
  }

  // prologue: K-tile 0 -> E (in the steady-state staging order), K-tile 1 -> O.B0 O.A1 O.B1; wait for K-tile 0
  stage(0, 2); stage(0, 1); stage(0, 3); stage(0, 0);
  if (nt > 1) { stage(1, 6); stage(1, 5); stage(1, 7); }
  if (nt > 1) vm_wait6();
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (STAG && wave >= 4) __builtin_amdgcn_s_barrier();
  if (SPRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);

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
  // FP8: the inline-asm MFMAs are invisible to the hazard recognizer -- pad before any VALU reads an accumulator
  if constexpr (RT) {
    // LoRA K-tail from register operands (K2 <= 64 in steps of 32 = one MFMA k-depth): this lane's fragments are
    // 16-B global loads -- A2 row m0 + 128 ha + 32 wr + 16 i + fr and W2 row n0 + hb*BH0 + wc*CW0 + 16 j + fr, k =
    // kb + 8 fk .. +8 -- u / sB are small and L2-resident.  Rows >= tail_m (the reference half of a paired pass)
    // and k >= K2 are zeros.
    if (has_tail) {
      const bf16x8 z8 = __builtin_bit_cast(bf16x8, make_uint4(0u, 0u, 0u, 0u));
      for (int kb = 0; kb < g.K2; kb += 32) {
        const int k = kb + 8 * fk;
        bf16x8 ta2[2][MI], tw2[2][NJ];
#pragma unroll
        for (int ha = 0; ha < 2; ++ha)
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const int m = m0 + ha * 128 + wr * 32 + i * 16 + fr;
            ta2[ha][i] = (m < g.tail_m && k < g.K2)
                             ? *reinterpret_cast<const bf16x8*>(g.a2 + (long)m * g.lda2 + a2_col + k) : z8;
          }
#pragma unroll
        for (int hb = 0; hb < 2; ++hb)
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int n = n0 + hb * BH0 + wc * CW0 + j * 16 + fr;
            tw2[hb][j] = k < g.K2 ? *reinterpret_cast<const bf16x8*>(g.w2 + (long)n * g.ldw2 + k) : z8;
          }
#pragma unroll
        for (int ha = 0; ha < 2; ++ha)
#pragma unroll
          for (int hb = 0; hb < 2; ++hb)
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
              for (int j = 0; j < NJ; ++j)
                asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[ha][hb][i][j]) : "v"(tw2[hb][j]),
                             "v"(ta2[ha][i]));
      }
    }
  }
  if constexpr (FP8 || BN == 320) asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
  if (STAG && wave < 4) __builtin_amdgcn_s_barrier();
  if (SPRIO) __builtin_amdgcn_s_setprio(0);

  // ---- epilogue: lane holds out[m = m0 + 128 ha + 32 wr + 16 i + fr][n = n0 + 128 hb + 64 wc + 16 j + 4 fk + r] ----
  if (g.skip_epi) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < (b ? NJ1 : NJ0); ++j) asm volatile("" ::"v"(acc[a][b][i][j]));
    goto tile_end;
  }
  if constexpr (BN == 320) {
    // 256 x 320 tile through LDS in two 128-row halves (the whole tile would need 160 KB): rows at a 328-element
    // (656-B = 164-dword) pitch -- the ds_write_b64 of a 16-row fragment column hits 16 distinct bank pairs -- read
    // back as 40 16-B chunks per row and stored whole (640 B).  Register budget: the 160 accumulator registers are
    // live until a half is staged, so the bias is loaded per column half (20 registers) and the residual chunks only
    // once the half's accumulators are in LDS.
    __builtin_amdgcn_s_waitcnt(0xC07F & ~0x3F00);  // lgkmcnt(0): this wave's LDS traffic retired
    constexpr int TP = 328;
    bf16_t* tl = l8;
    const bool has_r = g.resid != nullptr;
    auto stage_half = [&](auto HA_) {
      constexpr int ha = decltype(HA_)::value;
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        float bv[NJ][4];
#pragma unroll
        for (int jt = 0; jt < NJ; ++jt) {
          const int n = n0 + hb * BH0 + wc * CW0 + jt * 16 + fk * 4;
          const uint2 v = g.bias ? *reinterpret_cast<const uint2*>(g.bias + n) : make_uint2(0u, 0u);
          bv[jt][0] = bf2f(v.x & 0xffff); bv[jt][1] = bf2f(v.x >> 16);
          bv[jt][2] = bf2f(v.y & 0xffff); bv[jt][3] = bf2f(v.y >> 16);
          if (CONV && g.rowbias) {  // the tile's image row of the per-image bias (H*W % 256 == 0)
            const uint2 w = *reinterpret_cast<const uint2*>(g.rowbias + (long)(m0 / (g.cv_H * g.cv_W)) * g.ld_rowbias + n);
            bv[jt][0] += bf2f(w.x & 0xffff); bv[jt][1] += bf2f(w.x >> 16);
            bv[jt][2] += bf2f(w.y & 0xffff); bv[jt][3] += bf2f(w.y >> 16);
          }
        }
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int R = wr * 32 + i * 16 + fr;
#pragma unroll
          for (int jt = 0; jt < NJ; ++jt) {
            const int col = hb * BH0 + wc * CW0 + jt * 16 + fk * 4;
            const f32x4 a = acc[ha][hb][i][jt];
            const float al = g.alpha;
            *reinterpret_cast<uint2*>(tl + R * TP + col) =
                make_uint2(pack2bf(a[0] * al + bv[jt][0], a[1] * al + bv[jt][1]),
                           pack2bf(a[2] * al + bv[jt][2], a[3] * al + bv[jt][3]));
          }
        }
      }
    };
    auto store_half = [&](int ha) {
      if constexpr (EPI == EPI8_GEGLU) {
        // the staged half IS the interleaved pre-activation ([h 32 | gate 32] per 64 columns, acc + bias rounded
        // once, as in the 256 x 256 form): its policy rows (< pre_rows) to out2, then out = h * gelu(gate) from it --
        // the 256 x 256 form's arithmetic on the same bf16 values, so the same bits
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (g.out2) {
#pragma unroll 2
          for (int p = 0; p < 10; ++p) {  // 128 rows x 40 chunks = 10 passes of 512
            const int idx = p * 512 + tid;
            const int R = idx / 40, c = idx - R * 40, m = m0 + ha * 128 + R;
            if (m < g.pre_rows && m < g.M)
              *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(g.out2) + (long)m * g.ldo2 + n0 + c * 8) =
                  *reinterpret_cast<const uint4*>(tl + R * TP + c * 8);
          }
        }
        // output chunk q (20 per row: 160 output columns) = h chunk (q / 4) * 8 + (q % 4), gate chunk + 4
#pragma unroll 1
        for (int p = 0; p < 5; ++p) {  // 128 rows x 20 chunks = 5 passes of 512
          const int idx = p * 512 + tid;
          const int R = idx / 20, q = idx - R * 20, m = m0 + ha * 128 + R;
          if (m >= g.M) continue;
          const int ch = (q >> 2) * 8 + (q & 3);
          const uint4 hv = *reinterpret_cast<const uint4*>(tl + R * TP + ch * 8);
          const uint4 gv = *reinterpret_cast<const uint4*>(tl + R * TP + (ch + 4) * 8);
          const uint32_t hw[4] = {hv.x, hv.y, hv.z, hv.w}, gw[4] = {gv.x, gv.y, gv.z, gv.w};
          uint32_t o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            o[e] = pack2bf(bf2f(hw[e] & 0xffff) * gelu_erf(bf2f(gw[e] & 0xffff)),
                           bf2f(hw[e] >> 16) * gelu_erf(bf2f(gw[e] >> 16)));
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(g.out) + (long)m * g.ldo + n0 / 2 + q * 8) =
              make_uint4(o[0], o[1], o[2], o[3]);
        }
        return;
      }
      if constexpr (EPI == EPI8_GEGLU_BWD) {
        // the staged half = dout (bf16, as the unfused path stores it); chunk c of row R = dout columns n .. n+7 ->
        // interleaved input-gradient positions ph .. ph+7 (h) and ph+32 .. (gate), ph = (n / 32) * 64 + n % 32, from
        // the interleaved pre-activation aux: 128 rows x 40 chunks = 10 passes of 512
        // the pre-activation chunks of 5 passes are requested together (the first 5 before the LDS barrier), so
        // the 10 passes wait for 2 global round trips instead of one per unrolled pair (C2 step: 8192 x 5120 x 1280
        // 717 -> 751 TF/s, 32768 x 2560 x 640 482 -> 518)
#pragma unroll
        for (int p5 = 0; p5 < 2; ++p5) {
        uint4 hvp[5], gvp[5];
#pragma unroll
        for (int u = 0; u < 5; ++u) {
          const int idx = (p5 * 5 + u) * 512 + tid;
          const int R = idx / 40, c = idx - R * 40, m = min(m0 + ha * 128 + R, g.M - 1);
          const int n = n0 + c * 8;
          const int ph = (n >> 5) * 64 + (n & 31);
          hvp[u] = *reinterpret_cast<const uint4*>(g.aux + (long)m * g.ldaux + ph);
          gvp[u] = *reinterpret_cast<const uint4*>(g.aux + (long)m * g.ldaux + ph + 32);
        }
        if (p5 == 0) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int u = 0; u < 5; ++u) {
          const int idx = (p5 * 5 + u) * 512 + tid;
          const int R = idx / 40, c = idx - R * 40, m = m0 + ha * 128 + R;
          if (m >= g.M) continue;
          const int n = n0 + c * 8;
          const int ph = (n >> 5) * 64 + (n & 31);
          const uint4 dv = *reinterpret_cast<const uint4*>(tl + R * TP + c * 8);
          const uint4 hv = hvp[u], gv = gvp[u];
          const uint32_t dw[4] = {dv.x, dv.y, dv.z, dv.w}, hw[4] = {hv.x, hv.y, hv.z, hv.w},
                         gw[4] = {gv.x, gv.y, gv.z, gv.w};
          uint32_t oh[4], og[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d0 = bf2f(dw[e] & 0xffff), d1 = bf2f(dw[e] >> 16);
            const float h0 = bf2f(hw[e] & 0xffff), h1 = bf2f(hw[e] >> 16);
            const float q0 = bf2f(gw[e] & 0xffff), q1 = bf2f(gw[e] >> 16);
            float c0, e0, c1, e1;
            gelu_erf_parts(q0, c0, e0);
            gelu_erf_parts(q1, c1, e1);
            oh[e] = pack2bf(d0 * q0 * c0, d1 * q1 * c1);
            og[e] = pack2bf(d0 * h0 * (c0 + 0.39894228040143268f * q0 * e0),
                            d1 * h1 * (c1 + 0.39894228040143268f * q1 * e1));
          }
          bf16_t* o = reinterpret_cast<bf16_t*>(g.out) + (long)m * g.ldo + ph;
          *reinterpret_cast<uint4*>(o) = make_uint4(oh[0], oh[1], oh[2], oh[3]);
          *reinterpret_cast<uint4*>(o + 32) = make_uint4(og[0], og[1], og[2], og[3]);
        }
        }
        return;
      }
      uint4 rvp[10];
#pragma unroll
      for (int p = 0; p < 10; ++p) {
        const int idx = p * 512 + tid;
        const int R = idx / 40, c = idx - R * 40, m = min(m0 + ha * 128 + R, g.M - 1);
        rvp[p] = has_r ? *reinterpret_cast<const uint4*>(g.resid + (long)m * g.ldr + n0 + c * 8) : make_uint4(0, 0, 0, 0);
      }
      // LDS-only barrier: the residual loads stay in flight across it
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
      for (int p = 0; p < 10; ++p) {  // 128 rows x 40 chunks = 10 passes of 512
        const int idx = p * 512 + tid;
        const int R = idx / 40, c = idx - R * 40, m = m0 + ha * 128 + R;
        if (m >= g.M) continue;
        uint4 y = *reinterpret_cast<const uint4*>(tl + R * TP + c * 8);
        if (has_r) {  // residual added to the bf16-rounded projection (the unfused Linear + add)
          const uint4 rv = rvp[p];
          const uint32_t yw[4] = {y.x, y.y, y.z, y.w}, rw[4] = {rv.x, rv.y, rv.z, rv.w};
          uint32_t o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            o[e] = pack2bf(bf2f(yw[e] & 0xffff) + bf2f(rw[e] & 0xffff), bf2f(yw[e] >> 16) + bf2f(rw[e] >> 16));
          y = make_uint4(o[0], o[1], o[2], o[3]);
        }
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(g.out) + (long)m * g.ldo + n0 + c * 8) = y;
      }
    };
    stage_half(ic8<0>{});
    store_half(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // the first half's LDS reads retired
    stage_half(ic8<1>{});
    store_half(1);
  } else if constexpr (BN == 160) {
    // 256 x 160 tile through LDS at a 168-element (336-B) row pitch: the ds_write_b64 of a 16-row fragment column hits
    // 16 distinct bank pairs (84 dwords per row), rows are read back as 20 16-B chunks and stored whole (320 B)
    __builtin_amdgcn_s_waitcnt(0xC07F & ~0x3F00);  // lgkmcnt(0): this wave's LDS traffic retired
    constexpr int TP = 168;
    bf16_t* tl = l8;
    // the residual chunks of all 10 store passes are requested first: their latency runs under the LDS staging
    const bool has_r = g.resid != nullptr;
    uint4 rvp[10];
#pragma unroll
    for (int p = 0; p < 10; ++p) {
      const int idx = p * 512 + tid;
      const int R = idx / 20, c = idx - R * 20, m = min(m0 + R, g.M - 1);
      rvp[p] = has_r ? *reinterpret_cast<const uint4*>(g.resid + (long)m * g.ldr + n0 + c * 8) : make_uint4(0, 0, 0, 0);
    }
    auto epi_half = [&](auto HB_) {
      constexpr int hb = decltype(HB_)::value, nj = hb ? NJ1 : NJ0;
      const int c0 = hb * BH0 + wc * (hb ? CW1 : CW0);
      float bv[nj][4];
#pragma unroll
      for (int jt = 0; jt < nj; ++jt) {
        const int n = n0 + c0 + jt * 16 + fk * 4;
        const uint2 v = g.bias ? *reinterpret_cast<const uint2*>(g.bias + n) : make_uint2(0u, 0u);
        bv[jt][0] = bf2f(v.x & 0xffff); bv[jt][1] = bf2f(v.x >> 16);
        bv[jt][2] = bf2f(v.y & 0xffff); bv[jt][3] = bf2f(v.y >> 16);
      }
#pragma unroll
      for (int ha = 0; ha < 2; ++ha)
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int R = ha * 128 + wr * 32 + i * 16 + fr;
#pragma unroll
          for (int jt = 0; jt < nj; ++jt) {
            const int col = c0 + jt * 16 + fk * 4;
            const f32x4 a = acc[ha][hb][i][jt];
            const float al = g.alpha;
            *reinterpret_cast<uint2*>(tl + R * TP + col) =
                make_uint2(pack2bf(a[0] * al + bv[jt][0], a[1] * al + bv[jt][1]),
                           pack2bf(a[2] * al + bv[jt][2], a[3] * al + bv[jt][3]));
          }
        }
    };
    epi_half(ic8<0>{});
    epi_half(ic8<1>{});
    // LDS-only barrier: the residual loads stay in flight across it (__syncthreads would wait for them)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int p = 0; p < 10; ++p) {  // 256 rows x 20 chunks = 10 passes of 512
      const int idx = p * 512 + tid;
      const int R = idx / 20, c = idx - R * 20, m = m0 + R;
      if (m >= g.M) continue;
      uint4 y = *reinterpret_cast<const uint4*>(tl + R * TP + c * 8);
      if (has_r) {  // residual added to the bf16-rounded projection (the unfused Linear + add)
        const uint4 rv = rvp[p];
        const uint32_t yw[4] = {y.x, y.y, y.z, y.w}, rw[4] = {rv.x, rv.y, rv.z, rv.w};
        uint32_t o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          o[e] = pack2bf(bf2f(yw[e] & 0xffff) + bf2f(rw[e] & 0xffff), bf2f(yw[e] >> 16) + bf2f(rw[e] >> 16));
        y = make_uint4(o[0], o[1], o[2], o[3]);
      }
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(g.out) + (long)m * g.ldo + n0 + c * 8) = y;
    }
  } else {
  // Epilogue through LDS: the operand ring (128 KB, free once the last phase's barrier has passed and no staging is
  // in flight) holds the whole 256 x 256 tile as bf16 (acc + bias, rounded once -- the unfused Linear's output),
  // then every wave stores whole 512-B rows in 16-B chunks (full 128-B lines per instruction) instead of the MFMA
  // layout's 16 rows x 32 B per store instruction.  Chunk c of row R sits at chunk c ^ (R & 31): the ds_write_b64 of
  // a 16-row fragment column is 2-way banked, the 16-lane ds_read_b128 of one row is conflict-free.
  __builtin_amdgcn_s_waitcnt(0xC07F & ~0x3F00);  // lgkmcnt(0): this wave's LDS traffic retired
  bf16_t* tl = l8;
  auto tix = [](int R, int c) { return R * 256 + ((c ^ (R & 31)) << 3); };  // element index of chunk c of row R
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
        const int R = ha * 128 + wr * 32 + i * 16 + fr;
#pragma unroll
        for (int jt = 0; jt < 4; ++jt) {
          const int col = hb * 128 + wc * 64 + jt * 16 + fk * 4;
          const f32x4 a = acc[ha][hb][i][jt];
          const float al = g.alpha;
          *reinterpret_cast<uint2*>(tl + tix(R, col >> 3) + (col & 7)) =
              make_uint2(pack2bf(a[0] * al + bv[jt][0], a[1] * al + bv[jt][1]),
                         pack2bf(a[2] * al + bv[jt][2], a[3] * al + bv[jt][3]));
        }
      }
  }
  __syncthreads();
  // 512 threads = 16 rows x 32 chunks per pass, 16 passes
  const int cq = tid & 31, rq = tid >> 5;
  if constexpr (EPI == EPI8_GEGLU) {
    // the staged tile IS the interleaved pre-activation ([h 32 | gate 32] per 64 columns): store its policy rows,
    // then form out = h * gelu(gate) from it (columns c and c + 32 of each 64-group -> 8 output columns per thread)
    if (g.out2) {
#pragma unroll 4
      for (int p = 0; p < 16; ++p) {
        const int R = p * 16 + rq, m = m0 + R;
        if (m < g.pre_rows && m < g.M)
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(g.out2) + (long)m * g.ldo2 + n0 + cq * 8) =
              *reinterpret_cast<const uint4*>(tl + tix(R, cq));
      }
    }
    // output chunk q (16 per row: 128 output columns) = h chunk (q / 4) * 8 + (q % 4), gate chunk + 4
    const int q = tid & 15, rr = tid >> 4;  // 32 rows per pass, 8 passes
    const int ch = (q >> 2) * 8 + (q & 3);
#pragma unroll 2
    for (int p = 0; p < 8; ++p) {
      const int R = p * 32 + rr, m = m0 + R;
      if (m >= g.M) continue;
      const uint4 hv = *reinterpret_cast<const uint4*>(tl + tix(R, ch));
      const uint4 gv = *reinterpret_cast<const uint4*>(tl + tix(R, ch + 4));
      const uint32_t hw[4] = {hv.x, hv.y, hv.z, hv.w}, gw[4] = {gv.x, gv.y, gv.z, gv.w};
      uint32_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = pack2bf(bf2f(hw[e] & 0xffff) * gelu_erf(bf2f(gw[e] & 0xffff)),
                       bf2f(hw[e] >> 16) * gelu_erf(bf2f(gw[e] >> 16)));
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(g.out) + (long)m * g.ldo + n0 / 2 + q * 8) =
          make_uint4(o[0], o[1], o[2], o[3]);
    }
  } else if constexpr (EPI == EPI8_GEGLU_BWD) {
    // staged tile = dout (bf16, as the unfused path stores it); chunk cq of row R = dout columns n .. n+7 ->
    // interleaved input-gradient positions ph .. ph+7 (h) and ph+32 .. (gate), ph = (n / 32) * 64 + n % 32
    const int n = n0 + cq * 8;
    const int ph = (n >> 5) * 64 + (n & 31);
#pragma unroll 2
    for (int p = 0; p < 16; ++p) {
      const int R = p * 16 + rq, m = m0 + R;
      if (m >= g.M) continue;
      const uint4 dv = *reinterpret_cast<const uint4*>(tl + tix(R, cq));
      const uint4 hv = *reinterpret_cast<const uint4*>(g.aux + (long)m * g.ldaux + ph);
      const uint4 gv = *reinterpret_cast<const uint4*>(g.aux + (long)m * g.ldaux + ph + 32);
      const uint32_t dw[4] = {dv.x, dv.y, dv.z, dv.w}, hw[4] = {hv.x, hv.y, hv.z, hv.w}, gw[4] = {gv.x, gv.y, gv.z, gv.w};
      uint32_t oh[4], og[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d0 = bf2f(dw[e] & 0xffff), d1 = bf2f(dw[e] >> 16);
        const float h0 = bf2f(hw[e] & 0xffff), h1 = bf2f(hw[e] >> 16);
        const float q0 = bf2f(gw[e] & 0xffff), q1 = bf2f(gw[e] >> 16);
        float c0, e0, c1, e1;
        gelu_erf_parts(q0, c0, e0);
        gelu_erf_parts(q1, c1, e1);
        oh[e] = pack2bf(d0 * q0 * c0, d1 * q1 * c1);
        og[e] = pack2bf(d0 * h0 * (c0 + 0.39894228040143268f * q0 * e0), d1 * h1 * (c1 + 0.39894228040143268f * q1 * e1));
      }
      bf16_t* o = reinterpret_cast<bf16_t*>(g.out) + (long)m * g.ldo + ph;
      *reinterpret_cast<uint4*>(o) = make_uint4(oh[0], oh[1], oh[2], oh[3]);
      *reinterpret_cast<uint4*>(o + 32) = make_uint4(og[0], og[1], og[2], og[3]);
    }
  } else {
    const bool has_r = g.resid != nullptr;
#pragma unroll 4
    for (int p = 0; p < 16; ++p) {
      const int R = p * 16 + rq, m = m0 + R;
      if (m >= g.M) continue;
      uint4 y = *reinterpret_cast<const uint4*>(tl + tix(R, cq));
      if (has_r) {  // residual added to the bf16-rounded projection (the unfused Linear + add)
        const uint4 rv = *reinterpret_cast<const uint4*>(g.resid + (long)m * g.ldr + n0 + cq * 8);
        const uint32_t yw[4] = {y.x, y.y, y.z, y.w}, rw[4] = {rv.x, rv.y, rv.z, rv.w};
        uint32_t o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          o[e] = pack2bf(bf2f(yw[e] & 0xffff) + bf2f(rw[e] & 0xffff), bf2f(yw[e] >> 16) + bf2f(rw[e] >> 16));
        y = make_uint4(o[0], o[1], o[2], o[3]);
      }
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(g.out) + (long)m * g.ldo + n0 + cq * 8) = y;
    }
  }
  }  // BN == 256
  tile_end:
  if constexpr (BN != 160) break;
  // every wave's epilogue LDS reads retired before the next tile's staging overwrites the ring (no vmcnt wait: the
  // stores keep draining)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }  // tiles
}

// persistent grid: one workgroup per CU (256 on MI355X; a multiple of 8 keeps every tile of a workgroup on its XCD)
// (benchmark knob PSO_GEMM8_GRID, tools build only: a larger value = one workgroup per tile)
#ifdef PSO_BENCH_KNOBS
static const int g_grid8 = [] {
  const char* e = getenv("PSO_GEMM8_GRID");
  return e ? atoi(e) : 256;
}();
#else
static constexpr int g_grid8 = 256;
#endif

template <int EPI, bool STAG, bool SPRIO, bool FP8 = false, int BN = 256, bool CONV = false>
int launch8(const Gemm8Args& g, hipStream_t st) {
  const int nblk = ((g.M + 255) / 256) * (g.N / BN);
  // 2 K-tile buffers: 128 KiB (256 x 256) / 104 KiB (256 x 160) / 144 KiB + a 4-KiB dummy slot (256 x 320)
  const size_t shm = (4 * HT + 4 * (BN / 2) * 64 + (BN == 320 ? 4 * 512 : 0)) * sizeof(bf16_t);
  static bool attr_done = false;
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)gemm8p_kernel<EPI, STAG, SPRIO, FP8, BN, CONV>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    attr_done = true;
  }
  // the demangled name rocprofv3 reports (every template argument), so traces and live attribution agree
  pso_note_kernel("gemm8p_kernel<%d, %s, %s, %s, %d, %s>", EPI, STAG ? "true" : "false", SPRIO ? "true" : "false",
                  FP8 ? "true" : "false", BN, CONV ? "true" : "false");
  // raster group aligned to the XCD chunks: each XCD walks nblk / 8 consecutive tile ids, so a group (group_m row
  // bands x all column tiles) that straddles two chunks puts a row band's column tiles on two XCDs and its A rows
  // are fetched into both L2s.  The largest group_m <= the requested one whose groups tile a chunk (C4's 12288 x
  // 1280 x 5120, 192 tiles: 1.97 -> 1.66x algorithmic fetch; profiles/r03_pmc_raster.txt; whole-round shapes keep 4)
  Gemm8Args ga = g;
  const int nbn = g.N / BN;
  if (pso_gemm_group_knob() == 0 && nblk >= 8 && nblk % 8 == 0) {  // (variant + 100 * rows forces a group)
    const int chunk = nblk / 8;
    int gm = g.group_m;
    while (gm > 1 && chunk % (gm * nbn) != 0) --gm;
    if (chunk % (gm * nbn) == 0) ga.group_m = gm;
  }
  gemm8p_kernel<EPI, STAG, SPRIO, FP8, BN, CONV><<<(BN == 160 && nblk > g_grid8) ? g_grid8 : nblk, 512, shm, st>>>(ga);
  return pso_check_launch(FP8 ? "pso_gemm_fp8" : "pso_gemm(8-phase)");
}

template <int EPI>
int launch8s(const Gemm8Args& g, hipStream_t st, int mode) {
#ifdef PSO_BENCH_KNOBS
  switch (mode & 3) {
    case 0: return launch8<EPI, true, false>(g, st);
    case 1: return launch8<EPI, false, false>(g, st);
    case 2: return launch8<EPI, true, true>(g, st);
    default: return launch8<EPI, false, true>(g, st);
  }
#else
  (void)mode;
  return launch8<EPI, true, false>(g, st);
#endif
}

}  // namespace

// Host entries used by gemm.hip (preconditions checked there): N % 256 == 0, K % 64 == 0, 16-B aligned rows, every
// operand's M * ld (or N * ld) below 2^30 elements (byte offsets of the buffer loads are 32-bit).
#ifdef PSO_BENCH_KNOBS
static int g_skip_epi8 = 0;
// benchmark knobs, bit 1: wave groups in lockstep (default: staggered by half a phase, +10-18 % on every UNet shape,
// tools/gemm8_ab.py); bit 2: static priority for waves 4-7
static int g_mode8 = 0;
extern "C" void pso_gemm8p_skip_epilogue(int on) { g_skip_epi8 = on & 1; g_mode8 = (on >> 1) & 3; }
#else
static constexpr int g_skip_epi8 = 0, g_mode8 = 0;
#endif

int pso_gemm8p_run(int epi, int M, int N, int K, const void* a, long lda, const void* w, long ldw, const void* a2,
                   long lda2, int K2, const void* w2, long ldw2, int tail_m, int tail_group_n, float alpha,
                   const void* bias, const void* resid, long ldr, void* out, long ldo, void* out2, long ldo2,
                   int pre_rows, const void* aux, long ldaux, int group_m, hipStream_t st) {
  Gemm8Args g{};
  g.a = (const bf16_t*)a; g.lda = lda; g.w = (const bf16_t*)w; g.ldw = ldw;
  g.M = M; g.N = N; g.K = K;
  g.a2 = (const bf16_t*)a2; g.lda2 = lda2; g.K2 = a2 ? K2 : 0; g.w2 = (const bf16_t*)w2; g.ldw2 = ldw2;
  g.tail_m = tail_m; g.tail_group_n = a2 ? tail_group_n : 0;
  g.alpha = alpha; g.bias = (const bf16_t*)bias; g.resid = (const bf16_t*)resid; g.ldr = ldr;
  g.out = out; g.ldo = ldo; g.out2 = out2; g.ldo2 = ldo2; g.pre_rows = pre_rows;
  g.aux = (const bf16_t*)aux; g.ldaux = ldaux;
  g.group_m = group_m; g.skip_epi = g_skip_epi8;
  if (epi == EPI8_GEGLU) return launch8s<EPI8_GEGLU>(g, st, g_mode8);
  if (epi == EPI8_GEGLU_BWD) return launch8s<EPI8_GEGLU_BWD>(g, st, g_mode8);
  return launch8s<EPI8_NONE>(g, st, g_mode8);
}

// 256 x 160 tiles (N % 160 == 0, K % 64 == 0, plain epilogue; preconditions checked in gemm.hip)
int pso_gemm8p160_run(int M, int N, int K, const void* a, long lda, const void* w, long ldw, const void* a2, long lda2,
                      int K2, const void* w2, long ldw2, int tail_m, int tail_group_n, float alpha, const void* bias,
                      const void* resid, long ldr, void* out, long ldo, int group_m, hipStream_t st) {
  Gemm8Args g{};
  g.a = (const bf16_t*)a; g.lda = lda; g.w = (const bf16_t*)w; g.ldw = ldw;
  g.M = M; g.N = N; g.K = K;
  g.a2 = (const bf16_t*)a2; g.lda2 = lda2; g.K2 = a2 ? K2 : 0; g.w2 = (const bf16_t*)w2; g.ldw2 = ldw2;
  g.tail_m = tail_m; g.tail_group_n = a2 ? tail_group_n : 0;
  g.alpha = alpha; g.bias = (const bf16_t*)bias; g.resid = (const bf16_t*)resid; g.ldr = ldr;
  g.out = out; g.ldo = ldo; g.group_m = group_m; g.skip_epi = g_skip_epi8;
  return launch8<EPI8_NONE, true, false, false, 160>(g, st);
}

// 256 x 320 tiles (N % 320 == 0, K % 64 == 0, plain epilogue; preconditions checked in gemm.hip)
int pso_gemm8p320_run(int M, int N, int K, const void* a, long lda, const void* w, long ldw, const void* a2, long lda2,
                      int K2, const void* w2, long ldw2, int tail_m, int tail_group_n, float alpha, const void* bias,
                      const void* resid, long ldr, void* out, long ldo, int group_m, hipStream_t st) {
  Gemm8Args g{};
  g.a = (const bf16_t*)a; g.lda = lda; g.w = (const bf16_t*)w; g.ldw = ldw;
  g.M = M; g.N = N; g.K = K;
  g.a2 = (const bf16_t*)a2; g.lda2 = lda2; g.K2 = a2 ? K2 : 0; g.w2 = (const bf16_t*)w2; g.ldw2 = ldw2;
  g.tail_m = tail_m; g.tail_group_n = a2 ? tail_group_n : 0;
  g.alpha = alpha; g.bias = (const bf16_t*)bias; g.resid = (const bf16_t*)resid; g.ldr = ldr;
  g.out = out; g.ldo = ldo; g.group_m = group_m; g.skip_epi = g_skip_epi8;
  return launch8<EPI8_NONE, true, false, false, 320>(g, st);
}

// GEGLU forward on 256 x 320 tiles (N % 320 == 0, lda == ldw; preconditions checked in gemm.hip): the interleaved
// pre-activation a . w^T + bias (rows < pre_rows to out2) and out = h * gelu(gate), bit-identical to the 256 x 256 form
int pso_gemm8p320_geglu_run(int M, int N, int K, const void* a, long lda, const void* w, long ldw, const void* bias,
                            void* out, long ldo, void* out2, long ldo2, int pre_rows, int group_m, hipStream_t st) {
  Gemm8Args g{};
  g.a = (const bf16_t*)a; g.lda = lda; g.w = (const bf16_t*)w; g.ldw = ldw;
  g.M = M; g.N = N; g.K = K; g.tail_m = M;
  g.alpha = 1.f; g.bias = (const bf16_t*)bias;
  g.out = out; g.ldo = ldo; g.out2 = out2; g.ldo2 = ldo2; g.pre_rows = pre_rows;
  g.group_m = group_m; g.skip_epi = g_skip_epi8;
  return launch8<EPI8_GEGLU, true, false, false, 320>(g, st);
}

// GEGLU backward on 256 x 320 tiles (N % 320 == 0, lda == ldw; preconditions checked in gemm.hip): dout = a . w^T,
// out = the interleaved [dout * gelu(g) | dout * h * gelu'(g)] from the interleaved pre-activation aux
int pso_gemm8p320_geglu_bwd_run(int M, int N, int K, const void* a, long lda, const void* w, long ldw, const void* aux,
                                long ldaux, void* out, long ldo, int group_m, hipStream_t st) {
  Gemm8Args g{};
  g.a = (const bf16_t*)a; g.lda = lda; g.w = (const bf16_t*)w; g.ldw = ldw;
  g.M = M; g.N = N; g.K = K; g.tail_m = M;
  g.alpha = 1.f; g.out = out; g.ldo = ldo; g.aux = (const bf16_t*)aux; g.ldaux = ldaux;
  g.group_m = group_m; g.skip_epi = g_skip_epi8;
  return launch8<EPI8_GEGLU_BWD, true, false, false, 320>(g, st);
}

// 3x3 / stride 1 / pad 1 implicit-GEMM convolution on 256 x 320 tiles (preconditions checked in gemm.hip: C % 64 == 0,
// H*W % 256 == 0, Cout % 320 == 0, weight rows [Cout][3][3][C], bf16 output)
int pso_gemm8p320_conv_run(int B, int H, int W, int C, const void* x, const void* w, int Cout, float alpha,
                           const void* bias, const void* rowbias, long ld_rowbias, const void* resid, long ldr,
                           void* out, long ldo, int group_m, hipStream_t st) {
  Gemm8Args g{};
  g.a = (const bf16_t*)x; g.lda = C; g.w = (const bf16_t*)w; g.ldw = 9L * C;
  g.M = B * H * W; g.N = Cout; g.K = 9 * C;
  g.tail_m = g.M;
  g.alpha = alpha; g.bias = (const bf16_t*)bias; g.resid = (const bf16_t*)resid; g.ldr = ldr;
  g.out = out; g.ldo = ldo; g.group_m = group_m; g.skip_epi = g_skip_epi8;
  g.cv_H = H; g.cv_W = W; g.cv_lh = __builtin_ctz(H); g.cv_lw = __builtin_ctz(W); g.cv_ct = C / 64; g.cv_recip = (1 << 20) / (C / 64) + 1;
  g.rowbias = (const bf16_t*)rowbias; g.ld_rowbias = ld_rowbias;
  return launch8<EPI8_NONE, true, false, false, 320, true>(g, st);
}

// FP8 form (pso_amd.h, pso_gemm_fp8): staggered wave groups, epilogue 0 (bias / alpha / residual) or 1 (GEGLU)
extern "C" int pso_gemm_fp8(int epi, int M, int N, int K, const void* a, long lda, const void* sa, const void* w,
                            long ldw, const void* sw, const void* a2, long lda2, int K2, const void* sa2,
                            const void* w2, long ldw2, const void* sw2, int tail_m, int tail_group_n, float alpha,
                            const void* bias, const void* resid, long ldr, void* out, long ldo, void* out_pre,
                            long ld_pre, int pre_rows, void* stream) {
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  PSO_ARG_CHECK(epi == EPI8_NONE || epi == EPI8_GEGLU, "pso_gemm_fp8: epi must be 0 (plain) or 1 (GEGLU)");
  PSO_ARG_CHECK(M > 0 && N > 0 && (N % 256) == 0 && K > 0 && (K % 128) == 0,
                "pso_gemm_fp8: need N %% 256 == 0, K %% 128 == 0 (M=%d N=%d K=%d)", M, N, K);
  PSO_ARG_CHECK(a && sa && w && sw && out, "pso_gemm_fp8: null operand");
  PSO_ARG_CHECK(a16(a) && a16(w) && (lda % 16) == 0 && (ldw % 16) == 0 && a16(out) && (ldo % 8) == 0,
                "pso_gemm_fp8: A / W / out need 16-B aligned rows");
  PSO_ARG_CHECK((long)M * lda < (1L << 31) && (long)N * ldw < (1L << 31), "pso_gemm_fp8: operand above 2 GiB");
  PSO_ARG_CHECK(!a2 || (w2 && sa2 && sw2 && K2 > 0 && (K2 % 16) == 0 && a16(a2) && a16(w2) && (lda2 % 16) == 0 &&
                        (ldw2 % 16) == 0 && tail_m > 0 && (long)tail_m * lda2 < (1L << 31) &&
                        (tail_group_n == 0 || (tail_group_n % 256) == 0)),
                "pso_gemm_fp8: bad LoRA tail operands");
  PSO_ARG_CHECK(!resid || (a16(resid) && (ldr % 8) == 0), "pso_gemm_fp8: residual needs 16-B aligned rows");
  PSO_ARG_CHECK(epi != EPI8_GEGLU || (bias && !resid && (!out_pre || (a16(out_pre) && (ld_pre % 8) == 0))),
                "pso_gemm_fp8: GEGLU needs a bias, no residual, aligned out_pre");
  Gemm8Args g{};
  g.a = (const bf16_t*)a; g.lda = lda; g.w = (const bf16_t*)w; g.ldw = ldw;
  g.M = M; g.N = N; g.K = K;
  g.a2 = (const bf16_t*)a2; g.lda2 = lda2; g.K2 = a2 ? K2 : 0; g.w2 = (const bf16_t*)w2; g.ldw2 = ldw2;
  g.tail_m = a2 ? (tail_m < M ? tail_m : M) : M; g.tail_group_n = a2 ? tail_group_n : 0;
  g.alpha = alpha; g.bias = (const bf16_t*)bias; g.resid = (const bf16_t*)resid; g.ldr = ldr;
  g.out = out; g.ldo = ldo; g.out2 = out_pre; g.ldo2 = ld_pre; g.pre_rows = pre_rows > 0 ? pre_rows : M;
  g.group_m = 4; g.skip_epi = g_skip_epi8;
  g.sa = (const uint8_t*)sa; g.sw = (const uint8_t*)sw; g.sa2 = (const uint8_t*)sa2; g.sw2 = (const uint8_t*)sw2;
  const hipStream_t st = (hipStream_t)stream;
  if (epi == EPI8_GEGLU) return launch8<EPI8_GEGLU, true, false, true>(g, st);
  return launch8<EPI8_NONE, true, false, true>(g, st);
}
