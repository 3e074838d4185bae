/* Benchmark knobs of the TOOLS build (libpso_amd_knobs.so: the same sources compiled with -DPSO_BENCH_KNOBS).
 *
 * The product library libpso_amd.so (include/pso_amd.h) has none of these: its dispatch is the automatic one, its knob
 * state is compile-time constant, and the measured-not-kept kernel forms are not compiled into it.  The knobs build
 * adds mutable process-wide dispatch overrides for A/B measurements (the tools/ scripts) and for the tests that pin an
 * alternative kernel form to the default's bits (run in a child process: tests/test_knobs_build.py).  Not
 * thread-safe; never on a product path.
 */
#ifndef PSO_AMD_KNOBS_H
#define PSO_AMD_KNOBS_H

#include "pso_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* GEMM dispatch override: v % 100 = variant (0 = automatic per shape; 1-29 force a tile shape, 30-56 flip one rule
 * of the automatic dispatch -- gemm.hip run_gemm), v / 100 = raster-group rows (0 = automatic). */
void pso_gemm_set_variant(int v);
/* 8-phase kernels: bit 0 = keep the accumulators live but store nothing (main-loop cost), bits 1-2 = wave-group
 * schedule (lockstep / static priority). */
void pso_gemm8p_skip_epilogue(int on);
/* Split count of pso_gemm_tn over the reduction rows (0 = automatic). */
void pso_gemm_tn_set_split(int ks);
/* Attention: ones digit = forward form (0 auto, 1 lane-local growth test, 2 / 4 force 32 / 64 rows per wave, 5-9 the
 * first-round loop), tens digit = backward form (0 default, 1 / 3 older forms, 4 64 keys per wave, 5 / 6 deeper
 * rings, 7 the dQ + dK/dV launches for short key sequences too (instead of the one-pass attn_bwd_x_kernel), 8 / 9 the
 * 8-wave ping-pong dK/dV), 100s = VALU row sums, 1000s = segment clock trace of the ping-pong form, 10000 * qs = the
 * query splits of attn_bwd_x_kernel (0 automatic). */
void pso_attention_set_variant(int v);
/* Segment-start clocks of the last traced ping-pong dK/dV launch (2 x 520 unsigned 64-bit, group-major). */
int pso_attn_pp_trace(unsigned long long* out);

#ifdef __cplusplus
}
#endif

#endif /* PSO_AMD_KNOBS_H */
