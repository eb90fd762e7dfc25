/*
 * csm_hip_prof.h -- tuning and profiling hooks of libcsm_hip.so.
 *
 * NOT part of the reference-facing ABI (include/csm_hip.h): no reference interface corresponds to
 * these.  bench.py uses csm_bench_dec_frame / csm_bench_gemv for the live roofline of the dominant kernel; the parity
 * tests use csm_set_option to A/B the opt-in fused paths against the default launches.
 */
#ifndef CSM_HIP_PROF_H
#define CSM_HIP_PROF_H

#include "csm_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Replay one projection of the frame `iters` times on the engine stream (one launch per layer in
 * turn, as the frame does), timed with HIP events on that stream.  which = stack*4 + kind, stack 0
 * backbone / 1 decoder, kind 0 = norm+gate/up+SiLU, 1 = down+residual, 2 = norm+QKV+RoPE,
 * 3 = o_proj+residual; M rows (M >= 8 on bf16 / int4 weights: the MFMA GEMM the batched frame runs).
 * *bytes = algorithmic bytes per launch (weights in their storage format + activations read and
 * written). */
int csm_bench_gemv(csm_engine* e, int which, int M, int iters, float* avg_us, double* bytes);

/* Replay the persistent frame decoder (dec_frame.hip: codebook0_head + 31 decoder steps of a batch-1
 * greedy frame, one launch) `iters` times on the engine stream from the current h_last, timed with HIP
 * events on that stream.  Needs an engine on which that kernel is active and a prefilled utterance.
 * *bytes = algorithmic bytes per launch: every head and decoder weight the frame reads once in bf16,
 * the folded-table rows, h_last, and the decoder K/V rows read and appended. */
int csm_bench_dec_frame(csm_engine* e, int iters, float* avg_us, double* bytes);
/* The persistent backbone step (bb_step.hip) replayed `iters` times for the last decoded row (same x,
 * same position; idempotent): average launch time (HIP events, engine stream) and the algorithmic
 * bytes one launch moves (every backbone weight in bf16 + the K/V rows).  CSM_ERR_STATE when the
 * engine does not run it (not batch-1 bf16 csm_1b shapes, or no frame run yet). */
int csm_bench_bb_step(csm_engine* e, int iters, float* avg_us, double* bytes);
/* The persistent batched decoder step (dec_step_xs.hip; batch 1..32 bf16 / 1..64 int4 on the streaming
 * path) replayed `iters` times for the last codebook step of the last frame (same partials, same
 * position; idempotent): average launch time and the algorithmic bytes one launch reads (decoder weights
 * in their storage format + the bf16 audio_head slice + folded table rows + K/V history).  CSM_ERR_STATE
 * when the step kernel is not active on this engine. */
int csm_bench_dec_xsd(csm_engine* e, int iters, float* avg_us, double* bytes);

/* Tuning / debug switches (re-capture the frame graphs), per engine: "fold_proj" (decoder steps >= 2
 * gather projection(E_a[c]) from a table built at csm_begin, default 1), "qkv0_tab" (decoder layer 0's
 * q, k, v gathered from a table at steps >= 2, default 1), "qkv0_tab_batched" (0: batched frames run
 * layer 0's QKV projection instead, default 1), "dec_frame" (batch-1 greedy bf16 frames on the
 * persistent frame decoder, dec_frame.hip: codebook0_head + 31 decoder steps in one launch, default 1),
 * "bb_step" (batch-1 bf16 backbone rows on the persistent backbone step, bb_step.hip: 16 blocks + the
 * final norm in one launch, default 1), "dec_frame_stamps" / "bb_step_stamps" (per-hand-off clock
 * stamps of the persistent kernels, read back with csm_debug_read, default 0), "linear_mfma" (csm_linear
 * runs the batched frame's MFMA GEMM at >= 8 rows instead of the GEMV, default 0: the GEMM's kernel
 * tests), "gemm_xs" (the batched depth decoder on the streaming matrix-core GEMM, gemm_xs.hip,
 * default 1), "bb_xs" (the batched backbone on it too, default 1), "prefill_rows" (row cap of one
 * csm_prefill_batch group, 0 = the engine's capacity), "attn_prefill" (prompt attention on the fp32 matrix
 * cores, a block per 64-row prompt run and kv head, default 1; 0 = one block per row, tests), "dec_xsd"
 * (codebook steps >= 2 of the streaming path on the persistent batched decoder step, dec_step_xs.hip:
 * <= 32 bf16 / <= 64 int4 rows, default 1), "dec_xsd_head" (its head in the same launch, default 1),
 * "dec_xsd_sample" (sampled top-k steps: sample_kernel's sampler in the same launch too, default 1),
 * "dec_xsd_stamps" (its per-role clock marks, csm_debug_read "dec_xsd_stamps", default 0),
 * "inject_handoff_error" (test hook).
 * Process-wide lab knobs are environment variables read once (CSM_NT_MASK, CSM_GEMV_XL, CSM_XS_*). */
int csm_set_option(csm_engine* e, const char* key, int value);

/* Launch geometry the streaming matrix-core GEMM (gemm_xs.hip) would use for an (N, K) projection at M
 * rows (head != 0: an arg-max / SiLU launch) with weights of dtype wdt (CSM_BF16 or CSM_Q4): out[4] =
 * {weight-row tiles of 32 per block, K slices, ring depth, waves per block}.  Returns 1 if the shape is
 * eligible for that dtype (every 64-deep K stage falls on exactly one wave of one slice; int4: at most
 * Q4_XG stages per slice), else 0.  Host-only (no device call). */
int csm_xs_shape(int N, int K, int M, int head, int wdt, int* out);

/* The int4 GEMV's tiling for an [N][K] matrix (q4_kernels.hip): out[3] = {threads per row group G, K
 * steps per thread, rows per 256-thread block}.  Returns 1 if the shape is supported, else 0.  Host-only. */
int csm_q4_gemv_shape(int N, int K, int* out);

/* The matrix-core GEMMs' int4 -> bf16 expansion (xs.h q4_word_bf16) of n uint32 words of MLX nibbles, on
 * the current device: out[4 n] = the bf16 pairs (low half first) of the nibbles in order.  Test hook
 * (tests/test_gemm_kernel_gpu.py checks every nibble value at every position).  Returns CSM_OK or an error. */
int csm_q4_expand(const uint32_t* words, int n, uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* CSM_HIP_PROF_H */
