/*
 * csm_hip.h -- C ABI of libcsm_hip.so, the MI355X (gfx950) engine behind the
 * csm_mlx drop-in API.  Plain pointers and sizes only; no torch types.
 *
 * Every entry point returns 0 on success or a negative csm_status; the message
 * of the last failure on the calling thread is available from csm_last_error().
 * The Python layer (csm-mlx_amd/csm_mlx/_lib.py) binds these with ctypes and
 * maps failures to the reference's exceptions.
 *
 * Reference interfaces replaced (all /root/reference/csm_mlx/...):
 *   csm_engine_create / csm_load_tensor    CSM(args) + Module.load_weights
 *                                          (models.py:31-77; README.md:38-40)
 *   csm_set_rope_table                     Llama3ScaledRoPE.rope_init cache (attention.py:57-92)
 *   csm_begin / csm_prefill                generate(): prompt assembly + first generate_frame
 *                                          backbone pass (generation.py:108-140)
 *   csm_run_frames                         the frame loop: generate_frame (generation.py:21-92)
 *                                          + EOS test (:151) + feedback row (:156-161)
 *   csm_read_codes                         the stacked samples (generation.py:154, :167-170)
 *   mimi_*                                 moshi_mlx Mimi encode / decode / decode_step /
 *                                          reset_state (tokenizers.py:14-21, 61-85, 148-150;
 *                                          generation.py:224-258)
 */
#ifndef CSM_HIP_H
#define CSM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum csm_status {
  CSM_OK = 0,
  CSM_ERR_ARG = -1,       /* bad argument / shape (ValueError) */
  CSM_ERR_HIP = -2,       /* HIP runtime failure (RuntimeError) */
  CSM_ERR_STATE = -3,     /* call out of order, e.g. weights missing */
  CSM_ERR_TOO_LONG = -4   /* prompt + frames exceed the 2048-position window (generation.py:132-137) */
};

/* CSM_Q4: MLX affine int4, group 64 (nn.quantize(model, 64, 4)); as a host source dtype, CSM_U32 marks
 * MLX-packed int4 weights (8 nibbles per uint32, element j at bits 4*(j%8)). */
enum csm_dtype { CSM_F32 = 0, CSM_BF16 = 1, CSM_Q4 = 2, CSM_U32 = 3 };

typedef struct csm_llama_dims {
  int n_layers, hidden, n_heads, n_kv_heads, head_dim, intermediate;
  float eps;
} csm_llama_dims;

typedef struct csm_dims {
  csm_llama_dims backbone, decoder;
  int n_text_vocab, n_audio_vocab, n_audio_codebooks;
  int max_seq_len; /* RoPE / KV window: 2048 (generation.py:132, attention.py:38) */
} csm_dims;

typedef struct csm_engine csm_engine;

const char* csm_last_error(void);
int csm_device_count(int* n);

/* weight_dtype: storage of every Linear/Embedding weight (CSM_F32 parity mode, CSM_BF16 perf, CSM_Q4 int4
 * g64: float weights loaded into it are quantized on the device; MLX-quantized checkpoints load as
 * <name>.weight (CSM_U32 [n][K/8]) + <name>.scales + <name>.biases ([n][K/64] f32 or bf16)).
 * audio_head is never quantized (bf16 in a CSM_Q4 engine). */
int csm_engine_create(const csm_dims* dims, int device, int weight_dtype, int max_batch, int max_frames,
                      csm_engine** out);
int csm_engine_destroy(csm_engine* e);
/* name: MLX parameter key; host: src_dtype data, C-contiguous, shape as in the checkpoint */
int csm_load_tensor(csm_engine* e, const char* name, const void* host, int src_dtype, const int64_t* shape,
                    int ndim);
/* which: 0 backbone, 1 decoder; table [max_seq_len][head_dim/2][2] = (cos, sin) float32 */
int csm_set_rope_table(csm_engine* e, int which, const float* table, int n_pos, int head_dim);
/* returns CSM_ERR_STATE and names the first missing tensor when weights are incomplete */
int csm_weights_ready(csm_engine* e);
/* Multi-GPU weight distribution (no reference counterpart: the reference is single-device).  The
 * engine's resident weight buffers -- every Linear / Embedding / norm / head matrix in kernel layout
 * and storage dtype, in a fixed order -- so one rank's loaded buffers can be broadcast device to
 * device (RCCL) into identically created engines.  *n = buffer count; up to cap (ptr, bytes) pairs
 * are written.  csm_weights_received then marks a receiving engine's weights as loaded (derived
 * tables and tiled copies rebuild at the next csm_begin). */
int csm_weight_buffers(csm_engine* e, void** ptrs, uint64_t* bytes, int cap, int* n);
int csm_weights_received(csm_engine* e);
/* nn.quantize(model, group_size, bits) (run_streaming_csm_mlx.py:811-818; README.md:108-111): convert every
 * loaded Linear / Embedding weight to int4 in place (MLX affine rule, oracle/quant_oracle.py).  Only
 * group_size 64, bits 4.  audio_head and the norms keep their dtype. */
int csm_quantize(csm_engine* e, int group_size, int bits);

/* Start a batch of B utterances.  temperature 0 = greedy (generation.py:51); top_k 0 = off.
 * seeds[B]: per-utterance sampling seeds (build's counter-based Gumbel sampler). */
int csm_begin(csm_engine* e, int B, const uint64_t* seeds, float temperature, int top_k);
/* mlx_lm make_sampler's filters beyond top_k (README.md:49, cli/generate.py:168-174: temp, top_p, min_p,
 * min_tokens_to_keep, top_k), applied in its order top_k -> top_p -> min_p to the log-probabilities
 * before the Gumbel-max draw (oracle/csm_oracle.py filter_keep).  top_p in (0, 1) and min_p != 0 are
 * active; call after csm_begin, before the first frame (csm_begin resets them to off). */
int csm_set_sampler_filters(csm_engine* e, double top_p, double min_p, int min_tokens_to_keep);
/* Prompt rows of utterance b: tokens/mask [T][K+1] (text id in the last column). */
int csm_prefill(csm_engine* e, int b, int T, const int32_t* tokens, const uint8_t* mask);
/* csm_prefill for several utterances at once (the rows of generate_batch's prompts): utts[i] gets
 * Ts[i] rows, rows of all of them concatenated in tokens / masks.  Up to max_seq_len rows per pass
 * run as ONE pass of every backbone projection (the weights stream once for all of them; each row
 * keeps its own utterance's KV cache and positions), so the results are those of csm_prefill per
 * utterance up to summation order.  No reference counterpart (the reference is batch-1). */
int csm_prefill_batch(csm_engine* e, int n, const int32_t* utts, const int32_t* Ts, const int32_t* tokens,
                      const uint8_t* masks);
/* Generate up to nframes frames for the whole batch (one HIP graph replay per frame).
 * *all_done (optional) = 1 when every utterance hit EOS. */
int csm_run_frames(csm_engine* e, int nframes, int* all_done);
/* csm_run_frames without waiting on this chunk: enqueues nframes frames, then waits for the PREVIOUS
 * chunk enqueued by this call (not for the frames just enqueued) and sets *prev_all_done = 1 when every
 * utterance had hit EOS by its end, 0 when not, -1 when there was no previous chunk.  The generation loop
 * (generation.py:139-161) thus tests EOS one chunk behind while the next chunk already runs, so the GPU
 * never idles on the host's poll; frames enqueued past an all-EOS chunk change no returned code or frame
 * count.  CSM_ERR_HIP if a persistent kernel's hand-off timed out in the polled chunk. */
int csm_run_frames_ahead(csm_engine* e, int nframes, int* prev_all_done);
/* One frame (generation.py:21-92 + the EOS test :151) with its result handed back: out_codes [B][K]
 * int32 = the frame's codes (the `sample` generate_frame returns), done [B] = utterances past EOS.
 * Either pointer may be NULL.  Equivalent to csm_run_frames(e, 1, NULL) followed by a read of the
 * frame's codes; CSM_ERR_STATE when the engine's frame capacity is exhausted. */
int csm_frame_step(csm_engine* e, int32_t* out_codes, uint8_t* done);
/* One frame split around a host hook on the c0 logits (logits_processors, generation.py:42-49):
 * csm_frame_c0_logits runs the backbone step + codebook0_head and copies logits [B][V] out;
 * csm_frame_finish takes the (processed) logits [B][V] back, picks c0 (arg-max when greedy, else the
 * engine's sampler) and runs the 31 decoder steps.  Replaces generate_frame's processor loop
 * (generation.py:44-49) -- called once per frame instead of csm_run_frames. */
int csm_frame_c0_logits(csm_engine* e, float* logits);
int csm_frame_finish(csm_engine* e, const float* logits, int* all_done);
/* A frame sampled on the host by an arbitrary sampler callable (the sampler= keyword the reference CLI
 * passes, cli/generate.py:168-174, :197-199; upstream csm-mlx applied it to every codebook's logits):
 * after csm_frame_c0_logits, call csm_frame_host_step K times; call i (1..K) hands the host's codes[B]
 * of codebook i-1 to the engine, which feeds them forward (as csm_frame_forced does) and runs decoder
 * step i + its head: logits [B][V] receive codebook i's logits for calls 1..K-1; call K finishes the
 * frame (history, EOS) and sets *all_done.  Replaces csm_frame_finish for that frame. */
int csm_frame_host_step(csm_engine* e, const int32_t* codes, float* logits, int* all_done);
/* Teacher-forced frame (the scoring form of trainer.py:203-318 compute_loss): the backbone step
 * consumes the previous frame, then every head stores its logits while the code fed forward is
 * codes[B][K] (the target frame).  c0_logits [B][V] and ci_logits [K-1][B][V] (optional, may be
 * NULL) receive the logits that predict codes[b][0] and codes[b][1..K-1]; ce [B][K] (optional)
 * their cross entropies logsumexp(logits) - logits[code], reduced on the device. */
int csm_frame_forced(csm_engine* e, const int32_t* codes, float* c0_logits, float* ci_logits, float* ce);
/* hist [F][B][K] int32 of the frames generated so far, n_frames[B] emitted frames (EOS excluded),
 * done[B].  Any pointer may be NULL. */
int csm_read_codes(csm_engine* e, int32_t* hist, int32_t* n_frames, uint8_t* done, int* frames_run);
/* Debug / parity taps: "h_last" [B][D], "c0_logits" [B][Vpad], "ci_logits" [K-1][B][Vpad], "codes" [B][K],
 * "audio_head" [K-1][Vpad][Dd] (f32 or bf16 bits),
 * "weight:<MLX name>" a whole (unfused) Linear / Embedding matrix in its device layout (int4: nibbles
 * [N][K/2] then {scale, bias} bf16 pairs [N][K/64]). */
int csm_debug_read(csm_engine* e, const char* what, void* host, int64_t nbytes, int64_t* needed);
/* The module views of CSM (models.py:53-92): rows[n] of a stored Linear / Embedding weight (MLX key,
 * e.g. "audio_embeddings.weight") as fp32 [n][in] (int4: the dequantized values the kernels use) --
 * CSM.embed_tokens / embed_audio / <module>.weight -- and a Linear applied on the GPU: y [M][out] =
 * x [M][in] . W^T (the GEMV's arithmetic) for a Linear key, or x [M][Dd] . audio_head[i] for
 * "audio_head.<i>" (generation.py:79). */
int csm_read_rows(csm_engine* e, const char* name, int n, const int32_t* rows, float* out);
int csm_linear(csm_engine* e, const char* name, int M, const float* x, float* y);
/* Device pointer of the code history [F][B][K] (for on-device Mimi decode) */
int csm_codes_device_ptr(csm_engine* e, void** dev_ptr);
int csm_synchronize(csm_engine* e);
/* ------------------------------------------------------------------ Mimi codec */
typedef struct mimi_dims {
  int channels, dimension, n_filters, n_ratios, ratios[8];
  int kernel_size, residual_kernel_size, last_kernel_size, compress;
  int num_heads, num_layers, dim_feedforward, context;
  int n_q, bins, codebook_dim, downsample_stride;
  float norm_eps;
  int gelu_erf;   /* 0: tanh approximation (mlx gelu_approx), 1: exact */
  int attn_mode;  /* 0: moshi_mlx (no mask inside a call), 1: causal sliding window */
} mimi_dims;

typedef struct mimi_codec mimi_codec;

int mimi_create(const mimi_dims* dims, int device, int max_batch, int max_frames, mimi_codec** out);
int mimi_destroy(mimi_codec* m);
int mimi_load_tensor(mimi_codec* m, const char* name, const void* host, int src_dtype, const int64_t* shape,
                     int ndim);
/* RoPE table for the codec transformer: [n_pos][head_dim/2][2] */
int mimi_set_rope_table(mimi_codec* m, const float* table, int n_pos, int head_dim);
int mimi_weights_ready(mimi_codec* m);
/* pcm [B][N] float32 host -> codes [B][n_q][Tf] int32 host; *n_frames_out = Tf */
int mimi_encode(mimi_codec* m, int B, int N, const float* pcm, int32_t* codes, int* n_frames_out);
/* as mimi_encode with utterance b's N samples at rows[b] (pcm NULL): the batched context encode of
   tokenize_segments_batch (reference tokenizers.py:61-85 per segment) without a host-side stacking copy */
int mimi_encode_rows(mimi_codec* m, int B, int N, const float* pcm, const float* const* rows, int32_t* codes,
                     int* n_frames_out);
/* codes [B][n_q][F] -> pcm [B][F*frame_size].  codes_on_device / pcm_on_device select device pointers;
 * codes_layout 0 = [B][n_q][F], 1 = engine history [F][B][n_q] */
int mimi_decode(mimi_codec* m, int B, int F, const int32_t* codes, int codes_on_device, int codes_layout,
                float* pcm, int pcm_on_device);
/* streaming: reset per-utterance state, then one frame at a time: codes [B][n_q] -> pcm [B][frame_size] */
int mimi_reset_state(mimi_codec* m, int B);
int mimi_decode_step(mimi_codec* m, int B, const int32_t* codes, float* pcm);

#ifdef __cplusplus
}
#endif
#endif /* CSM_HIP_H */
