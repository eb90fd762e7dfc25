// Kernel parameter blocks and launchers shared by the CSM engine and the Mimi codec.
#pragma once
#include <unordered_map>

#include "common.h"

enum { WDT_F32 = 0, WDT_BF16 = 1, WDT_Q4 = 2 };  // WDT_Q4: MLX affine int4, group 64 (common.h layout)
enum { EPI_STORE = 0, EPI_ADD = 1, EPI_SILU_MUL = 2, EPI_QKV = 3, EPI_GELU = 4, EPI_ARGMAX = 5 };
enum { ATTN_CAUSAL = 0, ATTN_WINDOW = 1, ATTN_BLOCK = 2 };

// MFMA-path state owned by one engine (csm_engine::ws): split-K slice partials and arrival tickets,
// sized by gemm_reserve outside graph capture, and the fragment-tiled copy of every weight matrix
// the matrix cores read (row-major matrix -> its tiled copy, gemm_retile).
struct GemmWs {
  float* kpart = nullptr;
  size_t bytes = 0;
  unsigned* tickets = nullptr;
  size_t n = 0;
  std::unordered_map<const void*, const void*> tiled;
};

struct GemvParams {
  const void* W;      // [N][K] weight (bf16 or f32)
  int N, K;
  const float* x;     // [M][xs] activations (row m at x + m*xs)
  int xs, M;
  const float* nw;    // RMSNorm weight (NORM=1)
  float eps;
  float* out;         // output rows (stride os)
  int os;
  const float* scale; // EPI_ADD: optional per-column scale (Mimi LayerScale)
  int gelu_erf;       // EPI_GELU: 1 = exact erf gelu, 0 = tanh approximation
  // EPI_QKV
  int Hq, Hkv, hd, S_cap;
  const float* rope;  // [S][hd/2][2] cos/sin
  float* kc;          // [B][Hkv][S_cap][hd]
  float* vc;
  RowMap rm;
  int epi;            // set by launch_gemv
  // EPI_ARGMAX: logits stored to out AND the block's best (value, first index) for each row
  // packed as (orderable float << 32 | ~index) into part[m * part_stride + blockIdx.x]
  unsigned long long* part;
  int part_stride, n_valid;
  // x gather mode (x_codes != null): row m of x is table[(code(m) + V*cb) * K] where code(m) is
  // the arg-max of xpart[b(m) * xpart_stride + 0..xpart_n); with x_step1 rows alternate
  // [x_dense row b (h_last), table row] (decoder step 1).  Block 0 writes codes[b*K_cb + cb].
  const unsigned long long* xpart;
  int xpart_stride, xpart_n;
  const void* xtab;
  int xV, xcb, x_step1, x_codes_K;
  int* x_codes;
  int xtab_f32;         // gathered table rows are fp32 (else the weight type)
  int xtab_q4_rows;     // int4 weights: total rows of the (quantized) gathered table
  float* x_copy;        // if set: block 0 also stores the raw (un-normed) x rows here [M][K]
  float* qkv_tab;       // EPI_QKV table build: rows [M][(Hq + 2 Hkv) hd] instead of q / KV cache
  // MFMA path split-K (set by launch_gemm_mfma from ws): slice partials [ksplit][M][N], sum-of-squares [ksplit][M]
  GemmWs* ws;            // the calling engine's scratch (host pointer; required for split launches)
  unsigned lab_launch;   // lab builds of gemm_xs (XS_STAMPS): launch index for the phase stamps
  const void* Wt;        // the weight's fragment-tiled copy (looked up in ws->tiled by launch_gemm_mfma)
  float* kpart;          // [tile][m chunk][slice][slab] split-K slice partials (+ sum x^2), written sc1
  unsigned* kticket;     // [tile][m chunk] arrival tickets (zero between launches)
  int ksplit;
  int no_mfma;           // keep the GEMV's per-row arithmetic at any M (folded-table builds)
  int row_chunk;         // gemv_xl_kernel: blockIdx.y takes rows [y*row_chunk, +row_chunk) (table builds)
  // Streaming matrix-core path (gemm_xs.hip; the batched depth decoder): the A operand arrives
  // pre-split (xs.h) instead of as fp32 rows x.  With nw set, the RMSNorm scale of row m is
  // rsqrt(sum_t ss_in[t * ss_stride + m] / K + eps) (ss_n producer partials, summed in order).
  const void* xs_in;
  const float* ss_in;
  int ss_n, ss_stride;
  // Producer side (gemm_xs epilogue, attention, row gathers): the rows this launch produces (EPI_ADD:
  // the new residual, EPI_STORE: the stored rows, EPI_SILU_MUL: silu(gate) * up) are also written
  // split into xs_out (xs_K columns, times xs_nw -- the consuming projection's RMSNorm weight -- when
  // set), with per-row partial sums of squares of the un-normed values in ss_out[tile * ss_stride + m].
  void* xs_out;
  const float* xs_nw;
  float* ss_out;
  int xs_K;
  // int4 consumers: half-group sums of the split rows (xs.h): produced into hs_out, consumed from hs_in
  float* hs_out;
  const float* hs_in;
};

// order-preserving float <-> uint32 keys (radix select of the top-k threshold)
__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
// The sampler's counter-based Gumbel-max (restated in oracle/csm_oracle.py gumbel_u): one key per
// (utterance seed, frame * K + codebook), one uniform per vocabulary entry, perturbed logit in double.
// Shared by sample_kernel and the persistent frame decoder so both pick identical codes.
__device__ __forceinline__ uint64_t gumbel_key(uint64_t seed, int step) {
  return splitmix64(splitmix64(seed) ^ (uint64_t)step);
}
__device__ __forceinline__ double gumbel_noise(uint64_t key, int v) {
  const uint64_t h = splitmix64(key ^ (uint64_t)v);
  const double u = ((double)(h >> 11) + 0.5) * 1.1102230246251565e-16;  // 2^-53
  return -log(-log(u));
}
__device__ __forceinline__ double gumbel_perturbed(float logit, float inv_t, uint64_t key, int v) {
  return (double)(logit * inv_t) + gumbel_noise(key, v);
}

__device__ __forceinline__ unsigned long long pack_argmax(float v, int idx) {
  const uint32_t u = __float_as_uint(v);
  const uint32_t key = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)key << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)idx);
}
__device__ __forceinline__ int unpack_argmax(unsigned long long p) { return (int)(0xFFFFFFFFu - (uint32_t)p); }
// Arg-max over n packed block partials pp[0..n) by one wave: each lane's loads (up to 16 per round)
// are all issued before the first compare -- one memory round trip for a head's ~500 partials --
// then a shuffle max.  Every lane returns the result.
__device__ __forceinline__ unsigned long long wave_argmax_partials(const unsigned long long* pp, int n, int lane) {
  unsigned long long best = 0;
  for (int i0 = 0; i0 < n; i0 += 64 * 16) {
    unsigned long long v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = i0 + lane + 64 * u;
      v[u] = i < n ? pp[i] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) best = v[u] > best ? v[u] : best;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long v = __shfl_xor(best, o, 64);
    best = v > best ? v : best;
  }
  return best;
}

// Pair epilogue shared by every GEMV kernel (rows n, n+1 of output row m).
__device__ __forceinline__ void gemv_epilogue_pair(const GemvParams& p, int m, int n, float a, float b) {
  switch (p.epi) {
    case EPI_STORE: {
      float* o = p.out + (size_t)m * p.os + n;
      o[0] = a;
      o[1] = b;
      break;
    }
    case EPI_GELU: {
      float* o = p.out + (size_t)m * p.os + n;
      o[0] = p.gelu_erf ? gelu_erf_f(a) : gelu_tanh_f(a);
      o[1] = p.gelu_erf ? gelu_erf_f(b) : gelu_tanh_f(b);
      break;
    }
    case EPI_ADD: {
      float* o = p.out + (size_t)m * p.os + n;
      if (p.scale) {
        a *= p.scale[n];
        b *= p.scale[n + 1];
      }
      o[0] += a;
      o[1] += b;
      break;
    }
    case EPI_ARGMAX: {  // logits (c0 / ci heads); the packed block arg-max is reduced by the caller
      float* o = p.out + (size_t)m * p.os + n;
      o[0] = a;
      o[1] = b;
      break;
    }
    case EPI_SILU_MUL:  // rows 2j (gate), 2j+1 (up) -> out[j]  (mlx_lm MLP: down(silu(gate)*up))
      p.out[(size_t)m * p.os + (n >> 1)] = silu_f(a) * b;
      break;
    case EPI_QKV: {
      // rows [q: Hq*hd | k: Hkv*hd | v: Hkv*hd]; RoPE on interleaved pairs (2i, 2i+1)
      // (attention.py:157-177) from the cos/sin table; K/V appended at pos (KVCache.update_and_fetch)
      const int qn = p.Hq * p.hd, kn = p.Hkv * p.hd;
      const int bb = p.rm.b(m), pos = p.rm.pos(m);
      const int nn = n < qn ? n : (n < qn + kn ? n - qn : n - qn - kn);
      const int d = nn % p.hd;
      if (n < qn + kn) {
        const float2 cs = *reinterpret_cast<const float2*>(p.rope + ((size_t)pos * (p.hd >> 1) + (d >> 1)) * 2);
        const float y0 = a * cs.x - b * cs.y, y1 = b * cs.x + a * cs.y;
        a = y0;
        b = y1;
      }
      float* o;
      if (p.qkv_tab) {  // table build: the whole (RoPE'd q, k | v) row of row m
        o = p.qkv_tab + (size_t)m * (qn + 2 * kn) + n;
      } else if (n < qn) {
        o = p.out + (size_t)m * p.os + n;
      } else {
        float* cache = n < qn + kn ? p.kc : p.vc;
        o = cache + (((size_t)bb * p.Hkv + nn / p.hd) * p.S_cap + pos) * p.hd + d;
      }
      *reinterpret_cast<float2*>(o) = make_float2(a, b);
      break;
    }
  }
}

struct EmbedParams {
  const int* tok;        // [M][K+1] prompt tokens (or null)
  const uint8_t* mask;   // [M][K+1]
  const int* codes;      // [M][K] decode-mode codes (or null)
  const void* text_emb;  // [Vt][D]
  const void* audio_emb; // [V*K][D]
  int V, K, D;
  float* out;            // [M][D]
  int* pos_inc;          // decode mode: pos[m] += 1 (position of the new backbone row)
  // streaming backbone (gemm_xs): rows also written split (x * xs_nw, xs.h, K = D) with per-row sums of
  // squares per 512-column block in ss_out[blockIdx.y * ss_stride + m]
  void* xs_out;
  const float* xs_nw;
  float* ss_out;
  int ss_stride;
  float* hs_out;         // int4 consumer: half-group sums of the split rows (xs.h)
};

struct AttnParams {
  const float* q;  // [M][qs] (head h at h*hd)
  int qs, M;
  const float* kc;
  const float* vc;
  int Hq, Hkv, S_cap;
  float scale;
  int mode, window;
  RowMap rm;
  float* out;
  int os;
  // Decoder layer 0 at codebook steps >= 2 (g_tab != null): the step's QKV rows are not computed but
  // gathered -- g_tab[code] = RoPE'd (q, k | v) of layer 0 for decoder input row proj_tab[cb][code]
  // (built at csm_begin by the QKV GEMV itself).  code = arg-max of the head partials g_part; the
  // block writes its kv head's K/V row at pos into the cache, kv head 0's block also writes
  // codes[b][g_cb] and the residual row g_xtab[code] -> g_xout[m].
  const float* g_tab;
  int g_row;  // floats per g_tab row = (Hq + 2 Hkv) * hd
  const unsigned long long* g_part;
  int g_part_stride, g_part_n, g_V;
  int* g_codes;
  int g_codes_K, g_cb;
  const float* g_xtab;
  float* g_xout;
  int g_D;
  // streaming matrix-core path: the attention output also written split (xs.h) for the o_proj GEMM
  // (+ its half-group sums for an int4 o_proj)
  void* xs_out;
  int xs_K;
  float* hs_out;
};

struct SampleParams {
  const float* logits;  // [B][ls]
  int ls, V;            // V = number of valid logits
  float temperature;
  int top_k;
  const uint64_t* seeds;
  const int* frame_ctr;
  int K, cb;
  int* codes;           // [B][K]
  unsigned long long* part;  // optional: publish the code as partial [b * part_stride]
  int part_stride;
  const int* forced;    // optional [B][K]: teacher forcing -- the code is forced[b][cb], logits untouched
  // mlx_lm filter chain beyond top-k (sample_filtered_kernel): top_p keeps entries whose ascending
  // cumulative probability > top_p_cut = float32(1 - top_p); min_p keeps lp >= best + log_min_p
  // (float32(log(min_p))) and the first min_keep ranks
  int use_top_p, use_min_p, min_keep;
  float top_p_cut, log_min_p;
};

struct AdvanceParams {
  int* codes;
  int* hist;      // [F_cap][B][K]
  int F_cap, B, K, V;
  uint8_t* done;
  int* n_frames;
  int* frame_ctr;
  const unsigned long long* last_part;  // greedy: partials of the last head (null: codes already final)
  int last_stride, last_n;
};

void launch_gemv(const GemvParams& p, int wdt, int epi, int norm, hipStream_t st, int tag = 2);
// folded-table builds: rows per call launch_gemv_table takes (same per-row arithmetic as launch_gemv)
int gemv_table_rows(int N, int K, int wdt, int tag);
void launch_gemv_table(const GemvParams& p, int wdt, int epi, int norm, hipStream_t st, int tag);
void launch_embed(const EmbedParams& p, int wdt, int M, hipStream_t st);
// out[i] = stored row idx[i] of a [Ntot][K] matrix (f32 / bf16 / int4) as fp32 (K % 8 == 0)
void launch_table_rows(const void* base, int wdt, int Ntot, int K, const int* idx, int n, float* out, hipStream_t st);
// dst[i] = float(src[i]) for n elements (n % 8 == 0)
void launch_to_f32(const void* src, int wdt, float* dst, size_t n, hipStream_t st);
void launch_attn(const AttnParams& p, int hd, hipStream_t st);
// dense rows -> the streaming GEMM's operand (x * nw), per-512-column sums of squares, half-group sums
void launch_xs_rows(const float* x, int xstride, int M, int K, const float* nw, void* xs_out, float* ss_out, int ss_stride,
                    float* hs_out, hipStream_t st);
// rows per block of the GEMV launch for (N, K, M): N must be a multiple of it
int gemv_rows_per_block(int N, int K, int M);
void launch_rmsnorm_rows(const float* x, int xs, const float* w, float eps, int D, float* out, int os, int M,
                         hipStream_t st);

// down_proj columns re-laid chunk-major [F/R][D][R] for the persistent kernels (dec_frame / bb_step):
// R = wdc_chunk(D) consecutive intermediate columns per chunk (0: no chunk-major copy for this width)
int wdc_chunk(int D);
bool gemv_nt(int tag);                       // non-temporal weight loads for this stack tag
void launch_sample(const SampleParams& p, int wdt, int B, hipStream_t st);
void launch_advance(const AdvanceParams& p, hipStream_t st);
// Teacher-forced cross entropy (mlx cross_entropy, trainer.py:271-312): out[b][cb] =
// logsumexp(logits[:V]) - logits[forced[b][cb]] for c0 rows [B][Vp] and ci rows [K-1][B][Vp].
void launch_forced_ce(const float* c0, const float* ci, const int* forced, float* out, int B, int K, int V, int Vp,
                      hipStream_t st);


// ---- int4 (q4_kernels.hip)
// quantize rows [0, n_rows) of a dense [n_rows][K] f32/bf16 device matrix into rows row0 + r*rstep of a
// quantized matrix with Ntot rows (MLX affine rule; oracle/quant_oracle.py)
void launch_q4_quantize(const void* src, int src_wdt, int n_rows, int K, void* dst, int Ntot, int row0, int rstep,
                        hipStream_t st);
// MLX scales / biases [n_rows][K/64] (f32 or bf16, device) -> sb words of rows row0 + r*rstep
void launch_q4_set_sb(const void* sc, const void* bi, int src_wdt, int n_rows, int K, void* dst, int Ntot, int row0,
                      int rstep, hipStream_t st);
void launch_q4_to_f32(const void* base, int Ntot, int K, int r0, int n, float* dst, hipStream_t st);
void launch_embed_q4(const EmbedParams& p, int n_text_rows, int M, hipStream_t st);
void launch_gemv_q4(const GemvParams& p, bool nt, hipStream_t st);
int gemv_q4_rows_per_block(int N, int K, int M);
bool gemv_q4_supported(int N, int K);
// the persistent kernels' chunk-major copy of an int4 [D][F] down_proj (q4_bytes(D, F) bytes)
void launch_q4_down_cm(const void* src, int D, int F, void* dst, hipStream_t st);

// ---- batched projections on MFMA (gemm_kernels.hip)
constexpr int GEMM_MFMA_MIN_M = 8;  // rows at which a bf16 projection leaves the GEMV for the matrix cores
bool gemm_mfma_eligible(int N, int K, int M, int wdt);
int gemm_tiles(int N, int K, int M, int wdt);  // row-tile blocks of an MFMA launch (= arg-max partials per row)
void launch_gemm_mfma(const GemvParams& p, int wdt, bool nt, hipStream_t st);
// pre-size ws for (N, K) at any row count <= M (outside graph capture); true if it reallocated
bool gemm_reserve(GemmWs& ws, int N, int K, int M);
// Streaming matrix-core GEMM over pre-split activations (gemm_xs.hip): bf16 weights, <= 64 rows
constexpr int GEMM_XS_MAX_M = 64;
bool gemm_xs_eligible(int N, int K, int M, int wdt);
// column tiles of a launch: sums-of-squares partials per row, or (head: an EPI_ARGMAX / SiLU launch) arg-max partials
int gemm_xs_tiles(int N, int K, int M, bool head = false);
void launch_gemm_xs(const GemvParams& p, int epi, hipStream_t st, bool nt = false, int wdt = WDT_BF16);
bool gemm_xs_reserve(GemmWs& ws, int N, int K, int M);
void gemm_xs_stamps_report(const char* tag);  // lab builds (-DXS_STAMPS=1): phase breakdown to stderr
// Fragment-tiled weight copy for the MFMA path: per 32-row tile and 64-K stage, the bytes each lane
// of a wave loads for v_mfma_f32_32x32x16_bf16's B operand, contiguous (bf16: 4 KB = 4 steps x 64
// lanes x 16 B; int4: 1 KB of nibbles, then a [tile][stage][32] block of scale|bias words); rows
// past N are zero.
size_t gemm_tiled_bytes(int N, int K, int wdt);
void launch_gemm_retile(const void* W, void* T, int N, int K, int wdt, hipStream_t st);
void gemm_ws_free(GemmWs& ws);
// dense decoder-input rows from a table (codes resolved from arg-max partials), see gather_rows_kernel
void launch_gather_rows(const GemvParams& p, int wdt, hipStream_t st);
// arg-max partial slots per row written by launch_gemv for this shape / dtype / row count
int gemv_partials(int N, int K, int M, int wdt);

// ---- persistent frame decoder (dec_frame.hip): c0 head + 31 depth-decoder steps of one greedy batch-1
// frame in one launch of 256 x 512 threads (one workgroup per CU), csm_1b decoder shapes, bf16 weights
// Persistent backbone step (bb_step.hip): the 16 backbone blocks of one batch-1 decode row (bf16,
// csm_1b shapes) + the final norm in one launch.
constexpr int BB_STEP_LAYERS = 16, BB_STEP_WGS = 256, BB_STEP_THREADS = 512;
struct BbStepArgs {
  const bf16_t* wqkv[BB_STEP_LAYERS];
  const bf16_t* wo[BB_STEP_LAYERS];
  const bf16_t* wgu[BB_STEP_LAYERS];     // gate/up rows interleaved
  const bf16_t* wdc[BB_STEP_LAYERS];     // down_proj chunk-major [F/8][D][8] (int4: q4_down_cm's copy)
  const float* n1[BB_STEP_LAYERS];
  const float* n2[BB_STEP_LAYERS];
  float* kc[BB_STEP_LAYERS];             // [Hkv][S_cap][HD] of utterance 0
  float* vc[BB_STEP_LAYERS];
  const float* norm;                     // backbone final norm
  const float* rope;                     // [S_cap][HD/2][2]
  int S_cap;
  float eps;
  const float* x;                        // [D] the embedded row
  const int* pos;                        // [1] its position (advanced by the embedding launch)
  float* h_last;                         // [D] norm(h) of the row
  unsigned long long* gbuf;              // hand-off granules (bb_step_gbuf_bytes)
  unsigned* epoch;                       // hand-off tag base
  int* err;                              // raised when a hand-off wait times out
  unsigned long long* stamps;            // optional [NWG][BB_STEP_STAMPS] s_memrealtime per hand-off (profiling)
};
constexpr int BB_STEP_STAMPS = 128;
size_t bb_step_gbuf_bytes();
// q4: the int4 kernel (wqkv / wo / wgu in the common.h int4 layout, wdc the q4_down_cm copy)
void launch_bb_step(const BbStepArgs& p, hipStream_t st, bool q4 = false);
const void* bb_step_kernel_ptr(bool q4 = false);

constexpr int DEC_FRAME_LAYERS = 4;
struct DecFrameArgs {
  const bf16_t* wqkv[DEC_FRAME_LAYERS];
  const bf16_t* wo[DEC_FRAME_LAYERS];
  const bf16_t* wgu[DEC_FRAME_LAYERS];   // gate/up rows interleaved
  const bf16_t* wdc[DEC_FRAME_LAYERS];   // down_proj chunk-major [F/16][D][16]
  const float* n1[DEC_FRAME_LAYERS];
  const float* n2[DEC_FRAME_LAYERS];
  const float* norm;                     // decoder final norm
  const float* rope;                     // [S_cap][HD/2][2]
  float* kc[DEC_FRAME_LAYERS];           // [Hkv][S_cap][HD] of utterance 0
  float* vc[DEC_FRAME_LAYERS];
  int S_cap;
  float eps;
  const bf16_t* c0_head;                 // [VP][2048]
  const bf16_t* proj;                    // [1024][2048]
  const bf16_t* audio_head;              // [K-1][VP][1024]
  const float* proj_tab;                 // [K-1][V][1024]
  const float* qkv0_tab;                 // [K-1][V][1536]
  const float* h_last;                   // [2048]
  int V, VP, K;
  int* codes;                            // [K] of utterance 0
  float* c0_logits;                      // [VP] (debug / parity taps, as the launch path stores them)
  float* ci_logits;                      // [K-1][VP]
  unsigned long long* gbuf;              // hand-off granules (dec_frame_gbuf_bytes)
  unsigned* epoch;                       // hand-off tag base (advanced by every frame)
  int* err;                              // raised when a hand-off wait times out
  unsigned long long* stamps;            // optional [NWG][DEC_FRAME_STAMPS] s_memrealtime per hand-off (profiling)
  int wnt, hnt;                          // non-temporal loads for the decoder weights / the heads
  // sampling (temperature > 0): every head's logits are handed to every workgroup, which picks the
  // code by the sampler's top-k threshold + Gumbel-max (gumbel_perturbed) redundantly
  float temperature;
  int top_k;
  const uint64_t* seeds;                 // [1] utterance 0's sampling seed
  const int* frame_ctr;                  // frame index (the sampler's counter)
};
constexpr int DEC_FRAME_STAMPS = 1024;
size_t dec_frame_gbuf_bytes();
constexpr int DEC_FRAME_WGS = 256, DEC_FRAME_THREADS = 512;
// q4: the int4 kernel (wqkv / wo / wgu / c0_head / proj in the common.h int4 layout, wdc the q4_down_cm copy;
// audio_head bf16)
void launch_dec_frame(const DecFrameArgs& p, hipStream_t st, bool q4 = false);
const void* dec_frame_kernel_ptr(bool q4 = false);  // for the occupancy query

// Persistent batched depth-decoder step (dec_step_xs.hip): the 4 decoder layers (+ the head) of codebook
// step `step` >= 2 for rows (utterances) 0..M-1 in one launch: M <= 32 with bf16 weights, M <= 64 int4.
constexpr int DEC_XSD_WGS = 256, DEC_XSD_THREADS = 512, DEC_XSD_MAX_M = 32, DEC_XSD_MAX_M_Q4 = 64;
struct DecStepXsArgs {
  const uint8_t* wqkv[DEC_FRAME_LAYERS];  // fragment-tiled bf16 copies (gemm_retile)
  const uint8_t* wo[DEC_FRAME_LAYERS];
  const uint8_t* wgu[DEC_FRAME_LAYERS];
  const uint8_t* wd[DEC_FRAME_LAYERS];
  const float* n1[DEC_FRAME_LAYERS];
  const float* n2[DEC_FRAME_LAYERS];
  const float* norm;                      // decoder final norm
  const float* rope;                      // [S_cap][HD/2][2]
  float* kc[DEC_FRAME_LAYERS];            // [B][Hkv][S_cap][HD]
  float* vc[DEC_FRAME_LAYERS];
  int S_cap;
  float eps;
  int M, step;                            // rows; codebook step (= the rows' position)
  const unsigned long long* part;         // the previous head's arg-max partials [B][part_stride]
  int part_stride, part_n, V;
  const float* qkv0_tab;                  // this step's folded tables: [V][1536] RoPE'd layer-0 q | k | v
  const float* proj_tab;                  // [V][1024] projection(E_a[c])
  int* codes;                             // [B][codes_K]: codes[m][step - 1] written
  int codes_K;
  // scratch (dec_step_xs_scratch_bytes) and outputs
  float* qkv;                             // [64][1536]
  void* xs_att;                           // split rows (xs.h), K = 1024
  void* xs_x;                             // K = 1024
  void* xs_h;                             // K = 8192
  void* xs_out;                           // K = 1024: x * (next n1 | final norm) -- the head's xs_in
  float* ss_out;                          // [32 tiles][ss_stride] sums of squares -- the head's ss_in
  int ss_stride;
  float* x_o;                             // [64][1024]
  float* x_d;                             // [64][1024]
  float* ss_o;                            // [32 tiles][64]
  float* dpart;                           // [8][64][1024]
  int* code_buf;                          // [64]
  // int4 consumers: half-group sums [k / 32][64] of the split rows (xs.h) -- attention out, x_o * n2, h,
  // and of xs_out (the engine's hs_D)
  float* hs_att;
  float* hs_x;
  float* hs_h;
  float* hs_out;
  unsigned* ctrl;                         // hand-off flags / counters (dec_step_xs_ctrl_bytes, zeroed once)
  unsigned* epoch;                        // advanced by every launch
  int* err;                               // raised when a hand-off wait times out
  unsigned long long* stamps;             // optional [NWG][DEC_XSD_STAMPS] s_memrealtime marks (profiling)
  // the step's head in the same launch (head_w null: a launch of its own after this one):
  // audio_head[step - 1]'s fragment-tiled copy (head_nt32 32-row tiles of the Vp padded rows), logits ->
  // head_out [M][Vp], one arg-max partial per 64-row tile (head_tiles of them) -> head_part[m][part_stride]
  const uint8_t* head_w;
  int head_nt32, head_tiles, Vp, n_valid;
  float* head_out;
  unsigned long long* head_part;
  // sampled steps (temperature > 0, top-k only; needs the head in the launch): workgroup m < M samples
  // row m from the head's logits as sample_kernel does (radix-select top-k threshold, Gumbel-max with
  // the counter key(seeds[m], frame_ctr[0] * K + cb)) -> codes[m][cb] and the single partial head_part[m][0]
  int sample, s_top_k, s_K, s_cb;
  float s_temperature;
  const uint64_t* s_seeds;
  const int* s_frame_ctr;
  float* qkvp;                            // bf16 XSD_QSPLIT: [2][RMAX][QKV] the QKV K halves' partial sums, then [48][RMAX] row scales
};
constexpr int DEC_XSD_STAMPS = 64;
constexpr int DEC_XSD_SAMPLE_NPT = 5;  // logits per thread of the in-launch sampler: V <= 512 x 5
size_t dec_step_xs_ctrl_bytes();
void launch_dec_step_xs(const DecStepXsArgs& p, hipStream_t st, bool q4);
const void* dec_step_xs_kernel_ptr(bool q4);
