// Kernel parameter blocks and launchers shared by the CSM engine and the Mimi codec.
#pragma once
#include "common.h"

enum { WDT_F32 = 0, WDT_BF16 = 1 };
enum { EPI_STORE = 0, EPI_ADD = 1, EPI_SILU_MUL = 2, EPI_QKV = 3, EPI_GELU = 4 };
enum { ATTN_CAUSAL = 0, ATTN_WINDOW = 1, ATTN_BLOCK = 2 };

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
};

struct EmbedParams {
  const int* tok;        // [M][K+1] prompt tokens (or null)
  const uint8_t* mask;   // [M][K+1]
  const int* codes;      // [M][K] decode-mode codes (or null)
  const void* text_emb;  // [Vt][D]
  const void* audio_emb; // [V*K][D]
  int V, K, D;
  float* out;            // [M][D]
  int* pos_inc;          // decode mode: pos[m] += 1 (position of the new backbone row)
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
  // fused next-input gather (null next_in = skip)
  float* next_in;
  const float* h_last;  // [B][D] (cb == 0: decoder step-1 rows are [h_last, E_a[c0]])
  const void* audio_emb;
  int V_emb, D;
};

struct AdvanceParams {
  const int* codes;
  int* hist;      // [F_cap][B][K]
  int F_cap, B, K;
  uint8_t* done;
  int* n_frames;
  int* frame_ctr;
};

void launch_gemv(const GemvParams& p, int wdt, int epi, int norm, hipStream_t st, int tag = 2);
void launch_embed(const EmbedParams& p, int wdt, int M, hipStream_t st);
void launch_attn(const AttnParams& p, int hd, hipStream_t st);
// rows per block of the GEMV launch for (N, K, M): N must be a multiple of it
int gemv_rows_per_block(int N, int K, int M);
void gemv_set_override(int G, int RPT);  // 0 = automatic
// fused attention (<= 64 keys, M <= 4 rows) + o_proj + residual for the depth decoder
void launch_attn_oproj(const GemvParams& p, const AttnParams& a, int wdt, int hd, hipStream_t st);
void launch_rmsnorm_rows(const float* x, int xs, const float* w, float eps, int D, float* out, int os, int M,
                         hipStream_t st);
void launch_sample(const SampleParams& p, int wdt, int B, hipStream_t st);
void launch_advance(const AdvanceParams& p, hipStream_t st);
