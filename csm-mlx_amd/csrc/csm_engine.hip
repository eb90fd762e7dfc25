// CSM engine: device-resident weights, KV caches and the graph-captured frame loop behind
// the C ABI of include/csm_hip.h.
//
// One frame (generation.py:21-92) is two captured HIP graphs replayed back to back:
//   body : embed(previous codes) -> 16 backbone layers (M = B rows) -> final RMSNorm -> h_last
//   head : c0 head -> sample c0 (+ gather decoder rows) -> 31 x [projection -> 4 decoder layers
//          -> ci head -> sample ci (+ gather next row)] -> advance (history, EOS, frame counter)
// All per-frame state (positions, codes, frame counter) lives in device memory so the same
// graphs replay every frame without host involvement; the host only polls EOS flags.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <memory>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/csm_hip.h"
#include "../../include/csm_hip_prof.h"
#include "csm_kernels.h"
#include "engine_util.h"
#include "xs.h"

namespace {

struct LayerW {
  void* wqkv = nullptr;  // [(Hq+2Hkv)*hd][D]
  void* wo = nullptr;    // [D][Hq*hd]
  void* wgu = nullptr;   // [2F][D] rows interleaved gate_j, up_j
  void* wd = nullptr;    // [D][F]
  void* wdc = nullptr;   // bf16 engines: down_proj re-laid chunk-major [F/R][D][R] for the fused MLP
  void* wdq = nullptr;   // int4 engines: the persistent kernels' chunk-major down copy (q4_down_cm), derived:
                         // rebuilt by build_tiled after any weight change, not a weight buffer
  float* n1 = nullptr;
  float* n2 = nullptr;
  float* kc = nullptr;   // [B][Hkv][S][hd]
  float* vc = nullptr;
};

struct Stack {
  csm_llama_dims d;
  std::vector<LayerW> L;
  float* norm = nullptr;
  float* rope = nullptr;  // [S][hd/2][2]
  int S_cap = 0;
  int qkv_rows() const { return (d.n_heads + 2 * d.n_kv_heads) * d.head_dim; }
  int q_dim() const { return d.n_heads * d.head_dim; }
};

}  // namespace

struct csm_engine {
  csm_dims dims;
  int dev = 0;
  int wdt = WDT_BF16;       // Linear / Embedding weights: WDT_F32, WDT_BF16 or WDT_Q4 (nn.quantize'd)
  int head_wdt = WDT_BF16;  // audio_head: never quantized (a raw array, models.py:65-67)
  size_t wsz = 2;           // bytes per element of the dense (non-q4) weight dtype
  // bytes of one [N][K] Linear/Embedding weight in the engine's storage dtype
  size_t wbytes(size_t N, size_t K) const { return wdt == WDT_Q4 ? q4_bytes(N, K) : N * K * wsz; }
  // pre-quantized MLX tensors wait here until .weight, .scales and .biases have all arrived
  struct PendingQ4 {
    std::vector<uint8_t> packed, scales, biases;
    int sdt = 0;
    int64_t n = 0, k = 0;
  };
  std::map<std::string, PendingQ4> pending_q4;
  int B_max = 0, F_cap = 0, M_cap = 0;
  hipStream_t st = nullptr;
  Stack bb, dec;
  int V = 0, Vpad = 0, K = 0, D = 0, Dd = 0;
  void* text_emb = nullptr;
  void* audio_emb = nullptr;
  void* proj = nullptr;      // [Dd][D]
  void* c0_head = nullptr;   // [Vpad][D]
  void* audio_head = nullptr;  // [K-1][Vpad][Dd]
  // projection folded into the decoder-input table: proj_tab[cb][code] = projection(E_a[code + V*cb])
  // (fp32, the exact output of the projection GEMV), cb < K-1.  Decoder steps >= 2 gather their
  // input row from it instead of running the projection GEMV.
  float* proj_tab = nullptr;
  bool proj_tab_dirty = true;
  bool c0_pending = false;  // csm_frame_c0_logits ran; csm_frame_finish (or csm_frame_host_step) must follow
  int host_piece = 1;       // csm_frame_host_step: the codebook whose code the next call feeds is host_piece - 1
  // decoder layer 0's QKV folded too: qkv0_tab[cb][code] = RoPE'd (q, k | v) of layer 0 for input row
  // proj_tab[cb][code] at position cb + 1 (fp32, built by the same QKV GEMV); codebook steps >= 2 then
  // skip layer 0's QKV launch and its attention gathers the row (AttnParams::g_tab).
  float* qkv0_tab = nullptr;
  bool use_qkv0_tab = [] { const char* v = getenv("CSM_QKV0_TAB"); return !(v && v[0] == '0'); }();  // csm_set_option "qkv0_tab"
  bool qkv0_built = false;
  // fragment-tiled copies of the matrices the MFMA path reads (build_tiled; ws.tiled maps them)
  std::vector<void*> tiled_bufs;
  bool tiled_dirty = true;
  std::set<std::string> loaded;
  std::vector<std::string> required;
  // activations
  float *x = nullptr, *q = nullptr, *att = nullptr, *mlp = nullptr;
  float *h_last = nullptr, *c0_logits = nullptr, *ci_logits = nullptr;
  int* force = nullptr;  // [B_max][K] teacher-forced codes (csm_frame_forced)
  float* force_ce = nullptr;  // [B_max][K] their cross entropies
  float *dx = nullptr, *din = nullptr, *dq = nullptr, *datt = nullptr, *dmlp = nullptr;
  int32_t* tok = nullptr;
  uint8_t* msk = nullptr;
  int *row_b = nullptr, *row_pos = nullptr;  // [M_cap] batched-prefill row tables
  int2* ptiles = nullptr;  // [M_cap / 64 + B_max + 2] prompt-prefill attention tiles (RowMap::tiles)
  // csm_run_frames_ahead: each chunk's done flags and the persistent kernels' error flags are copied to
  // pinned host memory behind its frames, with an event; a call waits for the previous chunk's only
  uint8_t* ahead_pin = nullptr;  // [2][ahead_bytes()]
  int2* ptiles_pin = nullptr;     // pinned staging of a single prompt's attention tiles (csm_prefill)
  hipEvent_t ahead_ev[2] = {nullptr, nullptr};
  int ahead_slot = 0;
  bool ahead_pending = false;
  size_t ahead_bytes() const { return (size_t)(B_max + 7) / 8 * 8 + 8; }
  bool attn_tiles_on = true;  // csm_set_option "attn_prefill": 0 = attn_block per row (A/B, tests)
  // per-batch state
  int *codes = nullptr, *hist = nullptr, *pos = nullptr, *n_frames = nullptr, *frame_ctr = nullptr;
  unsigned long long* part = nullptr;  // [K][B_max][part_stride] arg-max partials of the heads
  int part_stride = 0;
  uint8_t* done = nullptr;
  uint64_t* seeds = nullptr;
  int B = 0;
  float temperature = 0.f;
  int top_k = 0;
  // mlx_lm filter chain beyond top-k (csm_set_sampler_filters; reset by csm_begin)
  int use_top_p = 0, use_min_p = 0, min_keep = 1;
  float top_p_cut = 0.f, log_min_p = 0.f;
  int filters_id = 0, g_filters = -1;  // graphs capture the filter parameters by value
  int frames_run = 0;
  bool need_body = false;
  std::vector<int> prompt_len;
  // graphs
  hipGraphExec_t g_body = nullptr, g_head = nullptr;
  int g_B = -1;
  float g_temp = -1.f;
  int g_topk = -1;
  std::vector<void*> allocs;
  std::vector<void*> batch_allocs;
  std::vector<int> pos_host;
  bool fold_proj = true;  // csm_set_option "fold_proj": decoder steps >= 2 read the folded table
  bool linear_mfma = false;  // csm_set_option "linear_mfma": csm_linear on the MFMA GEMM (kernel tests)
  // csm_set_option "prefill_rows": row cap of one csm_prefill_batch group (0 = M_cap); lowering it makes
  // small test batches take the multi-group path that config 5's 64 x 248-row contexts take
  int prefill_rows = 0;
  // csm_set_option "qkv0_tab_batched" 0: batched (matrix-core) frames run layer 0's QKV projection
  // instead of gathering it from the folded table (A/B and parity checks)
  bool no_tab_batched = false;
  // batched depth decoder (8..64 utterances, bf16 or int4, codebook steps >= 2) on the streaming
  // matrix-core GEMM over pre-split activations (gemm_xs.hip): split rows x * norm [64][Dd], attention
  // output, SiLU*up rows [64][F] (xs.h layout), per-row partial sums of squares [64 tiles][64 rows],
  // half-group sums for int4.  Config 4 3917 vs 3729 frames/s on gemm_wide (r03).
  // csm_set_option "gemm_xs" / CSM_GEMM_XS=0 turn it off.
  bool xs_on = [] { const char* v = getenv("CSM_GEMM_XS"); return !(v && v[0] == '0'); }();
  // the depth decoder's step 1 (2 rows per utterance) on the streaming GEMM as well (CSM_XS_STEP1=0: on
  // gemm_wide, the A/B)
  bool xs_step1 = [] { const char* v = getenv("CSM_XS_STEP1"); return !(v && v[0] == '0'); }();
  void *xs_D = nullptr, *xs_A = nullptr, *xs_F = nullptr;
  float* xs_ss = nullptr;
  // the batched backbone on the streaming GEMM too (option bb_xs / CSM_BB_XS=0 off): with 8-wave blocks it
  // beats gemm_wide on every backbone shape -- int4 at 64 rows gate/up 40.4 -> 22.7, down 28.2 -> 18.9,
  // QKV 24.8 -> 18.3, o 15.8 -> 11.4 us; bf16 at 32 rows 63 -> 58 us per layer (profiles/r04_ab_xs_waves8.txt)
  bool bb_xs_on = [] { const char* v = getenv("CSM_BB_XS"); return !(v && v[0] == '0'); }();
  float *hs_D = nullptr, *hs_A = nullptr, *hs_F = nullptr;  // int4 engines: half-group sums of the split rows
  GemmWs ws;         // split-K slabs + tickets of this engine's MFMA launches (ensure_batch sizes them)
  // persistent frame decoder (dec_frame.hip) for batch-1 greedy bf16 frames: hand-off granules, tag
  // epoch, timeout flag; csm_set_option "dec_frame" / CSM_DEC_FRAME=0 turn it off
  void* df_gbuf = nullptr;
  unsigned* df_epoch = nullptr;
  int* df_err = nullptr;
  bool dec_frame = [] { const char* v = getenv("CSM_DEC_FRAME"); return !(v && v[0] == '0'); }();
  int df_hw = -1;    // 1: the device can hold one 512-thread workgroup on each of 256 CUs at once
  unsigned long long* df_stamps = nullptr;  // csm_set_option "dec_frame_stamps": per-hand-off clock stamps
  // persistent backbone step (bb_step.hip) for batch-1 bf16 csm_1b decode rows; csm_set_option
  // "bb_step" / CSM_BB_STEP=0 turn it off
  void* bb_gbuf = nullptr;
  unsigned* bb_epoch = nullptr;
  int* bb_err = nullptr;
  bool bb_step = [] { const char* v = getenv("CSM_BB_STEP"); return !(v && v[0] == '0'); }();
  int bb_hw = -1, bb_hw_q4 = -1;
  int df_hw_q4 = -1;
  unsigned long long* bb_stamps = nullptr;  // csm_set_option "bb_step_stamps": per-hand-off clock stamps
  // persistent batched depth-decoder step (dec_step_xs.hip): codebook steps >= 2 of 1..32 bf16 rows in one
  // launch instead of run_dec_xs's ~20; csm_set_option "dec_xsd" / CSM_DEC_XSD=0 turn it off
  bool xsd_on = [] { const char* v = getenv("CSM_DEC_XSD"); return !(v && v[0] == '0'); }();
  int xsd_hw = -1, xsd_hw_q4 = -1;
  DecStepXsArgs xsd{};    // scratch pointers (ensure_batch) + control words
  unsigned* xsd_ctrl = nullptr;
  unsigned* xsd_epoch = nullptr;
  int* xsd_err = nullptr;
  unsigned long long* xsd_stamps = nullptr;  // csm_set_option "dec_xsd_stamps": per-role clock marks of the last launch
  bool xsd_head = [] { const char* v = getenv("CSM_DEC_XSD_HEAD"); return !(v && v[0] == '0'); }();  // "dec_xsd_head": the head in the same launch
  bool xsd_sample = [] { const char* v = getenv("CSM_DEC_XSD_SAMPLE"); return !(v && v[0] == '0'); }();  // "dec_xsd_sample": + the sampler
  bool xsd_sampled = false;  // the last launch_xsd sampled in the launch

  void* balloc(size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) throw CsmError(CSM_ERR_HIP, "hipMalloc(" + std::to_string(bytes) + ") failed");
    (void)hipMemset(p, 0, bytes);
    (void)hipDeviceSynchronize();  // the null-stream fill is not ordered with the engine's non-blocking stream
    batch_allocs.push_back(p);
    return p;
  }
  void* alloc(size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) throw CsmError(CSM_ERR_HIP, "hipMalloc(" + std::to_string(bytes) + ") failed");
    (void)hipMemset(p, 0, bytes);
    (void)hipDeviceSynchronize();  // the null-stream fill is not ordered with the engine's non-blocking stream
    allocs.push_back(p);
    return p;
  }
  void release(void* p) {
    for (auto& a : allocs)
      if (a == p) {
        (void)hipFree(p);
        a = allocs.back();
        allocs.pop_back();
        return;
      }
  }
  ~csm_engine() {
    for (hipEvent_t ev : ahead_ev)
      if (ev) (void)hipEventDestroy(ev);
    if (ahead_pin) (void)hipHostFree(ahead_pin);
    if (ptiles_pin) (void)hipHostFree(ptiles_pin);
    if (g_body) (void)hipGraphExecDestroy(g_body);
    if (g_head) (void)hipGraphExecDestroy(g_head);
    for (void* p : allocs) (void)hipFree(p);
    for (void* p : batch_allocs) (void)hipFree(p);
    gemm_ws_free(ws);
    if (st) (void)hipStreamDestroy(st);
  }
};

// ---------------------------------------------------------------------------------------------
namespace {

// GEMV / GEMM parameters bound to this engine's split-K scratch
GemvParams gp(csm_engine* e) {
  GemvParams g{};
  g.ws = &e->ws;
  return g;
}

void alloc_stack(csm_engine* e, Stack& s, const csm_llama_dims& d, int S_cap, const char* prefix) {
  s.d = d;
  s.S_cap = S_cap;
  s.L.resize(d.n_layers);
  const size_t D = d.hidden, F = d.intermediate, hd = d.head_dim;
  for (int i = 0; i < d.n_layers; ++i) {
    LayerW& l = s.L[i];
    l.wqkv = e->alloc(e->wbytes(s.qkv_rows(), D));
    l.wo = e->alloc(e->wbytes(D, s.q_dim()));
    l.wgu = e->alloc(e->wbytes(2 * F, D));
    l.wd = e->alloc(e->wbytes(D, F));
    if (e->wdt == WDT_BF16 && wdc_chunk((int)D) && F % wdc_chunk((int)D) == 0) l.wdc = e->alloc(D * F * 2);
    l.n1 = (float*)e->alloc(D * 4);
    l.n2 = (float*)e->alloc(D * 4);
    const std::string p = std::string(prefix) + ".layers." + std::to_string(i);
    for (const char* n : {".self_attn.q_proj.weight", ".self_attn.k_proj.weight", ".self_attn.v_proj.weight",
                          ".self_attn.o_proj.weight", ".mlp.gate_proj.weight", ".mlp.up_proj.weight",
                          ".mlp.down_proj.weight", ".input_layernorm.weight", ".post_attention_layernorm.weight"})
      e->required.push_back(p + n);
  }
  s.norm = (float*)e->alloc(D * 4);
  s.rope = (float*)e->alloc((size_t)S_cap * hd * 4);
  e->required.push_back(std::string(prefix) + ".norm.weight");
}

// Debug-only timing ablation (CSM_ABLATE bit mask, read at graph capture): skips kernels so their
// in-graph cost can be measured as a frame-time delta.  Results are garbage when set.
int ablate() {
  static int m = -1;
  if (m < 0) {
    const char* v = getenv("CSM_ABLATE");
    m = v ? atoi(v) : 0;
  }
  return m;
}

// One Llama block stack over M rows of the residual stream x (in place).
// gather0: x-gather fields for layer 0's QKV GEMV (its input rows come from a table; the GEMV also
// writes them to x as the residual stream).
void run_stack(csm_engine* e, Stack& s, float* x, int M, float* q, float* att, float* mlp, const RowMap& rm,
                     hipStream_t st, const GemvParams* gather0 = nullptr, const AttnParams* attn0 = nullptr) {
  const csm_llama_dims& d = s.d;
  const int tag = (&s == &e->dec) ? 1 : 0;
  const int D = d.hidden, F = d.intermediate, hd = d.head_dim, Hq = d.n_heads, Hkv = d.n_kv_heads;
  const int ab = tag ? ablate() : (ablate() >> 8) & 31;  // bits 0-4 decoder, 8-12 backbone
  for (int i = 0; i < d.n_layers; ++i) {
    LayerW& l = s.L[i];
    GemvParams g = gp(e);
    // norm1 + QKV + RoPE + KV append
    g.W = l.wqkv; g.N = s.qkv_rows(); g.K = D; g.x = x; g.xs = D; g.M = M; g.nw = l.n1; g.eps = d.eps;
    g.out = q; g.os = s.q_dim(); g.Hq = Hq; g.Hkv = Hkv; g.hd = hd; g.S_cap = s.S_cap; g.rope = s.rope;
    g.kc = l.kc; g.vc = l.vc; g.rm = rm;
    if (i == 0 && gather0) {
      g.xpart = gather0->xpart; g.xpart_stride = gather0->xpart_stride; g.xpart_n = gather0->xpart_n;
      g.xtab = gather0->xtab; g.xtab_f32 = gather0->xtab_f32; g.xV = gather0->xV; g.xcb = gather0->xcb;
      g.x_codes = gather0->x_codes; g.x_codes_K = gather0->x_codes_K; g.x_copy = x;
    }
    const bool gathered = (i == 0 && attn0);  // layer 0 QKV from the folded table (attention gathers it)
    if (!(ab & 2) && !gathered) launch_gemv(g, e->wdt, EPI_QKV, 1, st, tag);
    // attention, then o_proj + residual
    AttnParams a = gathered ? *attn0 : AttnParams{};
    a.q = q; a.qs = s.q_dim(); a.M = M; a.kc = l.kc; a.vc = l.vc; a.Hq = Hq; a.Hkv = Hkv; a.S_cap = s.S_cap;
    a.scale = 1.0f / sqrtf((float)hd); a.mode = ATTN_CAUSAL; a.window = 0; a.rm = rm; a.out = att;
    a.os = s.q_dim();
    g = gp(e);
    g.W = l.wo; g.N = D; g.K = s.q_dim(); g.x = att; g.xs = s.q_dim(); g.M = M; g.out = x; g.os = D;
    if (!(ab & 1)) launch_attn(a, hd, st);
    if (!(ab & 4)) launch_gemv(g, e->wdt, EPI_ADD, 0, st, tag);
    // norm2 + gate/up + SiLU*up
    g = gp(e);
    g.W = l.wgu; g.N = 2 * F; g.K = D; g.x = x; g.xs = D; g.M = M; g.nw = l.n2; g.eps = d.eps; g.out = mlp;
    g.os = F;
    if (!(ab & 8)) launch_gemv(g, e->wdt, EPI_SILU_MUL, 1, st, tag);
    // down + residual
    g = gp(e);
    g.W = l.wd; g.N = D; g.K = F; g.x = mlp; g.xs = F; g.M = M; g.out = x; g.os = D;
    if (!(ab & 16)) launch_gemv(g, e->wdt, EPI_ADD, 0, st, tag);
  }
}

// The batched depth decoder at codebook steps >= 2 (generation.py:72-89 at batch M) on the streaming
// matrix-core GEMM (gemm_xs.hip): layer 0's q | k | v and input row come from the folded tables (attn0),
// and every projection's epilogue writes the split activations of the next one (xs.h) -- o_proj:
// the new residual x * n2 (+ per-row sums of squares), gate/up: SiLU*up, down: the new residual x *
// (next layer's n1, or the final norm for the head) -- so no launch re-normalises or re-splits rows.
int head_blocks(int N, int K, int M, int wdt);

bool dec_xs_eligible(csm_engine* e, int M) {
  const Stack& s = e->dec;
  const int Dd = s.d.hidden, F = s.d.intermediate;
  return e->xs_on && e->xs_D && M >= GEMM_MFMA_MIN_M && M <= GEMM_XS_MAX_M && (e->wdt == WDT_BF16 || e->wdt == WDT_Q4) &&
         e->head_wdt == WDT_BF16 && s.d.head_dim == 128 && s.S_cap <= 32 &&
         gemm_xs_eligible(s.qkv_rows(), Dd, M, e->wdt) && gemm_xs_eligible(Dd, s.q_dim(), M, e->wdt) &&
         gemm_xs_eligible(2 * F, Dd, M, e->wdt) && gemm_xs_eligible(Dd, F, M, e->wdt) &&
         gemm_xs_eligible(e->Vpad, Dd, M, e->head_wdt) &&
         // the next step's row gather reads head_blocks() arg-max partials per row: the streaming head
         // must write exactly that many (one per 64-row tile)
         gemm_xs_tiles(e->Vpad, Dd, M, true) == head_blocks(e->Vpad, Dd, M, e->head_wdt) && gemm_xs_tiles(Dd, F, M) <= 64 &&
         gemm_xs_tiles(Dd, s.q_dim(), M) <= 64;
}

// l0_qkv: layer 0 also projects its q | k | v from split rows (step 1, whose rows launch_xs_rows split
// after the projection) instead of gathering them from the folded table (attn0).
void run_dec_xs(csm_engine* e, int M, const RowMap& rm, hipStream_t st, const AttnParams& attn0, bool l0_qkv = false) {
  Stack& s = e->dec;
  const csm_llama_dims& d = s.d;
  const int D = d.hidden, F = d.intermediate;
  const int ss_o = gemm_xs_tiles(D, s.q_dim(), M), ss_d = gemm_xs_tiles(D, F, M);
  const bool q4 = e->wdt == WDT_Q4;  // int4 consumers also read the half-group sums of their operand
  float* hsD = q4 ? e->hs_D : nullptr;
  float* hsA = q4 ? e->hs_A : nullptr;
  float* hsF = q4 ? e->hs_F : nullptr;
  for (int i = 0; i < d.n_layers; ++i) {
    LayerW& l = s.L[i];
    if (i > 0 || l0_qkv) {  // norm1 + QKV + RoPE + KV append from the split rows the previous down wrote
      GemvParams g = gp(e);
      g.W = l.wqkv; g.N = s.qkv_rows(); g.K = D; g.M = M; g.nw = l.n1; g.eps = d.eps;
      g.out = e->dq; g.os = s.q_dim(); g.Hq = d.n_heads; g.Hkv = d.n_kv_heads; g.hd = d.head_dim;
      g.S_cap = s.S_cap; g.rope = s.rope; g.kc = l.kc; g.vc = l.vc; g.rm = rm;
      g.xs_in = e->xs_D; g.ss_in = e->xs_ss; g.ss_n = i == 0 ? (D + 511) / 512 : ss_d; g.ss_stride = GEMM_XS_MAX_M; g.hs_in = hsD;
      launch_gemm_xs(g, EPI_QKV, st, false, e->wdt);
    }
    AttnParams a = i == 0 ? attn0 : AttnParams{};
    a.q = e->dq; a.qs = s.q_dim(); a.M = M; a.kc = l.kc; a.vc = l.vc; a.Hq = d.n_heads; a.Hkv = d.n_kv_heads;
    a.S_cap = s.S_cap; a.scale = 1.0f / sqrtf((float)d.head_dim); a.mode = ATTN_CAUSAL; a.window = 0; a.rm = rm;
    a.out = e->datt; a.os = s.q_dim(); a.xs_out = e->xs_A; a.xs_K = s.q_dim(); a.hs_out = hsA;
    launch_attn(a, d.head_dim, st);
    {  // o_proj + residual -> x; split (x * n2) + sums of squares for gate/up
      GemvParams g = gp(e);
      g.W = l.wo; g.N = D; g.K = s.q_dim(); g.M = M; g.out = e->dx; g.os = D; g.xs_in = e->xs_A;
      g.xs_out = e->xs_D; g.xs_nw = l.n2; g.ss_out = e->xs_ss; g.ss_stride = GEMM_XS_MAX_M; g.xs_K = D;
      g.hs_in = hsA; g.hs_out = hsD;
      launch_gemm_xs(g, EPI_ADD, st, false, e->wdt);
    }
    {  // norm2 + gate/up + SiLU*up -> split h
      GemvParams g = gp(e);
      g.W = l.wgu; g.N = 2 * F; g.K = D; g.M = M; g.nw = l.n2; g.eps = d.eps; g.out = nullptr; g.os = F;
      g.xs_in = e->xs_D; g.ss_in = e->xs_ss; g.ss_n = ss_o; g.ss_stride = GEMM_XS_MAX_M;
      g.xs_out = e->xs_F; g.xs_K = F; g.hs_in = hsD; g.hs_out = hsF;
      launch_gemm_xs(g, EPI_SILU_MUL, st, false, e->wdt);
    }
    {  // down + residual -> x; split (x * next norm) + sums of squares
      GemvParams g = gp(e);
      g.W = l.wd; g.N = D; g.K = F; g.M = M; g.out = e->dx; g.os = D; g.xs_in = e->xs_F;
      g.xs_out = e->xs_D; g.xs_nw = i + 1 < d.n_layers ? s.L[i + 1].n1 : s.norm; g.ss_out = e->xs_ss;
      g.ss_stride = GEMM_XS_MAX_M; g.xs_K = D; g.hs_in = hsF; g.hs_out = hsD;
      launch_gemm_xs(g, EPI_ADD, st, false, e->wdt);
    }
  }
}

// The batched backbone step (generation.py:39 at batch M, one decode row per utterance) on the same
// streaming path: the embedding gather writes split rows (x * n1[0]) + per-512-column sums of squares,
// then every projection's epilogue (and the attention) writes the next projection's operand.
bool bb_xs_eligible(csm_engine* e, int M) {
  const Stack& s = e->bb;
  const int D = s.d.hidden, F = s.d.intermediate;
  return e->xs_on && e->xs_D && M >= GEMM_MFMA_MIN_M && M <= GEMM_XS_MAX_M && (e->wdt == WDT_BF16 || e->wdt == WDT_Q4) &&
         D % 512 == 0 && D / 512 <= 64 && gemm_xs_eligible(s.qkv_rows(), D, M, e->wdt) &&
         gemm_xs_eligible(D, s.q_dim(), M, e->wdt) && gemm_xs_eligible(2 * F, D, M, e->wdt) &&
         gemm_xs_eligible(D, F, M, e->wdt) && gemm_xs_tiles(D, F, M) <= 64 && gemm_xs_tiles(D, s.q_dim(), M) <= 64;
}

void run_bb_xs(csm_engine* e, int M, const RowMap& rm, hipStream_t st) {
  Stack& s = e->bb;
  const csm_llama_dims& d = s.d;
  const int D = d.hidden, F = d.intermediate;
  const int ss_o = gemm_xs_tiles(D, s.q_dim(), M), ss_d = gemm_xs_tiles(D, F, M);
  const bool q4 = e->wdt == WDT_Q4;  // int4 consumers also read the half-group sums of their operand
  float* hsD = q4 ? e->hs_D : nullptr;
  float* hsA = q4 ? e->hs_A : nullptr;
  float* hsF = q4 ? e->hs_F : nullptr;
  for (int i = 0; i < d.n_layers; ++i) {
    LayerW& l = s.L[i];
    {  // norm1 + QKV + RoPE + KV append
      GemvParams g = gp(e);
      g.W = l.wqkv; g.N = s.qkv_rows(); g.K = D; g.M = M; g.nw = l.n1; g.eps = d.eps;
      g.out = e->q; g.os = s.q_dim(); g.Hq = d.n_heads; g.Hkv = d.n_kv_heads; g.hd = d.head_dim;
      g.S_cap = s.S_cap; g.rope = s.rope; g.kc = l.kc; g.vc = l.vc; g.rm = rm;
      g.xs_in = e->xs_D; g.ss_in = e->xs_ss; g.ss_n = i == 0 ? D / 512 : ss_d; g.ss_stride = GEMM_XS_MAX_M;
      g.hs_in = hsD;
      launch_gemm_xs(g, EPI_QKV, st, gemv_nt(0), e->wdt);
    }
    AttnParams a{};
    a.q = e->q; a.qs = s.q_dim(); a.M = M; a.kc = l.kc; a.vc = l.vc; a.Hq = d.n_heads; a.Hkv = d.n_kv_heads;
    a.S_cap = s.S_cap; a.scale = 1.0f / sqrtf((float)d.head_dim); a.mode = ATTN_CAUSAL; a.window = 0; a.rm = rm;
    a.out = e->att; a.os = s.q_dim(); a.xs_out = e->xs_A; a.xs_K = s.q_dim(); a.hs_out = hsA;
    launch_attn(a, d.head_dim, st);
    {  // o_proj + residual
      GemvParams g = gp(e);
      g.W = l.wo; g.N = D; g.K = s.q_dim(); g.M = M; g.out = e->x; g.os = D; g.xs_in = e->xs_A;
      g.xs_out = e->xs_D; g.xs_nw = l.n2; g.ss_out = e->xs_ss; g.ss_stride = GEMM_XS_MAX_M; g.xs_K = D;
      g.hs_in = hsA; g.hs_out = hsD;
      launch_gemm_xs(g, EPI_ADD, st, gemv_nt(0), e->wdt);
    }
    {  // norm2 + gate/up + SiLU*up
      GemvParams g = gp(e);
      g.W = l.wgu; g.N = 2 * F; g.K = D; g.M = M; g.nw = l.n2; g.eps = d.eps; g.out = nullptr; g.os = F;
      g.xs_in = e->xs_D; g.ss_in = e->xs_ss; g.ss_n = ss_o; g.ss_stride = GEMM_XS_MAX_M;
      g.xs_out = e->xs_F; g.xs_K = F; g.hs_in = hsD; g.hs_out = hsF;
      launch_gemm_xs(g, EPI_SILU_MUL, st, gemv_nt(0), e->wdt);
    }
    {  // down + residual (the last layer's rows go to the final norm in fp32 only)
      GemvParams g = gp(e);
      g.W = l.wd; g.N = D; g.K = F; g.M = M; g.out = e->x; g.os = D; g.xs_in = e->xs_F; g.hs_in = hsF;
      if (i + 1 < d.n_layers) {
        g.xs_out = e->xs_D; g.xs_nw = s.L[i + 1].n1; g.ss_out = e->xs_ss; g.ss_stride = GEMM_XS_MAX_M; g.xs_K = D;
        g.hs_out = hsD;
      }
      launch_gemm_xs(g, EPI_ADD, st, gemv_nt(0), e->wdt);
    }
  }
}

void embed(csm_engine* e, const EmbedParams& ep, int M, hipStream_t st) {
  if (e->wdt == WDT_Q4) launch_embed_q4(ep, e->dims.n_text_vocab, M, st);
  else launch_embed(ep, e->wdt, M, st);
}

// arg-max partial slots per row of a head launch (GEMV or MFMA path, dense or int4)
int head_blocks(int N, int K, int M, int wdt) { return gemv_partials(N, K, M, wdt); }

// The persistent backbone step runs the 16 blocks + final norm of a batch-1 decode row when the
// engine has csm_1b's backbone shapes in bf16 (with the chunk-major down copies) and the device has
// the 256 CUs its one-workgroup-per-CU grid assumes (every workgroup must be resident).
bool bb_step_eligible(csm_engine* e) {
  if (!e->bb_step || !e->bb_gbuf || e->B != 1 || (e->wdt != WDT_BF16 && e->wdt != WDT_Q4)) return false;
  const bool q4 = e->wdt == WDT_Q4;
  const csm_llama_dims& d = e->bb.d;
  if (d.hidden != 2048 || d.intermediate != 8192 || d.n_heads != 32 || d.n_kv_heads != 8 || d.head_dim != 64 ||
      d.n_layers != BB_STEP_LAYERS)
    return false;
  for (const LayerW& l : e->bb.L)
    if (!(q4 ? l.wdq : l.wdc)) return false;
  if (q4 && e->tiled_dirty) return false;  // (the int4 down copies are rebuilt at csm_begin)
  int& hw = q4 ? e->bb_hw_q4 : e->bb_hw;
  if (hw < 0) {
    hipDeviceProp_t prop;
    int per_cu = 0;
    hw = hipGetDeviceProperties(&prop, e->dev) == hipSuccess && prop.multiProcessorCount == BB_STEP_WGS &&
                 hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bb_step_kernel_ptr(q4), BB_STEP_THREADS, 0) ==
                     hipSuccess && per_cu >= 1
             ? 1 : 0;
  }
  return hw == 1;
}

void enqueue_bb_step(csm_engine* e, hipStream_t st) {
  BbStepArgs a{};
  for (int l = 0; l < BB_STEP_LAYERS; ++l) {
    const LayerW& w = e->bb.L[l];
    a.wqkv[l] = (const bf16_t*)w.wqkv; a.wo[l] = (const bf16_t*)w.wo; a.wgu[l] = (const bf16_t*)w.wgu;
    a.wdc[l] = (const bf16_t*)(e->wdt == WDT_Q4 ? w.wdq : w.wdc); a.n1[l] = w.n1; a.n2[l] = w.n2; a.kc[l] = w.kc; a.vc[l] = w.vc;
  }
  a.norm = e->bb.norm; a.rope = e->bb.rope; a.S_cap = e->bb.S_cap; a.eps = e->bb.d.eps;
  a.x = e->x; a.pos = e->pos; a.h_last = e->h_last;
  a.gbuf = (unsigned long long*)e->bb_gbuf; a.epoch = e->bb_epoch; a.err = e->bb_err; a.stamps = e->bb_stamps;
  launch_bb_step(a, st, e->wdt == WDT_Q4);
}

void enqueue_body(csm_engine* e, hipStream_t st) {
  const int B = e->B;
  EmbedParams ep{};
  ep.codes = e->codes; ep.text_emb = e->text_emb; ep.audio_emb = e->audio_emb; ep.V = e->V; ep.K = e->K;
  ep.D = e->D; ep.out = e->x; ep.pos_inc = e->pos;
  // batched backbone rows on the streaming GEMM (round 4 default; option bb_xs / CSM_BB_XS=0: gemm_wide)
  const bool bb_xs = e->bb_xs_on && !bb_step_eligible(e) && bb_xs_eligible(e, B);
  if (bb_xs) {
    ep.xs_out = e->xs_D; ep.xs_nw = e->bb.L[0].n1; ep.ss_out = e->xs_ss; ep.ss_stride = GEMM_XS_MAX_M;
    ep.hs_out = e->wdt == WDT_Q4 ? e->hs_D : nullptr;
  }
  embed(e, ep, B, st);
  if (bb_step_eligible(e)) {
    enqueue_bb_step(e, st);
    return;
  }
  RowMap rm{1, 0, e->pos, 0};
  if (bb_xs) {
    run_bb_xs(e, B, rm, st);
    launch_rmsnorm_rows(e->x, e->D, e->bb.norm, e->bb.d.eps, e->D, e->h_last, e->D, B, st);
    return;
  }
  run_stack(e, e->bb, e->x, B, e->q, e->att, e->mlp, rm, st);
  launch_rmsnorm_rows(e->x, e->D, e->bb.norm, e->bb.d.eps, e->D, e->h_last, e->D, B, st);
}

// The persistent frame decoder runs the whole head of a batch-1 frame (greedy, or sampled: its heads
// then hand every logit to every workgroup, which runs the sampler's top-k + Gumbel-max) when the engine has
// csm_1b's decoder shapes in bf16 and the folded tables, and the device has the 256 CUs its grid of
// one workgroup per CU assumes (every workgroup must be resident: the hand-offs spin).
bool dec_frame_eligible(csm_engine* e) {
  if (!e->dec_frame || e->B != 1 || (e->wdt != WDT_BF16 && e->wdt != WDT_Q4) || e->head_wdt != WDT_BF16) return false;
  const bool q4 = e->wdt == WDT_Q4;
  if (e->temperature > 0.f && (e->use_top_p || e->use_min_p)) return false;  // filters: sample_filtered_kernel
  const csm_llama_dims& d = e->dec.d;
  if (d.hidden != 1024 || d.intermediate != 8192 || d.n_heads != 8 || d.n_kv_heads != 2 || d.head_dim != 128 ||
      d.n_layers != DEC_FRAME_LAYERS || e->bb.d.hidden != 2048 || e->V <= 2048 || e->V > 2051 || e->K > 32 ||
      e->dec.S_cap != e->K)
    return false;
  for (const LayerW& l : e->dec.L)
    if (!(q4 ? l.wdq : l.wdc)) return false;
  if (q4 && e->tiled_dirty) return false;  // (the int4 down copies are rebuilt at csm_begin)
  if (!e->proj_tab || !e->fold_proj || !e->use_qkv0_tab || !e->qkv0_built || e->proj_tab_dirty) return false;
  int& hw = q4 ? e->df_hw_q4 : e->df_hw;
  if (hw < 0) {
    hipDeviceProp_t prop;
    int per_cu = 0;
    hw = hipGetDeviceProperties(&prop, e->dev) == hipSuccess && prop.multiProcessorCount == DEC_FRAME_WGS &&
                 hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dec_frame_kernel_ptr(q4), DEC_FRAME_THREADS, 0) ==
                     hipSuccess && per_cu >= 1
             ? 1 : 0;
  }
  return hw == 1;
}

void enqueue_dec_frame_only(csm_engine* e, hipStream_t st) {
  DecFrameArgs a{};
  for (int l = 0; l < DEC_FRAME_LAYERS; ++l) {
    const LayerW& w = e->dec.L[l];
    a.wqkv[l] = (const bf16_t*)w.wqkv; a.wo[l] = (const bf16_t*)w.wo; a.wgu[l] = (const bf16_t*)w.wgu;
    a.wdc[l] = (const bf16_t*)(e->wdt == WDT_Q4 ? w.wdq : w.wdc); a.n1[l] = w.n1; a.n2[l] = w.n2; a.kc[l] = w.kc; a.vc[l] = w.vc;
  }
  a.norm = e->dec.norm; a.rope = e->dec.rope; a.S_cap = e->dec.S_cap; a.eps = e->dec.d.eps;
  a.c0_head = (const bf16_t*)e->c0_head; a.proj = (const bf16_t*)e->proj; a.audio_head = (const bf16_t*)e->audio_head;
  a.proj_tab = e->proj_tab; a.qkv0_tab = e->qkv0_tab; a.h_last = e->h_last;
  a.V = e->V; a.VP = e->Vpad; a.K = e->K; a.codes = e->codes; a.c0_logits = e->c0_logits; a.ci_logits = e->ci_logits;
  a.gbuf = (unsigned long long*)e->df_gbuf; a.epoch = e->df_epoch; a.err = e->df_err; a.stamps = e->df_stamps;
  static const int wnt = [] { const char* v = getenv("CSM_DF_WNT"); return v ? atoi(v) : 0; }();
  static const int hnt = [] { const char* v = getenv("CSM_DF_HNT"); return v ? atoi(v) : 1; }();
  a.wnt = wnt; a.hnt = hnt;
  a.temperature = e->temperature; a.top_k = e->top_k; a.seeds = e->seeds; a.frame_ctr = e->frame_ctr;
  launch_dec_frame(a, st, e->wdt == WDT_Q4);
}

void enqueue_dec_frame(csm_engine* e, hipStream_t st) {
  enqueue_dec_frame_only(e, st);
  AdvanceParams ap{};  // codes are final: EOS test, history, frame counter
  ap.codes = e->codes; ap.hist = e->hist; ap.F_cap = e->F_cap; ap.B = e->B; ap.K = e->K; ap.V = e->V; ap.done = e->done;
  ap.n_frames = e->n_frames; ap.frame_ctr = e->frame_ctr;
  launch_advance(ap, st);
}

// The persistent batched decoder step (dec_step_xs.hip) runs a codebook step >= 2 of the streaming
// matrix-core path (xs_dec) when the decoder has csm_1b's shapes in bf16, the rows fit one 32-row tile and
// the device holds one 512-thread workgroup on each of its 256 CUs (every workgroup must be resident).
bool xsd_eligible(csm_engine* e, int M) {
  const bool q4 = e->wdt == WDT_Q4;
  if (!e->xsd_on || !e->xsd_ctrl || M < 1 || M > (q4 ? DEC_XSD_MAX_M_Q4 : DEC_XSD_MAX_M) || (e->wdt != WDT_BF16 && !q4) ||
      e->head_wdt != WDT_BF16 || e->tiled_dirty || GEMM_XS_MAX_M != 64)
    return false;
  const csm_llama_dims& d = e->dec.d;
  if (d.hidden != 1024 || d.intermediate != 8192 || d.n_heads != 8 || d.n_kv_heads != 2 || d.head_dim != 128 ||
      d.n_layers != DEC_FRAME_LAYERS || e->dec.S_cap > 32)
    return false;
  int& hw = q4 ? e->xsd_hw_q4 : e->xsd_hw;
  if (hw < 0) {
    hipDeviceProp_t prop;
    int per_cu = 0;
    hw = hipGetDeviceProperties(&prop, e->dev) == hipSuccess && prop.multiProcessorCount == DEC_XSD_WGS &&
                 hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dec_step_xs_kernel_ptr(q4), DEC_XSD_THREADS, 0) ==
                     hipSuccess && per_cu >= 1
             ? 1 : 0;
  }
  return hw == 1;
}

// step i >= 2 of the batched decoder: M rows (utterances 0..M-1) at position i; the codes of codebook
// i - 1 come from the head partials part_prev (part_n per row)
// returns true when the step's head ran in the same launch (its logits and arg-max partials are written)
bool launch_xsd(csm_engine* e, int M, int i, const unsigned long long* part_prev, int part_n, unsigned long long* part_out,
                hipStream_t st, bool sample = false) {
  DecStepXsArgs a = e->xsd;
  const Stack& s = e->dec;
  for (int l = 0; l < DEC_FRAME_LAYERS; ++l) {
    const LayerW& w = s.L[l];
    a.wqkv[l] = (const uint8_t*)e->ws.tiled.at(w.wqkv); a.wo[l] = (const uint8_t*)e->ws.tiled.at(w.wo);
    a.wgu[l] = (const uint8_t*)e->ws.tiled.at(w.wgu); a.wd[l] = (const uint8_t*)e->ws.tiled.at(w.wd);
    a.n1[l] = w.n1; a.n2[l] = w.n2; a.kc[l] = w.kc; a.vc[l] = w.vc;
  }
  a.norm = s.norm; a.rope = s.rope; a.S_cap = s.S_cap; a.eps = s.d.eps;
  a.M = M; a.step = i;
  a.part = part_prev; a.part_stride = e->part_stride; a.part_n = part_n; a.V = e->V;
  a.qkv0_tab = e->qkv0_tab + (size_t)(i - 1) * e->V * s.qkv_rows();
  a.proj_tab = e->proj_tab + (size_t)(i - 1) * e->V * e->Dd;
  a.codes = e->codes; a.codes_K = e->K;
  a.xs_out = e->xs_D; a.ss_out = e->xs_ss; a.ss_stride = GEMM_XS_MAX_M;
  a.hs_out = e->hs_D;  // (int4: the half-group sums of xs_out)
  a.ctrl = e->xsd_ctrl; a.epoch = e->xsd_epoch; a.err = e->xsd_err; a.stamps = e->xsd_stamps;
  // the head in the same launch: 64-row tiles, one arg-max partial each -- the launch path's partial count
  const int Vp = e->Vpad, ht = (Vp + 63) / 64;
  const void* hw = (const char*)e->audio_head + (size_t)(i - 1) * Vp * e->Dd * 2;
  auto it = e->ws.tiled.find(hw);
  // (int4: the head's (tile, row tile) pairs on the 64 attention + 32 plain workgroups: <= 48 tiles)
  if (e->xsd_head && it != e->ws.tiled.end() && ht == head_blocks(Vp, e->Dd, M, e->head_wdt) && ht <= (e->wdt == WDT_Q4 ? 48 : 64)) {
    a.head_w = (const uint8_t*)it->second; a.head_nt32 = (Vp + 31) / 32; a.head_tiles = ht; a.Vp = Vp; a.n_valid = e->V;
    a.head_out = e->ci_logits + (size_t)(i - 1) * e->B * Vp; a.head_part = part_out;
    // the sampled step's sampler in the same launch (option dec_xsd_sample; V within the sampler's reach)
    if (sample && e->xsd_sample && e->V <= DEC_XSD_THREADS * DEC_XSD_SAMPLE_NPT) {
      a.sample = 1; a.s_top_k = e->top_k; a.s_K = e->K; a.s_cb = i; a.s_temperature = e->temperature;
      a.s_seeds = e->seeds; a.s_frame_ctr = e->frame_ctr;
    }
  }
  launch_dec_step_xs(a, st, e->wdt == WDT_Q4);
  e->xsd_sampled = a.sample != 0;
  return a.head_w != nullptr;
}

// A hand-off wait of a persistent kernel that timed out leaves its flag raised: report it.
// Every raised flag is cleared and named in the one error.
void check_dec_frame(csm_engine* e) {
  std::string who;
  for (int* f : {e->df_err, e->bb_err, e->xsd_err}) {
    if (!f) continue;
    int v = 0;
    HIPCHK(hipMemcpy(&v, f, 4, hipMemcpyDeviceToHost));
    if (v) {
      HIPCHK(hipMemset(f, 0, 4));
      if (f == e->xsd_err) {  // counters and flags are out of step with the epoch: start both afresh
        HIPCHK(hipMemset(e->xsd_ctrl, 0, dec_step_xs_ctrl_bytes()));
        HIPCHK(hipMemset(e->xsd_epoch, 0, 4));
      }
      who += std::string(who.empty() ? "" : " and ") +
             (f == e->df_err ? "persistent frame decoder" : (f == e->bb_err ? "persistent backbone step" : "persistent batched decoder step"));
    }
  }
  if (!who.empty()) throw CsmError(CSM_ERR_HIP, who + ": a hand-off wait timed out (results of this batch are invalid)");
}

// phase 0: the whole head (what the frame graph captures).  phase 1: c0 logits only, stored for the
// host (logits processors, generation.py:44-49).  phase 2: the rest of the frame from c0 logits the
// host wrote back: c0 is picked by the sample kernel (arg-max when greedy, published as one partial),
// then steps 1..K-1 as in phase 0.
// phase 3: teacher forcing -- every head stores its logits and the code fed forward is the caller's
// (e->force [B][K]), as compute_loss feeds the target frame (trainer.py:233-262).
// phase 4: one piece of a host-sampled frame (a sampler callable on the host, csm_frame_host_step):
// piece p feeds the host's code for codebook p - 1 forward (e->force, as teacher forcing) and runs
// decoder step p + its head (logits stored); piece K feeds the last code and advances the frame.  The
// c0 head ran as phase 1 (csm_frame_c0_logits).
void enqueue_head_phase(csm_engine* e, hipStream_t st, int phase, int piece = 0) {
  if (phase == 0 && dec_frame_eligible(e)) {
    enqueue_dec_frame(e, st);
    return;
  }
  const int B = e->B, K = e->K, D = e->D, Dd = e->Dd, V = e->V, Vp = e->Vpad;
  const bool greedy = e->temperature <= 0.f && phase != 3 && phase != 4;
  const bool c0_sampled = !greedy || phase == 2;  // c0 published by sample_kernel as a single partial
  const int n0 = head_blocks(Vp, D, B, e->wdt);        // c0-head blocks (partials per row)
  const int ni = head_blocks(Vp, Dd, B, e->head_wdt);  // ci-head blocks
  auto part = [&](int cb) { return e->part + (size_t)cb * e->B_max * e->part_stride; };
  SampleParams sp{};
  sp.ls = Vp; sp.V = V; sp.temperature = e->temperature; sp.top_k = e->top_k; sp.seeds = e->seeds;
  sp.frame_ctr = e->frame_ctr; sp.K = K; sp.codes = e->codes; sp.part_stride = e->part_stride;
  sp.use_top_p = e->use_top_p; sp.use_min_p = e->use_min_p; sp.min_keep = e->min_keep;
  sp.top_p_cut = e->top_p_cut; sp.log_min_p = e->log_min_p;
  sp.forced = (phase == 3 || phase == 4) ? e->force : nullptr;
  // c0 = codebook0_head(h_last) (generation.py:42); greedy arg-max fused into the GEMV epilogue
  GemvParams g = gp(e);
  g.W = e->c0_head; g.N = Vp; g.K = D; g.x = e->h_last; g.xs = D; g.M = B; g.out = e->c0_logits; g.os = Vp;
  g.part = part(0); g.part_stride = e->part_stride; g.n_valid = V;
  if (phase != 2 && phase != 4) launch_gemv(g, e->wdt, (greedy && phase == 0) ? EPI_ARGMAX : EPI_STORE, 0, st);
  if (phase == 1) return;
  const int cb_first = phase == 4 ? piece - 1 : 0;  // the code fed forward before the first step below
  if (c0_sampled) {
    sp.logits = e->c0_logits; sp.cb = cb_first; sp.part = part(cb_first);
    launch_sample(sp, e->wdt, B, st);
  }
  const int i_lo = phase == 4 ? piece : 1, i_hi = phase == 4 ? std::min(piece + 1, K) : K;
  for (int i = i_lo; i < i_hi; ++i) {
    const int M = (i == 1) ? 2 * B : B;
    // decoder(projection(decoder_inputs)) (generation.py:74-77): the projection gathers its input
    // rows itself -- [h_last, E_a[c0]] at step 1 (:62-64), E_a[c_{i-1} + V*(i-1)] after (:87-89)
    g = gp(e);
    g.W = e->proj; g.N = Dd; g.K = D; g.x = e->h_last; g.xs = D; g.M = M; g.out = e->dx; g.os = Dd;
    g.xpart = part(i - 1); g.xpart_stride = e->part_stride; g.xpart_n = i == 1 ? (c0_sampled ? 1 : n0) : (greedy ? ni : 1);
    g.xtab = e->audio_emb; g.xV = V; g.xcb = i - 1; g.x_step1 = (i == 1); g.x_codes = e->codes; g.x_codes_K = K;
    g.xtab_q4_rows = e->wdt == WDT_Q4 ? V * K : 0;
    const bool folded = i >= 2 && e->proj_tab && e->fold_proj;
    GemvParams g0 = g;  // steps >= 2: layer 0 gathers projection(E_a[c]) from the folded table
    g0.xtab = e->proj_tab; g0.xtab_f32 = 1; g0.xtab_q4_rows = 0;
    RowMap rm = (i == 1) ? RowMap{2, 0, nullptr, 0} : RowMap{1, 0, nullptr, i};
    const bool use_tab = folded && e->use_qkv0_tab && e->qkv0_built && !e->no_tab_batched;
    const bool xs_dec = use_tab && dec_xs_eligible(e, M);  // streaming matrix-core decoder + head
    bool xsd_used = false;  // the persistent step ran (its combines wrote 32 sum-of-squares tiles)
    bool xsd_head_done = false;  // ... and the head in the same launch
    bool xsd_sampled = false;    // ... and the sampler
    // step 1 (two rows per utterance) on the streaming GEMM too: the projected rows split once, layer 0's
    // QKV projected from them; the head stays on the dense path (it reads one row of each pair)
    const bool xs_s1 = i == 1 && !folded && e->xs_step1 && dec_xs_eligible(e, M) && Dd % 512 == 0;
    if (!use_tab && (gemm_mfma_eligible(Dd, D, M, e->wdt) || gemm_mfma_eligible(e->dec.qkv_rows(), Dd, M, e->wdt))) {
      // batched: materialise the gathered rows densely, then every projection runs on the matrix cores
      if (!folded) {
        GemvParams gr = g;
        gr.K = D; gr.out = e->din; gr.os = D;
        launch_gather_rows(gr, e->wdt, st);
        GemvParams gj = gp(e);
        gj.W = e->proj; gj.N = Dd; gj.K = D; gj.x = e->din; gj.xs = D; gj.M = M; gj.out = e->dx; gj.os = Dd;
        launch_gemv(gj, e->wdt, EPI_STORE, 0, st);
      } else {
        GemvParams gr = g0;
        gr.K = Dd; gr.out = e->dx; gr.os = Dd;
        launch_gather_rows(gr, e->wdt, st);
      }
      if (xs_s1) {
        launch_xs_rows(e->dx, (int)Dd, M, (int)Dd, e->dec.L[0].n1, e->xs_D, e->xs_ss, GEMM_XS_MAX_M,
                       e->wdt == WDT_Q4 ? e->hs_D : nullptr, st);
        run_dec_xs(e, M, rm, st, AttnParams{}, true);
      } else {
        run_stack(e, e->dec, e->dx, M, e->dq, e->datt, e->dmlp, rm, st, nullptr);
      }
    } else if (use_tab) {
      // layer 0's q | k | v and input row gathered from the folded tables by the attention (no layer-0
      // QKV projection); at >= 8 rows the other projections run on the matrix cores
      AttnParams a0{};
      a0.g_tab = e->qkv0_tab + (size_t)(i - 1) * V * e->dec.qkv_rows(); a0.g_row = e->dec.qkv_rows();
      a0.g_part = g.xpart; a0.g_part_stride = g.xpart_stride; a0.g_part_n = g.xpart_n; a0.g_V = V;
      a0.g_codes = e->codes; a0.g_codes_K = K; a0.g_cb = i - 1;
      a0.g_xtab = e->proj_tab + (size_t)(i - 1) * V * Dd; a0.g_xout = e->dx; a0.g_D = Dd;
      if (xs_dec && xsd_eligible(e, M)) {
        // sampled frames (phases 0 / 2; top-k only): the sampler runs in the step's launch too
        const bool fuse_sample = !greedy && (phase == 0 || phase == 2) && !e->use_top_p && !e->use_min_p;
        xsd_head_done = launch_xsd(e, M, i, g.xpart, g.xpart_n, part(i), st, fuse_sample);
        xsd_sampled = xsd_head_done && e->xsd_sampled;
        xsd_used = true;
      } else if (xs_dec) {
        run_dec_xs(e, M, rm, st, a0);
      } else {
        run_stack(e, e->dec, e->dx, M, e->dq, e->datt, e->dmlp, rm, st, nullptr, &a0);
      }
    } else {
      if (!folded) launch_gemv(g, e->wdt, EPI_STORE, 0, st);
      run_stack(e, e->dec, e->dx, M, e->dq, e->datt, e->dmlp, rm, st, folded ? &g0 : nullptr);
    }
    // ci_logits = norm(hidden[:, -1]) @ audio_head[i-1]  (generation.py:79)
    g = gp(e);
    g.W = (const char*)e->audio_head + (size_t)(i - 1) * Vp * Dd * (e->head_wdt == WDT_F32 ? 4 : 2); g.N = Vp; g.K = Dd;
    g.x = e->dx + (i == 1 ? Dd : 0); g.xs = (i == 1 ? 2 * Dd : Dd); g.M = B; g.nw = e->dec.norm;
    g.eps = e->dec.d.eps; g.out = e->ci_logits + (size_t)(i - 1) * B * Vp; g.os = Vp;
    g.part = part(i); g.part_stride = e->part_stride; g.n_valid = V;
    if (xsd_head_done) {
      // (logits and arg-max partials written by the persistent step)
    } else if (xs_dec) {  // the head reads the split rows (x * final norm) the last down wrote
      g.xs_in = e->xs_D; g.ss_in = e->xs_ss; g.ss_n = xsd_used ? 32 : gemm_xs_tiles(Dd, e->dec.d.intermediate, M);
      g.ss_stride = GEMM_XS_MAX_M;
      launch_gemm_xs(g, greedy ? EPI_ARGMAX : EPI_STORE, st, gemv_nt(2), e->head_wdt);
    } else if (!(ablate() & 64)) {
      launch_gemv(g, e->head_wdt, greedy ? EPI_ARGMAX : EPI_STORE, 1, st);
    }
    if (!greedy && phase != 4 && !xsd_sampled) {
      sp.logits = e->ci_logits + (size_t)(i - 1) * B * Vp; sp.cb = i; sp.part = part(i);
      launch_sample(sp, e->wdt, B, st);
    }
  }
  if (phase == 4 && piece < K) return;  // the frame continues with the host's next code
  AdvanceParams ap{};
  ap.codes = e->codes; ap.hist = e->hist; ap.F_cap = e->F_cap; ap.B = B; ap.K = K; ap.V = V; ap.done = e->done;
  ap.n_frames = e->n_frames; ap.frame_ctr = e->frame_ctr;
  if (greedy) {
    ap.last_part = part(K - 1); ap.last_stride = e->part_stride; ap.last_n = ni;
  }
  launch_advance(ap, st);
}

void enqueue_head(csm_engine* e, hipStream_t st) { enqueue_head_phase(e, st, 0); }

hipGraphExec_t capture(csm_engine* e, void (*fn)(csm_engine*, hipStream_t)) {
  hipGraph_t graph;
  HIPCHK(hipStreamBeginCapture(e->st, hipStreamCaptureModeThreadLocal));
  fn(e, e->st);
  HIPCHK(hipStreamEndCapture(e->st, &graph));
  hipGraphExec_t exec;
  HIPCHK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  (void)hipGraphDestroy(graph);
  return exec;
}

// (Re)allocate everything sized by the batch: KV caches, decoder activations, code history.
void ensure_batch(csm_engine* e, int B) {
  if (B <= e->B_max && !e->batch_allocs.empty()) return;
  HIPCHK(hipDeviceSynchronize());
  for (void* p : e->batch_allocs) (void)hipFree(p);
  e->batch_allocs.clear();
  if (e->g_body) { (void)hipGraphExecDestroy(e->g_body); e->g_body = nullptr; }
  if (e->g_head) { (void)hipGraphExecDestroy(e->g_head); e->g_head = nullptr; }
  e->g_B = -1;
  e->B_max = std::max(B, e->B_max);
  const size_t Bm = e->B_max, D = e->D, Dd = e->Dd, K = e->K, Vp = e->Vpad;
  for (Stack* s : {&e->bb, &e->dec}) {
    const size_t kv = Bm * s->d.n_kv_heads * (size_t)s->S_cap * s->d.head_dim * 4;
    for (LayerW& l : s->L) {
      l.kc = (float*)e->balloc(kv);
      l.vc = (float*)e->balloc(kv);
    }
  }
  e->h_last = (float*)e->balloc(Bm * D * 4);
  e->c0_logits = (float*)e->balloc(Bm * Vp * 4);
  e->force = (int*)e->balloc(Bm * K * 4);
  e->force_ce = (float*)e->balloc(Bm * K * 4);
  e->ci_logits = (float*)e->balloc((K - 1) * Bm * Vp * 4);
  e->dx = (float*)e->balloc(2 * Bm * Dd * 4);
  e->din = (float*)e->balloc(2 * Bm * D * 4);
  e->dq = (float*)e->balloc(2 * Bm * e->dec.q_dim() * 4);
  e->datt = (float*)e->balloc(2 * Bm * e->dec.q_dim() * 4);
  e->dmlp = (float*)e->balloc(2 * Bm * (size_t)e->dec.d.intermediate * 4);
  e->codes = (int*)e->balloc(Bm * K * 4);
  e->hist = (int*)e->balloc((size_t)e->F_cap * Bm * K * 4);
  e->pos = (int*)e->balloc(Bm * 4);
  e->n_frames = (int*)e->balloc(Bm * 4);
  e->done = (uint8_t*)e->balloc(Bm);
  e->seeds = (uint64_t*)e->balloc(Bm * 8);
  // partial slots per row: enough for any head tiling (c0 / ci heads, dense or q4; >= Vp/2 blocks never occur)
  e->part_stride = (int)(Vp / 2);
  e->part = (unsigned long long*)e->balloc(K * Bm * (size_t)e->part_stride * 8);
  // split-K scratch of the MFMA path for every projection shape at its largest row count
  for (Stack* s : {&e->bb, &e->dec}) {
    const int Dm = s->d.hidden, F = s->d.intermediate, rows = (s == &e->bb) ? std::max(e->M_cap, (int)Bm) : 2 * (int)Bm;
    gemm_reserve(e->ws, s->qkv_rows(), Dm, rows);
    gemm_reserve(e->ws, Dm, s->q_dim(), rows);
    gemm_reserve(e->ws, 2 * F, Dm, rows);
    gemm_reserve(e->ws, Dm, F, rows);
  }
  gemm_reserve(e->ws, (int)Dd, (int)D, 2 * (int)Bm);
  gemm_reserve(e->ws, (int)Vp, (int)D, (int)Bm);   // c0 head
  gemm_reserve(e->ws, (int)Vp, (int)Dd, (int)Bm);  // ci heads
  // the streaming decoder path (gemm_xs): split-row buffers for up to GEMM_XS_MAX_M rows + its scratch
  {
    // (shared by the backbone and the decoder: their launches never overlap)
    // (2 Bm: the depth decoder's step 1 carries two rows per utterance)
    const int xm = GEMM_XS_MAX_M, rows = std::min(2 * (int)Bm, xm);
    size_t bD = 0, bA = 0, bF = 0;
    for (Stack* s : {&e->bb, &e->dec}) {
      const int Dm = s->d.hidden, F = s->d.intermediate;
      bD = std::max(bD, xs::bytes(xm, Dm));
      bA = std::max(bA, xs::bytes(xm, s->q_dim()));
      bF = std::max(bF, xs::bytes(xm, F));
      gemm_xs_reserve(e->ws, s->qkv_rows(), Dm, rows);
      gemm_xs_reserve(e->ws, Dm, s->q_dim(), rows);
      gemm_xs_reserve(e->ws, 2 * F, Dm, rows);
      gemm_xs_reserve(e->ws, Dm, F, rows);
    }
    gemm_xs_reserve(e->ws, (int)Vp, (int)Dd, rows);
    e->xs_D = e->balloc(bD);
    e->xs_A = e->balloc(bA);
    e->xs_F = e->balloc(bF);
    e->xs_ss = (float*)e->balloc((size_t)64 * xm * 4);
    for (float** h : {&e->hs_D, &e->hs_A, &e->hs_F}) *h = (float*)e->balloc(bF / xs::XS_EB / xm / 32 * xs::HS_ROWS * 4 + 4096);
  }
  // the persistent batched decoder step's scratch (csm_1b decoder shapes only; control words once per engine)
  {
    const csm_llama_dims& d = e->dec.d;
    if (d.hidden == 1024 && d.intermediate == 8192 && d.head_dim == 128 && d.n_heads == 8 && d.n_kv_heads == 2) {
      const size_t R = DEC_XSD_MAX_M_Q4;
      DecStepXsArgs& x = e->xsd;
      x.qkv = (float*)e->balloc(R * e->dec.qkv_rows() * 4);
      x.qkvp = (float*)e->balloc((2 * R * e->dec.qkv_rows() + (size_t)e->dec.qkv_rows() / 32 * R) * 4);  // + row scales [48][R]
      x.xs_att = e->balloc(xs::bytes(R, 1024));
      x.xs_x = e->balloc(xs::bytes(R, 1024));
      x.xs_h = e->balloc(xs::bytes(R, 8192));
      x.x_o = (float*)e->balloc(R * 1024 * 4);
      x.x_d = (float*)e->balloc(R * 1024 * 4);
      x.ss_o = (float*)e->balloc(32 * R * 4);
      x.dpart = (float*)e->balloc(8 * R * 1024 * 4);
      x.code_buf = (int*)e->balloc(R * 4);
      x.hs_att = (float*)e->balloc(1024 / 32 * R * 4);
      x.hs_x = (float*)e->balloc(1024 / 32 * R * 4);
      x.hs_h = (float*)e->balloc(8192 / 32 * R * 4);
      if (!e->xsd_ctrl) {
        e->xsd_ctrl = (unsigned*)e->alloc(dec_step_xs_ctrl_bytes());
        e->xsd_epoch = (unsigned*)e->alloc(16);
        e->xsd_err = (int*)e->alloc(16);
      }
    }
  }
}

// Fragment-tiled copies (launch_gemm_retile) of every matrix the batched MFMA path reads -- stack
// projections, projection, codebook0_head, the bf16 audio_head slices -- rebuilt in place after any
// weight change (csm_load_tensor, csm_quantize), at csm_begin, before graphs capture them.
void build_tiled(csm_engine* e) {
  // pass 0 allocates (alloc's zero fill runs on the null stream: drained before pass 1 writes the
  // copies on the engine stream), pass 1 re-lays every matrix
  for (int pass = 0; pass < 2; ++pass) {
  size_t idx = 0;
  auto one = [&](const void* W, int N, int K, int wdt) {
    if (wdt != WDT_BF16 && wdt != WDT_Q4) return;
    if (pass == 0) {
      if (idx++ == e->tiled_bufs.size()) e->tiled_bufs.push_back(e->alloc(gemm_tiled_bytes(N, K, wdt)));
      return;
    }
    void* T = e->tiled_bufs[idx++];
    launch_gemm_retile(W, T, N, K, wdt, e->st);
    e->ws.tiled[W] = T;
  };
  for (Stack* s : {&e->bb, &e->dec})
    for (LayerW& l : s->L) {
      const int D = s->d.hidden, F = s->d.intermediate;
      one(l.wqkv, s->qkv_rows(), D, e->wdt);
      one(l.wo, D, s->q_dim(), e->wdt);
      one(l.wgu, 2 * F, D, e->wdt);
      one(l.wd, D, F, e->wdt);
    }
  one(e->proj, e->Dd, e->D, e->wdt);
  one(e->c0_head, e->Vpad, e->D, e->wdt);
  if (e->wdt == WDT_Q4)  // the persistent kernels' chunk-major down copies (bb_step_q4 / dec_frame_q4)
    for (Stack* s : {&e->bb, &e->dec})
      for (LayerW& l : s->L) {
        const int D = s->d.hidden, F = s->d.intermediate;
        if (F % 64) continue;
        if (pass == 0) { if (!l.wdq) l.wdq = e->alloc(q4_bytes(D, F)); }
        else launch_q4_down_cm(l.wd, D, F, l.wdq, e->st);
      }
  if (e->head_wdt == WDT_BF16)
    for (int cb = 0; cb < e->K - 1; ++cb) one((const char*)e->audio_head + (size_t)cb * e->Vpad * e->Dd * 2, e->Vpad, e->Dd, WDT_BF16);
  HIPCHK(hipDeviceSynchronize());
  }
  HIPCHK(hipGetLastError());
  e->tiled_dirty = false;
}

// proj_tab[cb] = projection(E_a rows of codebook cb), computed by the projection GEMV itself
// (per-row arithmetic identical to the per-step launch it replaces).
void build_proj_table(csm_engine* e) {
  const int V = e->V, D = e->D, Dd = e->Dd;
  float* scratch = e->mlp;  // [M_cap][F] fp32: >= V*D floats (checked at create)
  for (int cb = 0; cb < e->K - 1; ++cb) {
    if (e->wdt == WDT_Q4) launch_q4_to_f32(e->audio_emb, V * e->K, D, cb * V, V, scratch, e->st);
    else launch_to_f32((const char*)e->audio_emb + (size_t)cb * V * D * e->wsz, e->wdt, scratch, (size_t)V * D, e->st);
    GemvParams g = gp(e);
    g.W = e->proj; g.N = Dd; g.K = D; g.x = scratch; g.xs = D; g.M = V;
    g.out = e->proj_tab + (size_t)cb * V * Dd; g.os = Dd;
    g.no_mfma = 1;  // the GEMV's per-row arithmetic (the step-1 launch's), never the matrix cores
    launch_gemv_table(g, e->wdt, EPI_STORE, 0, e->st, 1);
  }
  HIPCHK(hipStreamSynchronize(e->st));
  HIPCHK(hipGetLastError());
  e->proj_tab_dirty = false;
  // layer-0 QKV of every folded decoder input row, by the frame's own QKV GEMV (one launch per
  // codebook where the shape allows, else 4 rows per launch: per-row arithmetic of the 1-row launch)
  if (!e->use_qkv0_tab) return;  // built at the next csm_begin after csm_set_option("qkv0_tab", 1)
  const Stack& s = e->dec;
  const LayerW& l0 = s.L[0];
  for (int cb = 1; cb < e->K - 1; ++cb) {
    GemvParams g = gp(e);
    g.W = l0.wqkv; g.N = s.qkv_rows(); g.K = Dd; g.x = e->proj_tab + (size_t)cb * V * Dd; g.xs = Dd;
    g.M = V; g.nw = l0.n1; g.eps = s.d.eps; g.Hq = s.d.n_heads; g.Hkv = s.d.n_kv_heads;
    g.hd = s.d.head_dim; g.S_cap = s.S_cap; g.rope = s.rope; g.rm = RowMap{1, 0, nullptr, cb + 1};
    g.qkv_tab = e->qkv0_tab + (size_t)cb * V * s.qkv_rows();
    launch_gemv_table(g, e->wdt, EPI_QKV, 1, e->st, 1);
  }
  HIPCHK(hipStreamSynchronize(e->st));
  HIPCHK(hipGetLastError());
  e->qkv0_built = true;
}



// Where an MLX Linear/Embedding weight lives in the engine: rows row0 + r*rstep (r < n) of a
// [Ntot][K] matrix at base.  False for parameters nn.quantize leaves alone (norms, audio_head).
struct Place {
  void* base = nullptr;
  int Ntot = 0, K = 0, row0 = 0, rstep = 1, n = 0;
};

bool weight_place(csm_engine* e, const std::string& name, Place& pl) {
  for (int which = 0; which < 2; ++which) {
    Stack& s = which == 0 ? e->bb : e->dec;
    const std::string pre = which == 0 ? "backbone.layers." : "decoder.layers.";
    if (name.rfind(pre, 0) != 0) continue;
    int li = -1;
    char tail[128] = {0};
    if (sscanf(name.c_str() + pre.size(), "%d.%127s", &li, tail) != 2 || li < 0 || li >= s.d.n_layers) return false;
    LayerW& l = s.L[li];
    const std::string t(tail);
    const int D = s.d.hidden, F = s.d.intermediate, qd = s.q_dim(), kvd = s.d.n_kv_heads * s.d.head_dim;
    const int qkv = s.qkv_rows();
    if (t == "self_attn.q_proj.weight") pl = Place{l.wqkv, qkv, D, 0, 1, qd};
    else if (t == "self_attn.k_proj.weight") pl = Place{l.wqkv, qkv, D, qd, 1, kvd};
    else if (t == "self_attn.v_proj.weight") pl = Place{l.wqkv, qkv, D, qd + kvd, 1, kvd};
    else if (t == "self_attn.o_proj.weight") pl = Place{l.wo, D, qd, 0, 1, D};
    else if (t == "mlp.gate_proj.weight") pl = Place{l.wgu, 2 * F, D, 0, 2, F};
    else if (t == "mlp.up_proj.weight") pl = Place{l.wgu, 2 * F, D, 1, 2, F};
    else if (t == "mlp.down_proj.weight") pl = Place{l.wd, D, F, 0, 1, D};
    else return false;
    return true;
  }
  const int D = e->D, Dd = e->Dd, V = e->V, K = e->K, Vp = e->Vpad;
  if (name == "text_embeddings.weight") pl = Place{e->text_emb, e->dims.n_text_vocab, D, 0, 1, e->dims.n_text_vocab};
  else if (name == "audio_embeddings.weight") pl = Place{e->audio_emb, V * K, D, 0, 1, V * K};
  else if (name == "projection.weight") pl = Place{e->proj, Dd, D, 0, 1, Dd};
  else if (name == "codebook0_head.weight") pl = Place{e->c0_head, Vp, D, 0, 1, V};
  else return false;
  return true;
}

// Device scratch for load-time conversions (grown on demand, freed after each load)
struct DevBuf {
  void* p = nullptr;
  explicit DevBuf(size_t n) { HIPCHK(hipMalloc(&p, n)); }
  ~DevBuf() { if (p) (void)hipFree(p); }
};

// int4 engine: an MLX float weight is quantized on the device; a pre-quantized one (uint32
// .weight + .scales + .biases, MLX QuantizedLinear / QuantizedEmbedding keys) is placed once all
// three parts have arrived.  Returns false for names that are not quantized parameters.
bool load_q4(csm_engine* e, const std::string& name, const void* host, int src_dtype, const std::vector<int64_t>& shp) {
  std::string base = name, part = "weight";
  for (const char* suf : {".scales", ".biases"})
    if (name.size() > strlen(suf) && name.compare(name.size() - strlen(suf), strlen(suf), suf) == 0) {
      base = name.substr(0, name.size() - strlen(suf)) + ".weight";
      part = suf + 1;
    }
  Place pl;
  if (!weight_place(e, base, pl)) return false;
  size_t numel = 1;
  for (auto v : shp) numel *= (size_t)v;
  if (part == "weight" && src_dtype != CSM_U32) {  // float weight -> quantize (nn.quantize)
    if (shp != std::vector<int64_t>{pl.n, pl.K}) throw CsmError(CSM_ERR_ARG, "shape mismatch for " + name);
    auto h = convert_to(host, src_dtype, numel, WDT_F32);
    DevBuf tmp(h.size());
    HIPCHK(hipMemcpy(tmp.p, h.data(), h.size(), hipMemcpyHostToDevice));
    launch_q4_quantize(tmp.p, WDT_F32, pl.n, pl.K, pl.base, pl.Ntot, pl.row0, pl.rstep, e->st);
    HIPCHK(hipStreamSynchronize(e->st));
    HIPCHK(hipGetLastError());
    e->loaded.insert(base);
    if (base == "audio_embeddings.weight" || base == "projection.weight") e->proj_tab_dirty = true;
    return true;
  }
  auto& pq = e->pending_q4[base];
  const size_t es = src_dtype == CSM_F32 || src_dtype == CSM_U32 ? 4 : 2;
  if (part == "weight") {
    if (shp != std::vector<int64_t>{pl.n, pl.K / 8}) throw CsmError(CSM_ERR_ARG, "packed shape mismatch for " + name);
    pq.packed.assign((const uint8_t*)host, (const uint8_t*)host + numel * 4);
  } else {
    if (src_dtype != CSM_F32 && src_dtype != CSM_BF16) throw CsmError(CSM_ERR_ARG, name + " must be f32 or bf16");
    if (shp != std::vector<int64_t>{pl.n, pl.K / Q4_GROUP}) throw CsmError(CSM_ERR_ARG, "shape mismatch for " + name);
    if (!pq.scales.empty() || !pq.biases.empty())
      if (pq.sdt != src_dtype) throw CsmError(CSM_ERR_ARG, "scales / biases dtypes differ for " + base);
    pq.sdt = src_dtype;
    (part == "scales" ? pq.scales : pq.biases).assign((const uint8_t*)host, (const uint8_t*)host + numel * es);
  }
  if (pq.packed.empty() || pq.scales.empty() || pq.biases.empty()) return true;
  // all three parts present: nibble rows (strided for interleaved gate/up) + sb words
  const size_t rowb = (size_t)pl.K / 2;
  HIPCHK(hipMemcpy2D((uint8_t*)pl.base + (size_t)pl.row0 * rowb, rowb * pl.rstep, pq.packed.data(), rowb, rowb, pl.n,
                     hipMemcpyHostToDevice));
  DevBuf sc(pq.scales.size()), bi(pq.biases.size());
  HIPCHK(hipMemcpy(sc.p, pq.scales.data(), pq.scales.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(bi.p, pq.biases.data(), pq.biases.size(), hipMemcpyHostToDevice));
  launch_q4_set_sb(sc.p, bi.p, pq.sdt == CSM_BF16 ? WDT_BF16 : WDT_F32, pl.n, pl.K, pl.base, pl.Ntot, pl.row0,
                   pl.rstep, e->st);
  HIPCHK(hipStreamSynchronize(e->st));
  HIPCHK(hipGetLastError());
  e->pending_q4.erase(base);
  e->loaded.insert(base);
  if (base == "audio_embeddings.weight" || base == "projection.weight") e->proj_tab_dirty = true;
  return true;
}

}  // namespace

// =============================================================================== C ABI
extern "C" {

int csm_device_count(int* n) {
  CSM_TRY {
    int c = 0;
    HIPCHK(hipGetDeviceCount(&c));
    if (n) *n = c;
  }
  CSM_CATCH
}

int csm_engine_create(const csm_dims* dims, int device, int weight_dtype, int max_batch, int max_frames,
                      csm_engine** out) {
  CSM_TRY {
    if (!dims || !out || max_batch <= 0 || max_frames <= 0) throw CsmError(CSM_ERR_ARG, "bad engine arguments");
    const csm_llama_dims& b = dims->backbone;
    const csm_llama_dims& d = dims->decoder;
    for (const csm_llama_dims* x : {&b, &d}) {
      if (x->head_dim != 64 && x->head_dim != 128) throw CsmError(CSM_ERR_ARG, "head_dim must be 64 or 128");
      if (x->hidden % 256 || x->intermediate % 256 || (x->n_heads * x->head_dim) % 256)
        throw CsmError(CSM_ERR_ARG, "hidden/intermediate widths must be multiples of 256");
      if (x->n_heads % x->n_kv_heads) throw CsmError(CSM_ERR_ARG, "n_heads % n_kv_heads != 0");
    }
    if (b.n_heads * b.head_dim != b.hidden) throw CsmError(CSM_ERR_ARG, "backbone hidden != heads*head_dim");
    for (const csm_llama_dims* x : {&b, &d})
      if (x->n_heads / x->n_kv_heads > 4) throw CsmError(CSM_ERR_ARG, "GQA group > 4 unsupported");
    if (weight_dtype != CSM_F32 && weight_dtype != CSM_BF16 && weight_dtype != CSM_Q4)
      throw CsmError(CSM_ERR_ARG, "weight_dtype must be CSM_F32, CSM_BF16 or CSM_Q4");
    {  // every GEMV shape must tile into whole blocks (q4: any even N whose K the q4 tiling covers)
      const int Vp = (dims->n_audio_vocab + 7) / 8 * 8;
      std::vector<std::pair<int, int>> shapes = {{Vp, b.hidden}, {Vp, d.hidden}, {d.hidden, b.hidden}};
      for (const csm_llama_dims* x : {&b, &d}) {
        shapes.push_back({(x->n_heads + 2 * x->n_kv_heads) * x->head_dim, x->hidden});
        shapes.push_back({x->hidden, x->n_heads * x->head_dim});
        shapes.push_back({2 * x->intermediate, x->hidden});
        shapes.push_back({x->hidden, x->intermediate});
      }
      for (auto [N, Kd] : shapes) {
        for (int M : {1, 4})
          if (N % gemv_rows_per_block(N, Kd, M)) throw CsmError(CSM_ERR_ARG, "GEMV shape does not tile");
        if (!gemv_q4_supported(N, Kd) && weight_dtype == CSM_Q4)
          throw CsmError(CSM_ERR_ARG, "int4 GEMV does not support this shape");
      }
    }
    HIPCHK(hipSetDevice(device));
    std::unique_ptr<csm_engine> e(new csm_engine());
    e->dims = *dims;
    e->dev = device;
    e->wdt = weight_dtype == CSM_F32 ? WDT_F32 : (weight_dtype == CSM_Q4 ? WDT_Q4 : WDT_BF16);
    e->head_wdt = e->wdt == WDT_F32 ? WDT_F32 : WDT_BF16;
    e->wsz = e->wdt == WDT_F32 ? 4 : 2;
    e->B_max = max_batch;
    e->F_cap = max_frames;
    e->K = dims->n_audio_codebooks;
    e->V = dims->n_audio_vocab;
    e->Vpad = (e->V + 7) / 8 * 8;
    e->D = b.hidden;
    e->Dd = d.hidden;
    const int S = dims->max_seq_len;
    e->M_cap = std::max(S, 2 * max_batch);
    if (const char* v = getenv("CSM_ATTN_PREFILL")) e->attn_tiles_on = atoi(v) != 0;  // lab: 0 = per-row prompt attention (A/B)
    if (const char* v = getenv("CSM_STREAM_PRIO"); !v || atoi(v) != 0) {  // the engine's stream first (mimi_create)
      int least = 0, greatest = 0;
      HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      HIPCHK(hipStreamCreateWithPriority(&e->st, hipStreamNonBlocking, greatest));
    } else {
      HIPCHK(hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking));
    }
    alloc_stack(e.get(), e->bb, b, S, "backbone");
    alloc_stack(e.get(), e->dec, d, e->K, "decoder");
    const size_t D = e->D, Dd = e->Dd, K = e->K, Vp = e->Vpad, B = max_batch;
    e->text_emb = e->alloc(e->wbytes(dims->n_text_vocab, D));
    e->audio_emb = e->alloc(e->wbytes((size_t)e->V * K, D));
    e->proj = e->alloc(e->wbytes(Dd, D));
    e->c0_head = e->alloc(e->wbytes(Vp, D));
    e->audio_head = e->alloc((K - 1) * Vp * Dd * (e->head_wdt == WDT_F32 ? 4 : 2));
    e->proj_tab = (float*)e->alloc((K - 1) * (size_t)e->V * Dd * 4);
    e->qkv0_tab = (float*)e->alloc((K - 1) * (size_t)e->V * e->dec.qkv_rows() * 4);
    for (const char* n : {"text_embeddings.weight", "audio_embeddings.weight", "projection.weight",
                          "codebook0_head.weight", "audio_head"})
      e->required.push_back(n);
    const size_t M = e->M_cap;
    e->x = (float*)e->alloc(M * D * 4);
    e->q = (float*)e->alloc(M * e->bb.q_dim() * 4);
    e->att = (float*)e->alloc(M * e->bb.q_dim() * 4);
    e->mlp = (float*)e->alloc(M * b.intermediate * 4);
    if (M * (size_t)b.intermediate < (size_t)e->V * e->D)
      throw CsmError(CSM_ERR_ARG, "activation scratch too small for the projection table build");
    e->tok = (int32_t*)e->alloc(M * (K + 1) * 4);
    e->msk = (uint8_t*)e->alloc(M * (K + 1));
    e->row_b = (int*)e->alloc(M * 4);
    e->row_pos = (int*)e->alloc(M * 4);
    e->ptiles = (int2*)e->alloc((M / 64 + (size_t)max_batch + 2) * sizeof(int2));
    e->frame_ctr = (int*)e->alloc(16);
    e->df_gbuf = e->alloc(dec_frame_gbuf_bytes());
    e->df_epoch = (unsigned*)e->alloc(16);
    e->df_err = (int*)e->alloc(16);
    if ((e->wdt == WDT_BF16 || e->wdt == WDT_Q4) && b.hidden == 2048 && b.n_layers == BB_STEP_LAYERS) {
      e->bb_gbuf = e->alloc(bb_step_gbuf_bytes());
      e->bb_epoch = (unsigned*)e->alloc(16);
      e->bb_err = (int*)e->alloc(16);
    }
    (void)Vp;
    (void)B;
    ensure_batch(e.get(), max_batch);
    HIPCHK(hipDeviceSynchronize());
    *out = e.release();
  }
  CSM_CATCH
}

int csm_engine_destroy(csm_engine* e) {
  CSM_TRY { delete e; }
  CSM_CATCH
}

int csm_set_rope_table(csm_engine* e, int which, const float* table, int n_pos, int head_dim) {
  CSM_TRY {
    Stack& s = which == 0 ? e->bb : e->dec;
    if (head_dim != s.d.head_dim || n_pos < s.S_cap) throw CsmError(CSM_ERR_ARG, "rope table shape mismatch");
    HIPCHK(hipSetDevice(e->dev));
    HIPCHK(hipMemcpy(s.rope, table, (size_t)s.S_cap * head_dim * 4, hipMemcpyHostToDevice));
  }
  CSM_CATCH
}

int csm_load_tensor(csm_engine* e, const char* cname, const void* host, int src_dtype, const int64_t* shape,
                    int ndim) {
  CSM_TRY {
    HIPCHK(hipSetDevice(e->dev));
    const std::string name(cname);
    std::vector<int64_t> shp(shape, shape + ndim);
    auto numel = [&]() { int64_t n = 1; for (auto s : shp) n *= s; return (size_t)n; };
    auto expect = [&](std::initializer_list<int64_t> want) {
      if (shp != std::vector<int64_t>(want)) throw CsmError(CSM_ERR_ARG, "shape mismatch for " + name);
    };
    if (name.rfind("decoder.layers.0.", 0) == 0) e->proj_tab_dirty = true;  // feeds the folded layer-0 QKV table
    e->tiled_dirty = true;
    if (e->wdt == WDT_Q4 && load_q4(e, name, host, src_dtype, shp)) return CSM_OK;
    if (src_dtype == CSM_U32) throw CsmError(CSM_ERR_ARG, "packed int4 tensor " + name + " needs a CSM_Q4 engine");
    const size_t es = e->wsz;
    auto conv = [&](size_t n) { return convert_to(host, src_dtype, n, e->wdt); };
    auto conv_f32 = [&](size_t n) { return convert_to(host, src_dtype, n, WDT_F32); };

    // --- stack parameters
    for (int which = 0; which < 2; ++which) {
      Stack& s = which == 0 ? e->bb : e->dec;
      const std::string pre = which == 0 ? "backbone." : "decoder.";
      if (name.rfind(pre, 0) != 0) continue;
      const int D = s.d.hidden, F = s.d.intermediate, hd = s.d.head_dim;
      const int qd = s.q_dim(), kvd = s.d.n_kv_heads * hd;
      if (name == pre + "norm.weight") {
        expect({D});
        auto h = conv_f32(D);
        HIPCHK(hipMemcpy(s.norm, h.data(), D * 4, hipMemcpyHostToDevice));
        e->loaded.insert(name);
        return CSM_OK;
      }
      int li = -1;
      char tail[128] = {0};
      if (sscanf(name.c_str() + pre.size(), "layers.%d.%127s", &li, tail) != 2 || li < 0 || li >= s.d.n_layers)
        throw CsmError(CSM_ERR_ARG, "unknown tensor " + name);
      LayerW& l = s.L[li];
      const std::string t(tail);
      if (t == "self_attn.q_proj.weight") {
        expect({qd, D});
        auto h = conv(numel());
        HIPCHK(hipMemcpy(l.wqkv, h.data(), h.size(), hipMemcpyHostToDevice));
      } else if (t == "self_attn.k_proj.weight" || t == "self_attn.v_proj.weight") {
        expect({kvd, D});
        auto h = conv(numel());
        const size_t row0 = qd + (t[10] == 'k' ? 0 : kvd);
        HIPCHK(hipMemcpy((char*)l.wqkv + row0 * D * es, h.data(), h.size(), hipMemcpyHostToDevice));
      } else if (t == "self_attn.o_proj.weight") {
        expect({D, qd});
        auto h = conv(numel());
        HIPCHK(hipMemcpy(l.wo, h.data(), h.size(), hipMemcpyHostToDevice));
      } else if (t == "mlp.gate_proj.weight" || t == "mlp.up_proj.weight") {
        expect({F, D});
        auto h = conv(numel());
        const size_t off = (t[4] == 'g') ? 0 : 1;  // interleave: row 2j gate, 2j+1 up
        HIPCHK(hipMemcpy2D((char*)l.wgu + off * D * es, 2 * D * es, h.data(), D * es, D * es, F,
                           hipMemcpyHostToDevice));
      } else if (t == "mlp.down_proj.weight") {
        expect({D, F});
        auto h = conv(numel());
        HIPCHK(hipMemcpy(l.wd, h.data(), h.size(), hipMemcpyHostToDevice));
        if (l.wdc) {  // persistent kernels: columns chunk-major [F/R][D][R] (bf16)
          const int R = wdc_chunk(D);
          const uint16_t* src = reinterpret_cast<const uint16_t*>(h.data());
          std::vector<uint16_t> t2((size_t)D * F);
          for (int c = 0; c < F / R; ++c)
            for (int n = 0; n < D; ++n)
              memcpy(&t2[((size_t)c * D + n) * R], src + (size_t)n * F + (size_t)c * R, R * 2);
          HIPCHK(hipMemcpy(l.wdc, t2.data(), t2.size() * 2, hipMemcpyHostToDevice));
        }
      } else if (t == "input_layernorm.weight" || t == "post_attention_layernorm.weight") {
        expect({D});
        auto h = conv_f32(D);
        HIPCHK(hipMemcpy(t[0] == 'i' ? l.n1 : l.n2, h.data(), D * 4, hipMemcpyHostToDevice));
      } else {
        throw CsmError(CSM_ERR_ARG, "unknown tensor " + name);
      }
      e->loaded.insert(name);
      return CSM_OK;
    }
    const int64_t D = e->D, Dd = e->Dd, V = e->V, K = e->K, Vp = e->Vpad;
    if (name == "text_embeddings.weight") {
      expect({e->dims.n_text_vocab, D});
      auto h = conv(numel());
      HIPCHK(hipMemcpy(e->text_emb, h.data(), h.size(), hipMemcpyHostToDevice));
    } else if (name == "audio_embeddings.weight") {
      e->proj_tab_dirty = true;
      expect({V * K, D});
      auto h = conv(numel());
      HIPCHK(hipMemcpy(e->audio_emb, h.data(), h.size(), hipMemcpyHostToDevice));
    } else if (name == "projection.weight") {
      e->proj_tab_dirty = true;
      expect({Dd, D});
      auto h = conv(numel());
      HIPCHK(hipMemcpy(e->proj, h.data(), h.size(), hipMemcpyHostToDevice));
    } else if (name == "codebook0_head.weight") {
      expect({V, D});
      auto h = conv(numel());  // rows V..Vpad stay zero (padding)
      HIPCHK(hipMemcpy(e->c0_head, h.data(), h.size(), hipMemcpyHostToDevice));
    } else if (name == "audio_head") {
      expect({K - 1, Dd, V});
      // (in,out) layout -> per-codebook (out,in) GEMV rows: [K-1][Vpad][Dd]
      auto f = conv_f32(numel());
      const float* src = reinterpret_cast<const float*>(f.data());
      std::vector<float> t((size_t)(K - 1) * Vp * Dd, 0.f);
      for (int64_t c = 0; c < K - 1; ++c)
        for (int64_t i = 0; i < Dd; ++i)
          for (int64_t v = 0; v < V; ++v) t[((size_t)c * Vp + v) * Dd + i] = src[((size_t)c * Dd + i) * V + v];
      auto h = convert_to(t.data(), CSM_F32, t.size(), e->head_wdt);
      HIPCHK(hipMemcpy(e->audio_head, h.data(), h.size(), hipMemcpyHostToDevice));
    } else {
      throw CsmError(CSM_ERR_ARG, "unknown tensor " + name);
    }
    e->loaded.insert(name);
  }
  CSM_CATCH
}

int csm_weights_ready(csm_engine* e) {
  CSM_TRY {
    for (const auto& n : e->required)
      if (!e->loaded.count(n)) throw CsmError(CSM_ERR_STATE, "missing weight " + n);
  }
  CSM_CATCH
}

// resident weight buffers in a fixed order (identical across engines of the same dims / dtype)
static std::vector<std::pair<void*, size_t>> weight_buffers(csm_engine* e) {
  std::vector<std::pair<void*, size_t>> b;
  for (Stack* s : {&e->bb, &e->dec}) {
    const size_t D = s->d.hidden, F = s->d.intermediate;
    b.emplace_back(s->norm, D * 4);
    for (LayerW& l : s->L) {
      b.emplace_back(l.wqkv, e->wbytes(s->qkv_rows(), D));
      b.emplace_back(l.wo, e->wbytes(D, s->q_dim()));
      b.emplace_back(l.wgu, e->wbytes(2 * F, D));
      b.emplace_back(l.wd, e->wbytes(D, F));
      if (l.wdc) b.emplace_back(l.wdc, D * F * 2);
      b.emplace_back(l.n1, D * 4);
      b.emplace_back(l.n2, D * 4);
    }
  }
  const size_t D = e->D, Dd = e->Dd, V = e->V, K = e->K, Vp = e->Vpad;
  b.emplace_back(e->text_emb, e->wbytes(e->dims.n_text_vocab, D));
  b.emplace_back(e->audio_emb, e->wbytes(V * K, D));
  b.emplace_back(e->proj, e->wbytes(Dd, D));
  b.emplace_back(e->c0_head, e->wbytes(Vp, D));
  b.emplace_back(e->audio_head, (K - 1) * Vp * Dd * (e->head_wdt == WDT_F32 ? 4 : 2));
  return b;
}

int csm_weight_buffers(csm_engine* e, void** ptrs, uint64_t* bytes, int cap, int* n) {
  CSM_TRY {
    if (!e || !n || cap < 0) throw CsmError(CSM_ERR_ARG, "bad csm_weight_buffers arguments");
    const auto b = weight_buffers(e);
    *n = (int)b.size();
    for (int i = 0; i < cap && i < (int)b.size(); ++i) {
      if (ptrs) ptrs[i] = b[i].first;
      if (bytes) bytes[i] = b[i].second;
    }
  }
  CSM_CATCH
}

int csm_weights_received(csm_engine* e) {
  CSM_TRY {
    HIPCHK(hipSetDevice(e->dev));
    HIPCHK(hipDeviceSynchronize());
    for (const auto& nm : e->required) e->loaded.insert(nm);
    e->tiled_dirty = true;
    e->proj_tab_dirty = true;
    e->g_B = -1;
  }
  CSM_CATCH
}

int csm_quantize(csm_engine* e, int group_size, int bits) {
  CSM_TRY {
    if (group_size != Q4_GROUP || bits != 4) throw CsmError(CSM_ERR_ARG, "only group_size=64, bits=4 is supported");
    if (e->wdt == WDT_Q4) return CSM_OK;  // already quantized (nn.quantize on a quantized model is a no-op here)
    HIPCHK(hipSetDevice(e->dev));
    HIPCHK(hipDeviceSynchronize());
    const int old = e->wdt;
    const size_t old_es = e->wsz;
    // every Linear / Embedding matrix, whole (all rows of fused / interleaved layouts): row order kept
    std::vector<std::tuple<void**, int, int>> mats;
    for (Stack* s : {&e->bb, &e->dec})
      for (LayerW& l : s->L) {
        const int D = s->d.hidden, F = s->d.intermediate;
        mats.emplace_back(&l.wqkv, s->qkv_rows(), D);
        mats.emplace_back(&l.wo, D, s->q_dim());
        mats.emplace_back(&l.wgu, 2 * F, D);
        mats.emplace_back(&l.wd, D, F);
      }
    mats.emplace_back(&e->text_emb, e->dims.n_text_vocab, e->D);
    mats.emplace_back(&e->audio_emb, e->V * e->K, e->D);
    mats.emplace_back(&e->proj, e->Dd, e->D);
    mats.emplace_back(&e->c0_head, e->Vpad, e->D);
    for (auto& [pp, N, Kd] : mats)
      if (!gemv_q4_supported(N, Kd)) throw CsmError(CSM_ERR_ARG, "int4 GEMV does not support this shape");
    // the bf16 chunk-major down_proj copies serve only the bf16 persistent kernels: freed, so an
    // nn.quantize'd engine lists the same weight buffers as one created as CSM_Q4 (csm_weight_buffers)
    for (Stack* s : {&e->bb, &e->dec})
      for (LayerW& l : s->L)
        if (l.wdc) { e->release(l.wdc); l.wdc = nullptr; }
    for (auto& [pp, N, Kd] : mats) {
      void* q = e->alloc(q4_bytes(N, Kd));
      launch_q4_quantize(*pp, old, N, Kd, q, N, 0, 1, e->st);
      HIPCHK(hipStreamSynchronize(e->st));
      HIPCHK(hipGetLastError());
      e->release(*pp);
      *pp = q;
    }
    (void)old_es;
    e->head_wdt = old;
    e->wdt = WDT_Q4;
    e->proj_tab_dirty = true;
    for (void* t : e->tiled_bufs) e->release(t);  // re-sized for int4 at the next csm_begin
    e->tiled_bufs.clear();
    e->ws.tiled.clear();
    e->tiled_dirty = true;
    e->g_B = -1;
  }
  CSM_CATCH
}

int csm_begin(csm_engine* e, int B, const uint64_t* seeds, float temperature, int top_k) {
  CSM_TRY {
    e->c0_pending = false;
    if (e->ahead_pending) {  // the last chunk's pinned copies land before the slots are reused
      HIPCHK(hipStreamSynchronize(e->st));
      e->ahead_pending = false;
    }
    if (B <= 0) throw CsmError(CSM_ERR_ARG, "batch size out of range");
    if (temperature < 0.f) throw CsmError(CSM_ERR_ARG, "temperature must be >= 0");
    HIPCHK(hipSetDevice(e->dev));
    ensure_batch(e, B);
    if (e->tiled_dirty) build_tiled(e);
    if (e->proj_tab_dirty) build_proj_table(e);
    e->pos_host.assign(B, -1);
    e->B = B;
    e->temperature = temperature;
    e->top_k = top_k;
    e->use_top_p = e->use_min_p = 0;
    e->min_keep = 1;
    e->top_p_cut = e->log_min_p = 0.f;
    ++e->filters_id;
    e->frames_run = 0;
    e->need_body = false;
    e->prompt_len.assign(B, -1);
    std::vector<uint64_t> s(B, 0);
    if (seeds) memcpy(s.data(), seeds, B * 8);
    HIPCHK(hipMemcpyAsync(e->seeds, s.data(), B * 8, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipMemsetAsync(e->done, 0, B, e->st));
    HIPCHK(hipMemsetAsync(e->n_frames, 0, B * 4, e->st));
    HIPCHK(hipMemsetAsync(e->frame_ctr, 0, 16, e->st));
    HIPCHK(hipMemsetAsync(e->codes, 0, (size_t)B * e->K * 4, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
  }
  CSM_CATCH
}

int csm_set_sampler_filters(csm_engine* e, double top_p, double min_p, int min_tokens_to_keep) {
  CSM_TRY {
    if (!e) throw CsmError(CSM_ERR_ARG, "null engine");
    if (e->frames_run > 0 || e->c0_pending) throw CsmError(CSM_ERR_STATE, "set the sampler filters before the first frame");
    if (!(top_p >= 0.0 && top_p <= 1.0) || !(min_p >= 0.0 && min_p <= 1.0) || min_tokens_to_keep < 1)
      throw CsmError(CSM_ERR_ARG, "top_p and min_p must lie in [0, 1], min_tokens_to_keep >= 1");
    // mlx_lm make_sampler: top_p active in (0, 1), min_p when != 0; the cuts are the float32 values
    // its comparisons use: 1 - top_p and log(min_p) evaluated in double, then rounded
    e->use_top_p = top_p > 0.0 && top_p < 1.0;
    e->use_min_p = min_p != 0.0;
    e->top_p_cut = (float)(1.0 - top_p);
    e->log_min_p = e->use_min_p ? (float)std::log(min_p) : 0.f;
    e->min_keep = min_tokens_to_keep;
    ++e->filters_id;
  }
  CSM_CATCH
}

int csm_prefill(csm_engine* e, int b, int T, const int32_t* tokens, const uint8_t* mask) {
  CSM_TRY {
    if (b < 0 || b >= e->B) throw CsmError(CSM_ERR_ARG, "utterance index out of range");
    if (T <= 0 || T > e->M_cap) throw CsmError(CSM_ERR_ARG, "prompt length out of range");
    const int start = e->pos_host[b] + 1;  // rows append after what the backbone already holds
    if (start + T > e->dims.max_seq_len)
      throw CsmError(CSM_ERR_TOO_LONG, "rows exceed the 2048-position window");
    HIPCHK(hipSetDevice(e->dev));
    const int K = e->K;
    HIPCHK(hipMemcpyAsync(e->tok, tokens, (size_t)T * (K + 1) * 4, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipMemcpyAsync(e->msk, mask, (size_t)T * (K + 1), hipMemcpyHostToDevice, e->st));
    EmbedParams ep{};
    ep.tok = e->tok; ep.mask = e->msk; ep.text_emb = e->text_emb; ep.audio_emb = e->audio_emb; ep.V = e->V;
    ep.K = K; ep.D = e->D; ep.out = e->x;
    embed(e, ep, T, e->st);
    RowMap rm{T, b, nullptr, start};
    if (e->attn_tiles_on && T >= 16) {  // attention tiles: <= 64 consecutive rows (launch_attn's >= 16-row bar)
      // staged in pinned memory: the copy stays asynchronous (this call's closing synchronize is what
      // makes the staging reusable by the next csm_prefill)
      const int nt = (T + 63) / 64;
      if (!e->ptiles_pin) HIPCHK(hipHostMalloc((void**)&e->ptiles_pin, (e->M_cap / 64 + 1) * sizeof(int2), hipHostMallocDefault));
      for (int t = 0; t < nt; ++t) e->ptiles_pin[t] = make_int2(64 * t, std::min(64, T - 64 * t));
      HIPCHK(hipMemcpyAsync(e->ptiles, e->ptiles_pin, nt * sizeof(int2), hipMemcpyHostToDevice, e->st));
      rm.tiles = e->ptiles;
      rm.ntiles = nt;
    }
    run_stack(e, e->bb, e->x, T, e->q, e->att, e->mlp, rm, e->st);
    launch_rmsnorm_rows(e->x + (size_t)(T - 1) * e->D, e->D, e->bb.norm, e->bb.d.eps, e->D,
                        e->h_last + (size_t)b * e->D, e->D, 1, e->st);
    e->pos_host[b] = start + T - 1;  // position of the last processed backbone row
    HIPCHK(hipMemcpyAsync(e->pos + b, &e->pos_host[b], 4, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    HIPCHK(hipGetLastError());
    e->prompt_len[b] = std::max(e->prompt_len[b], 0) + T;
    e->need_body = false;
  }
  CSM_CATCH
}

int csm_prefill_batch(csm_engine* e, int n, const int32_t* utts, const int32_t* Ts, const int32_t* tokens,
                      const uint8_t* masks) {
  CSM_TRY {
    if (n <= 0 || !utts || !Ts || !tokens || !masks) throw CsmError(CSM_ERR_ARG, "bad csm_prefill_batch arguments");
    const int K = e->K;
    std::vector<int> start(n);
    std::vector<size_t> row0(n + 1, 0);
    std::vector<char> seen(e->B, 0);
    for (int i = 0; i < n; ++i) {
      const int b = utts[i], T = Ts[i];
      if (b < 0 || b >= e->B || seen[b]) throw CsmError(CSM_ERR_ARG, "utterance index out of range or repeated");
      seen[b] = 1;
      if (T <= 0 || T > e->M_cap) throw CsmError(CSM_ERR_ARG, "prompt length out of range");
      start[i] = e->pos_host[b] + 1;
      if (start[i] + T > e->dims.max_seq_len) throw CsmError(CSM_ERR_TOO_LONG, "rows exceed the 2048-position window");
      row0[i + 1] = row0[i] + T;
    }
    HIPCHK(hipSetDevice(e->dev));
    const size_t cap = e->prefill_rows > 0 ? std::min(e->prefill_rows, e->M_cap) : e->M_cap;
    // utterances in groups of at most M_cap rows: one pass of every projection per group (the
    // weights stream once for all of the group's rows), rows mapped to (utterance, position)
    std::vector<int> rb, rp;
    std::vector<int2> tl;
    for (int i0 = 0; i0 < n;) {
      int i1 = i0;
      while (i1 < n && row0[i1 + 1] - row0[i0] <= cap) ++i1;
      if (i1 == i0) i1 = i0 + 1;  // one utterance longer than a lowered cap: a group of its own (T <= M_cap)
      const int R = (int)(row0[i1] - row0[i0]);
      rb.assign(R, 0);
      rp.assign(R, 0);
      for (int i = i0; i < i1; ++i)
        for (int t = 0; t < Ts[i]; ++t) {
          rb[row0[i] - row0[i0] + t] = utts[i];
          rp[row0[i] - row0[i0] + t] = start[i] + t;
        }
      HIPCHK(hipMemcpyAsync(e->tok, tokens + row0[i0] * (K + 1), (size_t)R * (K + 1) * 4, hipMemcpyHostToDevice, e->st));
      HIPCHK(hipMemcpyAsync(e->msk, masks + row0[i0] * (K + 1), (size_t)R * (K + 1), hipMemcpyHostToDevice, e->st));
      HIPCHK(hipMemcpyAsync(e->row_b, rb.data(), (size_t)R * 4, hipMemcpyHostToDevice, e->st));
      HIPCHK(hipMemcpyAsync(e->row_pos, rp.data(), (size_t)R * 4, hipMemcpyHostToDevice, e->st));
      tl.clear();  // attention tiles: <= 64 consecutive rows of one utterance
      for (int i = i0; i < i1; ++i)
        for (int t0 = 0; t0 < Ts[i]; t0 += 64) tl.push_back(make_int2((int)(row0[i] - row0[i0]) + t0, std::min(64, Ts[i] - t0)));
      HIPCHK(hipMemcpyAsync(e->ptiles, tl.data(), tl.size() * sizeof(int2), hipMemcpyHostToDevice, e->st));
      EmbedParams ep{};
      ep.tok = e->tok; ep.mask = e->msk; ep.text_emb = e->text_emb; ep.audio_emb = e->audio_emb; ep.V = e->V;
      ep.K = K; ep.D = e->D; ep.out = e->x;
      embed(e, ep, R, e->st);
      RowMap rm{1, 0, nullptr, 0};
      rm.row_b = e->row_b;
      rm.row_pos = e->row_pos;
      if (e->attn_tiles_on) {
        rm.tiles = e->ptiles;
        rm.ntiles = (int)tl.size();
      }
      run_stack(e, e->bb, e->x, R, e->q, e->att, e->mlp, rm, e->st);
      for (int i = i0; i < i1; ++i) {  // h_last = norm(last row) of each utterance
        const size_t last = row0[i + 1] - 1 - row0[i0];
        launch_rmsnorm_rows(e->x + last * e->D, e->D, e->bb.norm, e->bb.d.eps, e->D, e->h_last + (size_t)utts[i] * e->D,
                            e->D, 1, e->st);
      }
      HIPCHK(hipStreamSynchronize(e->st));  // the host row tables are reused by the next group
      HIPCHK(hipGetLastError());
      i0 = i1;
    }
    for (int i = 0; i < n; ++i) {
      const int b = utts[i];
      e->pos_host[b] = start[i] + Ts[i] - 1;
      HIPCHK(hipMemcpyAsync(e->pos + b, &e->pos_host[b], 4, hipMemcpyHostToDevice, e->st));
      e->prompt_len[b] = std::max(e->prompt_len[b], 0) + Ts[i];
    }
    HIPCHK(hipStreamSynchronize(e->st));
    e->need_body = false;
  }
  CSM_CATCH
}

int csm_run_frames(csm_engine* e, int nframes, int* all_done) {
  CSM_TRY {
    if (e->c0_pending) throw CsmError(CSM_ERR_STATE, "csm_frame_finish pending");
    for (int b = 0; b < e->B; ++b)
      if (e->prompt_len[b] < 0) throw CsmError(CSM_ERR_STATE, "csm_prefill not called for every utterance");
    HIPCHK(hipSetDevice(e->dev));
    if (e->frames_run + nframes > e->F_cap) nframes = e->F_cap - e->frames_run;
    int maxpos = 0;
    for (int b = 0; b < e->B; ++b) maxpos = std::max(maxpos, e->pos_host[b]);
    if (maxpos + nframes + (e->need_body ? 1 : 0) > e->dims.max_seq_len)
      throw CsmError(CSM_ERR_TOO_LONG, "frames exceed the 2048-position window");
    if (nframes <= 0) { if (all_done) *all_done = 0; return CSM_OK; }
    // CSM_GRAPH=0: eager launches of the same kernels (rocprofv3 kernel tracing of graph
    // replays crashes on ROCm 7.2, so profiling runs use this mode).
    static const bool use_graph = [] {
      const char* v = getenv("CSM_GRAPH");
      return !(v && v[0] == '0');
    }();
    if (!use_graph) {
      for (int f = 0; f < nframes; ++f) {
        if (e->need_body) {
          enqueue_body(e, e->st);
          for (int b = 0; b < e->B; ++b) e->pos_host[b] += 1;
        }
        enqueue_head(e, e->st);
        e->need_body = true;
        e->frames_run++;
      }
      HIPCHK(hipGetLastError());
      nframes = 0;
    }
    if (use_graph && (e->g_B != e->B || e->g_temp != e->temperature || e->g_topk != e->top_k ||
                      e->g_filters != e->filters_id || !e->g_head)) {
      if (e->g_body) (void)hipGraphExecDestroy(e->g_body);
      if (e->g_head) (void)hipGraphExecDestroy(e->g_head);
      e->g_body = capture(e, enqueue_body);
      e->g_head = capture(e, enqueue_head);
      e->g_B = e->B;
      e->g_temp = e->temperature;
      e->g_topk = e->top_k;
      e->g_filters = e->filters_id;
    }
    for (int f = 0; f < nframes; ++f) {
      if (e->need_body) {
        HIPCHK(hipGraphLaunch(e->g_body, e->st));
        for (int b = 0; b < e->B; ++b) e->pos_host[b] += 1;
      }
      HIPCHK(hipGraphLaunch(e->g_head, e->st));
      e->need_body = true;
      e->frames_run++;
    }
    if (all_done) {
      std::vector<uint8_t> d(e->B);
      HIPCHK(hipMemcpyAsync(d.data(), e->done, e->B, hipMemcpyDeviceToHost, e->st));
      HIPCHK(hipStreamSynchronize(e->st));
      check_dec_frame(e);
      int all = 1;
      for (auto v : d) all &= (v != 0);
      *all_done = all;
    }
  }
  CSM_CATCH
}

int csm_run_frames_ahead(csm_engine* e, int nframes, int* prev_all_done) {
  if (!e || !prev_all_done) { csm_set_error("null engine or result pointer"); return CSM_ERR_ARG; }
  const int rc = csm_run_frames(e, nframes, nullptr);  // enqueued, no wait
  if (rc != CSM_OK) return rc;
  CSM_TRY {
    if (!e->ahead_pin) {
      HIPCHK(hipHostMalloc((void**)&e->ahead_pin, 2 * e->ahead_bytes(), hipHostMallocDefault));
      for (hipEvent_t& ev : e->ahead_ev) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    const int s = e->ahead_slot;
    uint8_t* pin = e->ahead_pin + s * e->ahead_bytes();
    int* perr = reinterpret_cast<int*>(pin + e->ahead_bytes() - 8);
    perr[0] = perr[1] = 0;  // (slot s was last read two chunks ago, after its event)
    HIPCHK(hipMemcpyAsync(pin, e->done, e->B, hipMemcpyDeviceToHost, e->st));
    if (e->df_err) HIPCHK(hipMemcpyAsync(perr, e->df_err, 4, hipMemcpyDeviceToHost, e->st));
    if (e->bb_err) HIPCHK(hipMemcpyAsync(perr + 1, e->bb_err, 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipEventRecord(e->ahead_ev[s], e->st));
    int res = -1;
    if (e->ahead_pending) {
      const int q = s ^ 1;
      HIPCHK(hipEventSynchronize(e->ahead_ev[q]));
      const uint8_t* pq = e->ahead_pin + q * e->ahead_bytes();
      const int* qerr = reinterpret_cast<const int*>(pq + e->ahead_bytes() - 8);
      if (qerr[0] || qerr[1]) {
        // the chunk just enqueued has written slot s behind its event: drain the stream and forget both
        // slots, so a later call (with or without csm_begin) never polls a stale done state
        HIPCHK(hipStreamSynchronize(e->st));
        e->ahead_pending = false;
        e->ahead_slot = 0;
        check_dec_frame(e);  // resets the device flags and raises
      }
      res = 1;
      for (int b = 0; b < e->B; ++b) res &= pq[b] != 0;
    }
    e->ahead_slot = s ^ 1;
    e->ahead_pending = true;
    *prev_all_done = res;
  }
  CSM_CATCH
}

int csm_frame_step(csm_engine* e, int32_t* out_codes, uint8_t* done) {
  if (!e) { csm_set_error("null engine"); return CSM_ERR_ARG; }
  if (e->frames_run >= e->F_cap) { csm_set_error("frame capacity reached"); return CSM_ERR_STATE; }
  const int rc = csm_run_frames(e, 1, nullptr);
  if (rc != CSM_OK) return rc;
  CSM_TRY {
    if (out_codes)
      HIPCHK(hipMemcpyAsync(out_codes, e->codes, (size_t)e->B * e->K * 4, hipMemcpyDeviceToHost, e->st));
    if (done) HIPCHK(hipMemcpyAsync(done, e->done, e->B, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    check_dec_frame(e);
  }
  CSM_CATCH
}

// One frame in two halves around a host hook on the c0 logits (generation.py:42-49): eager launches
// of the same kernels the frame graph holds.
int csm_frame_c0_logits(csm_engine* e, float* logits) {
  CSM_TRY {
    for (int b = 0; b < e->B; ++b)
      if (e->prompt_len[b] < 0) throw CsmError(CSM_ERR_STATE, "csm_prefill not called for every utterance");
    if (e->c0_pending) throw CsmError(CSM_ERR_STATE, "csm_frame_c0_logits called again before csm_frame_finish");
    if (!logits) throw CsmError(CSM_ERR_ARG, "null logits buffer");
    HIPCHK(hipSetDevice(e->dev));
    if (e->frames_run + 1 > e->F_cap) throw CsmError(CSM_ERR_STATE, "frame capacity reached");
    int maxpos = 0;
    for (int b = 0; b < e->B; ++b) maxpos = std::max(maxpos, e->pos_host[b]);
    if (maxpos + 1 + (e->need_body ? 1 : 0) > e->dims.max_seq_len)
      throw CsmError(CSM_ERR_TOO_LONG, "frames exceed the 2048-position window");
    if (e->need_body) {
      enqueue_body(e, e->st);
      for (int b = 0; b < e->B; ++b) e->pos_host[b] += 1;
      e->need_body = false;
    }
    enqueue_head_phase(e, e->st, 1);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy2DAsync(logits, (size_t)e->V * 4, e->c0_logits, (size_t)e->Vpad * 4, (size_t)e->V * 4, e->B,
                            hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    check_dec_frame(e);  // the backbone row may have run on the persistent step
    e->c0_pending = true;
    e->host_piece = 1;
  }
  CSM_CATCH
}

int csm_frame_finish(csm_engine* e, const float* logits, int* all_done) {
  CSM_TRY {
    if (!e->c0_pending) throw CsmError(CSM_ERR_STATE, "csm_frame_finish without csm_frame_c0_logits");
    if (!logits) throw CsmError(CSM_ERR_ARG, "null logits buffer");
    HIPCHK(hipSetDevice(e->dev));
    HIPCHK(hipMemcpy2DAsync(e->c0_logits, (size_t)e->Vpad * 4, logits, (size_t)e->V * 4, (size_t)e->V * 4, e->B,
                            hipMemcpyHostToDevice, e->st));
    enqueue_head_phase(e, e->st, 2);
    HIPCHK(hipGetLastError());
    e->c0_pending = false;
    e->need_body = true;
    e->frames_run++;
    if (all_done) {
      std::vector<uint8_t> d(e->B);
      HIPCHK(hipMemcpyAsync(d.data(), e->done, e->B, hipMemcpyDeviceToHost, e->st));
      HIPCHK(hipStreamSynchronize(e->st));
      int all = 1;
      for (auto v : d) all &= (v != 0);
      *all_done = all;
    } else {
      HIPCHK(hipStreamSynchronize(e->st));  // the host logits buffer may be released on return
    }
    check_dec_frame(e);
  }
  CSM_CATCH
}

int csm_frame_host_step(csm_engine* e, const int32_t* codes, float* logits, int* all_done) {
  CSM_TRY {
    if (!e->c0_pending) throw CsmError(CSM_ERR_STATE, "csm_frame_host_step without csm_frame_c0_logits");
    if (!codes) throw CsmError(CSM_ERR_ARG, "null codes");
    const int piece = e->host_piece;  // codes are those of codebook piece - 1
    if (piece < e->K && !logits) throw CsmError(CSM_ERR_ARG, "null logits buffer");
    for (int b = 0; b < e->B; ++b)
      if (codes[b] < 0 || codes[b] >= e->V) throw CsmError(CSM_ERR_ARG, "host-sampled code out of range");
    HIPCHK(hipSetDevice(e->dev));
    HIPCHK(hipMemcpy2DAsync(e->force + (piece - 1), (size_t)e->K * 4, codes, 4, 4, e->B, hipMemcpyHostToDevice, e->st));
    enqueue_head_phase(e, e->st, 4, piece);
    HIPCHK(hipGetLastError());
    if (piece < e->K) {
      HIPCHK(hipMemcpy2DAsync(logits, (size_t)e->V * 4, e->ci_logits + (size_t)(piece - 1) * e->B * e->Vpad,
                              (size_t)e->Vpad * 4, (size_t)e->V * 4, e->B, hipMemcpyDeviceToHost, e->st));
      HIPCHK(hipStreamSynchronize(e->st));
      e->host_piece = piece + 1;
      if (all_done) *all_done = 0;
    } else {
      e->c0_pending = false;
      e->host_piece = 1;
      e->need_body = true;
      e->frames_run++;
      std::vector<uint8_t> d(e->B);
      HIPCHK(hipMemcpyAsync(d.data(), e->done, e->B, hipMemcpyDeviceToHost, e->st));
      HIPCHK(hipStreamSynchronize(e->st));
      int all = 1;
      for (auto v : d) all &= (v != 0);
      if (all_done) *all_done = all;
    }
    check_dec_frame(e);
  }
  CSM_CATCH
}

int csm_frame_forced(csm_engine* e, const int32_t* codes, float* c0_logits, float* ci_logits, float* ce) {
  CSM_TRY {
    for (int b = 0; b < e->B; ++b)
      if (e->prompt_len[b] < 0) throw CsmError(CSM_ERR_STATE, "csm_prefill not called for every utterance");
    if (e->c0_pending) throw CsmError(CSM_ERR_STATE, "csm_frame_finish pending");
    if (!codes) throw CsmError(CSM_ERR_ARG, "null codes");
    HIPCHK(hipSetDevice(e->dev));
    if (e->frames_run + 1 > e->F_cap) throw CsmError(CSM_ERR_STATE, "frame capacity reached");
    int maxpos = 0;
    for (int b = 0; b < e->B; ++b) maxpos = std::max(maxpos, e->pos_host[b]);
    if (maxpos + 1 + (e->need_body ? 1 : 0) > e->dims.max_seq_len)
      throw CsmError(CSM_ERR_TOO_LONG, "frames exceed the 2048-position window");
    for (int i = 0; i < e->B * e->K; ++i)
      if (codes[i] < 0 || codes[i] >= e->V) throw CsmError(CSM_ERR_ARG, "forced code out of range");
    HIPCHK(hipMemcpyAsync(e->force, codes, (size_t)e->B * e->K * 4, hipMemcpyHostToDevice, e->st));
    if (e->need_body) {
      enqueue_body(e, e->st);
      for (int b = 0; b < e->B; ++b) e->pos_host[b] += 1;
    }
    enqueue_head_phase(e, e->st, 3);
    if (ce) launch_forced_ce(e->c0_logits, e->ci_logits, e->force, e->force_ce, e->B, e->K, e->V, e->Vpad, e->st);
    HIPCHK(hipGetLastError());
    e->need_body = true;
    e->frames_run++;
    const size_t V = e->V, Vp = e->Vpad, B = e->B;
    if (c0_logits)
      HIPCHK(hipMemcpy2DAsync(c0_logits, V * 4, e->c0_logits, Vp * 4, V * 4, B, hipMemcpyDeviceToHost, e->st));
    if (ci_logits)
      HIPCHK(hipMemcpy2DAsync(ci_logits, V * 4, e->ci_logits, Vp * 4, V * 4, (size_t)(e->K - 1) * B,
                              hipMemcpyDeviceToHost, e->st));
    if (ce) HIPCHK(hipMemcpyAsync(ce, e->force_ce, B * e->K * 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    check_dec_frame(e);  // the backbone row may have run on the persistent step
  }
  CSM_CATCH
}

int csm_read_codes(csm_engine* e, int32_t* hist, int32_t* n_frames, uint8_t* done, int* frames_run) {
  CSM_TRY {
    HIPCHK(hipSetDevice(e->dev));
    HIPCHK(hipStreamSynchronize(e->st));
    check_dec_frame(e);
    if (hist)
      HIPCHK(hipMemcpy(hist, e->hist, (size_t)e->frames_run * e->B * e->K * 4, hipMemcpyDeviceToHost));
    if (n_frames) HIPCHK(hipMemcpy(n_frames, e->n_frames, e->B * 4, hipMemcpyDeviceToHost));
    if (done) HIPCHK(hipMemcpy(done, e->done, e->B, hipMemcpyDeviceToHost));
    if (frames_run) *frames_run = e->frames_run;
  }
  CSM_CATCH
}

int csm_debug_read(csm_engine* e, const char* what, void* host, int64_t nbytes, int64_t* needed) {
  CSM_TRY {
    HIPCHK(hipSetDevice(e->dev));
    HIPCHK(hipStreamSynchronize(e->st));
    const std::string w(what);
    const void* src = nullptr;
    size_t n = 0;
    const size_t B = e->B, Vp = e->Vpad;
    if (w == "h_last") { src = e->h_last; n = B * e->D * 4; }
    else if (w == "c0_logits") { src = e->c0_logits; n = B * Vp * 4; }
    else if (w == "ci_logits") { src = e->ci_logits; n = (e->K - 1) * B * Vp * 4; }
    else if (w == "codes") { src = e->codes; n = B * e->K * 4; }
    else if (w == "pos") { src = e->pos; n = B * 4; }
    else if (w == "dec_frame_epoch") { src = e->df_epoch; n = 4; }
    else if (w == "dec_xsd_epoch") { src = e->xsd_epoch; n = 4; }
    else if (w == "dec_xsd_stamps" && e->xsd_stamps) { src = e->xsd_stamps; n = (size_t)DEC_XSD_WGS * DEC_XSD_STAMPS * 8; }
    else if (w == "bb_step_epoch" && e->bb_epoch) { src = e->bb_epoch; n = 4; }  // advances by 80 per row it ran
    else if (w == "bb_step_stamps" && e->bb_stamps) { src = e->bb_stamps; n = (size_t)BB_STEP_WGS * BB_STEP_STAMPS * 8; }  // advances by the hand-offs of every frame it ran
    else if (w == "dec_frame_stamps" && e->df_stamps) { src = e->df_stamps; n = (size_t)DEC_FRAME_WGS * DEC_FRAME_STAMPS * 8; }
    else if (w == "audio_head") {  // device layout [K-1][Vpad][Dd], f32 or bf16 bits
      src = e->audio_head; n = (size_t)(e->K - 1) * Vp * e->Dd * (e->head_wdt == WDT_F32 ? 4 : 2);
    }
    else if (w.rfind("weight:", 0) == 0) {  // a whole stored matrix in its device layout (not fused ones)
      Place pl;
      if (!weight_place(e, w.substr(7), pl) || pl.n != pl.Ntot) throw CsmError(CSM_ERR_ARG, "no whole matrix " + w);
      src = pl.base;
      n = e->wbytes(pl.Ntot, pl.K);
    }
    else throw CsmError(CSM_ERR_ARG, "unknown debug tap " + w);
    if (needed) *needed = (int64_t)n;
    if (host) {
      if ((size_t)nbytes < n) throw CsmError(CSM_ERR_ARG, "debug buffer too small");
      HIPCHK(hipMemcpy(host, src, n, hipMemcpyDeviceToHost));
    }
  }
  CSM_CATCH
}

int csm_read_rows(csm_engine* e, const char* name, int n, const int32_t* rows, float* out) {
  CSM_TRY {
    if (!name || n < 0 || (n > 0 && (!rows || !out))) throw CsmError(CSM_ERR_ARG, "bad csm_read_rows arguments");
    Place pl;
    if (!weight_place(e, name, pl)) throw CsmError(CSM_ERR_ARG, std::string("not a Linear / Embedding weight: ") + name);
    if (!e->loaded.count(name)) throw CsmError(CSM_ERR_STATE, std::string("weight not loaded: ") + name);
    std::vector<int> idx(n);
    for (int i = 0; i < n; ++i) {
      if (rows[i] < 0 || rows[i] >= pl.n) throw CsmError(CSM_ERR_ARG, "row index out of range");
      idx[i] = pl.row0 + rows[i] * pl.rstep;
    }
    if (n == 0) return CSM_OK;
    HIPCHK(hipSetDevice(e->dev));
    DevBuf di((size_t)n * 4), dout((size_t)n * pl.K * 4);
    HIPCHK(hipMemcpyAsync(di.p, idx.data(), (size_t)n * 4, hipMemcpyHostToDevice, e->st));
    launch_table_rows(pl.base, e->wdt, pl.Ntot, pl.K, (const int*)di.p, n, (float*)dout.p, e->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, dout.p, (size_t)n * pl.K * 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
  }
  CSM_CATCH
}

int csm_linear(csm_engine* e, const char* name, int M, const float* x, float* y) {
  CSM_TRY {
    if (!name || M <= 0 || !x || !y) throw CsmError(CSM_ERR_ARG, "bad csm_linear arguments");
    const std::string nm(name);
    const void* W = nullptr;
    int wdt = e->wdt, N = 0, K = 0, row0 = 0, rstep = 1, n_out = 0;
    if (nm.rfind("audio_head.", 0) == 0) {  // audio_head[i] (in, out): x @ audio_head[i] (generation.py:79)
      char* end = nullptr;
      const long i = strtol(nm.c_str() + 11, &end, 10);
      if (!end || *end || i < 0 || i >= e->K - 1) throw CsmError(CSM_ERR_ARG, "audio_head index out of range");
      if (!e->loaded.count("audio_head")) throw CsmError(CSM_ERR_STATE, "weight not loaded: audio_head");
      wdt = e->head_wdt;
      W = (const char*)e->audio_head + (size_t)i * e->Vpad * e->Dd * (wdt == WDT_F32 ? 4 : 2);
      N = e->Vpad; K = e->Dd; n_out = e->V;
    } else {
      Place pl;
      if (!weight_place(e, nm, pl) || nm.find("embeddings") != std::string::npos)
        throw CsmError(CSM_ERR_ARG, "not a Linear weight: " + nm);
      if (!e->loaded.count(nm)) throw CsmError(CSM_ERR_STATE, "weight not loaded: " + nm);
      W = pl.base; N = pl.Ntot; K = pl.K; row0 = pl.row0; rstep = pl.rstep; n_out = pl.n;
    }
    HIPCHK(hipSetDevice(e->dev));
    DevBuf dx((size_t)M * K * 4), dy((size_t)M * N * 4);
    HIPCHK(hipMemcpyAsync(dx.p, x, (size_t)M * K * 4, hipMemcpyHostToDevice, e->st));
    GemvParams g = gp(e);
    g.W = W; g.N = N; g.K = K; g.x = (const float*)dx.p; g.xs = K; g.M = M; g.out = (float*)dy.p; g.os = N;
    // default: the GEMV's fp32 arithmetic at any row count; option "linear_mfma": the batched
    // frame's MFMA GEMM where eligible (its split-K scratch reserved here: captured graphs re-capture)
    g.no_mfma = !(e->linear_mfma && gemm_mfma_eligible(N, K, M, wdt));
    if (!g.no_mfma) {
      if (e->tiled_dirty) build_tiled(e);
      if (gemm_reserve(e->ws, N, K, M)) e->g_B = -1;
    }
    launch_gemv(g, wdt, EPI_STORE, 0, e->st, 2);
    HIPCHK(hipGetLastError());
    std::vector<float> full((size_t)M * N);
    HIPCHK(hipMemcpyAsync(full.data(), dy.p, full.size() * 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    for (int m = 0; m < M; ++m)
      for (int j = 0; j < n_out; ++j) y[(size_t)m * n_out + j] = full[(size_t)m * N + row0 + (size_t)j * rstep];
  }
  CSM_CATCH
}

int csm_codes_device_ptr(csm_engine* e, void** p) {
  CSM_TRY { *p = e->hist; }
  CSM_CATCH
}

int csm_bench_gemv(csm_engine* e, int which, int M, int iters, float* avg_us, double* bytes) {
  CSM_TRY {
    if (M <= 0 || M > 2 * e->B_max || iters <= 0) throw CsmError(CSM_ERR_ARG, "bad bench arguments");
    HIPCHK(hipSetDevice(e->dev));
    if (e->tiled_dirty) build_tiled(e);
    const int stack = (which & 7) / 4;
    Stack& s = stack == 0 ? e->bb : e->dec;
    const int tag = stack == 0 ? 0 : 1;
    float* x = stack == 0 ? e->x : e->dx;
    float* mlp = stack == 0 ? e->mlp : e->dmlp;
    const int D = s.d.hidden, F = s.d.intermediate;
    const int kind = which % 4;
    // one launch per layer in turn, as the frame does, so the weight working set (and hence
    // L2 / Infinity-Cache residency) matches the real frame: backbone 16 x 67 MB streams from
    // HBM, decoder 4 x 33.5 MB stays within the 256 MiB Infinity Cache.
    auto params = [&](int layer, int& epi, int& norm) {
      const LayerW& l = s.L[layer];
      GemvParams g = gp(e);
      if (kind == 0) {  // norm + gate/up + SiLU
        g.W = l.wgu; g.N = 2 * F; g.K = D; g.x = x; g.xs = D; g.M = M; g.nw = l.n2; g.eps = s.d.eps;
        g.out = mlp; g.os = F; epi = EPI_SILU_MUL; norm = 1;
      } else if (kind == 1) {  // down + residual
        g.W = l.wd; g.N = D; g.K = F; g.x = mlp; g.xs = F; g.M = M; g.out = x; g.os = D; epi = EPI_ADD; norm = 0;
      } else if (kind == 2) {  // norm + QKV + RoPE + KV append (position 0)
        g.W = l.wqkv; g.N = s.qkv_rows(); g.K = D; g.x = x; g.xs = D; g.M = M; g.nw = l.n1; g.eps = s.d.eps;
        g.out = stack == 0 ? e->q : e->dq; g.os = s.q_dim(); g.Hq = s.d.n_heads; g.Hkv = s.d.n_kv_heads;
        g.hd = s.d.head_dim; g.S_cap = s.S_cap; g.rope = s.rope; g.kc = l.kc; g.vc = l.vc; g.rm = RowMap{1, 0, nullptr, 0};
        epi = EPI_QKV; norm = 1;
      } else {  // o_proj + residual
        g.W = l.wo; g.N = D; g.K = s.q_dim(); g.x = stack == 0 ? e->att : e->datt; g.xs = s.q_dim(); g.M = M;
        g.out = x; g.os = D; epi = EPI_ADD; norm = 0;
      }
      return g;
    };
    // which & 8: the streaming matrix-core GEMM (gemm_xs) of the same projection at M rows, with the
    // decoder path's operands and producer outputs (split rows in, split rows + sums out; lab timing)
    const bool xsb = (which & 8) != 0;
    auto xs_params = [&](GemvParams g, int epi) {
      const int Dm = s.d.hidden;
      g.x = nullptr;
      g.xs_in = (epi == EPI_ADD && g.K == F) ? e->xs_F : (epi == EPI_ADD ? e->xs_A : e->xs_D);
      g.ss_in = e->xs_ss; g.ss_n = gemm_xs_tiles(Dm, F, M); g.ss_stride = GEMM_XS_MAX_M;
      const bool noprod = (which & 16) != 0;  // lab: without the producer outputs (their cost)
      if (epi == EPI_SILU_MUL) { g.out = noprod ? mlp : nullptr; if (!noprod) { g.xs_out = e->xs_F; g.xs_K = F; } }
      if (epi == EPI_ADD && !noprod) { g.xs_out = e->xs_D; g.xs_nw = s.L[0].n1; g.ss_out = e->xs_ss; g.xs_K = Dm; }
      if (e->wdt == WDT_Q4) { g.hs_in = e->hs_D; g.hs_out = (epi == EPI_SILU_MUL) ? e->hs_F : e->hs_A; }
      return g;
    };
    int epi = 0, norm = 0;
    GemvParams g = params(0, epi, norm);
    size_t nbytes = e->wbytes(g.N, g.K);
    nbytes += (size_t)M * g.K * 4 + (size_t)M * (epi == EPI_SILU_MUL ? F : D) * 4 * (epi == EPI_ADD ? 2 : 1);
    const char* lenv = getenv("CSM_BENCH_LAYERS");  // lab: rotate over fewer layers (cache residency)
    const int nl = lenv ? std::max(1, std::min(atoi(lenv), s.d.n_layers)) : s.d.n_layers;
    auto run1 = [&](int i) {
      GemvParams gi = params(i % nl, epi, norm);
      if (xsb) {
        if (!norm) gi.nw = nullptr;
        launch_gemm_xs(xs_params(gi, epi), epi, e->st, tag == 0 && gemv_nt(0), e->wdt);
      } else {
        launch_gemv(gi, e->wdt, epi, norm, e->st, tag);
      }
    };
    for (int i = 0; i < nl; ++i) run1(i);
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    if (xsb) gemm_xs_stamps_report("warm");  // lab builds: clears the stamps of the warm-up launches
    HIPCHK(hipEventRecord(a, e->st));
    for (int i = 0; i < iters; ++i) run1(i);
    HIPCHK(hipEventRecord(b, e->st));
    HIPCHK(hipEventSynchronize(b));
    if (xsb) gemm_xs_stamps_report((std::string(stack ? "dec" : "bb") + " kind " + std::to_string(kind) + " M " + std::to_string(M)).c_str());
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (avg_us) *avg_us = ms * 1000.f / iters;
    if (bytes) *bytes = (double)nbytes;
  }
  CSM_CATCH
}

int csm_bench_dec_frame(csm_engine* e, int iters, float* avg_us, double* bytes) {
  CSM_TRY {
    if (!e || iters <= 0) throw CsmError(CSM_ERR_ARG, "bad bench arguments");
    if (!dec_frame_eligible(e)) throw CsmError(CSM_ERR_STATE, "the persistent frame decoder is not active on this engine");
    if (e->prompt_len.empty() || e->prompt_len[0] < 0) throw CsmError(CSM_ERR_STATE, "csm_prefill first (the replay needs h_last)");
    HIPCHK(hipSetDevice(e->dev));
    // The replay recomputes the last frame's head from the same h_last: the same codes, logits and
    // decoder K/V rows are written again (the advance launch is not replayed).
    const size_t D = e->Dd, DB = e->D, V = e->V, F = e->dec.d.intermediate, QKV = e->dec.qkv_rows();
    const size_t HKV = e->dec.d.n_kv_heads, HD = e->dec.d.head_dim;
    // every weight in its storage format (bf16, or int4 nibbles + affine words); audio_head stays bf16
    auto wb = [&](size_t n, size_t k) { return (double)e->wbytes(n, k); };
    double nb = wb(V, DB) + DB * 4 + wb(D, DB);                       // codebook0_head, h_last, projection
    for (int step = 1; step < e->K; ++step) {
      const int rows = step == 1 ? 2 : 1, pos = step == 1 ? 1 : step;
      for (int l = 0; l < DEC_FRAME_LAYERS; ++l) {
        nb += (l == 0 && step > 1) ? (double)QKV * 4 : wb(QKV, D);          // folded qkv0 table row / QKV
        nb += wb(D, D) + wb(2 * F, D) + wb(D, F);                           // o, gate/up, down
        nb += 2.0 * HKV * (pos + 1) * HD * 4 + 2.0 * HKV * rows * HD * 4;    // K/V history read + append
      }
      nb += (double)V * D * 2 + D * 4;                                      // audio_head[step-1], next x row
    }
    for (int i = 0; i < 2; ++i) enqueue_dec_frame_only(e, e->st);
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    HIPCHK(hipEventRecord(a, e->st));
    for (int i = 0; i < iters; ++i) enqueue_dec_frame_only(e, e->st);
    HIPCHK(hipEventRecord(b, e->st));
    HIPCHK(hipEventSynchronize(b));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    check_dec_frame(e);
    if (avg_us) *avg_us = ms * 1000.f / iters;
    if (bytes) *bytes = nb;
  }
  CSM_CATCH
}

int csm_bench_dec_xsd(csm_engine* e, int iters, float* avg_us, double* bytes) {
  CSM_TRY {
    if (!e || iters <= 0) throw CsmError(CSM_ERR_ARG, "bad bench arguments");
    const int M = e->B, K = e->K;
    if (e->frames_run < 1 || !xsd_eligible(e, M)) throw CsmError(CSM_ERR_STATE, "the persistent batched decoder step is not active on this engine");
    HIPCHK(hipSetDevice(e->dev));
    // The replay recomputes the last frame's last codebook step (i = K - 1) from the same partials of
    // step K - 2: the same K/V rows, codes, logits and partials are written again.
    const int Vp = e->Vpad, i = K - 1;
    const bool greedy = e->temperature <= 0.f;
    auto part = [&](int cb) { return e->part + (size_t)cb * e->B_max * e->part_stride; };
    const int pn = greedy ? head_blocks(Vp, e->Dd, M, e->head_wdt) : 1;
    const size_t D = e->Dd, F = e->dec.d.intermediate, QKV = e->dec.qkv_rows(), HKV = e->dec.d.n_kv_heads, HD = e->dec.d.head_dim;
    auto wb = [&](size_t n, size_t k) { return (double)e->wbytes(n, k); };
    double nb = (double)M * (QKV + D) * 4;                                  // layer 0: folded table rows
    for (int l = 0; l < DEC_FRAME_LAYERS; ++l) {
      if (l > 0) nb += wb(QKV, D);
      nb += wb(D, D) + wb(2 * F, D) + wb(D, F);                             // weights in their storage format
      nb += 2.0 * M * HKV * (i + 1) * HD * 4;                               // K/V history read + append
    }
    nb += (double)Vp * D * 2;                                               // audio_head[i - 1] (bf16)
    for (int r = 0; r < 2; ++r) launch_xsd(e, M, i, part(i - 1), pn, part(i), e->st);
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    HIPCHK(hipEventRecord(a, e->st));
    for (int r = 0; r < iters; ++r) launch_xsd(e, M, i, part(i - 1), pn, part(i), e->st);
    HIPCHK(hipEventRecord(b, e->st));
    HIPCHK(hipEventSynchronize(b));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    check_dec_frame(e);
    if (avg_us) *avg_us = ms * 1000.f / (float)iters;
    if (bytes) *bytes = nb;
  }
  CSM_CATCH
}

int csm_bench_bb_step(csm_engine* e, int iters, float* avg_us, double* bytes) {
  CSM_TRY {
    if (!e || iters <= 0) throw CsmError(CSM_ERR_ARG, "bad bench arguments");
    if (!bb_step_eligible(e)) throw CsmError(CSM_ERR_STATE, "the persistent backbone step is not active on this engine");
    if (e->frames_run < 2) throw CsmError(CSM_ERR_STATE, "run two frames first (the replay needs an embedded decode row)");
    HIPCHK(hipSetDevice(e->dev));
    // The replay recomputes the last backbone row from the same embedded x at the same position: the
    // same K/V rows and h_last are written again.
    int pos = 0;
    HIPCHK(hipMemcpy(&pos, e->pos, 4, hipMemcpyDeviceToHost));
    const csm_llama_dims& d = e->bb.d;
    const double D = d.hidden, F = d.intermediate, QKV = e->bb.qkv_rows(), HKV = d.n_kv_heads, HD = d.head_dim;
    double nb = D * 4 * 2;                                                     // x in, h_last out
    for (int l = 0; l < d.n_layers; ++l) {
      nb += (double)e->wbytes((size_t)QKV, (size_t)D) + (double)e->wbytes((size_t)D, (size_t)D) +   // weights in
            (double)e->wbytes(2 * (size_t)F, (size_t)D) + (double)e->wbytes((size_t)D, (size_t)F) +     // their storage
            2 * D * 4;                                                          // format; norm weights
      nb += 2 * HKV * (double)pos * HD * 4 + 2 * HKV * HD * 4;                  // K/V history read + append
    }
    for (int i = 0; i < 2; ++i) enqueue_bb_step(e, e->st);
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    HIPCHK(hipEventRecord(a, e->st));
    for (int i = 0; i < iters; ++i) enqueue_bb_step(e, e->st);
    HIPCHK(hipEventRecord(b, e->st));
    HIPCHK(hipEventSynchronize(b));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    check_dec_frame(e);
    if (avg_us) *avg_us = ms * 1000.f / iters;
    if (bytes) *bytes = nb;
  }
  CSM_CATCH
}

int csm_set_option(csm_engine* e, const char* key, int value) {
  CSM_TRY {
    const std::string k(key ? key : "");
    if (k == "linear_mfma") {
      if (!e) throw CsmError(CSM_ERR_ARG, "linear_mfma needs an engine");
      e->linear_mfma = value != 0;
    } else if (k == "fold_proj") {
      if (!e) throw CsmError(CSM_ERR_ARG, "fold_proj needs an engine");
      e->fold_proj = value != 0;
    }
    else if (k == "qkv0_tab") {
      if (!e) throw CsmError(CSM_ERR_ARG, "qkv0_tab needs an engine");
      e->use_qkv0_tab = value != 0;
      if (e->use_qkv0_tab && !e->qkv0_built) e->proj_tab_dirty = true;  // built at the next csm_begin
    }
    else if (k == "dec_frame_stamps") {
      if (!e) throw CsmError(CSM_ERR_ARG, "dec_frame_stamps needs an engine");
      if (value && !e->df_stamps) e->df_stamps = (unsigned long long*)e->alloc((size_t)DEC_FRAME_WGS * DEC_FRAME_STAMPS * 8);
      if (!value && e->df_stamps) { e->release(e->df_stamps); e->df_stamps = nullptr; }
    }
    else if (k == "dec_frame") {
      if (!e) throw CsmError(CSM_ERR_ARG, "dec_frame needs an engine");
      e->dec_frame = value != 0;
    }
    else if (k == "bb_step_stamps") {
      if (!e) throw CsmError(CSM_ERR_ARG, "bb_step_stamps needs an engine");
      if (value && !e->bb_stamps) e->bb_stamps = (unsigned long long*)e->alloc((size_t)BB_STEP_WGS * BB_STEP_STAMPS * 8);
      if (!value && e->bb_stamps) { e->release(e->bb_stamps); e->bb_stamps = nullptr; }
    }
    else if (k == "dec_xsd_stamps") {
      if (!e) throw CsmError(CSM_ERR_ARG, "dec_xsd_stamps needs an engine");
      if (value && !e->xsd_stamps) e->xsd_stamps = (unsigned long long*)e->alloc((size_t)DEC_XSD_WGS * DEC_XSD_STAMPS * 8);
      if (!value && e->xsd_stamps) { e->release(e->xsd_stamps); e->xsd_stamps = nullptr; }
      e->g_B = -1;
    }
    else if (k == "dec_xsd_head") {
      if (!e) throw CsmError(CSM_ERR_ARG, "dec_xsd_head needs an engine");
      e->xsd_head = value != 0;
      e->g_B = -1;
    }
    else if (k == "dec_xsd_sample") {
      if (!e) throw CsmError(CSM_ERR_ARG, "dec_xsd_sample needs an engine");
      e->xsd_sample = value != 0;
      e->g_B = -1;
    }
    else if (k == "dec_xsd") {
      if (!e) throw CsmError(CSM_ERR_ARG, "dec_xsd needs an engine");
      e->xsd_on = value != 0;
      e->g_B = -1;  // captured frame graphs hold the previous path
    }
    else if (k == "bb_step") {
      if (!e) throw CsmError(CSM_ERR_ARG, "bb_step needs an engine");
      e->bb_step = value != 0;
    }
    else if (k == "gemm_xs") {
      if (!e) throw CsmError(CSM_ERR_ARG, "gemm_xs needs an engine");
      e->xs_on = value != 0;
    }
    else if (k == "bb_xs") {
      if (!e) throw CsmError(CSM_ERR_ARG, "bb_xs needs an engine");
      e->bb_xs_on = value != 0;
    }
    else if (k == "qkv0_tab_batched") {
      if (!e) throw CsmError(CSM_ERR_ARG, "qkv0_tab_batched needs an engine");
      e->no_tab_batched = value == 0;
    }
    else if (k == "attn_prefill") {
      if (!e) throw CsmError(CSM_ERR_ARG, "attn_prefill needs an engine");
      e->attn_tiles_on = value != 0;
    }
    else if (k == "prefill_rows") {
      if (!e || value < 0) throw CsmError(CSM_ERR_ARG, "prefill_rows needs an engine and a row count >= 0");
      e->prefill_rows = value;
    }
    else if (k == "inject_handoff_error") {  // test hook: raise the persistent kernels' timeout flags
      if (!e) throw CsmError(CSM_ERR_ARG, "inject_handoff_error needs an engine");
      const int one = 1;
      for (int* f : {e->df_err, e->bb_err, e->xsd_err})
        if (f && value) HIPCHK(hipMemcpy(f, &one, 4, hipMemcpyHostToDevice));
    }
    else throw CsmError(CSM_ERR_ARG, "unknown option " + k);
    if (e) e->g_B = -1;  // re-capture the frame graphs with the new setting
  }
  CSM_CATCH
}

int csm_synchronize(csm_engine* e) {
  CSM_TRY {
    HIPCHK(hipSetDevice(e->dev));
    HIPCHK(hipStreamSynchronize(e->st));
    check_dec_frame(e);
    HIPCHK(hipGetLastError());
  }
  CSM_CATCH
}

}  // extern "C"
