// Mimi codec engine behind the mimi_* C ABI (include/csm_hip.h).
//
// Reference: moshi_mlx Mimi(mimi_202407(n_q)) as used by /root/reference/csm_mlx/tokenizers.py:14-21,
// 61-85, 148-150 and generation.py:224-258; restated in oracle/mimi_oracle.py.
//
// Layout: SEANet activations are [B][C][T] fp32, transformer rows [B*T][C].  The decoder SEANet
// has only stride-1 causal convs and k = 2s transposed convs, so every op is evaluated on an
// input *window* = [history (pad samples) | new samples]; one-shot decode is one window with a
// zero history, decode_step is the same code with n = 2 new latent steps per frame and the
// history carried between calls (per-utterance state, unlike the reference's process-global Mimi).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "../../include/csm_hip.h"
#include "engine_util.h"
#include "mimi_kernels.h"

namespace {

struct MConv {
  int cin, cout, k, stride, dil, elu;
  float* w = nullptr;
  float* b = nullptr;
};
struct MConvTr {
  int cin, cout, k, s, elu;
  float* wt = nullptr;  // [s][cout][cin][2]
  float* b = nullptr;
};
struct MRes {
  int ch, hid, k, dil;
  MConv c1, c2;
};
struct MOp {
  int kind;  // 0 conv, 1 convtr, 2 res
  int idx;
};
struct MTLayer {
  float *in_w, *out_w, *n1w, *n1b, *n2w, *n2b, *l1, *l2, *ls1, *ls2;
};
struct Dest {
  float* ptr;
  size_t numel;
  int kind;  // 0 plain, 1 convtr rearrange, 2 codebook sum, 3 codebook usage
  int a, b, c;  // convtr: cin, cout, k ; codebook: flat index
  std::vector<int64_t> shape;
};

}  // namespace

struct mimi_codec {
  mimi_dims d;
  int dev = 0;
  hipStream_t st = nullptr;
  int B_max = 0, F_max = 0, S_cap = 0, hd = 0;
  std::vector<MConv> convs;
  std::vector<MConvTr> convtrs;
  std::vector<MRes> res;
  std::vector<MOp> enc_ops, dec_ops;
  std::vector<MTLayer> etr, dtr;
  float *down_w = nullptr, *up_w = nullptr;
  float* rvq_in[2] = {nullptr, nullptr};
  float* rvq_out[2] = {nullptr, nullptr};
  float *cb = nullptr, *c2half = nullptr;  // [n_q][bins][cd], [n_q][bins]
  float* cbT = nullptr;                    // [n_q][cd][bins]: codebooks dims-major (RVQ encode distance GEMM)
  float* rvq_r = nullptr;                  // RVQ encode scratch: 2 x [M][cd] residuals, 2 x [M][bins / 256] partials
  size_t rvq_r_n = 0;
  unsigned long long* rvq_p = nullptr;
  size_t rvq_p_n = 0;
  float* rope = nullptr;
  std::map<std::string, Dest> dest;
  std::set<std::string> loaded;
  std::vector<std::vector<float>> cb_sum, cb_usage;
  std::vector<void*> allocs;
  // workspace (grown on demand)
  size_t ws_big = 0, ws_rows = 0;
  float *W0 = nullptr, *W1 = nullptr, *H = nullptr, *E = nullptr;  // E: ELU of the encoder's current buffer
  float* ks_ws = nullptr;  // split-K scratch of the codec GEMMs (MIMI_KS_WS_FLOATS, mimi_kernels.h)
  float *R = nullptr, *Rh = nullptr, *Rqkv = nullptr, *Rq = nullptr, *Ratt = nullptr, *Rf = nullptr;
  int* dcodes = nullptr;
  size_t dcodes_n = 0;
  float* dpcm = nullptr;
  size_t dpcm_n = 0;
  // transformer KV (encoder one-shot; decoder one-shot + streaming)
  std::vector<float*> ekc, evc, dkc, dvc;
  // streaming state
  int s_B = 0, s_off = 0;
  std::vector<float*> hist;  // per decoder op input history [B_max][cin][pad]
  float* up_hist = nullptr;  // [B_max][dim][1]
  std::vector<int> hist_pad;

  void* alloc(size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) throw CsmError(CSM_ERR_HIP, "hipMalloc(" + std::to_string(bytes) + ") failed");
    (void)hipMemset(p, 0, bytes);
    (void)hipDeviceSynchronize();  // the null-stream fill is not ordered with the engine's non-blocking stream
    allocs.push_back(p);
    return p;
  }
  ~mimi_codec() {
    for (void* p : allocs) (void)hipFree(p);
    for (float* p : {W0, W1, H, E, R, Rh, Rqkv, Rq, Ratt, Rf, dpcm}) if (p) (void)hipFree(p);
    if (dcodes) (void)hipFree(dcodes);
    if (rvq_r) (void)hipFree(rvq_r);
    if (rvq_p) (void)hipFree(rvq_p);
    if (st) (void)hipStreamDestroy(st);
  }
  int op_cin(const MOp& o) const {
    return o.kind == 0 ? convs[o.idx].cin : (o.kind == 1 ? convtrs[o.idx].cin : res[o.idx].ch);
  }
  int op_cout(const MOp& o) const {
    return o.kind == 0 ? convs[o.idx].cout : (o.kind == 1 ? convtrs[o.idx].cout : res[o.idx].ch);
  }
  // history samples an op needs in front of its new input (stride-1 conv: k_eff - 1; convtr: 1; res: k_eff - 1)
  int op_pad(const MOp& o) const {
    if (o.kind == 0) return (convs[o.idx].k - 1) * convs[o.idx].dil + 1 - convs[o.idx].stride;
    if (o.kind == 1) return 1;
    return (res[o.idx].k - 1) * res[o.idx].dil;
  }
};

namespace {

void add_dest(mimi_codec* m, const std::string& name, float* ptr, std::vector<int64_t> shape, int kind = 0, int a = 0,
              int b = 0, int c = 0) {
  size_t n = 1;
  for (auto s : shape) n *= (size_t)s;
  m->dest[name] = Dest{ptr, n, kind, a, b, c, shape};
}

void build_layout(mimi_codec* m) {
  const mimi_dims& d = m->d;
  auto conv = [&](const std::string& key, int cin, int cout, int k, int stride, int dil, int elu) {
    MConv c{cin, cout, k, stride, dil, elu};
    c.w = (float*)m->alloc((size_t)cout * cin * k * 4);
    c.b = (float*)m->alloc((size_t)cout * 4);
    add_dest(m, key + ".conv.conv.weight", c.w, {cout, cin, k});
    add_dest(m, key + ".conv.conv.bias", c.b, {cout});
    return c;
  };
  auto add_res = [&](const std::string& key, int ch) {
    MRes r{ch, ch / d.compress, d.residual_kernel_size, 1};
    r.c1 = conv(key + ".block.1", ch, r.hid, r.k, 1, r.dil, 1);
    r.c2 = conv(key + ".block.3", r.hid, ch, 1, 1, 1, 1);
    m->res.push_back(r);
    return MOp{2, (int)m->res.size() - 1};
  };
  auto add_conv = [&](const std::string& key, int cin, int cout, int k, int stride, int elu) {
    m->convs.push_back(conv(key, cin, cout, k, stride, 1, elu));
    return MOp{0, (int)m->convs.size() - 1};
  };
  auto add_convtr = [&](const std::string& key, int cin, int cout, int s) {
    MConvTr t{cin, cout, 2 * s, s, 1};
    t.wt = (float*)m->alloc((size_t)s * cout * cin * 2 * 4);
    t.b = (float*)m->alloc((size_t)cout * 4);
    add_dest(m, key + ".convtr.convtr.weight", t.wt, {cin, cout, 2 * s}, 1, cin, cout, 2 * s);
    add_dest(m, key + ".convtr.convtr.bias", t.b, {cout});
    m->convtrs.push_back(t);
    return MOp{1, (int)m->convtrs.size() - 1};
  };
  const int nf = d.n_filters;
  // encoder (moshi SEANetEncoder indices; ELU modules occupy indices)
  int idx = 0, mult = 1;
  m->enc_ops.push_back(add_conv("encoder.model.0", d.channels, nf, d.kernel_size, 1, 0));
  idx = 1;
  for (int r = d.n_ratios - 1; r >= 0; --r) {
    const int ratio = d.ratios[r], ch = mult * nf;
    m->enc_ops.push_back(add_res("encoder.model." + std::to_string(idx), ch));
    idx += 2;
    m->enc_ops.push_back(add_conv("encoder.model." + std::to_string(idx), ch, 2 * ch, 2 * ratio, ratio, 1));
    idx += 1;
    mult *= 2;
  }
  idx += 1;
  m->enc_ops.push_back(add_conv("encoder.model." + std::to_string(idx), mult * nf, d.dimension, d.last_kernel_size, 1, 1));
  // decoder
  mult = 1 << d.n_ratios;
  m->dec_ops.push_back(add_conv("decoder.model.0", d.dimension, mult * nf, d.kernel_size, 1, 0));
  idx = 1;
  for (int r = 0; r < d.n_ratios; ++r) {
    const int ratio = d.ratios[r], ch = mult * nf;
    idx += 1;
    m->dec_ops.push_back(add_convtr("decoder.model." + std::to_string(idx), ch, ch / 2, ratio));
    idx += 1;
    m->dec_ops.push_back(add_res("decoder.model." + std::to_string(idx), ch / 2));
    idx += 1;
    mult /= 2;
  }
  idx += 1;
  m->dec_ops.push_back(add_conv("decoder.model." + std::to_string(idx), nf, d.channels, d.last_kernel_size, 1, 1));
  // transformers
  const int D = d.dimension, F = d.dim_feedforward;
  for (int which = 0; which < 2; ++which) {
    auto& T = which == 0 ? m->etr : m->dtr;
    const std::string pre = which == 0 ? "encoder_transformer" : "decoder_transformer";
    T.resize(d.num_layers);
    for (int l = 0; l < d.num_layers; ++l) {
      MTLayer& L = T[l];
      const std::string p = pre + ".transformer.layers." + std::to_string(l);
      L.in_w = (float*)m->alloc((size_t)3 * D * D * 4);
      L.out_w = (float*)m->alloc((size_t)D * D * 4);
      L.l1 = (float*)m->alloc((size_t)F * D * 4);
      L.l2 = (float*)m->alloc((size_t)D * F * 4);
      for (float** v : {&L.n1w, &L.n1b, &L.n2w, &L.n2b, &L.ls1, &L.ls2}) *v = (float*)m->alloc((size_t)D * 4);
      add_dest(m, p + ".self_attn.in_proj_weight", L.in_w, {3 * D, D});
      add_dest(m, p + ".self_attn.out_proj.weight", L.out_w, {D, D});
      add_dest(m, p + ".linear1.weight", L.l1, {F, D});
      add_dest(m, p + ".linear2.weight", L.l2, {D, F});
      add_dest(m, p + ".norm1.weight", L.n1w, {D});
      add_dest(m, p + ".norm1.bias", L.n1b, {D});
      add_dest(m, p + ".norm2.weight", L.n2w, {D});
      add_dest(m, p + ".norm2.bias", L.n2b, {D});
      add_dest(m, p + ".layer_scale_1.scale", L.ls1, {D});
      add_dest(m, p + ".layer_scale_2.scale", L.ls2, {D});
    }
  }
  const int s = d.downsample_stride;
  m->down_w = (float*)m->alloc((size_t)D * D * 2 * s * 4);
  m->up_w = (float*)m->alloc((size_t)D * 2 * s * 4);
  add_dest(m, "downsample.conv.conv.conv.weight", m->down_w, {D, D, 2 * s});
  add_dest(m, "upsample.convtr.convtr.convtr.weight", m->up_w, {D, 1, 2 * s});
  const int cd = d.codebook_dim;
  const char* qn[2] = {"rvq_first", "rvq_rest"};
  for (int q = 0; q < 2; ++q) {
    m->rvq_in[q] = (float*)m->alloc((size_t)cd * D * 4);
    m->rvq_out[q] = (float*)m->alloc((size_t)D * cd * 4);
    add_dest(m, std::string("quantizer.") + qn[q] + ".input_proj.weight", m->rvq_in[q], {cd, D, 1});
    add_dest(m, std::string("quantizer.") + qn[q] + ".output_proj.weight", m->rvq_out[q], {D, cd, 1});
  }
  m->cb = (float*)m->alloc((size_t)d.n_q * d.bins * cd * 4);
  m->c2half = (float*)m->alloc((size_t)d.n_q * d.bins * 4);
  m->cbT = (float*)m->alloc((size_t)d.n_q * d.bins * cd * 4);
  m->cb_sum.assign(d.n_q, {});
  m->cb_usage.assign(d.n_q, {});
  for (int k = 0; k < d.n_q; ++k) {
    const std::string p = k == 0 ? std::string("quantizer.rvq_first.vq.layers.0._codebook")
                                 : "quantizer.rvq_rest.vq.layers." + std::to_string(k - 1) + "._codebook";
    add_dest(m, p + ".embedding_sum", nullptr, {d.bins, cd}, 2, k);
    add_dest(m, p + ".cluster_usage", nullptr, {d.bins}, 3, k);
  }
}

void finish_codebook(mimi_codec* m, int k) {
  const int bins = m->d.bins, cd = m->d.codebook_dim;
  auto& s = m->cb_sum[k];
  auto& u = m->cb_usage[k];
  if (s.empty() || u.empty()) return;
  std::vector<float> e((size_t)bins * cd), c2(bins);
  for (int i = 0; i < bins; ++i) {
    const float us = std::max(u[i], 1e-5f);  // embedding_sum / clamp(cluster_usage, eps)
    double acc = 0.0;
    for (int j = 0; j < cd; ++j) {
      const float v = s[(size_t)i * cd + j] / us;
      e[(size_t)i * cd + j] = v;
      acc += (double)v * (double)v;
    }
    c2[i] = (float)(acc / 2.0);
  }
  HIPCHK(hipMemcpy(m->cb + (size_t)k * bins * cd, e.data(), e.size() * 4, hipMemcpyHostToDevice));
  std::vector<float> et((size_t)bins * cd);
  for (int i = 0; i < bins; ++i)
    for (int j = 0; j < cd; ++j) et[(size_t)j * bins + i] = e[(size_t)i * cd + j];
  HIPCHK(hipMemcpy(m->cbT + (size_t)k * bins * cd, et.data(), et.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(m->c2half + (size_t)k * bins, c2.data(), c2.size() * 4, hipMemcpyHostToDevice));
}

template <typename T>
void grow(T*& p, size_t& cap, size_t n) {
  if (n <= cap) return;
  if (p) (void)hipFree(p);
  p = nullptr;
  if (hipMalloc((void**)&p, n * sizeof(T)) != hipSuccess) throw CsmError(CSM_ERR_HIP, "workspace allocation failed");
  cap = n;
}

void ensure_ws(mimi_codec* m, size_t big, size_t rows_M) {
  if (big > m->ws_big) {
    for (float** p : {&m->W0, &m->W1, &m->H, &m->E})
      if (*p) (void)hipFree(*p);
    for (float** p : {&m->W0, &m->W1, &m->H, &m->E})
      if (hipMalloc((void**)p, big * 4) != hipSuccess) throw CsmError(CSM_ERR_HIP, "workspace allocation failed");
    m->ws_big = big;
  }
  if (rows_M > m->ws_rows) {
    const size_t D = m->d.dimension, F = m->d.dim_feedforward;
    for (float** p : {&m->R, &m->Rh, &m->Rqkv, &m->Rq, &m->Ratt, &m->Rf})
      if (*p) (void)hipFree(*p);
    auto A = [&](float** p, size_t n) {
      if (hipMalloc((void**)p, n * 4) != hipSuccess) throw CsmError(CSM_ERR_HIP, "workspace allocation failed");
    };
    A(&m->R, rows_M * D);
    A(&m->Rh, rows_M * std::max(D, (size_t)m->d.codebook_dim));
    A(&m->Rqkv, rows_M * 3 * D);
    A(&m->Rq, rows_M * D);
    A(&m->Ratt, rows_M * D);
    A(&m->Rf, rows_M * F);
    m->ws_rows = rows_M;
  }
}

// x rows [M = B*T][D] in place through the codec transformer; positions offset..offset+T-1
void run_transformer(mimi_codec* m, std::vector<MTLayer>& T, std::vector<float*>& kc, std::vector<float*>& vc, int B,
                     int Tn, int offset) {
  const mimi_dims& d = m->d;
  const int D = d.dimension, M = B * Tn, H = d.num_heads, hd = m->hd, F = d.dim_feedforward;
  hipStream_t st = m->st;
  RowMap rm{Tn, 0, nullptr, offset};
  for (size_t l = 0; l < T.size(); ++l) {
    MTLayer& L = T[l];
    launch_layernorm_rows(m->R, D, L.n1w, L.n1b, d.norm_eps, m->Rh, M, st);
    LinParams lp{};
    lp.ks_ws = m->ks_ws;
    lp.x = m->Rh; lp.M = M; lp.K = D; lp.xs = D; lp.W = L.in_w; lp.N = 3 * D; lp.out = m->Rqkv; lp.os = 3 * D;
    lp.epi = EPI_STORE;
    launch_linear(lp, st);
    launch_rope_append(m->Rqkv, M, D, H, hd, m->rope, rm, m->Rq, kc[l], vc[l], m->S_cap, st);
    AttnParams a{};
    a.q = m->Rq; a.qs = D; a.M = M; a.kc = kc[l]; a.vc = vc[l]; a.Hq = H; a.Hkv = H; a.S_cap = m->S_cap;
    a.scale = 1.0f / sqrtf((float)hd); a.window = d.context; a.rm = rm; a.out = m->Ratt; a.os = D;
    a.mode = d.attn_mode == 0 ? ATTN_BLOCK : ATTN_WINDOW;
    launch_attn(a, hd, st);
    lp = LinParams{};
    lp.ks_ws = m->ks_ws;
    lp.x = m->Ratt; lp.M = M; lp.K = D; lp.xs = D; lp.W = L.out_w; lp.N = D; lp.out = m->R; lp.os = D;
    lp.epi = EPI_ADD; lp.scale = L.ls1;
    launch_linear(lp, st);
    launch_layernorm_rows(m->R, D, L.n2w, L.n2b, d.norm_eps, m->Rh, M, st);
    lp = LinParams{};
    lp.ks_ws = m->ks_ws;
    lp.x = m->Rh; lp.M = M; lp.K = D; lp.xs = D; lp.W = L.l1; lp.N = F; lp.out = m->Rf; lp.os = F;
    lp.epi = EPI_GELU; lp.gelu_erf = d.gelu_erf;
    launch_linear(lp, st);
    lp = LinParams{};
    lp.ks_ws = m->ks_ws;
    lp.x = m->Rf; lp.M = M; lp.K = F; lp.xs = F; lp.W = L.l2; lp.N = D; lp.out = m->R; lp.os = D;
    lp.epi = EPI_ADD; lp.scale = L.ls2;
    launch_linear(lp, st);
  }
}

int64_t conv_out_len(int64_t T, int k_eff, int stride) {  // causal conv with right "extra" padding
  const int pad = k_eff - stride;
  const double n_frames = (double)(T - k_eff + pad) / stride + 1.0;
  const int64_t ideal = ((int64_t)std::ceil(n_frames) - 1) * stride + (k_eff - pad);
  const int64_t extra = ideal - T;
  return (T + pad + extra - k_eff) / stride + 1;
}

// CSM_MIMI_ELU_PRE=0: ELU in every consumer's staging loads (A/B); else once, by the producer
bool mimi_elu_pre() {
  static const bool v = [] { const char* e = getenv("CSM_MIMI_ELU_PRE"); return !(e && e[0] == '0'); }();
  return v;
}

// One decoder-SEANet op on a window buffer: input window [B][cin][P + n] in `in` (channel stride
// cs_in), output [B][cout][P' + n'] written at offset P' (the next op's history length) of `out`.
// in_elu: the window holds ELU(x) (its producer stored it so); out_elu: store ELU(y) for an ELU-input
// next op (histories copy whichever the window holds, so the two stay consistent from call to call)
void run_window_op(mimi_codec* m, const MOp& o, const float* in, int cs_in, int P, int n, float* out, int cs_out,
                   int P_next, int B, bool in_elu = false, bool out_elu = false) {
  hipStream_t st = m->st;
  if (o.kind == 0) {
    const MConv& c = m->convs[o.idx];
    ConvParams p{};
    p.ks_ws = m->ks_ws;
    p.x = in; p.Cin = c.cin; p.Tin = P + n; p.x_bstride = c.cin * cs_in; p.x_cstride = cs_in; p.x_off = 0;
    p.w = c.w; p.bias = c.b; p.Cout = c.cout; p.k = c.k; p.stride = 1; p.dil = c.dil; p.pad_l = 0;
    p.replicate = 0; p.elu_in = c.elu && !in_elu; p.y = out; p.Tout = n; p.y_bstride = c.cout * cs_out; p.y_cstride = cs_out;
    p.y_off = P_next; p.B = B; p.elu_out = out_elu;
    launch_conv1d(p, st);
  } else if (o.kind == 1) {
    const MConvTr& t = m->convtrs[o.idx];
    ConvTrParams p{};
    p.ks_ws = m->ks_ws;
    p.x = in; p.Cin = t.cin; p.Tin = P + n; p.x_bstride = t.cin * cs_in; p.x_cstride = cs_in; p.x_off = 0;
    p.wt = t.wt; p.bias = t.b; p.Cout = t.cout; p.s = t.s; p.elu_in = t.elu && !in_elu; p.t_in0 = P; p.n_in = n; p.y = out;
    p.y_bstride = t.cout * cs_out; p.y_cstride = cs_out; p.y_off = P_next; p.B = B;
    launch_convtr(p, st);
  } else {
    const MRes& r = m->res[o.idx];
    ConvParams p{};
    p.ks_ws = m->ks_ws;  // block.1: ELU -> conv(k, ch -> hid) over the window
    p.x = in; p.Cin = r.ch; p.Tin = P + n; p.x_bstride = r.ch * cs_in; p.x_cstride = cs_in; p.x_off = 0;
    p.w = r.c1.w; p.bias = r.c1.b; p.Cout = r.hid; p.k = r.k; p.stride = 1; p.dil = r.dil; p.pad_l = 0;
    p.elu_in = 1; p.y = m->H; p.Tout = n; p.y_bstride = r.hid * n; p.y_cstride = n; p.y_off = 0; p.B = B;
    p.elu_out = mimi_elu_pre();  // H feeds only block.3's ELU
    launch_conv1d(p, st);
    ConvParams q{};
    q.ks_ws = m->ks_ws;  // block.3: ELU -> conv(1, hid -> ch) + identity skip (true_skip)
    q.x = m->H; q.Cin = r.hid; q.Tin = n; q.x_bstride = r.hid * n; q.x_cstride = n; q.x_off = 0;
    q.w = r.c2.w; q.bias = r.c2.b; q.Cout = r.ch; q.k = 1; q.stride = 1; q.dil = 1; q.pad_l = 0;
    q.elu_in = !mimi_elu_pre();
    q.y = out; q.Tout = n; q.y_bstride = r.ch * cs_out; q.y_cstride = cs_out; q.y_off = P_next;
    q.resid = in; q.r_bstride = r.ch * cs_in; q.r_cstride = cs_in; q.r_off = P; q.B = B; q.elu_out = out_elu;
    launch_conv1d(q, st);
  }
}

// Decoder from latent rows (already through the transformer): conv layout x [B][dim][n] in m->W0
// at offset P0 (history slot).  Returns pcm in the final window (device).  `stream` = keep histories.
const float* run_decoder_seanet(mimi_codec* m, int B, int n_lat, bool use_hist) {
  const auto& ops = m->dec_ops;
  float* bufs[2] = {m->W0, m->W1};
  int n = n_lat;
  int cur = 0;
  bool in_elu = false;
  auto elu_input = [&](const MOp& o) {
    return (o.kind == 0 && m->convs[o.idx].elu) || (o.kind == 1 && m->convtrs[o.idx].elu);
  };
  for (size_t i = 0; i < ops.size(); ++i) {
    const MOp& o = ops[i];
    const int P = m->op_pad(o);
    const int cin = m->op_cin(o);
    const int cs_in = P + n;
    float* in = bufs[cur];
    // history -> window head (zeros for one-shot)
    if (P > 0) {
      if (use_hist) {
        launch_copy_window(m->hist[i], B, cin, cin * P, P, 0, in, cin * cs_in, cs_in, 0, P, m->st);
      } else {
        // the B utterances' cin rows are B * cin rows of pitch cs_in: one 2-D fill for all (not one per utterance)
        HIPCHK(hipMemset2DAsync(in, (size_t)cs_in * 4, 0, (size_t)P * 4, (size_t)cin * B, m->st));
      }
    }
    const int n_out = o.kind == 1 ? n * m->convtrs[o.idx].s : n;
    const bool last = i + 1 == ops.size();
    const int P_next = last ? 0 : m->op_pad(ops[i + 1]);
    const int cs_out = P_next + n_out;
    // an output that only an ELU-input op reads is stored as ELU(y) (a transposed conv's output feeds a
    // residual block, whose skip needs y itself)
    const bool out_elu = mimi_elu_pre() && !last && o.kind != 1 && elu_input(ops[i + 1]);
    run_window_op(m, o, in, cs_in, P, n, bufs[cur ^ 1], cs_out, P_next, B, in_elu, out_elu);
    in_elu = out_elu;
    // window tail -> history for the next call
    if (use_hist && P > 0) launch_copy_window(in, B, cin, cin * cs_in, cs_in, n, m->hist[i], cin * P, P, 0, P, m->st);
    n = n_out;
    cur ^= 1;
  }
  return bufs[cur];
}

size_t decoder_ws(mimi_codec* m, int n_lat) {  // max window elements per utterance
  size_t best = (size_t)m->d.dimension * (n_lat + 8);
  int n = n_lat;
  for (const MOp& o : m->dec_ops) {
    const int P = m->op_pad(o);
    best = std::max(best, (size_t)m->op_cin(o) * (P + n));
    if (o.kind == 1) n *= m->convtrs[o.idx].s;
    best = std::max(best, (size_t)m->op_cout(o) * (n + 8));
  }
  return best;
}

}  // namespace

// =============================================================================== C ABI
extern "C" {

int mimi_create(const mimi_dims* dims, int device, int max_batch, int max_frames, mimi_codec** out) {
  CSM_TRY {
    if (!dims || !out || max_batch <= 0 || max_frames <= 0) throw CsmError(CSM_ERR_ARG, "bad codec arguments");
    if (dims->dimension % dims->num_heads) throw CsmError(CSM_ERR_ARG, "dimension % heads");
    const int hd = dims->dimension / dims->num_heads;
    if (hd != 64 && hd != 128) throw CsmError(CSM_ERR_ARG, "codec head_dim must be 64 or 128");
    if (dims->codebook_dim % 4 || dims->codebook_dim > 1024) throw CsmError(CSM_ERR_ARG, "codebook_dim");
    if (dims->n_ratios <= 0 || dims->n_ratios > 8) throw CsmError(CSM_ERR_ARG, "ratios");
    HIPCHK(hipSetDevice(device));
    std::unique_ptr<mimi_codec> m(new mimi_codec());
    m->d = *dims;
    m->dev = device;
    m->hd = hd;
    m->B_max = max_batch;
    m->F_max = max_frames;
    int hop = 1;
    for (int i = 0; i < dims->n_ratios; ++i) hop *= dims->ratios[i];
    (void)hop;
    m->S_cap = 2 * max_frames * dims->downsample_stride / 2 + 16;  // latent (25 Hz) positions
    m->S_cap = std::max(m->S_cap, 2 * max_frames + 16);
    // the codec's stream at the lowest priority (the engine's at the highest), so a streaming decode_step
    // overlapping the frame engine yields the CUs to the engine's dependent launches: config 3 +0.4-0.5 %
    // in two alternating pairs (profiles/r06_ab_stream_prio.txt).  CSM_STREAM_PRIO=0: default priorities
    if (const char* v = getenv("CSM_STREAM_PRIO"); !v || atoi(v) != 0) {
      int least = 0, greatest = 0;
      HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      HIPCHK(hipStreamCreateWithPriority(&m->st, hipStreamNonBlocking, least));
    } else {
      HIPCHK(hipStreamCreateWithFlags(&m->st, hipStreamNonBlocking));
    }
    build_layout(m.get());
    m->rope = (float*)m->alloc((size_t)m->S_cap * hd * 4);
    const size_t kv = (size_t)max_batch * dims->num_heads * m->S_cap * hd * 4;
    for (int l = 0; l < dims->num_layers; ++l) {
      m->ekc.push_back((float*)m->alloc(kv));
      m->evc.push_back((float*)m->alloc(kv));
      m->dkc.push_back((float*)m->alloc(kv));
      m->dvc.push_back((float*)m->alloc(kv));
    }
    for (const MOp& o : m->dec_ops) {
      const int P = m->op_pad(o);
      m->hist_pad.push_back(P);
      m->hist.push_back(P > 0 ? (float*)m->alloc((size_t)max_batch * m->op_cin(o) * P * 4) : nullptr);
    }
    m->up_hist = (float*)m->alloc((size_t)max_batch * dims->dimension * 4);
    m->ks_ws = (float*)m->alloc(MIMI_KS_WS_FLOATS * 4);
    HIPCHK(hipDeviceSynchronize());
    *out = m.release();
  }
  CSM_CATCH
}

int mimi_destroy(mimi_codec* m) {
  CSM_TRY { delete m; }
  CSM_CATCH
}

int mimi_set_rope_table(mimi_codec* m, const float* table, int n_pos, int head_dim) {
  CSM_TRY {
    if (head_dim != m->hd || n_pos < m->S_cap) throw CsmError(CSM_ERR_ARG, "codec rope table shape mismatch");
    HIPCHK(hipSetDevice(m->dev));
    HIPCHK(hipMemcpy(m->rope, table, (size_t)m->S_cap * head_dim * 4, hipMemcpyHostToDevice));
    m->loaded.insert("__rope__");
  }
  CSM_CATCH
}

int mimi_load_tensor(mimi_codec* m, const char* cname, const void* host, int src_dtype, const int64_t* shape,
                     int ndim) {
  CSM_TRY {
    HIPCHK(hipSetDevice(m->dev));
    const std::string name(cname);
    auto it = m->dest.find(name);
    if (it == m->dest.end()) throw CsmError(CSM_ERR_ARG, "unknown tensor " + name);
    const Dest& d = it->second;
    if (std::vector<int64_t>(shape, shape + ndim) != d.shape) throw CsmError(CSM_ERR_ARG, "shape mismatch for " + name);
    auto h = convert_to(host, src_dtype, d.numel, 0);
    const float* f = reinterpret_cast<const float*>(h.data());
    if (d.kind == 0) {
      HIPCHK(hipMemcpy(d.ptr, f, d.numel * 4, hipMemcpyHostToDevice));
    } else if (d.kind == 1) {  // ConvTranspose (cin, cout, k=2s) -> [s][cout][cin][2]
      const int cin = d.a, cout = d.b, k = d.c, s = k / 2;
      std::vector<float> t((size_t)s * cout * cin * 2);
      for (int ci = 0; ci < cin; ++ci)
        for (int co = 0; co < cout; ++co)
          for (int j = 0; j < k; ++j) {
            const int r = j % s, e = j / s;
            t[(((size_t)r * cout + co) * cin + ci) * 2 + e] = f[((size_t)ci * cout + co) * k + j];
          }
      HIPCHK(hipMemcpy(d.ptr, t.data(), t.size() * 4, hipMemcpyHostToDevice));
    } else if (d.kind == 2) {
      m->cb_sum[d.a].assign(f, f + d.numel);
      finish_codebook(m, d.a);
    } else {
      m->cb_usage[d.a].assign(f, f + d.numel);
      finish_codebook(m, d.a);
    }
    m->loaded.insert(name);
  }
  CSM_CATCH
}

int mimi_weights_ready(mimi_codec* m) {
  CSM_TRY {
    for (const auto& kv : m->dest)
      if (!m->loaded.count(kv.first)) throw CsmError(CSM_ERR_STATE, "missing codec weight " + kv.first);
    if (!m->loaded.count("__rope__")) throw CsmError(CSM_ERR_STATE, "codec rope table not set");
  }
  CSM_CATCH
}

int mimi_encode(mimi_codec* m, int B, int N, const float* pcm, int32_t* codes, int* n_frames_out) {
  return mimi_encode_rows(m, B, N, pcm, nullptr, codes, n_frames_out);
}

int mimi_encode_rows(mimi_codec* m, int B, int N, const float* pcm, const float* const* rows, int32_t* codes,
                     int* n_frames_out) {
  CSM_TRY {
    if (B <= 0 || B > m->B_max || N <= 0) throw CsmError(CSM_ERR_ARG, "bad encode shape");
    if (!pcm && !rows) throw CsmError(CSM_ERR_ARG, "encode: no audio");
    HIPCHK(hipSetDevice(m->dev));
    const mimi_dims& d = m->d;
    hipStream_t st = m->st;
    // lengths through the encoder
    std::vector<int64_t> lens{N};
    size_t big = (size_t)N * std::max(d.n_filters, d.channels) + 64;
    int64_t T = N;
    for (const MOp& o : m->enc_ops) {
      if (o.kind == 0) {
        const MConv& c = m->convs[o.idx];
        T = conv_out_len(T, (c.k - 1) * c.dil + 1, c.stride);
      }
      big = std::max(big, (size_t)m->op_cout(o) * (T + 8));
      lens.push_back(T);
    }
    const int64_t T25 = T;
    if (T25 + 4 > m->S_cap) throw CsmError(CSM_ERR_ARG, "audio longer than the codec capacity");
    const int s = d.downsample_stride;
    const int64_t Tf = conv_out_len(T25, 2 * s, s);
    big = std::max(big, (size_t)d.dimension * (T25 + 8));
    ensure_ws(m, big * B, (size_t)B * std::max<int64_t>(T25, Tf) + 8);
    if (pcm) {
      HIPCHK(hipMemcpyAsync(m->W0, pcm, (size_t)B * N * 4, hipMemcpyHostToDevice, st));
    } else {  // one host row per utterance, straight into its slot (no host-side stacking copy)
      for (int b = 0; b < B; ++b)
        HIPCHK(hipMemcpyAsync(m->W0 + (size_t)b * N, rows[b], (size_t)N * 4, hipMemcpyHostToDevice, st));
    }
    float* bufs[2] = {m->W0, m->W1};
    int cur = 0;
    int64_t Tin = N;
    // ELU once per element (CSM_MIMI_ELU_PRE=0: in every consumer's staging loads, A/B): an op whose
    // next op is an ELU-input conv stores ELU(y) in place of y; one whose next op is a residual block
    // (ELU for its first conv, y itself for the skip) also writes ELU(y) to m->E.  in_elu: bufs[cur]
    // holds ELU(x); have_e: m->E holds ELU(bufs[cur]).
    const bool elu_pre = mimi_elu_pre();
    bool in_elu = false, have_e = false;
    auto out_elu = [&](size_t i, ConvParams& p) {
      const MOp* nx = i + 1 < m->enc_ops.size() ? &m->enc_ops[i + 1] : nullptr;
      if (!elu_pre || !nx) return;
      if (nx->kind == 0 && m->convs[nx->idx].elu) p.elu_out = 1;
      else if (nx->kind != 0) p.y2 = m->E;
    };
    for (size_t i = 0; i < m->enc_ops.size(); ++i) {
      const MOp& o = m->enc_ops[i];
      float* in = bufs[cur];
      float* out = bufs[cur ^ 1];
      bool nx_in_elu = false, nx_have_e = false;
      if (o.kind == 0) {
        const MConv& c = m->convs[o.idx];
        const int k_eff = (c.k - 1) * c.dil + 1;
        const int64_t Tout = lens[i + 1];
        ConvParams p{};
        p.ks_ws = m->ks_ws;
        p.x = in; p.Cin = c.cin; p.Tin = (int)Tin; p.x_bstride = c.cin * (int)Tin; p.x_cstride = (int)Tin;
        p.w = c.w; p.bias = c.b; p.Cout = c.cout; p.k = c.k; p.stride = c.stride; p.dil = c.dil;
        p.pad_l = k_eff - c.stride; p.elu_in = c.elu; p.y = out; p.Tout = (int)Tout;
        p.y_bstride = c.cout * (int)Tout; p.y_cstride = (int)Tout; p.B = B;
        if (in_elu && !c.elu) throw CsmError(CSM_ERR_HIP, "mimi encoder: ELU bookkeeping");
        if (in_elu) p.elu_in = 0;
        out_elu(i, p);
        nx_in_elu = p.elu_out != 0;
        nx_have_e = p.y2 != nullptr;
        launch_conv1d(p, st);
        Tin = Tout;
      } else {  // resblock on the full sequence (causal, zero left pad)
        const MRes& r = m->res[o.idx];
        ConvParams p{};
        p.ks_ws = m->ks_ws;
        p.x = in; p.Cin = r.ch; p.Tin = (int)Tin; p.x_bstride = r.ch * (int)Tin; p.x_cstride = (int)Tin;
        p.w = r.c1.w; p.bias = r.c1.b; p.Cout = r.hid; p.k = r.k; p.stride = 1; p.dil = r.dil;
        p.pad_l = (r.k - 1) * r.dil; p.elu_in = 1; p.y = m->H; p.Tout = (int)Tin; p.y_bstride = r.hid * (int)Tin;
        p.y_cstride = (int)Tin; p.B = B;
        if (in_elu) throw CsmError(CSM_ERR_HIP, "mimi encoder: ELU bookkeeping");
        if (have_e) { p.x = m->E; p.elu_in = 0; }
        p.elu_out = elu_pre;  // H feeds only the block's second (ELU-input) conv
        launch_conv1d(p, st);
        ConvParams q{};
        q.ks_ws = m->ks_ws;
        q.x = m->H; q.Cin = r.hid; q.Tin = (int)Tin; q.x_bstride = r.hid * (int)Tin; q.x_cstride = (int)Tin;
        q.w = r.c2.w; q.bias = r.c2.b; q.Cout = r.ch; q.k = 1; q.stride = 1; q.dil = 1; q.elu_in = elu_pre ? 0 : 1; q.y = out;
        q.Tout = (int)Tin; q.y_bstride = r.ch * (int)Tin; q.y_cstride = (int)Tin; q.resid = in;
        q.r_bstride = r.ch * (int)Tin; q.r_cstride = (int)Tin; q.B = B;
        out_elu(i, q);
        nx_in_elu = q.elu_out != 0;
        nx_have_e = q.y2 != nullptr;
        launch_conv1d(q, st);
      }
      in_elu = nx_in_elu;
      have_e = nx_have_e;
      cur ^= 1;
    }
    // transformer on [B][dim][T25]
    const int D = d.dimension;
    launch_conv_to_rows(bufs[cur], B, D, (int)T25, D * (int)T25, (int)T25, 0, m->R, st);
    run_transformer(m, m->etr, m->ekc, m->evc, B, (int)T25, 0);
    launch_rows_to_conv(m->R, B, D, (int)T25, bufs[cur ^ 1], D * (int)T25, (int)T25, 0, st);
    cur ^= 1;
    // downsample: k = 2s, stride s, replicate pad, no bias
    {
      ConvParams p{};
      p.ks_ws = m->ks_ws;
      p.x = bufs[cur]; p.Cin = D; p.Tin = (int)T25; p.x_bstride = D * (int)T25; p.x_cstride = (int)T25;
      p.w = m->down_w; p.Cout = D; p.k = 2 * s; p.stride = s; p.dil = 1; p.pad_l = s; p.replicate = 1;
      p.y = bufs[cur ^ 1]; p.Tout = (int)Tf; p.y_bstride = D * (int)Tf; p.y_cstride = (int)Tf; p.B = B;
      launch_conv1d(p, st);
      cur ^= 1;
    }
    // split RVQ: semantic and acoustic both quantize the same latent
    launch_conv_to_rows(bufs[cur], B, D, (int)Tf, D * (int)Tf, (int)Tf, 0, m->R, st);
    const int M = B * (int)Tf, cd = d.codebook_dim;
    grow(m->dcodes, m->dcodes_n, (size_t)B * d.n_q * Tf);
    for (int q = 0; q < 2; ++q) {
      LinParams lp{};
      lp.ks_ws = m->ks_ws;
      lp.x = m->R; lp.M = M; lp.K = D; lp.xs = D; lp.W = m->rvq_in[q]; lp.N = cd; lp.out = m->Rh; lp.os = cd;
      lp.epi = EPI_STORE;
      launch_linear(lp, st);
      const int k0 = q == 0 ? 0 : 1, k1 = q == 0 ? 1 : d.n_q;
      if (k1 <= k0) continue;
      // many rows: one distance GEMM launch per codebook (CSM_RVQ_GEMM=0: the tiled / per-row kernels)
      static const bool gemm_on = [] { const char* e = getenv("CSM_RVQ_GEMM"); return !(e && e[0] == '0'); }();
      if (gemm_on && M >= 256 && rvq_gemm_eligible(cd, d.bins)) {
        grow(m->rvq_r, m->rvq_r_n, (size_t)2 * M * cd);
        grow(m->rvq_p, m->rvq_p_n, 2 * rvq_gemm_parts(M, d.bins));
        launch_rvq_encode_gemm(m->Rh, M, (int)Tf, cd, m->cb, m->cbT, m->c2half, d.bins, k0, k1, d.n_q, m->dcodes,
                               m->rvq_r, m->rvq_p, st);
      } else {
        launch_rvq_encode(m->Rh, M, (int)Tf, cd, m->cb, m->c2half, d.bins, k0, k1, d.n_q, m->dcodes, st);
      }
    }
    HIPCHK(hipMemcpyAsync(codes, m->dcodes, (size_t)B * d.n_q * Tf * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipGetLastError());
    if (n_frames_out) *n_frames_out = (int)Tf;
  }
  CSM_CATCH
}

static void decode_frames(mimi_codec* m, int B, int F, const int32_t* dcodes, int layout, bool stream) {
  const mimi_dims& d = m->d;
  hipStream_t st = m->st;
  const int D = d.dimension, cd = d.codebook_dim, s = d.downsample_stride;
  const int n_lat = F * s;
  const int M = B * F;
  // RVQ decode: semantic + acoustic gathers, output projections summed into conv layout [B][D][F]
  launch_rvq_gather(dcodes, layout, B, F, d.n_q, 0, 1, m->cb, d.bins, cd, m->Rh, st);
  LinParams lp{};
  lp.ks_ws = m->ks_ws;
  lp.x = m->Rh; lp.M = M; lp.K = cd; lp.xs = cd; lp.W = m->rvq_out[0]; lp.N = D; lp.conv_T = F;
  lp.conv_bstride = D * F; lp.out = m->W1; lp.accumulate = 0;
  launch_linear(lp, st);
  if (d.n_q > 1) {
    launch_rvq_gather(dcodes, layout, B, F, d.n_q, 1, d.n_q, m->cb, d.bins, cd, m->Rh, st);
    lp.W = m->rvq_out[1];
    lp.accumulate = 1;
    launch_linear(lp, st);
  }
  // upsample (depthwise ConvTranspose k=2s): window [1 history | F new] in H
  const int cs = F + 1;
  if (stream) {
    launch_copy_window(m->up_hist, B, D, D, 1, 0, m->H, D * cs, cs, 0, 1, st);
  } else {
    HIPCHK(hipMemset2DAsync(m->H, (size_t)cs * 4, 0, 4, (size_t)D * B, st));  // B * D rows of pitch cs
  }
  launch_copy_window(m->W1, B, D, D * F, F, 0, m->H, D * cs, cs, 1, F, st);
  if (stream) launch_copy_window(m->H, B, D, D * cs, cs, F, m->up_hist, D, 1, 0, 1, st);
  launch_upsample_dw(m->H, B, D, D * cs, cs, 0, m->up_w, s, 1, F, m->W1, D * n_lat, n_lat, 0, st);
  // transformer on the latent steps
  launch_conv_to_rows(m->W1, B, D, n_lat, D * n_lat, n_lat, 0, m->R, st);
  run_transformer(m, m->dtr, m->dkc, m->dvc, B, n_lat, m->s_off);
  m->s_off += n_lat;
  const int P0 = m->op_pad(m->dec_ops[0]);
  launch_rows_to_conv(m->R, B, D, n_lat, m->W0, D * (P0 + n_lat), P0 + n_lat, P0, st);
  run_decoder_seanet(m, B, n_lat, stream);
}

int mimi_decode(mimi_codec* m, int B, int F, const int32_t* codes, int codes_on_device, int codes_layout, float* pcm,
                int pcm_on_device) {
  CSM_TRY {
    if (B <= 0 || B > m->B_max || F <= 0) throw CsmError(CSM_ERR_ARG, "bad decode shape");
    if (2 * F + 4 > m->S_cap) throw CsmError(CSM_ERR_ARG, "more frames than the codec capacity");
    HIPCHK(hipSetDevice(m->dev));
    const mimi_dims& d = m->d;
    const int s = d.downsample_stride;
    const size_t per = decoder_ws(m, F * s);
    ensure_ws(m, per * B + 64, (size_t)B * F * s + 8);
    // Mimi.decode resets the decoder state first (moshi_mlx), so a one-shot decode starts at position 0
    m->s_off = 0;
    const int32_t* dc = codes;
    if (!codes_on_device) {
      grow(m->dcodes, m->dcodes_n, (size_t)B * d.n_q * F);
      HIPCHK(hipMemcpyAsync(m->dcodes, codes, (size_t)B * d.n_q * F * 4, hipMemcpyHostToDevice, m->st));
      dc = m->dcodes;
    }
    decode_frames(m, B, F, dc, codes_layout, false);
    m->s_off = 0;
    // final window: [B][1][F*frame] in whichever ping-pong buffer run_decoder_seanet ended in
    const int n_out = F * s;
    int n = n_out;
    for (const MOp& o : m->dec_ops)
      if (o.kind == 1) n *= m->convtrs[o.idx].s;
    const float* src = (m->dec_ops.size() % 2 == 0) ? m->W0 : m->W1;
    const size_t bytes = (size_t)B * n * 4;
    HIPCHK(hipMemcpyAsync(pcm, src, bytes, pcm_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, m->st));
    HIPCHK(hipStreamSynchronize(m->st));
    HIPCHK(hipGetLastError());
  }
  CSM_CATCH
}

int mimi_reset_state(mimi_codec* m, int B) {
  CSM_TRY {
    if (B <= 0 || B > m->B_max) throw CsmError(CSM_ERR_ARG, "bad batch");
    HIPCHK(hipSetDevice(m->dev));
    m->s_B = B;
    m->s_off = 0;
    for (size_t i = 0; i < m->hist.size(); ++i)
      if (m->hist[i])
        HIPCHK(hipMemsetAsync(m->hist[i], 0, (size_t)B * m->op_cin(m->dec_ops[i]) * m->hist_pad[i] * 4, m->st));
    HIPCHK(hipMemsetAsync(m->up_hist, 0, (size_t)B * m->d.dimension * 4, m->st));
    HIPCHK(hipStreamSynchronize(m->st));
  }
  CSM_CATCH
}

int mimi_decode_step(mimi_codec* m, int B, const int32_t* codes, float* pcm) {
  CSM_TRY {
    if (B != m->s_B) throw CsmError(CSM_ERR_STATE, "mimi_reset_state(B) must precede decode_step");
    const int s = m->d.downsample_stride;
    if (m->s_off + s + 4 > m->S_cap) throw CsmError(CSM_ERR_ARG, "stream longer than the codec capacity");
    HIPCHK(hipSetDevice(m->dev));
    const size_t per = decoder_ws(m, s);
    ensure_ws(m, per * B + 64, (size_t)B * s + 8);
    grow(m->dcodes, m->dcodes_n, (size_t)B * m->d.n_q);
    HIPCHK(hipMemcpyAsync(m->dcodes, codes, (size_t)B * m->d.n_q * 4, hipMemcpyHostToDevice, m->st));
    decode_frames(m, B, 1, m->dcodes, 0, true);
    int n = s;
    for (const MOp& o : m->dec_ops)
      if (o.kind == 1) n *= m->convtrs[o.idx].s;
    const float* src = (m->dec_ops.size() % 2 == 0) ? m->W0 : m->W1;
    HIPCHK(hipMemcpyAsync(pcm, src, (size_t)B * n * 4, hipMemcpyDeviceToHost, m->st));
    HIPCHK(hipStreamSynchronize(m->st));
    HIPCHK(hipGetLastError());
  }
  CSM_CATCH
}

}  // extern "C"
