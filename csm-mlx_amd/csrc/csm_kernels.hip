// CSM hot-path kernels for gfx950 (MI355X, wave64).
//
// Everything the reference's frame step dispatches to MLX
// (/root/reference/csm_mlx/generation.py:21-92) is one of these kernels:
//   embed_rows     models.py:82-92 + generation.py:32-36 (gather 33 rows, masked sum)
//   gemv           every nn.Linear / audio_head matmul, with fused RMSNorm prologue and
//                  residual / SiLU*up / GELU / RoPE+KV-append epilogues
//   attn           mlx_lm SDPA (attention.py:242-249), GQA without materialising repeats
//   rmsnorm_rows   the final LlamaModel norm for h_last (generation.py:40)
//   sample         argmax / top-k + Gumbel sampling (generation.py:51-54, :81-84) fused with
//                  the next decoder input gather (embed_audio, models.py:79-80)
//   advance        EOS flag (generation.py:151), code history, frame counter
// Weights are streamed straight to VGPRs with 16-B loads (GEMV / M <= 16 regime: no LDS
// round trip); x rows are tiny and served from L1/L2.
#include "csm_kernels.h"

// ============================================================================ embed
template <typename WT>
__global__ __launch_bounds__(256) void embed_rows_kernel(EmbedParams p) {
  const int m = blockIdx.x;
  const int ncol = p.K + 1;
  float* out = p.out + (size_t)m * p.D;
  const int* tok = p.codes ? p.codes + (size_t)m * p.K : p.tok + (size_t)m * ncol;
  if (p.pos_inc && threadIdx.x == 0) p.pos_inc[m] += 1;
  for (int d = threadIdx.x; d < p.D; d += blockDim.x) {
    float acc = 0.f;
    for (int j = 0; j < ncol; ++j) {
      bool on;
      int t;
      if (p.codes) {  // decode: row = [codes, 0], mask = [1]*K + [0]  (generation.py:156-161)
        on = j < p.K;
        t = on ? tok[j] : 0;
      } else {
        on = p.mask[(size_t)m * ncol + j] != 0;
        t = tok[j];
      }
      if (!on) continue;  // masked rows contribute exact zeros
      const WT* row = (j < p.K) ? (const WT*)p.audio_emb + ((size_t)t + (size_t)p.V * j) * p.D
                                : (const WT*)p.text_emb + (size_t)t * p.D;
      acc += ld1<WT>(row + d);
    }
    out[d] = acc;
  }
}

// ============================================================================ GEMV
// y[m, n] = sum_k norm(x)[m, k] * W[n, k]   (W row-major [N][K], MLX (out,in) layout)
// One wave owns RPW consecutive weight rows for MT x-rows at a time; lanes stride K by 8
// elements (one 16-B bf16 load per row per step).  NORM=1 fuses RMSNorm of x (weight nw)
// as a per-row scale applied after the reduction.
template <int EPI, int RPW>
__device__ __forceinline__ void gemv_epilogue(const GemvParams& p, int m, int row0, const float (&v)[RPW],
                                              int lane) {
  if constexpr (EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_ADD) {
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      if (lane == r) {
        const int n = row0 + r;
        float* o = p.out + (size_t)m * p.os + n;
        float val = v[r];
        if constexpr (EPI == EPI_GELU) val = p.gelu_erf ? gelu_erf_f(val) : gelu_tanh_f(val);
        if constexpr (EPI == EPI_ADD) {
          if (p.scale) val *= p.scale[n];
          val += *o;
        }
        *o = val;
      }
    }
  } else if constexpr (EPI == EPI_SILU_MUL) {
#pragma unroll
    for (int r = 0; r < RPW; r += 2) {
      if (lane == r) {
        const int j = (row0 + r) >> 1;
        p.out[(size_t)m * p.os + j] = silu_f(v[r]) * v[r + 1];
      }
    }
  } else if constexpr (EPI == EPI_QKV) {
    // rows: [q: Hq*hd | k: Hkv*hd | v: Hkv*hd]; RoPE on interleaved pairs (2i, 2i+1)
    // (attention.py:157-177) with the cos/sin table; K/V appended at pos (KVCache.update_and_fetch)
#pragma unroll
    for (int r = 0; r < RPW; r += 2) {
      if (lane == r) {
        const int n = row0 + r;
        const int qn = p.Hq * p.hd, kn = p.Hkv * p.hd;
        float a = v[r], b = v[r + 1];
        const int bb = p.rm.b(m), pos = p.rm.pos(m);
        const int d = (n < qn ? n : (n < qn + kn ? n - qn : n - qn - kn)) % p.hd;
        if (n < qn + kn) {
          const float* cs = p.rope + ((size_t)pos * (p.hd >> 1) + (d >> 1)) * 2;
          const float c = cs[0], s = cs[1];
          const float y0 = a * c - b * s, y1 = b * c + a * s;
          a = y0;
          b = y1;
        }
        if (n < qn) {
          float* o = p.out + (size_t)m * p.os + n;
          o[0] = a;
          o[1] = b;
        } else {
          const int nn = n < qn + kn ? n - qn : n - qn - kn;
          const int kvh = nn / p.hd;
          float* cache = n < qn + kn ? p.kc : p.vc;
          float* o = cache + (((size_t)bb * p.Hkv + kvh) * p.S_cap + pos) * p.hd + d;
          o[0] = a;
          o[1] = b;
        }
      }
    }
  }
}

// TAG only separates kernel symbols per call site (0 backbone, 1 decoder, 2 heads/codec) so rocprof
// reports the dominant decoder GEMV on its own row; it does not change the code.
template <typename WT, int RPW, int MT, int EPI, int NORM, int TAG>
__global__ __launch_bounds__(256) void gemv_kernel(GemvParams p) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int row0 = (blockIdx.x * 4 + wave) * RPW;
  if (row0 >= p.N) return;
  const WT* W = (const WT*)p.W;
  for (int m0 = 0; m0 < p.M; m0 += MT) {
    float acc[MT][RPW];
    float ss[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      ss[i] = 0.f;
#pragma unroll
      for (int r = 0; r < RPW; ++r) acc[i][r] = 0.f;
    }
#pragma unroll 2
    for (int k = lane * 8; k < p.K; k += 512) {
      float w[RPW][8];
#pragma unroll
      for (int r = 0; r < RPW; ++r) W8<WT>::load(W + (size_t)(row0 + r) * p.K + k, w[r]);
      float nw[8];
      if constexpr (NORM) W8<float>::load(p.nw + k, nw);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if (m0 + i < p.M) {
          float xv[8];
          W8<float>::load(p.x + (size_t)(m0 + i) * p.xs + k, xv);
          if constexpr (NORM) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              ss[i] += xv[j] * xv[j];
              xv[j] *= nw[j];
            }
          }
#pragma unroll
          for (int r = 0; r < RPW; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][r] = fmaf(w[r][j], xv[j], acc[i][r]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (m0 + i >= p.M) break;
      float scale = 1.f;
      if constexpr (NORM) scale = rsqrtf(wave_sum(ss[i]) / (float)p.K + p.eps);
      float v[RPW];
#pragma unroll
      for (int r = 0; r < RPW; ++r) v[r] = wave_sum(acc[i][r]) * scale;
      gemv_epilogue<EPI, RPW>(p, m0 + i, row0, v, lane);
    }
  }
}

// ============================================================================ attention
// One wave per (query row m, q head h).  Keys [k0, k1] of utterance b(m), online softmax
// over 64-key chunks (lane = key for q.k, lane = head dim for p.V).  GQA: kv head h/(Hq/Hkv).
template <int HD>
__global__ __launch_bounds__(256) void attn_kernel(AttnParams p) {
  __shared__ __attribute__((aligned(16))) float qs[4][HD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int gid = blockIdx.x * 4 + wave;
  const int m = gid / p.Hq, h = gid % p.Hq;
  const bool active = m < p.M;
  const int mm = active ? m : 0;
  const float* q = p.q + (size_t)mm * p.qs + h * HD;
  for (int d = lane; d < HD; d += 64) qs[wave][d] = q[d];
  __syncthreads();
  if (!active) return;
  const int b = p.rm.b(m), pos = p.rm.pos(m);
  int k0, k1;
  if (p.mode == ATTN_CAUSAL) {
    k0 = 0;
    k1 = pos;
  } else if (p.mode == ATTN_WINDOW) {
    k0 = max(0, pos - p.window + 1);
    k1 = pos;
  } else {  // ATTN_BLOCK: moshi_mlx -- every key of the call visible, past trimmed to `window`
    const int off = pos - (m % p.rm.T);
    k0 = max(0, off - p.window);
    k1 = off + p.rm.T - 1;
  }
  const int kvh = h / (p.Hq / p.Hkv);
  const float* K = p.kc + ((size_t)b * p.Hkv + kvh) * p.S_cap * HD;
  const float* V = p.vc + ((size_t)b * p.Hkv + kvh) * p.S_cap * HD;
  constexpr int NO = HD / 64;
  float o[NO];
#pragma unroll
  for (int i = 0; i < NO; ++i) o[i] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  for (int c = k0; c <= k1; c += 64) {
    const int j = c + lane;
    float s = -INFINITY;
    if (j <= k1) {
      const float4* kr = reinterpret_cast<const float4*>(K + (size_t)j * HD);
      const float4* qr = reinterpret_cast<const float4*>(qs[wave]);
      float dot = 0.f;
#pragma unroll
      for (int d4 = 0; d4 < HD / 4; ++d4) {
        const float4 kk = kr[d4], qq = qr[d4];
        dot = fmaf(qq.x, kk.x, dot);
        dot = fmaf(qq.y, kk.y, dot);
        dot = fmaf(qq.z, kk.z, dot);
        dot = fmaf(qq.w, kk.w, dot);
      }
      s = dot * p.scale;
    }
    const float cmax = wave_max(s);
    const float new_m = fmaxf(m_run, cmax);
    const float alpha = (m_run == -INFINITY) ? 0.f : expf(m_run - new_m);
    const float pj = (j <= k1) ? expf(s - new_m) : 0.f;
    l_run = l_run * alpha + wave_sum(pj);
#pragma unroll
    for (int i = 0; i < NO; ++i) o[i] *= alpha;
    const int n = min(64, k1 - c + 1);
    for (int jj = 0; jj < n; ++jj) {
      const float pb = __shfl(pj, jj, 64);
      const float* vr = V + (size_t)(c + jj) * HD;
#pragma unroll
      for (int i = 0; i < NO; ++i) o[i] = fmaf(pb, vr[lane + 64 * i], o[i]);
    }
    m_run = new_m;
  }
  const float inv = 1.f / l_run;
  float* out = p.out + (size_t)m * p.os + h * HD;
#pragma unroll
  for (int i = 0; i < NO; ++i) out[lane + 64 * i] = o[i] * inv;
}

// ============================================================================ rmsnorm rows
// out[m] = rmsnorm(x[row(m)]) ; optionally also scatter to dec_in[2m] (decoder step-1 rows).
__global__ __launch_bounds__(256) void rmsnorm_rows_kernel(const float* x, int xs, const float* w, float eps, int D,
                                                            float* out, int os) {
  __shared__ float red[4];
  const int m = blockIdx.x;
  const float* xr = x + (size_t)m * xs;
  float ss = 0.f;
  for (int d = threadIdx.x; d < D; d += blockDim.x) ss += xr[d] * xr[d];
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float sc = rsqrtf(tot / (float)D + eps);
  for (int d = threadIdx.x; d < D; d += blockDim.x) out[(size_t)m * os + d] = xr[d] * sc * w[d];
}

// ============================================================================ sampling
__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

struct BestPair {
  double v;
  int i;
};
__device__ __forceinline__ BestPair best_of(BestPair a, BestPair b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}

// One block per utterance.  Greedy: first max (mx.argmax).  Else Gumbel-max over
// logits*(1/temp) restricted to values >= the top_k-th largest (radix select).
template <typename WT>
__global__ __launch_bounds__(256) void sample_kernel(SampleParams p) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t sh_prefix, sh_remain;
  __shared__ double red_v[256];
  __shared__ int red_i[256];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const float* lg = p.logits + (size_t)b * p.ls;
  const int V = p.V;
  float thr = -INFINITY;
  const bool greedy = p.temperature <= 0.f;
  if (!greedy && p.top_k > 0 && p.top_k < V) {
    uint32_t prefix = 0, maskbits = 0;
    if (tid == 0) sh_remain = (uint32_t)p.top_k;
    for (int shift = 24; shift >= 0; shift -= 8) {
      hist[tid] = 0;
      __syncthreads();
      for (int v = tid; v < V; v += 256) {
        const uint32_t key = f2key(lg[v]);
        if ((key & maskbits) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (tid == 0) {
        uint32_t cum = 0, rem = sh_remain;
        int dsel = 0;
        for (int dgt = 255; dgt >= 0; --dgt) {
          if (cum + hist[dgt] >= rem) {
            dsel = dgt;
            rem -= cum;
            break;
          }
          cum += hist[dgt];
        }
        sh_remain = rem;
        sh_prefix = prefix | ((uint32_t)dsel << shift);
      }
      __syncthreads();
      prefix = sh_prefix;
      maskbits |= 255u << shift;
    }
    thr = key2f(prefix);
  }
  const int step = p.frame_ctr[0] * p.K + p.cb;
  uint64_t key = 0;
  if (!greedy) key = splitmix64(splitmix64(p.seeds[b]) ^ (uint64_t)step);
  const double inv_t = greedy ? 1.0 : (double)(1.0f / p.temperature);
  BestPair best{-INFINITY, 0x7fffffff};
  for (int v = tid; v < V; v += 256) {
    const float l = lg[v];
    double val;
    if (greedy) {
      val = (double)l;
    } else {
      if (!(l >= thr)) continue;
      const uint64_t h = splitmix64(key ^ (uint64_t)v);
      const double u = ((double)(h >> 11) + 0.5) * 1.1102230246251565e-16;  // 2^-53
      val = (double)(l * (float)inv_t) + (-log(-log(u)));
    }
    best = best_of(best, BestPair{val, v});
  }
  red_v[tid] = best.v;
  red_i[tid] = best.i;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) {
      const BestPair o = best_of(BestPair{red_v[tid], red_i[tid]}, BestPair{red_v[tid + s], red_i[tid + s]});
      red_v[tid] = o.v;
      red_i[tid] = o.i;
    }
    __syncthreads();
  }
  // NaN logits leave no winner; clamp so a bad row can never index outside the embedding table
  const int code = min(max(red_i[0], 0), V - 1);
  if (tid == 0) p.codes[(size_t)b * p.K + p.cb] = code;
  // fused embed_audio for the next decoder input (generation.py:57-64, :87-89)
  if (p.next_in) {
    const int D = p.D;
    const WT* emb = (const WT*)p.audio_emb + ((size_t)code + (size_t)p.V_emb * p.cb) * D;
    if (p.cb == 0) {
      float* r0 = p.next_in + (size_t)(2 * b) * D;
      float* r1 = r0 + D;
      const float* hl = p.h_last + (size_t)b * D;
      for (int d = tid; d < D; d += 256) {
        r0[d] = hl[d];
        r1[d] = ld1<WT>(emb + d);
      }
    } else {
      float* r = p.next_in + (size_t)b * D;
      for (int d = tid; d < D; d += 256) r[d] = ld1<WT>(emb + d);
    }
  }
}

// ============================================================================ advance
__global__ void advance_kernel(AdvanceParams p) {
  const int f = p.frame_ctr[0];
  for (int b = threadIdx.x; b < p.B; b += blockDim.x) {
    bool any = false;
    for (int k = 0; k < p.K; ++k) {
      const int c = p.codes[(size_t)b * p.K + k];
      any |= (c != 0);
      if (f < p.F_cap) p.hist[((size_t)f * p.B + b) * p.K + k] = c;
    }
    if (!any && !p.done[b]) {  // EOS: all-zero frame, not emitted (generation.py:151)
      p.done[b] = 1;
      p.n_frames[b] = f;
    }
    if (!p.done[b]) p.n_frames[b] = f + 1;
  }
  __syncthreads();
  if (threadIdx.x == 0) p.frame_ctr[0] = f + 1;
}

// ============================================================================ launchers
template <typename WT, int TAG>
static void launch_gemv_t(const GemvParams& p, int epi, int norm, hipStream_t st) {
  const int M = p.M;
  // rows per wave: 4 for tall matrices, 2 otherwise (keeps >= ~1k waves in flight)
  const int rpw = (p.N >= 8192) ? 4 : 2;
  const int blocks = (p.N + 4 * rpw - 1) / (4 * rpw);
#define GEMV_CASE(RPW, MT, E, NM) \
  hipLaunchKernelGGL((gemv_kernel<WT, RPW, MT, E, NM, TAG>), dim3(blocks), dim3(256), 0, st, p)
#define GEMV_NORM(RPW, MT, E) \
  do { if (norm) GEMV_CASE(RPW, MT, E, 1); else GEMV_CASE(RPW, MT, E, 0); } while (0)
#define GEMV_EPI(RPW, MT)                                   \
  do {                                                      \
    switch (epi) {                                          \
      case EPI_STORE: GEMV_NORM(RPW, MT, EPI_STORE); break;   \
      case EPI_ADD: GEMV_NORM(RPW, MT, EPI_ADD); break;       \
      case EPI_SILU_MUL: GEMV_NORM(RPW, MT, EPI_SILU_MUL); break; \
      case EPI_QKV: GEMV_NORM(RPW, MT, EPI_QKV); break;       \
      case EPI_GELU: GEMV_NORM(RPW, MT, EPI_GELU); break;     \
    }                                                       \
  } while (0)
  if (rpw == 4) {
    if (M <= 1) GEMV_EPI(4, 1); else if (M <= 2) GEMV_EPI(4, 2); else GEMV_EPI(4, 4);
  } else {
    if (M <= 1) GEMV_EPI(2, 1); else if (M <= 2) GEMV_EPI(2, 2); else GEMV_EPI(2, 4);
  }
#undef GEMV_EPI
#undef GEMV_NORM
#undef GEMV_CASE
}

void launch_gemv(const GemvParams& p, int wdt, int epi, int norm, hipStream_t st, int tag) {
  if (wdt == WDT_BF16) {
    if (tag == 1) launch_gemv_t<bf16_t, 1>(p, epi, norm, st);
    else if (tag == 2) launch_gemv_t<bf16_t, 2>(p, epi, norm, st);
    else launch_gemv_t<bf16_t, 0>(p, epi, norm, st);
  } else {
    if (tag == 1) launch_gemv_t<float, 1>(p, epi, norm, st);
    else if (tag == 2) launch_gemv_t<float, 2>(p, epi, norm, st);
    else launch_gemv_t<float, 0>(p, epi, norm, st);
  }
}

void launch_embed(const EmbedParams& p, int wdt, int M, hipStream_t st) {
  if (wdt == WDT_BF16) hipLaunchKernelGGL(embed_rows_kernel<bf16_t>, dim3(M), dim3(256), 0, st, p);
  else hipLaunchKernelGGL(embed_rows_kernel<float>, dim3(M), dim3(256), 0, st, p);
}

void launch_attn(const AttnParams& p, int hd, hipStream_t st) {
  const int waves = p.M * p.Hq;
  const int blocks = (waves + 3) / 4;
  if (hd == 64) hipLaunchKernelGGL(attn_kernel<64>, dim3(blocks), dim3(256), 0, st, p);
  else if (hd == 128) hipLaunchKernelGGL(attn_kernel<128>, dim3(blocks), dim3(256), 0, st, p);
}

void launch_rmsnorm_rows(const float* x, int xs, const float* w, float eps, int D, float* out, int os, int M,
                         hipStream_t st) {
  hipLaunchKernelGGL(rmsnorm_rows_kernel, dim3(M), dim3(256), 0, st, x, xs, w, eps, D, out, os);
}

void launch_sample(const SampleParams& p, int wdt, int B, hipStream_t st) {
  if (wdt == WDT_BF16) hipLaunchKernelGGL(sample_kernel<bf16_t>, dim3(B), dim3(256), 0, st, p);
  else hipLaunchKernelGGL(sample_kernel<float>, dim3(B), dim3(256), 0, st, p);
}

void launch_advance(const AdvanceParams& p, hipStream_t st) {
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(256), 0, st, p);
}
