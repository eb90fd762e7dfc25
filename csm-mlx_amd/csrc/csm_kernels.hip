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
#include "engine_util.h"
#include "xs.h"

#include <cstdlib>

// ============================================================================ embed
// x[m] = sum_j mask[m,j] * table_j[tok[m,j]]  over the K audio columns (row tok + V*j of the
// audio table) then the text column -- the order of the reference's .sum(-2) over 33 rows
// (generation.py:34-36).  Row pointers are resolved once into LDS; each thread then sums 8
// consecutive dims with independent 16-B loads.
template <typename WT>
__global__ __launch_bounds__(64) void embed_rows_kernel(EmbedParams p) {
  // one wave per 512 columns of row m.  Lane j (< K + 1 <= 64) resolves column j's table row (one
  // vector load of all codes / tokens / masks at once), then every row's 16-B slice is loaded
  // before any is summed (one memory round trip for all K + 1 rows), added in column order j = 0..K.
  constexpr int CH = 33;
  const int m = blockIdx.x, t = threadIdx.x;
  const int ncol = p.K + 1;
  if (p.pos_inc && blockIdx.y == 0 && t == 0) p.pos_inc[m] += 1;
  long long off = -1;  // element offset of column t's row in its table, -1 when masked
  if (t < ncol) {
    if (p.codes) {  // decode: row = [codes, 0], mask = [1]*K + [0]  (generation.py:156-161)
      if (t < p.K) off = ((long long)p.codes[(size_t)m * p.K + t] + (long long)p.V * t) * p.D;
    } else if (p.mask[(size_t)m * ncol + t]) {
      const long long tk = p.tok[(size_t)m * ncol + t];
      off = t < p.K ? (tk + (long long)p.V * t) * p.D : tk * p.D;
    }
  }
  const int off_lo = (int)(unsigned long long)off, off_hi = (int)((unsigned long long)off >> 32);
  const int d0 = (blockIdx.y * 64 + t) * 8;
  if (d0 >= p.D) return;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < ncol; j0 += CH) {
    Raw8<WT> raw[CH];
    bool live[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int j = j0 + u;
      long long o = -1;
      if (j < ncol)
        o = (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane(off_hi, j) << 32) |
                        (unsigned)__builtin_amdgcn_readlane(off_lo, j));
      live[u] = o >= 0;
      const WT* base = (const WT*)(j < p.K ? p.audio_emb : p.text_emb);
      raw[u].template load<false>(base + (o >= 0 ? o : 0) + d0);
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      if (!live[u]) continue;  // masked columns contribute exact zeros
      float w[8];
      raw[u].get(w);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += w[e];
    }
  }
  float* out = p.out + (size_t)m * p.D;
  *reinterpret_cast<float4*>(out + d0) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  *reinterpret_cast<float4*>(out + d0 + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  if (p.xs_out) {  // the streaming backbone QKV's operand: split (x * n1), + this block's sum of squares
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s = fmaf(acc[e], acc[e], s);
    s = wave_sum(s);
    if (t == 0) p.ss_out[(size_t)blockIdx.y * p.ss_stride + m] = s;
    float hsum = 0.f;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = acc[4 * hf + u] * p.xs_nw[d0 + 4 * hf + u];
        hsum += v[u];
      }
      xs::store4(p.xs_out, p.D, m, d0 + 4 * hf, v);
    }
    if (p.hs_out) {  // half-group sums (32 columns = 4 lanes, in column order) for int4 consumers
      const int b4 = t & ~3;
      const float h0 = __shfl(hsum, b4, 64), h1 = __shfl(hsum, b4 + 1, 64), h2 = __shfl(hsum, b4 + 2, 64),
                  h3 = __shfl(hsum, b4 + 3, 64);
      if ((t & 3) == 0) p.hs_out[(size_t)(d0 / 32) * xs::HS_ROWS + m] = ((h0 + h1) + h2) + h3;
    }
  }
}

// ============================================================================ split rows
// The streaming GEMM's operand (xs.h) from dense rows: x[m] * nw in fragment order, per-row sums of
// squares of x per 512-column block (ss_out[blockIdx.y * ss_stride + m]) and, for int4 consumers, the
// half-group sums -- the embedding producer's outputs (embed_rows_kernel), for rows another kernel
// wrote densely (the depth decoder's step-1 rows after the projection).  One wave per 512 columns.
__global__ __launch_bounds__(64) void xs_rows_kernel(const float* x, int xstride, int K, const float* nw, void* xs_out,
                                                     float* ss_out, int ss_stride, float* hs_out) {
  const int m = blockIdx.x, t = threadIdx.x, d0 = (blockIdx.y * 64 + t) * 8;
  if (d0 >= K) return;
  const float* xr = x + (size_t)m * xstride + d0;
  const float4 a = *reinterpret_cast<const float4*>(xr), b = *reinterpret_cast<const float4*>(xr + 4);
  const float v8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  float sq = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) sq = fmaf(v8[e], v8[e], sq);
  sq = wave_sum(sq);
  if (t == 0) ss_out[(size_t)blockIdx.y * ss_stride + m] = sq;
  float hsum = 0.f;
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v[u] = v8[4 * hf + u] * nw[d0 + 4 * hf + u];
      hsum += v[u];
    }
    xs::store4(xs_out, K, m, d0 + 4 * hf, v);
  }
  if (hs_out) {
    const int b4 = t & ~3;
    const float h0 = __shfl(hsum, b4, 64), h1 = __shfl(hsum, b4 + 1, 64), h2 = __shfl(hsum, b4 + 2, 64),
                h3 = __shfl(hsum, b4 + 3, 64);
    if ((t & 3) == 0) hs_out[(size_t)(d0 / 32) * xs::HS_ROWS + m] = ((h0 + h1) + h2) + h3;
  }
}

void launch_xs_rows(const float* x, int xstride, int M, int K, const float* nw, void* xs_out, float* ss_out, int ss_stride,
                    float* hs_out, hipStream_t st) {
  hipLaunchKernelGGL(xs_rows_kernel, dim3(M, (K + 511) / 512), dim3(64), 0, st, x, xstride, K, nw, xs_out, ss_out, ss_stride, hs_out);
}

// ============================================================================ GEMV
// y[m, n] = sum_k norm(x)[m, k] * W[n, k]   (W row-major [N][K], MLX (out,in) layout)
//
// A 256-thread block owns RPB = (256/G)*RPT consecutive weight rows.  The block is split into
// 256/G row groups of G threads; a group walks K in strides of G*8 elements (one 16-B bf16 load
// per row per step, straight to VGPRs -- the GEMV / M <= 16 regime: no LDS staging of the weight
// stream), each thread carrying RPT rows x MT activation rows of fp32 accumulators.  Partials are
// reduced with wave shuffles, then across the group's waves through LDS.  G is chosen so a group
// covers K in 1-4 steps (G = 128 at K = 1024, 256 at K >= 2048): thousands of waves in flight for
// the 16-67 MB projections.  NORM fuses RMSNorm of x (weight nw) as a per-row scale applied
// after the reduction; the epilogue (store / residual add / SiLU*up / GELU / RoPE + KV append)
// runs on row pairs so RoPE pairs and interleaved gate/up rows stay in one thread.
template <typename WT, int G, int RPT, int MT, int TAG>
__global__ __launch_bounds__(256) void gemv_kernel(GemvParams p) {
  constexpr int NG = 256 / G;
  constexpr int RPB = NG * RPT;
  __shared__ float red[4][MT][RPT + 1];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int grp = tid / G, gt = tid % G;
  const int row0 = blockIdx.x * RPB + grp * RPT;
  const bool norm = p.nw != nullptr;
  const WT* W = (const WT*)p.W;
  // x gather mode: resolve each needed row's code from the producer's block partials once
  __shared__ int gcode[512];  // codes of the gathered rows (M <= 512)
  if (p.xpart) {
    for (int m = wave; m < p.M; m += 4) {
      const int bb = p.x_step1 ? (m >> 1) : m;
      if (p.x_step1 && !(m & 1)) continue;
      const unsigned long long best = wave_argmax_partials(p.xpart + (size_t)bb * p.xpart_stride, p.xpart_n, lane);
      if (lane == 0) {
        const int c = min(max(unpack_argmax(best), 0), p.xV - 1);
        gcode[m] = c;
        if (blockIdx.x == 0) p.x_codes[(size_t)bb * p.x_codes_K + p.xcb] = c;
      }
    }
    __syncthreads();
  }
  for (int m0 = 0; m0 < p.M; m0 += MT) {
    float acc[MT][RPT];
    float ss[MT];
    const float* xf[MT];
    const WT* xw[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int m = m0 + i;
      xf[i] = p.x + (size_t)m * p.xs;
      xw[i] = nullptr;
      if (p.xpart && m < p.M && !(p.x_step1 && !(m & 1))) {
        const size_t trow = ((size_t)gcode[m] + (size_t)p.xV * p.xcb) * p.K;
        if (p.xtab_f32) xf[i] = (const float*)p.xtab + trow;
        else xw[i] = (const WT*)p.xtab + trow;
      } else if (p.x_step1) {
        xf[i] = p.x + (size_t)(m >> 1) * p.xs;
      }
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      ss[i] = 0.f;
#pragma unroll
      for (int r = 0; r < RPT; ++r) acc[i][r] = 0.f;
    }
#pragma unroll 2
    for (int k = gt * 8; k < p.K; k += G * 8) {
      float w[RPT][8];
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        if constexpr ((TAG & 4) != 0) W8<WT>::load_nt(W + (size_t)(row0 + r) * p.K + k, w[r]);
        else W8<WT>::load(W + (size_t)(row0 + r) * p.K + k, w[r]);
      }
      float nw[8];
      if (norm) W8<float>::load(p.nw + k, nw);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if (m0 + i < p.M) {
          float xv[8];
          if (xw[i]) W8<WT>::load(xw[i] + k, xv);
          else W8<float>::load(xf[i] + k, xv);
          if (p.x_copy && blockIdx.x == 0 && grp == 0) {  // group 0 of block 0 walks all of K
            float* xc = p.x_copy + (size_t)(m0 + i) * p.K + k;
            *reinterpret_cast<float4*>(xc) = make_float4(xv[0], xv[1], xv[2], xv[3]);
            *reinterpret_cast<float4*>(xc + 4) = make_float4(xv[4], xv[5], xv[6], xv[7]);
          }
          if (norm) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              ss[i] = fmaf(xv[j], xv[j], ss[i]);
              xv[j] *= nw[j];
            }
          }
#pragma unroll
          for (int r = 0; r < RPT; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][r] = fmaf(w[r][j], xv[j], acc[i][r]);
        }
      }
    }
    // reduce: wave shuffles, then the G/64 waves of the group through LDS
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const float v = wave_sum(acc[i][r]);
        if (lane == 0) red[wave][i][r] = v;
      }
      if (norm) {
        const float v = wave_sum(ss[i]);
        if (lane == 0) red[wave][i][RPT] = v;
      }
    }
    __syncthreads();
    constexpr int WPG = G / 64;  // waves per group
    constexpr int NPAIR = NG * MT * (RPT / 2);
    unsigned long long akey = 0;
    int arow = -1;
    if (tid < NPAIR) {
      const int g = tid / (MT * (RPT / 2));
      const int rem = tid % (MT * (RPT / 2));
      const int i = rem / (RPT / 2), rp = (rem % (RPT / 2)) * 2;
      const int m = m0 + i;
      if (m < p.M) {
        float a = 0.f, b = 0.f, sq = 0.f;
#pragma unroll
        for (int w = 0; w < WPG; ++w) {
          a += red[g * WPG + w][i][rp];
          b += red[g * WPG + w][i][rp + 1];
          sq += red[g * WPG + w][i][RPT];
        }
        if (norm) {
          const float sc = rsqrtf(sq / (float)p.K + p.eps);
          a *= sc;
          b *= sc;
        }
        gemv_epilogue_pair(p, m, blockIdx.x * RPB + g * RPT + rp, a, b);
        if (p.epi == EPI_ARGMAX) {
          const int n = blockIdx.x * RPB + g * RPT + rp;
          unsigned long long key = 0;
          if (n < p.n_valid) key = pack_argmax(a, n);
          if (n + 1 < p.n_valid) {
            const unsigned long long kb = pack_argmax(b, n + 1);
            key = kb > key ? kb : key;
          }
          akey = key;
          arow = i;
        }
      }
    }
    if (p.epi == EPI_ARGMAX && wave == 0) {  // block arg-max per row -> partial slot
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        unsigned long long v = (tid < NPAIR && arow == i) ? akey : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const unsigned long long w = __shfl_xor(v, o, 64);
          v = w > v ? w : v;
        }
        if (lane == 0 && m0 + i < p.M) p.part[(size_t)(m0 + i) * p.part_stride + blockIdx.x] = v;
      }
    }
    __syncthreads();
  }
}

// ============================================================================ GEMV, activations in LDS
// Decode-regime variant (M <= MT, K <= XL_KMAX) of gemv_kernel.  Profiling (tools/lab.py) showed
// the register-direct kernel at ~half the streaming rate on the K = 1024/2048 matrices: every
// wave re-read the fp32 activation row AND the RMSNorm weight for its K slice through the vector
// memory path -- 2x the weight bytes per CU.  Here the block (1) puts ALL of its weight K-steps in
// flight into VGPRs first, (2) stages x (dense or gathered table rows) times the norm weight into
// LDS once, reducing sum(x^2) per row once per block, (3) runs the dot products from LDS.  Per
// thread the weight K-slices, accumulation order and pair epilogues are those of gemv_kernel.
constexpr int XL_KMAX = 2048;
constexpr int XL_KMAX_WIDE = 8192;  // down projections (K = 8192) at M = 1: 32 KB of LDS

template <typename WT, int G, int RPT, int MT, int TAG, int KMAX = XL_KMAX>
__global__ __launch_bounds__(256) void gemv_xl_kernel(GemvParams p) {
  if (p.row_chunk) {  // table builds: one launch covers every row, MT rows per grid row
    const int y0 = blockIdx.y * p.row_chunk;
    p.x += (size_t)y0 * p.xs;
    if (p.out) p.out += (size_t)y0 * p.os;
    if (p.qkv_tab) p.qkv_tab += (size_t)y0 * p.N;
    p.M = min(p.row_chunk, p.M - y0);
  }
  constexpr int NG = 256 / G;
  constexpr int RPB = NG * RPT;
  constexpr int NKM = KMAX / (G * 8);  // K-steps per thread at most
  constexpr bool NT = (TAG & 4) != 0;
  __shared__ __attribute__((aligned(16))) float xl[MT][KMAX];
  __shared__ float red[4][MT][RPT];
  __shared__ float rss[4][MT];
  __shared__ int gcode[MT];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int grp = tid / G, gt = tid % G;
  const int row0 = blockIdx.x * RPB + grp * RPT;
  const bool norm = p.nw != nullptr;
  const WT* W = (const WT*)p.W;
  // (1) every weight K-step of this thread in flight before anything else
  Raw8<WT> wr[NKM][RPT];
#pragma unroll
  for (int s = 0; s < NKM; ++s) {
    const int k = gt * 8 + s * G * 8;
    if (k < p.K) {
#pragma unroll
      for (int r = 0; r < RPT; ++r) wr[s][r].template load<NT>(W + (size_t)(row0 + r) * p.K + k);
    }
  }
  // (2a) gather mode: resolve the rows' codes from the producer's arg-max partials
  if (p.xpart) {
    for (int m = wave; m < p.M; m += 4) {
      const int bb = p.x_step1 ? (m >> 1) : m;
      if (p.x_step1 && !(m & 1)) continue;
      const unsigned long long best = wave_argmax_partials(p.xpart + (size_t)bb * p.xpart_stride, p.xpart_n, lane);
      if (lane == 0) {
        const int c = min(max(unpack_argmax(best), 0), p.xV - 1);
        gcode[m] = c;
        if (blockIdx.x == 0) p.x_codes[(size_t)bb * p.x_codes_K + p.xcb] = c;
      }
    }
    __syncthreads();
  }
  // (2b) stage x (* norm weight) into LDS; sum(x^2) per row once per block
  float ssp[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    ssp[i] = 0.f;
    if (i < p.M) {
      const bool gathered = p.xpart && !(p.x_step1 && !(i & 1));
      const size_t trow = gathered ? ((size_t)gcode[i] + (size_t)p.xV * p.xcb) * p.K : 0;
      const bool g16 = gathered && !p.xtab_f32;
      const WT* xw = g16 ? (const WT*)p.xtab + trow : nullptr;
      const float* xf = gathered ? (const float*)p.xtab + trow : p.x + (size_t)(p.x_step1 ? (i >> 1) : i) * p.xs;
      float* xc = (p.x_copy && blockIdx.x == 0) ? p.x_copy + (size_t)i * p.K : nullptr;
      for (int k = tid * 8; k < p.K; k += 256 * 8) {
        float xv[8];
        if (g16) W8<WT>::load(xw + k, xv);
        else W8<float>::load(xf + k, xv);
        if (xc) {
          *reinterpret_cast<float4*>(xc + k) = make_float4(xv[0], xv[1], xv[2], xv[3]);
          *reinterpret_cast<float4*>(xc + k + 4) = make_float4(xv[4], xv[5], xv[6], xv[7]);
        }
        if (norm) {
          float nw[8];
          W8<float>::load(p.nw + k, nw);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            ssp[i] = fmaf(xv[j], xv[j], ssp[i]);
            xv[j] *= nw[j];
          }
        }
        *reinterpret_cast<float4*>(&xl[i][k]) = make_float4(xv[0], xv[1], xv[2], xv[3]);
        *reinterpret_cast<float4*>(&xl[i][k + 4]) = make_float4(xv[4], xv[5], xv[6], xv[7]);
      }
    }
    if (norm) {
      const float v = wave_sum(ssp[i]);
      if (lane == 0) rss[wave][i] = v;
    }
  }
  __syncthreads();
  // (3) dot products from LDS
  float acc[MT][RPT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < RPT; ++r) acc[i][r] = 0.f;
#pragma unroll
  for (int s = 0; s < NKM; ++s) {
    const int k = gt * 8 + s * G * 8;
    if (k < p.K) {
      float w[RPT][8];
#pragma unroll
      for (int r = 0; r < RPT; ++r) wr[s][r].get(w[r]);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if (i < p.M) {
          const float4 x0 = *reinterpret_cast<const float4*>(&xl[i][k]);
          const float4 x1 = *reinterpret_cast<const float4*>(&xl[i][k + 4]);
          const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
          for (int r = 0; r < RPT; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][r] = fmaf(w[r][j], xv[j], acc[i][r]);
        }
      }
    }
  }
  // (4) reduce: wave shuffles, then the G/64 waves of each group through LDS; pair epilogues
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      const float v = wave_sum(acc[i][r]);
      if (lane == 0) red[wave][i][r] = v;
    }
  __syncthreads();
  constexpr int WPG = G / 64;
  constexpr int NPAIR = NG * MT * (RPT / 2);
  unsigned long long akey = 0;
  int arow = -1;
  if (tid < NPAIR) {
    const int g = tid / (MT * (RPT / 2));
    const int rem = tid % (MT * (RPT / 2));
    const int i = rem / (RPT / 2), rp = (rem % (RPT / 2)) * 2;
    if (i < p.M) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w = 0; w < WPG; ++w) {
        a += red[g * WPG + w][i][rp];
        b += red[g * WPG + w][i][rp + 1];
      }
      if (norm) {
        const float sq = (rss[0][i] + rss[1][i]) + (rss[2][i] + rss[3][i]);
        const float sc = rsqrtf(sq / (float)p.K + p.eps);
        a *= sc;
        b *= sc;
      }
      const int n = blockIdx.x * RPB + g * RPT + rp;
      gemv_epilogue_pair(p, i, n, a, b);
      if (p.epi == EPI_ARGMAX) {
        unsigned long long key = 0;
        if (n < p.n_valid) key = pack_argmax(a, n);
        if (n + 1 < p.n_valid) {
          const unsigned long long kb = pack_argmax(b, n + 1);
          key = kb > key ? kb : key;
        }
        akey = key;
        arow = i;
      }
    }
  }
  if (p.epi == EPI_ARGMAX && wave == 0) {  // block arg-max per row -> partial slot
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      unsigned long long v = (tid < NPAIR && arow == i) ? akey : 0ull;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = __shfl_xor(v, o, 64);
        v = w > v ? w : v;
      }
      if (lane == 0 && i < p.M) p.part[(size_t)i * p.part_stride + blockIdx.x] = v;
    }
  }
}

// ============================================================================ attention
// Decode-shaped GQA attention for one (query row m, kv head) per 256-thread block; wave w serves
// q head kvh*G + w (G = Hq/Hkv <= 4).  Keys [k0, k1] of utterance b(m) stream through LDS in chunks
// of 64 rows; the chunk loads are software-pipelined through registers (chunk c+1 is in flight while
// chunk c is scored), all 256 threads issuing coalesced 16-B loads.  Each wave scores its head
// (lane = key, K rows padded by 16 B: conflict-free ds_read_b128), online softmax in fp32, and
// P.V with lane = head dim reading V rows from LDS.
// One wave scores one head against a chunk of n <= 64 keys held in LDS (K rows padded to KP floats,
// V rows HD floats) with online-softmax state (m_run, l_run, o).  The q.k dot runs as four
// independent FMA chains (one per float4 lane) and P.V broadcasts p_j with v_readlane (scalar, no
// LDS round trip) four keys at a time so the V reads are in flight together: the single-chain /
// ds_bpermute form spent ~3 us of dependent latency per head at 32 keys.
template <int HD>
__device__ __forceinline__ void attn_chunk(const float* qr_, const float* Kc, const float* Vc, int n, int lane,
                                           float& m_run, float& l_run, float (&o)[HD / 64]) {
  constexpr int KP = HD + 4, V4 = HD / 4, NO = HD / 64;
  float s = -INFINITY;
  if (lane < n) {
    const float4* kr = reinterpret_cast<const float4*>(Kc + lane * KP);
    const float4* qr = reinterpret_cast<const float4*>(qr_);
    float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
#pragma unroll
    for (int d4 = 0; d4 < V4; ++d4) {
      const float4 a = kr[d4], q4 = qr[d4];
      d0 = fmaf(q4.x, a.x, d0);
      d1 = fmaf(q4.y, a.y, d1);
      d2 = fmaf(q4.z, a.z, d2);
      d3 = fmaf(q4.w, a.w, d3);
    }
    s = (d0 + d1) + (d2 + d3);
  }
  const float new_m = fmaxf(m_run, wave_max(s));
  const float alpha = (m_run == -INFINITY) ? 0.f : expf(m_run - new_m);
  const float pj = (lane < n) ? expf(s - new_m) : 0.f;
  l_run = l_run * alpha + wave_sum(pj);
#pragma unroll
  for (int i = 0; i < NO; ++i) o[i] *= alpha;
  const int pji = __float_as_int(pj);
  int j = 0;
  for (; j + 4 <= n; j += 4) {
    float v[4][NO];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < NO; ++i) v[u][i] = Vc[(j + u) * HD + lane + 64 * i];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float pb = __int_as_float(__builtin_amdgcn_readlane(pji, j + u));
#pragma unroll
      for (int i = 0; i < NO; ++i) o[i] = fmaf(pb, v[u][i], o[i]);
    }
  }
  for (; j < n; ++j) {
    const float pb = __int_as_float(__builtin_amdgcn_readlane(pji, j));
#pragma unroll
    for (int i = 0; i < NO; ++i) o[i] = fmaf(pb, Vc[j * HD + lane + 64 * i], o[i]);
  }
  m_run = new_m;
}

template <int HD>
struct AttnLds {
  float Ks[64 * (HD + 4)];
  float Vs[64 * HD];
  float qs[4][HD];
};

// Half-group sums of one wave's 64 consecutive split values (column c0 + lane): a butterfly over each
// 32-lane half (every lane of a half ends with the same sum), written by lanes 0 and 32.
__device__ __forceinline__ void xs_half_sum(float* hs, int m, int c0, float v, int lane) {
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);
  if ((lane & 31) == 0) hs[(size_t)((c0 + lane) / 32) * xs::HS_ROWS + m] = v;
}

template <int HD>
__device__ __forceinline__ void attn_block(const AttnParams& p, int m, int kvh, AttnLds<HD>& L) {
  constexpr int KP = HD + 4;  // padded K row (floats)
  constexpr int V4 = HD / 4;  // float4 per row
  constexpr int PER = 64 * V4 / 256;  // float4 per thread per tensor for a full chunk (4 or 8)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = p.Hq / p.Hkv;
  const int h = kvh * G + wave;
  const bool head_ok = wave < G;
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
  const float* qrow = p.q + (size_t)m * p.qs;
  if (p.g_tab) {  // decoder layer 0, steps >= 2: gather this row's QKV from the layer-0 table
    __shared__ int gcode;
    if (wave == 0) {
      const unsigned long long best = wave_argmax_partials(p.g_part + (size_t)b * p.g_part_stride, p.g_part_n, lane);
      if (lane == 0) gcode = min(max(unpack_argmax(best), 0), p.g_V - 1);
    }
    __syncthreads();
    const int c = gcode;
    const float* trow = p.g_tab + (size_t)c * p.g_row;
    qrow = trow;
    const int qd = p.Hq * HD, kvd = p.Hkv * HD;
    float* kd = const_cast<float*>(p.kc) + (((size_t)b * p.Hkv + kvh) * p.S_cap + pos) * HD;
    float* vd = const_cast<float*>(p.vc) + (((size_t)b * p.Hkv + kvh) * p.S_cap + pos) * HD;
    for (int d = tid; d < HD; d += 256) {
      kd[d] = trow[qd + kvh * HD + d];
      vd[d] = trow[qd + kvd + kvh * HD + d];
    }
    if (kvh == 0) {
      if (tid == 0) p.g_codes[(size_t)b * p.g_codes_K + p.g_cb] = c;
      const float* xs = p.g_xtab + (size_t)c * p.g_D;
      float* xo = p.g_xout + (size_t)m * p.g_D;
      for (int d = tid * 4; d < p.g_D; d += 256 * 4)
        *reinterpret_cast<float4*>(xo + d) = *reinterpret_cast<const float4*>(xs + d);
    }
    __syncthreads();  // the K/V row at pos is visible to this block's fetches below
  }
  const float* K = p.kc + ((size_t)b * p.Hkv + kvh) * p.S_cap * HD;
  const float* V = p.vc + ((size_t)b * p.Hkv + kvh) * p.S_cap * HD;
  // chunk loads through registers; rows past the live range re-read the last live row (always a
  // valid address), so the register array is written unconditionally and stays in VGPRs.
  // Native ext-vector (not HIP's float4 struct, whose copies lower to memcpy and defeat SROA).
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  f32x4 kk[PER], vv[PER];
  auto fetch = [&](const int c_) {
    const int n_ = min(64, k1 - c_ + 1);
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int t = u * 256 + tid, j = min(t / V4, n_ - 1), d4 = t % V4;
      kk[u] = *reinterpret_cast<const f32x4*>(K + (size_t)(c_ + j) * HD + d4 * 4);
      vv[u] = *reinterpret_cast<const f32x4*>(V + (size_t)(c_ + j) * HD + d4 * 4);
    }
  };
  fetch(k0);  // first chunk in flight together with q
  if (head_ok) {
    const float* q = qrow + h * HD;
    for (int d = lane; d < HD; d += 64) L.qs[wave][d] = q[d] * p.scale;
  }
  constexpr int NO = HD / 64;
  float o[NO];
#pragma unroll
  for (int i = 0; i < NO; ++i) o[i] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  for (int c = k0; c <= k1; c += 64) {
    const int n = min(64, k1 - c + 1);
    __syncthreads();  // previous chunk consumed (and qs visible on the first pass)
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int t = u * 256 + tid, j = t / V4, d4 = t % V4;
      if (j < n) {
        *reinterpret_cast<f32x4*>(&L.Ks[j * KP + d4 * 4]) = kk[u];
        *reinterpret_cast<f32x4*>(&L.Vs[j * HD + d4 * 4]) = vv[u];
      }
    }
    __syncthreads();
    fetch(min(c + 64, k1));  // next chunk streams while this one is scored (clamped: unconditional)
    if (!head_ok) continue;
    attn_chunk<HD>(L.qs[wave], L.Ks, L.Vs, n, lane, m_run, l_run, o);
  }
  if (!head_ok) return;
  const float inv = 1.f / l_run;
  float* out = p.out + (size_t)m * p.os + h * HD;
#pragma unroll
  for (int i = 0; i < NO; ++i) {
    out[lane + 64 * i] = o[i] * inv;
    if (p.xs_out) {  // streaming o_proj (+ half-group sums for an int4 one)
      xs::store1(p.xs_out, p.xs_K, m, h * HD + lane + 64 * i, o[i] * inv);
      if (p.hs_out) xs_half_sum(p.hs_out, m, h * HD + 64 * i, o[i] * inv, lane);
    }
  }
}

// Short causal attention (depth decoder: <= 32 cached positions, generation.py:70-77): one wave per
// (row, q head); lanes (key j, half of the head dims) compute the scores.  Every K half-row and V row
// is loaded up front with 16-B loads straight to VGPRs -- one memory round trip instead of
// attn_block's staged chunk pipeline.  P.V (as dec_frame's DF_PV 2): lane = (key half kv = lane >> 5:
// keys 16 kv .. 16 kv + 15, dims 4 dq .. 4 dq + 3, dq = lane & 31), so a key's V row is one 16-B load
// per lane (16 loads per wave instead of 64 of 4 B); each half sums its keys in order and the halves
// are added once (keys 0-15 first); lanes dq < 32 return dims 4 dq .. 4 dq + 3.  fp32 throughout:
// scores, softmax (max-subtracted, one pass: all keys fit one wave).  With g_tab set (decoder layer 0,
// codebook steps >= 2) the row's q and its key/value at pos come from the folded layer-0 table (see
// AttnParams).
template <int HD, int NMAX>
__device__ __forceinline__ void attn_short_head(const AttnParams& p, int m, int h, int lane, float* qsh,
                                                float (&o)[4], bool write_kv, bool write_code, bool copy_res,
                                                int* code_out) {
  static_assert(HD == 128 && NMAX == 32, "key halves of 16 x 32 lanes x 4 dims");
  constexpr int V4 = HD / 4;
  const int G = p.Hq / p.Hkv, kvh = h / G;
  const int b = p.rm.b(m), pos = p.rm.pos(m);
  const int n = pos + 1;
  const float* K = p.kc + ((size_t)b * p.Hkv + kvh) * p.S_cap * HD;
  const float* V = p.vc + ((size_t)b * p.Hkv + kvh) * p.S_cap * HD;
  const bool gath = p.g_tab != nullptr;
  const int jc = gath ? pos : n;  // keys read from the cache (the gathered row's own key comes from the table)
  // cached keys / values first (independent of the gathered code).  Scores: lane = (key kj = lane & 31,
  // half hh = lane >> 5 of the head dims); the two halves' partial dots are added with one shuffle.
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  constexpr int H4 = V4 / 2;
  const int kj = lane & 31, hh = lane >> 5;
  f32x4 kr[H4];
  const int jl = min(kj, max(jc - 1, 0));
  const f32x4* ksrc = reinterpret_cast<const f32x4*>(K + (size_t)jl * HD + hh * (HD / 2));
#pragma unroll
  for (int d4 = 0; d4 < H4; ++d4) kr[d4] = ksrc[d4];
  const int kv = lane >> 5, dq = lane & 31;
  f32x4 vv[NMAX / 2];
#pragma unroll
  for (int u = 0; u < NMAX / 2; ++u) {
    const int j = 16 * kv + u;
    vv[u] = (j < jc) ? *reinterpret_cast<const f32x4*>(V + (size_t)j * HD + 4 * dq) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const float* qrow = p.q + (size_t)m * p.qs;
  if (gath) {
    const unsigned long long best = wave_argmax_partials(p.g_part + (size_t)b * p.g_part_stride, p.g_part_n, lane);
    const int c = min(max(unpack_argmax(best), 0), p.g_V - 1);
    if (code_out) *code_out = c;
    const float* trow = p.g_tab + (size_t)c * p.g_row;
    qrow = trow;
    const int qd = p.Hq * HD, kvd = p.Hkv * HD;
    const float* tk = trow + qd + kvh * HD;
    const float* tv = trow + qd + kvd + kvh * HD;
    if (kj == pos) {
      const f32x4* t4 = reinterpret_cast<const f32x4*>(tk + hh * (HD / 2));
#pragma unroll
      for (int d4 = 0; d4 < H4; ++d4) kr[d4] = t4[d4];
    }
#pragma unroll
    for (int u = 0; u < NMAX / 2; ++u)
      if (16 * kv + u == pos) vv[u] = *reinterpret_cast<const f32x4*>(tv + 4 * dq);
    if (write_kv && h % G == 0) {  // this kv head's K/V row at pos -> cache (read by the later codebook steps)
      float* kd = const_cast<float*>(K) + (size_t)pos * HD;
      float* vd = const_cast<float*>(V) + (size_t)pos * HD;
      for (int d = lane; d < HD; d += 64) {
        kd[d] = tk[d];
        vd[d] = tv[d];
      }
    }
    if (write_code && h == 0 && lane == 0) p.g_codes[(size_t)b * p.g_codes_K + p.g_cb] = c;
    if (copy_res && h == 0) {
      const float* xs = p.g_xtab + (size_t)c * p.g_D;
      float* xo = p.g_xout + (size_t)m * p.g_D;
      for (int d = lane * 4; d < p.g_D; d += 64 * 4)
        *reinterpret_cast<float4*>(xo + d) = *reinterpret_cast<const float4*>(xs + d);
    }
  }
  for (int d = lane; d < HD; d += 64) qsh[d] = qrow[h * HD + d] * p.scale;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // scores (fp32), softmax over the n live keys, P.V in key order
  float s;
  {
    const f32x4* qr = reinterpret_cast<const f32x4*>(qsh + hh * (HD / 2));
    float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
#pragma unroll
    for (int d4 = 0; d4 < H4; ++d4) {
      const f32x4 a = kr[d4], q4 = qr[d4];
      d0 = fmaf(q4.x, a.x, d0);
      d1 = fmaf(q4.y, a.y, d1);
      d2 = fmaf(q4.z, a.z, d2);
      d3 = fmaf(q4.w, a.w, d3);
    }
    const float part = (d0 + d1) + (d2 + d3);
    const float other = __shfl_xor(part, 32, 64);
    s = hh == 0 ? part + other : other + part;  // half 0 + half 1 on both lanes of a key
    if (kj >= n) s = -INFINITY;
  }
  const float new_m = wave_max(s);
  const float pj = (kj < n) ? expf(s - new_m) : 0.f;
  const float l_run = wave_sum(hh == 0 ? pj : 0.f);
  const int pji = __float_as_int(pj);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < NMAX / 2; ++u) {
    const float pa = __int_as_float(__builtin_amdgcn_readlane(pji, u));
    const float pb = __int_as_float(__builtin_amdgcn_readlane(pji, 16 + u));
    const float pw = kv ? pb : pa;
    if (16 * kv + u < n) {
      acc.x = fmaf(pw, vv[u].x, acc.x);
      acc.y = fmaf(pw, vv[u].y, acc.y);
      acc.z = fmaf(pw, vv[u].z, acc.z);
      acc.w = fmaf(pw, vv[u].w, acc.w);
    }
  }
  const float inv = 1.f / l_run;
  const float t0 = __shfl_xor(acc.x, 32, 64), t1 = __shfl_xor(acc.y, 32, 64), t2 = __shfl_xor(acc.z, 32, 64),
              t3 = __shfl_xor(acc.w, 32, 64);
  o[0] = (acc.x + t0) * inv;  // (lanes < 32: keys 0-15 + keys 16-31)
  o[1] = (acc.y + t1) * inv;
  o[2] = (acc.z + t2) * inv;
  o[3] = (acc.w + t3) * inv;
}

template <int HD, int NMAX>
__global__ __launch_bounds__(64) void attn_short_kernel(AttnParams p) {
  __shared__ __attribute__((aligned(16))) float qsh[HD];
  const int m = blockIdx.x / p.Hq, h = blockIdx.x % p.Hq, lane = threadIdx.x, dq = lane & 31;
  float o[4];
  attn_short_head<HD, NMAX>(p, m, h, lane, qsh, o, true, true, true, nullptr);
  // half-group sums for an int4 o_proj: 32 columns = 8 lanes, each lane's 4 in column order, then
  // the lanes' sums in a butterfly (lanes 32-63 mirror 0-31 and store nothing)
  float hsum = (o[0] + o[1]) + (o[2] + o[3]);
#pragma unroll
  for (int x = 1; x < 8; x <<= 1) hsum += __shfl_xor(hsum, x, 64);
  if (lane < 32) {
    float* out = p.out + (size_t)m * p.os + h * HD + 4 * dq;
    *reinterpret_cast<float4*>(out) = make_float4(o[0], o[1], o[2], o[3]);
    if (p.xs_out) {  // the operand of the streaming o_proj GEMM (gemm_xs.hip)
      xs::store4(p.xs_out, p.xs_K, m, h * HD + 4 * dq, o);
      if (p.hs_out && (dq & 7) == 0) p.hs_out[(size_t)((h * HD + 4 * dq) / 32) * xs::HS_ROWS + m] = hsum;
    }
  }
}

template <int HD>
__global__ __launch_bounds__(256) void attn_kernel(AttnParams p) {
  __shared__ __attribute__((aligned(16))) AttnLds<HD> L;
  attn_block<HD>(p, blockIdx.x / p.Hkv, blockIdx.x % p.Hkv, L);
}

// Prompt-prefill causal attention on the fp32 matrix cores (v_mfma_f32_32x32x2f32).  A prompt's rows
// are one utterance at consecutive positions, so one 256-thread block takes a tile of <= 64 of them
// and one kv head; wave w = q head kvh*G + w over the tile's two 32-row MFMA tiles.  Keys 0 .. the
// tile's last position stream through LDS in 64-key chunks, the next chunk's loads in flight in
// registers while this one is scored (as attn_block).  Scores are computed transposed, S^T = K Q^T:
// accumulator register r of lane (c, hh) is query row c against key (r & 3) + 8 (r >> 2) + 4 hh, so
// a row's online-softmax max / sum are the lane's own registers plus one swap with lane ^ 32, and the
// same registers are the B operand of O^T = V^T P^T once the MFMA K steps walk the keys in that order
// (step s, half hh <-> key (s & 3) + 8 (s >> 2) + 4 hh; the score steps walk dims 32 hh + s).  fp32
// products and fp32 accumulation as attn_block, summed in another order.  attn_block runs one
// (row, kv head) per block: config 5's 15,872 prompt rows were 127k blocks and ~26 ms of latency
// chains (profiles/r04_prof_config5_prefill_codec.txt).
template <int HD>
__global__ __launch_bounds__(256) void attn_prefill_kernel(AttnParams p) {
  static_assert(HD == 64, "one 64-dim head per wave: 32 K steps over dims, two 32-dim output tiles");
  constexpr int KP = HD + 4, V4 = HD / 4, PER = 64 * V4 / 256;
  __shared__ __attribute__((aligned(16))) float Ks[64 * KP];
  __shared__ __attribute__((aligned(16))) float Vs[64 * HD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, c32 = lane & 31, hh = lane >> 5;
  const int kvh = blockIdx.x % p.Hkv, tile = blockIdx.x / p.Hkv;
  int m0, n;
  if (p.rm.tiles) {
    const int2 tl = p.rm.tiles[tile];
    m0 = tl.x;
    n = tl.y;
  } else {  // uniform calls (the codec transformer): rm.T rows per utterance, ceil(T / 64) tiles each
    const int tpu = (p.rm.T + 63) / 64, r0 = 64 * (tile % tpu);
    m0 = (tile / tpu) * p.rm.T + r0;
    n = min(64, p.rm.T - r0);
  }
  const int G = p.Hq / p.Hkv;
  const bool head_ok = wave < G;
  const int h = kvh * G + min(wave, G - 1);
  const int b = p.rm.b(m0), pos0 = p.rm.pos(m0);
  // keys kbeg .. kmax: causal -- 0 .. the tile's last position, each row masked past its own; ATTN_BLOCK
  // (moshi_mlx, as attn_block) -- every row of the call sees the call's keys and `window` past ones
  int kbeg = 0, kmax = pos0 + n - 1;
  if (p.mode == ATTN_BLOCK) {
    const int off = pos0 - (m0 % p.rm.T);
    kbeg = max(0, off - p.window);
    kmax = off + p.rm.T - 1;
  }
  const float* K = p.kc + ((size_t)b * p.Hkv + kvh) * p.S_cap * HD;
  const float* V = p.vc + ((size_t)b * p.Hkv + kvh) * p.S_cap * HD;
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  f32x4 kk[PER], vv[PER];
  auto fetch = [&](int c_) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int t = u * 256 + tid, j = min(c_ + t / V4, kmax), d4 = t % V4;
      kk[u] = *reinterpret_cast<const f32x4*>(K + (size_t)j * HD + d4 * 4);
      vv[u] = *reinterpret_cast<const f32x4*>(V + (size_t)j * HD + d4 * 4);
    }
  };
  fetch(kbeg);
  // this lane's query rows (clamped: rows past the tile repeat its last row, never stored), scaled,
  // dims 32 hh .. 32 hh + 31 (the score steps' B operand)
  float qv[2][HD / 2];
  int rpos[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int r = min(32 * rt + c32, n - 1);
    rpos[rt] = p.mode == ATTN_BLOCK ? kmax : pos0 + r;
    const f32x4* qp = reinterpret_cast<const f32x4*>(p.q + (size_t)(m0 + r) * p.qs + h * HD + 32 * hh);
#pragma unroll
    for (int s4 = 0; s4 < HD / 8; ++s4) {
      const f32x4 v = qp[s4];
      qv[rt][4 * s4] = v.x * p.scale;
      qv[rt][4 * s4 + 1] = v.y * p.scale;
      qv[rt][4 * s4 + 2] = v.z * p.scale;
      qv[rt][4 * s4 + 3] = v.w * p.scale;
    }
  }
  f32x16 o[2][2];
  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) o[rt][dt] = f32x16{};
  for (int c = kbeg; c <= kmax; c += 64) {
    __syncthreads();  // the previous chunk consumed
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int t = u * 256 + tid, j = t / V4, d4 = t % V4;
      *reinterpret_cast<f32x4*>(&Ks[j * KP + d4 * 4]) = kk[u];
      *reinterpret_cast<f32x4*>(&Vs[j * HD + d4 * 4]) = vv[u];
    }
    __syncthreads();
    fetch(min(c + 64, kmax));  // (clamped: unconditional)
    if (!head_ok) continue;
    f32x16 sc[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      float ka[HD / 2];
#pragma unroll
      for (int s4 = 0; s4 < HD / 8; ++s4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(&Ks[(32 * kt + c32) * KP + 32 * hh + 4 * s4]);
        ka[4 * s4] = v.x; ka[4 * s4 + 1] = v.y; ka[4 * s4 + 2] = v.z; ka[4 * s4 + 3] = v.w;
      }
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) sc[rt][kt] = f32x16{};
#pragma unroll
      for (int s = 0; s < HD / 2; ++s)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) sc[rt][kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(ka[s], qv[rt][s], sc[rt][kt], 0, 0, 0);
    }
    // online softmax per query row (this lane's column), causal mask key > row position
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = c + 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (key > rpos[rt]) sc[rt][kt][r] = -INFINITY;
          mx = fmaxf(mx, sc[rt][kt][r]);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float new_m = fmaxf(m_run[rt], mx);
      const float alpha = (m_run[rt] == -INFINITY) ? 0.f : expf(m_run[rt] - new_m);
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pj = expf(sc[rt][kt][r] - new_m);
          sc[rt][kt][r] = pj;
          rs += pj;
        }
      rs += __shfl_xor(rs, 32, 64);
      l_run[rt] = l_run[rt] * alpha + rs;
      m_run[rt] = new_m;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) o[rt][dt] *= alpha;
    }
    // O^T[dim][row] += V[key][dim] P[row][key], K steps in the score registers' key order
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int key = 32 * kt + (s & 3) + 8 * (s >> 2) + 4 * hh;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const float va = Vs[key * HD + 32 * dt + c32];
#pragma unroll
          for (int rt = 0; rt < 2; ++rt) o[rt][dt] = __builtin_amdgcn_mfma_f32_32x32x2f32(va, sc[rt][kt][s], o[rt][dt], 0, 0, 0);
        }
      }
  }
  if (!head_ok) return;
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int r = 32 * rt + c32;
    if (r >= n) continue;
    const float inv = 1.f / l_run[rt];
    float* out = p.out + (size_t)(m0 + r) * p.os + h * HD;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4)
        *reinterpret_cast<f32x4*>(out + 32 * dt + 8 * r4 + 4 * hh) =
            f32x4{o[rt][dt][4 * r4] * inv, o[rt][dt][4 * r4 + 1] * inv, o[rt][dt][4 * r4 + 2] * inv, o[rt][dt][4 * r4 + 3] * inv};
  }
}

// ============================================================================ rmsnorm rows
// out[m] = rmsnorm(x[row(m)]) ; optionally also scatter to dec_in[2m] (decoder step-1 rows).
__global__ __launch_bounds__(256) void rmsnorm_rows_kernel(const float* x, int xs, const float* w, float eps, int D,
                                                            float* out, int os) {
  __shared__ float red[4];
  const int m = blockIdx.x;
  const float* xr = x + (size_t)m * xs;
  auto xv = [&](int d) { return xr[d]; };
  float ss = 0.f;
  for (int d = threadIdx.x; d < D; d += blockDim.x) ss += xv(d) * xv(d);
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float sc = rsqrtf(tot / (float)D + eps);
  for (int d = threadIdx.x; d < D; d += blockDim.x) out[(size_t)m * os + d] = xv(d) * sc * w[d];
}

// ============================================================================ sampling

// (value, index) arg-max with the first-max tie rule of mx.argmax
template <typename T>
__device__ __forceinline__ void argmax_merge(T& v, int& i, T ov, int oi) {
  if (ov > v || (ov == v && oi < i)) {
    v = ov;
    i = oi;
  }
}
template <typename T>
__device__ __forceinline__ int block_argmax(T v, int i, T* sv, int* si) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const T ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(i, o, 64);
    argmax_merge(v, i, ov, oi);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    sv[wave] = v;
    si[wave] = i;
  }
  __syncthreads();
  T bv = sv[0];
  int bi = si[0];
  for (int w = 1; w < 4; ++w) argmax_merge(bv, bi, sv[w], si[w]);
  return bi;
}

// One block per utterance.  Greedy: first max (mx.argmax, generation.py:51-52).  Else Gumbel-max
// over logits*(1/temp) restricted to values >= the top_k-th largest (radix select) -- mlx_lm
// make_sampler(temp, top_k) semantics with the build's counter-based RNG.  The chosen code's
// audio embedding (embed_audio, models.py:79-80) is gathered into the next decoder input row.
constexpr int SAMPLE_NPT = 16;  // logits per thread: V <= 4096 (checked at launch)
constexpr int SAMPLE_CMAX = 512;  // compacted top-k survivors (more ties than this: the in-place loop)
// The top_k-th largest of a 256-thread block's logits (lv[i] = logit tid + 256 i, i < SAMPLE_NPT):
// radix select of its order-preserving key, 8 bits per pass; the digit is found by a parallel suffix
// count over the 256 bins (thread t holds digit 255 - t), not a serial scan.  Every logit >= the
// result is in the top-k set (ties at the k-th value kept).
__device__ float topk_threshold_256(const float (&lv)[SAMPLE_NPT], int V, int k, uint32_t* hist, uint32_t* wsum,
                                    uint32_t* sh) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t prefix = 0, maskbits = 0, rem = (uint32_t)k;
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < SAMPLE_NPT; ++i) {
      const uint32_t key = f2key(lv[i]);
      if (tid + 256 * i < V && (key & maskbits) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    const uint32_t h = hist[255 - tid];
    uint32_t c = h;  // inclusive prefix over t = count of keys with digit >= 255 - t
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(c, o, 64);
      if (lane >= o) c += u;
    }
    if (lane == 63) wsum[wave] = c;
    __syncthreads();
    for (int w = 0; w < wave; ++w) c += wsum[w];
    const uint32_t above = c - h;
    if (h > 0 && above < rem && rem <= c) {  // exactly one digit
      sh[0] = prefix | ((uint32_t)(255 - tid) << shift);
      sh[1] = rem - above;
    }
    __syncthreads();
    prefix = sh[0];
    rem = sh[1];
    maskbits |= 255u << shift;
    __syncthreads();  // hist / sh reused by the next pass
  }
  return key2f(prefix);
}

template <typename WT>
__global__ __launch_bounds__(256) void sample_kernel(SampleParams p) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t sh[2];
  __shared__ double sdv[4];
  __shared__ float sfv[4];
  __shared__ int si[4];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const float* lg = p.logits + (size_t)b * p.ls;
  const int V = p.V;
  int code;
  if (p.forced) {  // block-uniform: no barrier below is reached by part of the block
    if (tid == 0) {
      code = min(max(p.forced[(size_t)b * p.K + p.cb], 0), V - 1);
      p.codes[(size_t)b * p.K + p.cb] = code;
      if (p.part) p.part[(size_t)b * p.part_stride] = pack_argmax(0.f, code);
    }
    return;
  }
  if (p.temperature <= 0.f) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int v = tid; v < V; v += 256) {
      const float l = lg[v];
      if (l > best) {  // increasing v per thread: first max kept
        best = l;
        bi = v;
      }
    }
    code = block_argmax<float>(best, bi, sfv, si);
  } else {
    // the row's logits stay in registers for the radix passes and the Gumbel pass
    float lv[SAMPLE_NPT];
#pragma unroll
    for (int i = 0; i < SAMPLE_NPT; ++i) {
      const int v = tid + 256 * i;
      lv[i] = v < V ? lg[v] : 0.f;
    }
    const bool topk = p.top_k > 0 && p.top_k < V;
    const float thr = topk ? topk_threshold_256(lv, V, p.top_k, hist, wsum, sh) : -INFINITY;
    const uint64_t key = gumbel_key(p.seeds[b], p.frame_ctr[0] * p.K + p.cb);
    const float inv_t = 1.0f / p.temperature;
    double best = -INFINITY;
    int bi = 0x7fffffff;
    // With a top-k threshold the kept entries (k plus ties, ~2 % of the row) are compacted into LDS
    // first, so the double-precision Gumbel noise is drawn for them alone: in place, nearly every wave
    // had a kept entry in nearly every slot and paid the two double logs for all 16 slots.  The
    // winner is the same -- max perturbed value, lowest index on ties -- whatever the visiting order.
    __shared__ int cidx[SAMPLE_CMAX];
    __shared__ float clv[SAMPLE_CMAX];
    __shared__ int wcnt[4];
    int kept_n = SAMPLE_CMAX + 1;
    if (topk) {
      const int lane = tid & 63, wave = tid >> 6;
      const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
      uint64_t mk[SAMPLE_NPT];
      int mine = 0;
#pragma unroll
      for (int i = 0; i < SAMPLE_NPT; ++i) {
        mk[i] = __ballot(tid + 256 * i < V && lv[i] >= thr);
        mine += __popcll(mk[i]);
      }
      if (lane == 0) wcnt[wave] = mine;
      __syncthreads();
      int base = 0;
      kept_n = 0;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        base += w < wave ? wcnt[w] : 0;
        kept_n += wcnt[w];
      }
      if (kept_n <= SAMPLE_CMAX) {
#pragma unroll
        for (int i = 0; i < SAMPLE_NPT; ++i) {
          if ((mk[i] >> lane) & 1ull) {
            const int at = base + __popcll(mk[i] & below);
            cidx[at] = tid + 256 * i;
            clv[at] = lv[i];
          }
          base += __popcll(mk[i]);
        }
      }
      __syncthreads();
    }
    if (kept_n <= SAMPLE_CMAX) {
      for (int j = tid; j < kept_n; j += 256) {
        const int v = cidx[j];
        const double val = gumbel_perturbed(clv[j], inv_t, key, v);
        if (val > best || (val == best && v < bi)) {
          best = val;
          bi = v;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < SAMPLE_NPT; ++i) {
        const int v = tid + 256 * i;
        const float l = lv[i];
        if (v >= V || !(l >= thr)) continue;
        const double val = gumbel_perturbed(l, inv_t, key, v);
        if (val > best) {
          best = val;
          bi = v;
        }
      }
    }
    code = block_argmax<double>(best, bi, sdv, si);
  }
  // NaN logits leave no winner; clamp so a bad row can never index outside the embedding table
  code = min(max(code, 0), V - 1);
  if (tid == 0) {
    p.codes[(size_t)b * p.K + p.cb] = code;
    if (p.part) p.part[(size_t)b * p.part_stride] = pack_argmax(0.f, code);  // consumed as a 1-entry partial
  }
}

// Sampling with mlx_lm's filter chain beyond top-k (make_sampler(temp, top_p, min_p,
// min_tokens_to_keep, top_k): apply_top_k -> apply_top_p -> apply_min_p -> categorical), restated in
// oracle/csm_oracle.py filter_keep on the log-probabilities lp = logits - logsumexp(logits).  One
// block per utterance: the top-k threshold (radix select), lse (fixed-order block sums), a bitonic
// sort of (lp desc, index asc) in LDS, the ascending cumulative probability of the kept entries as
// suffix sums of that order (top_p), the min_p cut against the best kept lp with the first
// min_keep ranks always kept, then the Gumbel-max of sample_kernel over the survivors.
constexpr int SORT_N = 256 * SAMPLE_NPT;  // 4096 >= V
__global__ __launch_bounds__(256) void sample_filtered_kernel(SampleParams p) {
  __shared__ unsigned long long srt[SORT_N];  // (key(l) << 32) | ~index, sorted descending
  __shared__ float lgs[SORT_N];               // the row's logits by index
  __shared__ uint8_t keep[SORT_N];
  __shared__ uint32_t hist[256];
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t sh[2];
  __shared__ float fred[8];
  __shared__ double sdv[4];
  __shared__ int si[4];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* lg = p.logits + (size_t)b * p.ls;
  const int V = p.V;
  float lv[SAMPLE_NPT];
#pragma unroll
  for (int i = 0; i < SAMPLE_NPT; ++i) {
    const int v = tid + 256 * i;
    lv[i] = v < V ? lg[v] : -INFINITY;
    lgs[v] = lv[i];
    keep[v] = 0;
  }
  const float thr = (p.top_k > 0 && p.top_k < V) ? topk_threshold_256(lv, V, p.top_k, hist, wsum, sh) : -INFINITY;
  // lse = max + log(sum exp(l - max)) over the valid logits (per-thread sums in i order, waves by
  // DPP reductions, the 4 waves in order)
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < SAMPLE_NPT; ++i) mx = fmaxf(mx, lv[i]);
  mx = wave_max(mx);
  if (lane == 0) fred[wave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(fred[0], fred[1]), fmaxf(fred[2], fred[3]));
  float se = 0.f;
#pragma unroll
  for (int i = 0; i < SAMPLE_NPT; ++i)
    if (tid + 256 * i < V) se += expf(lv[i] - mx);
  se = wave_sum(se);
  __syncthreads();
  if (lane == 0) fred[4 + wave] = se;
  __syncthreads();
  const float lse = mx + logf(((fred[4] + fred[5]) + fred[6]) + fred[7]);
  // sort entries by (lp desc, index asc), lp = l - lse in fp32 (rounding can tie distinct logits)
#pragma unroll
  for (int i = 0; i < SAMPLE_NPT; ++i) {
    const int v = tid + 256 * i;
    srt[v] = v < V ? (((unsigned long long)f2key(lv[i] - lse) << 32) | (0xFFFFFFFFu - (uint32_t)v)) : 0ull;
  }
  __syncthreads();
  for (int k = 2; k <= SORT_N; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll 4
      for (int t = tid; t < SORT_N / 2; t += 256) {
        const int i = 2 * t - (t & (j - 1)), ixj = i + j;
        const unsigned long long a = srt[i], c = srt[ixj];
        if (((i & k) == 0) ? (a < c) : (a > c)) { srt[i] = c; srt[ixj] = a; }
      }
      __syncthreads();
    }
  // thread t owns sorted positions 16t .. 16t+15
  int idx[SAMPLE_NPT];
  bool kp[SAMPLE_NPT];
  float lpv[SAMPLE_NPT];
#pragma unroll
  for (int r = 0; r < SAMPLE_NPT; ++r) {
    const unsigned long long e = srt[SAMPLE_NPT * tid + r];
    idx[r] = (int)(0xFFFFFFFFu - (uint32_t)e);
    const bool valid = e != 0ull && idx[r] < V;
    const float l = valid ? lgs[idx[r]] : -INFINITY;
    lpv[r] = l - lse;
    kp[r] = valid && l >= thr;
  }
  if (p.use_top_p) {
    // cum_asc at sorted position r = sum of exp(lp) of kept entries at positions >= r
    float suf[SAMPLE_NPT];
    float acc = 0.f;
#pragma unroll
    for (int r = SAMPLE_NPT - 1; r >= 0; --r) {
      acc += kp[r] ? expf(lpv[r]) : 0.f;
      suf[r] = acc;
    }
    // exclusive suffix of the thread totals over threads > tid: reverse inclusive scan in each
    // wave, then the later waves' totals
    float c = acc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float u = __shfl_down(c, o, 64);
      if (lane + o < 64) c += u;
    }
    __syncthreads();
    if (lane == 0) fred[wave] = c;  // wave total
    __syncthreads();
    float later = c - acc;          // threads after tid in this wave
    for (int w2 = 3; w2 > wave; --w2) later += fred[w2];
#pragma unroll
    for (int r = 0; r < SAMPLE_NPT; ++r) kp[r] = kp[r] && (suf[r] + later > p.top_p_cut);
  }
  if (p.use_min_p) {
    // the best kept lp, a block max over the kept entries (oracle filter_keep: lp[keep].max()).  Not
    // simply sorted position 0: top_k keeps by the raw logit while the sort is by the fp32-rounded
    // lp = l - lse with index-ascending ties, so a dropped entry can sort ahead of a kept one.
    float bm = -INFINITY;
#pragma unroll
    for (int r = 0; r < SAMPLE_NPT; ++r)
      if (kp[r]) bm = fmaxf(bm, lpv[r]);
    bm = wave_max(bm);
    __syncthreads();
    if (lane == 0) fred[wave] = bm;
    __syncthreads();
    const float tmin = fmaxf(fmaxf(fred[0], fred[1]), fmaxf(fred[2], fred[3])) + p.log_min_p;
#pragma unroll
    for (int r = 0; r < SAMPLE_NPT; ++r) kp[r] = kp[r] && (!(lpv[r] < tmin) || SAMPLE_NPT * tid + r < p.min_keep);
  }
#pragma unroll
  for (int r = 0; r < SAMPLE_NPT; ++r)
    if (kp[r]) keep[idx[r]] = 1;
  __syncthreads();
  const uint64_t key = gumbel_key(p.seeds[b], p.frame_ctr[0] * p.K + p.cb);
  const float inv_t = 1.0f / p.temperature;
  double best = -INFINITY;
  int bi = 0x7fffffff;
  float bl = -INFINITY;
  int bli = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < SAMPLE_NPT; ++i) {
    const int v = tid + 256 * i;
    if (v >= V) continue;
    if (lv[i] > bl) { bl = lv[i]; bli = v; }  // fallback: the arg-max when nothing survives
    if (!keep[v]) continue;
    const double val = gumbel_perturbed(lv[i], inv_t, key, v);
    if (val > best) {
      best = val;
      bi = v;
    }
  }
  int code = block_argmax<double>(best, bi, sdv, si);
  if (code == 0x7fffffff) {
    __syncthreads();
    code = block_argmax<float>(bl, bli, fred, si);
  }
  code = min(max(code, 0), V - 1);
  if (tid == 0) {
    p.codes[(size_t)b * p.K + p.cb] = code;
    if (p.part) p.part[(size_t)b * p.part_stride] = pack_argmax(0.f, code);
  }
}

// ============================================================================ advance
__global__ void advance_kernel(AdvanceParams p) {
  const int f = p.frame_ctr[0];
  if (p.last_part) {  // greedy: arg-max of the last head's block partials -> codes[b][K-1]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int b = wave; b < p.B; b += blockDim.x / 64) {
      const unsigned long long best = wave_argmax_partials(p.last_part + (size_t)b * p.last_stride, p.last_n, lane);
      if (lane == 0) p.codes[(size_t)b * p.K + p.K - 1] = min(max(unpack_argmax(best), 0), p.V - 1);
    }
    __syncthreads();
  }
  {  // one wave per utterance, lane k = codebook k (K <= 64): codes read once, history row written
     // coalesced, the all-zero test by a wave vote
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int b = wave; b < p.B; b += nw) {
      const int c = lane < p.K ? p.codes[(size_t)b * p.K + lane] : 0;
      if (lane < p.K && f < p.F_cap) p.hist[((size_t)f * p.B + b) * p.K + lane] = c;
      const bool any = __any(c != 0);
      if (lane == 0) {
        if (!any && !p.done[b]) {  // EOS: all-zero frame, not emitted (generation.py:151)
          p.done[b] = 1;
          p.n_frames[b] = f;
        }
        if (!p.done[b]) p.n_frames[b] = f + 1;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) p.frame_ctr[0] = f + 1;
}

// ============================================================================ launchers
// tiling choice (G threads per row group, RPT rows per thread)

// Measured on MI355X (tools/gemv_sweep.py, bf16, M = 1): tall gate/up matrices want one wave per
// row group (G = 64: no cross-wave reduction, 2-4 K-steps per thread); the K = 8192 down
// projections want the whole block on a row pair (G = 256 at N = 1024, 128 at N = 2048); every
// other shape is latency-bound and best at G = 128 (K >= 1024).  RPT = 2 wins everywhere at M = 1.
// LDS-staged activations for the decode regime (gemv_xl_kernel): 1 = on for K <= 2048, 3 = also the
// K = 8192 down projections (measured slower: dec down 5.96 vs 5.77 us, 231.6 vs 234.8 frames/s),
// 0 = off.  CSM_GEMV_XL overrides the default (A/B runs; read once per process).
static const int g_gemv_xl = [] { const char* e = getenv("CSM_GEMV_XL"); return e ? atoi(e) : 1; }();

static void gemv_tiling(int N, int K, int M, int& G, int& RPT) {
  (void)M;
  if (N >= 8192) G = 64;
  else if (K >= 8192) G = N <= 1024 ? 256 : 128;
  else G = K >= 1024 ? 128 : 64;
  RPT = 2;
}

template <typename WT, int TAG>
static void launch_gemv_t(const GemvParams& p, hipStream_t st) {
  int G, RPT;
  gemv_tiling(p.N, p.K, p.M, G, RPT);
  const int blocks = p.N / ((256 / G) * RPT);
  const bool mt1 = p.M == 1;
  const bool xl = g_gemv_xl && p.M <= 4 && p.K <= XL_KMAX && p.K % 8 == 0;
  // K = 8192 at M = 1 (down projections): LDS-staged x, every weight K-step in flight first
  const bool xlw = (g_gemv_xl & 2) != 0 && mt1 && p.K > XL_KMAX && p.K <= XL_KMAX_WIDE && p.K % 8 == 0 &&
                   G >= 128;
  if (xlw && G == 256 && RPT == 2) {
    hipLaunchKernelGGL((gemv_xl_kernel<WT, 256, 2, 1, TAG, XL_KMAX_WIDE>), dim3(blocks), dim3(256), 0, st, p);
    return;
  }
  if (xlw && G == 128 && RPT == 2) {
    hipLaunchKernelGGL((gemv_xl_kernel<WT, 128, 2, 1, TAG, XL_KMAX_WIDE>), dim3(blocks), dim3(256), 0, st, p);
    return;
  }
#define GEMV_L(G_, R_, M_)                                                                            \
  do {                                                                                                \
    if (xl) hipLaunchKernelGGL((gemv_xl_kernel<WT, G_, R_, M_, TAG>), dim3(blocks), dim3(256), 0, st, p); \
    else hipLaunchKernelGGL((gemv_kernel<WT, G_, R_, M_, TAG>), dim3(blocks), dim3(256), 0, st, p);  \
  } while (0)
#define GEMV_M(G_, R_) do { if (mt1) GEMV_L(G_, R_, 1); else GEMV_L(G_, R_, 4); } while (0)
#define GEMV_R(G_) do { if (RPT == 4) GEMV_M(G_, 4); else GEMV_M(G_, 2); } while (0)
  if (G == 256) GEMV_R(256);
  else if (G == 128) GEMV_R(128);
  else GEMV_R(64);
#undef GEMV_R
#undef GEMV_M
#undef GEMV_L
}

int gemv_partials(int N, int K, int M, int wdt) {
  if (gemm_mfma_eligible(N, K, M, wdt)) return gemm_tiles(N, K, M, wdt);
  const int rpb = wdt == WDT_Q4 ? gemv_q4_rows_per_block(N, K, M) : gemv_rows_per_block(N, K, M);
  return (N + rpb - 1) / rpb;
}

int gemv_rows_per_block(int N, int K, int M) {
  int G, RPT;
  gemv_tiling(N, K, M, G, RPT);
  return (256 / G) * RPT;
}

// Weight-load cache policy per stack tag (bit t set -> non-temporal loads for tag t).  The
// backbone streams 1.95 GB per frame once; the decoder's 221 MB are re-read 31x per frame and
// can stay resident in the 256 MiB Infinity Cache if the backbone stream does not evict them.
// CSM_NT_MASK overrides the default (A/B runs; read once per process).
static int gemv_nt_mask() {
  static const int m = [] { const char* e = getenv("CSM_NT_MASK"); return e ? atoi(e) : 5; }();  // backbone + heads (measured: 209.9 vs 202.0 fps all-default)
  return m;
}

// Folded-table builds (csm_engine.hip build_proj_table): every row of a table in ONE launch of
// gemv_xl_kernel<WT, 128, 2, MT, 1, KMAX> with grid.y over chunks of MT rows (MT = 14 at K <= 1024,
// 7 at K <= 2048: <= 56 KB of LDS) -- per row the arithmetic of the frame's own launch (same
// K-slices, reduction order and epilogue for every MT; without a norm also gemv_kernel's).  Other
// shapes / weight types fall back to launch_gemv in chunks of 4 rows.
int gemv_table_rows(int N, int K, int wdt, int tag) {
  int G, RPT;
  gemv_tiling(N, K, 1, G, RPT);
  const bool ok = g_gemv_xl && (wdt == WDT_BF16 || wdt == WDT_F32) && K <= 2048 && K % 8 == 0 && G == 128 &&
                  RPT == 2 && tag == 1 && !((gemv_nt_mask() >> tag) & 1);
  return ok ? (K <= 1024 ? 14 : 7) : 4;
}
void launch_gemv_table(const GemvParams& p0, int wdt, int epi, int norm, hipStream_t st, int tag) {
  const int rows = gemv_table_rows(p0.N, p0.K, wdt, tag);
  if (rows == 4 || p0.xpart) {
    for (int m0 = 0; m0 < p0.M; m0 += 4) {
      GemvParams g = p0;
      g.M = std::min(4, p0.M - m0);
      g.x = p0.x + (size_t)m0 * p0.xs;
      if (g.out) g.out = p0.out + (size_t)m0 * p0.os;
      if (g.qkv_tab) g.qkv_tab = p0.qkv_tab + (size_t)m0 * p0.N;
      launch_gemv(g, wdt, epi, norm, st, tag);
    }
    return;
  }
  GemvParams p = p0;
  p.epi = epi;
  if (!norm) p.nw = nullptr;
  p.row_chunk = rows;
  const dim3 grid(p.N / ((256 / 128) * 2), (p.M + rows - 1) / rows);
#define TAB_L(WT_, MT_, KM_) hipLaunchKernelGGL((gemv_xl_kernel<WT_, 128, 2, MT_, 1, KM_>), grid, dim3(256), 0, st, p)
  if (rows == 14) { if (wdt == WDT_BF16) TAB_L(bf16_t, 14, 1024); else TAB_L(float, 14, 1024); }
  else { if (wdt == WDT_BF16) TAB_L(bf16_t, 7, 2048); else TAB_L(float, 7, 2048); }
#undef TAB_L
}

void launch_gemv(const GemvParams& p0, int wdt, int epi, int norm, hipStream_t st, int tag) {
  GemvParams p = p0;
  p.epi = epi;
  if (!norm) p.nw = nullptr;
  const bool nt = (gemv_nt_mask() >> tag) & 1;
  if (!p.xpart && !p.x_copy && !p.no_mfma && gemm_mfma_eligible(p.N, p.K, p.M, wdt)) {
    launch_gemm_mfma(p, wdt, nt, st);
  } else if (wdt == WDT_Q4) {
    launch_gemv_q4(p, nt, st);
  } else if (wdt == WDT_BF16) {
    if (tag == 1) nt ? launch_gemv_t<bf16_t, 5>(p, st) : launch_gemv_t<bf16_t, 1>(p, st);
    else if (tag == 2) nt ? launch_gemv_t<bf16_t, 6>(p, st) : launch_gemv_t<bf16_t, 2>(p, st);
    else nt ? launch_gemv_t<bf16_t, 4>(p, st) : launch_gemv_t<bf16_t, 0>(p, st);
  } else {
    if (tag == 1) launch_gemv_t<float, 1>(p, st);
    else if (tag == 2) launch_gemv_t<float, 2>(p, st);
    else launch_gemv_t<float, 0>(p, st);
  }
}

template <typename WT>
__global__ __launch_bounds__(256) void to_f32_kernel(const WT* src, float* dst, size_t n) {
  const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= n) return;
  float v[8];
  W8<WT>::load(src + i, v);
  *reinterpret_cast<float4*>(dst + i) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(dst + i + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

void launch_to_f32(const void* src, int wdt, float* dst, size_t n, hipStream_t st) {
  const int blocks = (int)((n / 8 + 255) / 256);
  if (wdt == WDT_BF16) hipLaunchKernelGGL(to_f32_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)src, dst, n);
  else hipLaunchKernelGGL(to_f32_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)src, dst, n);
}

void launch_embed(const EmbedParams& p, int wdt, int M, hipStream_t st) {
  if (p.K + 1 > 64) throw CsmError(CSM_ERR_ARG, "embedding gather: at most 63 codebooks");
  const dim3 grid(M, (p.D + 511) / 512);
  if (wdt == WDT_BF16) hipLaunchKernelGGL(embed_rows_kernel<bf16_t>, grid, dim3(64), 0, st, p);
  else hipLaunchKernelGGL(embed_rows_kernel<float>, grid, dim3(64), 0, st, p);
}

static bool g_attn_short = [] { const char* e = getenv("CSM_ATTN_SHORT"); return !(e && e[0] == '0'); }();

void launch_attn(const AttnParams& p, int hd, hipStream_t st) {
  if (p.xs_out && p.g_tab && !(hd == 128 && p.mode == ATTN_CAUSAL && p.S_cap <= 32)) {
    fprintf(stderr, "csm: table-gathered attention with split output only on the depth decoder's short attention\n");
    abort();
  }
  if ((g_attn_short || (p.xs_out && p.g_tab)) && hd == 128 && p.mode == ATTN_CAUSAL && p.S_cap <= 32) {  // depth decoder
    hipLaunchKernelGGL((attn_short_kernel<128, 32>), dim3(p.M * p.Hq), dim3(64), 0, st, p);
    return;
  }
  // prompt rows with a tile table (csm_prefill / csm_prefill_batch) of >= 16 rows a tile on average
  if (p.rm.tiles && p.rm.ntiles > 0 && p.M >= 16 * p.rm.ntiles && hd == 64 && p.mode == ATTN_CAUSAL && !p.g_tab &&
      !p.xs_out && p.Hq / p.Hkv <= 4) {
    hipLaunchKernelGGL(attn_prefill_kernel<64>, dim3(p.rm.ntiles * p.Hkv), dim3(256), 0, st, p);
    return;
  }
  // the codec transformer's whole-call rows (Mimi encode / decode: rm.T rows per utterance, every key of
  // the call visible): the same matrix-core tiles, tiles derived from rm.T (CSM_MIMI_ATTN_TILES=0: per row)
  static const bool mimi_tiles = [] { const char* e = getenv("CSM_MIMI_ATTN_TILES"); return !(e && e[0] == '0'); }();
  if (mimi_tiles && !p.rm.tiles && !p.rm.row_b && !p.rm.row_pos && p.mode == ATTN_BLOCK && hd == 64 && !p.g_tab &&
      !p.xs_out && p.rm.T >= 16 && p.M % p.rm.T == 0 && p.Hq / p.Hkv <= 4) {
    AttnParams q = p;
    q.rm.ntiles = p.M / p.rm.T * ((p.rm.T + 63) / 64);
    hipLaunchKernelGGL(attn_prefill_kernel<64>, dim3(q.rm.ntiles * q.Hkv), dim3(256), 0, st, q);
    return;
  }
  const int blocks = p.M * p.Hkv;
  if (hd == 64) hipLaunchKernelGGL(attn_kernel<64>, dim3(blocks), dim3(256), 0, st, p);
  else if (hd == 128) hipLaunchKernelGGL(attn_kernel<128>, dim3(blocks), dim3(256), 0, st, p);
}

void launch_rmsnorm_rows(const float* x, int xs, const float* w, float eps, int D, float* out, int os, int M,
                         hipStream_t st) {
  hipLaunchKernelGGL(rmsnorm_rows_kernel, dim3(M), dim3(256), 0, st, x, xs, w, eps, D, out, os);
}

int wdc_chunk(int D) { return D == 1024 ? 16 : (D == 2048 ? 8 : 0); }

bool gemv_nt(int tag) { return (gemv_nt_mask() >> tag) & 1; }

void launch_sample(const SampleParams& p, int wdt, int B, hipStream_t st) {
  if (p.V > 256 * SAMPLE_NPT) {
    fprintf(stderr, "csm: sampler supports V <= %d (got %d)\n", 256 * SAMPLE_NPT, p.V);
    abort();
  }
  if (!p.forced && p.temperature > 0.f && (p.use_top_p || p.use_min_p)) {
    hipLaunchKernelGGL(sample_filtered_kernel, dim3(B), dim3(256), 0, st, p);
    return;
  }
  if (wdt == WDT_BF16) hipLaunchKernelGGL(sample_kernel<bf16_t>, dim3(B), dim3(256), 0, st, p);
  else hipLaunchKernelGGL(sample_kernel<float>, dim3(B), dim3(256), 0, st, p);
}

// One block per (codebook, utterance) row: max, then sum of exp(l - max) in fp32 (wave shuffles +
// a 4-entry LDS combine), lse - l[target].
__global__ __launch_bounds__(256) void forced_ce_kernel(const float* c0, const float* ci, const int* forced,
                                                        float* out, int B, int K, int V, int Vp) {
  __shared__ float red[4];
  const int cb = blockIdx.x / B, b = blockIdx.x % B;
  const float* lg = cb == 0 ? c0 + (size_t)b * Vp : ci + ((size_t)(cb - 1) * B + b) * Vp;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float m = -INFINITY;
  for (int v = tid; v < V; v += 256) m = fmaxf(m, lg[v]);
  m = wave_max(m);
  if (lane == 0) red[wave] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int v = tid; v < V; v += 256) sum += expf(lg[v] - m);
  sum = wave_sum(sum);
  if (lane == 0) red[wave] = sum;
  __syncthreads();
  if (tid == 0) {
    const int t = min(max(forced[(size_t)b * K + cb], 0), V - 1);
    out[(size_t)b * K + cb] = (logf((red[0] + red[1]) + (red[2] + red[3])) + m) - lg[t];
  }
}

void launch_forced_ce(const float* c0, const float* ci, const int* forced, float* out, int B, int K, int V, int Vp,
                      hipStream_t st) {
  hipLaunchKernelGGL(forced_ce_kernel, dim3(B * K), dim3(256), 0, st, c0, ci, forced, out, B, K, V, Vp);
}

void launch_advance(const AdvanceParams& p, hipStream_t st) {
  if (p.K > 64) throw CsmError(CSM_ERR_ARG, "advance: at most 64 codebooks");
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(256), 0, st, p);
}

// ============================================================================ stored-row reads
// out[i] = row idx[i] of a stored [Ntot][K] matrix as fp32 (int4: dequantized w = scale * q + bias,
// the value every kernel computes with) -- the CSM.embed_tokens / embed_audio / weight views.
template <typename WT>
__global__ __launch_bounds__(256) void table_rows_kernel(const void* base, int Ntot, int K, const int* idx,
                                                         float* out, int q4) {
  const size_t r = (size_t)idx[blockIdx.x];
  float* o = out + (size_t)blockIdx.x * K;
  for (int k = threadIdx.x * 8; k < K; k += 256 * 8) {
    float v[8];
    if (q4) q4_load8((const uint8_t*)base, (size_t)Ntot, K, r, k, v);
    else W8<WT>::load((const WT*)base + r * K + k, v);
    *reinterpret_cast<float4*>(o + k) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(o + k + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

void launch_table_rows(const void* base, int wdt, int Ntot, int K, const int* idx, int n, float* out, hipStream_t st) {
  if (n <= 0) return;
  if (wdt == WDT_F32) hipLaunchKernelGGL(table_rows_kernel<float>, dim3(n), dim3(256), 0, st, base, Ntot, K, idx, out, 0);
  else hipLaunchKernelGGL(table_rows_kernel<bf16_t>, dim3(n), dim3(256), 0, st, base, Ntot, K, idx, out,
                          wdt == WDT_Q4 ? 1 : 0);
}
