// int4 (MLX affine, group 64) kernels for gfx950: load-time quantization, dequantization, the
// quantized GEMV behind every QuantizedLinear of an nn.quantize'd CSM, and the quantized
// embedding gather (QuantizedEmbedding).
//
// Reference: nn.quantize(model, group_size=64, bits=4) (run_streaming_csm_mlx.py:811-818,
// README.md:108-111).  The quantization rule restated here and in oracle/quant_oracle.py is
// mlx's affine ``quantize`` (un-vendored dependency mlx>=0.22.1, pyproject.toml:13); the layout
// is common.h's q4 layout.
#include <climits>

#include "../../include/csm_hip_prof.h"
#include "csm_kernels.h"
#include "xs.h"

// ============================================================================ quantize
// One thread per (row, group of 64): MLX affine rule in fp32 (IEEE div / rint, as numpy does in the
// oracle), scale and bias rounded to bf16, q = clip(rint((w - bias) / scale), 0, 15).
// Source rows r < n_rows of a [n_rows][K] f32 / bf16 matrix; destination row = row0 + r * rstep of
// a quantized matrix with Ntot rows (fused QKV offsets, interleaved gate/up rows).
template <typename ST>
__global__ __launch_bounds__(256) void q4_quantize_kernel(const ST* src, int n_rows, int K, uint8_t* dst, int Ntot,
                                                         int row0, int rstep) {
  const int KG = K / Q4_GROUP;
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= (long long)n_rows * KG) return;
  const int r = (int)(t / KG), g = (int)(t % KG);
  const ST* w = src + (size_t)r * K + (size_t)g * Q4_GROUP;
  float v[Q4_GROUP];
  float mx = -INFINITY, mn = INFINITY;
#pragma unroll
  for (int j = 0; j < Q4_GROUP; ++j) {
    v[j] = ld1<ST>(w + j);
    mx = fmaxf(mx, v[j]);
    mn = fminf(mn, v[j]);
  }
  const bool mask = fabsf(mn) > fabsf(mx);
  float scale = fmaxf((mx - mn) / 15.0f, 1e-7f);
  scale = mask ? scale : -scale;
  const float edge = mask ? mn : mx;
  const float q0 = rintf(edge / scale);
  float bias = 0.f;
  if (q0 != 0.f) {
    scale = edge / q0;
    bias = edge;
  }
  const uint32_t sbits = st_cast<bf16_t>(scale), bbits = st_cast<bf16_t>(bias);
  scale = __uint_as_float(sbits << 16);
  bias = __uint_as_float(bbits << 16);
  const size_t dr = (size_t)row0 + (size_t)r * rstep;
  uint32_t* q = reinterpret_cast<uint32_t*>(dst + dr * (K / 2) + (size_t)g * (Q4_GROUP / 2));
#pragma unroll
  for (int wd = 0; wd < Q4_GROUP / 8; ++wd) {
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float qf = fminf(fmaxf(rintf((v[wd * 8 + j] - bias) / scale), 0.f), 15.f);
      word |= (uint32_t)qf << (4 * j);
    }
    q[wd] = word;
  }
  reinterpret_cast<uint32_t*>(dst + q4_sb_offset(Ntot, K))[dr * KG + g] = sbits | (bbits << 16);
}

void launch_q4_quantize(const void* src, int src_wdt, int n_rows, int K, void* dst, int Ntot, int row0, int rstep,
                        hipStream_t st) {
  const long long n = (long long)n_rows * (K / Q4_GROUP);
  const int blocks = (int)((n + 255) / 256);
  if (src_wdt == WDT_BF16)
    hipLaunchKernelGGL(q4_quantize_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)src, n_rows, K,
                       (uint8_t*)dst, Ntot, row0, rstep);
  else
    hipLaunchKernelGGL(q4_quantize_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)src, n_rows, K,
                       (uint8_t*)dst, Ntot, row0, rstep);
}

// Pre-quantized MLX tensors: packed uint32 [n][K/8] (copied as bytes by the host) + scales / biases
// [n][K/64] (f32 or bf16 on the host) -> the sb words of rows row0 + r*rstep.
template <typename ST>
__global__ void q4_set_sb_kernel(const ST* sc, const ST* bi, int n_rows, int K, uint8_t* dst, int Ntot, int row0,
                                 int rstep) {
  const int KG = K / Q4_GROUP;
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= (long long)n_rows * KG) return;
  const int r = (int)(t / KG), g = (int)(t % KG);
  const uint32_t s = st_cast<bf16_t>(ld1<ST>(sc + t)), b = st_cast<bf16_t>(ld1<ST>(bi + t));
  const size_t dr = (size_t)row0 + (size_t)r * rstep;
  reinterpret_cast<uint32_t*>(dst + q4_sb_offset(Ntot, K))[dr * KG + g] = s | (b << 16);
}

void launch_q4_set_sb(const void* sc, const void* bi, int src_wdt, int n_rows, int K, void* dst, int Ntot, int row0,
                      int rstep, hipStream_t st) {
  const long long n = (long long)n_rows * (K / Q4_GROUP);
  const int blocks = (int)((n + 255) / 256);
  if (src_wdt == WDT_BF16)
    hipLaunchKernelGGL(q4_set_sb_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)sc,
                       (const bf16_t*)bi, n_rows, K, (uint8_t*)dst, Ntot, row0, rstep);
  else
    hipLaunchKernelGGL(q4_set_sb_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)sc, (const float*)bi,
                       n_rows, K, (uint8_t*)dst, Ntot, row0, rstep);
}

// rows [r0, r0 + n) of a quantized [Ntot][K] matrix -> dense f32 [n][K]  (mx.dequantize)
__global__ __launch_bounds__(256) void q4_to_f32_kernel(const uint8_t* base, int Ntot, int K, int r0, int n,
                                                         float* dst) {
  const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= (size_t)n * K) return;
  const size_t r = i / K;
  const int k = (int)(i % K);
  float w[8];
  q4_load8(base, Ntot, K, (size_t)r0 + r, k, w);
  *reinterpret_cast<float4*>(dst + i) = make_float4(w[0], w[1], w[2], w[3]);
  *reinterpret_cast<float4*>(dst + i + 4) = make_float4(w[4], w[5], w[6], w[7]);
}

void launch_q4_to_f32(const void* base, int Ntot, int K, int r0, int n, float* dst, hipStream_t st) {
  const size_t tot = (size_t)n * K / 8;
  hipLaunchKernelGGL(q4_to_f32_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const uint8_t*)base,
                     Ntot, K, r0, n, dst);
}

// [D][F] quantized down_proj -> the persistent kernels' chunk-major copy: nibbles [F/32][D][16 B] (columns
// 32c .. 32c + 31 of row n, the 16 bytes of the standard layout, contiguous per column chunk), then the
// affine words [F/64][D] -- a workgroup's 32-column slice of every row is one contiguous stream.
__global__ __launch_bounds__(256) void q4_down_cm_kernel(const uint8_t* src, int D, int F, uint8_t* dst) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t nch = (size_t)(F / 32) * D;
  if (i < nch) {
    const size_t c = i / D, n = i % D;
    *reinterpret_cast<uint4*>(dst + i * 16) = *reinterpret_cast<const uint4*>(src + n * (F / 2) + c * 16);
  }
  if (i < (size_t)(F / Q4_GROUP) * D) {
    const size_t g = i / D, n = i % D;
    reinterpret_cast<uint32_t*>(dst + (size_t)D * F / 2)[i] =
        reinterpret_cast<const uint32_t*>(src + q4_sb_offset(D, F))[n * (F / Q4_GROUP) + g];
  }
}

void launch_q4_down_cm(const void* src, int D, int F, void* dst, hipStream_t st) {
  const size_t n = (size_t)(F / 32) * D;
  hipLaunchKernelGGL(q4_down_cm_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const uint8_t*)src, D, F,
                     (uint8_t*)dst);
}

// ============================================================================ embedding (QuantizedEmbedding)
// embed_rows_kernel with dequantized rows: x[m] = sum_j mask * (scale * q + bias) of row tok + V*j of
// the audio table, then the text column (generation.py:32-36 order).
__global__ __launch_bounds__(256) void embed_rows_q4_kernel(EmbedParams p, int n_text_rows) {
  __shared__ long long rows[64];  // table row (audio rows >= 0, text rows encoded as -(row+1)), or LLONG_MIN
  const int m = blockIdx.x;
  const int ncol = p.K + 1;
  if (threadIdx.x < ncol) {
    const int j = threadIdx.x;
    long long r = LLONG_MIN;
    if (p.codes) {
      if (j < p.K) r = (long long)p.codes[(size_t)m * p.K + j] + (long long)p.V * j;
    } else if (p.mask[(size_t)m * ncol + j]) {
      const int t = p.tok[(size_t)m * ncol + j];
      r = (j < p.K) ? (long long)t + (long long)p.V * j : -(long long)t - 1;
    }
    rows[j] = r;
  }
  __syncthreads();
  if (p.pos_inc && threadIdx.x == 0) p.pos_inc[m] += 1;
  const size_t Na = (size_t)p.V * p.K;
  float* out = p.out + (size_t)m * p.D;
  for (int d0 = threadIdx.x * 8; d0 < p.D; d0 += blockDim.x * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < ncol; ++j) {
      const long long r = rows[j];
      if (r == LLONG_MIN) continue;
      float w[8];
      if (r >= 0) q4_load8((const uint8_t*)p.audio_emb, Na, p.D, (size_t)r, d0, w);
      else q4_load8((const uint8_t*)p.text_emb, (size_t)n_text_rows, p.D, (size_t)(-r - 1), d0, w);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += w[e];
    }
    *reinterpret_cast<float4*>(out + d0) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *reinterpret_cast<float4*>(out + d0 + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
    if (p.xs_out) {  // streaming backbone operand, as embed_rows_kernel: split (x * n1), sums of squares
      const int t = threadIdx.x & 63;  // per 512 columns (one wave), half-group sums per 32 (4 lanes)
      float sq = 0.f, hsum = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) sq = fmaf(acc[e], acc[e], sq);
      sq = wave_sum(sq);
      if (t == 0) p.ss_out[(size_t)(d0 / 512) * p.ss_stride + m] = sq;
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
      if (p.hs_out) {
        const int b4 = t & ~3;
        const float h0 = __shfl(hsum, b4, 64), h1 = __shfl(hsum, b4 + 1, 64), h2 = __shfl(hsum, b4 + 2, 64),
                    h3 = __shfl(hsum, b4 + 3, 64);
        if ((t & 3) == 0) p.hs_out[(size_t)(d0 / 32) * xs::HS_ROWS + m] = ((h0 + h1) + h2) + h3;
      }
    }
  }
}

void launch_embed_q4(const EmbedParams& p, int n_text_rows, int M, hipStream_t st) {
  hipLaunchKernelGGL(embed_rows_q4_kernel, dim3(M), dim3(256), 0, st, p, n_text_rows);
}

// ============================================================================ quantized GEMV
// y[m, n] = sum_k norm(x)[m, k] * w_hat[n, k],  w_hat = s_g * q + b_g  (QuantizedLinear, transpose=True)
// evaluated per half group of 32 as  s_g * sum(q * x) + b_g * sum(x).
//
// A 256-thread block owns RPB = (256/G)*RPT rows; a group of G threads covers K in KS steps of
// G*32 elements, each lane one 16-B load (32 nibbles = half a group) per row and step plus the
// group's {scale, bias} word.  Structure as gemv_xl_kernel: (1) every weight load of the thread is
// issued first and stays in VGPRs for the whole launch, (2) MT activation rows at a time are staged
// in LDS as x * norm_weight with their half-group sums and sum(x^2), (3) dot products from LDS,
// (4) shuffle + LDS reduction and the shared pair epilogues.  M > MT loops over (2)-(4) with the
// weights still in registers, so every weight byte is read once per launch at any M.
template <int G, int KS, int RPT, int MT, bool NT>
__global__ __launch_bounds__(256) void gemv_q4_kernel(GemvParams p) {
  constexpr int NG = 256 / G;
  constexpr int RPB = NG * RPT;
  constexpr int LW = G < 64 ? G : 64;    // lanes of a group inside one wave
  constexpr int WPG = G < 64 ? 1 : G / 64;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) float q4_smem[];
  const int K = p.K;
  // x * nw in LDS, each 32-element half group padded to 36 floats: lane gt's ds_read_b128 of its
  // half group (stride 144 B) then hits distinct banks across a 16-lane group (no conflicts)
  const int KP = K / 32 * 36;
  float* xl = q4_smem;                    // [MT][KP]
  float* xh = q4_smem + MT * KP;          // [MT][K/32] half-group sums of x*nw
  __shared__ float red[4][MT][RPT + 1];   // per wave: (row of block, RPT partials) -- G >= 64 path
  __shared__ float rss[4][MT];
  __shared__ int gcode[64];
  __shared__ unsigned long long bk[4][MT];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int grp = tid / G, gt = tid % G;
  const int row0 = blockIdx.x * RPB + grp * RPT;
  const bool norm = p.nw != nullptr;
  const uint8_t* Wq = (const uint8_t*)p.W;
  const uint32_t* SB = reinterpret_cast<const uint32_t*>(Wq + q4_sb_offset(p.N, K));
  const int KG = K / Q4_GROUP;
  // (1) weights in flight
  u32x4 wq[KS][RPT];
  uint32_t sb[KS][RPT];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    // K need not fill the group's G x 32 span (K = 1280: G = 64, lanes gt >= 40 idle): a lane past K
    // holds zero weights and skips its dot products
    const int k = min(gt * 32 + s * G * 32, K - 32);
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      const size_t row = (size_t)min(row0 + r, p.N - 1);  // partial last block: re-read a valid row
      const u32x4* src = reinterpret_cast<const u32x4*>(Wq + row * (K / 2) + k / 2);
      if constexpr (NT) wq[s][r] = __builtin_nontemporal_load(src);
      else wq[s][r] = *src;
      sb[s][r] = SB[row * KG + k / Q4_GROUP];
    }
  }
  for (int m0 = 0; m0 < p.M; m0 += MT) {
    const int mn = min(MT, p.M - m0);
    // (2a) gather mode: codes of the gathered rows from the producer's arg-max partials
    if (p.xpart) {
      for (int i = wave; i < mn; i += 4) {
        const int m = m0 + i;
        const int bb = p.x_step1 ? (m >> 1) : m;
        if (p.x_step1 && !(m & 1)) continue;
        const unsigned long long best = wave_argmax_partials(p.xpart + (size_t)bb * p.xpart_stride, p.xpart_n, lane);
        if (lane == 0) {
          const int c = min(max(unpack_argmax(best), 0), p.xV - 1);
          gcode[i] = c;
          if (blockIdx.x == 0) p.x_codes[(size_t)bb * p.x_codes_K + p.xcb] = c;
        }
      }
      __syncthreads();
    }
    // (2b) stage x * nw, half-group sums, sum(x^2)
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float ssp = 0.f;
      if (i < mn) {
        const int m = m0 + i;
        const bool gathered = p.xpart && !(p.x_step1 && !(m & 1));
        const size_t trow = gathered ? (size_t)gcode[i] + (size_t)p.xV * p.xcb : 0;
        const bool gq4 = gathered && !p.xtab_f32;
        const float* xf = gathered ? (const float*)p.xtab + trow * K : p.x + (size_t)(p.x_step1 ? (m >> 1) : m) * p.xs;
        float* xc = (p.x_copy && blockIdx.x == 0) ? p.x_copy + (size_t)m * K : nullptr;
        for (int k = tid * 8; k < K; k += 256 * 8) {
          float xv[8];
          if (gq4) q4_load8((const uint8_t*)p.xtab, (size_t)p.xtab_q4_rows, K, trow, k, xv);
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
              ssp = fmaf(xv[j], xv[j], ssp);
              xv[j] *= nw[j];
            }
          }
          float* xd = &xl[i * KP + (k >> 5) * 36 + (k & 31)];
          *reinterpret_cast<float4*>(xd) = make_float4(xv[0], xv[1], xv[2], xv[3]);
          *reinterpret_cast<float4*>(xd + 4) = make_float4(xv[4], xv[5], xv[6], xv[7]);
          float hs = ((xv[0] + xv[1]) + (xv[2] + xv[3])) + ((xv[4] + xv[5]) + (xv[6] + xv[7]));
          hs += __shfl_xor(hs, 1, 64);
          hs += __shfl_xor(hs, 2, 64);
          if ((tid & 3) == 0) xh[i * (K / 32) + k / 32] = hs;
        }
      }
      if (norm) {
        const float v = wave_sum(ssp);
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
    for (int s = 0; s < KS; ++s) {
      const int k = gt * 32 + s * G * 32;
      if (k >= K) continue;  // (idle lane of a K that does not fill the span)
      float qf[RPT][32];
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const uint32_t u = wq[s][r][w];
          const uint32_t lo = u & 0x0F0F0F0Fu, hi = (u >> 4) & 0x0F0F0F0Fu;
          qf[r][w * 8 + 0] = (float)((lo >> 0) & 0xFFu);
          qf[r][w * 8 + 1] = (float)((hi >> 0) & 0xFFu);
          qf[r][w * 8 + 2] = (float)((lo >> 8) & 0xFFu);
          qf[r][w * 8 + 3] = (float)((hi >> 8) & 0xFFu);
          qf[r][w * 8 + 4] = (float)((lo >> 16) & 0xFFu);
          qf[r][w * 8 + 5] = (float)((hi >> 16) & 0xFFu);
          qf[r][w * 8 + 6] = (float)((lo >> 24) & 0xFFu);
          qf[r][w * 8 + 7] = (float)((hi >> 24) & 0xFFu);
        }
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if (i < mn) {
          const float4* xr = reinterpret_cast<const float4*>(&xl[i * KP + (k >> 5) * 36]);
          float xv[32];
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            const float4 v = xr[c];
            xv[c * 4 + 0] = v.x; xv[c * 4 + 1] = v.y; xv[c * 4 + 2] = v.z; xv[c * 4 + 3] = v.w;
          }
          const float hsum = xh[i * (K / 32) + k / 32];
#pragma unroll
          for (int r = 0; r < RPT; ++r) {
            float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
#pragma unroll
            for (int j = 0; j < 32; j += 4) {
              d0 = fmaf(qf[r][j + 0], xv[j + 0], d0);
              d1 = fmaf(qf[r][j + 1], xv[j + 1], d1);
              d2 = fmaf(qf[r][j + 2], xv[j + 2], d2);
              d3 = fmaf(qf[r][j + 3], xv[j + 3], d3);
            }
            const float dq = (d0 + d1) + (d2 + d3);
            acc[i][r] = fmaf(bf16_lo(sb[s][r]), dq, fmaf(bf16_hi(sb[s][r]), hsum, acc[i][r]));
          }
        }
      }
    }
    // (4) reduce over the group's lanes (and waves), pair epilogues
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        float v = acc[i][r];
#pragma unroll
        for (int o = LW / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        acc[i][r] = v;
      }
    if (WPG > 1 && lane == 0) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < RPT; ++r) red[wave][i][r] = acc[i][r];
    }
    __syncthreads();
    float sc[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      sc[i] = 1.f;
      if (norm) {
        const float sq = (rss[0][i] + rss[1][i]) + (rss[2][i] + rss[3][i]);
        sc[i] = rsqrtf(sq / (float)K + p.eps);
      }
    }
    unsigned long long akey[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) akey[i] = 0ull;
    auto emit = [&](int i, int n, float a, float b) {
      if (n >= p.N) return;  // partial last block
      gemv_epilogue_pair(p, m0 + i, n, a, b);
      if (p.epi == EPI_ARGMAX) {
        unsigned long long key = n < p.n_valid ? pack_argmax(a, n) : 0ull;
        if (n + 1 < p.n_valid) {
          const unsigned long long kb = pack_argmax(b, n + 1);
          key = kb > key ? kb : key;
        }
        akey[i] = key > akey[i] ? key : akey[i];
      }
    };
    if constexpr (WPG > 1) {
      constexpr int NPAIR = NG * MT * (RPT / 2);
      if (tid < NPAIR) {
        const int g = tid / (MT * (RPT / 2));
        const int rem = tid % (MT * (RPT / 2));
        const int i = rem / (RPT / 2), rp = (rem % (RPT / 2)) * 2;
#pragma unroll
        for (int ii = 0; ii < MT; ++ii) {
          if (ii == i && i < mn) {
            float a = 0.f, b = 0.f;
#pragma unroll
            for (int w = 0; w < WPG; ++w) {
              a += red[g * WPG + w][ii][rp];
              b += red[g * WPG + w][ii][rp + 1];
            }
            emit(ii, blockIdx.x * RPB + g * RPT + rp, a * sc[ii], b * sc[ii]);
          }
        }
      }
    } else if (gt == 0) {  // groups inside one wave: lane 0 of each group owns its rows
#pragma unroll
      for (int i = 0; i < MT; ++i)
        if (i < mn)
#pragma unroll
          for (int rp = 0; rp < RPT; rp += 2) emit(i, row0 + rp, acc[i][rp] * sc[i], acc[i][rp + 1] * sc[i]);
    }
    if (p.epi == EPI_ARGMAX) {  // block arg-max per row -> partial slot
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        unsigned long long v = akey[i];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const unsigned long long w = __shfl_xor(v, o, 64);
          v = w > v ? w : v;
        }
        if (lane == 0) bk[wave][i] = v;
      }
      __syncthreads();
      if (tid < mn) {
        unsigned long long v = bk[0][tid];
        for (int w = 1; w < 4; ++w) v = bk[w][tid] > v ? bk[w][tid] : v;
        p.part[(size_t)(m0 + tid) * p.part_stride + blockIdx.x] = v;
      }
    }
    __syncthreads();
  }
}

// Tiling: one K step per thread (G = K / 32 rounded up to a power of two >= 8, capped at 256; K = 8192
// runs G = 256; K = 1280 runs G = 64 with lanes 40..63 of each group idle); RPT = 2.
static void q4_tiling(int K, int& G, int& KS) {
  G = 8;
  while (G < K / 32 && G < 256) G *= 2;
  KS = (K / 32 + G - 1) / G;
}

int gemv_q4_rows_per_block(int N, int K, int M) {
  (void)N;
  (void)M;
  int G, KS;
  q4_tiling(K, G, KS);
  return (256 / G) * 2;
}

// shapes the launcher handles (rows need not fill the last block; N even for the pair epilogue)
bool gemv_q4_supported(int N, int K) {
  int G, KS;
  q4_tiling(K, G, KS);
  return K % Q4_GROUP == 0 && K >= Q4_GROUP && N % 2 == 0 && KS == 1;
}

extern "C" int csm_q4_gemv_shape(int N, int K, int* out) {
  if (K <= 0 || N <= 0) return 0;
  int G, KS;
  q4_tiling(K, G, KS);
  out[0] = G; out[1] = KS; out[2] = (256 / G) * 2;
  return gemv_q4_supported(N, K) ? 1 : 0;
}

template <int G, bool NT>
static void launch_q4_g(const GemvParams& p, hipStream_t st) {
  const int rpb = (256 / G) * 2;
  const int blocks = (p.N + rpb - 1) / rpb;
  const bool mt1 = p.M == 1;
  const size_t lds = (size_t)(mt1 ? 1 : 4) * (p.K / 32 * 36 + p.K / 32) * 4;
  static bool attr_set = false;  // > 64 KB of dynamic LDS (K = 8192 at MT = 4)
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemv_q4_kernel<G, 1, 2, 1, NT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 158 * 1024);
    (void)hipFuncSetAttribute((const void*)gemv_q4_kernel<G, 1, 2, 4, NT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 158 * 1024);
    attr_set = true;
  }
  if (mt1) hipLaunchKernelGGL((gemv_q4_kernel<G, 1, 2, 1, NT>), dim3(blocks), dim3(256), lds, st, p);
  else hipLaunchKernelGGL((gemv_q4_kernel<G, 1, 2, 4, NT>), dim3(blocks), dim3(256), lds, st, p);
}

void launch_gemv_q4(const GemvParams& p, bool nt, hipStream_t st) {
  int G, KS;
  q4_tiling(p.K, G, KS);
#define Q4_G(G_) do { if (nt) launch_q4_g<G_, true>(p, st); else launch_q4_g<G_, false>(p, st); } while (0)
  switch (G) {
    case 8: Q4_G(8); break;
    case 16: Q4_G(16); break;
    case 32: Q4_G(32); break;
    case 64: Q4_G(64); break;
    case 128: Q4_G(128); break;
    default: Q4_G(256); break;
  }
#undef Q4_G
}
