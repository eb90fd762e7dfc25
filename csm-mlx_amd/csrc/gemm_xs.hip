// Streaming matrix-core GEMM for the batched depth decoder: y[m, n] = sum_k A[m, k] W[n, k] at
// M <= 64 batch rows (generation.py:72-90 at batch B: the projection, QKV / o / gate-up / down of
// every decoder layer and the audio_head slices, once per codebook step).
//
// Why a second MFMA kernel beside gemm_wide_kernel (gemm_kernels.hip): at 32 rows the decoder's
// projections are latency- and VALU-bound there -- every block re-normalises and re-splits the
// same fp32 activation rows into three bf16 parts through LDS with a barrier per 64-K stage, at one
// wave per SIMD.  Here the producer of a row block (the previous projection's epilogue, the
// attention, the row gather) writes it ONCE already split, in MFMA fragment order (xs.h); every
// block then streams both operands straight into registers through a ring of PD stages whose loads
// are pinned at issue (compiler barrier: no sinking to the use), with no LDS and no barrier in the
// K loop.  Lab (profiles/r03_lab_gemm_stream.txt): decoder gate/up at 32 rows 8.8 us against
// 14.7 us for gemm_wide_kernel, QKV 3.3 against 10.4 (before the split-K combine).
//
// Block = 2 waves over one K slice (the slice's stages split between them, partial tiles added in a
// fixed order through LDS), 32 * RTW weight rows, 32 * MT batch rows.  Exactness as gemm_wide: the
// activation parts are exact, products exact in fp32, fp32 accumulation; the RMSNorm row scale is
// applied after the dot product (the producer multiplied the norm weight in before splitting).
// Split-K slices publish write-through (sc1) partial tiles and take an arrival ticket; the last
// slice of a tile sums them in slice order and runs the epilogue (deterministic).
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "csm_kernels.h"
#include "xs.h"

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned int gu32;

constexpr int XK = 64;                 // K per stage
constexpr int XW = 2;                  // waves per block
constexpr int RSRC3 = 0x00020000;      // buffer descriptor word 3 (raw 32-bit format)
constexpr int SC1 = 16;                // cache policy: sc1 (agent-coherent)
constexpr int MAX_SLICES = 16;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, RSRC3);
}

template <int MT, int RTW, int PD, bool NT>
__global__ __launch_bounds__(64 * XW) void gemm_xs_kernel(GemvParams p) {
  constexpr int NB = 32 * MT, NBR = 32 * RTW, NTH = 64 * XW;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tile = blockIdx.x, n0 = tile * NBR;
  const int nks = p.K / XK, nt32 = (p.N + 31) / 32;
  const int ks = p.ksplit, nst = nks / ks, wst = nst / XW, ws0 = blockIdx.y * nst + wave * wst;
  const __amdgpu_buffer_rsrc_t wrs = rsrc(p.Wt, 0x7fffffff), ars = rsrc(p.xs_in, 0x7fffffff), zrs = rsrc(p.Wt, 0);
  int wv[RTW];
#pragma unroll
  for (int i = 0; i < RTW; ++i) wv[i] = (min(n0 / 32 + i, nt32 - 1) * nks * 4 * 64 + lane) * 16;
  struct St {
    u32x4_t w[RTW][4];
    u32x4_t a[MT][3][4];
  };
  // stage j of this wave (j >= wst: zero-sized descriptors, no traffic) -- straight-line loads
  auto load = [&](int j, St& g) {
    const bool live = j < wst;
    const int st = ws0 + (live ? j : 0);
    const __amdgpu_buffer_rsrc_t wr = live ? wrs : zrs, ar = live ? ars : zrs;
#pragma unroll
    for (int i = 0; i < RTW; ++i)
#pragma unroll
      for (int s = 0; s < 4; ++s)
        g.w[i][s] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(wr, wv[i], (st * 4 + s) * 1024, NT ? 2 : 0));
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int s = 0; s < 4; ++s)
          g.a[t][q][s] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(ar, lane * 16, ((t * nks + st) * 12 + q * 4 + s) * 1024, 0));
  };
  f32x16_t acc[MT][RTW];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < RTW; ++i) acc[t][i] = f32x16_t{};
  St g[PD];
#pragma unroll
  for (int d = 0; d < PD; ++d) load(d, g[d]);
  asm volatile("" ::: "memory");  // the ring's loads stay where they are issued (no sinking to their use)
  for (int j0 = 0; j0 < wst; j0 += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
          for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int i = 0; i < RTW; ++i)
              acc[t][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, g[d].a[t][q][s]),
                                                                   __builtin_bit_cast(bf16x8_t, g[d].w[i][s]), acc[t][i], 0, 0, 0);
      load(j0 + d + PD, g[d]);
      asm volatile("" ::: "memory");
    }
  }
  // the waves' partial tiles -> ct[batch row][weight row], added in wave order.  Accumulator register
  // j of lane (r, h): batch row (j & 3) + 8 (j >> 2) + 4 h of tile t, weight row r of tile i.
  __shared__ float red[XW][MT * RTW * 16][64];
  __shared__ float ct[NB][NBR + 1];
  __shared__ float hb[NB][NBR / 2 + 1];
  __shared__ float rsc[NB];
  __shared__ int last;
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < RTW; ++i)
#pragma unroll
      for (int j = 0; j < 16; ++j) red[wave][(t * RTW + i) * 16 + j][lane] = acc[t][i][j];
  __syncthreads();
  for (int e = tid; e < NB * NBR; e += NTH) {
    const int ml = e / NBR, c = e % NBR, rr = ml & 31;
    const int idx = ((ml >> 5) * RTW + (c >> 5)) * 16 + (rr & 3) + 4 * (rr >> 3), ln = (c & 31) + 32 * ((rr >> 2) & 1);
    float v = red[0][idx][ln];
#pragma unroll
    for (int w = 1; w < XW; ++w) v += red[w][idx][ln];
    ct[ml][c] = v;
  }
  __syncthreads();
  const int mrows = min(NB, p.M);
  if (ks > 1) {
    // slice partial [NB][NBR] write-through, ticket; the last slice to arrive sums all in slice order
    const int slab_f = NB * NBR;
    float* slab = p.kpart + (size_t)tile * ks * slab_f;
    const __amdgpu_buffer_rsrc_t rs = rsrc(slab, ks * slab_f * 4);
    const int mine = blockIdx.y * slab_f * 4;
    for (int q = tid; q < mrows * (NBR / 4); q += NTH) {
      const int ml = q / (NBR / 4), j = (q % (NBR / 4)) * 4;
      const f32x4_t v = {ct[ml][j], ct[ml][j + 1], ct[ml][j + 2], ct[ml][j + 3]};
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, q * 16, mine, SC1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      gu32* tk = (gu32*)p.kticket + tile;
      const unsigned old = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = (old == (unsigned)ks - 1);
      if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
    }
    __syncthreads();
    if (!last) return;
    for (int q = tid; q < mrows * (NBR / 4); q += NTH) {
      f32x4_t v[MAX_SLICES];
#pragma unroll
      for (int s = 0; s < MAX_SLICES; ++s)
        if (s < ks) v[s] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, q * 16, s * slab_f * 4, SC1));
      f32x4_t sum = v[0];
#pragma unroll
      for (int s = 1; s < MAX_SLICES; ++s)
        if (s < ks) sum += v[s];
      const int ml = q / (NBR / 4), j = (q % (NBR / 4)) * 4;
      ct[ml][j] = sum.x;
      ct[ml][j + 1] = sum.y;
      ct[ml][j + 2] = sum.z;
      ct[ml][j + 3] = sum.w;
    }
    __syncthreads();
  }
  // ---- epilogue
  const bool norm = p.nw != nullptr;
  if (norm && tid < mrows) {
    float s = 0.f;
    for (int t = 0; t < p.ss_n; ++t) s += p.ss_in[(size_t)t * p.ss_stride + tid];
    rsc[tid] = rsqrtf(s / (float)p.K + p.eps);
  }
  __syncthreads();
  const bool prod = p.xs_out != nullptr;
  const bool silu = p.epi == EPI_SILU_MUL;
  for (int e = tid; e < mrows * (NBR / 2); e += NTH) {
    const int ml = e / (NBR / 2), rp = (e % (NBR / 2)) * 2, n = n0 + rp;
    float va = ct[ml][rp], vb = ct[ml][rp + 1];
    if (norm) {
      va *= rsc[ml];
      vb *= rsc[ml];
    }
    if (n >= p.N) continue;
    if (p.epi == EPI_ADD) {  // residual add (no fused-MLP accumulator / column scale on this path)
      float* o = p.out + (size_t)ml * p.os + n;
      va = o[0] + va;
      vb = o[1] + vb;
      o[0] = va;
      o[1] = vb;
    } else if (silu) {  // rows 2j (gate), 2j+1 (up) -> h[j]
      const float hv = silu_f(va) * vb;
      if (p.out) p.out[(size_t)ml * p.os + (n >> 1)] = hv;
      hb[ml][rp >> 1] = hv;
    } else {
      gemv_epilogue_pair(p, ml, n, va, vb);
    }
    ct[ml][rp] = va;
    ct[ml][rp + 1] = vb;
  }
  if (prod || p.epi == EPI_ARGMAX) __syncthreads();
  if (prod) {
    const int ncol = silu ? NBR / 2 : NBR, col0 = silu ? n0 / 2 : n0, colN = silu ? p.N / 2 : p.N;
    for (int q = tid; q < mrows * (ncol / 4); q += NTH) {
      const int ml = q / (ncol / 4), c = (q % (ncol / 4)) * 4, col = col0 + c;
      if (col >= colN) continue;
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = silu ? hb[ml][c + u] : ct[ml][c + u];
        if (p.xs_nw) v[u] *= p.xs_nw[col + u];
      }
      xs::store4(p.xs_out, p.xs_K, ml, col, v);
    }
    if (p.ss_out && !silu && tid < mrows) {  // sum of squares of this tile's new values, column order
      float s = 0.f;
      for (int c = 0; c < ncol && col0 + c < colN; ++c) s = fmaf(ct[tid][c], ct[tid][c], s);
      p.ss_out[(size_t)tile * p.ss_stride + tid] = s;
    }
  }
  if (p.epi == EPI_ARGMAX && tid < mrows) {
    unsigned long long best = 0;
    for (int j = 0; j < NBR; ++j) {
      const int n = n0 + j;
      if (n < p.n_valid) {
        const unsigned long long key = pack_argmax(ct[tid][j], n);
        best = key > best ? key : best;
      }
    }
    p.part[(size_t)tid * p.part_stride + tile] = best;
  }
}

// Launch shape: RTW 2 (64-row tiles) for the wide and the long-K projections and for the heads (the
// arg-max partial count then equals gemm_wide's 64-row tiles), else 1; K slices doubled until the grid
// has >= 256 blocks while every wave keeps >= 1 stage; ring depth <= 4 stages (<= 2 at 64 rows).
void xs_shape(int N, int K, int M, bool head, int& rtw, int& ks, int& pd) {
  const int nks = K / XK;
  rtw = (N >= 4096 || K >= 4096 || head) ? 2 : 1;
  const int tiles = (N + 32 * rtw - 1) / (32 * rtw);
  ks = 1;
  while (tiles * ks < 256 && ks < MAX_SLICES && nks / (ks * 2) >= XW && nks % (ks * 2) == 0) ks *= 2;
  const int wst = nks / ks / XW;
  const int cap = M > 32 ? (rtw == 2 ? 1 : 2) : 4;
  pd = 1;
  while (pd * 2 <= cap && wst % (pd * 2) == 0) pd *= 2;
}

size_t xs_need(int N, int K, int M, bool head, size_t& tk) {
  int rtw, ks, pd;
  xs_shape(N, K, M, head, rtw, ks, pd);
  const size_t tiles = (N + 32 * rtw - 1) / (32 * rtw);
  tk = tiles;
  return ks > 1 ? tiles * ks * (size_t)(M > 32 ? 64 : 32) * 32 * rtw * 4 : 0;
}

}  // namespace

bool gemm_xs_eligible(int N, int K, int M, int wdt) {
  return wdt == WDT_BF16 && M >= 1 && M <= GEMM_XS_MAX_M && N % 2 == 0 && K % XK == 0 && K / XK >= XW;
}

int gemm_xs_tiles(int N, int K, int M) {
  int rtw, ks, pd;
  xs_shape(N, K, M, false, rtw, ks, pd);
  return (N + 32 * rtw - 1) / (32 * rtw);
}

bool gemm_xs_reserve(GemmWs& ws, int N, int K, int Mmax) {
  size_t slab = 0, tk = 0;
  for (int m = 1; m <= std::min(Mmax, GEMM_XS_MAX_M); ++m)
    for (int h = 0; h < 2; ++h) {
      size_t t = 0;
      slab = std::max(slab, xs_need(N, K, m, h == 1, t));
      tk = std::max(tk, t);
    }
  bool moved = false;
  if (slab > ws.bytes) {
    if (ws.kpart) (void)hipFree(ws.kpart);
    ws.kpart = nullptr;
    ws.bytes = 0;
    if (hipMalloc(&ws.kpart, slab) == hipSuccess) ws.bytes = slab;
    moved = true;
  }
  if (tk > ws.n) {
    if (ws.tickets) (void)hipFree(ws.tickets);
    ws.tickets = nullptr;
    ws.n = 0;
    if (hipMalloc(&ws.tickets, tk * 4) == hipSuccess && hipMemset(ws.tickets, 0, tk * 4) == hipSuccess &&
        hipDeviceSynchronize() == hipSuccess)
      ws.n = tk;
    moved = true;
  }
  return moved;
}

void launch_gemm_xs(const GemvParams& p0, int epi, hipStream_t st, bool nt_w) {
  GemvParams p = p0;
  p.epi = epi;
  p.Wt = nullptr;
  if (p.ws) {
    const auto ti = p.ws->tiled.find(p.W);
    if (ti != p.ws->tiled.end()) p.Wt = ti->second;
  }
  if (!p.Wt || !p.xs_in || p.M > GEMM_XS_MAX_M || p.xacc || p.oacc || p.scale) {
    fprintf(stderr, "csm: gemm_xs launch without a tiled weight / split activations, or with an unsupported option (N=%d K=%d M=%d)\n",
            p.N, p.K, p.M);
    abort();
  }
  const bool head = epi == EPI_ARGMAX;
  int rtw, ks, pd;
  xs_shape(p.N, p.K, p.M, head, rtw, ks, pd);
  p.ksplit = ks;
  const int tiles = (p.N + 32 * rtw - 1) / (32 * rtw);
  if (ks > 1) {
    size_t tk = 0;
    const size_t need = xs_need(p.N, p.K, p.M, head, tk);
    if (!p.ws || need > p.ws->bytes || tk > p.ws->n) {  // reserved by gemm_xs_reserve outside graph capture
      fprintf(stderr, "csm: gemm_xs split-K scratch not reserved for N=%d K=%d M=%d\n", p.N, p.K, p.M);
      abort();
    }
    p.kpart = p.ws->kpart;
    p.kticket = p.ws->tickets;
  }
  // non-temporal weight loads: the audio_head slices and the backbone (read once per frame) stay out of the
  // caches the decoder's weights are re-read from
  const bool nt = head || nt_w;
  const dim3 grid(tiles, ks);
#define GX_K(MT_, RTW_, PD_) do { if (nt) hipLaunchKernelGGL((gemm_xs_kernel<MT_, RTW_, PD_, true>), grid, dim3(64 * XW), 0, st, p); \
                                  else hipLaunchKernelGGL((gemm_xs_kernel<MT_, RTW_, PD_, false>), grid, dim3(64 * XW), 0, st, p); } while (0)
#define GX_P(MT_, RTW_) do { if (pd == 4) GX_K(MT_, RTW_, (MT_ == 1 ? 4 : 2)); else if (pd == 2) GX_K(MT_, RTW_, 2); else GX_K(MT_, RTW_, 1); } while (0)
  if (p.M > 32) { if (rtw == 2) GX_P(2, 2); else GX_P(2, 1); }
  else { if (rtw == 2) GX_P(1, 2); else GX_P(1, 1); }
#undef GX_P
#undef GX_K
}
