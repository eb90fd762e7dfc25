// Streaming matrix-core GEMM for the batched depth decoder: y[m, n] = sum_k A[m, k] W[n, k] at
// M <= 64 batch rows (generation.py:72-90 at batch B: the projection, QKV / o / gate-up / down of
// every decoder layer and the audio_head slices, once per codebook step).
//
// Why a second MFMA kernel beside gemm_wide_kernel (gemm_kernels.hip): at 32 rows the decoder's
// projections are latency- and VALU-bound there -- every block re-normalises and re-splits the
// same fp32 activation rows into three bf16 parts through LDS with a barrier per 64-K stage, at one
// wave per SIMD.  Here the producer of a row block (the previous projection's epilogue, the
// attention, the row gather) writes it ONCE in MFMA fragment order (xs.h: fp32, split into the three
// parts in registers by the consumer); every
// block then streams both operands straight into registers through a ring of PD stages whose loads
// are pinned at issue (compiler barrier: no sinking to the use), with no LDS and no barrier in the
// K loop.  Lab (profiles/r03_lab_gemm_stream.txt): decoder gate/up at 32 rows 8.8 us against
// 14.7 us for gemm_wide_kernel, QKV 3.3 against 10.4 (before the split-K combine).
//
// Block = 4 waves (2 where K is short) over one K slice (the slice's stages split between them, partial tiles added in a
// fixed order through LDS), 32 * RTW weight rows, 32 * MT batch rows.  Exactness as gemm_wide: the
// activation parts are exact, products exact in fp32, fp32 accumulation; the RMSNorm row scale is
// applied after the dot product (the producer multiplied the norm weight in before splitting).
// Split-K slices publish write-through (sc1) partial tiles and take an arrival ticket; the last
// slice of a tile sums them in slice order and runs the epilogue (deterministic).
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "../../include/csm_hip.h"
#include "../../include/csm_hip_prof.h"
#include "csm_kernels.h"
#include "xs.h"

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned int gu32;

constexpr int XK = 64;                 // K per stage
constexpr int XW_MAX = 4;              // waves per block: 2, or 4 where the grid would leave SIMDs idle
constexpr int RSRC3 = 0x00020000;      // buffer descriptor word 3 (raw 32-bit format)
constexpr int SC1 = 16;                // cache policy: sc1 (agent-coherent)
constexpr int MAX_SLICES = 16;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, RSRC3);
}

// Q4: int4 weights (MLX affine, group 64 = one stage) from the fragment-tiled int4 copy: the nibbles
// enter the matrix cores as exact bf16 integers, per stage S_g = sum q x (three products per step as
// for bf16), folded as acc += scale * S_g + bias * X_g with X_g the stage's activation sum per row
// (the producers' half-group sums, xs.h) -- the arithmetic of gemm_wide_kernel's int4 path.
constexpr int Q4_XG = 64;  // stages per block whose X_g an int4 block stages in LDS (Q4_XG / XW per wave)
constexpr int SS_MAX = 64 * 64;  // sums-of-squares partials a normed launch stages (tiles x rows)

// Split-K combine by the last slice to arrive: every slice's partial tile read with 16-B sc1 loads, up
// to 32 loads in flight per thread (UB vectors x KS slices per round), summed in slice order.
template <int KS, int NB, int NBR, int NTH>
__device__ __forceinline__ void combine(__amdgpu_buffer_rsrc_t rs, float (*ct)[NBR + 1], int mrows, int slab_f, int tid) {
  constexpr int NQ = NB * NBR / 4, U = (NQ + NTH - 1) / NTH, UB = (32 / KS) < 1 ? 1 : (32 / KS);
  const int nq = mrows * (NBR / 4);
#pragma unroll
  for (int u0 = 0; u0 < U; u0 += UB) {
    f32x4_t v[UB][KS];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int q = min(tid + NTH * (u0 + u), nq - 1);
#pragma unroll
      for (int s = 0; s < KS; ++s) v[u][s] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, q * 16, s * slab_f * 4, SC1));
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int q = tid + NTH * (u0 + u);
      if (u0 + u < U && q < nq) {
        f32x4_t sum = v[u][0];
#pragma unroll
        for (int s = 1; s < KS; ++s) sum += v[u][s];
        const int ml = q / (NBR / 4), j = (q % (NBR / 4)) * 4;
        ct[ml][j] = sum.x;
        ct[ml][j + 1] = sum.y;
        ct[ml][j + 2] = sum.z;
        ct[ml][j + 3] = sum.w;
      }
    }
  }
}

// Lab build only (tools/variant.sh -DXS_STAMPS=1): per-block clock stamps of the phases, 100 MHz
// s_memrealtime, for the first XS_ST_BLOCKS blocks of every launch, reported by gemm_xs_stamps_report.
#ifndef XS_STAMPS
#define XS_STAMPS 0
#endif
constexpr int XS_ST_N = 8, XS_ST_BLOCKS = 1024, XS_ST_LAUNCHES = 64;
__device__ unsigned long long g_xs_st[XS_ST_LAUNCHES][XS_ST_BLOCKS][XS_ST_N];
__device__ unsigned g_xs_launch;
#define XS_STAMP(k) do { if constexpr (XS_STAMPS != 0) { if (threadIdx.x == 0) { \
    const unsigned bl = blockIdx.x + gridDim.x * blockIdx.y, ln = p.lab_launch % XS_ST_LAUNCHES; \
    if (bl < XS_ST_BLOCKS) g_xs_st[ln][bl][k] = __builtin_amdgcn_s_memrealtime(); } } } while (0)

// ROLE: a name tag only (1 QKV, 2 o_proj, 3 down): the decoder's small projections share one shape at
// 32 bf16 / 64 int4 rows, and a tagged instantiation per role lets a rocprofv3 counter pass attribute
// FETCH_SIZE to each (launch_gemm_xs); the code is identical.
template <bool Q4, int MT, int RTW, int PD, bool NT, int XW, int ROLE = 0>
__global__ __launch_bounds__(64 * XW) void gemm_xs_kernel(GemvParams p) {
  XS_STAMP(0);
  constexpr int NB = 32 * MT, NBR = 32 * RTW, NTH = 64 * XW;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware (tile, slice) placement for the int4 64-row launches with >= 8 K slices (the decoder's QKV
  // and down at configs[4]'s B = 64): blocks are dealt round-robin over the 8 XCDs (linear id % 8 share
  // one L2; MI355X_MICROARCH.md, placement is speed only, never correctness), and with tile-major ids
  // every XCD read every slice of the 64-row fp32 operand -- its 2 MB (down) crossed into all 8 L2s,
  // 3.7x the launch's algorithmic bytes (round-4 PMC pass).  Here the blocks of XCD x take slices
  // [x S/8, (x + 1) S/8), so each operand slice reaches one L2.  Same (tile, slice) work items, same
  // combine order: outputs unchanged.  (At 32 bf16 rows the operand is half the size and the tile-major
  // order, which keeps a tile's slices and its combine inside one XCD, measured faster: r04_ab_xcd_map.)
#ifndef XS_XCD_Q4
#define XS_XCD_Q4 1  // lab: 0 keeps the tile-major placement (A/B)
#endif
  int tile = blockIdx.x, slice = blockIdx.y;
  if constexpr (Q4 && MT == 2 && XS_XCD_Q4 != 0) {
    const int T = gridDim.x, S = gridDim.y, L = blockIdx.x + T * blockIdx.y;
    if (S % 8 == 0) {
      slice = (L & 7) * (S / 8) + (L >> 3) / T;
      tile = (L >> 3) % T;
    }
  }
  const int n0 = tile * NBR;
  const int nks = p.K / XK, nt32 = (p.N + 31) / 32;
  const int ks = p.ksplit, nst = nks / ks, wst = nst / XW, ws0 = slice * nst + wave * wst;
  const __amdgpu_buffer_rsrc_t wrs = rsrc(p.Wt, 0x7fffffff), ars = rsrc(p.xs_in, 0x7fffffff), zrs = rsrc(p.Wt, 0);
  int wv[RTW], sv[RTW];
#pragma unroll
  for (int i = 0; i < RTW; ++i) {
    const int T = min(n0 / 32 + i, nt32 - 1);
    wv[i] = Q4 ? T * nks * 1024 + 16 * lane : (T * nks * 4 * 64 + lane) * 16;
    sv[i] = nt32 * nks * 1024 + (T * nks * 32 + (lane & 31)) * 4;  // int4: the lane's scale|bias words
  }
  __shared__ __attribute__((aligned(16))) float xg[Q4 ? XW : 1][Q4 ? Q4_XG / XW : 1][NB];
  if constexpr (Q4) {  // X_g of this block's stages: the two half-group sums, in order
    for (int e = tid; e < XW * wst * NB; e += NTH) {
      const int w = e / (wst * NB), j = (e / NB) % wst, m = e % NB;
      const int st = slice * nst + w * wst + j;
      xg[w][j][m] = p.hs_in[(size_t)(2 * st) * xs::HS_ROWS + m] + p.hs_in[(size_t)(2 * st + 1) * xs::HS_ROWS + m];
    }
    __syncthreads();
  }
  struct St {
    u32x4_t w[RTW][Q4 ? 1 : 4];
    uint32_t sb[RTW];
    u32x4_t a[MT][XS_F32 ? 4 : 3][XS_F32 ? 2 : 4];  // XS_F32: [t][s][half] fp32; else [t][part][s]
  };
  // the three bf16 parts of row tile t, step s (XS_F32: split here from the fp32 fragment)
  auto parts = [&](const St& g, int t, int s, u32x4_t (&pt)[3]) {
    if constexpr (XS_F32 != 0) {
      xs::split_frag(g.a[t][s][0], g.a[t][s][1], pt);
    } else {
#pragma unroll
      for (int q = 0; q < 3; ++q) pt[q] = g.a[t][q][s];
    }
  };
  // stage j of this wave (j >= wst: zero-sized descriptors, no traffic) -- straight-line loads
  auto load = [&](int j, St& g) {
    const bool live = j < wst;
    const int st = ws0 + (live ? j : 0);
#ifndef XS_LAB
#define XS_LAB 0  // lab ablations (tools/variant.sh -DXS_LAB=bits, results invalid): 1 no MFMA, 2 no activation
                  // traffic, 4 no weight traffic, 8 no split-K exchange / epilogue, 16 stop after the waves'
                  // reduction
#endif
    const __amdgpu_buffer_rsrc_t wr = (live && !(XS_LAB & 4)) ? wrs : zrs, ar = (live && !(XS_LAB & 2)) ? ars : zrs;
#pragma unroll
    for (int i = 0; i < RTW; ++i) {
      if constexpr (Q4) {
        g.w[i][0] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(wr, wv[i], st * 1024, NT ? 2 : 0));
        g.sb[i] = __builtin_amdgcn_raw_buffer_load_b32(wr, sv[i], st * 128, 0);
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s)
          g.w[i][s] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(wr, wv[i], (st * 4 + s) * 1024, NT ? 2 : 0));
      }
    }
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      if constexpr (XS_F32 != 0) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int hf = 0; hf < 2; ++hf)
            g.a[t][s][hf] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(ar, lane * 16, (((t * nks + st) * 4 + s) * 2 + hf) * 1024, 0));
      } else {
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
          for (int s = 0; s < 4; ++s)
            g.a[t][q][s] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(ar, lane * 16, ((t * nks + st) * 12 + q * 4 + s) * 1024, 0));
      }
    }
  };
  f32x16_t acc[MT][RTW];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < RTW; ++i) acc[t][i] = f32x16_t{};
  // Epilogue operands prefetched into LDS by LDS-DMA before the first weight stage (no registers held
  // across the K loop, no dependent global round trips after it): the RMSNorm sums-of-squares partials,
  // the residual rows of an EPI_ADD tile, the producer's norm-weight columns.
  __shared__ float sss[SS_MAX + 2 * 64 * XW];  // [t][NB] partial sums of squares
  __shared__ float res[NB * NBR + 64 * XW];    // [NB][NBR] residual rows (EPI_ADD)
  __shared__ float nws[64];                    // xs_nw[col0 .. col0 + ncol)
  const bool norm = p.nw != nullptr;
  const bool silu = p.epi == EPI_SILU_MUL;
  const int mrows = min(NB, p.M);
  {
    if (norm) {
      const int tot = p.ss_n * NB;
      for (int i0 = wave * 64; i0 < tot; i0 += NTH) {
        const int i = min(i0 + lane, tot - 1), t = i / NB, m = min(i % NB, mrows - 1);
        __builtin_amdgcn_global_load_lds(p.ss_in + (size_t)t * p.ss_stride + m, &sss[i0], 4, 0, 0);
      }
    }
    if (p.epi == EPI_ADD) {
      const int tot = mrows * NBR;
      for (int i0 = wave * 64; i0 < tot; i0 += NTH) {
        const int i = min(i0 + lane, tot - 1), m = i / NBR, n = min(n0 + i % NBR, p.N - 1);
        __builtin_amdgcn_global_load_lds(p.out + (size_t)m * p.os + n, &res[i0], 4, 0, 0);
      }
    }
    if (p.xs_out && p.xs_nw && wave == 0) {
      const int col0 = silu ? n0 / 2 : n0, ncol = silu ? NBR / 2 : NBR, colN = silu ? p.N / 2 : p.N;
      __builtin_amdgcn_global_load_lds(p.xs_nw + min(col0 + min(lane, ncol - 1), colN - 1), &nws[0], 4, 0, 0);
    }
  }
  St g[PD];
#pragma unroll
  for (int d = 0; d < PD; ++d) load(d, g[d]);
  asm volatile("" ::: "memory");  // the ring's loads stay where they are issued (no sinking to their use)
  XS_STAMP(1);
  const int hrow = 4 * (lane >> 5);  // int4 fold: lane (r, h) register jj holds batch row (jj & 3) + 8 (jj >> 2) + 4 h
  for (int j0 = 0; j0 < wst; j0 += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      if constexpr (Q4) {
        f32x16_t gq[MT][RTW];
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int i = 0; i < RTW; ++i) gq[t][i] = f32x16_t{};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          bf16x8_t b[RTW];
#pragma unroll
          for (int i = 0; i < RTW; ++i) b[i] = __builtin_bit_cast(bf16x8_t, xs::q4_word_bf16(g[d].w[i][0][s]));
          // (row tiles have their own accumulators: t outside q gives every accumulator the same
          // MFMA sequence as q outside t, with one tile's parts live at a time)
#pragma unroll
          for (int t = 0; t < MT; ++t) {
            u32x4_t pt[3];
            parts(g[d], t, s, pt);
#pragma unroll
            for (int q = 0; q < 3; ++q)
#pragma unroll
              for (int i = 0; i < RTW; ++i)
                gq[t][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, pt[q]), b[i], gq[t][i], 0, 0, 0);
            if constexpr (XS_F32 != 0 && MT > 1) __builtin_amdgcn_sched_barrier(0);  // one tile's parts live at a time (no spills)
          }
        }
        const int jst = j0 + d;
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          float xr[16];
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            const f32x4_t x4 = *reinterpret_cast<const f32x4_t*>(&xg[wave][jst][32 * t + 8 * q4 + hrow]);
            xr[4 * q4] = x4.x; xr[4 * q4 + 1] = x4.y; xr[4 * q4 + 2] = x4.z; xr[4 * q4 + 3] = x4.w;
          }
#pragma unroll
          for (int i = 0; i < RTW; ++i) {
            const float sc = bf16_lo(g[d].sb[i]), bi = bf16_hi(g[d].sb[i]);
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
              acc[t][i][jj] = fmaf(sc, gq[t][i][jj], acc[t][i][jj]);
              acc[t][i][jj] = fmaf(bi, xr[jj], acc[t][i][jj]);
            }
          }
        }
      } else if constexpr ((XS_LAB & 1) != 0) {  // lab: operands consumed by one VALU op each, no MFMA
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          u32x4_t pt[MT][3];
#pragma unroll
          for (int t = 0; t < MT; ++t) parts(g[d], t, s, pt[t]);
#pragma unroll
          for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int t = 0; t < MT; ++t) acc[t][0][s] += __uint_as_float(pt[t][q].x ^ pt[t][q].w);
#pragma unroll
          for (int i = 0; i < RTW; ++i) acc[0][i][4 + s] += __uint_as_float(g[d].w[i][s].y ^ g[d].w[i][s].z);
        }
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int t = 0; t < MT; ++t) {  // (t outside q: the same MFMA sequence per accumulator)
            u32x4_t pt[3];
            parts(g[d], t, s, pt);
#pragma unroll
            for (int q = 0; q < 3; ++q)
#pragma unroll
              for (int i = 0; i < RTW; ++i)
                acc[t][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, pt[q]),
                                                                     __builtin_bit_cast(bf16x8_t, g[d].w[i][s]), acc[t][i], 0, 0, 0);
          }
        }
      }
      load(j0 + d + PD, g[d]);
      asm volatile("" ::: "memory");
    }
  }
  // the waves' partial tiles -> ct[batch row][weight row], added in wave order.  Accumulator register
  // j of lane (r, h): batch row (j & 3) + 8 (j >> 2) + 4 h of tile t, weight row r of tile i.
  // reduction slots: one per wave where the slab fits 64 KB (then every wave stores once and the
  // ct pass adds (w, w + 4) pairs in the pre-add's order -- one barrier and one LDS round trip
  // fewer, same sums); else 8-wave blocks pre-add waves w + 4 into w through 4 slots
  // RED_HALF (8 waves, two row tiles, 128 KB of partials): the same single pass per row tile in turn
  // -- every wave stores its row tile t partials into its own slot, the ct pass builds rows 32 t ..
  // 32 t + 31 -- instead of the 4-slot pre-add (whose phases leave half the waves idle)
  constexpr bool RED_ALL = XW > 4 && MT * RTW * 16 * 64 * 4 * XW <= 65536;
  constexpr bool RED_HALF = !RED_ALL && XW > 4 && MT == 2 && RTW * 16 * 64 * 4 * XW <= 65536;
  constexpr int RW = (RED_ALL || RED_HALF) ? XW : (XW > 4 ? 4 : XW);
  __shared__ float red[RW][(RED_HALF ? 1 : MT) * RTW * 16][64];
  __shared__ float ct[NB][NBR + 1];
  __shared__ float hb[NB][NBR / 2 + 1];
  __shared__ float rsc[NB];
  __shared__ float pss[NB][NBR / 8 + 1], phs[NB][NBR / 8 + 1];  // producer: 8-column partial sums
  __shared__ int last;
  XS_STAMP(2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the LDS-DMA prefetch too; the barrier below publishes it)
  if constexpr ((XS_LAB & 8) != 0) {  // lab: the K loop alone (one store keeps it live)
    float v = 0.f;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int i = 0; i < RTW; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) v += acc[t][i][j];
    if (v == 1.2345f) p.out[tid] = v;
    return;
  }
  if constexpr (RED_HALF) {
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      if (t > 0) __syncthreads();  // row tile t - 1's partials consumed
#pragma unroll
      for (int i = 0; i < RTW; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) red[wave][i * 16 + j][lane] = acc[t][i][j];
      __syncthreads();
      for (int e = tid; e < 32 * NBR; e += NTH) {
        const int rr = e / NBR, c = e % NBR;
        const int idx = (c >> 5) * 16 + (rr & 3) + 4 * (rr >> 3), ln = (c & 31) + 32 * ((rr >> 2) & 1);
        float v = red[0][idx][ln] + red[4][idx][ln];  // the 4-slot pre-add's sums, in its order
#pragma unroll
        for (int w = 1; w < 4; ++w) v += red[w][idx][ln] + red[w + 4][idx][ln];
        ct[32 * t + rr][c] = v;
      }
    }
  }
  if constexpr (XW > 4 && !RED_ALL && !RED_HALF) {  // waves 4..7 hand their tiles to waves 0..3 (added in registers)
    if (wave >= 4) {
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int i = 0; i < RTW; ++i)
#pragma unroll
          for (int j = 0; j < 16; ++j) red[wave - 4][(t * RTW + i) * 16 + j][lane] = acc[t][i][j];
    }
    __syncthreads();
    if (wave < 4) {
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int i = 0; i < RTW; ++i)
#pragma unroll
          for (int j = 0; j < 16; ++j) acc[t][i][j] += red[wave][(t * RTW + i) * 16 + j][lane];
    }
    __syncthreads();
  }
  if constexpr (!RED_HALF) {
  if (wave < RW) {
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int i = 0; i < RTW; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) red[wave][(t * RTW + i) * 16 + j][lane] = acc[t][i][j];
  }
  __syncthreads();
  for (int e = tid; e < NB * NBR; e += NTH) {
    const int ml = e / NBR, c = e % NBR, rr = ml & 31;
    const int idx = ((ml >> 5) * RTW + (c >> 5)) * 16 + (rr & 3) + 4 * (rr >> 3), ln = (c & 31) + 32 * ((rr >> 2) & 1);
    float v;
    if constexpr (RED_ALL) {  // ((s0 + s1) + s2) + s3 with s_w = wave w + wave w + 4, as the pre-add
      v = red[0][idx][ln] + red[4][idx][ln];
#pragma unroll
      for (int w = 1; w < 4; ++w) v += red[w][idx][ln] + red[w + 4][idx][ln];
    } else {
      v = red[0][idx][ln];
#pragma unroll
      for (int w = 1; w < RW; ++w) v += red[w][idx][ln];
    }
    ct[ml][c] = v;
  }
  }
  __syncthreads();
  XS_STAMP(3);
  if constexpr ((XS_LAB & 16) != 0) {  // lab: stop after the waves' reduction (no exchange, no epilogue)
    if (ct[tid & 31][0] == 1.2345f) p.out[tid] = 0.f;
    return;
  }
  if (ks > 1) {
    // slice partial [NB][NBR] write-through, ticket; the last slice to arrive sums all in slice order
    const int slab_f = NB * NBR;
    float* slab = p.kpart + (size_t)tile * ks * slab_f;
    const __amdgpu_buffer_rsrc_t rs = rsrc(slab, ks * slab_f * 4);
    const int mine = slice * slab_f * 4;
    for (int q = tid; q < mrows * (NBR / 4); q += NTH) {
      const int ml = q / (NBR / 4), j = (q % (NBR / 4)) * 4;
      const f32x4_t v = {ct[ml][j], ct[ml][j + 1], ct[ml][j + 2], ct[ml][j + 3]};
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, q * 16, mine, SC1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    XS_STAMP(4);
    if (tid == 0) {
      gu32* tk = (gu32*)p.kticket + tile;
      const unsigned old = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = (old == (unsigned)ks - 1);
      if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
    }
    __syncthreads();
    XS_STAMP(5);
    if (!last) return;
    switch (ks) {
      case 2: combine<2, NB, NBR, NTH>(rs, ct, mrows, slab_f, tid); break;
      case 4: combine<4, NB, NBR, NTH>(rs, ct, mrows, slab_f, tid); break;
      case 8: combine<8, NB, NBR, NTH>(rs, ct, mrows, slab_f, tid); break;
      default: combine<16, NB, NBR, NTH>(rs, ct, mrows, slab_f, tid); break;
    }
    __syncthreads();
    XS_STAMP(6);
  }
  // ---- epilogue
  if (norm && tid < mrows) {
    float s = 0.f;
    for (int t = 0; t < p.ss_n; ++t) s += sss[t * NB + tid];
    rsc[tid] = rsqrtf(s / (float)p.K + p.eps);
  }
  __syncthreads();
  const bool prod = p.xs_out != nullptr;
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
      va = res[ml * NBR + rp] + va;
      vb = res[ml * NBR + rp + 1] + vb;
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
    // the produced rows, 8 columns (one 16-B fragment per part) per thread step; per-row sums of squares
    // (un-normed values) and half-group sums (split values) as 8-column partials in LDS, then summed in
    // column order
    const int ncol = silu ? NBR / 2 : NBR, col0 = silu ? n0 / 2 : n0, colN = silu ? p.N / 2 : p.N;
    const int ng = ncol / 8;
    for (int q = tid; q < mrows * ng; q += NTH) {
      const int ml = q / ng, g8 = q % ng, c = 8 * g8, col = col0 + c;
      float v[8], sq = 0.f, hsum = 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float x = silu ? hb[ml][c + u] : ct[ml][c + u];
        sq = fmaf(x, x, sq);
        v[u] = p.xs_nw ? x * nws[c + u] : x;
        hsum += v[u];
      }
      if (col < colN) xs::store8(p.xs_out, p.xs_K, ml, col, v);
      pss[ml][g8] = sq;
      phs[ml][g8] = hsum;
    }
    __syncthreads();
    if (p.ss_out && !silu && tid < mrows) {
      float sq = 0.f;
      for (int g8 = 0; g8 < ng; ++g8) sq += pss[tid][g8];
      p.ss_out[(size_t)tile * p.ss_stride + tid] = sq;
    }
    if (p.hs_out)  // 32-column halves (4 partials each)
      for (int q = tid; q < mrows * (ncol / 32); q += NTH) {
        const int ml = q / (ncol / 32), hh = q % (ncol / 32);
        if (col0 + 32 * hh >= colN) continue;
        p.hs_out[(size_t)((col0 + 32 * hh) / 32) * xs::HS_ROWS + ml] =
            ((phs[ml][4 * hh] + phs[ml][4 * hh + 1]) + phs[ml][4 * hh + 2]) + phs[ml][4 * hh + 3];
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
  if constexpr (XS_STAMPS != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    XS_STAMP(7);
  }
}

// Launch shape: RTW 2 (64-row tiles) for the wide and the long-K projections and for the heads (the
// arg-max partial count then equals gemm_wide's 64-row tiles), else 1; K slices doubled until the grid
// has >= 256 blocks while every wave keeps >= 1 stage; ring depth <= 4 stages (<= 2 at 64 rows).
void xs_shape(int N, int K, int M, bool head, int& rtw, int& ks, int& pd, int& xw) {
  const int nks = K / XK;
  // long-K projections (down) on 32-row tiles: twice the tiles, half the split-K slices and a quarter of
  // the partial bytes to combine -- 12.1 vs 16.7 us for the decoder down at 32 rows (tools/gemm_bench.py)
  static const int rtw_long = [] { const char* v = getenv("CSM_XS_LONGK_RTW"); return v ? atoi(v) : 1; }();
  rtw = (N >= 4096 || head) ? 2 : (K >= 4096 ? rtw_long : 1);
  const int tiles = (N + 32 * rtw - 1) / (32 * rtw);
  // split-K slices until the grid has >= `target` blocks (CSM_XS_BLOCKS lab knob).  The depth decoder's
  // small projections at <= 32 rows (QKV / o, N x K <= 1536 x 1024) take none (target 1,
  // CSM_XS_SMALL_BLOCKS): one K slice over 8 waves, no partial exchange -- decoder QKV 7.2 -> 6.3 us,
  // o 6.7 -> 6.2 us, config 4 4347 -> 4378 frames/s (profiles/r04_ab_step1_small.txt); the backbone's
  // o (2048 x 2048) measured ~2 us slower that way and keeps its slices (profiles/r04_prof_config4_per_frame_final.txt)
  static const int target = [] { const char* v = getenv("CSM_XS_BLOCKS"); return v ? atoi(v) : 256; }();
  static const int small_target = [] { const char* v = getenv("CSM_XS_SMALL_BLOCKS"); return v ? atoi(v) : 1; }();
  const bool dec_small = (size_t)N * K <= (size_t)1536 * 1024 && M <= 32 && !head;
  // the arg-max heads (N not a multiple of 64: the padded vocabulary): CSM_XS_HEAD_BLOCKS lab knob
  static const int head_target = [] { const char* v = getenv("CSM_XS_HEAD_BLOCKS"); return v ? atoi(v) : 256; }();
  const int tgt = dec_small ? small_target : (head && N % 64 != 0 ? head_target : target);
  // waves per block; the block's K slice is split between them.  4 (one per SIMD of the CU the block
  // occupies) against 2: QKV 9.4 -> 7.2 us and o 8.0 -> 6.8 us at 32 bf16 rows, int4 gate/up 24.7 -> 16.1
  // and down 20.6 -> 16.1 us at 64 rows; config 4 3667 -> 3816, config 5 3501 -> 4035 frames/s
  // (profiles/r04_ab_xs_waves.txt).  8 (two per SIMD: one wave's loads / int4 fold overlap the other's
  // MFMAs) everywhere but the depth decoder's QKV / o at <= 32 rows (o 6.8 vs 7.2 us): gate/up 13.1 -> 11.6
  // and down 12.3 -> 11.3 us at 32 bf16 rows, int4 gate/up 16.1 -> 13.8, down 15.5 -> 13.8, QKV 10.6 ->
  // 9.8 us at 64 rows, the backbone's projections 4-14 % (profiles/r04_ab_xs_waves8.txt).  Lab knob
  // CSM_XS_WAVES=2 / 4 / 8 forces one count everywhere.
  static const int waves = [] { const char* v = getenv("CSM_XS_WAVES"); const int w = v ? atoi(v) : 0; return w == 2 || w == 4 || w == 8 ? w : 0; }();
  // the heads (arg-max epilogue, 64-row tiles, ~33 of them): fewer waves per block leave room for
  // more K slices, spreading the head's bytes over more CUs (CSM_XS_HEAD_WAVES lab knob).  4 waves (4 K
  // slices, 132 blocks at 32 rows) against 8 (2 slices, 66 blocks): config 4 4383-4409 -> 4496 frames/s,
  // config 5 5408 -> 5413; 2 waves 4352-4435 (profiles/r05_ab_head_waves.txt)
  static const int head_waves = [] { const char* v = getenv("CSM_XS_HEAD_WAVES"); const int w = v ? atoi(v) : 0; return w == 2 || w == 4 || w == 8 ? w : 4; }();
  // (the decoder's QKV / o at <= 32 rows: 8 waves now that they take one K slice; 4 with split-K)
  static const int small_waves = [] { const char* v = getenv("CSM_XS_SMALL_WAVES"); const int w = v ? atoi(v) : 0; return w == 2 || w == 4 || w == 8 ? w : 8; }();
  const int want = waves ? waves : (head && N % 64 != 0 ? head_waves : (dec_small ? small_waves : 8));
  xw = nks >= 2 * want ? want : (nks >= 8 ? 4 : 2);
  // every wave takes wst = nks / ks / xw whole stages: the waves must divide the slice's stages (K = 640:
  // 10 stages -> 2 waves), or the leftover stages would never be computed (gemm_xs_eligible rejects a
  // shape whose stage count no wave count divides)
  while (xw > 2 && nks % xw != 0) xw /= 2;
  ks = 1;
  while (tiles * ks < tgt && ks < MAX_SLICES && nks / (ks * 2) >= xw && nks % (ks * 2) == 0 && (nks / (ks * 2)) % xw == 0)
    ks *= 2;
  const int wst = nks / ks / xw;
  // ring depth at 64 rows with 64-row tiles (lab knob CSM_XS_PD64, default 1: register budget)
  static const int cap64 = [] { const char* v = getenv("CSM_XS_PD64"); return v ? std::max(1, atoi(v)) : 1; }();
  int cap = M > 32 ? (rtw == 2 ? cap64 : 2) : 4;
  if (xw == 8) cap = std::min(cap, M > 32 ? 1 : 2);  // two waves per SIMD: <= 256 registers, no spills
  pd = 1;
  while (pd * 2 <= cap && wst % (pd * 2) == 0) pd *= 2;
}

size_t xs_need(int N, int K, int M, bool head, size_t& tk) {
  int rtw, ks, pd, xw;
  xs_shape(N, K, M, head, rtw, ks, pd, xw);
  const size_t tiles = (N + 32 * rtw - 1) / (32 * rtw);
  tk = tiles;
  return ks > 1 ? tiles * ks * (size_t)(M > 32 ? 64 : 32) * 32 * rtw * 4 : 0;
}

}  // namespace

// Lab (XS_STAMPS builds): mean phase durations over the recorded launches, per launch shape, to stderr.
// Phases: 0 start, 1 ring issued, 2 K loop done, 3 waves reduced, 4 partial published, 5 ticket taken,
// 6 combined (last slice), 7 end.  No-op in product builds.
void gemm_xs_stamps_report(const char* tag) {
  if constexpr (XS_STAMPS == 0) {
    (void)tag;
  } else {
    static unsigned long long h[XS_ST_LAUNCHES][XS_ST_BLOCKS][XS_ST_N];
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(h, HIP_SYMBOL(g_xs_st), sizeof(h)) != hipSuccess) return;
    double sum[XS_ST_N] = {0};
    double cnt[XS_ST_N] = {0};
    for (int l = 0; l < XS_ST_LAUNCHES; ++l) {
      unsigned long long t0 = ~0ull;
      for (int b = 0; b < XS_ST_BLOCKS; ++b)
        if (h[l][b][0]) t0 = std::min(t0, h[l][b][0]);
      if (t0 == ~0ull) continue;
      for (int b = 0; b < XS_ST_BLOCKS; ++b)
        for (int k = 0; k < XS_ST_N; ++k)
          if (h[l][b][k] >= t0 && h[l][b][0]) { sum[k] += (double)(h[l][b][k] - t0) * 0.01; cnt[k] += 1; }
    }
    fprintf(stderr, "xs_stamps %s (us after the launch's first block start, mean over blocks):", tag);
    for (int k = 0; k < XS_ST_N; ++k) fprintf(stderr, " %d:%.2f(%d)", k, cnt[k] ? sum[k] / cnt[k] : -1.0, (int)cnt[k]);
    fprintf(stderr, "\n");
    static unsigned long long z[XS_ST_LAUNCHES][XS_ST_BLOCKS][XS_ST_N];
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_xs_st), z, sizeof(z));
  }
}

bool gemm_xs_eligible(int N, int K, int M, int wdt) {
  if (!(wdt == WDT_BF16 || wdt == WDT_Q4) || M < 1 || M > GEMM_XS_MAX_M || N % 2 || K % XK || K / XK < 2) return false;
  for (int h = 0; h < 2; ++h) {
    int rtw, ks, pd, xw;
    xs_shape(N, K, M, h == 1, rtw, ks, pd, xw);
    if ((K / XK) % ks != 0 || (K / XK / ks) % xw != 0) return false;  // every stage on exactly one wave
    if (wdt == WDT_Q4 && K / XK / ks > Q4_XG) return false;            // the X_g stage table holds <= Q4_XG stages
  }
  return true;
}

// Host-side shape query (csm_hip_prof.h csm_xs_shape): the launch geometry gemm_xs would use, for the
// CPU tests of the stage-coverage rule.
extern "C" int csm_xs_shape(int N, int K, int M, int head, int wdt, int* out) {
  int rtw, ks, pd, xw;
  xs_shape(N, K, M, head != 0, rtw, ks, pd, xw);
  out[0] = rtw; out[1] = ks; out[2] = pd; out[3] = xw;
  const int w = wdt == CSM_Q4 ? WDT_Q4 : (wdt == CSM_BF16 ? WDT_BF16 : -1);
  return w >= 0 && gemm_xs_eligible(N, K, M, w) ? 1 : 0;
}

__global__ void q4_expand_kernel(const uint32_t* w, int n, u32x4_t* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = xs::q4_word_bf16(w[i]);
}

extern "C" int csm_q4_expand(const uint32_t* words, int n, uint32_t* out) {
  if (!words || !out || n <= 0) return CSM_ERR_ARG;
  uint32_t* dw = nullptr;
  u32x4_t* dout = nullptr;
  int rc = CSM_ERR_HIP;
  if (hipMalloc(&dw, (size_t)n * 4) == hipSuccess && hipMalloc(&dout, (size_t)n * 16) == hipSuccess &&
      hipMemcpy(dw, words, (size_t)n * 4, hipMemcpyHostToDevice) == hipSuccess) {
    hipLaunchKernelGGL(q4_expand_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, dw, n, dout);
    if (hipGetLastError() == hipSuccess && hipMemcpy(out, dout, (size_t)n * 16, hipMemcpyDeviceToHost) == hipSuccess)
      rc = CSM_OK;
  }
  if (dw) (void)hipFree(dw);
  if (dout) (void)hipFree(dout);
  return rc;
}

int gemm_xs_tiles(int N, int K, int M, bool head) {
  int rtw, ks, pd, xw;
  xs_shape(N, K, M, head, rtw, ks, pd, xw);
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

void launch_gemm_xs(const GemvParams& p0, int epi, hipStream_t st, bool nt_w, int wdt) {
  GemvParams p = p0;
  p.epi = epi;
  p.Wt = nullptr;
  if (p.ws) {
    const auto ti = p.ws->tiled.find(p.W);
    if (ti != p.ws->tiled.end()) p.Wt = ti->second;
  }
  if (!p.Wt || !p.xs_in || p.M > GEMM_XS_MAX_M || p.scale || (wdt == WDT_Q4 && !p.hs_in) ||
      !gemm_xs_eligible(p.N, p.K, p.M, wdt)) {
    fprintf(stderr, "csm: gemm_xs launch without a tiled weight / split activations, or with an unsupported option (N=%d K=%d M=%d)\n",
            p.N, p.K, p.M);
    abort();
  }
  // 64-row tiles for the heads (arg-max partial count) and for SiLU*up producers (32 whole output
  // columns per tile: the int4 consumer's half-group sums never span two tiles)
  const bool head = epi == EPI_ARGMAX || epi == EPI_SILU_MUL;
  int rtw, ks, pd, xw;
  xs_shape(p.N, p.K, p.M, head, rtw, ks, pd, xw);
  if (wdt == WDT_Q4 && rtw == 2 && pd > 2) pd = 2;  // the int4 fold's per-group products: a shorter ring (no spills)
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
  const bool nt = epi == EPI_ARGMAX || nt_w;
  const dim3 grid(tiles, ks);
  if constexpr (XS_STAMPS != 0) {
    static unsigned n = 0;
    p.lab_launch = n++;
  }
#define GX_W(Q_, MT_, RTW_, PD_, NT_) do { if (xw == 4) hipLaunchKernelGGL((gemm_xs_kernel<Q_, MT_, RTW_, PD_, NT_, 4>), grid, dim3(256), 0, st, p); \
                                             else if (xw == 8) hipLaunchKernelGGL((gemm_xs_kernel<Q_, MT_, RTW_, PD_, NT_, 8>), grid, dim3(512), 0, st, p); \
                                             else hipLaunchKernelGGL((gemm_xs_kernel<Q_, MT_, RTW_, PD_, NT_, 2>), grid, dim3(128), 0, st, p); } while (0)
#define GX_K(Q_, MT_, RTW_, PD_) do { if (nt) GX_W(Q_, MT_, RTW_, PD_, true); else GX_W(Q_, MT_, RTW_, PD_, false); } while (0)
#define GX_P(Q_, MT_, RTW_) do { if (pd == 4) GX_K(Q_, MT_, RTW_, (MT_ == 1 ? 4 : 2)); else if (pd == 2) GX_K(Q_, MT_, RTW_, 2); \
                                 else GX_K(Q_, MT_, RTW_, 1); } while (0)
#define GX_M(Q_) do { if (p.M > 32) { if (rtw == 2) GX_P(Q_, 2, 2); else GX_P(Q_, 2, 1); } \
                      else { if (rtw == 2) GX_P(Q_, 1, 2); else GX_P(Q_, 1, 1); } } while (0)
  const int role = p.epi == EPI_QKV ? 1 : (p.epi == EPI_ADD ? (p.K > p.N ? 3 : 2) : 0);
#ifndef XS_ROLES
#define XS_ROLES 1  // lab: 0 launches the untagged instantiations (A/B)
#endif
  if (XS_ROLES && role && !nt && xw == 8 && rtw == 1 && ((wdt == WDT_Q4 && p.M > 32 && pd == 1) || (wdt == WDT_BF16 && p.M <= 32 && pd == 2))) {
#define GX_R(Q_, MT_, PD_) do { if (role == 1) hipLaunchKernelGGL((gemm_xs_kernel<Q_, MT_, 1, PD_, false, 8, 1>), grid, dim3(512), 0, st, p); \
                                else if (role == 2) hipLaunchKernelGGL((gemm_xs_kernel<Q_, MT_, 1, PD_, false, 8, 2>), grid, dim3(512), 0, st, p); \
                                else hipLaunchKernelGGL((gemm_xs_kernel<Q_, MT_, 1, PD_, false, 8, 3>), grid, dim3(512), 0, st, p); } while (0)
    if (wdt == WDT_Q4) GX_R(true, 2, 1);
    else GX_R(false, 1, 2);
#undef GX_R
  } else if (wdt == WDT_Q4) {
    GX_M(true);
  } else {
    GX_M(false);
  }
#undef GX_M
#undef GX_P
#undef GX_K
#undef GX_W
}
