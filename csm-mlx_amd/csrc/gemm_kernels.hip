// Batched projections on the matrix cores (gfx950 MFMA) for B >= 8 utterances and prompt prefill.
//
// y[m, n] = sum_k norm(x)[m, k] * W[n, k]   -- every nn.Linear of the backbone / decoder and the
// codebook heads (models.py:50-67, generation.py:42, :74-79) once the row count M makes the
// GEMV's per-row loop (gemv_kernel re-streams the weights every MT rows) the bottleneck.
//
// Exactness.  The greedy bar is bit-exact RVQ codes against an fp32 reference, so every product
// must be an fp32-exact one:
//   * activations (fp32, RMSNorm-weighted) are split into three bf16 parts x = hi + mid + lo
//     (hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid)); the three parts hold all 24
//     significant bits of x, and each part times a bf16 weight is exact in fp32 -- three
//     v_mfma_f32_32x32x16_bf16 per K-step, fp32 accumulation: the arithmetic of an fp32 GEMV up to
//     summation order;
//   * int4 weights (MLX affine, group 64: w = scale * q + bias) are NOT dequantized: the nibbles
//     q in [0, 15] are exact bf16 operands, so per group g the matrix cores give
//     S_g = sum_k q_k x_k (three products per K-step as above) and the staging threads give
//     X_g = sum_k x_k; the accumulator folds acc += scale_g * S_g + bias_g * X_g per group
//     (scale, bias bf16 as stored).  Same operand count as a bf16 weight.
// v_mfma_f32_32x32x16_bf16 fragments: lane l = (r = l & 31, h = l >> 5) holds A[row r][k 8h..8h+7]
// and B[k 8h..8h+7][col r]; C[row (j&3) + 8(j>>2) + 4h][col r] in accumulator register j.
//
// Kernel "pipe": the block's weight tile AND activation tile go through LDS with coalesced global
// loads into a register ring of PD stages (loads of stages c+1..c+PD in flight while stage c runs
// on the matrix cores from a double-buffered LDS tile; PD = 1 / 2 / 4 by the stage count).  Block =
// 64 weight rows x 32*MT batch rows over one K slice, stages of 64 K (4 MFMA steps = one int4
// group); every fragment is stored in MFMA-lane order (one conflict-free ds_read_b128 per operand).
// MT = 2: 2 x 2 waves over (row tile, batch tile); MT = 1: 2 waves per row tile split each stage's
// K steps and are summed in a fixed order.  Split-K: each slice publishes its tile write-through
// (16-B sc1 stores, drained), takes an arrival ticket; the last slice of a tile to arrive reads
// every partial back with 16-B sc1 loads (MI355X_MICROARCH.md hand-off table, single-counter row),
// sums them in slice order (deterministic) and runs the epilogue -- RoPE + KV append, residual
// add, SiLU*up or the heads' arg-max partials -- no second launch.  The slabs and tickets belong
// to the calling engine (GemmWs), sized outside graph capture by gemm_reserve.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "csm_kernels.h"
#include "xs.h"

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) const f32x4_t gcf32x4;

constexpr int GP_KC = 64;  // K per stage (= Q4_GROUP)
constexpr int GK_MAX_SLICES = 16;
static_assert(GP_KC == Q4_GROUP, "one int4 group per stage");


// x -> three bf16 parts holding all 24 significant bits, by truncation: hi = x with its low 16
// bits cleared (8 significant bits), r = x - hi (exact, <= 16 bits), mid = r truncated the same
// way, lo = r - mid (exact, <= 8 bits: a bf16 value) -- x = hi + mid + lo exactly, and each part
// times a bf16 weight is exact in fp32.  Pairs are packed by v_perm (the high halves of two floats).
__device__ __forceinline__ void split3_4(const float (&v)[4], u32x2_t& hi, u32x2_t& mid, u32x2_t& lo) {
  uint32_t h[4], m[4], l[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t u = __float_as_uint(v[q]);
    h[q] = u & 0xFFFF0000u;
    const float r = v[q] - __uint_as_float(h[q]);
    m[q] = __float_as_uint(r) & 0xFFFF0000u;
    l[q] = __float_as_uint(r - __uint_as_float(m[q]));
  }
  hi = u32x2_t{__builtin_amdgcn_perm(h[1], h[0], 0x07060302u), __builtin_amdgcn_perm(h[3], h[2], 0x07060302u)};
  mid = u32x2_t{__builtin_amdgcn_perm(m[1], m[0], 0x07060302u), __builtin_amdgcn_perm(m[3], m[2], 0x07060302u)};
  lo = u32x2_t{__builtin_amdgcn_perm(l[1], l[0], 0x07060302u), __builtin_amdgcn_perm(l[3], l[2], 0x07060302u)};
}

// sum over each row of 16 lanes by DPP (row rotations by 8 and 4, then quad swaps): every lane of
// the row gets the sum, in an order fixed by its position
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));  // row_ror:8
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false));  // row_ror:4
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  return v;
}

// Split-K combine (the last slice of a tile to arrive): every slice's partial is read with 16-B sc1
// buffer loads, KS * U of them in flight per thread before the first add, and summed in slice order
// (deterministic).
constexpr int GP_RSRC3 = 0x00020000;  // buffer descriptor word 3 (raw 32-bit format)
constexpr int GP_SC1 = 16;            // cache policy: sc1 (agent-coherent, as __hip_atomic_load/store)
constexpr int GP_NT = 2;              // cache policy: non-temporal
template <int KS, int NB, int NBR, int NTH>
__device__ __forceinline__ void gp_combine(__amdgpu_buffer_rsrc_t rs, float (*ct)[NBR + 1], float* ssb,
                                           int mrows, bool norm, int slab_f, int tid) {
  constexpr int U = KS >= 16 ? 1 : 16 / KS;
  const int nq = mrows * (NBR / 4);
  for (int q0 = tid; q0 < nq; q0 += NTH * U) {
    f32x4_t v[U][KS];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = min(q0 + NTH * u, nq - 1);
#pragma unroll
      for (int s = 0; s < KS; ++s) v[u][s] = __builtin_amdgcn_raw_buffer_load_b128(rs, q * 16, s * slab_f * 4, GP_SC1);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = q0 + NTH * u;
      if (q < nq) {
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
  if (norm && tid < mrows) {
    float v[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s)
      v[s] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (NB * NBR + tid) * 4, s * slab_f * 4, GP_SC1));
    float sum = v[0];
#pragma unroll
    for (int s = 1; s < KS; ++s) sum += v[s];
    ssb[tid] = sum;
  }
}

// Block = NW waves (4; 8 for long prompts: two per SIMD, so one wave's staging / int4 fold runs
// beside the other's MFMAs) over NBR weight rows x 32*MT batch rows x one K slice, stages of 64 K
// (one int4 group).  The activations are the MFMA A operand (rows = batch rows), the weights the B operand
// (columns = weight rows): every lane's 16 accumulators then share ONE weight row, whose int4
// scale / bias it loaded itself.  Weights go global -> registers in fragment order (no LDS): with
// the K order permuted inside a stage (step s, half h <-> k = 32h + 8s + j, the same permutation on
// both operands) lane (r, h) reads 64 contiguous bytes of weight row r per bf16 stage (16 for int4).
// Activations go global -> registers -> (RMSNorm weight, sum of squares, hi/mid/lo split) -> LDS
// once per stage and are shared by the block's NBR / 32 row tiles.  4 waves: NBR = 256: 2 row tiles
// per wave; 128: one; 64: two waves per row tile split each stage's steps (summed in a fixed order);
// 8 waves: 256: one row tile per wave; 128 / 64: 2 / 4 waves per row tile.
#ifdef GEMM_STAMPS  // lab build only (tools/variant.sh ... -DGEMM_STAMPS): per-block phase clocks
__device__ unsigned long long g_gemm_stamps[1024][6];
#define GSTAMP(i) do { if (threadIdx.x == 0 && blin < 1024) g_gemm_stamps[blin][i] = __builtin_amdgcn_s_memrealtime(); } while (0)
extern "C" int csm_gemm_stamps(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gemm_stamps), sizeof(unsigned long long) * 6 * (size_t)(n < 1024 ? n : 1024)) == hipSuccess ? 0 : 1;
}
#else
#define GSTAMP(i) do {} while (0)
#endif

#ifndef GW_LAB
#define GW_LAB 0  // lab ablations (tools/variant.sh -DGW_LAB=bits, results invalid): 1 staging without norm / split /
                  // group sums, 2 no int4 scale / bias fold, 4 no MFMA (operands consumed by one VALU op), 8 no int4
                  // -> bf16 expansion, 16 no LDS reads of the activation fragments
#endif
template <bool Q4, int MT, int NBR, int PD, bool NT, int NW = 4>
__global__ __launch_bounds__(64 * NW) void gemm_wide_kernel(GemvParams p) {
  constexpr int NB = MT * 32, NTH = 64 * NW;
  constexpr int NTILE = NBR / 32;                            // 32-row tiles of the block
  constexpr int RTW = NTILE > NW ? NTILE / NW : 1;           // row tiles per wave
  constexpr int KW = NW > NTILE ? NW / NTILE : 1;            // waves per row tile (they split the steps)
  constexpr int NGRP = NTILE / RTW;                          // wave groups (one per RTW row tiles)
  constexpr int NS = 4 / KW;                                 // k-steps per wave per stage
  constexpr int RPT = NTH / 16, NI = NB / RPT;               // activation staging: rows per pass, passes
  static_assert(NI >= 1 && NS >= 1 && NGRP * KW == NW, "wave layout");
  constexpr int SLOTS = 65;                // 16-B slots per (part, batch tile, step) block: lane l at l + l / 32
  constexpr int XS_BYTES = 2 * 3 * MT * 4 * SLOTS * 16;
  constexpr int CT_BYTES = NB * (NBR + 1) * 4;
  constexpr int SM = XS_BYTES > CT_BYTES ? XS_BYTES : CT_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM];
  // GW_QB: the int4 bias term sum_g bias_g[n] X_g[m] on the matrix cores, 16 stages at a time (X_g split in
  // three exact bf16 parts, the bf16 biases as the B operand: three MFMAs per tile pair) instead of an fmaf per
  // accumulator per stage; X_g and the biases wait in 32-stage rings
#ifndef GW_QB
#define GW_QB 1
#endif
  constexpr bool QB = Q4 && GW_QB != 0;
  __shared__ __attribute__((aligned(16))) float xsum[QB ? 32 : 2][NB];  // int4: the stage's sum of x per batch row
  __shared__ uint16_t bsh[QB ? 32 : 1][QB ? NBR : 1];
  __shared__ float ssb[NB];
  __shared__ int last;
  auto Xs = [&](int buf, int part, int t, int s) {
    return reinterpret_cast<u32x4_t*>(smem) + (((buf * 3 + part) * MT + t) * 4 + s) * SLOTS;
  };
  float (*ct)[NBR + 1] = reinterpret_cast<float (*)[NBR + 1]>(smem);  // after the K loop
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5, slot = lane + h;
  // grid (row tile, K slice, batch chunk): tiles fastest in dispatch order (measured: the
  // chunk-major order cost configs 4 / 5 3-4 %)
  const int tile = blockIdx.x, n0 = tile * NBR;
  const int blin = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  (void)blin;
  GSTAMP(0);
  const int mc = blockIdx.z, m0 = mc * NB, nchunks = gridDim.z;
  const int Kblk = p.K / p.ksplit, kslice = blockIdx.y * Kblk, nst = Kblk / GP_KC;
  const bool norm = p.nw != nullptr;
  const int kh = wave / NGRP;
  const int rt0 = (wave % NGRP) * RTW;
  // this lane's weight bytes in the fragment-tiled copy (gemm_retile): row tile T, stage kst at
  // T * nks + kst blocks of 4 KB (bf16; + 1 KB per step) or 1 KB (int4; scale|bias words after)
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.Wt), 0, 0x7fffffff, GP_RSRC3);
  const int nks = p.K / GP_KC, nt32 = (p.N + 31) / 32;
  int wv[RTW], sv[RTW];
#pragma unroll
  for (int i = 0; i < RTW; ++i) {
    const int T = min(n0 / 32 + rt0 + i, nt32 - 1);
    wv[i] = Q4 ? T * nks * 1024 + 16 * lane : T * nks * 4096 + 16 * lane + 1024 * NS * kh;
    sv[i] = nt32 * nks * 1024 + (T * nks * 32 + r) * 4;
  }
  // activation staging map: thread -> batch row x_c + 16 i, k x_k4 .. x_k4 + 3 of the stage
  const int x_c = tid >> 4, x_k4 = (tid & 15) * 4;
  const int st_h = x_k4 >> 5, st_s = (x_k4 >> 3) & 3, st_j = (x_k4 >> 2) & 1;
  float ss[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) ss[i] = 0.f;
  struct Stage {
    u32x4_t w[RTW][Q4 ? 1 : NS];
    uint32_t sb[RTW];
    f32x4_t xr[NI];
    f32x4_t nwr;
  };
  Stage sg[PD];
  const float* nwp = norm ? p.nw : p.x;
  // Straight-line loads (no branch between a load and the waits that follow it, so the compiler's
  // vmcnt counts stay exact): stages past the slice read through zero-sized buffer descriptors
  // (out of range: zeros, no memory traffic).  Activations first: a wait for the next stage's
  // activations (its LDS store) then leaves every younger weight load of the ring in flight
  // (vmcnt retires in issue order).
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.x), 0, 0x7fffffff, GP_RSRC3);
  const __amdgpu_buffer_rsrc_t nrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(nwp), 0, 0x7fffffff, GP_RSRC3);
  const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.Wt), 0, 0, GP_RSRC3);
  int xv[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) xv[i] = (min(m0 + x_c + RPT * i, p.M - 1) * p.xs + x_k4) * 4;
  auto load = [&](int st, Stage& g) {
    const bool live = st < nst;
    const int kc = kslice + (live ? st : 0) * GP_KC;
    const __amdgpu_buffer_rsrc_t xr = live ? xrs : zrs, nr = live ? nrs : zrs, wr = live ? wrs : zrs;
#pragma unroll
    for (int i = 0; i < NI; ++i) g.xr[i] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(xr, xv[i], kc * 4, 0));
    g.nwr = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(nr, x_k4 * 4, kc * 4, 0));
#pragma unroll
    for (int i = 0; i < RTW; ++i) {
      if constexpr (Q4) {
        g.w[i][0] = __builtin_amdgcn_raw_buffer_load_b128(wr, wv[i], (kc / GP_KC) * 1024, NT ? GP_NT : 0);
        g.sb[i] = __builtin_amdgcn_raw_buffer_load_b32(wr, sv[i], (kc / GP_KC) * 128, 0);
      } else {
#pragma unroll
        for (int s = 0; s < NS; ++s) g.w[i][s] = __builtin_amdgcn_raw_buffer_load_b128(wr, wv[i], (kc / GP_KC) * 4096 + 1024 * s, NT ? GP_NT : 0);
      }
    }
  };
  auto store = [&](const Stage& g, int buf, bool live, int st) {
    const int xslot = QB ? (st & 31) : buf;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int c = x_c + RPT * i;
      float v[4] = {g.xr[i].x, g.xr[i].y, g.xr[i].z, g.xr[i].w};
      if constexpr ((GW_LAB & 1) != 0) {  // the same LDS stores of raw bits: the staging's memory side only
        const u32x2_t raw = {__float_as_uint(v[0]) ^ __float_as_uint(g.nwr.x), __float_as_uint(v[2])};
        const int sl = (c & 31) + 33 * st_h;
        *(reinterpret_cast<u32x2_t*>(&Xs(buf, 0, c >> 5, st_s)[sl]) + st_j) = raw;
        *(reinterpret_cast<u32x2_t*>(&Xs(buf, 1, c >> 5, st_s)[sl]) + st_j) = raw;
        *(reinterpret_cast<u32x2_t*>(&Xs(buf, 2, c >> 5, st_s)[sl]) + st_j) = raw;
        if (live && (tid & 15) == 0) xsum[xslot][c] = v[1];
        continue;
      }
      if (norm) {
        const float nw4[4] = {g.nwr.x, g.nwr.y, g.nwr.z, g.nwr.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ss[i] = live ? fmaf(v[q], v[q], ss[i]) : ss[i];
          v[q] *= nw4[q];
        }
      }
      if constexpr (Q4) {  // sum of the group's 64 values of row c: 16 threads x 4, fixed order
        const float sum = row16_sum((v[0] + v[1]) + (v[2] + v[3]));
        if ((tid & 15) == 0) xsum[xslot][c] = sum;
      }
      u32x2_t hi, mid, lo;
      split3_4(v, hi, mid, lo);
      const int sl = (c & 31) + 33 * st_h;
      *(reinterpret_cast<u32x2_t*>(&Xs(buf, 0, c >> 5, st_s)[sl]) + st_j) = hi;
      *(reinterpret_cast<u32x2_t*>(&Xs(buf, 1, c >> 5, st_s)[sl]) + st_j) = mid;
      *(reinterpret_cast<u32x2_t*>(&Xs(buf, 2, c >> 5, st_s)[sl]) + st_j) = lo;
    }
  };
  f32x16_t acc[MT][RTW];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < RTW; ++i) acc[t][i] = f32x16_t{};
#pragma unroll
  for (int d = 0; d < PD; ++d) load(d, sg[d]);
  store(sg[0], 0, true, 0);
  __syncthreads();
  GSTAMP(1);
  for (int it0 = 0; it0 < nst; it0 += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      const int it = it0 + d, buf = it & 1;
      const Stage& g = sg[d];
      f32x16_t gq[MT][RTW];
      if constexpr (Q4) {
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int i = 0; i < RTW; ++i) gq[t][i] = f32x16_t{};
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int step = NS * kh + s;
        bf16x8_t b[RTW];
#pragma unroll
        for (int i = 0; i < RTW; ++i) {
          if constexpr (Q4) {  // (KW > 1: the wave's share of the 4 words, selected without indexing)
            uint32_t word = g.w[i][0][s];
            if constexpr (KW == 2) word = kh ? g.w[i][0][NS + s] : g.w[i][0][s];
            if constexpr (KW == 4) word = kh == 0 ? g.w[i][0][0] : (kh == 1 ? g.w[i][0][1] : (kh == 2 ? g.w[i][0][2] : g.w[i][0][3]));
            if constexpr ((GW_LAB & 8) != 0) b[i] = __builtin_bit_cast(bf16x8_t, u32x4_t{word, word ^ 1u, word ^ 2u, word ^ 3u});
            else b[i] = __builtin_bit_cast(bf16x8_t, xs::q4_word_bf16(word));
          } else {
            b[i] = __builtin_bit_cast(bf16x8_t, g.w[i][s]);
          }
        }
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int part = 0; part < 3; ++part) {
            const bf16x8_t a = (GW_LAB & 16) != 0 ? __builtin_bit_cast(bf16x8_t, u32x4_t{(uint32_t)slot, (uint32_t)part, (uint32_t)t, (uint32_t)(step + it)})
                                                  : __builtin_bit_cast(bf16x8_t, Xs(buf, part, t, step)[slot]);
#pragma unroll
            for (int i = 0; i < RTW; ++i) {
              if constexpr ((GW_LAB & 4) != 0) gq[t][i][part] += __builtin_bit_cast(float, __builtin_bit_cast(u32x4_t, a).x ^ __builtin_bit_cast(u32x4_t, b[i]).y);
              else if constexpr (Q4) gq[t][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[i], gq[t][i], 0, 0, 0);
              else acc[t][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[i], acc[t][i], 0, 0, 0);
            }
          }
      }
      if constexpr (QB) {  // acc += scale * S_g; the biases to their ring, their products every 16 stages
        if (kh == 0 && lane < 32)
#pragma unroll
          for (int i = 0; i < RTW; ++i) bsh[it & 31][32 * (rt0 + i) + lane] = (uint16_t)(g.sb[i] >> 16);
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int i = 0; i < RTW; ++i) {
            const float sc = bf16_lo(g.sb[i]);
#pragma unroll
            for (int j = 0; j < 16; ++j) acc[t][i][j] = fmaf(sc, gq[t][i][j], acc[t][i][j]);
          }
        if (kh == 0 && ((it & 15) == 15 || it == nst - 1)) {
          const int c0 = it & ~15;
#pragma unroll
          for (int t = 0; t < MT; ++t) {
            uint32_t xa[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const int gi = c0 + 8 * h + k;
              xa[k] = gi <= it ? __float_as_uint(xsum[gi & 31][32 * t + r]) : 0u;
            }
            u32x4_t pa[3];
            xs::split_frag(u32x4_t{xa[0], xa[1], xa[2], xa[3]}, u32x4_t{xa[4], xa[5], xa[6], xa[7]}, pa);
#pragma unroll
            for (int i = 0; i < RTW; ++i) {
              u32x4_t bw;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int gi = c0 + 8 * h + 2 * e;
                const uint32_t lo = gi <= it ? bsh[gi & 31][32 * (rt0 + i) + r] : 0u;
                const uint32_t hi = gi + 1 <= it ? bsh[(gi + 1) & 31][32 * (rt0 + i) + r] : 0u;
                bw[e] = lo | (hi << 16);
              }
#pragma unroll
              for (int q = 0; q < 3; ++q)
                acc[t][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, pa[q]), __builtin_bit_cast(bf16x8_t, bw), acc[t][i], 0, 0, 0);
            }
          }
        }
      } else if constexpr (Q4) {  // acc += scale * S_g + bias * X_g: this lane's weight row, 16 batch rows
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          float xs[16];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4_t x4 = kh == 0 ? *reinterpret_cast<const f32x4_t*>(&xsum[buf][32 * t + 8 * q + 4 * h]) : f32x4_t{};
            xs[4 * q] = x4.x; xs[4 * q + 1] = x4.y; xs[4 * q + 2] = x4.z; xs[4 * q + 3] = x4.w;
          }
#pragma unroll
          for (int i = 0; i < RTW; ++i) {
            const float sc = bf16_lo(g.sb[i]), bi = bf16_hi(g.sb[i]);
#pragma unroll
            for (int j = 0; j < 16; ++j) {
              if constexpr ((GW_LAB & 2) != 0) { acc[t][i][j] += gq[t][i][j]; continue; }
              acc[t][i][j] = fmaf(sc, gq[t][i][j], acc[t][i][j]);
              acc[t][i][j] = fmaf(bi, xs[j], acc[t][i][j]);
            }
          }
        }
      }
      if constexpr (PD == 1) {  // one slot (mostly one-stage slices): refill it first, nothing to protect
        if (it + 1 < nst) {
          load(it + 1, sg[0]);
          store(sg[0], buf ^ 1, true, it + 1);
        }
      } else {
        store(sg[(d + 1) % PD], buf ^ 1, it + 1 < nst, it + 1);  // past the slice: zeros into the idle buffer
        load(it + PD, sg[d]);
      }
      __syncthreads();
    }
  }
  GSTAMP(2);
  // sum of squares per batch row: the 16 threads of a row share it
  if (norm) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const float v = row16_sum(ss[i]);
      if ((tid & 15) == 0) ssb[x_c + RPT * i] = v;
    }
  }
  // accumulators -> C tile [batch row][weight row]; lane (r, h) register j: batch row
  // (j & 3) + 8 (j >> 2) + 4 h of tile t, weight row r of row tile rt0 + i
  if (kh == 0) {
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int i = 0; i < RTW; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) ct[32 * t + (j & 3) + 8 * (j >> 2) + 4 * h][32 * (rt0 + i) + r] = acc[t][i][j];
  }
  __syncthreads();
#pragma unroll
  for (int kk = 1; kk < KW; ++kk) {  // the later step shares, added in a fixed order
    if (kh == kk) {
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int j = 0; j < 16; ++j) ct[32 * t + (j & 3) + 8 * (j >> 2) + 4 * h][32 * rt0 + r] += acc[t][0][j];
    }
    __syncthreads();
  }
  const int mrows = min(NB, p.M - m0);
  if (p.ksplit > 1) {
    // slice partial = [NB][NBR] tile values, then [NB] sums of squares; 16-B write-through stores
    const int slab_f = NB * NBR + NB;
    float* slab = p.kpart + ((size_t)(tile * nchunks + mc) * p.ksplit) * slab_f;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slab, 0, p.ksplit * slab_f * 4, GP_RSRC3);
    const int mine = blockIdx.y * slab_f * 4;
    for (int q = tid; q < mrows * (NBR / 4); q += NTH) {
      const int ml = q / (NBR / 4), j = (q % (NBR / 4)) * 4;
      const f32x4_t v = {ct[ml][j], ct[ml][j + 1], ct[ml][j + 2], ct[ml][j + 3]};
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, q * 16, mine, GP_SC1);
    }
    if (norm && tid < mrows) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ssb[tid]), rs, (NB * NBR + tid) * 4, mine, GP_SC1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      gu32* tk = (gu32*)p.kticket + tile * nchunks + mc;
      const unsigned old = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = (old == (unsigned)p.ksplit - 1);
      if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
    }
    __syncthreads();
    GSTAMP(3);
    if (!last) return;
    switch (p.ksplit) {
      case 2: gp_combine<2, NB, NBR, NTH>(rs, ct, ssb, mrows, norm, slab_f, tid); break;
      case 4: gp_combine<4, NB, NBR, NTH>(rs, ct, ssb, mrows, norm, slab_f, tid); break;
      case 8: gp_combine<8, NB, NBR, NTH>(rs, ct, ssb, mrows, norm, slab_f, tid); break;
      default: gp_combine<16, NB, NBR, NTH>(rs, ct, ssb, mrows, norm, slab_f, tid); break;
    }
    __syncthreads();
  }
  for (int e = tid; e < mrows * (NBR / 2); e += NTH) {
    const int ml = e / (NBR / 2), rp = (e % (NBR / 2)) * 2;
    const int n = n0 + rp;
    float va = ct[ml][rp], vb = ct[ml][rp + 1];
    if (norm) {
      const float sc = rsqrtf(ssb[ml] / (float)p.K + p.eps);
      va *= sc;
      vb *= sc;
    }
    if (n < p.N) gemv_epilogue_pair(p, m0 + ml, n, va, vb);
    if (p.epi == EPI_ARGMAX) {
      ct[ml][rp] = va;
      ct[ml][rp + 1] = vb;
    }
  }
  if (p.epi == EPI_ARGMAX) {
    __syncthreads();
    if (tid < mrows) {
      unsigned long long best = 0;
      for (int j = 0; j < NBR; ++j) {
        const int n = n0 + j;
        if (n < p.n_valid) {
          const unsigned long long key = pack_argmax(ct[tid][j], n);
          best = key > best ? key : best;
        }
      }
      p.part[(size_t)(m0 + tid) * p.part_stride + tile] = best;
    }
  }
  GSTAMP(4);
}

// ---------------------------------------------------------------------------- host side
// Shape of one launch: rows per block (NBR) and K slices, from csm_1b microbenchmarks
// (tools/gemm_bench.py, profiles/r02_gemm_shapes.txt).  256-row blocks pay off only for the int4
// backbone gate/up (the activation split shared by 8 row tiles outweighs the longer split-K combine);
// 128 for the other wide int4 projections and the bf16 gate/up at 64 batch rows; 64 elsewhere.  K
// slices are doubled until the grid has >= 256 blocks (every CU streaming) while each slice keeps
// whole stages.  CSM_GEMM_NBR / CSM_GEMM_BLOCKS override (lab sweeps).
static int g_nbr_env = [] { const char* e = getenv("CSM_GEMM_NBR"); return e ? atoi(e) : 0; }();
static int g_blocks_env = [] { const char* e = getenv("CSM_GEMM_BLOCKS"); return e ? atoi(e) : 0; }();
// int4 prompt prefill (>= 256 rows, the 8-wave blocks): 256 weight rows per block for every shape (the
// block's activation staging -- norm, three-part split, group sums -- is shared by twice the columns):
// config 5's prefill 0.155 -> 0.140 s (profiles/r04_ab_prefill_nbr.txt).  CSM_GEMM_PREFILL_NBR=0: the
// per-shape widths below.
static int g_prefill_nbr = [] { const char* e = getenv("CSM_GEMM_PREFILL_NBR"); return e ? atoi(e) : 256; }();
static int gemm_nbr(int N, int K, int M, bool q4) {
  if (g_nbr_env == 64 || g_nbr_env == 128 || g_nbr_env == 256) return g_nbr_env;
  if (q4 && M >= 256 && (g_prefill_nbr == 128 || g_prefill_nbr == 256)) return g_prefill_nbr;
  if (q4) {
    if (N >= 8192 && K >= 2048) return 256;
    if (N >= 8192 || (N >= 2048 && (N >= 3072 || K >= 8192))) return 128;
    return 64;
  }
  return (N >= 8192 && M > 32) ? 128 : 64;
}
static int g_prefill_blocks = [] { const char* e = getenv("CSM_GEMM_PREFILL_BLOCKS"); return !e || atoi(e) != 0; }();
static int gemm_ksplit(int N, int K, int M, bool q4) {
  const int nbr = gemm_nbr(N, K, M, q4);
  const int tiles = (N + nbr - 1) / nbr, chunks = (M + 63) / 64;
  // half the slices (fewer partials to combine) where it measured faster (tools/gemm_bench.py): the
  // depth decoder's QKV / o_proj (bf16 at 32 rows 11.1 -> 10.0 and 9.4 -> 8.4 us; int4 at 64 rows
  // 16.2 -> 15.4 and 12.7 -> 12.2) and the int4 backbone QKV (30.5 -> 25.2 us); every other
  // csm_1b shape is slower so
  const bool half = (size_t)N * K <= (size_t)1536 * 1024 || (q4 && N == 3072 && K == 2048);
  // the int4 prompt prefill (>= 256 rows on 256-row blocks): 128 too (its o / down at 248 blocks then run
  // unsplit; profiles/r04_ab_prefill_blocks.txt)
  const bool prefill = q4 && M >= 256 && g_prefill_blocks;
  const int target = g_blocks_env > 0 ? g_blocks_env : ((half || prefill) ? 128 : 256);
  int ks = 1;
  while (tiles * chunks * ks < target && ks < GK_MAX_SLICES && K % (GP_KC * ks * 2) == 0) ks *= 2;
  return ks;
}

bool gemm_mfma_eligible(int N, int K, int M, int wdt) {
  return M >= GEMM_MFMA_MIN_M && N % 2 == 0 && (wdt == WDT_BF16 || wdt == WDT_Q4) && K % GP_KC == 0;
}

int gemm_tiles(int N, int K, int M, int wdt) { const int nbr = gemm_nbr(N, K, M, wdt == WDT_Q4); return (N + nbr - 1) / nbr; }

// split-K slab bytes and ticket count of one (N, K, M) launch
static size_t gemm_need(int N, int K, int M, bool q4, size_t& tk) {
  const int ks = gemm_ksplit(N, K, M, q4);
  const int MT = M > 32 ? 2 : 1, nbr = gemm_nbr(N, K, M, q4);
  const size_t tiles = (N + nbr - 1) / nbr, chunks = (M + MT * 32 - 1) / (MT * 32);
  tk = tiles * chunks;
  return ks > 1 ? tiles * chunks * ks * (size_t)MT * 32 * (nbr + 1) * 4 : 0;
}

static constexpr int gemm_pd_cap(bool q4, int mt, int nbr) { return nbr == 256 ? ((q4 && mt == 2) ? 2 : 4) : ((mt == 2 || q4) ? 4 : 8); }

// 8-wave blocks (two waves per SIMD: one wave's activation staging and int4 fold beside the other's
// MFMAs) for long prompts (>= GEMM_W8_MIN_M rows: the prompt prefill), where the 4-wave block holds
// 256 VGPRs + AGPRs at one wave per SIMD.  CSM_GEMM_W8=0: always 4 (A/B).
constexpr int GEMM_W8_MIN_M = 256;
static bool gemm_w8(int M) {
  static const bool on = [] { const char* e = getenv("CSM_GEMM_W8"); return !e || atoi(e) != 0; }();
  return on && M >= GEMM_W8_MIN_M;
}

void launch_gemm_mfma(const GemvParams& p0, int wdt, bool nt, hipStream_t st) {
  GemvParams p = p0;
  const bool q4 = wdt == WDT_Q4;
  p.Wt = nullptr;
  if (p.ws) {
    const auto ti = p.ws->tiled.find(p.W);
    if (ti != p.ws->tiled.end()) p.Wt = ti->second;
  }
  if (!p.Wt) {  // built by the engine (launch_gemm_retile) outside graph capture
    fprintf(stderr, "csm: no fragment-tiled copy of an N=%d K=%d weight for the MFMA path\n", p.N, p.K);
    abort();
  }
  const int ks = gemm_ksplit(p.N, p.K, p.M, q4);
  p.ksplit = ks;
  if (ks > 1) {
    size_t tk = 0;
    const size_t need = gemm_need(p.N, p.K, p.M, q4, tk);
    if (!p.ws || need > p.ws->bytes || tk > p.ws->n) {  // reserved by gemm_reserve outside graph capture
      fprintf(stderr, "csm: split-K scratch not reserved for N=%d K=%d M=%d\n", p.N, p.K, p.M);
      abort();
    }
    p.kpart = p.ws->kpart;
    p.kticket = p.ws->tickets;
  }
  // batch chunks of 64 (MT 2) or one chunk of 32 (MT 1) on grid.z
  const int MT = p.M > 32 ? 2 : 1, nbr = gemm_nbr(p.N, p.K, p.M, q4);
  const dim3 g3((p.N + nbr - 1) / nbr, ks, (p.M + MT * 32 - 1) / (MT * 32));
  const int nst = p.K / ks / GP_KC;
  // ring depth (stages of weights in flight per wave): 4 on 256-row blocks (32 KB a stage per
  // block), 8 on the smaller ones at 32 batch rows, 4 at 64; 2 where 4 would spill (int4 at 64
  // batch rows x 256 weight rows)
  const int pd_cap = gemm_pd_cap(wdt == WDT_Q4, MT, nbr);
  int pd = 1;  // the deepest ring within the cap that divides the stage count
  while (pd * 2 <= pd_cap && nst % (pd * 2) == 0) pd *= 2;
  const bool w8 = MT == 2 && gemm_w8(p.M);
#define GW_W(Q_, MT_, NBR_, PD_, NT_) do { if (w8 && MT_ == 2) hipLaunchKernelGGL((gemm_wide_kernel<Q_, MT_, NBR_, (PD_ > 2 ? 2 : PD_), NT_, 8>), g3, dim3(512), 0, st, p); \
                                           else hipLaunchKernelGGL((gemm_wide_kernel<Q_, MT_, NBR_, PD_, NT_>), g3, dim3(256), 0, st, p); } while (0)
#define GW_K(Q_, MT_, NBR_, PD_) do { if (nt) GW_W(Q_, MT_, NBR_, PD_, true); else GW_W(Q_, MT_, NBR_, PD_, false); } while (0)
#define GW_C(Q_, MT_, NBR_, PD_) (PD_ < gemm_pd_cap(Q_, MT_, NBR_) ? PD_ : gemm_pd_cap(Q_, MT_, NBR_))
#define GW_P(Q_, MT_, NBR_) do { if (pd == 8) GW_K(Q_, MT_, NBR_, GW_C(Q_, MT_, NBR_, 8)); else if (pd == 4) GW_K(Q_, MT_, NBR_, GW_C(Q_, MT_, NBR_, 4)); \
                                 else if (pd == 2) GW_K(Q_, MT_, NBR_, 2); else GW_K(Q_, MT_, NBR_, 1); } while (0)
#define GW_N(Q_, MT_) do { if (nbr == 256) GW_P(Q_, MT_, 256); else if (nbr == 128) GW_P(Q_, MT_, 128); else GW_P(Q_, MT_, 64); } while (0)
  if (wdt == WDT_Q4) { if (MT == 2) GW_N(true, 2); else GW_N(true, 1); }
  else { if (MT == 2) GW_N(false, 2); else GW_N(false, 1); }
#undef GW_N
#undef GW_C
#undef GW_P
#undef GW_K
#undef GW_W
}

// ---------------------------------------------------------------------------- tiled weight copies
size_t gemm_tiled_bytes(int N, int K, int wdt) {
  const size_t rows = (size_t)(N + 31) / 32 * 32;
  return wdt == WDT_Q4 ? rows * K / 2 + rows * (K / Q4_GROUP) * 4 : rows * K * 2;
}

// block = one (row tile, stage): 64 lanes; lane (r, h) copies row 32T + r, k 64 kst + 32h + 8s + 0..7
// (bf16, step s) or the 32 nibbles at k 64 kst + 32h (int4) -- the B-fragment permutation of
// gemm_wide_kernel -- and lanes < 32 the int4 scale|bias word of row 32T + lane
template <bool Q4>
__global__ __launch_bounds__(64) void gemm_retile_kernel(const uint8_t* W, uint8_t* T, int N, int K) {
  const int nks = K / GP_KC, nt32 = (N + 31) / 32;
  const int tile = blockIdx.x / nks, kst = blockIdx.x % nks, lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  const int row = 32 * tile + r;
  const bool live = row < N;
  if constexpr (Q4) {
    const u32x4_t v = live ? *reinterpret_cast<const u32x4_t*>(W + (size_t)row * (K / 2) + (64 * kst + 32 * h) / 2) : u32x4_t{};
    *reinterpret_cast<u32x4_t*>(T + ((size_t)blockIdx.x * 64 + lane) * 16) = v;
    if (lane < 32) {
      const uint32_t* SB = reinterpret_cast<const uint32_t*>(W + q4_sb_offset(N, K));
      reinterpret_cast<uint32_t*>(T + (size_t)nt32 * 32 * K / 2)[(size_t)blockIdx.x * 32 + lane] =
          live ? SB[(size_t)row * nks + kst] : 0u;
    }
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const u32x4_t v = live ? *reinterpret_cast<const u32x4_t*>(W + ((size_t)row * K + 64 * kst + 32 * h + 8 * s) * 2) : u32x4_t{};
      *reinterpret_cast<u32x4_t*>(T + (((size_t)blockIdx.x * 4 + s) * 64 + lane) * 16) = v;
    }
  }
}

void launch_gemm_retile(const void* W, void* T, int N, int K, int wdt, hipStream_t st) {
  const int blocks = (N + 31) / 32 * (K / GP_KC);
  if (wdt == WDT_Q4) hipLaunchKernelGGL(gemm_retile_kernel<true>, dim3(blocks), dim3(64), 0, st, (const uint8_t*)W, (uint8_t*)T, N, K);
  else hipLaunchKernelGGL(gemm_retile_kernel<false>, dim3(blocks), dim3(64), 0, st, (const uint8_t*)W, (uint8_t*)T, N, K);
}

// Pre-size the engine's split-K slab and tickets for an (N, K) launched at any M <= Mmax (outside
// capture).  Returns true when the buffers were reallocated (graphs holding the old ones are stale).
bool gemm_reserve(GemmWs& ws, int N, int K, int Mmax) {
  size_t slab = 0, tk = 0;
  for (int m = GEMM_MFMA_MIN_M; m <= Mmax; ++m) {  // cheap host loop (Mmax <= a few thousand)
    for (int q = 0; q < 2; ++q) {  // either weight format (an int4 engine keeps bf16 heads)
      size_t t = 0;
      slab = std::max(slab, gemm_need(N, K, m, q == 1, t));
      tk = std::max(tk, t);
    }
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
        hipDeviceSynchronize() == hipSuccess)  // (null-stream fill, drained before engine-stream use)
      ws.n = tk;
    moved = true;
  }
  return moved;
}

void gemm_ws_free(GemmWs& ws) {
  if (ws.kpart) (void)hipFree(ws.kpart);
  if (ws.tickets) (void)hipFree(ws.tickets);
  ws = GemmWs{};  // (the tiled copies are engine allocations)
}

// ---------------------------------------------------------------------------- row gather
// Batched decode: materialise the decoder-input rows a gathering GEMV would read (the next code's
// table row, resolved from the head's arg-max partials or the sampler's code) as dense fp32 rows,
// so the following projection runs on the matrix cores.  Block m: row m of the output; with
// x_step1, rows alternate [x row b (h_last), table row of c0] (generation.py:57-64).
template <typename WT>
__global__ __launch_bounds__(256) void gather_rows_kernel(GemvParams p) {
  __shared__ int code;
  const int m = blockIdx.x;
  const int bb = p.x_step1 ? (m >> 1) : m;
  const bool dense = p.x_step1 && !(m & 1);
  if (!dense && threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned long long best = wave_argmax_partials(p.xpart + (size_t)bb * p.xpart_stride, p.xpart_n, lane);
    if (lane == 0) {
      const int c = min(max(unpack_argmax(best), 0), p.xV - 1);
      code = c;
      p.x_codes[(size_t)bb * p.x_codes_K + p.xcb] = c;
    }
  }
  __syncthreads();
  float* out = p.out + (size_t)m * p.os;
  const size_t trow = dense ? 0 : (size_t)code + (size_t)p.xV * p.xcb;
  for (int k = threadIdx.x * 8; k < p.K; k += 256 * 8) {
    float v[8];
    if (dense) W8<float>::load(p.x + (size_t)bb * p.xs + k, v);
    else if (p.xtab_f32) W8<float>::load((const float*)p.xtab + trow * p.K + k, v);
    else if (p.xtab_q4_rows) q4_load8((const uint8_t*)p.xtab, (size_t)p.xtab_q4_rows, p.K, trow, k, v);
    else W8<WT>::load((const WT*)p.xtab + trow * p.K + k, v);
    *reinterpret_cast<float4*>(out + k) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(out + k + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

void launch_gather_rows(const GemvParams& p, int wdt, hipStream_t st) {
  if (wdt == WDT_F32) hipLaunchKernelGGL(gather_rows_kernel<float>, dim3(p.M), dim3(256), 0, st, p);
  else hipLaunchKernelGGL(gather_rows_kernel<bf16_t>, dim3(p.M), dim3(256), 0, st, p);
}
