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

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) const f32x4_t gcf32x4;

constexpr int GP_ROWS = 64, GP_KC = 64;  // weight rows per block, K per stage (= Q4_GROUP)
constexpr int GK_MAX_SLICES = 16;
static_assert(GP_KC == Q4_GROUP, "one int4 group per stage");

__device__ __forceinline__ unsigned short bf16_bits_rne(float v) { return (unsigned short)st_cast<bf16_t>(v); }

// x -> three bf16 parts holding all 24 significant bits (finite inputs; parts may be zero)
__device__ __forceinline__ void split3_4(const float (&v)[4], u32x2_t& hi, u32x2_t& mid, u32x2_t& lo) {
  unsigned short h[4], m[4], l[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    h[q] = bf16_bits_rne(v[q]);
    const float r1 = v[q] - __uint_as_float((unsigned)h[q] << 16);  // exact
    m[q] = bf16_bits_rne(r1);
    const float r2 = r1 - __uint_as_float((unsigned)m[q] << 16);    // exact, <= 8 significant bits
    l[q] = bf16_bits_rne(r2);
  }
  hi = u32x2_t{h[0] | ((unsigned)h[1] << 16), h[2] | ((unsigned)h[3] << 16)};
  mid = u32x2_t{m[0] | ((unsigned)m[1] << 16), m[2] | ((unsigned)m[3] << 16)};
  lo = u32x2_t{l[0] | ((unsigned)l[1] << 16), l[2] | ((unsigned)l[3] << 16)};
}

// bf16 bits of the small integer n in [0, 15] (exact)
__device__ __forceinline__ unsigned q_bits(unsigned n) { return __float_as_uint((float)n) >> 16; }

// Split-K combine (the last slice of a tile to arrive): every slice's partial is read with 16-B sc1
// buffer loads, KS * U of them in flight per thread before the first add (one round trip per 4096
// floats at U * KS = 16), and summed in slice order (deterministic).
constexpr int GP_RSRC3 = 0x00020000;  // buffer descriptor word 3 (raw 32-bit format)
constexpr int GP_SC1 = 16;            // cache policy: sc1 (agent-coherent, as __hip_atomic_load/store)
template <int KS, int NB>
__device__ __forceinline__ void gp_combine(__amdgpu_buffer_rsrc_t rs, float (*ct)[GP_ROWS + 1], float* ssb,
                                           int mrows, bool norm, int slab_f, int tid) {
  constexpr int U = KS >= 16 ? 1 : 16 / KS;
  const int nq = mrows * (GP_ROWS / 4);
  for (int q0 = tid; q0 < nq; q0 += 256 * U) {
    f32x4_t v[U][KS];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = min(q0 + 256 * u, nq - 1);
#pragma unroll
      for (int s = 0; s < KS; ++s) v[u][s] = __builtin_amdgcn_raw_buffer_load_b128(rs, q * 16, s * slab_f * 4, GP_SC1);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = q0 + 256 * u;
      if (q < nq) {
        f32x4_t sum = v[u][0];
#pragma unroll
        for (int s = 1; s < KS; ++s) sum += v[u][s];
        const int ml = q / (GP_ROWS / 4), j = (q % (GP_ROWS / 4)) * 4;
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
      v[s] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (NB * GP_ROWS + tid) * 4, s * slab_f * 4, GP_SC1));
    float sum = v[0];
#pragma unroll
    for (int s = 1; s < KS; ++s) sum += v[s];
    ssb[tid] = sum;
  }
}

template <bool Q4, int MT, bool NT, int PD>
__global__ __launch_bounds__(256) void gemm_pipe_kernel(GemvParams p) {
  constexpr int NB = MT * 32;
  constexpr int A_BYTES = 2 * 2 * 4 * 64 * 16;        // [buf][row tile][step][lane] x 16 B
  constexpr int B_BYTES = 2 * 3 * MT * 4 * 64 * 16;   // [buf][hi/mid/lo][batch tile][step][lane] x 16 B
  __shared__ __attribute__((aligned(16))) unsigned char smem[A_BYTES + B_BYTES];
  __shared__ __attribute__((aligned(16))) uint32_t sbs[2][GP_ROWS];  // int4: {scale, bias} of the stage's group
  __shared__ float xsum[2][NB];                                      // int4: sum of the stage's x per batch row
  __shared__ float ssb[NB];
  __shared__ int last;
  auto As = [&](int buf, int t, int s) { return reinterpret_cast<u32x4_t*>(smem) + ((buf * 2 + t) * 4 + s) * 64; };
  auto Bs = [&](int buf, int part, int t, int s) {
    return reinterpret_cast<u32x4_t*>(smem + A_BYTES) + (((buf * 3 + part) * MT + t) * 4 + s) * 64;
  };
  static_assert(NB * (GP_ROWS + 1) * 4 <= A_BYTES + B_BYTES, "C tile aliases the operand tiles");
  float (*ct)[GP_ROWS + 1] = reinterpret_cast<float (*)[GP_ROWS + 1]>(smem);  // after the K loop
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int wr = wave & 1, wc = wave >> 1;  // MT = 2: batch tile; MT = 1: K-step half
  const int tile = blockIdx.x, n0 = tile * GP_ROWS;
  const int mc = blockIdx.z, m0 = mc * NB, nchunks = gridDim.z;
  const int Kblk = p.K / p.ksplit, kslice = blockIdx.y * Kblk, nst = Kblk / GP_KC;
  const bool norm = p.nw != nullptr;
  // staging maps
  const int a_row = Q4 ? (tid >> 1) : (tid >> 2), a_seg = Q4 ? (tid & 1) : (tid & 3);
  const bool a_on = !Q4 || tid < 128;
  const size_t a_grow = (size_t)min(n0 + a_row, p.N - 1);
  const uint8_t* Wq = (const uint8_t*)p.W;
  const uint32_t* SB = Q4 ? reinterpret_cast<const uint32_t*>(Wq + q4_sb_offset(p.N, p.K)) : nullptr;
  const int x_c = tid >> 4, x_k4 = (tid & 15) * 4;
  float ss[NB / 16];
#pragma unroll
  for (int i = 0; i < NB / 16; ++i) ss[i] = 0.f;
  // register ring: PD stages in flight while one is multiplied (nst % PD == 0, host-checked)
  struct Stage {
    u32x4_t ar[2];
    uint32_t asb;
    f32x4_t xr[NB / 16];
    f32x4_t nwr;
  };
  Stage sg[PD];
  // stage st >= nst is a placeholder: loads from the (L2-hot) activation row, nothing used
  const float* nwp = norm ? p.nw : p.x;
  auto load = [&](int st, Stage& g) {
    const bool junk = st >= nst;
    const int kc = kslice + min(st, nst - 1) * GP_KC;
    if (a_on) {
      if constexpr (Q4) {
        const u32x4_t* src = junk ? reinterpret_cast<const u32x4_t*>(p.x)
                                  : reinterpret_cast<const u32x4_t*>(Wq + a_grow * (p.K / 2) + (kc + 32 * a_seg) / 2);
        g.ar[0] = NT ? __builtin_nontemporal_load(src) : *src;
        const uint32_t* sbp = junk ? reinterpret_cast<const uint32_t*>(p.x) : SB + a_grow * (p.K / Q4_GROUP) + kc / Q4_GROUP;
        g.asb = *sbp;
      } else {
        const u32x4_t* src = junk ? reinterpret_cast<const u32x4_t*>(p.x)
                                  : reinterpret_cast<const u32x4_t*>((const bf16_t*)p.W + a_grow * p.K + kc + 16 * a_seg);
        g.ar[0] = NT ? __builtin_nontemporal_load(src) : src[0];
        g.ar[1] = NT ? __builtin_nontemporal_load(src + 1) : src[1];
      }
    }
#pragma unroll
    for (int i = 0; i < NB / 16; ++i) {
      const int m = min(m0 + x_c + 16 * i, p.M - 1);
      g.xr[i] = *(const gcf32x4*)(p.x + (size_t)m * p.xs + kc + x_k4);
    }
    g.nwr = *(const gcf32x4*)(nwp + kc + x_k4);
  };
  auto store = [&](const Stage& g, int buf, bool live) {
    if (a_on) {
      const int t = a_row >> 5, ln = a_row & 31;
      if constexpr (Q4) {
#pragma unroll
        for (int w = 0; w < 4; ++w) {  // 8 consecutive k per word: step 2*seg + w/2, half w&1
          const uint32_t u = g.ar[0][w];
          unsigned b[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) b[j] = q_bits((u >> (4 * j)) & 15u);
          const int s = 2 * a_seg + (w >> 1), hh = w & 1;
          As(buf, t, s)[ln + 32 * hh] = u32x4_t{b[0] | (b[1] << 16), b[2] | (b[3] << 16), b[4] | (b[5] << 16), b[6] | (b[7] << 16)};
        }
        if (a_seg == 0) sbs[buf][a_row] = g.asb;
      } else {
        As(buf, t, a_seg)[ln] = g.ar[0];
        As(buf, t, a_seg)[ln + 32] = g.ar[1];
      }
    }
    const int s = x_k4 >> 4, hh = (x_k4 >> 3) & 1, j0 = x_k4 & 7;
#pragma unroll
    for (int i = 0; i < NB / 16; ++i) {
      const int c = x_c + 16 * i;
      float v[4] = {g.xr[i].x, g.xr[i].y, g.xr[i].z, g.xr[i].w};
      if (norm) {
        const float nw4[4] = {g.nwr.x, g.nwr.y, g.nwr.z, g.nwr.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ss[i] = live ? fmaf(v[q], v[q], ss[i]) : ss[i];
          v[q] *= nw4[q];
        }
      }
      if constexpr (Q4) {  // sum of the group's 64 values of row c: 16 threads x 4, fixed order
        float sum = (v[0] + v[1]) + (v[2] + v[3]);
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) sum += __shfl_xor(sum, o, 64);
        if ((tid & 15) == 0) xsum[buf][c] = sum;
      }
      u32x2_t hi, mid, lo;
      split3_4(v, hi, mid, lo);
      const int ln = (c & 31) + 32 * hh;
      *(reinterpret_cast<u32x2_t*>(&Bs(buf, 0, c >> 5, s)[ln]) + (j0 >> 2)) = hi;
      *(reinterpret_cast<u32x2_t*>(&Bs(buf, 1, c >> 5, s)[ln]) + (j0 >> 2)) = mid;
      *(reinterpret_cast<u32x2_t*>(&Bs(buf, 2, c >> 5, s)[ln]) + (j0 >> 2)) = lo;
    }
  };
  f32x16_t acc = f32x16_t{};
#pragma unroll
  for (int d = 0; d < PD; ++d) load(d, sg[d]);
  store(sg[0], 0, true);
  __syncthreads();
  const int s0 = MT == 2 ? 0 : 2 * wc, s1 = MT == 2 ? 4 : 2 * wc + 2;
  const int bt = MT == 2 ? wc : 0;
  for (int it0 = 0; it0 < nst; it0 += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      const int it = it0 + d, buf = it & 1;
      load(it + PD, sg[d]);  // slot d's stage (it) is already in LDS
      f32x16_t g = f32x16_t{};
#pragma unroll
      for (int s = s0; s < s1; ++s) {
        const bf16x8_t a = __builtin_bit_cast(bf16x8_t, As(buf, wr, s)[lane]);
#pragma unroll
        for (int part = 0; part < 3; ++part) {
          const bf16x8_t b = __builtin_bit_cast(bf16x8_t, Bs(buf, part, bt, s)[lane]);
          if constexpr (Q4) g = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, g, 0, 0, 0);
          else acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        }
      }
      if constexpr (Q4) {  // acc += scale * S_g + bias * X_g for this lane's 16 weight rows
        const float xs = (MT == 2 || wc == 0) ? xsum[buf][32 * bt + r] : 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const u32x4_t sb = *reinterpret_cast<const u32x4_t*>(&sbs[buf][32 * wr + 8 * q + 4 * h]);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int j = 4 * q + e;
            acc[j] = fmaf(bf16_lo(sb[e]), g[j], acc[j]);
            acc[j] = fmaf(bf16_hi(sb[e]), xs, acc[j]);
          }
        }
      }
      store(sg[(d + 1) % PD], buf ^ 1, it + 1 < nst);  // the last one stores a placeholder
      __syncthreads();
    }
  }
  // sum of squares per batch row: the 16 threads of a row share it
  if (norm) {
#pragma unroll
    for (int i = 0; i < NB / 16; ++i) {
      float v = ss[i];
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if ((tid & 15) == 0) ssb[x_c + 16 * i] = v;
    }
  }
  // accumulators -> C tile [batch row][weight row]
  if (MT == 2 || wc == 0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) ct[32 * (MT == 2 ? wc : 0) + r][32 * wr + (j & 3) + 8 * (j >> 2) + 4 * h] = acc[j];
  }
  __syncthreads();
  if (MT == 1 && wc == 1) {  // second K-step half, added in a fixed order
#pragma unroll
    for (int j = 0; j < 16; ++j) ct[r][32 * wr + (j & 3) + 8 * (j >> 2) + 4 * h] += acc[j];
  }
  __syncthreads();
  const int mrows = min(NB, p.M - m0);
  if (p.ksplit > 1) {
    // slice partial = [NB][64] tile values, then [NB] sums of squares; 16-B write-through stores
    const int slab_f = NB * (GP_ROWS + 1);
    float* slab = p.kpart + ((size_t)(tile * nchunks + mc) * p.ksplit) * slab_f;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slab, 0, p.ksplit * slab_f * 4, GP_RSRC3);
    const int mine = blockIdx.y * slab_f * 4;
    for (int q = tid; q < mrows * (GP_ROWS / 4); q += 256) {
      const int ml = q / (GP_ROWS / 4), j = (q % (GP_ROWS / 4)) * 4;
      const f32x4_t v = {ct[ml][j], ct[ml][j + 1], ct[ml][j + 2], ct[ml][j + 3]};
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, q * 16, mine, GP_SC1);
    }
    if (norm && tid < mrows) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ssb[tid]), rs, (NB * GP_ROWS + tid) * 4, mine, GP_SC1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      gu32* tk = (gu32*)p.kticket + tile * nchunks + mc;
      const unsigned old = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = (old == (unsigned)p.ksplit - 1);
      if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
    }
    __syncthreads();
    if (!last) return;
    switch (p.ksplit) {
      case 2: gp_combine<2, NB>(rs, ct, ssb, mrows, norm, slab_f, tid); break;
      case 4: gp_combine<4, NB>(rs, ct, ssb, mrows, norm, slab_f, tid); break;
      case 8: gp_combine<8, NB>(rs, ct, ssb, mrows, norm, slab_f, tid); break;
      default: gp_combine<16, NB>(rs, ct, ssb, mrows, norm, slab_f, tid); break;
    }
    __syncthreads();
  }
  for (int e = tid; e < mrows * (GP_ROWS / 2); e += 256) {
    const int ml = e / (GP_ROWS / 2), rp = (e % (GP_ROWS / 2)) * 2;
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
      for (int j = 0; j < GP_ROWS; ++j) {
        const int n = n0 + j;
        if (n < p.n_valid) {
          const unsigned long long key = pack_argmax(ct[tid][j], n);
          best = key > best ? key : best;
        }
      }
      p.part[(size_t)(m0 + tid) * p.part_stride + blockIdx.x] = best;
    }
  }
}

// ---------------------------------------------------------------------------- host side
// K slices are added until the grid has this many blocks (measured best: 256 for <= 32 batch rows,
// 512 above -- configs 4 / 5); CSM_PIPE_BLOCKS overrides (lab sweeps)
static int g_pipe_target_env = [] { const char* e = getenv("CSM_PIPE_BLOCKS"); return e ? atoi(e) : 0; }();
static int pipe_target(int M) { return g_pipe_target_env > 0 ? g_pipe_target_env : (M > 32 ? 512 : 256); }
// deepest register prefetch ring (stages in flight, 1 / 2 / 4: 4 for <= 32 batch rows, 2 above, where
// the 64-row stages cost twice the registers); CSM_PIPE_PD overrides
static int g_pipe_pd_env = [] { const char* e = getenv("CSM_PIPE_PD"); return e ? atoi(e) : 0; }();
static int pipe_pd_cap(int M) { return g_pipe_pd_env > 0 ? g_pipe_pd_env : (M > 32 ? 2 : 4); }

// K slices: doubled while the grid has fewer than pipe_target(M) blocks and every slice keeps >= 2
// stages; arg-max heads are split too (the last slice runs the arg-max epilogue).
static int gemm_ksplit(int N, int K, int M) {
  const int tiles = (N + GP_ROWS - 1) / GP_ROWS, chunks = (M + 63) / 64;
  int ks = 1;
  while (tiles * chunks * ks < pipe_target(M) && ks < GK_MAX_SLICES && K % (GP_KC * ks * 2) == 0 &&
         K / (ks * 2) >= 2 * GP_KC)
    ks *= 2;
  return ks;
}

bool gemm_mfma_eligible(int N, int K, int M, int wdt) {
  return M >= GEMM_MFMA_MIN_M && N % 2 == 0 && (wdt == WDT_BF16 || wdt == WDT_Q4) && K % GP_KC == 0;
}

int gemm_blocks(int N) { return (N + GP_ROWS - 1) / GP_ROWS; }

// split-K slab bytes and ticket count of one (N, K, M) launch
static size_t gemm_need(int N, int K, int M, size_t& tk) {
  const int ks = gemm_ksplit(N, K, M);
  const int MT = M > 32 ? 2 : 1;
  const size_t tiles = gemm_blocks(N), chunks = (M + MT * 32 - 1) / (MT * 32);
  tk = tiles * chunks;
  return ks > 1 ? tiles * chunks * ks * (size_t)MT * 32 * (GP_ROWS + 1) * 4 : 0;
}

void launch_gemm_mfma(const GemvParams& p0, int wdt, bool nt, hipStream_t st) {
  GemvParams p = p0;
  const int ks = gemm_ksplit(p.N, p.K, p.M);
  p.ksplit = ks;
  if (ks > 1) {
    size_t tk = 0;
    const size_t need = gemm_need(p.N, p.K, p.M, tk);
    if (!p.ws || need > p.ws->bytes || tk > p.ws->n) {  // reserved by gemm_reserve outside graph capture
      fprintf(stderr, "csm: split-K scratch not reserved for N=%d K=%d M=%d\n", p.N, p.K, p.M);
      abort();
    }
    p.kpart = p.ws->kpart;
    p.kticket = p.ws->tickets;
  }
  // batch chunks of 64 (MT 2) or one chunk of 32 (MT 1) on grid.z
  const int MT = p.M > 32 ? 2 : 1;
  const dim3 g3(gemm_blocks(p.N), ks, (p.M + MT * 32 - 1) / (MT * 32));
  const int nst = p.K / ks / GP_KC;
  const int cap = pipe_pd_cap(p.M);
  const int pd = (nst % 4 == 0 && cap >= 4) ? 4 : ((nst % 2 == 0 && cap >= 2) ? 2 : 1);
#define GP_K(Q_, MT_, PD_) do { if (nt) hipLaunchKernelGGL((gemm_pipe_kernel<Q_, MT_, true, PD_>), g3, dim3(256), 0, st, p); \
                                else hipLaunchKernelGGL((gemm_pipe_kernel<Q_, MT_, false, PD_>), g3, dim3(256), 0, st, p); } while (0)
#define GP_L(Q_, MT_) do { if (pd == 4) GP_K(Q_, MT_, 4); else if (pd == 2) GP_K(Q_, MT_, 2); else GP_K(Q_, MT_, 1); } while (0)
  if (wdt == WDT_Q4) { if (MT == 2) GP_L(true, 2); else GP_L(true, 1); }
  else { if (MT == 2) GP_L(false, 2); else GP_L(false, 1); }
#undef GP_L
#undef GP_K
}

// Pre-size the engine's split-K slab and tickets for an (N, K) launched at any M <= Mmax (outside
// capture).  Returns true when the buffers were reallocated (graphs holding the old ones are stale).
bool gemm_reserve(GemmWs& ws, int N, int K, int Mmax) {
  size_t slab = 0, tk = 0;
  for (int m = GEMM_MFMA_MIN_M; m <= Mmax; ++m) {  // cheap host loop (Mmax <= a few thousand)
    size_t t = 0;
    slab = std::max(slab, gemm_need(N, K, m, t));
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
    if (hipMalloc(&ws.tickets, tk * 4) == hipSuccess && hipMemset(ws.tickets, 0, tk * 4) == hipSuccess) ws.n = tk;
    moved = true;
  }
  return moved;
}

void gemm_ws_free(GemmWs& ws) {
  if (ws.kpart) (void)hipFree(ws.kpart);
  if (ws.tickets) (void)hipFree(ws.tickets);
  ws = GemmWs{};
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
