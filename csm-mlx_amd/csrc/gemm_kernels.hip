// Batched projections on the matrix cores (gfx950 MFMA) for B >= 8 utterances and prompt prefill.
//
// y[m, n] = sum_k norm(x)[m, k] * W[n, k]   -- every nn.Linear of the backbone / decoder and the
// codebook heads (models.py:50-67, generation.py:42, :74-79) once the row count M makes the
// GEMV's per-row loop (gemv_kernel re-streams the weights every MT rows) the bottleneck.
//
// Operands: W bf16 [N][K] as stored (MLX (out,in) layout) is the MFMA A operand (32 weight rows per
// wave); the fp32 activations are the B operand (32 batch rows per tile), each value split into two
// bf16 parts x = hi + lo (hi = bf16(x), lo = bf16(x - hi)) with both products accumulated in fp32:
// the activation keeps ~16 significant bits, so results stay within the bf16-weight parity bar of
// the fp32 GEMV (tests/test_gemm_gpu.py).  v_mfma_f32_32x32x16_bf16: lane l = (r = l & 31, h = l >> 5)
// holds A[row r][k 8h..8h+7] and B[k 8h..8h+7][col r]; C[row (j&3) + 8(j>>2) + 4h][col r].
//
// Block = 4 waves = 128 weight rows (wave w: rows 32w..32w+31) x up to 64 batch rows per pass, over
// one K slice of K / ksplit, in sub-chunks of 128 K: (1) the block's coalesced 16-B loads of the
// activation sub-chunk and every wave's weight loads for it are issued together (weights straight to
// VGPRs: each weight byte is used by one wave only), (2) the activations are RMSNorm-weighted,
// split hi/lo and written to LDS in MFMA-fragment order (one conflict-free ds_read_b128 per
// fragment, shared by the 4 waves), (3) 8 K-steps of MFMA.  ksplit == 1: pair epilogues straight
// from the accumulators (rows (j, j+1) sit in registers j, j+1 of one lane).  ksplit > 1: each slice
// publishes its accumulators write-through (sc1 stores, drained) and takes an arrival ticket; the
// last slice of a tile to arrive reads every partial back with sc1 loads (MI355X_MICROARCH.md
// hand-off table, single-counter row), sums them in slice order (deterministic) and runs the
// epilogue -- no second launch.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "csm_kernels.h"

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) float gfloat;
typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) const f32x4_t gcf32x4;

constexpr int GM_WROWS = 128;  // weight rows per block (4 waves x one 32-row MFMA tile)
constexpr int GM_KS = 128;     // K per sub-chunk (8 MFMA steps)

__device__ __forceinline__ unsigned short bf16_bits_rne(float v) { return (unsigned short)st_cast<bf16_t>(v); }

constexpr int GK_MAX_SLICES = 16;
// Split-K combine: element e of every slice partial (sc1 loads, all issued before the first add so
// the slices cost one round trip), summed in slice order.
__device__ __forceinline__ float slab_sum(const gfloat* slab, size_t slab_f, size_t e, int ks) {
  float v[GK_MAX_SLICES];
#pragma unroll
  for (int sl = 0; sl < GK_MAX_SLICES; ++sl)
    v[sl] = sl < ks ? __hip_atomic_load(slab + (size_t)sl * slab_f + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
  float sum = 0.f;
#pragma unroll
  for (int sl = 0; sl < GK_MAX_SLICES; ++sl)
    if (sl < ks) sum += v[sl];
  return sum;
}

template <int MT, bool NT>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(GemvParams p) {
  // activation fragments of one sub-chunk: [hi/lo][tile][step][lane] x 8 bf16 (16 B)
  __shared__ __attribute__((aligned(16))) u32x4_t xs[2][MT][GM_KS / 16][64];
  __shared__ float ssb[MT * 32];
  __shared__ float ct[MT * 32][GM_WROWS + 1];  // C tile [batch row][weight row]
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int tile = blockIdx.x;
  const int nw0 = tile * GM_WROWS + wave * 32;  // this wave's first weight row
  const int Kblk = p.K / p.ksplit;
  const int kslice = blockIdx.y * Kblk;
  const bool norm = p.nw != nullptr;
  const bf16_t* wrow = (const bf16_t*)p.W + (size_t)min(nw0 + r, p.N - 1) * p.K;
  const int nchunks = (p.M + MT * 32 - 1) / (MT * 32);
  // staging map: thread t, load i covers batch row (t >> 5) + 8i, k offset 4 * (t & 31) of the sub-chunk
  const int sk = 4 * (tid & 31);
  const int s_step = sk >> 4, s_h = (sk >> 3) & 1, s_j = sk & 7;
  for (int mc = 0; mc < nchunks; ++mc) {
    const int m0 = mc * MT * 32;
    f32x16_t acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = f32x16_t{};
    float ss[MT * 4];
#pragma unroll
    for (int i = 0; i < MT * 4; ++i) ss[i] = 0.f;
    for (int kc = kslice; kc < kslice + Kblk; kc += GM_KS) {
      // (1) activation sub-chunk (+ norm weights) and this wave's weights, all in flight
      f32x4_t xv[MT * 4];
#pragma unroll
      for (int i = 0; i < MT * 4; ++i) {
        const int m = min(m0 + (tid >> 5) + 8 * i, p.M - 1);
        xv[i] = *(const gcf32x4*)(p.x + (size_t)m * p.xs + kc + sk);
      }
      f32x4_t nwv = {1.f, 1.f, 1.f, 1.f};
      if (norm) nwv = *(const gcf32x4*)(p.nw + kc + sk);
      u32x4_t wa[GM_KS / 16];
#pragma unroll
      for (int s = 0; s < GM_KS / 16; ++s) {
        const u32x4_t* src = reinterpret_cast<const u32x4_t*>(wrow + kc + s * 16 + 8 * h);
        if constexpr (NT) wa[s] = __builtin_nontemporal_load(src);
        else wa[s] = *src;
      }
      __syncthreads();  // previous sub-chunk's fragments consumed
      // (2) x * nw, sum(x^2), hi/lo split -> fragment-ordered LDS
#pragma unroll
      for (int i = 0; i < MT * 4; ++i) {
        const int ml = (tid >> 5) + 8 * i;  // batch row inside the chunk
        const float v4[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
        const float n4[4] = {nwv.x, nwv.y, nwv.z, nwv.w};
        unsigned short hb[4], lb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v = v4[q];
          if (norm) {
            ss[i] = fmaf(v, v, ss[i]);
            v *= n4[q];
          }
          hb[q] = bf16_bits_rne(v);
          lb[q] = bf16_bits_rne(v - __uint_as_float((unsigned)hb[q] << 16));
        }
        const int t = ml >> 5, fl = (ml & 31) + 32 * s_h;
        unsigned int* dh = reinterpret_cast<unsigned int*>(&xs[0][t][s_step][fl]) + (s_j >> 1);
        unsigned int* dl = reinterpret_cast<unsigned int*>(&xs[1][t][s_step][fl]) + (s_j >> 1);
        *reinterpret_cast<u32x2_t*>(dh) = u32x2_t{hb[0] | ((unsigned)hb[1] << 16), hb[2] | ((unsigned)hb[3] << 16)};
        *reinterpret_cast<u32x2_t*>(dl) = u32x2_t{lb[0] | ((unsigned)lb[1] << 16), lb[2] | ((unsigned)lb[3] << 16)};
      }
      __syncthreads();
      // (3) MFMA over the sub-chunk
#pragma unroll
      for (int s = 0; s < GM_KS / 16; ++s) {
        const bf16x8_t a = __builtin_bit_cast(bf16x8_t, wa[s]);
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const bf16x8_t bh = __builtin_bit_cast(bf16x8_t, xs[0][t][s][lane]);
          const bf16x8_t bl = __builtin_bit_cast(bf16x8_t, xs[1][t][s][lane]);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bh, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bl, acc[t], 0, 0, 0);
        }
      }
    }
    // sum(x^2) of the slice per batch row: the 32 threads of a half-wave share rows
    if (norm) {
#pragma unroll
      for (int i = 0; i < MT * 4; ++i) {
        float v = ss[i];
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if ((tid & 31) == 0) ssb[(tid >> 5) + 8 * i] = v;
      }
    }
    // accumulators -> C tile in LDS [batch row][weight row of the block]
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int j = 0; j < 16; ++j) ct[32 * t + r][wave * 32 + (j & 3) + 8 * (j >> 2) + 4 * h] = acc[t][j];
    __syncthreads();
    const int mrows = min(MT * 32, p.M - m0);
    if (p.ksplit > 1) {
      // publish the slice partial write-through, take a ticket; the last slice to arrive combines
      const size_t slab_f = (size_t)MT * 32 * (GM_WROWS + 1);  // [batch row][128 rows + sum(x^2)]
      gfloat* slab = (gfloat*)p.kpart + ((size_t)(tile * nchunks + mc) * p.ksplit) * slab_f;
      gfloat* mine = slab + (size_t)blockIdx.y * slab_f;
      for (int e = tid; e < mrows * (GM_WROWS + 1); e += 256) {
        const int ml = e / (GM_WROWS + 1), j = e % (GM_WROWS + 1);
        __hip_atomic_store(mine + e, j < GM_WROWS ? ct[ml][j] : (norm ? ssb[ml] : 0.f), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        gu32* tk = (gu32*)p.kticket + tile * nchunks + mc;
        const unsigned old = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = (old == (unsigned)p.ksplit - 1);
        if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
      }
      __syncthreads();
      if (!last) continue;  // uniform per block
      for (int e = tid; e < mrows * (GM_WROWS + 1); e += 256) {
        const float v = slab_sum(slab, slab_f, e, p.ksplit);
        const int ml = e / (GM_WROWS + 1), j = e % (GM_WROWS + 1);
        if (j < GM_WROWS) ct[ml][j] = v;
        else ssb[ml] = v;
      }
      __syncthreads();
    }
    // pair epilogues: thread -> (batch row, weight-row pair)
    for (int e = tid; e < mrows * (GM_WROWS / 2); e += 256) {
      const int ml = e / (GM_WROWS / 2), rp = (e % (GM_WROWS / 2)) * 2;
      const int n = tile * GM_WROWS + rp;
      float a = ct[ml][rp], b = ct[ml][rp + 1];
      if (norm) {
        const float sc = rsqrtf(ssb[ml] / (float)p.K + p.eps);
        a *= sc;
        b *= sc;
      }
      if (n < p.N) gemv_epilogue_pair(p, m0 + ml, n, a, b);
      if (p.epi == EPI_ARGMAX) {
        ct[ml][rp] = a;
        ct[ml][rp + 1] = b;
      }
    }
    if (p.epi == EPI_ARGMAX) {  // block arg-max per batch row -> partial slot
      __syncthreads();
      if (tid < mrows) {
        unsigned long long best = 0;
        for (int j = 0; j < GM_WROWS; ++j) {
          const int n = tile * GM_WROWS + j;
          if (n < p.n_valid) {
            const unsigned long long key = pack_argmax(ct[tid][j], n);
            best = key > best ? key : best;
          }
        }
        p.part[(size_t)(m0 + tid) * p.part_stride + blockIdx.x] = best;
      }
    }
    __syncthreads();
  }
}

// Variant "wk" (CSM_GEMM=wk): 32 weight rows per block, the four waves split the block's K slice
// (each activation fragment read by one wave only, straight from L2 into VGPRs), loads run PF
// MFMA steps ahead of use through a register ring (in-order vmcnt: the wait for step s leaves the
// PF-1 younger steps in flight).  Wave tiles are summed in LDS in a fixed order; split-K as above.
constexpr int GW_ROWS = 32;
template <int MT, int PF, bool NT, bool LO = true>
__global__ __launch_bounds__(256) void gemm_bf16_wk_kernel(GemvParams p) {
  __shared__ float red[4][MT * 32][GW_ROWS + 1];
  __shared__ float ssw[4][MT * 32];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int tile = blockIdx.x, n0 = tile * GW_ROWS;
  const int Kblk = p.K / p.ksplit, kw = Kblk / 4;
  const int kbeg = blockIdx.y * Kblk + wave * kw;
  const int nsteps = kw / 16;  // multiple of PF (plan)
  const bool norm = p.nw != nullptr;
  const bf16_t* wrow = (const bf16_t*)p.W + (size_t)min(n0 + r, p.N - 1) * p.K + kbeg + 8 * h;
  const float* nwp = norm ? p.nw + kbeg + 8 * h : nullptr;
  const int nchunks = (p.M + MT * 32 - 1) / (MT * 32);
  for (int mc = 0; mc < nchunks; ++mc) {
    const int m0 = mc * MT * 32;
    const float* xr[MT];
    f32x16_t acc[MT];
    float ss[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      xr[t] = p.x + (size_t)min(m0 + t * 32 + r, p.M - 1) * p.xs + kbeg + 8 * h;
      acc[t] = f32x16_t{};
      ss[t] = 0.f;
    }
    u32x4_t wq[PF];
    f32x4_t xq[PF][MT][2];
    f32x4_t nq[PF][2];
    auto issue = [&](int u, int s) {
      const int k = s * 16;
      if constexpr (NT) wq[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(wrow + k));
      else wq[u] = *reinterpret_cast<const u32x4_t*>(wrow + k);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        xq[u][t][0] = ((gcf32x4*)(xr[t] + k))[0];
        xq[u][t][1] = ((gcf32x4*)(xr[t] + k))[1];
      }
      if (norm) {
        nq[u][0] = ((gcf32x4*)(nwp + k))[0];
        nq[u][1] = ((gcf32x4*)(nwp + k))[1];
      }
    };
#pragma unroll
    for (int u = 0; u < PF; ++u) issue(u, u);
    for (int s0 = 0; s0 < nsteps; s0 += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const bf16x8_t a = __builtin_bit_cast(bf16x8_t, wq[u]);
        const float nw[8] = {nq[u][0].x, nq[u][0].y, nq[u][0].z, nq[u][0].w, nq[u][1].x, nq[u][1].y, nq[u][1].z, nq[u][1].w};
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const float xv[8] = {xq[u][t][0].x, xq[u][t][0].y, xq[u][t][0].z, xq[u][t][0].w,
                               xq[u][t][1].x, xq[u][t][1].y, xq[u][t][1].z, xq[u][t][1].w};
          bf16x8_t bh, bl;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float v = xv[j];
            if (norm) {
              ss[t] = fmaf(v, v, ss[t]);
              v *= nw[j];
            }
            const __bf16 hi = (__bf16)v;
            bh[j] = hi;
            bl[j] = (__bf16)(v - (float)hi);
          }
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bh, acc[t], 0, 0, 0);
          if constexpr (LO) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bl, acc[t], 0, 0, 0);
        }
        if (s0 + u + PF < nsteps) issue(u, s0 + u + PF);
      }
    }
#pragma unroll
    for (int t = 0; t < MT; ++t) {
#pragma unroll
      for (int j = 0; j < 16; ++j) red[wave][t * 32 + r][(j & 3) + 8 * (j >> 2) + 4 * h] = acc[t][j];
      const float sv = ss[t] + __shfl_xor(ss[t], 32, 64);
      if (h == 0) ssw[wave][t * 32 + r] = sv;
    }
    __syncthreads();
    const int mrows = min(MT * 32, p.M - m0);
    gfloat* slab = nullptr;
    const size_t slab_f = (size_t)MT * 32 * (GW_ROWS + 1);
    if (p.ksplit > 1) {
      slab = (gfloat*)p.kpart + ((size_t)(tile * nchunks + mc) * p.ksplit) * slab_f;
      gfloat* mine = slab + (size_t)blockIdx.y * slab_f;
      for (int e = tid; e < mrows * (GW_ROWS + 1); e += 256) {
        const int mi = e / (GW_ROWS + 1), j = e % (GW_ROWS + 1);
        const float v = j < GW_ROWS ? (red[0][mi][j] + red[1][mi][j]) + (red[2][mi][j] + red[3][mi][j])
                                    : (ssw[0][mi] + ssw[1][mi]) + (ssw[2][mi] + ssw[3][mi]);
        __hip_atomic_store(mine + e, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        gu32* tk = (gu32*)p.kticket + tile * nchunks + mc;
        const unsigned old = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = (old == (unsigned)p.ksplit - 1);
        if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (!last) continue;  // uniform per block
    }
    for (int e = tid; e < mrows * (GW_ROWS / 2); e += 256) {
      const int mi = e / (GW_ROWS / 2), rp = (e % (GW_ROWS / 2)) * 2;
      const int n = n0 + rp;
      float a, b, sq;
      if (slab) {
        a = 0.f; b = 0.f; sq = 0.f;
        const size_t e0 = (size_t)mi * (GW_ROWS + 1);
        a = slab_sum(slab, slab_f, e0 + rp, p.ksplit);
        b = slab_sum(slab, slab_f, e0 + rp + 1, p.ksplit);
        sq = slab_sum(slab, slab_f, e0 + GW_ROWS, p.ksplit);
      } else {
        a = (red[0][mi][rp] + red[1][mi][rp]) + (red[2][mi][rp] + red[3][mi][rp]);
        b = (red[0][mi][rp + 1] + red[1][mi][rp + 1]) + (red[2][mi][rp + 1] + red[3][mi][rp + 1]);
        sq = (ssw[0][mi] + ssw[1][mi]) + (ssw[2][mi] + ssw[3][mi]);
      }
      if (norm) {
        const float sc = rsqrtf(sq / (float)p.K + p.eps);
        a *= sc;
        b *= sc;
      }
      if (n < p.N) gemv_epilogue_pair(p, m0 + mi, n, a, b);
      if (p.epi == EPI_ARGMAX) {
        red[0][mi][rp] = a;
        red[0][mi][rp + 1] = b;
      }
    }
    if (p.epi == EPI_ARGMAX) {
      __syncthreads();
      if (tid < mrows) {
        unsigned long long best = 0;
        for (int j = 0; j < GW_ROWS; ++j) {
          const int n = n0 + j;
          if (n < p.n_valid) {
            const unsigned long long key = pack_argmax(red[0][tid][j], n);
            best = key > best ? key : best;
          }
        }
        p.part[(size_t)(m0 + tid) * p.part_stride + blockIdx.x] = best;
      }
    }
    __syncthreads();
  }
}

// Variant "pipe" (default): the block's weight tile AND activation tile go through LDS with
// coalesced global loads into a register ring of PD stages (loads of stages c+1..c+PD in flight
// while stage c runs on the matrix cores from a double-buffered LDS tile; PD = 1 / 2 / 4 by the
// stage count).  Block = 64 weight rows x 32*MT batch rows over one K slice, stages of 64 K
// (4 MFMA steps); every fragment is stored in MFMA-lane order (one conflict-free ds_read_b128 per
// operand).  MT = 2: 2 x 2 waves over (row tile, batch tile); MT = 1: 2 waves per row tile split
// each stage's K steps and are summed in a fixed order.  int4 weights (Q4) are dequantized while
// staging (w = scale * q + bias in fp32, split hi/lo like the activations) and run three products
// (hi*hi, hi*lo, lo*hi).  Split-K fixup as the kernels above, except the combine (gp_combine: 16-B
// loads, 16 in flight per thread); arg-max heads are split too (the last slice runs the arg-max).
constexpr int GP_ROWS = 64, GP_KC = 64;
typedef unsigned short u16x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split4(const float (&v)[4], u32x2_t& hi, u32x2_t& lo) {
  unsigned short h[4], l[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    h[q] = bf16_bits_rne(v[q]);
    l[q] = bf16_bits_rne(v[q] - __uint_as_float((unsigned)h[q] << 16));
  }
  hi = u32x2_t{h[0] | ((unsigned)h[1] << 16), h[2] | ((unsigned)h[3] << 16)};
  lo = u32x2_t{l[0] | ((unsigned)l[1] << 16), l[2] | ((unsigned)l[3] << 16)};
}

// Split-K combine of the pipe kernel (the last slice of a tile to arrive): every slice's partial is
// read with 16-B sc1 buffer loads, KS * U of them in flight per thread before the first add (one
// round trip per 4096 floats at U * KS = 16), and summed in slice order (deterministic, the same
// order as slab_sum).
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
  constexpr int NB = MT * 32, NA = Q4 ? 2 : 1;
  constexpr int A_BYTES = 2 * NA * 2 * 4 * 64 * 16, B_BYTES = 2 * 2 * MT * 4 * 64 * 16;
  __shared__ __attribute__((aligned(16))) unsigned char smem[A_BYTES + B_BYTES];
  __shared__ float ssb[NB];
  __shared__ int last;
  // As[buf][hi/lo][row tile][step][lane], Bs[buf][hi/lo][batch tile][step][lane] (16 B each)
  auto As = [&](int buf, int hl, int t, int s) { return reinterpret_cast<u32x4_t*>(smem) + (((buf * NA + hl) * 2 + t) * 4 + s) * 64; };
  auto Bs = [&](int buf, int hl, int t, int s) {
    return reinterpret_cast<u32x4_t*>(smem + A_BYTES) + (((buf * 2 + hl) * MT + t) * 4 + s) * 64;
  };
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
  // stage st >= nst is a placeholder: weights from the (L2-hot) activation row, nothing used
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
        const float sc = bf16_lo(g.asb), bi = bf16_hi(g.asb);
#pragma unroll
        for (int w = 0; w < 4; ++w) {  // 8 consecutive k per word: step 2*seg + w/2, half w&1
          const uint32_t u = g.ar[0][w];
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = fmaf(sc, (float)((u >> (4 * j)) & 15u), bi);
          u32x2_t h0, l0, h1, l1;
          const float v0[4] = {v[0], v[1], v[2], v[3]}, v1[4] = {v[4], v[5], v[6], v[7]};
          split4(v0, h0, l0);
          split4(v1, h1, l1);
          const int s = 2 * a_seg + (w >> 1), hh = w & 1;
          As(buf, 0, t, s)[ln + 32 * hh] = u32x4_t{h0.x, h0.y, h1.x, h1.y};
          As(buf, 1, t, s)[ln + 32 * hh] = u32x4_t{l0.x, l0.y, l1.x, l1.y};
        }
      } else {
        As(buf, 0, t, a_seg)[ln] = g.ar[0];
        As(buf, 0, t, a_seg)[ln + 32] = g.ar[1];
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
      u32x2_t hi, lo;
      split4(v, hi, lo);
      const int ln = (c & 31) + 32 * hh;
      *(reinterpret_cast<u32x2_t*>(&Bs(buf, 0, c >> 5, s)[ln]) + (j0 >> 2)) = hi;
      *(reinterpret_cast<u32x2_t*>(&Bs(buf, 1, c >> 5, s)[ln]) + (j0 >> 2)) = lo;
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
#pragma unroll
      for (int s = s0; s < s1; ++s) {
        const bf16x8_t a = __builtin_bit_cast(bf16x8_t, As(buf, 0, wr, s)[lane]);
        const bf16x8_t bh = __builtin_bit_cast(bf16x8_t, Bs(buf, 0, bt, s)[lane]);
        const bf16x8_t bl = __builtin_bit_cast(bf16x8_t, Bs(buf, 1, bt, s)[lane]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bl, acc, 0, 0, 0);
        if constexpr (Q4) {
          const bf16x8_t al = __builtin_bit_cast(bf16x8_t, As(buf, 1, wr, s)[lane]);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
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
      if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
static int gemm_variant() {  // 2 = "pipe" (default), 0 = "wk" (CSM_GEMM=wk), 1 = "lds" (CSM_GEMM=lds)
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CSM_GEMM");
    v = (e && e[0] == 'l') ? 1 : ((e && e[0] == 'w') ? 0 : 2);
  }
  return v;
}
static int gemm_rows() { return gemm_variant() == 1 ? GM_WROWS : (gemm_variant() == 2 ? GP_ROWS : GW_ROWS); }
constexpr int GW_PF = 4;  // wk: MFMA steps in flight per wave
// pipe: K slices are added until the grid has this many blocks (measured best: 256 for <= 32 batch
// rows, 512 above -- configs 4 / 5); CSM_PIPE_BLOCKS overrides (lab sweeps)
static int g_pipe_target_env = [] { const char* e = getenv("CSM_PIPE_BLOCKS"); return e ? atoi(e) : 0; }();
static int pipe_target(int M) { return g_pipe_target_env > 0 ? g_pipe_target_env : (M > 32 ? 512 : 256); }
// pipe: deepest register prefetch ring (stages in flight, 1 / 2 / 4: 4 for <= 32 batch rows, 2 above,
// where the 64-row stages cost twice the registers); CSM_PIPE_PD overrides
static int g_pipe_pd_env = [] { const char* e = getenv("CSM_PIPE_PD"); return e ? atoi(e) : 0; }();
static int pipe_pd_cap(int M) { return g_pipe_pd_env > 0 ? g_pipe_pd_env : (M > 32 ? 2 : 4); }

// K slices: doubled while the grid has < 256 blocks (wk: while each wave keeps >= 2 rings of PF
// steps; lds: up to 8); wk / lds arg-max heads keep whole rows.
static void gemm_plan(int N, int K, int M, int epi, int& ks) {
  const int rows = gemm_rows();
  const int tiles = (N + rows - 1) / rows;
  const int chunks = (M + 63) / 64;
  ks = 1;
  if (epi == EPI_ARGMAX && gemm_variant() != 2) return;  // pipe: the last slice runs the arg-max epilogue
  if (gemm_variant() == 2) {
    while (tiles * chunks * ks < pipe_target(M) && ks < 16 && K % (GP_KC * ks * 2) == 0 && K / (ks * 2) >= 2 * GP_KC) ks *= 2;
  } else if (gemm_variant() == 1) {
    while (tiles * chunks * ks < 256 && ks < 8 && K % (GM_KS * ks * 2) == 0) ks *= 2;
  } else {
    while (tiles * chunks * ks < 512 && K % (ks * 2 * 4 * 16 * GW_PF * 2) == 0) ks *= 2;
  }
}

static size_t gemm_slab_floats(int MT) { return (size_t)MT * 32 * (gemm_rows() + 1); }

bool gemm_mfma_eligible(int N, int K, int M, int wdt) {
  if (M < GEMM_MFMA_MIN_M || N % 2) return false;
  if (gemm_variant() == 2) return (wdt == WDT_BF16 || wdt == WDT_Q4) && K % GP_KC == 0;
  return wdt == WDT_BF16 && K % (4 * 16 * GW_PF) == 0 && K % GM_KS == 0;
}

int gemm_blocks(int N) { return (N + gemm_rows() - 1) / gemm_rows(); }

static float* g_kscratch = nullptr;
static size_t g_kscratch_bytes = 0;
static unsigned* g_ktickets = nullptr;
static size_t g_ktickets_n = 0;

static size_t gemm_need(int N, int K, int M, size_t& tk) {
  int ks;
  gemm_plan(N, K, M, EPI_STORE, ks);
  const int MT = (M > 32 || gemm_variant() == 2) ? 2 : 1;
  const size_t tiles = gemm_blocks(N), chunks = (M + MT * 32 - 1) / (MT * 32);
  tk = tiles * chunks;
  return ks > 1 ? tiles * chunks * ks * gemm_slab_floats(MT) * 4 : 0;
}

void launch_gemm_mfma(const GemvParams& p0, int wdt, bool nt, hipStream_t st) {
  const bool p_is_q4 = wdt == WDT_Q4;
  GemvParams p = p0;
  int ks;
  gemm_plan(p.N, p.K, p.M, p.epi, ks);
  p.ksplit = ks;
  if (ks > 1) {
    size_t tk = 0;
    const size_t need = gemm_need(p.N, p.K, p.M, tk);
    if (need > g_kscratch_bytes || tk > g_ktickets_n) {  // reserved by gemm_reserve outside graph capture
      fprintf(stderr, "csm: split-K scratch not reserved for N=%d K=%d M=%d\n", p.N, p.K, p.M);
      abort();
    }
    p.kpart = g_kscratch;
    p.kticket = g_ktickets;
  }
  if (gemm_variant() == 2) {  // pipe: batch chunks of 64 (MT 2) or one chunk of 32 (MT 1) on grid.z
    const int MT = p.M > 32 ? 2 : 1;
    const dim3 g3(gemm_blocks(p.N), ks, (p.M + MT * 32 - 1) / (MT * 32));
    const int nst = p.K / ks / GP_KC;
    const int cap = pipe_pd_cap(p.M);
    const int pd = (nst % 4 == 0 && cap >= 4) ? 4 : ((nst % 2 == 0 && cap >= 2) ? 2 : 1);
#define GP_K(Q_, MT_, PD_) do { if (nt) hipLaunchKernelGGL((gemm_pipe_kernel<Q_, MT_, true, PD_>), g3, dim3(256), 0, st, p); \
                                else hipLaunchKernelGGL((gemm_pipe_kernel<Q_, MT_, false, PD_>), g3, dim3(256), 0, st, p); } while (0)
#define GP_L(Q_, MT_) do { if (pd == 4) GP_K(Q_, MT_, 4); else if (pd == 2) GP_K(Q_, MT_, 2); else GP_K(Q_, MT_, 1); } while (0)
    if (p_is_q4) { if (MT == 2) GP_L(true, 2); else GP_L(true, 1); }
    else { if (MT == 2) GP_L(false, 2); else GP_L(false, 1); }
#undef GP_L
#undef GP_K
    return;
  }
  const dim3 grid(gemm_blocks(p.N), ks);
  static const int lab_hl = [] { const char* e = getenv("CSM_GEMM_HL"); return e ? atoi(e) : 2; }();
  if (gemm_variant() == 0 && lab_hl == 1 && p.M <= 32) {  // lab only: hi part alone (not parity-grade)
    if (nt) hipLaunchKernelGGL((gemm_bf16_wk_kernel<1, GW_PF, true, false>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((gemm_bf16_wk_kernel<1, GW_PF, false, false>), grid, dim3(256), 0, st, p);
    return;
  }
  if (gemm_variant() == 0) {
    if (p.M > 32) {
      if (nt) hipLaunchKernelGGL((gemm_bf16_wk_kernel<2, GW_PF, true>), grid, dim3(256), 0, st, p);
      else hipLaunchKernelGGL((gemm_bf16_wk_kernel<2, GW_PF, false>), grid, dim3(256), 0, st, p);
    } else {
      if (nt) hipLaunchKernelGGL((gemm_bf16_wk_kernel<1, GW_PF, true>), grid, dim3(256), 0, st, p);
      else hipLaunchKernelGGL((gemm_bf16_wk_kernel<1, GW_PF, false>), grid, dim3(256), 0, st, p);
    }
    return;
  }
  if (p.M > 32) {
    if (nt) hipLaunchKernelGGL((gemm_bf16_kernel<2, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((gemm_bf16_kernel<2, false>), grid, dim3(256), 0, st, p);
  } else {
    if (nt) hipLaunchKernelGGL((gemm_bf16_kernel<1, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((gemm_bf16_kernel<1, false>), grid, dim3(256), 0, st, p);
  }
}

// Pre-size the split-K slab and tickets for an (N, K) launched at any M <= Mmax (call outside capture).
void gemm_reserve(int N, int K, int Mmax) {
  size_t slab = 0, tk = 0;
  for (int m = GEMM_MFMA_MIN_M; m <= Mmax; ++m) {  // cheap host loop (Mmax <= a few thousand)
    size_t t = 0;
    slab = std::max(slab, gemm_need(N, K, m, t));
    tk = std::max(tk, t);
  }
  if (slab > g_kscratch_bytes) {
    if (g_kscratch) (void)hipFree(g_kscratch);
    g_kscratch = nullptr;
    g_kscratch_bytes = 0;
    if (hipMalloc(&g_kscratch, slab) == hipSuccess) g_kscratch_bytes = slab;
  }
  if (tk > g_ktickets_n) {
    if (g_ktickets) (void)hipFree(g_ktickets);
    g_ktickets = nullptr;
    g_ktickets_n = 0;
    if (hipMalloc(&g_ktickets, tk * 4) == hipSuccess && hipMemset(g_ktickets, 0, tk * 4) == hipSuccess) g_ktickets_n = tk;
  }
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
