// Persistent batched depth-decoder step: the 4 decoder layers + the head of one codebook step i >= 2 for
// up to 32 (bf16 weights) or 64 (int4 g64 weights, MLX affine: nn.quantize) utterance rows
// (/root/reference/csm_mlx/generation.py:72-89 at batch B: decoder(projection(E_a[c])), then
// audio_head[i - 1]) in ONE launch, matrix cores for every projection.
//
// Why: on the launch path (run_dec_xs + the head launch) a step is ~21 dependent launches (QKV,
// attention, o_proj, gate/up, down per layer; the head); at 32-64 rows each is latency-bound -- ramp,
// first weight loads, split-K combine, drain: ~44 us per layer for ~53 MB of MALL-resident bf16 weights
// (profiles/r05_prof_config4_per_frame_roles.txt).  Here every CU keeps one workgroup for the step, owns
// fixed weight tiles of every projection and loads them into registers AHEAD of the hand-off that
// releases their activations, so the weight stream and the first-load latency sit under the waits.
//
// Roles (NWG = 256 workgroups x 8 waves, w = blockIdx.x; MR = 32 MT rows, MT row tiles of 32), per layer:
//   Q  w < 48         QKV tile w (32 of the 1536 rows), full K: x * n1 (split rows) -> RoPE, q | k | v
//                     rows + the K/V cache row at pos                               -> flag F1[w]
//   O  48 <= w < 80   o_proj tile j = w - 48 (32 columns), full K: + residual -> x_o, x_o * n2 (split),
//                     row sums of squares (int4: + half-group sums)               -> flag F3[j]
//   A  80 <= w < 80 + MR  attention of row m = w - 80, query head h = wave, keys 0..pos (the cached rows
//                     staged in LDS at the layer start; layer 0 takes q | k | v of the row's code from the
//                     folded table)                                               -> flag F2[m]
//   G  every w        gate/up tiles 2b, 2b + 1, b = 32 (w % 8) + w / 8 (the SiLU*up columns 32b..32b+31)
//                                                                                 -> flag FH[w]
//   D  every w        down, output tile j = w / 8 over h columns 1024 g .. + 1023, g = w % 8 (the G
//                     workgroups of group g: the same XCD under round-robin placement, speed only)
//                     -> partial tile; arrival ticket C4[j]; the eighth arrival sums the 8 partials in group
//                     order + residual -> x_d, x_d * (next n1 | final norm) split, row sums of squares
//                                                                                 -> flag F5[j]
//   H  80 + MR <= w   after the last layer: audio_head[i - 1] rows 64 t .. 64 t + 63 (bf16 tiles): logits
//                     and one arg-max partial per row -- the launch path's head partial layout
//
// Hand-offs (MI355X_MICROARCH.md, inter-workgroup visibility, valid form "ONE lane of each storing
// workgroup ... sc1 flag store or agent-scope atomic add"): every payload byte is stored sc1 and loaded
// sc1; each storing wave drains (s_waitcnt vmcnt(0)) before the workgroup barrier behind which one lane
// stores the flag / adds to the ticket; consumers poll with sc1 loads (one lane per flag), then a
// barrier.  Flags carry tag = epoch * 4 + layer + 1 and the tickets count monotonically from the epoch
// the launch read at its start (advanced by workgroup 0 at its end), so nothing is reset.  Every spin is
// bounded: on timeout a workgroup raises the error word and stops waiting (results garbage, the host
// raises) -- the grid always drains.  Single scratch buffers suffice: every rewrite of a buffer is
// ordered (through the hand-off chain) after every read of its previous contents.
//
// Arithmetic: the activations are fp32, split into three bf16 parts in registers (xs.h split_frag), so
// the matrix-core products are exact in fp32 and accumulate in fp32 (gemm_xs's arithmetic; summation
// order differs); int4: the nibbles enter the matrix cores as exact bf16 integers, per 64-column group
// acc += scale * sum_k q a + bias * sum_k a (the producers publish the half-group sums of the split
// rows, xs.h); RMSNorm folded as the streaming path's (x * norm weight split, row scale
// rsqrt(sum x^2 / D + eps) after the dot product); softmax with max subtraction in fp32.
#include "csm_kernels.h"
#include "handoff.h"
#include "xs.h"

namespace {

using namespace handoff;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

constexpr int NWG = DEC_XSD_WGS, NT = DEC_XSD_THREADS, NWV = NT / 64;
constexpr int D = 1024, F = 8192, HQ = 8, HKV = 2, HD = 128, NL = DEC_FRAME_LAYERS, QKV = (HQ + 2 * HKV) * HD;
constexpr int KS_D = D / 64, KS_F = F / 64;  // K stages of 64
constexpr int NQT = QKV / 32, NDT = D / 32;   // 48 QKV tiles; 32 o_proj / down / combine tiles
constexpr int NGRP = 8;                       // down K groups (1024 h columns each)
constexpr int O_WG0 = NQT;                    // o_proj workgroups 48 .. 79
constexpr int A_WG0 = O_WG0 + 32;             // attention workgroups 80 .. 80 + MR - 1
constexpr int RMAX = 64;                      // rows of the scratch buffers (row stride of sums)
constexpr unsigned SPIN_LIMIT = 1u << 22;
constexpr int SC1 = 16;  // buffer cache policy: sc1 (agent-coherent)
static_assert(NWG == 256 && NWV == 8, "roles assume 256 workgroups of 8 waves");
static_assert(KS_D == 2 * NWV && KS_F / NGRP == 2 * NWV, "every wave takes two K stages of its tile");
static_assert(RMAX == xs::HS_ROWS, "half-group sums use the xs.h row stride");

// control words (u32), one per 128-B line
// (F1 / F3: one flag per (tile, row tile) -- the int4 kernel's QKV and o_proj row tiles run on separate
// workgroups)
enum { CW_F1 = 0, CW_F2 = CW_F1 + 2 * NQT, CW_F3 = CW_F2 + RMAX, CW_FH = CW_F3 + 2 * NDT, CW_C4 = CW_FH + NWG,
       CW_F5 = CW_C4 + NDT, CW_FS = CW_F5 + NDT, CW_N = CW_FS + 128 };  // FS: head (tile, row tile)s done (sampled steps)
// int4 (two row tiles): the second row tile's QKV and o_proj workgroups
constexpr int Q1_WG0 = A_WG0 + 64, O1_WG0 = Q1_WG0 + NQT;
// XSD_QSPLIT (bf16): each QKV tile's K split over two workgroups (stages 0-7 on w < 48, 8-15 on QB_WG0 +
// the tile: workgroups idle until gate/up), one K stage per wave; they publish raw partial sums and the
// attention adds the halves, applies the row scale and RoPE and appends its row's K / V.  0: one
// workgroup per tile (A/B).
#ifndef XSD_QSPLIT
#define XSD_QSPLIT 1
#endif
constexpr int QB_WG0 = NWG - NQT;
constexpr int CW_STRIDE = 32;

#ifndef XSD_UNION
#define XSD_UNION 1  // lab: 0 keeps the attention buffers apart from the MFMA reduction slots
#endif
struct Lds {
#if XSD_UNION
  union {
#else
  struct {
#endif
    float red[NWV][2][16][64];  // MFMA roles: the per-wave accumulators of up to two tiles
    struct {                    // attention workgroups (wave = query head): cached keys / values 0..pos-1 of
      float Ks[HKV][32][HD + 4];//   both kv heads (rows padded: conflict-free row-parallel reads), each
      float Vs[HKV][32][HD];    //   wave's scaled query and the new key / value row at pos
      float qsh[HQ][HD];
      float kn[HQ][HD];
      float vn[HQ][HD];
    } at;
  };
  float ct[2][2][32][33];  // reduced tiles [row tile][tile][batch row][column]
  float rsp[8][RMAX];      // row scales: partial sums of squares (row_scales)
  float xg[NWV][2][RMAX];  // int4: X_g = sum over the stage's 64 columns of the split rows, per wave stage
  int flag;
};

struct Ctx {
  const DecStepXsArgs& p;
  Lds& L;
  int w, tid, lane, wave;
  unsigned ep;  // launch epoch
  int l = 0;    // layer (profiling marks)
  __device__ unsigned* cw(int i) const { return p.ctrl + (size_t)i * CW_STRIDE; }
  // profiling: the 100 MHz real-time clock at mark k of this layer (DEC_XSD_STAMPS slots per workgroup)
  __device__ void mark(int k) const {
    if (p.stamps && tid == 0) p.stamps[(size_t)w * DEC_XSD_STAMPS + 12 * l + k] = __builtin_amdgcn_s_memrealtime();
  }
  // sub-phase marks of layer 1 (slots 48..63)
  __device__ void sub(int k) const {
    if (p.stamps && tid == 0 && l == 1) p.stamps[(size_t)w * DEC_XSD_STAMPS + 48 + k] = __builtin_amdgcn_s_memrealtime();
  }
};

__device__ __forceinline__ bool spin_fail(const Ctx& c, unsigned spin) {
  if (spin >= SPIN_LIMIT || ((spin & 255) == 255 && __hip_atomic_load(c.p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
    __hip_atomic_store(c.p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  return false;
}
__device__ __forceinline__ unsigned ld_cw(const unsigned* a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// lanes < n of wave 0 wait until word idx(lane) has reached `target` (flags hold tags, tickets counts:
// both only grow), then the workgroup barrier
template <typename Idx>
__device__ __forceinline__ void wait_words(const Ctx& c, int n, Idx&& idx, unsigned target) {
  if (c.wave == 0 && c.lane < n) {
    const unsigned* a = c.cw(idx(c.lane));
    __builtin_amdgcn_s_sleep(8);
    for (unsigned spin = 0; (int)(ld_cw(a) - target) < 0; ++spin) {
      if (spin_fail(c, spin)) break;
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}
// after every storing wave drained: one lane publishes (the caller's barrier precedes)
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void set_flag(unsigned* a, unsigned tag) { __hip_atomic_store(a, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ unsigned add_ctr(unsigned* a) { return __hip_atomic_fetch_add(a, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
// (base wave-uniform -- it rides in the buffer descriptor; a per-lane base would make the compiler loop
// over the lanes' distinct descriptors -- and the lane's byte offset in the vector offset)
__device__ __forceinline__ void st16(void* base, size_t off, f32x4_t v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rsrc(base), (int)off, 0, SC1);
}
__device__ __forceinline__ f32x4_t ld16(const void* base, size_t off) {
  return __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), (int)off, 0, SC1));
}
__device__ __forceinline__ float2 ld8(const float* base, int off) {
  return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rsrc(base), off, 0, SC1));
}
__device__ __forceinline__ void st4(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// sum over the 8 lanes of a row group (lanes 8r .. 8r + 7), fixed butterfly order
__device__ __forceinline__ float sum8(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}

// ---- matrix-core tiles.  Weight tile registers: the wave's two K stages (st0, st0 + 1) of one 32-row
// tile of a fragment-tiled copy (gemm_retile) -- bf16: [tile][stage][s][lane] x 16 B; int4: [tile][stage]
// [lane] x 16 B of nibbles (word s = sub-step s) + the rows' {scale, bias} words after all nibbles.
// Activation registers: the same stages of one 32-row tile of the split rows (xs.h XS_F32 layout).
template <bool Q4> struct WTile;
template <> struct WTile<false> { u32x4_t a[2][4]; };
template <> struct WTile<true> { u32x4_t a[2]; unsigned sb[2]; };
struct AF { u32x4_t a[2][4][2]; };

// nt32: the matrix's 32-row tile count (int4: where the {scale, bias} words start)
template <bool Q4, int NS = 2>
__device__ __forceinline__ void load_wt(const uint8_t* T, int tile, int nks, int nt32, int st0, int lane, WTile<Q4>& r) {
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int ts = tile * nks + st0 + q;
    if constexpr (Q4) {
      r.a[q] = bload<0>(T, lane * 16, __builtin_amdgcn_readfirstlane(ts * 1024));
      r.sb[q] = bload4<0>(T, (lane & 31) * 4, __builtin_amdgcn_readfirstlane(nt32 * nks * 1024 + ts * 128));
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) r.a[q][s] = bload<0>(T, lane * 16, __builtin_amdgcn_readfirstlane((ts * 4 + s) * 1024));
    }
  }
}
// row tile t of split rows with nks K stages
template <int NS = 2>
__device__ __forceinline__ void load_af(const void* X, int nks, int t, int st0, int lane, AF& r) {
  const __amdgpu_buffer_rsrc_t rs = rsrc(X);
#pragma unroll
  for (int q = 0; q < NS; ++q)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
        r.a[q][s][hf] = __builtin_amdgcn_raw_buffer_load_b128(
            rs, lane * 16, __builtin_amdgcn_readfirstlane((((t * nks + st0 + q) * 4 + s) * 2 + hf) * 1024), SC1);
}
// int4: X_g of the wave's two stages for every row -> L.xg[wave] (from the producer's half-group sums
// hs[k / 32][RMAX]); a barrier follows before use
__device__ __forceinline__ void stage_xg(Ctx& c, const float* hs, int st0) {
  const __amdgpu_buffer_rsrc_t rs = rsrc(hs);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int st = st0 + q;
    const float a = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, c.lane * 4, __builtin_amdgcn_readfirstlane(2 * st * RMAX * 4), SC1));
    const float b = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, c.lane * 4, __builtin_amdgcn_readfirstlane((2 * st + 1) * RMAX * 4), SC1));
    c.L.xg[c.wave][q][c.lane] = a + b;
  }
}
// the wave's partial tiles of row tile t.  Accumulator register j of lane (r, h): batch row (j & 3) +
// 8 (j >> 2) + 4 h of the row tile, column r.
template <bool Q4, int NTL, int NS = 2>
__device__ __forceinline__ void mma(const Ctx& c, const AF& A, const WTile<Q4> (&W)[NTL], int t, f32x16_t (&acc)[NTL]) {
#pragma unroll
  for (int i = 0; i < NTL; ++i) acc[i] = f32x16_t{};
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    if constexpr (Q4) {
      f32x16_t gq[NTL];
#pragma unroll
      for (int i = 0; i < NTL; ++i) gq[i] = f32x16_t{};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8_t bq[NTL];
#pragma unroll
        for (int i = 0; i < NTL; ++i) bq[i] = __builtin_bit_cast(bf16x8_t, xs::q4_word_bf16(W[i].a[q][s]));
        u32x4_t pt[3];
        xs::split_frag(A.a[q][s][0], A.a[q][s][1], pt);
#pragma unroll
        for (int pp = 0; pp < 3; ++pp)
#pragma unroll
          for (int i = 0; i < NTL; ++i)
            gq[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, pt[pp]), bq[i], gq[i], 0, 0, 0);
      }
      // per-group fold: acc += scale * S_g + bias * X_g (the row's stage sum)
      const int hrow = 32 * t + 4 * (c.lane >> 5);
      float xr[16];
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const f32x4_t x4 = *reinterpret_cast<const f32x4_t*>(&c.L.xg[c.wave][q][hrow + 8 * j4]);
        xr[4 * j4] = x4.x; xr[4 * j4 + 1] = x4.y; xr[4 * j4 + 2] = x4.z; xr[4 * j4 + 3] = x4.w;
      }
#pragma unroll
      for (int i = 0; i < NTL; ++i) {
        const float sc = bf16_lo(W[i].sb[q]), bi = bf16_hi(W[i].sb[q]);
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
          acc[i][jj] = fmaf(sc, gq[i][jj], acc[i][jj]);
          acc[i][jj] = fmaf(bi, xr[jj], acc[i][jj]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one stage's temporaries live at a time
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        u32x4_t pt[3];
        xs::split_frag(A.a[q][s][0], A.a[q][s][1], pt);
#pragma unroll
        for (int pp = 0; pp < 3; ++pp)
#pragma unroll
          for (int i = 0; i < NTL; ++i)
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, pt[pp]),
                                                            __builtin_bit_cast(bf16x8_t, W[i].a[q][s]), acc[i], 0, 0, 0);
      }
    }
  }
}
// the 8 waves' partial tiles -> L.ct[t][i][batch row][column], added in wave order
template <int NTL>
__device__ __forceinline__ void reduce_tiles(Ctx& c, const f32x16_t (&acc)[NTL], int t) {
#pragma unroll
  for (int i = 0; i < NTL; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) c.L.red[c.wave][i][j][c.lane] = acc[i][j];
  __syncthreads();
#pragma unroll
  for (int e0 = 0; e0 < NTL * 1024; e0 += NT) {
    const int e = e0 + c.tid, i = e >> 10, m = (e >> 5) & 31, col = e & 31;
    const int j = (m & 3) + 4 * (m >> 3), ln = col + 32 * ((m >> 2) & 1);
    float v = c.L.red[0][i][j][ln];
#pragma unroll
    for (int wv = 1; wv < NWV; ++wv) v += c.L.red[wv][i][j][ln];
    c.L.ct[t][i][m][col] = v;
  }
  __syncthreads();
}
// one projection role's tiles for every row tile: split rows X (nks stages; int4: half-group sums hs)
// against the weight tiles W over the wave's stages st0, st0 + 1 -> L.ct.  The second row tile's operand
// loads are issued once the first tile's products are (its registers are then free).
// pre(): the role's other loads (row scales, residual), issued after the first operand loads (vmcnt
// retires in issue order: a load whose value is consumed first must be issued first).
template <bool Q4, int MT, int NTL, int T0 = 0, int NS = 2, typename Pre>
__device__ __forceinline__ void gemm_tiles(Ctx& c, const void* X, const float* hs, int nks, int st0, const WTile<Q4> (&W)[NTL], Pre&& pre) {
  static_assert(!Q4 || NS == 2, "int4: two stages per wave (stage_xg)");
  AF A;
  load_af<NS>(X, nks, T0, st0, c.lane, A);
  pre();
  if constexpr (Q4) {
    stage_xg(c, hs, st0);
    __syncthreads();
  }
#pragma unroll
  for (int t = T0; t < MT; ++t) {
    f32x16_t acc[NTL];
    mma<Q4, NTL, NS>(c, A, W, t, acc);
    if (t + 1 < MT) load_af<NS>(X, nks, t + 1, st0, c.lane, A);
    reduce_tiles<NTL>(c, acc, t);
  }
}

// Row scales rsqrt(sum_t ss[t][m] / D + eps) from 32 tiles' partial sums of squares (sc1, row stride
// RMAX): every thread adds 4 tiles of one row (loads in flight together) into L.rsp[part][row];
// row_scale() adds the 8 parts in order once a barrier (reduce_tiles') has published them
__device__ __forceinline__ void row_scales(Ctx& c, const float* ss) {
  const int m = c.tid & (RMAX - 1), q = c.tid / RMAX;  // (q wave-uniform)
  const __amdgpu_buffer_rsrc_t rs = rsrc(ss);
  float v[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
    v[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, m * 4, __builtin_amdgcn_readfirstlane((4 * q + t) * RMAX * 4), SC1));
  c.L.rsp[q][m] = ((v[0] + v[1]) + v[2]) + v[3];
}
__device__ __forceinline__ float row_scale(const Ctx& c, int m) {
  float s = c.L.rsp[0][m];
#pragma unroll
  for (int q = 1; q < 8; ++q) s += c.L.rsp[q][m];
  return rsqrtf(s / (float)D + c.p.eps);
}

// ---------------------------------------------------------------------------------------------------
// Q: QKV tile T of layer l (l >= 1)
// (row tiles RT0 .. RT1 - 1)
template <bool Q4, int RT0, int RT1>
__device__ __forceinline__ void role_q(Ctx& c, int l, int T, const WTile<Q4>& W) {
  const DecStepXsArgs& p = c.p;
  const unsigned tag = c.ep * NL + l;  // the previous layer's combine flags
  wait_words(c, NDT, [](int i) { return CW_F5 + i; }, tag);
  c.mark(1);
  gemm_tiles<Q4, RT1, 1, RT0>(c, p.xs_out, p.hs_out, KS_D, 2 * c.wave, reinterpret_cast<const WTile<Q4>(&)[1]>(W),
                              [&] { row_scales(c, p.ss_out); });
  c.sub(0);
  // rows m = tid / 16 (+ 32 per pass), columns 2 (tid % 16) + {0, 1} (RoPE pairs)
#pragma unroll
  for (int t = RT0; t < RT1; ++t) {
    const int ml = c.tid >> 4, m = 32 * t + ml, cc = 2 * (c.tid & 15), n = 32 * T + cc;
    const float r = row_scale(c, m);
    float a = c.L.ct[t][0][ml][cc] * r, b = c.L.ct[t][0][ml][cc + 1] * r;
    if (n < (HQ + HKV) * HD) {
      const float2 cs = reinterpret_cast<const float2*>(p.rope)[(size_t)p.step * (HD / 2) + (n % HD) / 2];
      const float y0 = a * cs.x - b * cs.y, y1 = b * cs.x + a * cs.y;
      a = y0;
      b = y1;
    }
    if (m < p.M) {
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, make_float2(a, b)), rsrc(p.qkv), (int)(((size_t)m * QKV + n) * 4), 0, SC1);
      if (n >= HQ * HD) {  // KVCache.update_and_fetch: the row at pos for the later codebook steps
        const int nn = n < (HQ + HKV) * HD ? n - HQ * HD : n - (HQ + HKV) * HD;
        float* cache = n < (HQ + HKV) * HD ? p.kc[l] : p.vc[l];
        *reinterpret_cast<float2*>(cache + (((size_t)m * HKV + nn / HD) * p.S_cap + p.step) * HD + nn % HD) = make_float2(a, b);
      }
    }
  }
  c.sub(1);
  drain();
  __syncthreads();
  if (c.tid == 0) set_flag(c.cw(CW_F1 + T + NQT * RT0), tag + 1);
  c.mark(2);
}

// bf16 XSD_QSPLIT: QKV tile T over K half HALF (stages 8 HALF .. 8 HALF + 7, one per wave) -> the raw
// partial sums qkvp[HALF][m][n] (role_a adds the halves, scales, rotates); the half-0 workgroups also
// publish the row scales (row_scales / row_scale, their loads under the operand loads) in qkvr[T][m]
template <int HALF>
__device__ __forceinline__ void role_qh(Ctx& c, int l, int T, const WTile<false>& W) {
  const DecStepXsArgs& p = c.p;
  const unsigned tag = c.ep * NL + l;  // the previous layer's combine flags
  wait_words(c, NDT, [](int i) { return CW_F5 + i; }, tag);
  c.mark(1);
  gemm_tiles<false, 1, 1, 0, 1>(c, p.xs_out, nullptr, KS_D, 8 * HALF + c.wave, reinterpret_cast<const WTile<false>(&)[1]>(W), [&] {
    if constexpr (HALF == 0) row_scales(c, p.ss_out);
  });
  c.sub(0);
  {
    const int m = c.tid >> 4, cc = 2 * (c.tid & 15), n = 32 * T + cc;
    if (m < p.M) {
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, make_float2(c.L.ct[0][0][m][cc], c.L.ct[0][0][m][cc + 1])),
                                            rsrc(p.qkvp + (size_t)HALF * RMAX * QKV), (int)(((size_t)m * QKV + n) * 4), 0, SC1);
      if (HALF == 0 && (c.tid & 15) == 0)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(row_scale(c, m)), rsrc(p.qkvp + (size_t)2 * RMAX * QKV),
                                              (T * RMAX + m) * 4, 0, SC1);
    }
  }
  c.sub(1);
  drain();
  __syncthreads();
  if (c.tid == 0) set_flag(c.cw(CW_F1 + T + NQT * HALF), tag + 1);
  c.mark(2);
}

// The cached K / V rows 0..pos-1 of the attention workgroup's row, both kv heads -> LDS (written by earlier
// launches: plain loads), at the start of the layer, before any hand-off wait of the workgroup
__device__ __forceinline__ void stage_kv(Ctx& c, int l) {
  const DecStepXsArgs& p = c.p;
  const int m = c.w - A_WG0, pos = p.step;
  if (m < 0 || m >= p.M) return;
  typedef float f4 __attribute__((ext_vector_type(4)));
  // 2 kv heads x pos rows x 32 float4 of K and of V: <= 8 float4 per thread, all in flight together
  constexpr int PER = HKV * 32 * (HD / 4) / NT;
  const int n4 = pos * (HD / 4);
  f4 t[2][PER];
#pragma unroll
  for (int kv = 0; kv < 2; ++kv)
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = c.tid + u * NT, g = e / (32 * (HD / 4)), r = e % (32 * (HD / 4));
      if (r < n4) t[kv][u] = *reinterpret_cast<const f4*>((kv ? p.vc[l] : p.kc[l]) + (((size_t)m * HKV + g) * p.S_cap) * HD + 4 * (size_t)r);
    }
#pragma unroll
  for (int kv = 0; kv < 2; ++kv)
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = c.tid + u * NT, g = e / (32 * (HD / 4)), r = e % (32 * (HD / 4));
      if (r < n4) {
        float* dst = kv ? &c.L.at.Vs[g][r / (HD / 4)][4 * (r % (HD / 4))] : &c.L.at.Ks[g][r / (HD / 4)][4 * (r % (HD / 4))];
        *reinterpret_cast<f4*>(dst) = t[kv][u];
      }
    }
}

// A (workgroups A_WG0 .. A_WG0 + MR - 1): attention of row m = w - A_WG0, query head h = wave, keys
// 0..pos -> xs_att (split rows of the o_proj; int4: + half-group sums).  The cached K / V rows are in LDS
// (stage_kv); each wave fetches its query and the new key / value row at pos (layer 0: of the row's code,
// from the folded table; else from the QKV tiles, after their flags) and computes.
template <bool Q4>
__device__ __forceinline__ void role_a(Ctx& c, int l) {
  const DecStepXsArgs& p = c.p;
  const int m = c.w - A_WG0, h = c.wave, g = h / (HQ / HKV), pos = p.step, n = pos + 1;
  const unsigned tag = c.ep * NL + l + 1;
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int lane = c.lane;
  c.sub(7);
  if (m < p.M) {
    const float scale = 0.08838834764831845f;  // 1 / sqrt(128)
    float2 qv, kv2, vv2;
    if (l == 0) {
      // the row's code: arg-max of the previous head's partials (or the sampler's single partial)
      const unsigned long long best = wave_argmax_partials(p.part + (size_t)m * p.part_stride, p.part_n, lane);
      const int code = min(max(unpack_argmax(best), 0), p.V - 1);
      const float* trow = p.qkv0_tab + (size_t)code * QKV;  // RoPE'd q | k | v of layer 0 (static table)
      qv = reinterpret_cast<const float2*>(trow + h * HD)[lane];
      kv2 = reinterpret_cast<const float2*>(trow + HQ * HD + g * HD)[lane];
      vv2 = reinterpret_cast<const float2*>(trow + (HQ + HKV) * HD + g * HD)[lane];
      if (h % (HQ / HKV) == 0) {  // this kv head's row at pos -> cache (later codebook steps)
        const size_t o = (((size_t)m * HKV + g) * p.S_cap + pos) * HD + 2 * lane;
        *reinterpret_cast<float2*>(p.kc[0] + o) = kv2;
        *reinterpret_cast<float2*>(p.vc[0] + o) = vv2;
      }
      if (h == 0 && lane == 0) {
        p.codes[(size_t)m * p.codes_K + pos - 1] = code;
        __hip_atomic_store(p.code_buf + m, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      // q tiles 4h..4h+3, k tiles 32 + 4g.., v tiles 40 + 4g.. (XSD_QSPLIT: of both K halves)
      constexpr bool QS = !Q4 && XSD_QSPLIT;
      if (lane < (QS ? 24 : 12)) {
        const int lt = lane % 12;
        const int t = lt < 4 ? 4 * h + lt : (lt < 8 ? HQ * 4 + 4 * g + lt - 4 : (HQ + HKV) * 4 + 4 * g + lt - 8);
        const unsigned* a = c.cw(CW_F1 + t + NQT * (QS ? lane / 12 : (m >> 5)));  // the K half / the row's row tile
        __builtin_amdgcn_s_sleep(8);
        for (unsigned spin = 0; (int)(ld_cw(a) - tag) < 0; ++spin) {
          if (spin_fail(c, spin)) break;
          __builtin_amdgcn_s_sleep(2);
        }
      }
      // (the wave leaves the poll loop once every polling lane has matched)
      c.sub(8);
      if constexpr (QS) {
        // the halves' sums, the row scale (row_scales' order: 4 tiles a part, the 8 parts in turn), RoPE,
        // the K / V row at pos -> cache (each kv head by its first query head's wave)
        const float* r0 = p.qkvp + (size_t)m * QKV;
        const float* r1 = r0 + (size_t)RMAX * QKV;
        const float2 q0 = ld8(r0, (h * HD + 2 * lane) * 4), q1 = ld8(r1, (h * HD + 2 * lane) * 4);
        const float2 k0 = ld8(r0, (HQ * HD + g * HD + 2 * lane) * 4), k1 = ld8(r1, (HQ * HD + g * HD + 2 * lane) * 4);
        const float2 v0 = ld8(r0, ((HQ + HKV) * HD + g * HD + 2 * lane) * 4), v1 = ld8(r1, ((HQ + HKV) * HD + g * HD + 2 * lane) * 4);
        // the row scale the q tile 4h's half-0 workgroup published (its flag was polled above)
        const float rs = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc(p.qkvp + (size_t)2 * RMAX * QKV),
                                                                                       (4 * h * RMAX + m) * 4, 0, SC1));
        const float2 cs = reinterpret_cast<const float2*>(p.rope)[(size_t)pos * (HD / 2) + lane];
        auto rot = [&](float a, float b) { return make_float2(a * cs.x - b * cs.y, b * cs.x + a * cs.y); };
        qv = rot((q0.x + q1.x) * rs, (q0.y + q1.y) * rs);
        kv2 = rot((k0.x + k1.x) * rs, (k0.y + k1.y) * rs);
        vv2 = make_float2((v0.x + v1.x) * rs, (v0.y + v1.y) * rs);
        if (h % (HQ / HKV) == 0) {  // KVCache.update_and_fetch: this kv head's row at pos
          const size_t o = (((size_t)m * HKV + g) * p.S_cap + pos) * HD + 2 * lane;
          *reinterpret_cast<float2*>(p.kc[l] + o) = kv2;
          *reinterpret_cast<float2*>(p.vc[l] + o) = vv2;
        }
      } else {
        const float* row = p.qkv + (size_t)m * QKV;
        qv = ld8(row, (h * HD + 2 * lane) * 4);
        kv2 = ld8(row, (HQ * HD + g * HD + 2 * lane) * 4);
        vv2 = ld8(row, ((HQ + HKV) * HD + g * HD + 2 * lane) * 4);
      }
    }
    *reinterpret_cast<float2*>(&c.L.at.qsh[h][2 * lane]) = make_float2(qv.x * scale, qv.y * scale);
    *reinterpret_cast<float2*>(&c.L.at.kn[h][2 * lane]) = kv2;
    *reinterpret_cast<float2*>(&c.L.at.vn[h][2 * lane]) = vv2;
    c.sub(9);
  }
  __syncthreads();  // stage_kv's rows (every wave) and this wave's own rows
  c.mark(3);
  if (m < p.M) {
    // lane = (key kj = lane & 31, half hh of the head dims): scores from two half dots added by one
    // shuffle, max-subtracted softmax, P.V in key order (lane = key half kv, dims 4 dq .. + 3)
    const int kj = lane & 31, hh = lane >> 5, kv = lane >> 5, dq = lane & 31;
    float s;
    {
      const float* krow = kj < pos ? &c.L.at.Ks[g][kj][0] : &c.L.at.kn[h][0];
      const f4* kr = reinterpret_cast<const f4*>(krow + hh * (HD / 2));
      const f4* qr = reinterpret_cast<const f4*>(&c.L.at.qsh[h][hh * (HD / 2)]);
      float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
#pragma unroll
      for (int d4 = 0; d4 < HD / 8; ++d4) {
        const f4 a = kr[d4], q4 = qr[d4];
        d0 = fmaf(q4.x, a.x, d0);
        d1 = fmaf(q4.y, a.y, d1);
        d2 = fmaf(q4.z, a.z, d2);
        d3 = fmaf(q4.w, a.w, d3);
      }
      const float part = (d0 + d1) + (d2 + d3);
      const float other = __shfl_xor(part, 32, 64);
      s = hh == 0 ? part + other : other + part;
      if (kj >= n) s = -INFINITY;
    }
    const float mx = wave_max(s);
    const float pj = kj < n ? expf(s - mx) : 0.f;
    const float l_run = wave_sum(hh == 0 ? pj : 0.f);
    const int pji = __float_as_int(pj);
    f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u0 = 0; u0 < 16; u0 += 8) {
      if (u0 < n) {
        f4 vv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int jj = 16 * kv + u0 + u;
          vv[u] = *reinterpret_cast<const f4*>(jj < pos ? &c.L.at.Vs[g][jj][4 * dq] : &c.L.at.vn[h][4 * dq]);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float pa = __int_as_float(__builtin_amdgcn_readlane(pji, u0 + u));
          const float pb = __int_as_float(__builtin_amdgcn_readlane(pji, 16 + u0 + u));
          const float pw = kv ? pb : pa;
          if (16 * kv + u0 + u < n) {
            acc.x = fmaf(pw, vv[u].x, acc.x);
            acc.y = fmaf(pw, vv[u].y, acc.y);
            acc.z = fmaf(pw, vv[u].z, acc.z);
            acc.w = fmaf(pw, vv[u].w, acc.w);
          }
        }
      }
    }
    const float inv = 1.f / l_run;
    const float t0 = __shfl_xor(acc.x, 32, 64), t1 = __shfl_xor(acc.y, 32, 64), t2 = __shfl_xor(acc.z, 32, 64),
                t3 = __shfl_xor(acc.w, 32, 64);
    const f32x4_t o = {(acc.x + t0) * inv, (acc.y + t1) * inv, (acc.z + t2) * inv, (acc.w + t3) * inv};
    if (lane < 32) st16(p.xs_att, xs::off(D, m, h * HD + 4 * dq), o);
    if constexpr (Q4) {  // half group (h * 128 + 4 dq) / 32: lanes dq = 8j .. 8j + 7, columns in order
      const float hs = sum8((o.x + o.y) + (o.z + o.w));
      if (lane < 32 && (dq & 7) == 0) st4(p.hs_att + (size_t)((h * HD + 4 * dq) / 32) * RMAX + m, hs);
    }
  }
  drain();
  __syncthreads();
  // one flag per attention workgroup (rows past M publish without work)
  if (c.tid == 0) set_flag(c.cw(CW_F2 + m), tag);
  c.mark(4);
}

// O: o_proj tile j (+ residual) -> x_o, split x_o * n2, row sums of squares (int4: half-group sums)
// (row tiles RT0 .. RT1 - 1: the attention rows 32 RT0 .. 32 RT1 - 1)
template <bool Q4, int RT0, int RT1>
__device__ __forceinline__ void role_o(Ctx& c, int l, int j, const WTile<Q4>& W) {
  const DecStepXsArgs& p = c.p;
  const unsigned tag = c.ep * NL + l + 1;
  wait_words(c, 32 * (RT1 - RT0), [](int i) { return CW_F2 + 32 * RT0 + i; }, tag);
  c.mark(5);
  // residual: layer 0 the projected input row proj_tab[code], else the previous layer's x_d
  const int mm = c.tid >> 3, m = 32 * RT0 + mm, q = c.tid & 7, n = 32 * j + 4 * q;
  f32x4_t res = {0.f, 0.f, 0.f, 0.f}, nw;
  gemm_tiles<Q4, RT1, 1, RT0>(c, p.xs_att, p.hs_att, KS_D, 2 * c.wave, reinterpret_cast<const WTile<Q4>(&)[1]>(W), [&] {
    if (mm < 32 * (RT1 - RT0) && m < p.M) {
      if (l == 0) {
        const int code = __hip_atomic_load(p.code_buf + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        res = *reinterpret_cast<const f32x4_t*>(p.proj_tab + (size_t)code * D + n);
      } else {
        res = ld16(p.x_d, ((size_t)m * D + n) * 4);
      }
    }
    nw = *reinterpret_cast<const f32x4_t*>(p.n2[l] + n);
  });
  c.sub(6);
  if (mm < 32 * (RT1 - RT0)) {
    f32x4_t x = {0.f, 0.f, 0.f, 0.f};
    const int t = m >> 5, ml = m & 31;
    if (m < p.M) x = res + f32x4_t{c.L.ct[t][0][ml][4 * q], c.L.ct[t][0][ml][4 * q + 1], c.L.ct[t][0][ml][4 * q + 2], c.L.ct[t][0][ml][4 * q + 3]};
    const f32x4_t xn = x * nw;
    st16(p.x_o, ((size_t)m * D + n) * 4, x);
    st16(p.xs_x, xs::off(D, m, n), xn);
    const float sq = sum8(fmaf(x.w, x.w, fmaf(x.z, x.z, fmaf(x.y, x.y, x.x * x.x))));
    if (q == 0) st4(p.ss_o + (size_t)j * RMAX + m, sq);
    if constexpr (Q4) {
      const float hs = sum8((xn.x + xn.y) + (xn.z + xn.w));
      if (q == 0) st4(p.hs_x + (size_t)j * RMAX + m, hs);
    }
  }
  drain();
  __syncthreads();
  if (c.tid == 0) set_flag(c.cw(CW_F3 + j + NDT * RT0), tag);
  c.mark(6);
}

// G: gate/up tiles 2b, 2b + 1 -> SiLU*up columns 32b .. 32b + 31 (split, K = F; int4: + half-group sums)
template <bool Q4, int MT>
__device__ __forceinline__ void role_g(Ctx& c, int l, const WTile<Q4> (&W)[2]) {
  const DecStepXsArgs& p = c.p;
  const int b = 32 * (c.w & 7) + (c.w >> 3);
  const unsigned tag = c.ep * NL + l + 1;
  wait_words(c, NDT * MT, [](int i) { return CW_F3 + i; }, tag);  // every (o_proj tile, row tile)
  c.mark(7);
  gemm_tiles<Q4, MT, 2>(c, p.xs_x, p.hs_x, KS_D, 2 * c.wave, W, [&] { row_scales(c, p.ss_o); });
  c.sub(3);
  const int m = c.tid >> 3, q = c.tid & 7;
  if (m < 32 * MT) {
    const int t = m >> 5, ml = m & 31;
    const float r = row_scale(c, m);
    float hv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pc = 4 * q + i, ti = pc >> 4, cc = 2 * (pc & 15);  // wgu rows interleave gate_j, up_j
      const float gt = c.L.ct[t][ti][ml][cc] * r, up = c.L.ct[t][ti][ml][cc + 1] * r;
      hv[i] = silu_f(gt) * up;
    }
    st16(p.xs_h, xs::off(F, m, 32 * b + 4 * q), f32x4_t{hv[0], hv[1], hv[2], hv[3]});
    if constexpr (Q4) {
      const float hs = sum8((hv[0] + hv[1]) + (hv[2] + hv[3]));
      if (q == 0) st4(p.hs_h + (size_t)b * RMAX + m, hs);
    }
  }
  c.sub(4);
  drain();
  __syncthreads();
  if (c.tid == 0) set_flag(c.cw(CW_FH + c.w), tag);
  c.mark(8);
}

// D: down tile j over K group g -> partial; the eighth arrival combines
template <bool Q4, int MT>
__device__ __forceinline__ void role_d(Ctx& c, int l, const WTile<Q4>& W) {
  const DecStepXsArgs& p = c.p;
  const int g = c.w & 7, j = c.w >> 3;
  const unsigned tag = c.ep * NL + l + 1;
  wait_words(c, 32, [g](int i) { return CW_FH + g + 8 * i; }, tag);  // the G workgroups of group g
  c.mark(9);
  gemm_tiles<Q4, MT, 1>(c, p.xs_h, p.hs_h, KS_F, 16 * g + 2 * c.wave, reinterpret_cast<const WTile<Q4>(&)[1]>(W), [] {});
  c.sub(5);
  const int m = c.tid >> 3, q = c.tid & 7, n = 32 * j + 4 * q;
  if (m < 32 * MT) {
    const int t = m >> 5, ml = m & 31;
    st16(p.dpart, (((size_t)g * RMAX + m) * D + n) * 4,
         f32x4_t{c.L.ct[t][0][ml][4 * q], c.L.ct[t][0][ml][4 * q + 1], c.L.ct[t][0][ml][4 * q + 2], c.L.ct[t][0][ml][4 * q + 3]});
  }
  drain();
  __syncthreads();
  if (c.tid == 0) c.L.flag = add_ctr(c.cw(CW_C4 + j)) + 1u == tag * NGRP;
  __syncthreads();
  c.mark(10);
  if (!c.L.flag) return;
  // combine (the last of the tile's 8 groups): x_d = x_o + sum_g partial_g, split with the next norm
  const float* nwp = l + 1 < NL ? p.n1[l + 1] : p.norm;
  if (m < 32 * MT) {
    f32x4_t pp[NGRP];
#pragma unroll
    for (int gg = 0; gg < NGRP; ++gg) pp[gg] = ld16(p.dpart, (((size_t)gg * RMAX + m) * D + n) * 4);
    const f32x4_t xo = ld16(p.x_o, ((size_t)m * D + n) * 4);
    const f32x4_t nw = *reinterpret_cast<const f32x4_t*>(nwp + n);
    f32x4_t s = pp[0];
#pragma unroll
    for (int gg = 1; gg < NGRP; ++gg) s += pp[gg];
    f32x4_t x = {0.f, 0.f, 0.f, 0.f};
    if (m < p.M) x = xo + s;
    const f32x4_t xn = x * nw;
    st16(p.x_d, ((size_t)m * D + n) * 4, x);
    st16(p.xs_out, xs::off(D, m, n), xn);
    const float sq = sum8(fmaf(x.w, x.w, fmaf(x.z, x.z, fmaf(x.y, x.y, x.x * x.x))));
    if (q == 0) st4(p.ss_out + (size_t)j * RMAX + m, sq);
    if constexpr (Q4) {
      const float hs = sum8((xn.x + xn.y) + (xn.z + xn.w));
      if (q == 0) st4(p.hs_out + (size_t)j * RMAX + m, hs);
    }
  }
  drain();
  __syncthreads();
  if (c.tid == 0) set_flag(c.cw(CW_F5 + j), tag);
  c.mark(11);
}

// H: audio_head[step - 1] rows 64 t .. 64 t + 63 (two bf16 32-row tiles) of the final-normed rows (the
// last combines' split x * norm + sums of squares) -> logits [row][Vp] and the tile's arg-max partial
// per row (pack_argmax: the largest logit, the first index on ties), exactly the partial layout of the
// launch path's head (gemm_xs EPI_ARGMAX, 64-row tiles), which the next step / advance_kernel reduce
// (head tile t, row tiles RT0 .. RT1 - 1: the int4 kernel's two row tiles on separate workgroups)
template <int RT0, int RT1>
__device__ __forceinline__ void role_h(Ctx& c, int t, const WTile<false> (&W)[2]) {
  const DecStepXsArgs& p = c.p;
  const unsigned tag = c.ep * NL + NL;  // the last layer's combine flags
  wait_words(c, NDT, [](int i) { return CW_F5 + i; }, tag);
  gemm_tiles<false, RT1, 2, RT0>(c, p.xs_out, nullptr, KS_D, 2 * c.wave, W, [&] { row_scales(c, p.ss_out); });
  // row m = tid / 16 (+ 32 per row tile), columns 4 (tid % 16) .. + 3 of the 64
#pragma unroll
  for (int rt = RT0; rt < RT1; ++rt) {
    const int ml = c.tid >> 4, m = 32 * rt + ml, c4 = 4 * (c.tid & 15), n = 64 * t + c4;
    const float r = row_scale(c, m);
    unsigned long long best = 0;
    if (m < p.M && n < p.Vp) {
      const float* ct = &c.L.ct[rt][c4 >> 5][ml][c4 & 31];
      const float4 v = make_float4(ct[0] * r, ct[1] * r, ct[2] * r, ct[3] * r);
      if (p.sample) st16(p.head_out, ((size_t)m * p.Vp + n) * 4, f32x4_t{v.x, v.y, v.z, v.w});  // (role_s reads them)
      else *reinterpret_cast<float4*>(p.head_out + (size_t)m * p.Vp + n) = v;
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (n + i < p.n_valid) {
          const unsigned long long k = pack_argmax(vv[i], n + i);
          best = k > best ? k : best;
        }
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const unsigned long long v = __shfl_xor(best, o, 64);
      best = v > best ? v : best;
    }
    // (sampled steps: role_s publishes the row's single partial; slot 0 written here too would race it
    // across the XCDs' L2s)
    if (m < p.M && (c.tid & 15) == 0 && !p.sample) p.head_part[(size_t)m * p.part_stride + t] = best;
  }
  if (p.sample) {  // this tile's logits -> the sampling workgroups
    drain();
    __syncthreads();
    if (c.tid == 0) set_flag(c.cw(CW_FS + t + 64 * RT0), c.ep + 1u);
  }
}

// S (sampled steps; workgroup m < M, after its layers): row m's code from the head's logits -- the sampler
// of sample_kernel (csm_kernels.hip) on 512 threads, as dec_frame.hip's sample_code: the top_k-th largest
// logit by radix select (keys >= it kept, ties included), then the Gumbel-max of logit * (1 / T) + noise
// over the kept entries, the lowest index on ties (the same winner whatever the visiting order) ->
// codes[m][cb] and the 1-entry partial the next step reads.
__device__ __forceinline__ void role_s(Ctx& c) {
  constexpr int NPT = DEC_XSD_SAMPLE_NPT;
  const DecStepXsArgs& p = c.p;
  const int m = c.w, V = p.n_valid;
  // the Gumbel noise does not depend on the logits: drawn before the wait
  const uint64_t key = gumbel_key(p.s_seeds[m], p.s_frame_ctr[0] * p.s_K + p.s_cb);
  double gn[NPT];
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int v = c.tid + NT * i;
    gn[i] = v < V ? gumbel_noise(key, v) : 0.0;
  }
  const int fs0 = CW_FS + 64 * (m >> 5);  // the head tiles of the row's row tile
  wait_words(c, p.head_tiles, [fs0](int i) { return fs0 + i; }, c.ep + 1u);
  float lg[NPT];
  const __amdgpu_buffer_rsrc_t rs = rsrc(p.head_out + (size_t)m * p.Vp);
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int v = c.tid + NT * i;
    lg[i] = v < V ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, v * 4, 0, SC1)) : 0.f;
  }
  float thr = -INFINITY;
  uint32_t* hist = reinterpret_cast<uint32_t*>(&c.L.red[0][0][0][0]);
  uint32_t* wsum = hist + 256;
  uint32_t* sh = hist + 264;  // [prefix, remain]
  if (p.s_top_k > 0 && p.s_top_k < V) {  // radix select, 8 bits per pass; threads 0..255 hold digit 255 - tid
    uint32_t prefix = 0, maskbits = 0, rem = (uint32_t)p.s_top_k;
    for (int shift = 24; shift >= 0; shift -= 8) {
      if (c.tid < 256) hist[c.tid] = 0;
      __syncthreads();
#pragma unroll
      for (int i = 0; i < NPT; ++i) {
        const int v = c.tid + NT * i;
        if (v < V) {
          const uint32_t k = f2key(lg[i]);
          if ((k & maskbits) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
        }
      }
      __syncthreads();
      uint32_t h = 0, cnt = 0;
      if (c.tid < 256) {
        h = hist[255 - c.tid];
        cnt = h;  // inclusive prefix over t = count of keys with digit >= 255 - t
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t u = __shfl_up(cnt, o, 64);
          if (c.lane >= o) cnt += u;
        }
        if (c.lane == 63) wsum[c.wave] = cnt;
      }
      __syncthreads();
      if (c.tid < 256) {
        for (int w = 0; w < c.wave; ++w) cnt += wsum[w];
        const uint32_t above = cnt - h;
        if (h > 0 && above < rem && rem <= cnt) {  // exactly one digit
          sh[0] = prefix | ((uint32_t)(255 - c.tid) << shift);
          sh[1] = rem - above;
        }
      }
      __syncthreads();
      prefix = sh[0];
      rem = sh[1];
      maskbits |= 255u << shift;
      __syncthreads();  // hist / sh reused by the next pass
    }
    thr = key2f(prefix);
  }
  const float inv_t = 1.0f / p.s_temperature;
  double best = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int v = c.tid + NT * i;
    if (v >= V || !(lg[i] >= thr)) continue;
    const double val = (double)(lg[i] * inv_t) + gn[i];  // = gumbel_perturbed(l, inv_t, key, v)
    if (val > best) {  // increasing v per thread: first max kept
      best = val;
      bi = v;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  double* sv = reinterpret_cast<double*>(hist + 272);
  int* si = reinterpret_cast<int*>(sv + NWV);
  if (c.lane == 0) { sv[c.wave] = best; si[c.wave] = bi; }
  __syncthreads();
  if (c.tid == 0) {
    double bv = sv[0];
    int b = si[0];
    for (int w2 = 1; w2 < NWV; ++w2)
      if (sv[w2] > bv || (sv[w2] == bv && si[w2] < b)) { bv = sv[w2]; b = si[w2]; }
    const int code = min(max(b, 0), V - 1);  // NaN logits leave no winner: clamp (as sample_kernel)
    p.codes[(size_t)m * p.codes_K + p.s_cb] = code;
    p.head_part[(size_t)m * p.part_stride] = pack_argmax(0.f, code);  // consumed as a 1-entry partial
  }
}

// The layer loop of one workgroup class (each its own straight-line code: exact register liveness per
// class, no merged paths holding another class's prefetch registers).  CLS: 0 QKV, 1 o_proj,
// 2 attention, 3 head (+ plain), 4 plain (gate/up + down only), 5 / 6 QKV / o_proj of the second row
// tile (int4).  int4: the head runs on the attention workgroups (their registers are free after the last
// layer), the head class does not exist.
enum { C_Q = 0, C_O = 1, C_A = 2, C_H = 3, C_P = 4, C_Q1 = 5, C_O1 = 6, C_QB = 7 };
template <bool Q4, int CLS>
__device__ __forceinline__ void run_layers(Ctx& c) {
  static_assert(CLS >= C_Q && CLS <= C_QB, "workgroup class");
  constexpr int MT = Q4 ? 2 : 1;
  constexpr bool IS_Q = CLS == C_Q || CLS == C_Q1 || CLS == C_QB, IS_O = CLS == C_O || CLS == C_O1;
  constexpr int RT0 = (CLS == C_Q1 || CLS == C_O1) ? 1 : 0, RT1 = Q4 ? RT0 + 1 : MT;
  constexpr bool QS = !Q4 && XSD_QSPLIT;  // bf16 QKV K halves: stage 8 HALF + wave
  constexpr int QHALF = CLS == C_QB ? 1 : 0, QNS = QS ? 1 : 2;
  const int qst = QS ? 8 * QHALF + c.wave : 2 * c.wave;
  const int qt = c.w - (CLS == C_Q1 ? Q1_WG0 : (CLS == C_QB ? QB_WG0 : 0)), ot = c.w - (CLS == C_O1 ? O1_WG0 : O_WG0);
  const DecStepXsArgs& p = c.p;
  const int b = 32 * (c.w & 7) + (c.w >> 3), g = c.w & 7, j = c.w >> 3;
  WTile<Q4> wq, wgu[2], wd;
  // vmcnt retires in issue order and every publish drains it: a prefetch issued just before a hand-off
  // poll or a latency-critical operand load holds that back, so each class issues its next tiles after
  // its own latency-critical steps (Q, A: after their publish).  The plain and head classes (the most
  // registers to spare) fetch their down tile with gate/up; the others during the h hand-off.
  constexpr bool WD_EARLY = CLS == C_P || CLS == C_H;
  auto ld_gu = [&](int l) {
    load_wt<Q4>(p.wgu[l], 2 * b, KS_D, 2 * F / 32, 2 * c.wave, c.lane, wgu[0]);
    load_wt<Q4>(p.wgu[l], 2 * b + 1, KS_D, 2 * F / 32, 2 * c.wave, c.lane, wgu[1]);
    if constexpr (WD_EARLY) load_wt<Q4>(p.wd[l], j, KS_F, D / 32, 16 * g + 2 * c.wave, c.lane, wd);
  };
  if constexpr (IS_Q) load_wt<Q4, QNS>(p.wqkv[1], qt, KS_D, NQT, qst, c.lane, wq);
  if constexpr (IS_O) load_wt<Q4>(p.wo[0], ot, KS_D, NDT, 2 * c.wave, c.lane, wq);
  if constexpr (CLS != C_A) ld_gu(0);
  for (int l = 0; l < NL; ++l) {
    c.l = l;
    c.mark(0);
    if constexpr (IS_O || CLS == C_H || CLS == C_P) {
      if (l > 0) {
        if constexpr (IS_O) load_wt<Q4>(p.wo[l], ot, KS_D, NDT, 2 * c.wave, c.lane, wq);
        ld_gu(l);
      }
    }
    if constexpr (IS_Q) {
      if (l > 0) {
        if constexpr (QS) role_qh<QHALF>(c, l, qt, wq);
        else role_q<Q4, RT0, RT1>(c, l, qt, wq);
        ld_gu(l);
      }
    }
    if constexpr (CLS == C_A) {
      stage_kv(c, l);  // (role_a's barrier publishes the LDS rows)
      role_a<Q4>(c, l);
      ld_gu(l);
    }
    if constexpr (IS_O) role_o<Q4, RT0, RT1>(c, l, ot, wq);
    role_g<Q4, MT>(c, l, wgu);
    if constexpr (!WD_EARLY) load_wt<Q4>(p.wd[l], j, KS_F, D / 32, 16 * g + 2 * c.wave, c.lane, wd);  // during the h hand-off
    role_d<Q4, MT>(c, l, wd);
    // the next layer's QKV tile: during the combine the Q hand-off waits for
    if constexpr (IS_Q) {
      if (l > 0 && l + 1 < NL) load_wt<Q4, QNS>(p.wqkv[l + 1], qt, KS_D, NQT, qst, c.lane, wq);
    }
  }
  // bf16 head tiles (a 32-row tile past the last is clamped: its columns are never stored).  bf16: head
  // tile w - H_WG0 on the head class; int4: (tile, row tile) k = (k % tiles, k / tiles) on the attention
  // workgroups (k = w - A_WG0) and, past their 64, the first plain ones (k = 64 + w - P4_WG0)
  constexpr int H_WG0 = A_WG0 + 32 * MT, P4_WG0 = O1_WG0 + NDT;
  if constexpr (!Q4 && CLS == C_H) {
    WTile<false> wh[2];
    load_wt<false>(p.head_w, 2 * (c.w - H_WG0), KS_D, 0, 2 * c.wave, c.lane, wh[0]);
    load_wt<false>(p.head_w, min(2 * (c.w - H_WG0) + 1, p.head_nt32 - 1), KS_D, 0, 2 * c.wave, c.lane, wh[1]);
    role_h<0, 1>(c, c.w - H_WG0, wh);
  }
  if constexpr (Q4 && (CLS == C_A || CLS == C_P)) {
    const int k = CLS == C_A ? c.w - A_WG0 : 64 + c.w - P4_WG0;
    if (p.head_w && k < 2 * p.head_tiles) {
      const int t = k % p.head_tiles, rt = k / p.head_tiles;
      WTile<false> wh[2];
      load_wt<false>(p.head_w, 2 * t, KS_D, 0, 2 * c.wave, c.lane, wh[0]);
      load_wt<false>(p.head_w, min(2 * t + 1, p.head_nt32 - 1), KS_D, 0, 2 * c.wave, c.lane, wh[1]);
      if (rt == 0) role_h<0, 1>(c, t, wh);
      else role_h<1, 2>(c, t, wh);
    }
  }
}

template <bool Q4>
__device__ __forceinline__ void step_kernel(const DecStepXsArgs& p) {
  constexpr int MT = Q4 ? 2 : 1, H_WG0 = A_WG0 + 32 * MT;
  static_assert(!Q4 || O1_WG0 + NDT <= NWG, "int4 roles fit the grid");
  static_assert(H_WG0 + 64 <= QB_WG0 || Q4, "bf16: head tiles and the second QKV K half apart");
  __shared__ __attribute__((aligned(16))) Lds L;
  Ctx c{p, L, (int)blockIdx.x, (int)threadIdx.x, (int)(threadIdx.x & 63), __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), 0u};
  c.ep = __hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (c.w < NQT) run_layers<Q4, C_Q>(c);
  else if (c.w < O_WG0 + NDT) run_layers<Q4, C_O>(c);
  else if (c.w < A_WG0 + 32 * MT) run_layers<Q4, C_A>(c);
  else if constexpr (Q4) {
    if (c.w < Q1_WG0 + NQT) run_layers<Q4, C_Q1>(c);
    else if (c.w < O1_WG0 + NDT) run_layers<Q4, C_O1>(c);
    else run_layers<Q4, C_P>(c);
  } else if (p.head_w && c.w < H_WG0 + p.head_tiles) run_layers<Q4, C_H>(c);
  else if (XSD_QSPLIT && c.w >= QB_WG0) run_layers<Q4, C_QB>(c);
  else run_layers<Q4, C_P>(c);
  if (p.sample && c.w < p.M) role_s(c);
  if (p.stamps && c.tid == 0) p.stamps[(size_t)c.w * DEC_XSD_STAMPS + DEC_XSD_STAMPS - 1] = __builtin_amdgcn_s_memrealtime();
  if (c.w == 0 && c.tid == 0) __hip_atomic_store(p.epoch, c.ep + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

__global__ __launch_bounds__(NT, 1) void dec_step_xs_kernel(DecStepXsArgs p) { step_kernel<false>(p); }
__global__ __launch_bounds__(NT, 1) void dec_step_xs_q4_kernel(DecStepXsArgs p) { step_kernel<true>(p); }

size_t dec_step_xs_ctrl_bytes() { return (size_t)CW_N * CW_STRIDE * 4; }

void launch_dec_step_xs(const DecStepXsArgs& p, hipStream_t st, bool q4) {
  if (q4) hipLaunchKernelGGL(dec_step_xs_q4_kernel, dim3(NWG), dim3(NT), 0, st, p);
  else hipLaunchKernelGGL(dec_step_xs_kernel, dim3(NWG), dim3(NT), 0, st, p);
}

const void* dec_step_xs_kernel_ptr(bool q4) {
  return q4 ? reinterpret_cast<const void*>(&dec_step_xs_q4_kernel) : reinterpret_cast<const void*>(&dec_step_xs_kernel);
}
