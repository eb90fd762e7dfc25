// Persistent batched depth-decoder step: the 4 decoder layers of one codebook step i >= 2 for up to 32
// utterance rows (/root/reference/csm_mlx/generation.py:72-89 at batch B: decoder(projection(E_a[c]))
// over the step's rows) in ONE launch, bf16 weights, matrix cores for every projection.
//
// Why: on the launch path (run_dec_xs) a step is ~20 dependent launches (QKV, attention, o_proj, gate/up,
// down per layer); at 32 rows each is latency-bound -- ramp, first weight loads, split-K combine, drain:
// ~44 us per layer for ~53 MB of MALL-resident weights (profiles/r05_prof_config4_per_frame_roles.txt).
// Here every CU keeps one workgroup for the step, owns fixed weight tiles of every projection and
// loads them into registers AHEAD of the hand-off that releases their activations, so the weight
// stream and the first-load latency sit under the dependency waits.
//
// Roles (NWG = 256 workgroups x 8 waves, w = blockIdx.x), per layer:
//   Q  w < 48        QKV tile w (32 of the 1536 rows), full K: x * n1 (split rows) -> RoPE, q | k | v
//                    rows + the K/V cache row at pos                              -> flag F1[w]
//   A  80 <= w < 112 attention of row m = w - 80, query head h = wave, keys 0..pos (the cached rows staged in
//                    LDS at the layer start; layer 0 takes q | k | v of the row's code from the folded
//                    table)                                                      -> flag F2[m]
//   O  48 <= w < 80  o_proj tile j = w - 48 (32 columns), full K: + residual -> x_o, x_o * n2 (split),
//                    row sums of squares                                         -> flag F3[j]
//   G  every w       gate/up tiles 2b, 2b + 1, b = 32 (w % 8) + w / 8 (the SiLU*up columns 32b..32b+31)
//                                                                                -> flag FH[w]
//   D  every w       down, output tile j = w / 8 over h columns 1024 g .. + 1023, g = w % 8 (the G
//                    workgroups of group g: the same XCD under round-robin placement, speed only)
//                    -> partial tile; arrival ticket C4[j]; the eighth arrival sums the 8 partials in group
//                    order + residual -> x_d, x_d * (next n1 | final norm) split, row sums of squares
//                                                                                -> flag F5[j]
// The head (audio_head[i - 1], its arg-max or sampler) stays a launch of its own after this one: it reads
// the split rows + sums of squares the last layer's combines wrote (engine's xs_D / xs_ss, 32 tiles).
//
// Hand-offs (MI355X_MICROARCH.md, inter-workgroup visibility, valid form "ONE lane of each storing
// workgroup ... sc1 flag store or agent-scope atomic add"): every payload byte is stored sc1 and loaded
// sc1; each storing wave drains (s_waitcnt vmcnt(0)) before the workgroup barrier behind which one lane
// stores the flag / adds to the counter; consumers poll with sc1 loads (one lane per flag), then a
// barrier.  Flags carry tag = epoch * 4 + layer + 1 and counters count monotonically from the epoch the
// launch read at its start (advanced by workgroup 0 at its end), so nothing is reset.  Every spin is
// bounded: on timeout a workgroup raises the error word and stops waiting (results garbage, the host
// raises) -- the grid always drains.  Single scratch buffers suffice: every rewrite of a buffer is
// ordered (through the hand-off chain) after every read of its previous contents.
//
// Arithmetic: the activations are fp32, split into three bf16 parts in registers (xs.h split_frag), so
// the matrix-core products are exact in fp32 and accumulate in fp32 (gemm_xs's arithmetic; summation
// order differs); RMSNorm folded as the streaming path's (x * norm weight split, row scale
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
constexpr int O_WG0 = NQT;       // o_proj workgroups 48 .. 79
constexpr int A_WG0 = O_WG0 + 32; // attention workgroups 80 .. 111 (row m = w - 80, wave = query head)
constexpr int H_WG0 = A_WG0 + 32; // head workgroups 112 .. (64 padded-vocabulary rows each)
constexpr unsigned SPIN_LIMIT = 1u << 22;
constexpr int SC1 = 16;  // buffer cache policy: sc1 (agent-coherent)
static_assert(NWG == 256 && NWV == 8, "roles assume 256 workgroups of 8 waves");
static_assert(KS_D == 2 * NWV && KS_F / NGRP == 2 * NWV, "every wave takes two K stages of its tile");

// control words (u32), one per 128-B line
enum { CW_F1 = 0, CW_F2 = CW_F1 + NQT, CW_F3 = CW_F2 + 32, CW_FH = CW_F3 + NDT, CW_C4 = CW_FH + NWG, CW_F5 = CW_C4 + NDT,
       CW_N = CW_F5 + NDT };
constexpr int CW_STRIDE = 32;

struct Lds {
  float red[NWV][2][16][64];  // the per-wave accumulators of up to two tiles
  float ct[2][32][33];     // reduced tiles [batch row][column]
  float rsp[8][32];        // row scales: partial sums of squares (row_scales)
  // attention workgroups (wave = query head): cached keys / values 0..pos-1 of both kv heads (rows padded:
  // conflict-free row-parallel reads), each wave's scaled query and the new key / value row at pos
  float Ks[HKV][32][HD + 4];
  float Vs[HKV][32][HD];
  float qsh[HQ][HD];
  float kn[HQ][HD];
  float vn[HQ][HD];
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
// lanes < n of wave 0 wait until word idx(lane) has reached `target` (flags hold tags, counters counts:
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
__device__ __forceinline__ void st16(void* base, size_t off, f32x4_t v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rsrc(base), (int)off, 0, SC1);
}
__device__ __forceinline__ f32x4_t ld16(const void* base, size_t off) {
  return __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), (int)off, 0, SC1));
}
// 4-B sc1 load as a plain buffer load (not an atomic: independent loads issue back to back)
__device__ __forceinline__ float ld4(const float* p) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc(p), 0, 0, SC1));
}
// (base wave-uniform -- it rides in the buffer descriptor; a per-lane base would make the compiler
// loop over the lanes' distinct descriptors -- and the lane's byte offset in the vector offset)
__device__ __forceinline__ float2 ld8(const float* base, int off) {
  return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rsrc(base), off, 0, SC1));
}
__device__ __forceinline__ void st4(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// ---- matrix-core tiles.  Weight tile registers: the wave's two K stages (st0, st0 + 1) of one 32-row
// tile of a fragment-tiled copy (gemm_retile: [tile][stage][s][lane] x 16 B); activation registers: the
// same stages of the 32 split rows (xs.h XS_F32 layout, row tile 0).
struct WT { u32x4_t a[2][4]; };
struct AF { u32x4_t a[2][4][2]; };

__device__ __forceinline__ void load_wt(const uint8_t* T, int tile, int nks, int st0, int lane, WT& r) {
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int s = 0; s < 4; ++s) r.a[q][s] = bload<0>(T, lane * 16, __builtin_amdgcn_readfirstlane(((tile * nks + st0 + q) * 4 + s) * 1024));
}
__device__ __forceinline__ void load_af(const void* X, int st0, int lane, AF& r) {
  const __amdgpu_buffer_rsrc_t rs = rsrc(X);
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
        r.a[q][s][hf] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, __builtin_amdgcn_readfirstlane((((st0 + q) * 4 + s) * 2 + hf) * 1024), SC1);
}
template <int NTL>
__device__ __forceinline__ void mma(const AF& A, const WT (&W)[NTL], f32x16_t (&acc)[NTL]) {
#pragma unroll
  for (int t = 0; t < NTL; ++t) acc[t] = f32x16_t{};
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      u32x4_t pt[3];
      xs::split_frag(A.a[q][s][0], A.a[q][s][1], pt);
#pragma unroll
      for (int pp = 0; pp < 3; ++pp)
#pragma unroll
        for (int t = 0; t < NTL; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, pt[pp]),
                                                          __builtin_bit_cast(bf16x8_t, W[t].a[q][s]), acc[t], 0, 0, 0);
    }
}
// the 8 waves' partial tiles -> L.ct[t][batch row][column], added in wave order.  Accumulator register
// j of lane (r, h): batch row (j & 3) + 8 (j >> 2) + 4 h, column r.
template <int NTL>
__device__ __forceinline__ void reduce_tiles(Ctx& c, const f32x16_t (&acc)[NTL]) {
#pragma unroll
  for (int t = 0; t < NTL; ++t)
#pragma unroll
    for (int j = 0; j < 16; ++j) c.L.red[c.wave][t][j][c.lane] = acc[t][j];
  __syncthreads();
#pragma unroll
  for (int e0 = 0; e0 < NTL * 1024; e0 += NT) {
    const int e = e0 + c.tid, t = e >> 10, m = (e >> 5) & 31, col = e & 31;
    const int j = (m & 3) + 4 * (m >> 3), ln = col + 32 * ((m >> 2) & 1);
    float v = c.L.red[0][t][j][ln];
#pragma unroll
    for (int wv = 1; wv < NWV; ++wv) v += c.L.red[wv][t][j][ln];
    c.L.ct[t][m][col] = v;
  }
  __syncthreads();
}

// Row scales rsqrt(sum_t ss[t][m] / D + eps) from 32 tiles' partial sums of squares (sc1): threads < 256
// each add 4 tiles of one row (loads in flight together) into L.rsp[part][row]; row_scale() adds the 8
// parts in order once a barrier (reduce_tiles') has published them
__device__ __forceinline__ void row_scales(Ctx& c, const float* ss, int stride) {
  if (c.tid < 256) {
    const int m = c.tid & 31, q = c.tid >> 5;
    const __amdgpu_buffer_rsrc_t rs = rsrc(ss);
    float v[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
      v[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (m + 4 * q * stride) * 4, t * stride * 4, SC1));
    c.L.rsp[q][m] = ((v[0] + v[1]) + v[2]) + v[3];
  }
}
__device__ __forceinline__ float row_scale(const Ctx& c, int m) {
  float s = c.L.rsp[0][m];
#pragma unroll
  for (int q = 1; q < 8; ++q) s += c.L.rsp[q][m];
  return rsqrtf(s / (float)D + c.p.eps);
}

// sum over the 8 lanes of a row group (lanes 8r .. 8r + 7), fixed butterfly order
__device__ __forceinline__ float sum8(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}

// ---------------------------------------------------------------------------------------------------
// Q: QKV tile T of layer l (l >= 1)
__device__ __forceinline__ void role_q(Ctx& c, int l, const WT& W) {
  const DecStepXsArgs& p = c.p;
  const int T = c.w;
  const unsigned tag = c.ep * NL + l;  // the previous layer's combine flags
  wait_words(c, NDT, [](int i) { return CW_F5 + i; }, tag);
  c.mark(1);
  AF A;
  load_af(p.xs_out, 2 * c.wave, c.lane, A);
  row_scales(c, p.ss_out, p.ss_stride);
  f32x16_t acc[1];
  mma<1>(A, reinterpret_cast<const WT(&)[1]>(W), acc);
  reduce_tiles<1>(c, acc);
  c.sub(0);
  // rows m = tid / 16, columns 2 (tid % 16) + {0, 1} (RoPE pairs)
  const int m = c.tid >> 4, cc = 2 * (c.tid & 15), n = 32 * T + cc;
  const float r = row_scale(c, m);
  float a = c.L.ct[0][m][cc] * r, b = c.L.ct[0][m][cc + 1] * r;
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
  c.sub(1);
  drain();
  __syncthreads();
  if (c.tid == 0) set_flag(c.cw(CW_F1 + T), tag + 1);
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
        float* dst = kv ? &c.L.Vs[g][r / (HD / 4)][4 * (r % (HD / 4))] : &c.L.Ks[g][r / (HD / 4)][4 * (r % (HD / 4))];
        *reinterpret_cast<f4*>(dst) = t[kv][u];
      }
    }
}

// A (workgroups A_WG0 .. A_WG0 + 31): attention of row m = w - A_WG0, query head h = wave, keys 0..pos ->
// xs_att (split rows of the o_proj).  The cached K / V rows are in LDS (stage_kv); each wave fetches its
// query and the new key / value row at pos (layer 0: of the row's code, from the folded table; else from
// the QKV tiles, after their flags) and computes.
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
      // q tiles 4h..4h+3, k tiles 32 + 4g.., v tiles 40 + 4g..
      if (lane < 12) {
        const int t = lane < 4 ? 4 * h + lane : (lane < 8 ? HQ * 4 + 4 * g + lane - 4 : (HQ + HKV) * 4 + 4 * g + lane - 8);
        const unsigned* a = c.cw(CW_F1 + t);
        __builtin_amdgcn_s_sleep(8);
        for (unsigned spin = 0; (int)(ld_cw(a) - tag) < 0; ++spin) {
          if (spin_fail(c, spin)) break;
          __builtin_amdgcn_s_sleep(2);
        }
      }
      // (the wave leaves the poll loop once every polling lane has matched)
      c.sub(8);
      const float* row = p.qkv + (size_t)m * QKV;
      qv = ld8(row, (h * HD + 2 * lane) * 4);
      kv2 = ld8(row, (HQ * HD + g * HD + 2 * lane) * 4);
      vv2 = ld8(row, ((HQ + HKV) * HD + g * HD + 2 * lane) * 4);
    }
    *reinterpret_cast<float2*>(&c.L.qsh[h][2 * lane]) = make_float2(qv.x * scale, qv.y * scale);
    *reinterpret_cast<float2*>(&c.L.kn[h][2 * lane]) = kv2;
    *reinterpret_cast<float2*>(&c.L.vn[h][2 * lane]) = vv2;
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
      const float* krow = kj < pos ? &c.L.Ks[g][kj][0] : &c.L.kn[h][0];
      const f4* kr = reinterpret_cast<const f4*>(krow + hh * (HD / 2));
      const f4* qr = reinterpret_cast<const f4*>(&c.L.qsh[h][hh * (HD / 2)]);
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
          vv[u] = *reinterpret_cast<const f4*>(jj < pos ? &c.L.Vs[g][jj][4 * dq] : &c.L.vn[h][4 * dq]);
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
    if (lane < 32)
      st16(p.xs_att, xs::off(D, m, h * HD + 4 * dq),
           f32x4_t{(acc.x + t0) * inv, (acc.y + t1) * inv, (acc.z + t2) * inv, (acc.w + t3) * inv});
  }
  drain();
  __syncthreads();
  // one flag per attention workgroup (rows past M publish without work)
  if (c.tid == 0) set_flag(c.cw(CW_F2 + m), tag);
  c.mark(4);
}

// O: o_proj tile j (+ residual) -> x_o, split x_o * n2, row sums of squares
__device__ __forceinline__ void role_o(Ctx& c, int l, const WT& W) {
  const DecStepXsArgs& p = c.p;
  const int j = c.w - O_WG0;
  const unsigned tag = c.ep * NL + l + 1;
  wait_words(c, 32, [](int i) { return CW_F2 + i; }, tag);
  c.mark(5);
  AF A;
  load_af(p.xs_att, 2 * c.wave, c.lane, A);
  // residual: layer 0 the projected input row proj_tab[code], else the previous layer's x_d
  const int m = c.tid >> 3, q = c.tid & 7, n = 32 * j + 4 * q;
  f32x4_t res = {0.f, 0.f, 0.f, 0.f};
  if (c.tid < 256 && m < p.M) {
    if (l == 0) {
      const int code = __hip_atomic_load(p.code_buf + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      res = *reinterpret_cast<const f32x4_t*>(p.proj_tab + (size_t)code * D + n);
    } else {
      res = ld16(p.x_d, ((size_t)m * D + n) * 4);
    }
  }
  const f32x4_t nw = *reinterpret_cast<const f32x4_t*>(p.n2[l] + n);
  f32x16_t acc[1];
  mma<1>(A, reinterpret_cast<const WT(&)[1]>(W), acc);
  reduce_tiles<1>(c, acc);
  c.sub(6);
  if (c.tid < 256) {
    f32x4_t x = {0.f, 0.f, 0.f, 0.f};
    if (m < p.M) x = res + f32x4_t{c.L.ct[0][m][4 * q], c.L.ct[0][m][4 * q + 1], c.L.ct[0][m][4 * q + 2], c.L.ct[0][m][4 * q + 3]};
    st16(p.x_o, ((size_t)m * D + n) * 4, x);
    st16(p.xs_x, xs::off(D, m, n), x * nw);
    const float sq = sum8(fmaf(x.w, x.w, fmaf(x.z, x.z, fmaf(x.y, x.y, x.x * x.x))));
    if (q == 0) st4(p.ss_o + (size_t)j * 32 + m, sq);
  }
  drain();
  __syncthreads();
  if (c.tid == 0) set_flag(c.cw(CW_F3 + j), tag);
  c.mark(6);
}

// G: gate/up tiles 2b, 2b + 1 -> SiLU*up columns 32b .. 32b + 31 (split, K = F)
__device__ __forceinline__ void role_g(Ctx& c, int l, const WT (&W)[2]) {
  const DecStepXsArgs& p = c.p;
  const int b = 32 * (c.w & 7) + (c.w >> 3);
  const unsigned tag = c.ep * NL + l + 1;
  wait_words(c, NDT, [](int i) { return CW_F3 + i; }, tag);
  c.mark(7);
  AF A;
  load_af(p.xs_x, 2 * c.wave, c.lane, A);
  row_scales(c, p.ss_o, 32);
  f32x16_t acc[2];
  mma<2>(A, W, acc);
  c.sub(2);
  reduce_tiles<2>(c, acc);
  c.sub(3);
  if (c.tid < 256) {
    const int m = c.tid >> 3, q = c.tid & 7;
    const float r = row_scale(c, m);
    float hv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pc = 4 * q + i, t = pc >> 4, cc = 2 * (pc & 15);  // wgu rows interleave gate_j, up_j
      const float gt = c.L.ct[t][m][cc] * r, up = c.L.ct[t][m][cc + 1] * r;
      hv[i] = silu_f(gt) * up;
    }
    st16(p.xs_h, xs::off(F, m, 32 * b + 4 * q), f32x4_t{hv[0], hv[1], hv[2], hv[3]});
  }
  c.sub(4);
  drain();
  __syncthreads();
  if (c.tid == 0) set_flag(c.cw(CW_FH + c.w), tag);
  c.mark(8);
}

// D: down tile j over K group g -> partial; the eighth arrival combines
__device__ __forceinline__ void role_d(Ctx& c, int l, const WT& W) {
  const DecStepXsArgs& p = c.p;
  const int g = c.w & 7, j = c.w >> 3;
  const unsigned tag = c.ep * NL + l + 1;
  wait_words(c, 32, [g](int i) { return CW_FH + g + 8 * i; }, tag);  // the G workgroups of group g
  c.mark(9);
  AF A;
  load_af(p.xs_h, 16 * g + 2 * c.wave, c.lane, A);
  f32x16_t acc[1];
  mma<1>(A, reinterpret_cast<const WT(&)[1]>(W), acc);
  reduce_tiles<1>(c, acc);
  c.sub(5);
  const int m = c.tid >> 3, q = c.tid & 7, n = 32 * j + 4 * q;
  if (c.tid < 256)
    st16(p.dpart, (((size_t)g * 32 + m) * D + n) * 4,
         f32x4_t{c.L.ct[0][m][4 * q], c.L.ct[0][m][4 * q + 1], c.L.ct[0][m][4 * q + 2], c.L.ct[0][m][4 * q + 3]});
  drain();
  __syncthreads();
  if (c.tid == 0) c.L.flag = add_ctr(c.cw(CW_C4 + j)) + 1u == tag * NGRP;
  __syncthreads();
  c.mark(10);
  if (!c.L.flag) return;
  // combine (the last of the tile's 8 groups): x_d = x_o + sum_g partial_g, split with the next norm
  const float* nwp = l + 1 < NL ? p.n1[l + 1] : p.norm;
  if (c.tid < 256) {
    f32x4_t pp[NGRP];
#pragma unroll
    for (int gg = 0; gg < NGRP; ++gg) pp[gg] = ld16(p.dpart, (((size_t)gg * 32 + m) * D + n) * 4);
    const f32x4_t xo = ld16(p.x_o, ((size_t)m * D + n) * 4);
    const f32x4_t nw = *reinterpret_cast<const f32x4_t*>(nwp + n);
    f32x4_t s = pp[0];
#pragma unroll
    for (int gg = 1; gg < NGRP; ++gg) s += pp[gg];
    f32x4_t x = {0.f, 0.f, 0.f, 0.f};
    if (m < p.M) x = xo + s;
    st16(p.x_d, ((size_t)m * D + n) * 4, x);
    st16(p.xs_out, xs::off(D, m, n), x * nw);
    const float sq = sum8(fmaf(x.w, x.w, fmaf(x.z, x.z, fmaf(x.y, x.y, x.x * x.x))));
    if (q == 0) st4(p.ss_out + (size_t)j * p.ss_stride + m, sq);
  }
  drain();
  __syncthreads();
  if (c.tid == 0) set_flag(c.cw(CW_F5 + j), tag);
  c.mark(11);
}

// H: audio_head[step - 1] rows 64 t .. 64 t + 63 (two 32-row tiles) of the final-normed rows (the last
// combines' split x * norm + sums of squares) -> logits [row][Vp] and the tile's arg-max partial per row
// (pack_argmax: the largest logit, the first index on ties), exactly the partial layout of the launch
// path's head (gemm_xs EPI_ARGMAX, 64-row tiles), which the next step / advance_kernel reduce
__device__ __forceinline__ void role_h(Ctx& c, const WT (&W)[2]) {
  const DecStepXsArgs& p = c.p;
  const int t = c.w - H_WG0;
  const unsigned tag = c.ep * NL + NL;  // the last layer's combine flags
  wait_words(c, NDT, [](int i) { return CW_F5 + i; }, tag);
  AF A;
  load_af(p.xs_out, 2 * c.wave, c.lane, A);
  row_scales(c, p.ss_out, p.ss_stride);
  f32x16_t acc[2];
  mma<2>(A, W, acc);
  reduce_tiles<2>(c, acc);
  // row m = tid / 16, columns 4 (tid % 16) .. + 3 of the 64
  const int m = c.tid >> 4, c4 = 4 * (c.tid & 15), n = 64 * t + c4;
  const float r = row_scale(c, m);
  unsigned long long best = 0;
  if (m < p.M && n < p.Vp) {
    const float4 v = make_float4(c.L.ct[c4 >> 5][m][c4 & 31] * r, c.L.ct[c4 >> 5][m][(c4 & 31) + 1] * r,
                                 c.L.ct[c4 >> 5][m][(c4 & 31) + 2] * r, c.L.ct[c4 >> 5][m][(c4 & 31) + 3] * r);
    *reinterpret_cast<float4*>(p.head_out + (size_t)m * p.Vp + n) = v;
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
  if (m < p.M && (c.tid & 15) == 0) p.head_part[(size_t)m * p.part_stride + t] = best;
}

// The layer loop of one workgroup class (each its own straight-line code: exact register liveness per
// class, no merged paths holding another class's prefetch registers).  CLS: 0 QKV, 1 o_proj,
// 2 attention, 3 head (+ plain), 4 plain (gate/up + down only).
enum { C_Q = 0, C_O = 1, C_A = 2, C_H = 3, C_P = 4 };
template <int CLS>
__device__ __forceinline__ void run_layers(Ctx& c) {
  static_assert(CLS >= C_Q && CLS <= C_P, "workgroup class");
  const DecStepXsArgs& p = c.p;
  const int b = 32 * (c.w & 7) + (c.w >> 3), g = c.w & 7, j = c.w >> 3;
  WT wq, wgu[2], wd;
  // vmcnt retires in issue order and every publish drains it: a prefetch issued just before a hand-off
  // poll or a latency-critical operand load holds that back, so each class issues its next tiles after
  // its own latency-critical steps (Q, A: after their publish)
  // the plain and head classes (the most registers to spare) fetch their down tile with gate/up: a load
  // issued just before the h hand-off's poll would hold the poll back (vmcnt order)
  constexpr bool WD_EARLY = CLS == C_P || CLS == C_H;
  auto ld_gu = [&](int l) {
    load_wt(p.wgu[l], 2 * b, KS_D, 2 * c.wave, c.lane, wgu[0]);
    load_wt(p.wgu[l], 2 * b + 1, KS_D, 2 * c.wave, c.lane, wgu[1]);
    if constexpr (WD_EARLY) load_wt(p.wd[l], j, KS_F, 16 * g + 2 * c.wave, c.lane, wd);
  };
  if constexpr (CLS == C_Q) load_wt(p.wqkv[1], c.w, KS_D, 2 * c.wave, c.lane, wq);
  if constexpr (CLS == C_O) load_wt(p.wo[0], c.w - O_WG0, KS_D, 2 * c.wave, c.lane, wq);
  if constexpr (CLS != C_A) ld_gu(0);
  for (int l = 0; l < NL; ++l) {
    c.l = l;
    c.mark(0);
    if constexpr (CLS == C_O || CLS == C_H || CLS == C_P) {
      if (l > 0) {
        if constexpr (CLS == C_O) load_wt(p.wo[l], c.w - O_WG0, KS_D, 2 * c.wave, c.lane, wq);
        ld_gu(l);
      }
    }
    if constexpr (CLS == C_Q) {
      if (l > 0) {
        role_q(c, l, wq);
        ld_gu(l);
      }
    }
    if constexpr (CLS == C_A) {
      stage_kv(c, l);  // (role_a's barrier publishes the LDS rows)
      role_a(c, l);
      ld_gu(l);
    }
    if constexpr (CLS == C_O) role_o(c, l, wq);
    role_g(c, l, wgu);
    if constexpr (!WD_EARLY) load_wt(p.wd[l], j, KS_F, 16 * g + 2 * c.wave, c.lane, wd);  // during the h hand-off
    role_d(c, l, wd);
    // the next layer's QKV tile: during the combine the Q hand-off waits for
    if constexpr (CLS == C_Q) {
      if (l > 0 && l + 1 < NL) load_wt(p.wqkv[l + 1], c.w, KS_D, 2 * c.wave, c.lane, wq);
    }
  }
  if constexpr (CLS == C_H) {  // (a 32-row tile past the last is clamped: its columns are never stored)
    load_wt(p.head_w, 2 * (c.w - H_WG0), KS_D, 2 * c.wave, c.lane, wgu[0]);
    load_wt(p.head_w, min(2 * (c.w - H_WG0) + 1, p.head_nt32 - 1), KS_D, 2 * c.wave, c.lane, wgu[1]);
    role_h(c, wgu);
  }
}

}  // namespace

__global__ __launch_bounds__(NT, 1) void dec_step_xs_kernel(DecStepXsArgs p) {
  __shared__ __attribute__((aligned(16))) Lds L;
  Ctx c{p, L, (int)blockIdx.x, (int)threadIdx.x, (int)(threadIdx.x & 63), __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), 0u};
  c.ep = __hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (c.w < NQT) run_layers<C_Q>(c);
  else if (c.w < O_WG0 + NDT) run_layers<C_O>(c);
  else if (c.w < A_WG0 + 32) run_layers<C_A>(c);
  else if (p.head_w && c.w < H_WG0 + p.head_tiles) run_layers<C_H>(c);
  else run_layers<C_P>(c);
  if (p.stamps && c.tid == 0) p.stamps[(size_t)c.w * DEC_XSD_STAMPS + DEC_XSD_STAMPS - 1] = __builtin_amdgcn_s_memrealtime();
  if (c.w == 0 && c.tid == 0) __hip_atomic_store(p.epoch, c.ep + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

size_t dec_step_xs_ctrl_bytes() { return (size_t)CW_N * CW_STRIDE * 4; }

void launch_dec_step_xs(const DecStepXsArgs& p, hipStream_t st) {
  hipLaunchKernelGGL(dec_step_xs_kernel, dim3(NWG), dim3(NT), 0, st, p);
}

const void* dec_step_xs_kernel_ptr() { return reinterpret_cast<const void*>(&dec_step_xs_kernel); }
