// Persistent backbone step: the 16 Llama blocks of csm_1b's backbone for one decode row (batch 1,
// bf16 weights) plus the final RMSNorm -> h_last, in ONE launch (/root/reference/csm_mlx/models.py:
// 50-51 + generation.py:32-42: self.backbone(h, mask, cache) then norm(h[:, -1])).
//
// Why: at batch 1 the backbone is 16 x 5 dependent launches (QKV, attention, o_proj, gate/up, down);
// each pays a kernel boundary plus its own ramp and drain around a 8-67 MB weight stream.  Here every
// CU keeps one workgroup for the whole step, owns a fixed slice of every matrix and streams it into
// registers ahead of the hand-off that releases its input (the same machinery as dec_frame.hip).
//
// Work split (NWG = 256 workgroups = one per CU, 512 threads = 8 waves each), per layer:
//   QKV     3072 rows: 12 per WG (RoPE pairs stay inside a WG; k / v rows appended to the cache)
//                                                              -> q | k | v granules      (E1)
//   attention: WG a < 32 = query head a (group a / 4): gathers q_a, k_g, v_g (192 granules), keys
//           < pos from the cache, key pos from the granules; 8 waves x 64-key blocks, online softmax,
//           waves combined in fixed order                        -> att granules            (E2)
//   o_proj  2048 rows: 8 per WG, + residual                      -> x granules              (E3)
//   gate/up 16384 interleaved rows: 64 per WG (8 per wave) -> 32 SiLU*up columns
//   down    split-K over those 32 columns (chunk-major copy [F/8][D][8]) -> 2048 partials     (E4)
//           WG w sums rows 8w..8w+7 of every producer in a fixed order, + residual -> x       (E5)
// Five hand-offs per layer; after the last layer every WG holds x, WG 0 writes h_last.
//
// Arithmetic: fp32 accumulation of bf16 weights x fp32 activations, RMSNorm as the oracle
// (x * rsqrt(mean(x^2) + eps) * w), RoPE on interleaved pairs (attention.py:157-177, the engine's
// EPI_QKV convention), softmax with max subtraction, every reduction in a fixed order
// (deterministic run to run; summation order differs from the launch path's GEMVs).
#include <type_traits>

#include "csm_kernels.h"
#include "handoff.h"

namespace {

using namespace handoff;

constexpr int NWG = BB_STEP_WGS, NT = BB_STEP_THREADS;
constexpr int D = 2048, F = 8192, HQ = 32, HKV = 8, HD = 64, NL = BB_STEP_LAYERS;
constexpr int QKV = (HQ + 2 * HKV) * HD;  // 3072
constexpr int NATT = HQ;                  // attention workgroups: one per query head
constexpr unsigned SPIN_LIMIT = 1u << 22; // ~0.1 s of s_sleep per hand-off before declaring failure

// granule regions (u64 offsets), double-buffered by hand-off parity.  The all-gather regions (E2,
// E3, E5: every workgroup reads every granule) are written in REP replicas, workgroup w reading
// replica w % REP (dec_frame.hip: fewer readers per granule; speed only, never correctness).
// Measured: 581-584 us (REP 1 / 8) -> 569 us (REP 4) per row (profiles/r03_ab_replicas.txt).
#ifndef BB_REP
#define BB_REP 4
#endif
constexpr int REP = BB_REP;
__host__ __device__ constexpr size_t rs_of(size_t per) { return (per + 511) / 512 * 512 + 32; }
constexpr size_t G_QKV = 0;                                   // [2][QKV]
constexpr size_t G_ATT = G_QKV + 2 * QKV;                     // [2][REP][rs(D)]
constexpr size_t G_X = G_ATT + 2 * REP * rs_of(D);            // [2][REP][rs(D)]
constexpr size_t G_PART = G_X + 2 * REP * rs_of(D);           // [2][NWG][D]
constexpr size_t G_TOTAL = G_PART + (size_t)2 * NWG * D;

struct Lds {
  float x[D];            // residual
  float xn[D];           // normed projection input
  float att[D];          // attention output (o_proj input)
  float red[8][NWG];     // reduce-scatter staging [row][producer]
  float wsum[8][8];      // per-wave partial dots
  float sq[8];           // per-wave partial sums of squares of the gathered x (folded RMSNorm)
  alignas(16) float hb[32];  // this WG's SiLU*up columns
  float2 rope[HD / 2];   // (cos, sin) at the step's position
  float q[HD], kn[HD], vn[HD];          // attention WGs: the head's q and the new k / v row
  float am[8], al[8], ao[8][HD];        // attention WGs: per-wave online-softmax partials
  float Ks[128][HD + 4], Vs[128][HD];   // attention WGs: one pass of 128 keys (K rows padded)
  // int4 kernel (bb_step_q4_kernel): projection inputs in the padded half-group layout (handoff.h q4p)
  // with their half-group sums: x * norm weight (QKV / gate-up input) and the attention output (o_proj)
  alignas(16) float xq[D / 32][36];
  float xh[D / 32];
  alignas(16) float aq[D / 32][36];
  float ah[D / 32];
};

struct Ctx {
  const BbStepArgs& p;
  Lds& L;
  int w, tid, lane, wave;
  unsigned tag0;
  int e;  // hand-off counter
  __device__ void refresh() {
    tid = opaque_tid();
    lane = tid & 63;
    wave = tid >> 6;
  }
  __device__ unsigned tag() const { return tag0 + (unsigned)e; }
  __device__ u64* buf(size_t region, size_t per) const { return p.gbuf + region + (size_t)(e & 1) * per; }
  // replicated all-gather regions: this workgroup's replica (reads), and a store to every replica
  __device__ u64* rbuf(size_t region, size_t per) const {
    return p.gbuf + region + ((size_t)(e & 1) * REP + (size_t)(w % REP)) * rs_of(per);
  }
  // one replica r of granule i (publishing lanes spread over the replicas: one store each)
  __device__ void put(size_t region, size_t per, size_t i, float v, int r) const {
    gput(p.gbuf + region + ((size_t)(e & 1) * REP + (size_t)r) * rs_of(per) + i, v, tag());
  }
  // profiling: the 100 MHz real-time clock when this WG passed hand-off e (slot e + 1; slot 0 = start)
  __device__ void stamp(int slot) const {
    if (p.stamps && tid == 0 && slot < BB_STEP_STAMPS) p.stamps[(size_t)w * BB_STEP_STAMPS + slot] = __builtin_amdgcn_s_memrealtime();
  }
};

// BB_PROBE_DELAY: sleeps before the first probe of a hand-off wait (the producers are still working
// when a workgroup starts waiting; an early probe returns stale and its re-polls load the lines every
// workgroup polls -- dec_frame.hip measured -6 % per frame from the same delay).
#ifndef BB_PROBE_DELAY
#define BB_PROBE_DELAY 32
#endif
// BB_DELAY_E2: the E2 wait of the 224 workgroups that run no attention (they wait the whole attention)
#ifndef BB_ATTN_LATE_PF
#define BB_ATTN_LATE_PF 0
#endif
#ifndef BB_EARLY_MQ2
#define BB_EARLY_MQ2 1
#endif
#ifndef BB_DELAY_E2
#define BB_DELAY_E2 BB_PROBE_DELAY
#endif
template <int DELAY = BB_PROBE_DELAY>
__device__ __forceinline__ void probe_delay() {
  if (DELAY > 0) __builtin_amdgcn_s_sleep(DELAY);
}
__device__ __forceinline__ bool spin_fail(Ctx& c, unsigned spin) {
  if (spin >= SPIN_LIMIT || ((spin & 255) == 255 && __hip_atomic_load(c.p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
    __hip_atomic_store(c.p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  return false;
}

// Wait until granules [0, n) of buf carry this hand-off's tag; values -> out (LDS).
template <int GPT, int DELAY = BB_PROBE_DELAY>
__device__ __forceinline__ void gather(Ctx& c, const u64* buf, int n, float* out) {
#if BB_PAIR16
  // granule pairs 2t + D/2 h (n == D: every pair whole)
  const unsigned tag = c.tag();
  const int poff[GPT / 2] = {2 * c.tid, D / 2 + 2 * c.tid};
  poll_pairs<GPT / 2, DELAY, 1>(buf, 0x7fffffff, poff, tag, [&](unsigned spin) { return spin_fail(c, spin); },
                                [&](const u32x4_t (&g)[GPT / 2]) {
#pragma unroll
    for (int h = 0; h < GPT / 2; ++h)
      *reinterpret_cast<float2*>(&out[poff[h]]) = make_float2(__uint_as_float(g[h].x), __uint_as_float(g[h].z));
  });
  c.stamp(c.e + 1);
  __syncthreads();
  (void)n;
#else
  const unsigned tag = c.tag();
  u64 g[GPT];
  probe_delay<DELAY>();
#pragma unroll
  for (int u = 0; u < GPT; ++u) {
    const int i = c.tid + u * NT;
    g[u] = i < n ? gload(buf + i) : ((u64)tag << 32);
  }
  for (unsigned spin = 0;; ++spin) {
    bool ok = true;
#pragma unroll
    for (int u = 0; u < GPT; ++u) ok &= (unsigned)(g[u] >> 32) == tag;
    if (ok || spin_fail(c, spin)) break;
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int u = 0; u < GPT; ++u) {
      const int i = c.tid + u * NT;
      if (i < n && (unsigned)(g[u] >> 32) != tag) g[u] = gload(buf + i);
    }
  }
  c.stamp(c.e + 1);
#pragma unroll
  for (int u = 0; u < GPT; ++u) {
    const int i = c.tid + u * NT;
    if (i < n) out[i] = __uint_as_float((unsigned)g[u]);
  }
  __syncthreads();
#endif
}

// BB_PAIR16 (as dec_frame.hip DF_PAIR16): the x / attention-output hand-offs and the down partials
// polled as granule pairs, one 16-B load each; thread t then owns elements 2t, 2t + 1, 1024 + 2t,
// 1024 + 2t + 1 of a row (else t + 512 j)
#ifndef BB_PAIR16
#define BB_PAIR16 1
#endif
// BB_E4_16: each thread's down rows are el(k) and its partials go out two granules per 16-B store
#ifndef BB_E4_16
#define BB_E4_16 0
#endif
__device__ __forceinline__ int el(const Ctx& c, int j) {
  return BB_PAIR16 ? (j >> 1) * (D / 2) + 2 * c.tid + (j & 1) : c.tid + j * NT;
}
// xn[k] = x[k] * rsqrt(mean(x^2) + eps) * nw[k]; nw elements el(j) fetched a phase ahead
struct Nw { float v[D / NT]; };
__device__ __forceinline__ Nw nw_fetch(const Ctx& c, const float* nw) {
  Nw r;
#pragma unroll
  for (int j = 0; j < D / NT; ++j) r.v[j] = nw[el(c, j)];
  return r;
}
__device__ __forceinline__ void rms(Ctx& c, const Nw& nw, float* out) {
  if (c.wave == 0) {  // sum of squares in a fixed order
    float s = 0.f;
#pragma unroll 8
    for (int k = c.lane; k < D; k += 64) s = fmaf(c.L.x[k], c.L.x[k], s);
    s = wave_sum(s);
    if (c.lane == 0) c.L.wsum[0][0] = s;
  }
  __syncthreads();
  const float r = rsqrtf(c.L.wsum[0][0] / (float)D + c.p.eps);
#pragma unroll
  for (int j = 0; j < D / NT; ++j) out[el(c, j)] = c.L.x[el(c, j)] * r * nw.v[j];
  __syncthreads();
}

// Folded RMSNorm (BB_FOLD, as dec_frame.hip): an x hand-off is gathered into x and xn = x * nw (the
// next consumer's norm weight) with per-wave sums of squares; consumers dot against the
// un-normalised xn and scale by rsqrt(mean(x^2) + eps) -- one barrier and one serial pass fewer.
#ifndef BB_FOLD
#define BB_FOLD 1
#endif
__device__ __forceinline__ void gather_x(Ctx& c, const u64* buf, const Nw& nw) {
  constexpr int GPT = D / NT;
  const unsigned tag = c.tag();
  float sq = 0.f;
#if BB_PAIR16
  const int poff[GPT / 2] = {2 * c.tid, D / 2 + 2 * c.tid};
  poll_pairs<GPT / 2, BB_PROBE_DELAY, 1>(buf, 0x7fffffff, poff, tag, [&](unsigned spin) { return spin_fail(c, spin); },
                                         [&](const u32x4_t (&g)[GPT / 2]) {
#pragma unroll
    for (int h = 0; h < GPT / 2; ++h) {
      const float v0 = __uint_as_float(g[h].x), v1 = __uint_as_float(g[h].z);
      *reinterpret_cast<float2*>(&c.L.x[poff[h]]) = make_float2(v0, v1);
      *reinterpret_cast<float2*>(&c.L.xn[poff[h]]) = make_float2(v0 * nw.v[2 * h], v1 * nw.v[2 * h + 1]);
      sq = fmaf(v0, v0, sq);
      sq = fmaf(v1, v1, sq);
    }
  });
  c.stamp(c.e + 1);
#else
  u64 g[GPT];
  probe_delay();
#pragma unroll
  for (int u = 0; u < GPT; ++u) g[u] = gload(buf + c.tid + u * NT);
  for (unsigned spin = 0;; ++spin) {
    bool ok = true;
#pragma unroll
    for (int u = 0; u < GPT; ++u) ok &= (unsigned)(g[u] >> 32) == tag;
    if (ok || spin_fail(c, spin)) break;
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int u = 0; u < GPT; ++u)
      if ((unsigned)(g[u] >> 32) != tag) g[u] = gload(buf + c.tid + u * NT);
  }
  c.stamp(c.e + 1);
#pragma unroll
  for (int u = 0; u < GPT; ++u) {
    const float v = __uint_as_float((unsigned)g[u]);
    c.L.x[c.tid + u * NT] = v;
    c.L.xn[c.tid + u * NT] = v * nw.v[u];
    sq = fmaf(v, v, sq);
  }
#endif
  sq = wave_sum(sq);
  if (c.lane == 0) c.L.sq[c.wave] = sq;
  __syncthreads();
}
__device__ __forceinline__ float row_rs(const Ctx& c) {
  float s = c.L.sq[0];
#pragma unroll
  for (int w = 1; w < 8; ++w) s += c.L.sq[w];
  return rsqrtf(s / (float)D + c.p.eps);
}

// ---- weight slices held in registers
// QKV / o_proj: thread (half h = tid >> 8, chunk c = tid & 255) holds chunk c of rows 6h+i / 4h+i
struct WQ { u32x4_t a[6]; };
struct WO { u32x4_t a[4]; };
// MLP quarter Q (of the WG's 64 gate/up rows and 4 down column chunks): wave v holds gate/up rows
// 16Q + 2v, 16Q + 2v + 1 (one gate/up pair -> SiLU*up column 8Q + v), chunks lane + 64 j (j < 4);
// thread t holds down rows t + 512 k (k < 4) of column chunk 4w + Q (8 columns)
struct WMq { u32x4_t g[2][4]; u32x4_t d[4]; };

__device__ __forceinline__ void load_q(Ctx& c, int l, WQ& r) {
  const bf16_t* base = c.p.wqkv[l] + (size_t)(12 * c.w + 6 * (c.tid >> 8)) * D;
  const int v = (c.tid & 255) * 16;
#pragma unroll
  for (int i = 0; i < 6; ++i) r.a[i] = bload<2>(base, v, i * D * 2);
}
__device__ __forceinline__ void load_o(Ctx& c, int l, WO& r) {
  const bf16_t* base = c.p.wo[l] + (size_t)(8 * c.w + 4 * (c.tid >> 8)) * D;
  const int v = (c.tid & 255) * 16;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.a[i] = bload<2>(base, v, i * D * 2);
}
__device__ __forceinline__ void load_mq(Ctx& c, int l, int Q, WMq& r) {
  const bf16_t* g = c.p.wgu[l] + (size_t)(64 * c.w + 16 * Q + 2 * c.wave) * D;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) r.g[i][j] = bload<2>(g, c.lane * 16, i * D * 2 + j * 64 * 16);
  // chunk 4w + Q of [F/8][D][8]: row n at byte (n * 8) * 2
  const bf16_t* d = c.p.wdc[l] + (size_t)(4 * c.w + Q) * D * 8;
#pragma unroll
  for (int k = 0; k < 4; ++k)  // rows el(k): 2t + (k & 1) + 1024 (k >> 1) with BB_E4_16, else t + 512 k
    r.d[k] = BB_E4_16 ? bload<2>(d, c.tid * 32, ((k >> 1) * (D / 2) + (k & 1)) * 16) : bload<2>(d, c.tid * 16, k * NT * 8 * 2);
}

// per-row partial sums of a (half, chunk)-split projection: wave partials -> wsum[wave][i]
template <int R>
__device__ __forceinline__ void rows_reduce(Ctx& c, float (&s)[R]) {
#pragma unroll
  for (int i = 0; i < R; ++i) s[i] = wave_sum(s[i]);
  if (c.lane == 0) {
#pragma unroll
    for (int i = 0; i < R; ++i) c.L.wsum[c.wave][i] = s[i];
  }
  __syncthreads();
}
// row i of half h: waves 4h..4h+3 in order
__device__ __forceinline__ float row_total(const Ctx& c, int h, int i) {
  return ((c.L.wsum[4 * h][i] + c.L.wsum[4 * h + 1][i]) + c.L.wsum[4 * h + 2][i]) + c.L.wsum[4 * h + 3][i];
}

// QKV rows 12w.. (RoPE at pos), published to E1; k / v rows also appended to the cache at pos
__device__ __forceinline__ void phase_qkv(Ctx& c, int l, int pos, const WQ& W, bool sc) {
  float s[6];
  const float* xc = c.L.xn + 8 * (c.tid & 255);
#pragma unroll
  for (int i = 0; i < 6; ++i) s[i] = dot8(W.a[i], xc);
  rows_reduce<6>(c, s);
  if (c.tid < 6) {  // pair j: rows n, n + 1 of half h
    const int h = c.tid / 3, i0 = 2 * (c.tid % 3), n = 12 * c.w + 6 * h + i0;
    float a = row_total(c, h, i0), b = row_total(c, h, i0 + 1);
    if (sc) {  // folded RMSNorm: the row scale after the dot product
      const float rs = row_rs(c);
      a *= rs;
      b *= rs;
    }
    if (n < (HQ + HKV) * HD) {
      const float2 cs = c.L.rope[(n % HD) / 2];
      const float y0 = a * cs.x - b * cs.y, y1 = b * cs.x + a * cs.y;
      a = y0;
      b = y1;
    }
    u64* g = c.buf(G_QKV, QKV);
    gput(g + n, a, c.tag());
    gput(g + n + 1, b, c.tag());
    if (n >= HQ * HD) {  // KVCache.update_and_fetch: the new row at pos (read by later launches)
      const int nn = n < (HQ + HKV) * HD ? n - HQ * HD : n - (HQ + HKV) * HD;
      float* cache = n < (HQ + HKV) * HD ? c.p.kc[l] : c.p.vc[l];
      *reinterpret_cast<float2*>(cache + ((size_t)(nn / HD) * c.p.S_cap + pos) * HD + nn % HD) = make_float2(a, b);
    }
  }
}

// Attention of query head a (WG a < NATT) over keys 0..pos: keys < pos from the cache (written by
// earlier launches), key pos from the E1 granules.  Wave v takes 64-key blocks v, v + 8, ...: lane j
// scores key 64 b + j (q . k over 64 dims, four fixed FMA chains), online softmax per wave, P.V with
// lane = head dim over the block's keys in order; waves combined in order 0..7 -> E2.
struct KvPass { float4 kv[4], vv[4]; };  // one 128-key pass of K / V rows in flight

// K / V rows k0 .. k0 + 127 of the pass (keys < pos from the cache, key pos from the E1 granules)
__device__ __forceinline__ void kv_pass_load(const Ctx& c, const float* K, const float* V, int pos, int k0, KvPass& kp) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = c.tid + NT * u, r = idx >> 4, c4 = idx & 15, j = k0 + r;
    const float4* ks = reinterpret_cast<const float4*>(j < pos ? K + (size_t)j * HD : c.L.kn);
    const float4* vs = reinterpret_cast<const float4*>(j < pos ? V + (size_t)j * HD : c.L.vn);
    kp.kv[u] = j <= pos ? ks[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
    kp.vv[u] = j <= pos ? vs[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// Attention of query head a (WG a < NATT), in two parts so the caller can issue its weight prefetch
// between them (BB_ATTN_LATE_PF: after the E1 poll and the first pass's K / V loads, so neither
// queues behind it):
// attn_begin: the E1 wait (q_a, k_g, v_g) and the first pass's K / V loads.
__device__ __forceinline__ void attn_begin(Ctx& c, int l, int pos, KvPass& kp) {
  const int a = c.w, g = a / (HQ / HKV);
  {  // E1 (the hand-off before c.e): q_a, k_g, v_g
    const u64* buf = c.p.gbuf + G_QKV + (size_t)((c.e - 1) & 1) * QKV;
    const unsigned tag = c.tag() - 1u;
    if (c.tid < 3 * HD) {
      const int part = c.tid / HD, d = c.tid % HD;
      const int idx = part == 0 ? a * HD + d : (part == 1 ? HQ * HD + g * HD + d : (HQ + HKV) * HD + g * HD + d);
      probe_delay();
      u64 v = gload(buf + idx);
      for (unsigned spin = 0; (unsigned)(v >> 32) != tag; ++spin) {
        if (spin_fail(c, spin)) break;
        __builtin_amdgcn_s_sleep(1);
        v = gload(buf + idx);
      }
      const float f = __uint_as_float((unsigned)v);
      if (part == 0) c.L.q[d] = f * 0.125f;  // 1 / sqrt(64)
      else if (part == 1) c.L.kn[d] = f;
      else c.L.vn[d] = f;
    }
    __syncthreads();
    c.stamp(c.e);  // E1 (index e - 1) passed
  }
  kv_pass_load(c, c.p.kc[l] + (size_t)g * c.p.S_cap * HD, c.p.vc[l] + (size_t)g * c.p.S_cap * HD, pos, 0, kp);
}

// attn_rest: keys 0..pos over 8 waves x 64-key blocks (wave v takes blocks v, v + 8, ...), online
// softmax per wave, waves combined in order 0..7 -> E2.
__device__ __forceinline__ void attn_rest(Ctx& c, int l, int pos, KvPass& kp) {
  const int a = c.w, g = a / (HQ / HKV);
  const float* K = c.p.kc[l] + (size_t)g * c.p.S_cap * HD;
  const float* V = c.p.vc[l] + (size_t)g * c.p.S_cap * HD;
  const int n = pos + 1;
  float m_run = -INFINITY, l_run = 0.f, o = 0.f;
  // passes of 128 keys staged in LDS by all 512 threads (8 float4 each: few registers, so the
  // weight prefetch can stay in flight through the attention); 64-key block b of the pass is wave
  // (2 * pass + b) % 8's, so every wave still takes blocks v, v + 8, ... in increasing order
  for (int k0 = 0; k0 < n; k0 += 128) {
    if (k0 > 0) kv_pass_load(c, K, V, pos, k0, kp);  // (pass 0 was loaded by attn_begin)
    __syncthreads();  // the previous pass is consumed
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = c.tid + NT * u, r = idx >> 4, c4 = idx & 15;
      *reinterpret_cast<float4*>(&c.L.Ks[r][4 * c4]) = kp.kv[u];
      *reinterpret_cast<float4*>(&c.L.Vs[r][4 * c4]) = kp.vv[u];
    }
    __syncthreads();
    const int blk = c.wave - ((k0 >> 6) & 7);  // this wave's block within the pass (0 or 1), if any
    if (blk == 0 || blk == 1) {
      const int b0 = k0 + 64 * blk;
      if (b0 < n) {
        const int j = b0 + c.lane;
        const float4* kr = reinterpret_cast<const float4*>(c.L.Ks[64 * blk + c.lane]);
        const float4* q4 = reinterpret_cast<const float4*>(c.L.q);
        float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
#pragma unroll
        for (int d4 = 0; d4 < HD / 4; ++d4) {
          const float4 qq = q4[d4], kk = kr[d4];
          d0 = fmaf(qq.x, kk.x, d0);
          d1 = fmaf(qq.y, kk.y, d1);
          d2 = fmaf(qq.z, kk.z, d2);
          d3 = fmaf(qq.w, kk.w, d3);
        }
        const float sc = j <= pos ? (d0 + d1) + (d2 + d3) : -INFINITY;
        const float m_new = fmaxf(m_run, wave_max(sc));
        const float alpha = m_run == -INFINITY ? 0.f : expf(m_run - m_new);
        const float pj = j <= pos ? expf(sc - m_new) : 0.f;
        l_run = l_run * alpha + wave_sum(pj);
        o *= alpha;
        const int pji = __float_as_int(pj);
#pragma unroll
        for (int u = 0; u < 64; ++u)  // keys past pos: p = 0 and v = 0, an exact no-op
          o = fmaf(__int_as_float(__builtin_amdgcn_readlane(pji, u)), c.L.Vs[64 * blk + u][c.lane], o);
        m_run = m_new;
      }
    }
  }
  c.L.ao[c.wave][c.lane] = o;
  if (c.lane == 0) { c.L.am[c.wave] = m_run; c.L.al[c.wave] = l_run; }
  __syncthreads();
  if (c.wave < REP) {  // wave r combines (identically) and publishes replica r
    float M = -INFINITY;
#pragma unroll
    for (int v = 0; v < 8; ++v) M = fmaxf(M, c.L.am[v]);
    float Ls = 0.f, O = 0.f;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const float wv = c.L.am[v] == -INFINITY ? 0.f : expf(c.L.am[v] - M);
      Ls = fmaf(c.L.al[v], wv, Ls);
      O = fmaf(c.L.ao[v][c.lane], wv, O);
    }
    c.put(G_ATT, D, a * HD + c.lane, O / Ls, c.wave);  // E2
  }
}

// o_proj rows 8w.. (+ residual) -> E3
__device__ __forceinline__ void phase_o(Ctx& c, const WO& W) {
  float s[4];
  const float* xc = c.L.att + 8 * (c.tid & 255);
#pragma unroll
  for (int i = 0; i < 4; ++i) s[i] = dot8(W.a[i], xc);
  rows_reduce<4>(c, s);
  if (c.tid < 8 * REP) {
    const int q = c.tid / REP, h = q / 4, i = q % 4, n = 8 * c.w + q;
    c.put(G_X, D, n, c.L.x[n] + row_total(c, h, i), c.tid % REP);
  }
}

// MLP quarter Q: the wave's gate/up pair -> SiLU*up column 8Q + wave (LDS), then this quarter's 8
// columns of the down split-K into the four row accumulators (column chunks added in order 0..3)
template <int Q>
__device__ __forceinline__ void phase_mq(Ctx& c, const WMq& m, float (&acc)[4], float rs) {
  float t[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float s = dot8(m.g[i][0], c.L.xn + 8 * c.lane);
#pragma unroll
    for (int j = 1; j < 4; ++j) s += dot8(m.g[i][j], c.L.xn + 8 * (c.lane + 64 * j));
    t[i] = wave_sum(s);
  }
  if (c.lane == 0) c.L.hb[8 * Q + c.wave] = silu_f(rs * t[0]) * (rs * t[1]);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float v = dot8(m.d[k], c.L.hb + 8 * Q);
    acc[k] = Q == 0 ? v : acc[k] + v;
  }
}

// Reduce-scatter: rows 8w..8w+7 of every producer's partials (fixed order), + residual -> E5
__device__ __forceinline__ void phase_reduce(Ctx& c) {
  const unsigned tag = c.tag();
  const u64* g = c.buf(G_PART, (size_t)NWG * D);
  const int v = c.tid >> 1, half = c.tid & 1;
  const u64* src = g + (size_t)v * D + 8 * c.w + 4 * half;
#if BB_PAIR16
  const int poff[2] = {v * D + 8 * c.w + 4 * half, v * D + 8 * c.w + 4 * half + 2};
  poll_pairs<2, BB_PROBE_DELAY, 1>(g, 0x7fffffff, poff, tag, [&](unsigned spin) { return spin_fail(c, spin); },
                                   [&](const u32x4_t (&q)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      c.L.red[4 * half + 2 * h][v] = __uint_as_float(q[h].x);
      c.L.red[4 * half + 2 * h + 1][v] = __uint_as_float(q[h].z);
    }
  });
  c.stamp(c.e + 1);
  (void)src;
#else
  u64 q[4];
  probe_delay();
#pragma unroll
  for (int u = 0; u < 4; ++u) q[u] = gload(src + u);
  for (unsigned spin = 0;; ++spin) {
    bool ok = true;
#pragma unroll
    for (int u = 0; u < 4; ++u) ok &= (unsigned)(q[u] >> 32) == tag;
    if (ok || spin_fail(c, spin)) break;
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if ((unsigned)(q[u] >> 32) != tag) q[u] = gload(src + u);
  }
  c.stamp(c.e + 1);
#pragma unroll
  for (int u = 0; u < 4; ++u) c.L.red[4 * half + u][v] = __uint_as_float((unsigned)q[u]);
#endif
  __syncthreads();
  ++c.e;  // the x hand-off that follows
  {
    const float* r = c.L.red[c.wave];
    float s = ((r[4 * c.lane] + r[4 * c.lane + 1]) + r[4 * c.lane + 2]) + r[4 * c.lane + 3];
    s = wave_sum(s);
    if (c.lane < REP) {
      const int n = 8 * c.w + c.wave;
      c.put(G_X, D, n, c.L.x[n] + s, c.lane);
    }
  }
}

// ============================================================================ int4 weights
// The step of an nn.quantize'd engine (int4 g64, run_streaming_csm_mlx.py:811-818): the hand-offs, the
// attention and the reduce-scatter are the bf16 kernel's; every projection reads its weight rows as 16-B
// chunks of 32 nibbles -- one per lane, so a wave covers one 2048-wide row -- plus the half group's
// {scale, bias} word, against activations staged in the padded layout (q4p) with their half-group sums
// (handoff.h q4dot32: the int4 GEMV's per-half-group arithmetic).  Per workgroup: QKV wave v rows
// 12w + v and 12w + 8 + (v & 3) (waves 4-7 load a duplicate they do not use: no branch around a load);
// o_proj wave v row 8w + v; gate/up wave v rows 64w + 8v .. + 7 (SiLU*up columns 4v .. 4v + 3); down
// this workgroup's 32 columns (one half group) of rows t + 512 k from the chunk-major copy (q4_down_cm:
// nibbles [F/32][D][16 B], affine words [F/64][D]).  The RMSNorm is folded as in the bf16 kernel
// (staged x * nw, the row scale after the dot product), layer 0 included.
struct WQ4 { u32x4_t a[2]; unsigned s[2]; };
struct WO4 { u32x4_t a; unsigned s; };
struct WM4 { u32x4_t g[8]; unsigned gs[8]; u32x4_t d[4]; unsigned ds[4]; };
constexpr int RB = D / 2, SBR = D / 64 * 4;              // bytes of a row's nibbles / affine words (K = D)
constexpr int SB_QKV = QKV * RB, SB_O = D * RB, SB_GU = 2 * F * RB, SB_DN = D * F / 2;

__device__ __forceinline__ void load_q4(Ctx& c, int l, WQ4& r) {
  const char* W = reinterpret_cast<const char*>(c.p.wqkv[l]);
  const int r0 = 12 * c.w, va = c.wave * RB + c.lane * 16, vb = (8 + (c.wave & 3)) * RB + c.lane * 16;
  r.a[0] = bload<2>(W, va, r0 * RB);
  r.a[1] = bload<2>(W, vb, r0 * RB);
  const int sa = c.wave * SBR + (c.lane >> 1) * 4, sb = (8 + (c.wave & 3)) * SBR + (c.lane >> 1) * 4;
  r.s[0] = bload4(W, sa, SB_QKV + r0 * SBR);
  r.s[1] = bload4(W, sb, SB_QKV + r0 * SBR);
}
__device__ __forceinline__ void load_o4(Ctx& c, int l, WO4& r) {
  const char* W = reinterpret_cast<const char*>(c.p.wo[l]);
  r.a = bload<2>(W, c.wave * RB + c.lane * 16, 8 * c.w * RB);
  r.s = bload4(W, c.wave * SBR + (c.lane >> 1) * 4, SB_O + 8 * c.w * SBR);
}
__device__ __forceinline__ void load_m4(Ctx& c, int l, WM4& r) {
  const char* G = reinterpret_cast<const char*>(c.p.wgu[l]);
  const int r0 = 64 * c.w + 8 * c.wave;  // (wave-dependent: in the lane offset, not the scalar one)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r.g[i] = bload<2>(G, 8 * c.wave * RB + c.lane * 16, (64 * c.w + i) * RB);
    r.gs[i] = bload4(G, 8 * c.wave * SBR + (c.lane >> 1) * 4, SB_GU + (64 * c.w + i) * SBR);
  }
  (void)r0;
  const char* Dn = reinterpret_cast<const char*>(c.p.wdc[l]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    r.d[k] = bload<2>(Dn, c.tid * 16, (c.w * D + k * NT) * 16);
    r.ds[k] = bload4(Dn, c.tid * 4, SB_DN + ((c.w >> 1) * D + k * NT) * 4);
  }
}

// half-group sums of the staged pair (2t, 2t + 1) of each half: the 16 threads of a half group in order
__device__ __forceinline__ void half_group_sums(Ctx& c, const float (&pair)[2], float* out) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float v = pair[h];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    if ((c.tid & 15) == 0) out[(h * (D / 2) + 2 * c.tid) >> 5] = v;
  }
}
// an x hand-off (E3 / E5) -> x, xq = x * nw (padded), xh, per-wave sums of squares (folded RMSNorm)
__device__ __forceinline__ void gather_x4(Ctx& c, const u64* buf, const Nw& nw) {
  const int poff[2] = {2 * c.tid, D / 2 + 2 * c.tid};
  float sq = 0.f, pr[2];
  poll_pairs<2, BB_PROBE_DELAY, 1>(buf, 0x7fffffff, poff, c.tag(), [&](unsigned spin) { return spin_fail(c, spin); },
                                   [&](const u32x4_t (&g)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float v0 = __uint_as_float(g[h].x), v1 = __uint_as_float(g[h].z);
      const float a = v0 * nw.v[2 * h], b = v1 * nw.v[2 * h + 1];
      *reinterpret_cast<float2*>(&c.L.x[poff[h]]) = make_float2(v0, v1);
      *reinterpret_cast<float2*>(&c.L.xq[0][0] + q4p(poff[h])) = make_float2(a, b);
      sq = fmaf(v0, v0, sq);
      sq = fmaf(v1, v1, sq);
      pr[h] = a + b;
    }
  });
  c.stamp(c.e + 1);
  half_group_sums(c, pr, c.L.xh);
  sq = wave_sum(sq);
  if (c.lane == 0) c.L.sq[c.wave] = sq;
  __syncthreads();
}
// the same staging from L.x (the embedded row, layer 0)
__device__ __forceinline__ void stage_x4(Ctx& c, const Nw& nw) {
  float sq = 0.f, pr[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = h * (D / 2) + 2 * c.tid;
    const float v0 = c.L.x[k], v1 = c.L.x[k + 1];
    const float a = v0 * nw.v[2 * h], b = v1 * nw.v[2 * h + 1];
    *reinterpret_cast<float2*>(&c.L.xq[0][0] + q4p(k)) = make_float2(a, b);
    sq = fmaf(v0, v0, sq);
    sq = fmaf(v1, v1, sq);
    pr[h] = a + b;
  }
  half_group_sums(c, pr, c.L.xh);
  sq = wave_sum(sq);
  if (c.lane == 0) c.L.sq[c.wave] = sq;
  __syncthreads();
}
// the attention output hand-off (E2) -> aq (padded), ah
template <int DELAY = BB_PROBE_DELAY>
__device__ __forceinline__ void gather_att4(Ctx& c, const u64* buf) {
  const int poff[2] = {2 * c.tid, D / 2 + 2 * c.tid};
  float pr[2];
  poll_pairs<2, DELAY, 1>(buf, 0x7fffffff, poff, c.tag(), [&](unsigned spin) { return spin_fail(c, spin); },
                          [&](const u32x4_t (&g)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float v0 = __uint_as_float(g[h].x), v1 = __uint_as_float(g[h].z);
      *reinterpret_cast<float2*>(&c.L.aq[0][0] + q4p(poff[h])) = make_float2(v0, v1);
      pr[h] = v0 + v1;
    }
  });
  c.stamp(c.e + 1);
  half_group_sums(c, pr, c.L.ah);
  __syncthreads();
}

// QKV rows 12w.. (folded norm: the row scale after the dot; RoPE at pos) -> E1, k / v rows to the cache
__device__ __forceinline__ void phase_qkv4(Ctx& c, int l, int pos, const WQ4& W) {
  const float* xa = c.L.xq[c.lane];
  const float hs = c.L.xh[c.lane];
  float s0 = q4dot32(W.a[0], xa, W.s[0], hs), s1 = q4dot32(W.a[1], xa, W.s[1], hs);
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  if (c.lane == 0) { c.L.wsum[c.wave][0] = s0; c.L.wsum[c.wave][1] = s1; }
  __syncthreads();
  if (c.tid < 6) {  // pair j: rows i0, i0 + 1 of the slice (row i: wave i & 7, slot i >> 3)
    const int i0 = 2 * c.tid, n = 12 * c.w + i0;
    const float rs = row_rs(c);
    float a = c.L.wsum[i0 & 7][i0 >> 3] * rs, b = c.L.wsum[(i0 + 1) & 7][(i0 + 1) >> 3] * rs;
    if (n < (HQ + HKV) * HD) {
      const float2 cs = c.L.rope[(n % HD) / 2];
      const float y0 = a * cs.x - b * cs.y, y1 = b * cs.x + a * cs.y;
      a = y0;
      b = y1;
    }
    u64* g = c.buf(G_QKV, QKV);
    gput(g + n, a, c.tag());
    gput(g + n + 1, b, c.tag());
    if (n >= HQ * HD) {  // KVCache.update_and_fetch: the new row at pos
      const int nn = n < (HQ + HKV) * HD ? n - HQ * HD : n - (HQ + HKV) * HD;
      float* cache = n < (HQ + HKV) * HD ? c.p.kc[l] : c.p.vc[l];
      *reinterpret_cast<float2*>(cache + ((size_t)(nn / HD) * c.p.S_cap + pos) * HD + nn % HD) = make_float2(a, b);
    }
  }
}
// o_proj rows 8w + v (+ residual) -> E3
__device__ __forceinline__ void phase_o4(Ctx& c, const WO4& W) {
  float s = q4dot32(W.a, c.L.aq[c.lane], W.s, c.L.ah[c.lane]);
  s = wave_sum(s);
  if (c.lane == 0) c.L.wsum[c.wave][0] = s;
  __syncthreads();
  if (c.tid < 8 * REP) {
    const int q = c.tid / REP, n = 8 * c.w + q;
    c.put(G_X, D, n, c.L.x[n] + c.L.wsum[q][0], c.tid % REP);
  }
}
// gate/up (8 rows per wave -> 4 SiLU*up columns), then the down partials of rows t + 512 k over the
// workgroup's 32 columns
__device__ __forceinline__ void phase_m4(Ctx& c, const WM4& W, float (&acc)[4], float rs) {
  const float* xa = c.L.xq[c.lane];
  const float hs = c.L.xh[c.lane];
  float t[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = wave_sum(q4dot32(W.g[i], xa, W.gs[i], hs));
  if (c.lane < 4) {  // pair j = lane: rows 2j (gate), 2j + 1 (up) of the wave's 8
    const float gt = rs * (c.lane == 0 ? t[0] : (c.lane == 1 ? t[2] : (c.lane == 2 ? t[4] : t[6])));
    const float up = rs * (c.lane == 0 ? t[1] : (c.lane == 1 ? t[3] : (c.lane == 2 ? t[5] : t[7])));
    c.L.hb[4 * c.wave + c.lane] = silu_f(gt) * up;
  }
  __syncthreads();
  float hsum = 0.f;
#pragma unroll
  for (int j = 0; j < 32; j += 4) {
    const float4 v = *reinterpret_cast<const float4*>(&c.L.hb[j]);
    hsum += (v.x + v.y) + (v.z + v.w);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = q4dot32(W.d[k], c.L.hb, W.ds[k], hsum);
}

}  // namespace

__global__ __launch_bounds__(NT, 1) void bb_step_q4_kernel(BbStepArgs p) {
  __shared__ __attribute__((aligned(16))) Lds L;
  Ctx c{p, L, (int)blockIdx.x, (int)threadIdx.x, (int)(threadIdx.x & 63), (int)(threadIdx.x >> 6), 0u, 0};
  c.tag0 = __hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  c.stamp(0);
  const int pos = p.pos[0];
  WQ4 wq;
  WO4 wo;
  WM4 wm;
  load_q4(c, 0, wq);
  Nw nw1 = nw_fetch(c, p.n1[0]);
  for (int k = c.tid; k < D; k += NT) L.x[k] = p.x[k];
  if (c.tid < HD / 2) L.rope[c.tid] = reinterpret_cast<const float2*>(p.rope)[(size_t)pos * (HD / 2) + c.tid];
  __syncthreads();
  stage_x4(c, nw1);
  for (int l = 0; l < NL; ++l) {
    c.refresh();
    phase_qkv4(c, l, pos, wq);                        // -> E1
    ++c.e;
    const bool attn_wg = c.w < NATT;
    if (!attn_wg) {                                   // (the attention WGs fetch after their attention)
      load_o4(c, l, wo);
      load_m4(c, l, wm);
    }
    const Nw nw2 = nw_fetch(c, p.n2[l]);
    if (attn_wg) {
      KvPass kp;
      attn_begin(c, l, pos, kp);
      attn_rest(c, l, pos, kp);                       // -> E2
      load_o4(c, l, wo);
      load_m4(c, l, wm);
    }
    if (attn_wg) gather_att4(c, c.rbuf(G_ATT, D));   // E2
    else gather_att4<BB_DELAY_E2>(c, c.rbuf(G_ATT, D));
    ++c.e;
    c.refresh();
    phase_o4(c, wo);                                  // -> E3
    if (l + 1 < NL) load_q4(c, l + 1, wq);
    gather_x4(c, c.rbuf(G_X, D), nw2);                // E3 -> x, xq = x * n2
    const float rs2 = row_rs(c);
    ++c.e;
    c.refresh();
    float acc[4];
    phase_m4(c, wm, acc, rs2);
    {
      u64* g = c.buf(G_PART, (size_t)NWG * D) + (size_t)c.w * D;
#pragma unroll
      for (int k = 0; k < 4; ++k) gput(g + c.tid + NT * k, acc[k], c.tag());   // -> E4
    }
    nw1 = nw_fetch(c, l + 1 < NL ? p.n1[l + 1] : p.norm);
    c.refresh();
    phase_reduce(c);                                  // waits E4, -> E5
    gather_x4(c, c.rbuf(G_X, D), nw1);                // E5 -> x, xq = x * (next n1 | final norm)
    ++c.e;
  }
  c.refresh();
  if (c.w == 0) {
    const float rs = row_rs(c);
    for (int k = c.tid; k < D; k += NT) p.h_last[k] = (&L.xq[0][0])[q4p(k)] * rs;
  }
  c.stamp(BB_STEP_STAMPS - 1);
  if (c.w == 0 && c.tid == 0) __hip_atomic_store(p.epoch, c.tag0 - 1u + (unsigned)c.e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

namespace {
}  // namespace

__global__ __launch_bounds__(NT, 1) void bb_step_kernel(BbStepArgs p) {
  __shared__ __attribute__((aligned(16))) Lds L;
  Ctx c{p, L, (int)blockIdx.x, (int)threadIdx.x, (int)(threadIdx.x & 63), (int)(threadIdx.x >> 6), 0u, 0};
  c.tag0 = __hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  c.stamp(0);
  const int pos = p.pos[0];  // the new row's position (the embedding launch advanced it)
  WQ wq;
  WO wo;
  WMq mq[4];
  load_q(c, 0, wq);
  Nw nw1 = nw_fetch(c, p.n1[0]);
  for (int k = c.tid; k < D; k += NT) L.x[k] = p.x[k];
  if (c.tid < HD / 2) L.rope[c.tid] = reinterpret_cast<const float2*>(p.rope)[(size_t)pos * (HD / 2) + c.tid];
  __syncthreads();
  for (int l = 0; l < NL; ++l) {
    c.refresh();
    // layers >= 1 (folded): the previous layer's E5 gather already wrote xn = x * n1
    const bool fold1 = BB_FOLD && l > 0;
    if (!fold1) rms(c, nw1, L.xn);
    phase_qkv(c, l, pos, wq, fold1);                  // -> E1
    ++c.e;                                            // E1 is read by the attention workgroups only
    const bool attn_wg = c.w < NATT;
    // the o_proj rows and the first two MLP quarters stream while the attention runs; the attention
    // workgroups fetch their second quarter after it (their E1 poll would queue behind it in the
    // CU's memory pipeline, and E2 waits on them).  Measured alternatives: both
    // quarters after the attention, the third quarter during E3, the next layer's first quarter
    // during E4 / E5 -- none faster.
    KvPass kp;
    if (attn_wg && BB_ATTN_LATE_PF) attn_begin(c, l, pos, kp);  // waits E1, first K / V pass in flight
    load_o(c, l, wo);
    load_mq(c, l, 0, mq[0]);
    if (!attn_wg) {
      load_mq(c, l, 1, mq[1]);
      // BB_EARLY_MQ2: the 224 workgroups without attention wait the whole attention at E2, so their
      // third quarter streams there too instead of inside the MLP
      if (BB_EARLY_MQ2) load_mq(c, l, 2, mq[2]);
    }
    const Nw nw2 = nw_fetch(c, p.n2[l]);
    if (attn_wg) {
      if (!BB_ATTN_LATE_PF) attn_begin(c, l, pos, kp);
      attn_rest(c, l, pos, kp);                       // -> E2
      load_mq(c, l, 1, mq[1]);
    }
    if (attn_wg) gather<D / NT>(c, c.rbuf(G_ATT, D), D, L.att);  // E2
    else gather<D / NT, BB_DELAY_E2>(c, c.rbuf(G_ATT, D), D, L.att);
    ++c.e;
    c.refresh();
    phase_o(c, wo);                                   // -> E3
    if (l + 1 < NL) load_q(c, l + 1, wq);
#if BB_FOLD
    gather_x(c, c.rbuf(G_X, D), nw2);                 // E3 -> x, xn = x * n2
    const float rs2 = row_rs(c);
#else
    gather<D / NT>(c, c.rbuf(G_X, D), D, L.x);         // E3
    const float rs2 = 1.f;
#endif
    ++c.e;
    c.refresh();
    if (!BB_FOLD) rms(c, nw2, L.xn);
    float acc[4];
    phase_mq<0>(c, mq[0], acc, rs2);
    if (attn_wg || !BB_EARLY_MQ2) load_mq(c, l, 2, mq[2]);
    phase_mq<1>(c, mq[1], acc, rs2);
    load_mq(c, l, 3, mq[3]);
    phase_mq<2>(c, mq[2], acc, rs2);
    phase_mq<3>(c, mq[3], acc, rs2);
    {
      u64* g = c.buf(G_PART, (size_t)NWG * D) + (size_t)c.w * D;
      if (BB_E4_16) {  // rows 2t, 2t + 1 (+ 1024): two granules per 16-B sc1 store   -> E4
        const unsigned tg = c.tag();
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(g, 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const u32x4_t v = {__float_as_uint(acc[2 * h]), tg, __float_as_uint(acc[2 * h + 1]), tg};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rs, (h * (D / 2) + 2 * c.tid) * 8, 0, 16);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) gput(g + c.tid + NT * k, acc[k], c.tag());   // -> E4
      }
    }
    nw1 = nw_fetch(c, l + 1 < NL ? p.n1[l + 1] : p.norm);
    c.refresh();
    phase_reduce(c);                                  // waits E4, -> E5
#if BB_FOLD
    gather_x(c, c.rbuf(G_X, D), nw1);                 // E5 -> x, xn = x * (next n1 | final norm)
#else
    gather<D / NT>(c, c.rbuf(G_X, D), D, L.x);         // E5
#endif
    ++c.e;
  }
  // final norm of the last row -> h_last (generation.py:42 reads norm(h[:, -1]))
  c.refresh();
#if BB_FOLD
  if (c.w == 0) {
    const float rs = row_rs(c);
    for (int k = c.tid; k < D; k += NT) p.h_last[k] = L.xn[k] * rs;
  }
#else
  rms(c, nw1, L.xn);
  if (c.w == 0)
    for (int k = c.tid; k < D; k += NT) p.h_last[k] = L.xn[k];
#endif
  c.stamp(BB_STEP_STAMPS - 1);
  if (c.w == 0 && c.tid == 0) __hip_atomic_store(p.epoch, c.tag0 - 1u + (unsigned)c.e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

size_t bb_step_gbuf_bytes() { return G_TOTAL * sizeof(u64); }

void launch_bb_step(const BbStepArgs& p, hipStream_t st, bool q4) {
  if (q4) hipLaunchKernelGGL(bb_step_q4_kernel, dim3(NWG), dim3(NT), 0, st, p);
  else hipLaunchKernelGGL(bb_step_kernel, dim3(NWG), dim3(NT), 0, st, p);
}

const void* bb_step_kernel_ptr(bool q4) {
  return q4 ? reinterpret_cast<const void*>(&bb_step_q4_kernel) : reinterpret_cast<const void*>(&bb_step_kernel);
}
