// Persistent frame decoder: codebook0_head + the 31 depth-decoder steps of one frame
// (/root/reference/csm_mlx/generation.py:42-90) in ONE launch, batch 1, greedy, bf16 weights.
//
// Why: at batch 1 the depth decoder is a chain of 31 x (4 layers x 5 projections + attention + head)
// dependent launches of 2-34 MB each; every launch pays a kernel boundary plus its own ramp and
// drain, ~3.5 us apiece over ~650 launches per frame, while the weight bytes themselves stream in
// far less.  Here every CU keeps one workgroup for the whole frame, owns a fixed slice of every
// matrix, and streams its slices into registers one or two hand-offs AHEAD of use (the weights do not
// depend on the activations), so the weight stream overlaps the dependency latency.
//
// Work split (NWG = 256 workgroups = one per CU, 512 threads = 8 waves each):
//   QKV    1536 rows: 6 per WG (RoPE pairs stay inside a WG)        -> all-gather q|k|v  (E1)
//   attention: every WG computes all 8 heads redundantly (<= 32 keys) -> no hand-off
//   o_proj 1024 rows: 4 per WG, + residual                           -> all-gather x      (E3)
//   gate/up 16384 interleaved rows: 64 per WG -> h[32 columns];
//   down   split-K: WG w multiplies its 32 columns of W_down (chunk-major copy, [F/16][D][16])
//          by its h -> 1024 partials                                  -> reduce-scatter   (E4)
//          WG w sums the 256 partials of rows 4w..4w+3 in a fixed order, + residual
//                                                                      -> all-gather x      (E5)
//   heads  2051 rows: 8 per WG (+1 for WGs 0-2), arg-max partial       -> all-gather keys   (E6)
// Layer 0 of steps >= 2 reads q|k|v (RoPE'd) and the input row from the folded tables built at
// csm_begin (proj_tab / qkv0_tab), so it has no QKV hand-off.  16 hand-offs per step.
//
// Hand-offs are data-tagged granules (MI355X_MICROARCH.md hand-off price list, "Granule"): each value
// travels as one naturally aligned 8-byte {float bits, tag} written by ONE agent-scope relaxed store
// (sc1) and read with agent-scope relaxed loads (sc1) until the tag matches; tag = epoch + hand-off
// index (epoch advances by the frame's hand-off count, never reused).  Buffers alternate by hand-off
// parity: a WG can only overwrite a buffer after every WG has published the next hand-off, i.e. after
// every WG finished reading the previous use.  Every spin is bounded: on timeout a WG raises the
// error word and stops waiting (results garbage, the host raises) -- the grid always drains.
//
// Arithmetic: fp32 accumulation of bf16 weights x fp32 activations, RMSNorm as the oracle
// (x * rsqrt(mean(x^2) + eps) * w), RoPE on interleaved pairs from the cos/sin table, softmax with
// max subtraction, reductions in fixed orders (deterministic run to run).
#include <type_traits>

#include "csm_kernels.h"
#include "handoff.h"

namespace {

using namespace handoff;

constexpr int NWG = 256, NT = 512;
constexpr int D = 1024, F = 8192, HQ = 8, HKV = 2, HD = 128, NL = DEC_FRAME_LAYERS, DB = 2048;
constexpr int QKV = (HQ + 2 * HKV) * HD;  // 1536
constexpr int MAXM = 2;                   // rows per step (step 1: [h_last, E_a[c0]])
constexpr unsigned SPIN_LIMIT = 1u << 22; // ~0.1 s of s_sleep per hand-off before declaring failure
constexpr int VMAX = 2056;                // padded audio vocabulary (V <= 2051, checked by the engine)

// the same chunk against two activation rows (every weight converted once, used twice: no
// loop-invariant conversions for the compiler to hoist out of a row loop)
__device__ __forceinline__ void dot8x2(const u32x4_t w, const float* x0, const float* x1, float& s0, float& s1) {
  const float4 a0 = *reinterpret_cast<const float4*>(x0), b0 = *reinterpret_cast<const float4*>(x0 + 4);
  const float4 a1 = *reinterpret_cast<const float4*>(x1), b1 = *reinterpret_cast<const float4*>(x1 + 4);
  float t;
  t = bf16_lo(w.x); s0 = fmaf(t, a0.x, s0); s1 = fmaf(t, a1.x, s1);
  t = bf16_hi(w.x); s0 = fmaf(t, a0.y, s0); s1 = fmaf(t, a1.y, s1);
  t = bf16_lo(w.y); s0 = fmaf(t, a0.z, s0); s1 = fmaf(t, a1.z, s1);
  t = bf16_hi(w.y); s0 = fmaf(t, a0.w, s0); s1 = fmaf(t, a1.w, s1);
  t = bf16_lo(w.z); s0 = fmaf(t, b0.x, s0); s1 = fmaf(t, b1.x, s1);
  t = bf16_hi(w.z); s0 = fmaf(t, b0.y, s0); s1 = fmaf(t, b1.y, s1);
  t = bf16_lo(w.w); s0 = fmaf(t, b0.z, s0); s1 = fmaf(t, b1.z, s1);
  t = bf16_hi(w.w); s0 = fmaf(t, b0.w, s0); s1 = fmaf(t, b1.w, s1);
}

// dot8x2 for the step's rows only: M == 1 runs row 0's chain alone (the same fmaf order)
template <int M>
__device__ __forceinline__ void dotm(const u32x4_t w, const float* x0, const float* x1, float& s0, float& s1) {
  if constexpr (M == 2) {
    dot8x2(w, x0, x1, s0, s1);
  } else {
    const float4 a0 = *reinterpret_cast<const float4*>(x0), b0 = *reinterpret_cast<const float4*>(x0 + 4);
    s0 = fmaf(bf16_lo(w.x), a0.x, s0);
    s0 = fmaf(bf16_hi(w.x), a0.y, s0);
    s0 = fmaf(bf16_lo(w.y), a0.z, s0);
    s0 = fmaf(bf16_hi(w.y), a0.w, s0);
    s0 = fmaf(bf16_lo(w.z), b0.x, s0);
    s0 = fmaf(bf16_hi(w.z), b0.y, s0);
    s0 = fmaf(bf16_lo(w.w), b0.z, s0);
    s0 = fmaf(bf16_hi(w.w), b0.w, s0);
  }
}

__device__ __forceinline__ u32x4_t wload(const bf16_t* p) { return *reinterpret_cast<const u32x4_t*>(p); }

struct Lds {
  float x[MAXM][D];        // residual rows
  float xn[MAXM][DB];      // normed x * norm weight (GEMV input); h_last at frame start
  float qkv[MAXM][QKV];    // gathered q | k | v (RoPE'd)
  float att[MAXM][D];      // attention output
  float qs[HQ][HD];        // scaled query of one row per head
  float2 rope[MAXM][HD / 2];// (cos, sin) of this step's positions, staged once per step
  alignas(16) float hb[MAXM][32];  // this WG's h columns
  float red[4 * MAXM][256];// reduce-scatter staging [row][producer]
  float wsum[8][MAXM * 8]; // per-wave partial dots
  float sq[8][MAXM];       // per-wave partial sums of squares of the gathered x rows (folded RMSNorm)
  union {
    float Ks[HKV][32][HD + 4];// cached keys of this layer (rows padded: conflict-free row-parallel reads)
    struct {                  // int4 kernel, frame start only (before any step's K history): h_last in the
      float hq[DB / 32][36];  // padded half-group layout (handoff.h q4p) with its half-group sums
      float hh[DB / 32];
    } h0;
  };
  float Vs[HKV][32][HD];    // cached values
  float lg[VMAX];          // sampling: the head's logits, gathered from every workgroup
  int code;                // last arg-max
  int flag;
  // int4 kernel: projection inputs in the padded layout with their half-group sums -- x * norm weight
  // (QKV / gate-up / head input) and the attention output (o_proj input)
  alignas(16) float xq[MAXM][D / 32][36];
  float xh[MAXM][D / 32];
  alignas(16) float aq[MAXM][D / 32][36];
  float ah[MAXM][D / 32];
};

}  // namespace

namespace {

// Granule buffer regions (u64 offsets), each double-buffered by hand-off parity.  The all-gather
// regions (every workgroup reads every granule) are written in REP replicas: a producer stores each
// granule REP times, workgroup w polls replica w % REP -- the workgroups of one XCD under the
// observed round-robin placement (speed only, never correctness), so each granule has 256 / REP
// readers instead of 256 (MI355X_MICROARCH.md allgather row: 256 -> 32 readers of a 16 KB sweep
// -1.9 us).  Replicas are 4 KB-aligned plus a 256-B skew so they fall on different channels.
// The reduce-scatter region (G_PART: each granule has one reader) is not replicated.  Measured
// (profiles/r03_ab_replicas.txt): 2394 -> 2325 us per frame at REP 4 or 8 with the replica stores
// spread over lanes (stored serially by one lane, REP 8 cost more on the publish than it saved).
#ifndef DF_REP
#define DF_REP 4
#endif
constexpr int REP = DF_REP;
__host__ __device__ constexpr size_t rs_of(size_t per) { return (per + 511) / 512 * 512 + 32; }
constexpr size_t G_X = 0;                                               // [2][REP][rs(MAXM*D)] x slices
constexpr size_t G_QKV = G_X + 2 * REP * rs_of(MAXM * D);               // [2][REP][rs(MAXM*QKV)]
constexpr size_t G_PART = G_QKV + 2 * REP * rs_of(MAXM * QKV);          // [2][NWG][MAXM][D] down partials
constexpr size_t G_ARG = G_PART + (size_t)2 * NWG * MAXM * D;           // [2][REP][rs(NWG*2)] arg-max keys
constexpr size_t G_LOG = G_ARG + 2 * REP * rs_of(NWG * 2);              // [2][REP][rs(VMAX)] logits (sampling)
constexpr size_t G_GUM = G_LOG + 2 * REP * rs_of(VMAX);               // [2][REP][rs(NWG*3)] Gumbel-max keys
constexpr size_t G_TOTAL = G_GUM + 2 * REP * rs_of(NWG * 3);

struct Ctx {
  const DecFrameArgs& p;
  Lds& L;
  int w, tid, lane, wave;
  unsigned tag0;
  int e;  // hand-off counter
  int ps = 0;  // phase-mark counter (profiling stamps 512..1007)
  int code = 0;  // the last head's code (every thread holds it)
  __device__ void mark() {
    if (p.stamps && tid == 0 && ps < 496) p.stamps[(size_t)w * DEC_FRAME_STAMPS + 512 + ps] = __builtin_amdgcn_s_memrealtime();
    ++ps;
  }
  // profiling: the 100 MHz real-time clock when this WG's hand-off wait number e completed
  __device__ void stamp() const {
    if (p.stamps && tid == 0 && e < DEC_FRAME_STAMPS) p.stamps[(size_t)w * DEC_FRAME_STAMPS + e] = __builtin_amdgcn_s_memrealtime();
  }
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
  // one replica r of granule i: the publishing lanes are spread over the replicas (lane-parallel
  // stores, one per lane), so a hand-off costs its producer one store instruction, not REP
  __device__ void put(size_t region, size_t per, size_t i, float v, int r) const {
    gput(p.gbuf + region + ((size_t)(e & 1) * REP + (size_t)r) * rs_of(per) + i, v, tag());
  }
  __device__ void put_u(size_t region, size_t per, size_t i, unsigned v, int r) const {
    gput_u(p.gbuf + region + ((size_t)(e & 1) * REP + (size_t)r) * rs_of(per) + i, v, tag());
  }
};

// Hand-off waits (handoff.h poll_granules): DF_POLL2 keeps two probes in flight, DF_POLL_GAP
// sleeps apart.
#ifndef DF_DN_AFTER_E1
#define DF_DN_AFTER_E1 0
#endif
#ifndef DF_DN_EARLY
#define DF_DN_EARLY 0
#endif
#ifndef DF_GU_E45
#define DF_GU_E45 0   // gate/up rows per wave of the next layer fetched during E4 / E5 (<= GU_EARLY)
#endif
#ifndef DF_POLL2
#define DF_POLL2 0
#endif
#ifndef DF_PROBE_DELAY
#define DF_PROBE_DELAY 16
#endif
#ifndef DF_REPOLL
#define DF_REPOLL 2
#endif
// per hand-off kind (E1 q|k|v, E3 / E5 x, E4 down partials, E6 arg-max keys), default DF_PROBE_DELAY
#ifndef DF_DELAY_E1
#define DF_DELAY_E1 DF_PROBE_DELAY
#endif
#ifndef DF_DELAY_E3
#define DF_DELAY_E3 DF_PROBE_DELAY
#endif
#ifndef DF_DELAY_E4
#define DF_DELAY_E4 DF_PROBE_DELAY
#endif
#ifndef DF_DELAY_E5
#define DF_DELAY_E5 40
#endif
#ifndef DF_DELAY_E6
#define DF_DELAY_E6 DF_PROBE_DELAY
#endif
#ifndef DF_POLL_GAP
#define DF_POLL_GAP 8
#endif
__device__ __forceinline__ bool spin_fail(Ctx& c, unsigned spin) {
  if (spin >= SPIN_LIMIT || ((spin & 255) == 255 && __hip_atomic_load(c.p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
    __hip_atomic_store(c.p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  return false;
}
// use(x): the lane-local consumption of the matched probe
template <int GPT, int DELAY = DF_PROBE_DELAY, typename F>
__device__ __forceinline__ void poll(Ctx& c, const u64* base, const int (&off)[GPT], const bool (&val)[GPT], F&& use) {
  poll_granules<GPT, DF_POLL2 != 0, DF_POLL_GAP, DELAY, DF_REPOLL>(base, off, val, c.tag(), [&](unsigned spin) { return spin_fail(c, spin); }, use);
  c.stamp();
}

// Wait until granules [0, n) of buf carry `tag`; values -> out (LDS).  Threads take granules
// tid, tid + NT, ... (at most GPT each).
template <int GPT>
__device__ __forceinline__ void gather(Ctx& c, const u64* buf, int n, float* out) {
#if DF_PAIR16
  // granule pairs (2i, 2i + 1), i = tid, tid + NT, ...; a granule past n (odd n) counts as current
  constexpr int GPP = (GPT + 1) / 2;
  const int np = (n + 1) / 2;
  int poff[GPP];
#pragma unroll
  for (int u = 0; u < GPP; ++u) poff[u] = 2 * min(c.tid + u * NT, np - 1);
  const unsigned tag = c.tag();
  if (DF_PROBE_DELAY > 0) __builtin_amdgcn_s_sleep(DF_PROBE_DELAY);
  auto cur1 = [&](const u32x4_t& x, int i) { return x.y == tag && (i + 1 >= n || x.w == tag); };
  u32x4_t g[GPP];
#pragma unroll
  for (int u = 0; u < GPP; ++u) g[u] = sc1_load16(buf, poff[u] * 8, 0x7fffffff);
  for (unsigned spin = 0;; ++spin) {
    bool ok = true;
#pragma unroll
    for (int u = 0; u < GPP; ++u) ok &= cur1(g[u], poff[u]);
    if (ok || spin_fail(c, spin)) break;
    __builtin_amdgcn_s_sleep(DF_REPOLL);
#pragma unroll
    for (int u = 0; u < GPP; ++u)
      if (!cur1(g[u], poff[u])) g[u] = sc1_load16(buf, poff[u] * 8, 0x7fffffff);
  }
  c.stamp();
#pragma unroll
  for (int u = 0; u < GPP; ++u)
    if (c.tid + u * NT < np) {
      out[poff[u]] = __uint_as_float(g[u].x);
      if (poff[u] + 1 < n) out[poff[u] + 1] = __uint_as_float(g[u].z);
    }
#else
  int off[GPT];
  bool val[GPT];
#pragma unroll
  for (int u = 0; u < GPT; ++u) {
    off[u] = c.tid + u * NT;
    val[u] = off[u] < n;
  }
  poll<GPT>(c, buf, off, val, [&](const u64 (&g)[GPT]) {
#pragma unroll
    for (int u = 0; u < GPT; ++u)
      if (val[u]) out[off[u]] = __uint_as_float((unsigned)g[u]);
  });
#endif
  __syncthreads();
}

// xn[m][k] = x[m][k] * rsqrt(mean(x^2) + eps) * nw[k] for rows m < M (every WG computes the same)
// RMSNorm weight elements tid and tid + 512 (every element a thread scales), fetched a phase ahead
// DF_PAIR16: x hand-offs (E3 / E5) and the down partials (E4) polled as granule pairs, one 16-B load
// each (thread t owns elements 2t, 2t + 1 of a row instead of t, t + NT)
#ifndef DF_PAIR16
#define DF_PAIR16 1
#endif
__device__ __forceinline__ int el0(const Ctx& c) { return DF_PAIR16 ? 2 * c.tid : c.tid; }
__device__ __forceinline__ int el1(const Ctx& c) { return DF_PAIR16 ? 2 * c.tid + 1 : c.tid + NT; }
__device__ __forceinline__ float2 nw_fetch(const Ctx& c, const float* nw) { return make_float2(nw[el0(c)], nw[el1(c)]); }

template <int M>
__device__ __forceinline__ void rms_rows(Ctx& c, float2 nw, int m0 = 0) {
  static_assert(D == 2 * NT, "a thread scales elements tid and tid + NT of each row");
  // sum of squares: wave m sums row m in a fixed order
  if (c.wave < M) {
    const float* x = c.L.x[m0 + c.wave];
    float s = 0.f;
    for (int k = c.lane; k < D; k += 64) s = fmaf(x[k], x[k], s);
    s = wave_sum(s);
    if (c.lane == 0) c.L.wsum[0][c.wave] = s;
  }
  __syncthreads();
  for (int m = 0; m < M; ++m) {
    const float r = rsqrtf(c.L.wsum[0][m] / (float)D + c.p.eps);
    c.L.xn[m][el0(c)] = c.L.x[m0 + m][el0(c)] * r * nw.x;
    c.L.xn[m][el1(c)] = c.L.x[m0 + m][el1(c)] * r * nw.y;
  }
  __syncthreads();
}

// Folded RMSNorm (DF_FOLD): an x hand-off is gathered straight into x and into xn = x * nw (the next
// consumer's norm weight) with per-wave sums of squares; the consumer dots against the un-normalised
// xn and scales its results by rsqrt(mean(x^2) + eps) -- one barrier and one pass over the rows
// fewer per norm (the batched path's xs.h does the same: row scale after the dot product).
#ifndef DF_FOLD
#define DF_FOLD 1
#endif
template <int M, int DELAY>
__device__ __forceinline__ void gather_x(Ctx& c, const u64* buf, float2 nw) {
  static_assert(D == 2 * NT, "granule tid + NT u is element (u / 2, tid + NT (u % 2))");
  constexpr int GPT = M * D / NT;
  int off[GPT];
  bool val[GPT];
#pragma unroll
  for (int u = 0; u < GPT; ++u) {
    off[u] = c.tid + u * NT;
    val[u] = true;
  }
  float sq[MAXM];
#if DF_PAIR16
  int poff[M];
#pragma unroll
  for (int m = 0; m < M; ++m) poff[m] = m * D + 2 * c.tid;
  poll_pairs<M, DELAY, DF_REPOLL>(buf, 0x7fffffff, poff, c.tag(), [&](unsigned spin) { return spin_fail(c, spin); },
                                  [&](const u32x4_t (&g)[M]) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float v0 = __uint_as_float(g[m].x), v1 = __uint_as_float(g[m].z);
      *reinterpret_cast<float2*>(&c.L.x[m][2 * c.tid]) = make_float2(v0, v1);
      *reinterpret_cast<float2*>(&c.L.xn[m][2 * c.tid]) = make_float2(v0 * nw.x, v1 * nw.y);
      sq[m] = fmaf(v1, v1, v0 * v0);
    }
  });
  c.stamp();
  (void)off; (void)val;
#else
  poll<GPT, DELAY>(c, buf, off, val, [&](const u64 (&g)[GPT]) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float v0 = __uint_as_float((unsigned)g[2 * m]), v1 = __uint_as_float((unsigned)g[2 * m + 1]);
      c.L.x[m][c.tid] = v0;
      c.L.x[m][c.tid + NT] = v1;
      c.L.xn[m][c.tid] = v0 * nw.x;
      c.L.xn[m][c.tid + NT] = v1 * nw.y;
      sq[m] = fmaf(v1, v1, v0 * v0);
    }
  });
#endif
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const float t = wave_sum(sq[m]);
    if (c.lane == 0) c.L.sq[c.wave][m] = t;
  }
  __syncthreads();
}
// rsqrt(mean(x^2) + eps) of gathered row m (the 8 wave partials in order)
__device__ __forceinline__ float row_rs(const Ctx& c, int m) {
  float s = c.L.sq[0][m];
#pragma unroll
  for (int w = 1; w < 8; ++w) s += c.L.sq[w][m];
  return rsqrtf(s / (float)D + c.p.eps);
}

// ---- weight slices held in registers (issued ahead of use)
struct WQkv { u32x4_t a, b; };      // waves 0..5: row 6w+wave, chunks lane / lane+64
struct WO { u32x4_t a; };            // row 4w + wave/2, chunk (wave&1)*64 + lane
#ifndef GU_EARLY
#define GU_EARLY 4  // gate/up rows per wave fetched before the attention (the rest after o_proj)
#endif
struct WGu { u32x4_t a[8][2]; };     // rows 64w + 8*wave + r, chunks lane / lane+64
struct WDn { u32x4_t a[2][2][2]; };  // [row t / t+512][chunk 2w+q][16-B half]
struct WHd { u32x4_t a[2]; u32x4_t x[2]; };  // head row 8w+wave (+ row 2048+w for wave 0, w < 3)

__device__ __forceinline__ void load_qkv(Ctx& c, int l, WQkv& r) {
  if (c.wave < 6) {
    const bf16_t* row = c.p.wqkv[l] + (size_t)(6 * c.w) * D;  // uniform
    const int v = (c.wave * D + 8 * c.lane) * 2;
    r.a = bload(row, v, 0);
    r.b = bload(row, v, 1024);
  }
}
__device__ __forceinline__ void load_o(Ctx& c, int l, WO& r) {
  const bf16_t* row = c.p.wo[l] + (size_t)(4 * c.w) * D;
  r.a = bload(row, ((c.wave >> 1) * D + 8 * ((c.wave & 1) * 64 + c.lane)) * 2, 0);
}
template <int I0, int I1>
__device__ __forceinline__ void load_gu(Ctx& c, int l, WGu& r) {
  const bf16_t* base = c.p.wgu[l] + (size_t)(64 * c.w) * D;
  const int v = (8 * c.wave * D + 8 * c.lane) * 2;
#pragma unroll
  for (int i = I0; i < I1; ++i) {
    r.a[i][0] = bload(base, v, i * D * 2);
    r.a[i][1] = bload(base, v, i * D * 2 + 1024);
  }
}
// DF_E4_16: thread t computes down rows 2t, 2t + 1 (not t, t + 512) and publishes both partials in
// one 16-B sc1 store (two granules, each with its own tag)
#ifndef DF_E4_16
#define DF_E4_16 1
#endif
#ifndef DF_TAB16
#define DF_TAB16 1
#endif
__device__ __forceinline__ void load_dn(Ctx& c, int l, WDn& r) {
  const bf16_t* base = c.p.wdc[l] + (size_t)(2 * c.w) * D * 16;
  const int v = DF_E4_16 ? c.tid * 16 * 2 * 2 : c.tid * 16 * 2;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int so = DF_E4_16 ? (q * D * 16 + s * 16) * 2 : (q * D * 16 + 512 * s * 16) * 2;
      r.a[s][q][0] = bload(base, v, so);
      r.a[s][q][1] = bload(base, v, so + 16);
    }
}
__device__ __forceinline__ void load_head(Ctx& c, const bf16_t* W, int K, WHd& r) {
  // K = 1024 (ci heads): 128 chunks per row -> 2 per lane; non-temporal (read once per frame)
  const bf16_t* base = W + (size_t)(8 * c.w) * K;
  const int v = (c.wave * K + 8 * c.lane) * 2;
  r.a[0] = bload<2>(base, v, 0);
  r.a[1] = bload<2>(base, v, 1024);
  if (c.wave == 0 && c.w < 3) {
    const bf16_t* xr = W + (size_t)(2048 + c.w) * K;
    r.x[0] = bload<2>(xr, 16 * c.lane, 0);
    r.x[1] = bload<2>(xr, 16 * c.lane, 1024);
  }
}

// ---- int4 weight slices (an nn.quantize'd engine: dec_frame_kernel<true>).  A 16-B chunk holds 32
// nibbles (a half group), so one 1024-wide decoder row is 32 lanes: each wave covers two rows, lanes 0-31
// the first, 32-63 the second (half_sums reduces them apart); every chunk comes with its half group's
// affine word (handoff.h q4dot32).  Down reads the chunk-major copy (q4_down_cm: nibbles [F/32][D][16 B],
// affine words [F/64][D]) -- the WG's 32 columns are one half group of every row.
constexpr int RB = D / 2, SBR = D / 64 * 4;             // a 1024-wide row: nibble bytes, affine-word bytes
constexpr int RBH = DB / 2, SBRH = DB / 64 * 4;         // a 2048-wide row (codebook0_head, projection)
constexpr int SB_QKV = QKV * RB, SB_O = D * RB, SB_GU = 2 * F * RB, SB_DN = D * F / 2, SB_PROJ = D * RBH;
struct WQkv4 { u32x4_t a; unsigned s; };       // waves 0-2: rows 6w + 2v (lanes 0-31), 6w + 2v + 1 (32-63)
struct WO4 { u32x4_t a; unsigned s; };         // waves 0-1: rows 4w + 2v, + 1
struct WGu4 { u32x4_t a[4]; unsigned s[4]; };  // load i: rows 64w + 8v + 2i (gate, lanes 0-31), + 1 (up)
struct WDn4 { u32x4_t a[2]; unsigned s[2]; };  // rows 2t, 2t + 1 over the WG's 32 columns
__device__ __forceinline__ int hrow(const Ctx& c) { return c.lane >> 5; }  // which row of the wave's two
__device__ __forceinline__ int hgi(const Ctx& c) { return c.lane & 31; }   // the lane's half group

__device__ __forceinline__ void load_qkv4(Ctx& c, int l, WQkv4& r) {
  if (c.wave < 3) {
    const char* W = reinterpret_cast<const char*>(c.p.wqkv[l]);
    const int row = 2 * c.wave + hrow(c);
    r.a = bload(W, row * RB + hgi(c) * 16, 6 * c.w * RB);
    r.s = bload4(W, row * SBR + (hgi(c) >> 1) * 4, SB_QKV + 6 * c.w * SBR);
  }
}
__device__ __forceinline__ void load_o4(Ctx& c, int l, WO4& r) {
  if (c.wave < 2) {
    const char* W = reinterpret_cast<const char*>(c.p.wo[l]);
    const int row = 2 * c.wave + hrow(c);
    r.a = bload(W, row * RB + hgi(c) * 16, 4 * c.w * RB);
    r.s = bload4(W, row * SBR + (hgi(c) >> 1) * 4, SB_O + 4 * c.w * SBR);
  }
}
template <int I0, int I1>
__device__ __forceinline__ void load_gu4(Ctx& c, int l, WGu4& r) {
  const char* W = reinterpret_cast<const char*>(c.p.wgu[l]);
  const int row = 8 * c.wave + hrow(c);
#pragma unroll
  for (int i = I0; i < I1; ++i) {
    r.a[i] = bload(W, row * RB + hgi(c) * 16, (64 * c.w + 2 * i) * RB);
    r.s[i] = bload4(W, row * SBR + (hgi(c) >> 1) * 4, SB_GU + (64 * c.w + 2 * i) * SBR);
  }
}
__device__ __forceinline__ void load_dn4(Ctx& c, int l, WDn4& r) {
  const char* W = reinterpret_cast<const char*>(c.p.wdc[l]);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    r.a[k] = bload(W, (2 * c.tid + k) * 16, c.w * D * 16);
    r.s[k] = bload4(W, (2 * c.tid + k) * 4, SB_DN + (c.w >> 1) * D * 4);
  }
}

// half-group sums of the pair (2t, 2t + 1) of one 1024-wide row: the 16 threads of a half group in order
__device__ __forceinline__ void half_group_sum16(const Ctx& c, float v, float* out) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  if ((c.tid & 15) == 0) out[c.tid >> 4] = v;
}

// ---- phases
// QKV rows of this WG for M rows at positions pos0..pos0+M-1 (RoPE), published to E1.
template <int M, bool SC>
__device__ __forceinline__ void qkv_publish(Ctx& c, int pos0);
template <int M, bool SC>
__device__ __forceinline__ void phase_qkv(Ctx& c, int pos0, const WQkv& W) {
  if (c.wave < 6) {
    float s0 = 0.f, s1 = 0.f;
    dotm<M>(W.a, c.L.xn[0] + 8 * c.lane, c.L.xn[1] + 8 * c.lane, s0, s1);
    dotm<M>(W.b, c.L.xn[0] + 8 * (c.lane + 64), c.L.xn[1] + 8 * (c.lane + 64), s0, s1);
    s0 = wave_sum(s0);
    if constexpr (M == 2) s1 = wave_sum(s1);
    if (c.lane == 0) { c.L.wsum[c.wave][0] = s0; if constexpr (M == 2) c.L.wsum[c.wave][1] = s1; }
  }
  __syncthreads();
  qkv_publish<M, SC>(c, pos0);
}
// int4: waves 0-2, the wave's two rows from its two lane halves (row 2v + h -> wsum[2v + h], as above)
template <int M, bool SC>
__device__ __forceinline__ void phase_qkv4(Ctx& c, int pos0, const WQkv4& W) {
  if (c.wave < 3) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float2 h = half_sums(q4dot32(W.a, c.L.xq[m][hgi(c)], W.s, c.L.xh[m][hgi(c)]));
      if (c.lane == 0) { c.L.wsum[2 * c.wave][m] = h.x; c.L.wsum[2 * c.wave + 1][m] = h.y; }
    }
  }
  __syncthreads();
  qkv_publish<M, SC>(c, pos0);
}
// the WG's 6 rows (wsum[r][m]) -> folded row scale, RoPE pairs -> E1
template <int M, bool SC>
__device__ __forceinline__ void qkv_publish(Ctx& c, int pos0) {
  if (c.tid < 3 * M * REP) {  // RoPE pair j of row m: rows n, n+1 = 6w + 2j, +1 -> replica rr
    const int pr = c.tid / REP, rr = c.tid % REP, m = pr / 3, j = pr % 3, n = 6 * c.w + 2 * j;
    float a = c.L.wsum[2 * j][m], b = c.L.wsum[2 * j + 1][m];
    if (SC) {  // folded RMSNorm: the row scale after the dot product
      const float rs = row_rs(c, m);
      a *= rs;
      b *= rs;
    }
    if (n < (HQ + HKV) * HD) {
      const int d = n % HD;
      const float2 cs = c.L.rope[m][d / 2];
      const float y0 = a * cs.x - b * cs.y, y1 = b * cs.x + a * cs.y;
      a = y0;
      b = y1;
    }
    c.put(G_QKV, MAXM * QKV, (size_t)m * QKV + n, a, rr);
    c.put(G_QKV, MAXM * QKV, (size_t)m * QKV + n + 1, b, rr);
  }
}

// K / V rows 0..pos0-1 of this layer's cache (written by WG 0 in earlier steps, write-through) are
// fetched with sc1 loads into registers BEFORE the hand-off wait that precedes attention, and stored
// to LDS after it: chunk idx = tid + 512 u -> (kv head idx >> 10, key (idx >> 5) & 31, 16-B chunk idx & 31).
struct KvRegs { u32x4_t k[4], v[4]; };
__device__ __forceinline__ void kv_issue(Ctx& c, int layer, int pos0, KvRegs& r) {
  const int bytes = HKV * c.p.S_cap * HD * 4;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = c.tid + 512 * u, g = idx >> 10, j = (idx >> 5) & 31, q = idx & 31;
    if (j < pos0) {
      const int off = ((g * c.p.S_cap + j) * HD + 4 * q) * 4;
      r.k[u] = sc1_load16(c.p.kc[layer], off, bytes);
      r.v[u] = sc1_load16(c.p.vc[layer], off, bytes);
    }
  }
}
__device__ __forceinline__ void kv_store(Ctx& c, int pos0, const KvRegs& r) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = c.tid + 512 * u, g = idx >> 10, j = (idx >> 5) & 31, q = idx & 31;
    if (j < pos0) {
      *reinterpret_cast<u32x4_t*>(&c.L.Ks[g][j][4 * q]) = r.k[u];
      *reinterpret_cast<u32x4_t*>(&c.L.Vs[g][j][4 * q]) = r.v[u];
    }
  }
}

// The step's new K / V rows (positions pos0 .. pos0+M-1, gathered in L.qkv) appended to the LDS
// history, so the attention reads every key from one array.
template <int M>
__device__ __forceinline__ void kv_append(Ctx& c, int pos0) {
  for (int idx = c.tid; idx < M * HKV * HD; idx += NT) {
    const int m = idx / (HKV * HD), r = idx % (HKV * HD), g = r / HD, d = r % HD;
    c.L.Ks[g][pos0 + m][d] = c.L.qkv[m][HQ * HD + r];
    c.L.Vs[g][pos0 + m][d] = c.L.qkv[m][(HQ + HKV) * HD + r];
  }
}

// DF_KVDIRECT: the q | k | v hand-off (and layer 0's table row) is written straight to its places --
// q to L.qkv, the new k / v rows into the LDS history at pos0 + m -- so no kv_append pass and one
// barrier fewer before the attention.
#ifndef DF_KVDIRECT
#define DF_KVDIRECT 1
#endif
__device__ __forceinline__ void qkv_place(Ctx& c, int m, int r, int pos0, float v) {
  if (r < HQ * HD) c.L.qkv[m][r] = v;
  else if (r < (HQ + HKV) * HD) c.L.Ks[(r - HQ * HD) / HD][pos0 + m][r % HD] = v;
  else c.L.Vs[(r - (HQ + HKV) * HD) / HD][pos0 + m][r % HD] = v;
}
template <int M>
__device__ __forceinline__ void gather_qkv(Ctx& c, const u64* buf, int pos0, const KvRegs& kv) {
  constexpr int GPT = (M * QKV + NT - 1) / NT;
  int off[GPT];
  bool val[GPT];
#pragma unroll
  for (int u = 0; u < GPT; ++u) {
    off[u] = c.tid + u * NT;
    val[u] = off[u] < M * QKV;
  }
#if DF_PAIR16
  constexpr int NP = M * QKV / 2, GPP = (NP + NT - 1) / NT;  // granule pairs; thread t: pairs t, t + NT
  int poff[GPP];
#pragma unroll
  for (int u = 0; u < GPP; ++u) poff[u] = 2 * min(c.tid + u * NT, NP - 1);  // (a clamped pair is re-read, unused)
  poll_pairs<GPP, DF_DELAY_E1, DF_REPOLL>(buf, 0x7fffffff, poff, c.tag(), [&](unsigned spin) { return spin_fail(c, spin); },
                                          [&](const u32x4_t (&g)[GPP]) {
#pragma unroll
    for (int u = 0; u < GPP; ++u)
      if (c.tid + u * NT < NP) {
        const int i = poff[u];
        qkv_place(c, i / QKV, i % QKV, pos0, __uint_as_float(g[u].x));
        qkv_place(c, (i + 1) / QKV, (i + 1) % QKV, pos0, __uint_as_float(g[u].z));
      }
  });
  c.stamp();
  (void)off; (void)val;
#else
  poll<GPT, DF_DELAY_E1>(c, buf, off, val, [&](const u64 (&g)[GPT]) {
#pragma unroll
    for (int u = 0; u < GPT; ++u)
      if (val[u]) qkv_place(c, off[u] / QKV, off[u] % QKV, pos0, __uint_as_float((unsigned)g[u]));
  });
#endif
  kv_store(c, pos0, kv);
  __syncthreads();
}

// Attention of rows m < M (positions pos0 + m) over keys 0..pos0+m, all in c.L.Ks / Vs (kv_store +
// kv_append).  Every WG computes all heads (wave = head), as attn_short_head: lane = (key kj =
// lane & 31, half hh of the head dims), scores from two half dots added by one shuffle,
// max-subtracted softmax, P.V in key order with the V rows read 8 keys at a time (all in flight
// together; rows past the last key are read but not used).  The new K/V rows go to the cache,
// spread over the workgroups, for later steps.
// DF_PV: the P.V loop's V reads -- 0: two 4-B reads per key (dims lane, lane + 64); 1: one 8-B read
// (dims 2 lane, +1); 2: one 16-B read per key over key halves (lane >> 5), the halves' sums exchanged
#ifndef DF_PV
#define DF_PV 2
#endif
#ifndef DF_ATTN_SUB
#define DF_ATTN_SUB 0  // lab: 1 / 2 move the attention-end mark after the softmax / after P.V (tools/df_stamps.py)
#endif
template <int M, bool Q4 = false>
__device__ __forceinline__ void phase_attn(Ctx& c, int pos0, int layer) {
  static_assert(!Q4 || DF_PV == 2, "the int4 kernel stages the attention output from the DF_PV 2 loop");
  const int h = c.wave, g = h / (HQ / HKV);
  const float scale = 0.08838834764831845f;  // 1 / sqrt(128)
  const int kj = c.lane & 31, hh = c.lane >> 5;
  for (int m = 0; m < M; ++m) {
    const int pos = pos0 + m, n = pos + 1;
    for (int d = c.lane; d < HD; d += 64) c.L.qs[h][d] = c.L.qkv[m][h * HD + d] * scale;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float part = 0.f;
    {
      const float4* k4 = reinterpret_cast<const float4*>(c.L.Ks[g][kj] + hh * (HD / 2));
      const float4* q4 = reinterpret_cast<const float4*>(c.L.qs[h] + hh * (HD / 2));
      float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
#pragma unroll
      for (int d4 = 0; d4 < HD / 8; ++d4) {
        const float4 a = k4[d4], q = q4[d4];
        d0 = fmaf(q.x, a.x, d0);
        d1 = fmaf(q.y, a.y, d1);
        d2 = fmaf(q.z, a.z, d2);
        d3 = fmaf(q.w, a.w, d3);
      }
      part = (d0 + d1) + (d2 + d3);
    }
    const float other = __shfl_xor(part, 32, 64);
    float s = hh == 0 ? part + other : other + part;
    if (kj >= n) s = -INFINITY;
    const float mx = wave_max(s);
    const float pj = kj < n ? expf(s - mx) : 0.f;
    const float l_run = wave_sum(hh == 0 ? pj : 0.f);
    const int pji = __float_as_int(pj);
    if (DF_ATTN_SUB == 1 && m == M - 1) c.mark();  // lab: the attention mark after the softmax
#if DF_PV == 1
    // lane = dims 2 lane, 2 lane + 1 (one 8-B V read per key), keys in order
    float o0 = 0.f, o1 = 0.f;
#pragma unroll
    for (int j0 = 0; j0 < 32; j0 += 8) {
      if (j0 < n) {
        float2 vv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) vv[u] = *reinterpret_cast<const float2*>(&c.L.Vs[g][j0 + u][2 * c.lane]);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (j0 + u < n) {
            const float pb = __int_as_float(__builtin_amdgcn_readlane(pji, j0 + u));
            o0 = fmaf(pb, vv[u].x, o0);
            o1 = fmaf(pb, vv[u].y, o1);
          }
        }
      }
    }
    const float inv = 1.f / l_run;
    *reinterpret_cast<float2*>(&c.L.att[m][h * HD + 2 * c.lane]) = make_float2(o0 * inv, o1 * inv);
#elif DF_PV == 2
    // lane = (key half kv = lane >> 5: keys 16 kv + u, dims 4 (lane & 31) .. +3): one 16-B V read per
    // key, the halves' sums added (keys 0-15 first) by one exchange
    const int kv = c.lane >> 5, dq = c.lane & 31;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u0 = 0; u0 < 16; u0 += 8) {
      if (u0 < n) {
        float4 vv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) vv[u] = *reinterpret_cast<const float4*>(&c.L.Vs[g][16 * kv + u0 + u][4 * dq]);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float pa = __int_as_float(__builtin_amdgcn_readlane(pji, u0 + u));
          const float pb = __int_as_float(__builtin_amdgcn_readlane(pji, 16 + u0 + u));
          const float p = kv ? pb : pa;
          if (16 * kv + u0 + u < n) {
            o.x = fmaf(p, vv[u].x, o.x);
            o.y = fmaf(p, vv[u].y, o.y);
            o.z = fmaf(p, vv[u].z, o.z);
            o.w = fmaf(p, vv[u].w, o.w);
          }
        }
      }
    }
    float4 t;
    t.x = __shfl_xor(o.x, 32, 64);
    t.y = __shfl_xor(o.y, 32, 64);
    t.z = __shfl_xor(o.z, 32, 64);
    t.w = __shfl_xor(o.w, 32, 64);
    if constexpr (Q4) {
      // int4 o_proj input: the padded layout (q4p) and its half-group sums -- lanes dq = 8j .. 8j + 7 of
      // the kv == 0 half hold half group 4h + j
      const float inv = 1.f / l_run;
      const float4 ov = make_float4((o.x + t.x) * inv, (o.y + t.y) * inv, (o.z + t.z) * inv, (o.w + t.w) * inv);
      if (kv == 0) *reinterpret_cast<float4*>(&c.L.aq[m][0][0] + q4p(h * HD + 4 * dq)) = ov;
      float hs = (ov.x + ov.y) + (ov.z + ov.w);
      hs += __shfl_xor(hs, 1, 64);
      hs += __shfl_xor(hs, 2, 64);
      hs += __shfl_xor(hs, 4, 64);
      if (kv == 0 && (dq & 7) == 0) c.L.ah[m][4 * h + (dq >> 3)] = hs;
    } else if (kv == 0) {
      const float inv = 1.f / l_run;
      *reinterpret_cast<float4*>(&c.L.att[m][h * HD + 4 * dq]) =
          make_float4((o.x + t.x) * inv, (o.y + t.y) * inv, (o.z + t.z) * inv, (o.w + t.w) * inv);
    }
#else
    float o0 = 0.f, o1 = 0.f;
#pragma unroll
    for (int j0 = 0; j0 < 32; j0 += 8) {
      if (j0 < n) {
        float va[8], vb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          va[u] = c.L.Vs[g][j0 + u][c.lane];
          vb[u] = c.L.Vs[g][j0 + u][c.lane + 64];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (j0 + u < n) {
            const float pb = __int_as_float(__builtin_amdgcn_readlane(pji, j0 + u));
            o0 = fmaf(pb, va[u], o0);
            o1 = fmaf(pb, vb[u], o1);
          }
        }
      }
    }
    const float inv = 1.f / l_run;
    c.L.att[m][h * HD + c.lane] = o0 * inv;
    c.L.att[m][h * HD + c.lane + 64] = o1 * inv;
#endif
  }
  if (DF_ATTN_SUB == 2) c.mark();  // lab: the attention mark after P.V (before the K/V store + barrier)
  // the new K / V rows -> cache, spread over the workgroups (WG w stores element w of each row:
  // 2 heads x 128 = 256 elements), write-through; the storing threads drain them (vmcnt(0)) before
  // this WG's next publish (phase_mlp), so a reader that saw that hand-off reads them coherently
  if (c.tid < M) {
    const int m = c.tid, r = c.w, gg = r / HD, d = r % HD;
    const size_t off = ((size_t)gg * c.p.S_cap + pos0 + m) * HD + d;
    sc1_store_f(c.p.kc[layer] + off, c.L.Ks[gg][pos0 + m][d]);
    sc1_store_f(c.p.vc[layer] + off, c.L.Vs[gg][pos0 + m][d]);
  }
  __syncthreads();
}

// o_proj rows 4w..4w+3 (+ residual) -> E3 granules
template <int M>
__device__ __forceinline__ void phase_o(Ctx& c, const WO& W) {
  {
    const int k = 8 * ((c.wave & 1) * 64 + c.lane);
    float s0 = 0.f, s1 = 0.f;
    dotm<M>(W.a, c.L.att[0] + k, c.L.att[1] + k, s0, s1);
    s0 = wave_sum(s0);
    if constexpr (M == 2) s1 = wave_sum(s1);
    if (c.lane == 0) { c.L.wsum[c.wave][0] = s0; if constexpr (M == 2) c.L.wsum[c.wave][1] = s1; }
  }
  __syncthreads();
  if (c.tid < 4 * M * REP) {
    const int q = c.tid / REP, m = q / 4, r = q % 4, n = 4 * c.w + r;
    const float o = c.L.wsum[2 * r][m] + c.L.wsum[2 * r + 1][m];
    c.put(G_X, MAXM * D, (size_t)m * D + n, c.L.x[m][n] + o, c.tid % REP);
  }
}

// gate/up (64 rows -> h[32]) and the split-K down partials of this WG's columns -> E4 granules
template <int M, bool SC>
__device__ __forceinline__ void phase_mlp(Ctx& c, const WGu& G, const WDn& Wd) {
  {
    float s[8][2];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s[i][0] = 0.f;
      s[i][1] = 0.f;
      dotm<M>(G.a[i][0], c.L.xn[0] + 8 * c.lane, c.L.xn[1] + 8 * c.lane, s[i][0], s[i][1]);
      dotm<M>(G.a[i][1], c.L.xn[0] + 8 * (c.lane + 64), c.L.xn[1] + 8 * (c.lane + 64), s[i][0], s[i][1]);
    }
#pragma unroll
    for (int m = 0; m < MAXM; ++m) {
      if (m >= M) break;
      float t[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) t[i] = wave_sum(s[i][m]);
      if (c.lane < 4) {  // pair j = 4*wave + lane: rows 2j (gate), 2j+1 (up) of the WG slice
        const float rs = SC ? row_rs(c, m) : 1.f;
        const float gt = rs * (c.lane == 0 ? t[0] : (c.lane == 1 ? t[2] : (c.lane == 2 ? t[4] : t[6])));
        const float up = rs * (c.lane == 0 ? t[1] : (c.lane == 1 ? t[3] : (c.lane == 2 ? t[5] : t[7])));
        c.L.hb[m][4 * c.wave + c.lane] = silu_f(gt) * up;
      }
    }
  }
  if (c.tid < MAXM) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this layer's K/V cache stores
  __syncthreads();
  u64* g = c.buf(G_PART, (size_t)NWG * MAXM * D) + (size_t)c.w * MAXM * D;
  float a[2][2];  // [row 2t + s | t + 512 s][utterance row m]
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    a[s][0] = 0.f;
    a[s][1] = 0.f;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      dotm<M>(Wd.a[s][q][0], c.L.hb[0] + 16 * q, c.L.hb[1] + 16 * q, a[s][0], a[s][1]);
      dotm<M>(Wd.a[s][q][1], c.L.hb[0] + 16 * q + 8, c.L.hb[1] + 16 * q + 8, a[s][0], a[s][1]);
    }
  }
  if (DF_E4_16) {
    const unsigned tg = c.tag();
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(g, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const u32x4_t v = {__float_as_uint(a[0][m]), tg, __float_as_uint(a[1][m]), tg};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rs, (m * D + 2 * c.tid) * 8, 0, 16);  // sc1
    }
  } else {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      gput(g + c.tid + 512 * s, a[s][0], c.tag());
      if (M > 1) gput(g + D + c.tid + 512 * s, a[s][1], c.tag());
    }
  }
}

// Reduce-scatter: rows 4w..4w+3 of every producer's partials (fixed order), + residual -> E5
template <int M>
__device__ __forceinline__ void phase_reduce(Ctx& c) {
  const u64* g = c.buf(G_PART, (size_t)NWG * MAXM * D);
  const int v = c.tid >> 1, half = c.tid & 1;
  int off[2 * M];
  bool val[2 * M];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      off[2 * m + u] = (v * MAXM + m) * D + 4 * c.w + 2 * half + u;
      val[2 * m + u] = true;
    }
#if DF_PAIR16
  int poff[M];
#pragma unroll
  for (int m = 0; m < M; ++m) poff[m] = off[2 * m];
  poll_pairs<M, DF_DELAY_E4, DF_REPOLL>(g, 0x7fffffff, poff, c.tag(), [&](unsigned spin) { return spin_fail(c, spin); },
                                        [&](const u32x4_t (&q)[M]) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      c.L.red[4 * m + 2 * half][v] = __uint_as_float(q[m].x);
      c.L.red[4 * m + 2 * half + 1][v] = __uint_as_float(q[m].z);
    }
  });
  c.stamp();
  (void)val;
#else
  poll<2 * M, DF_DELAY_E4>(c, g, off, val, [&](const u64 (&q)[2 * M]) {
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int u = 0; u < 2; ++u) c.L.red[4 * m + 2 * half + u][v] = __uint_as_float((unsigned)q[2 * m + u]);
  });
#endif
  __syncthreads();
  ++c.e;  // the x hand-off that follows
  if (c.wave < 4 * M) {
    const float* r = c.L.red[c.wave];
    float s = ((r[4 * c.lane] + r[4 * c.lane + 1]) + r[4 * c.lane + 2]) + r[4 * c.lane + 3];
    s = wave_sum(s);
    if (c.lane < REP) {
      const int m = c.wave / 4, n = 4 * c.w + c.wave % 4;
      c.put(G_X, MAXM * D, (size_t)m * D + n, c.L.x[m][n] + s, c.lane);
    }
  }
}

// ---- int4 phases
// o_proj: waves 0-1, rows 4w + 2v + h (+ residual) -> E3
template <int M>
__device__ __forceinline__ void phase_o4(Ctx& c, const WO4& W) {
  if (c.wave < 2) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float2 h = half_sums(q4dot32(W.a, c.L.aq[m][hgi(c)], W.s, c.L.ah[m][hgi(c)]));
      if (c.lane == 0) { c.L.wsum[2 * c.wave][m] = h.x; c.L.wsum[2 * c.wave + 1][m] = h.y; }
    }
  }
  __syncthreads();
  if (c.tid < 4 * M * REP) {
    const int q = c.tid / REP, m = q / 4, r = q % 4, n = 4 * c.w + r;
    c.put(G_X, MAXM * D, (size_t)m * D + n, c.L.x[m][n] + c.L.wsum[r][m], c.tid % REP);
  }
}
// gate/up (load i of wave v: the SiLU*up column 4v + i from its two lane halves) and the down partials
// of rows 2t, 2t + 1 over the WG's 32 columns -> E4 (two granules per 16-B sc1 store, as DF_E4_16)
template <int M, bool SC>
__device__ __forceinline__ void phase_mlp4(Ctx& c, const WGu4& G, const WDn4& Wd) {
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const float rs = SC ? row_rs(c, m) : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float2 h = half_sums(q4dot32(G.a[i], c.L.xq[m][hgi(c)], G.s[i], c.L.xh[m][hgi(c)]));
      if (c.lane == i) c.L.hb[m][4 * c.wave + i] = silu_f(rs * h.x) * (rs * h.y);
    }
  }
  if (c.tid < MAXM) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this layer's K/V cache stores
  __syncthreads();
  u64* g = c.buf(G_PART, (size_t)NWG * MAXM * D) + (size_t)c.w * MAXM * D;
  const unsigned tg = c.tag();
  const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(g, 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int m = 0; m < M; ++m) {
    float hs = 0.f;
#pragma unroll
    for (int j = 0; j < 32; j += 4) {
      const float4 v = *reinterpret_cast<const float4*>(&c.L.hb[m][j]);
      hs += (v.x + v.y) + (v.z + v.w);
    }
    const float a0 = q4dot32(Wd.a[0], c.L.hb[m], Wd.s[0], hs), a1 = q4dot32(Wd.a[1], c.L.hb[m], Wd.s[1], hs);
    const u32x4_t v = {__float_as_uint(a0), tg, __float_as_uint(a1), tg};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rsc, (m * D + 2 * c.tid) * 8, 0, 16);  // sc1
  }
}
// an x hand-off (E3 / E5) -> x, xq = x * nw (padded), xh, per-wave sums of squares (folded RMSNorm)
template <int M, int DELAY>
__device__ __forceinline__ void gather_x4(Ctx& c, const u64* buf, float2 nw) {
  int poff[M];
#pragma unroll
  for (int m = 0; m < M; ++m) poff[m] = m * D + 2 * c.tid;
  float sq[MAXM], pr[MAXM];
  poll_pairs<M, DELAY, DF_REPOLL>(buf, 0x7fffffff, poff, c.tag(), [&](unsigned spin) { return spin_fail(c, spin); },
                                  [&](const u32x4_t (&g)[M]) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float v0 = __uint_as_float(g[m].x), v1 = __uint_as_float(g[m].z);
      const float a = v0 * nw.x, b = v1 * nw.y;
      *reinterpret_cast<float2*>(&c.L.x[m][2 * c.tid]) = make_float2(v0, v1);
      *reinterpret_cast<float2*>(&c.L.xq[m][0][0] + q4p(2 * c.tid)) = make_float2(a, b);
      sq[m] = fmaf(v1, v1, v0 * v0);
      pr[m] = a + b;
    }
  });
  c.stamp();
#pragma unroll
  for (int m = 0; m < M; ++m) {
    half_group_sum16(c, pr[m], c.L.xh[m]);
    const float t = wave_sum(sq[m]);
    if (c.lane == 0) c.L.sq[c.wave][m] = t;
  }
  __syncthreads();
}
// RMSNorm of rows m < M from L.x (step 1's layer 0: x * rsqrt(mean(x^2) + eps) * nw, as rms_rows) -> xq, xh
template <int M>
__device__ __forceinline__ void rms_rows4(Ctx& c, float2 nw) {
  if (c.wave < M) {
    const float* x = c.L.x[c.wave];
    float s = 0.f;
    for (int k = c.lane; k < D; k += 64) s = fmaf(x[k], x[k], s);
    s = wave_sum(s);
    if (c.lane == 0) c.L.wsum[0][c.wave] = s;
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const float r = rsqrtf(c.L.wsum[0][m] / (float)D + c.p.eps);
    const float a = c.L.x[m][2 * c.tid] * r * nw.x, b = c.L.x[m][2 * c.tid + 1] * r * nw.y;
    *reinterpret_cast<float2*>(&c.L.xq[m][0][0] + q4p(2 * c.tid)) = make_float2(a, b);
    half_group_sum16(c, a + b, c.L.xh[m]);
  }
  __syncthreads();
}

// Temperature sampling without a top-k threshold (the reference generate()'s default, generation.py:
// 51-54, :102): handled by per-workgroup Gumbel-max keys (phase_head / gumbel_code), not by handing
// every logit to every workgroup.
__device__ __forceinline__ bool gumbel_local(const DecFrameArgs& p) {
  return p.temperature > 0.f && (p.top_k <= 0 || p.top_k >= p.V);
}
// order-preserving double -> u64 (larger value, larger key; every non-NaN value above key 0)
__device__ __forceinline__ unsigned long long dkey(double d) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(d);
  return (u >> 63) ? ~u : (u | (1ull << 63));
}

// Head rows of this WG on row xn[0] (K = 1024 or 2048) -> arg-max key -> E6 granules (hi, lo words)
__device__ __forceinline__ void head_publish(Ctx& c, float s, float t, int n_valid, float* logits, int cb);
// PAD: the input row is the int4 kernel's padded xq[xm] (element k at q4p(k): an 8-element chunk stays
// contiguous), else L.xn[xm]
template <int KH, bool PAD = false>
__device__ __forceinline__ void phase_head(Ctx& c, const bf16_t* W, int n_valid, const u32x4_t (&wa)[KH / 512],
                                           const u32x4_t (&wx)[KH / 512], float* logits, int cb, int xm = 0, float rs = 1.f) {
  constexpr int CPL = KH / 512;  // chunks per lane
  static_assert(!PAD || KH == D, "the padded input holds one decoder row");
  // input row (folded RMSNorm: un-normalised, scaled by rs after the dot)
  auto xin = [&](int i) -> const float* {
    if constexpr (PAD) return &c.L.xq[xm][0][0] + q4p(8 * (c.lane + 64 * i));
    else return c.L.xn[xm] + 8 * (c.lane + 64 * i);
  };
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) s += dot8(wa[i], xin(i));
  s = wave_sum(s) * rs;
  float t = 0.f;
  if (c.wave == 0 && c.w < 3) {
#pragma unroll
    for (int i = 0; i < CPL; ++i) t += dot8(wx[i], xin(i));
    t = wave_sum(t) * rs;
  }
  head_publish(c, s, t, n_valid, logits, cb);
  (void)W;
}
// A head's rows of this WG -- s: row 8w + wave, t: row 2048 + w (wave 0 of WGs 0-2) -- -> logits taps
// and the hand-off: arg-max keys (E6), Gumbel-max keys, or every logit (sampling with a top-k)
__device__ __forceinline__ void head_publish(Ctx& c, float s, float t, int n_valid, float* logits, int cb) {
  const int row = 8 * c.w + c.wave;
  unsigned long long best = row < n_valid ? pack_argmax(s, row) : 0ull;
  if (c.lane == 0 && row < n_valid) logits[row] = s;
  const int xr = 2048 + c.w;
  if (c.wave == 0 && c.w < 3) {
    const unsigned long long k2 = xr < n_valid ? pack_argmax(t, xr) : 0ull;
    best = k2 > best ? k2 : best;
    if (c.lane == 0 && xr < n_valid) logits[xr] = t;
  }
  if (gumbel_local(c.p)) {
    // temperature sampling with no top-k filter: the Gumbel-max is a max over independent perturbed
    // logits, so each workgroup reduces its own rows and hands on one (value, index) key
    const float inv_t = 1.0f / c.p.temperature;
    const uint64_t key = gumbel_key(c.p.seeds[0], c.p.frame_ctr[0] * c.p.K + cb);
    unsigned long long bk = 0ull;
    int bi = 0x7fffffff;
    auto cand = [&](float l, int v) {  // sample_code's rule: perturbed value strictly above -inf, first max
      if (!(l >= -INFINITY)) return;   // NaN logits never win
      double val = (double)(l * inv_t) + gumbel_noise(key, v);
      if (!(val > -INFINITY)) return;
      if (val == 0.0) val = 0.0;       // -0 and +0 compare equal in sample_code: one key
      const unsigned long long k = dkey(val);
      if (k > bk || (k == bk && v < bi)) { bk = k; bi = v; }
    };
    if (c.lane == 0 && row < n_valid) cand(s, row);
    if (c.lane == 0 && c.wave == 0 && c.w < 3 && xr < n_valid) cand(t, xr);
    unsigned long long* gk = reinterpret_cast<unsigned long long*>(&c.L.wsum[0][0]);
    int* gi = reinterpret_cast<int*>(gk + 8);
    if (c.lane == 0) { gk[c.wave] = bk; gi[c.wave] = bi; }
    __syncthreads();
    if (c.tid < REP) {
      unsigned long long b = gk[0];
      int ib = gi[0];
      for (int i = 1; i < 8; ++i)
        if (gk[i] > b || (gk[i] == b && gi[i] < ib)) { b = gk[i]; ib = gi[i]; }
      c.put_u(G_GUM, NWG * 3, 3 * c.w, (unsigned)(b >> 32), c.tid);
      c.put_u(G_GUM, NWG * 3, 3 * c.w + 1, (unsigned)b, c.tid);
      c.put_u(G_GUM, NWG * 3, 3 * c.w + 2, (unsigned)ib, c.tid);
    }
    __syncthreads();
    return;
  }
  if (c.p.temperature > 0.f) {  // sampling with top-k: every logit to every workgroup (sample_code)
    if (c.lane < REP && row < n_valid) c.put(G_LOG, VMAX, row, s, c.lane);
    if (c.lane < REP && c.wave == 0 && c.w < 3 && xr < n_valid) c.put(G_LOG, VMAX, xr, t, c.lane);
    __syncthreads();
    return;
  }
  if (c.lane == 0) reinterpret_cast<unsigned long long*>(c.L.wsum)[c.wave] = best;
  __syncthreads();
  if (c.tid < REP) {
    const unsigned long long* k = reinterpret_cast<const unsigned long long*>(c.L.wsum);
    unsigned long long b = k[0];
    for (int i = 1; i < 8; ++i) b = k[i] > b ? k[i] : b;
    c.put_u(G_ARG, NWG * 2, 2 * c.w, (unsigned)(b >> 32), c.tid);
    c.put_u(G_ARG, NWG * 2, 2 * c.w + 1, (unsigned)b, c.tid);
  }
  __syncthreads();
}

// Gather the 256 arg-max keys -> code (every WG identical).  Thread t polls granule t (word t & 1 of
// key t / 2); the two words meet by one lane swap, every wave takes the max of its 32 keys, and one
// barrier joins the 8 wave maxima -- the max of exact keys, so the order is immaterial.
__device__ __forceinline__ int gather_code(Ctx& c, int V) {
  static_assert(NWG * 2 == NT, "one key word per thread");
#if DF_PAIR16
  // key t = granule pair t: threads t < NWG poll one pair each (the others hold key 0)
  unsigned long long b = 0ull;
  if (c.tid < NWG) {
    const int poff[1] = {2 * c.tid};
    poll_pairs<1, DF_DELAY_E6, DF_REPOLL>(c.rbuf(G_ARG, NWG * 2), 0x7fffffff, poff, c.tag(),
                                          [&](unsigned spin) { return spin_fail(c, spin); },
                                          [&](const u32x4_t (&g)[1]) { b = ((unsigned long long)g[0].x << 32) | g[0].z; });
  }
  c.stamp();
#else
  const int off[1] = {c.tid};
  const bool val[1] = {true};
  unsigned wv = 0;
  poll<1, DF_DELAY_E6>(c, c.rbuf(G_ARG, NWG * 2), off, val, [&](const u64 (&g)[1]) { wv = (unsigned)g[0]; });
  const unsigned ov = __shfl_xor(wv, 1, 64);
  unsigned long long b = (c.tid & 1) ? (((unsigned long long)ov << 32) | wv) : (((unsigned long long)wv << 32) | ov);
#endif
#pragma unroll
  for (int o = 32; o > (DF_PAIR16 ? 0 : 1); o >>= 1) {
    const unsigned long long t = __shfl_xor(b, o, 64);
    b = t > b ? t : b;
  }
  unsigned long long* wk = reinterpret_cast<unsigned long long*>(&c.L.red[0][0]);
  if (c.lane == 0) wk[c.wave] = b;
  __syncthreads();
  b = wk[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) b = wk[i] > b ? wk[i] : b;
  c.code = min(max(unpack_argmax(b), 0), V - 1);
  return c.code;
}

// Sampling (temperature > 0): gather the head's V logits, then -- identically in every workgroup --
// the sampler of sample_kernel (csm_kernels.hip): the top_k-th largest logit by radix select (keys
// >= it kept, ties included), then the Gumbel-max over logits * (1/temp) of the kept entries with
// the first-max tie rule.  cb: codebook index of the sampler's counter (frame * K + cb).
__device__ __forceinline__ int sample_code(Ctx& c, int V, int cb) {
  constexpr int NPT = (VMAX + NT - 1) / NT;  // logits per thread
  const DecFrameArgs& p = c.p;
  // the Gumbel noise does not depend on the logits: drawn before the hand-off wait (overlaps it)
  const uint64_t key = gumbel_key(p.seeds[0], p.frame_ctr[0] * p.K + cb);
  double gn[NPT];
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int v = c.tid + NT * i;
    gn[i] = v < V ? gumbel_noise(key, v) : 0.0;
  }
  gather<NPT>(c, c.rbuf(G_LOG, VMAX), V, c.L.lg);
  float thr = -INFINITY;
  if (p.top_k > 0 && p.top_k < V) {
    // radix select, 8 bits per pass; threads 0..255 hold digit 255 - tid for the suffix count
    uint32_t* hist = reinterpret_cast<uint32_t*>(&c.L.red[0][0]);
    uint32_t* wsum = hist + 256;
    uint32_t* sh = hist + 264;  // [prefix, remain]
    uint32_t prefix = 0, maskbits = 0, rem = (uint32_t)p.top_k;
    for (int shift = 24; shift >= 0; shift -= 8) {
      if (c.tid < 256) hist[c.tid] = 0;
      __syncthreads();
#pragma unroll
      for (int i = 0; i < NPT; ++i) {
        const int v = c.tid + NT * i;
        if (v < V) {
          const uint32_t key = f2key(c.L.lg[v]);
          if ((key & maskbits) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
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
      __syncthreads();  // sh / hist reused by the next pass
    }
    thr = key2f(prefix);
  }
  const float inv_t = 1.0f / p.temperature;
  double best = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int v = c.tid + NT * i;
    if (v >= V) continue;
    const float l = c.L.lg[v];
    if (!(l >= thr)) continue;
    const double val = (double)(l * inv_t) + gn[i];  // = gumbel_perturbed(l, inv_t, key, v)
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
  double* sv = reinterpret_cast<double*>(&c.L.wsum[0][0]);
  int* si = reinterpret_cast<int*>(sv + 8);
  if (c.lane == 0) { sv[c.wave] = best; si[c.wave] = bi; }
  __syncthreads();
  if (c.tid == 0) {
    double bv = sv[0];
    int b = si[0];
    for (int w2 = 1; w2 < NT / 64; ++w2)
      if (sv[w2] > bv || (sv[w2] == bv && si[w2] < b)) { bv = sv[w2]; b = si[w2]; }
    c.L.code = min(max(b, 0), V - 1);  // NaN logits leave no winner: clamp (as sample_kernel)
  }
  __syncthreads();
  c.code = c.L.code;
  return c.code;
}

// Gather the 256 workgroups' Gumbel-max keys (value key hi, lo, index) -> code: max value, lowest
// index on ties; no candidate anywhere (every logit NaN or -inf) -> V - 1, as sample_kernel.
__device__ __forceinline__ int gumbel_code(Ctx& c, int V) {
  constexpr int NG = NWG * 3, GPT = (NG + NT - 1) / NT;
  int off[GPT];
  bool val[GPT];
#pragma unroll
  for (int u = 0; u < GPT; ++u) {
    off[u] = c.tid + u * NT;
    val[u] = off[u] < NG;
  }
  unsigned* words = reinterpret_cast<unsigned*>(&c.L.red[0][0]);
  poll<GPT, DF_DELAY_E6>(c, c.rbuf(G_GUM, NWG * 3), off, val, [&](const u64 (&g)[GPT]) {
#pragma unroll
    for (int u = 0; u < GPT; ++u)
      if (val[u]) words[off[u]] = (unsigned)g[u];
  });
  __syncthreads();
  unsigned long long b = 0ull;
  int ib = 0x7fffffff;
  if (c.tid < NWG) {
    b = ((unsigned long long)words[3 * c.tid] << 32) | words[3 * c.tid + 1];
    ib = (int)words[3 * c.tid + 2];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long ob = __shfl_xor(b, o, 64);
    const int oi = __shfl_xor(ib, o, 64);
    if (ob > b || (ob == b && oi < ib)) { b = ob; ib = oi; }
  }
  unsigned long long* wk = reinterpret_cast<unsigned long long*>(&c.L.wsum[0][0]);
  int* wi = reinterpret_cast<int*>(wk + 8);
  __syncthreads();  // (words read by every wave before wsum is reused)
  if (c.lane == 0 && c.wave < NWG / 64) { wk[c.wave] = b; wi[c.wave] = ib; }
  __syncthreads();
  b = wk[0];
  ib = wi[0];
#pragma unroll
  for (int i = 1; i < NWG / 64; ++i)
    if (wk[i] > b || (wk[i] == b && wi[i] < ib)) { b = wk[i]; ib = wi[i]; }
  c.code = b == 0ull ? V - 1 : min(max(ib, 0), V - 1);
  return c.code;
}

// the code of a head: greedy arg-max of the published keys, or the sampler
__device__ __forceinline__ int head_code(Ctx& c, int V, int cb) {
  if (c.p.temperature <= 0.f) return gather_code(c, V);
  return gumbel_local(c.p) ? gumbel_code(c, V) : sample_code(c, V, cb);
}

// Registers carried between phases (prefetched weights, norm weights)
struct Pre {
  WQkv wq;
  WO wo;
  WGu wg;
  WDn wd;
  WHd wh;
  float2 nw1;
};
struct Pre4 {  // the int4 kernel's (the ci heads stay bf16: audio_head is not quantized)
  WQkv4 wq;
  WO4 wo;
  WGu4 wg;
  WDn4 wd;
  WHd wh;
  float2 nw1;
};
template <bool Q4> using PreT = std::conditional_t<Q4, Pre4, Pre>;
#ifndef DF_GU4_EARLY
#define DF_GU4_EARLY 2  // int4: gate/up loads per wave fetched before the attention (of 4; the rest after o_proj)
#endif
static_assert(DF_FOLD && DF_PAIR16 && DF_E4_16 && DF_KVDIRECT && DF_TAB16 && DF_GU_E45 == 0 && !DF_DN_EARLY &&
              !DF_DN_AFTER_E1, "the int4 kernel implements the default variants only");
// weight-format dispatch of the loaders / phases the layer calls
template <bool Q4, typename P> __device__ __forceinline__ void ld_dn(Ctx& c, int l, P& r) {
  if constexpr (Q4) load_dn4(c, l, r.wd); else load_dn(c, l, r.wd);
}
template <bool Q4, typename P> __device__ __forceinline__ void ld_qkv(Ctx& c, int l, P& r) {
  if constexpr (Q4) load_qkv4(c, l, r.wq); else load_qkv(c, l, r.wq);
}
template <bool Q4, typename P> __device__ __forceinline__ void ld_o(Ctx& c, int l, P& r) {
  if constexpr (Q4) load_o4(c, l, r.wo); else load_o(c, l, r.wo);
}
template <bool Q4, bool EARLY, typename P> __device__ __forceinline__ void ld_gu(Ctx& c, int l, P& r) {
  if constexpr (Q4) {
    if constexpr (EARLY) load_gu4<0, DF_GU4_EARLY>(c, l, r.wg); else load_gu4<DF_GU4_EARLY, 4>(c, l, r.wg);
  } else {
    if constexpr (EARLY) load_gu<0, GU_EARLY>(c, l, r.wg); else load_gu<GU_EARLY, 8>(c, l, r.wg);
  }
}

// One decoder layer of step `step` (M rows at positions pos0..).  FIRST: layer 0, which at steps
// >= 2 takes q | k | v (RoPE'd) from the folded qkv0 table and its input row from proj_tab (no QKV
// hand-off).  LAST: the final layer, which also fetches this step's head rows and the next step's
// layer-0 o / layer-1 QKV slices.
template <int M, bool FIRST, bool LAST, bool Q4>
__device__ __forceinline__ void decoder_layer(Ctx& c, int l, int step, int pos0, PreT<Q4>& r) {
  const DecFrameArgs& p = c.p;
  Lds& L = c.L;
  c.refresh();
  // FIRST: RoPE (cos, sin) of this step's positions, loaded with the layer's first loads and staged
  // in LDS for the QKV epilogues of every layer (no global round trip before a QKV publish)
  float2 rp = make_float2(0.f, 0.f);
  if (FIRST && c.tid < M * (HD / 2))
    rp = reinterpret_cast<const float2*>(p.rope)[(size_t)pos0 * (HD / 2) + c.tid];
  if (FIRST && step > 1) {
    // q | k | v of input row proj_tab[step - 1][code] at position `step`, and the row itself; both
    // loads are in flight together, ahead of the down prefetch (vmcnt retires in issue order)
    const float* t = p.qkv0_tab + ((size_t)(step - 1) * p.V + c.code) * QKV;
    const float* xr = p.proj_tab + ((size_t)(step - 1) * p.V + c.code) * D;
#if DF_TAB16
    // DF_TAB16: the two rows as 16-B loads (640 float4: q|k|v 0..383, x 384..639; thread t takes
    // float4 t and, t < 128, float4 512 + t), one round trip, fewer load instructions
    constexpr int NQ4 = QKV / 4, NX4 = D / 4;
    const float4* t4 = reinterpret_cast<const float4*>(t);
    const float4* x4 = reinterpret_cast<const float4*>(xr);
    const int i0 = c.tid, i1 = NT + c.tid;
    const float4 va = i0 < NQ4 ? t4[i0] : x4[i0 - NQ4];
    const float4 vb = i1 < NQ4 + NX4 ? x4[min(i1, NQ4 + NX4 - 1) - NQ4] : make_float4(0.f, 0.f, 0.f, 0.f);
    ld_dn<Q4>(c, l, r);
    auto put4 = [&](int i, const float4 v) {
      if (i < NQ4) {
        qkv_place(c, 0, 4 * i, pos0, v.x);
        qkv_place(c, 0, 4 * i + 1, pos0, v.y);
        qkv_place(c, 0, 4 * i + 2, pos0, v.z);
        qkv_place(c, 0, 4 * i + 3, pos0, v.w);
      } else {
        *reinterpret_cast<float4*>(&L.x[0][4 * (i - NQ4)]) = v;
      }
    };
    put4(i0, va);
    if (i1 < NQ4 + NX4) put4(i1, vb);
#else
    float tv[(QKV + NT - 1) / NT], xv[D / NT];
#pragma unroll
    for (int j = 0; j < (QKV + NT - 1) / NT; ++j) tv[j] = c.tid + j * NT < QKV ? t[c.tid + j * NT] : 0.f;
#pragma unroll
    for (int j = 0; j < D / NT; ++j) xv[j] = xr[c.tid + j * NT];
    load_dn(c, l, r.wd);
#pragma unroll
    for (int j = 0; j < (QKV + NT - 1) / NT; ++j)
      if (c.tid + j * NT < QKV) {
        if (DF_KVDIRECT) qkv_place(c, 0, c.tid + j * NT, pos0, tv[j]);
        else L.qkv[0][c.tid + j * NT] = tv[j];
      }
#pragma unroll
    for (int j = 0; j < D / NT; ++j) L.x[0][c.tid + j * NT] = xv[j];
#endif
    if (c.tid < M * (HD / 2)) L.rope[c.tid / (HD / 2)][c.tid % (HD / 2)] = rp;
    __syncthreads();  // L.qkv complete before kv_append reads it
    if (!DF_KVDIRECT) {
      kv_append<M>(c, pos0);
      __syncthreads();
    }
  } else {
    KvRegs kv;
    if (FIRST && c.tid < M * (HD / 2)) L.rope[c.tid / (HD / 2)][c.tid % (HD / 2)] = rp;
    // layers >= 1 (folded): the previous layer's E5 gather already wrote xn = x * n1
    if constexpr (Q4) {
      if (FIRST) rms_rows4<M>(c, r.nw1);               // (its barriers also publish the RoPE rows)
      phase_qkv4<M, !FIRST>(c, pos0, r.wq);            // -> E1
    } else {
      if (FIRST || !DF_FOLD) rms_rows<M>(c, r.nw1);  // (its barriers also publish the RoPE rows)
      phase_qkv<M, DF_FOLD && !FIRST>(c, pos0, r.wq);   // -> E1
    }
    // prefetches issued after the publish (its RoPE operand load would otherwise retire behind
    // them in vmcnt order), still ahead of the hand-off wait they hide under
    kv_issue(c, l, pos0, kv);
    if ((FIRST || !DF_DN_EARLY) && !DF_DN_AFTER_E1) ld_dn<Q4>(c, l, r);
#if DF_KVDIRECT
    gather_qkv<M>(c, c.rbuf(G_QKV, MAXM * QKV), pos0, kv);  // (its barrier publishes the history too)
    ++c.e;
#else
    gather<(M * QKV + NT - 1) / NT>(c, c.rbuf(G_QKV, MAXM * QKV), M * QKV, &L.qkv[0][0]);
    ++c.e;
    kv_store(c, pos0, kv);
    kv_append<M>(c, pos0);
    __syncthreads();
#endif
  }
  c.refresh();
  c.mark();
  const float2 nw2 = nw_fetch(c, p.n2[l]);
  // DF_DN_AFTER_E1: the down slices issued after the q|k|v wait (not ahead of it) on layers that wait
  if constexpr (!Q4) {
    if (DF_DN_AFTER_E1 && !(FIRST && step > 1)) load_dn(c, l, r.wd);
    if (FIRST || DF_GU_E45 == 0) load_gu<0, GU_EARLY>(c, l, r.wg);  // (layers >= 1: rows < DF_GU_E45 came at E4 / E5)
    else if (DF_GU_E45 < GU_EARLY) load_gu<DF_GU_E45, GU_EARLY>(c, l, r.wg);
  } else {
    ld_gu<Q4, true>(c, l, r);
  }
  phase_attn<M, Q4>(c, pos0, l);
  if (DF_ATTN_SUB == 0) c.mark();
  if constexpr (Q4) phase_o4<M>(c, r.wo);             // -> E3
  else phase_o<M>(c, r.wo);
  c.mark();
  ld_gu<Q4, false>(c, l, r);
  if (!LAST) { ld_qkv<Q4>(c, l + 1, r); ld_o<Q4>(c, l + 1, r); }
#if DF_FOLD
  if constexpr (Q4) gather_x4<M, DF_DELAY_E3>(c, c.rbuf(G_X, MAXM * D), nw2);  // E3 -> x, xq = x * n2
  else gather_x<M, DF_DELAY_E3>(c, c.rbuf(G_X, MAXM * D), nw2);  // E3 -> x, xn = x * n2
#else
  gather<M * D / NT>(c, c.rbuf(G_X, MAXM * D), M * D, &L.x[0][0]);
#endif
  ++c.e;
  c.refresh();
  if (!DF_FOLD) rms_rows<M>(c, nw2);
  if constexpr (Q4) phase_mlp4<M, true>(c, r.wg, r.wd);  // -> E4
  else phase_mlp<M, DF_FOLD>(c, r.wg, r.wd);                // -> E4
  // DF_DN_EARLY: the next layer's down slices stream during this layer's E4 / E5 (its registers
  // were just consumed) instead of during the next E1 wait
  if constexpr (!Q4) {
    if (DF_DN_EARLY && !LAST) load_dn(c, l + 1, r.wd);
    if (DF_GU_E45 > 0 && !LAST) load_gu<0, DF_GU_E45>(c, l + 1, r.wg);
  }
  r.nw1 = nw_fetch(c, LAST ? p.norm : p.n1[l + 1]);  // next layer's norm, or the final one
  c.mark();
  if (LAST) {
    load_head(c, p.audio_head + (size_t)(step - 1) * p.VP * D, D, r.wh);
    if (step + 1 < p.K) {
      ld_o<Q4>(c, 0, r);
      ld_qkv<Q4>(c, 1, r);
    }
  }
  c.refresh();
  phase_reduce<M>(c);                                 // waits E4, -> E5
#if DF_FOLD
  if constexpr (Q4) gather_x4<M, DF_DELAY_E5>(c, c.rbuf(G_X, MAXM * D), r.nw1);  // E5 -> x, xq
  else gather_x<M, DF_DELAY_E5>(c, c.rbuf(G_X, MAXM * D), r.nw1);  // E5 -> x, xn = x * (next n1 | final norm)
#else
  gather<M * D / NT>(c, c.rbuf(G_X, MAXM * D), M * D, &L.x[0][0]);
#endif
  ++c.e;
}

// One decoder step (generation.py:72-90): 4 layers over the step's M rows, the ci head, the arg-max.
template <int M, bool Q4>
__device__ __forceinline__ void run_step(Ctx& c, int step, PreT<Q4>& r) {
  const DecFrameArgs& p = c.p;
  const int pos0 = M == 2 ? 0 : step;  // step 1: positions 0, 1
  decoder_layer<M, true, false, Q4>(c, 0, step, pos0, r);
  for (int l = 1; l < NL - 1; ++l) decoder_layer<M, false, false, Q4>(c, l, step, pos0, r);
  decoder_layer<M, false, true, Q4>(c, NL - 1, step, pos0, r);
  // ci head on the last row: final norm, audio_head[step - 1] (generation.py:79)
  c.refresh();
#if DF_FOLD
  phase_head<D, Q4>(c, p.audio_head + (size_t)(step - 1) * p.VP * D, p.V, r.wh.a, r.wh.x, p.ci_logits + (size_t)(step - 1) * p.VP,
                    step, M - 1, row_rs(c, M - 1));  // -> E6
#else
  rms_rows<1>(c, r.nw1, M - 1);
  phase_head<D>(c, p.audio_head + (size_t)(step - 1) * p.VP * D, p.V, r.wh.a, r.wh.x, p.ci_logits + (size_t)(step - 1) * p.VP, step);  // -> E6
#endif
  KvRegs kv0;  // layer 0's cached K/V rows of the next step: in flight during the head's hand-off,
  if (step + 1 < p.K) kv_issue(c, 0, step + 1, kv0);
  const int ci = head_code(c, p.V, step);
  ++c.e;
  if (c.w == 0 && c.tid == 0) p.codes[step] = ci;
  if (step + 1 < p.K) kv_store(c, step + 1, kv0);  // and in LDS before the loop back-edge
}

// Frame start of the int4 kernel: codebook0_head (one 2048-wide row per wave: a chunk per lane) and the
// projection of h_last (waves 0-3, rows 4w + v) against h_last staged in the padded layout -> the same
// two hand-offs as the bf16 kernel's frame start
__device__ __forceinline__ void frame_start4(Ctx& c) {
  const DecFrameArgs& p = c.p;
  Lds& L = c.L;
  const char* H = reinterpret_cast<const char*>(p.c0_head);
  const char* P = reinterpret_cast<const char*>(p.proj);
  const int sbh = p.VP * RBH;  // codebook0_head's affine words follow its VP rows of nibbles
  const u32x4_t ha = bload(H, c.wave * RBH + c.lane * 16, 8 * c.w * RBH);
  const unsigned hs = bload4(H, c.wave * SBRH + (c.lane >> 1) * 4, sbh + 8 * c.w * SBRH);
  u32x4_t hx = {0u, 0u, 0u, 0u};
  unsigned hxs = 0u;
  if (c.wave == 0 && c.w < 3) {
    hx = bload(H, c.lane * 16, (2048 + c.w) * RBH);
    hxs = bload4(H, (c.lane >> 1) * 4, sbh + (2048 + c.w) * SBRH);
  }
  const int pw = min(c.wave, 3);  // waves 4-7 re-read row 4w + 3 (no branch around a load; unused)
  const u32x4_t pa = bload(P, pw * RBH + c.lane * 16, 4 * c.w * RBH);
  const unsigned ps = bload4(P, pw * SBRH + (c.lane >> 1) * 4, SB_PROJ + 4 * c.w * SBRH);
  // h_last -> hq (padded), hh: thread t stages elements 2t, 2t + 1 and 1024 + 2t, + 1
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = h * (DB / 2) + 2 * c.tid;
    const float2 v = *reinterpret_cast<const float2*>(p.h_last + k);
    *reinterpret_cast<float2*>(&L.h0.hq[0][0] + q4p(k)) = v;
    float sum = v.x + v.y;
    sum += __shfl_xor(sum, 1, 64);
    sum += __shfl_xor(sum, 2, 64);
    sum += __shfl_xor(sum, 4, 64);
    sum += __shfl_xor(sum, 8, 64);
    if ((c.tid & 15) == 0) L.h0.hh[k >> 5] = sum;
  }
  __syncthreads();
  const float s = wave_sum(q4dot32(ha, L.h0.hq[c.lane], hs, L.h0.hh[c.lane]));
  float t = 0.f;
  if (c.wave == 0 && c.w < 3) t = wave_sum(q4dot32(hx, L.h0.hq[c.lane], hxs, L.h0.hh[c.lane]));
  head_publish(c, s, t, p.V, p.c0_logits, 0);  // -> G_ARG (hand-off 0)
  const float pv = wave_sum(q4dot32(pa, L.h0.hq[c.lane], ps, L.h0.hh[c.lane]));
  if (c.lane == 0 && c.wave < 4) L.wsum[c.wave][0] = pv;
  __syncthreads();
  if (c.tid < 4 * REP) {
    const int q = c.tid / REP;
    c.put(G_X, MAXM * D, 4 * c.w + q, L.wsum[q][0], c.tid % REP);
  }
}
}  // namespace

template <bool Q4>
__global__ __launch_bounds__(NT, 1) void dec_frame_kernel(DecFrameArgs p) {
  __shared__ __attribute__((aligned(16))) Lds L;
  Ctx c{p, L, (int)blockIdx.x, (int)threadIdx.x, (int)(threadIdx.x & 63), (int)(threadIdx.x >> 6), 0u, 0};
  c.tag0 = __hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  if (p.stamps && c.tid == 0) p.stamps[(size_t)c.w * DEC_FRAME_STAMPS + DEC_FRAME_STAMPS - 2] = __builtin_amdgcn_s_memrealtime();
  PreT<Q4> r;
  if constexpr (Q4) {
    ld_qkv<Q4>(c, 0, r);
    ld_o<Q4>(c, 0, r);
    frame_start4(c);
  } else {
  // ---- frame start: codebook0_head (K = 2048, 8 rows per WG + 1 for WGs 0-2) and the projection of
  // h_last (rows 4w..4w+3) for decoder step 1, both published in one hand-off
  u32x4_t c0a[4], c0x[4], pa[2];
  {
    const bf16_t* row = p.c0_head + (size_t)(8 * c.w) * DB;
#pragma unroll
    for (int i = 0; i < 4; ++i) c0a[i] = bload(row, (c.wave * DB + 8 * c.lane) * 2, i * 1024);
    if (c.wave == 0 && c.w < 3) {
      const bf16_t* xr = p.c0_head + (size_t)(2048 + c.w) * DB;
#pragma unroll
      for (int i = 0; i < 4; ++i) c0x[i] = bload(xr, 16 * c.lane, i * 1024);
    }
    const bf16_t* pr = p.proj + (size_t)(4 * c.w) * DB;
    const int pv = ((c.wave >> 1) * DB + 8 * 128 * (c.wave & 1) + 8 * c.lane) * 2;
    pa[0] = bload(pr, pv, 0);
    pa[1] = bload(pr, pv, 1024);
  }
  load_qkv(c, 0, r.wq);
  load_o(c, 0, r.wo);
  for (int k = c.tid; k < DB; k += NT) L.xn[0][k] = p.h_last[k];
  __syncthreads();
  phase_head<DB>(c, p.c0_head, p.V, c0a, c0x, p.c0_logits, 0);  // -> G_ARG (hand-off 0)
  {
    float s = dot8(pa[0], L.xn[0] + 8 * (128 * (c.wave & 1) + c.lane)) + dot8(pa[1], L.xn[0] + 8 * (128 * (c.wave & 1) + c.lane + 64));
    s = wave_sum(s);
    if (c.lane == 0) L.wsum[c.wave][0] = s;
    __syncthreads();
    if (c.tid < 4 * REP) {
      const int q = c.tid / REP;
      c.put(G_X, MAXM * D, 4 * c.w + q, L.wsum[2 * q][0] + L.wsum[2 * q + 1][0], c.tid % REP);
    }
  }
  }
  const int c0 = head_code(c, p.V, 0);
  gather<2>(c, c.rbuf(G_X, MAXM * D), D, L.x[0]);  // x row 0 = projection(h_last)
  ++c.e;
  if (c.w == 0 && c.tid == 0) p.codes[0] = c0;
  // x row 1 = projection(E_a[c0]) from the folded table (bit-identical to the projection GEMV)
  for (int k = c.tid; k < D; k += NT) L.x[1][k] = p.proj_tab[(size_t)c0 * D + k];
  __syncthreads();

  // Register prefetch schedule (what is in flight during each hand-off wait):
  //   E1 (q|k|v): the cached K/V rows, this layer's down slices (issued after the QKV publish)
  //   E3 (x): this layer's gate/up slices, next layer's QKV / o
  //   E4 / E5 of the last layer: this step's head rows, the next step's o / QKV
  //   E6: the next step's layer-0 cached K/V rows
  // The first and last layers of a step are peeled out of the layer loop (decoder_layer<FIRST,
  // LAST>): a prefetch that crosses a step boundary (layer-0 K/V rows, head rows) is then live only
  // between its issue and its use, not around a loop back-edge, where it would hold its registers
  // through every layer and spill.
  r.nw1 = nw_fetch(c, p.n1[0]);  // RMSNorm weights, fetched a phase ahead of use
  // step 1 carries two rows ([h_last, E_a[c0]]), steps >= 2 one: each its own instantiation, so the
  // one-row steps compute and read nothing for a second row
  run_step<2, Q4>(c, 1, r);
  for (int step = 2; step < p.K; ++step) run_step<1, Q4>(c, step, r);
  if (p.stamps && c.tid == 0) p.stamps[(size_t)c.w * DEC_FRAME_STAMPS + DEC_FRAME_STAMPS - 1] = __builtin_amdgcn_s_memrealtime();
  if (c.w == 0 && c.tid == 0) __hip_atomic_store(p.epoch, c.tag0 - 1u + (unsigned)c.e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

size_t dec_frame_gbuf_bytes() { return G_TOTAL * sizeof(u64); }

void launch_dec_frame(const DecFrameArgs& p, hipStream_t st, bool q4) {
  if (q4) hipLaunchKernelGGL(dec_frame_kernel<true>, dim3(NWG), dim3(NT), 0, st, p);
  else hipLaunchKernelGGL(dec_frame_kernel<false>, dim3(NWG), dim3(NT), 0, st, p);
}

const void* dec_frame_kernel_ptr(bool q4) {
  return q4 ? reinterpret_cast<const void*>(&dec_frame_kernel<true>) : reinterpret_cast<const void*>(&dec_frame_kernel<false>);
}
