// Inter-workgroup hand-off primitives of the persistent kernels (dec_frame.hip, bb_step.hip).
// A value travels as one naturally aligned 8-byte granule {fp32 bits, tag} written by ONE agent-scope
// relaxed (sc1) store and read with agent-scope relaxed (sc1) loads until the tag matches
// (MI355X_MICROARCH.md, inter-workgroup visibility and the hand-off price list).
#pragma once
#include "common.h"

namespace handoff {

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

__device__ __forceinline__ u64 gload(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gput(u64* p, float v, unsigned tag) {
  __hip_atomic_store(p, ((u64)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gput_u(u64* p, unsigned v, unsigned tag) {
  __hip_atomic_store(p, ((u64)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sc1_store_f(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 16-B agent-coherent (sc1) load at byte offset `off` of a buffer of `bytes` bytes
__device__ __forceinline__ u32x4_t sc1_load16(const void* base, int off, int bytes) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
  return __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16));
}

// 8 products of one 16-B bf16 weight chunk with 8 consecutive fp32 activations (fixed order)
__device__ __forceinline__ float dot8(const u32x4_t w, const float* x) {
  const float4 a = *reinterpret_cast<const float4*>(x), b = *reinterpret_cast<const float4*>(x + 4);
  float s = bf16_lo(w.x) * a.x;
  s = fmaf(bf16_hi(w.x), a.y, s);
  s = fmaf(bf16_lo(w.y), a.z, s);
  s = fmaf(bf16_hi(w.y), a.w, s);
  s = fmaf(bf16_lo(w.z), b.x, s);
  s = fmaf(bf16_hi(w.z), b.y, s);
  s = fmaf(bf16_lo(w.w), b.z, s);
  s = fmaf(bf16_hi(w.w), b.w, s);
  return s;
}

// 16-B weight load as a raw buffer load: the matrix base rides in the (uniform) descriptor, the
// lane-dependent part in ONE voffset register shared by every layer and row, the row / chunk step in
// the scalar offset -- so per-layer weight addresses are not VGPR pairs the compiler keeps live
// across the frame loop.
// AUX: cache policy (2 = nt), a compile-time constant so no load sits in a branch of its own.
template <int AUX = 0>
__device__ __forceinline__ u32x4_t bload(const void* base, int voff, int soff) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
  return __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, AUX));
}

// Wait until this thread's granules base[off[u]] (u < GPT, val[u]) carry `tag`, then use(probe).
// TWO: two probes in flight, the second issued GAP sleeps after the first, each re-issued whole as
// soon as its predecessor returns stale -- a probe returns every half round trip, so a hand-off is
// seen about a quarter round trip sooner than by one probe re-polled on its return.  Every load is
// unconditional (an unused entry reads granule 0 and counts as current) and use() runs on the exit
// the matched probe left by: no branch around a load and no copy of a probe's registers at a merge,
// so the compiler's vmcnt waits stay exact (a check waits for its own probe, the other stays in
// flight).  A granule's tag only moves from stale to current during a wait (its buffer is rewritten
// only after every workgroup has published the next hand-off), so any all-current probe is the
// hand-off.  fail(spin): the bounded-spin / error-flag test.  DELAY: sleeps before the first probe
// (fewer wasted probes while the producers are still working); REPOLL: sleeps between re-polls.
// Measured (profiles/r03_ab_poll.txt): TWO costs the frame decoder +12 % (every re-issued probe adds
// sc1 traffic on the lines every workgroup polls), so both kernels keep one probe.
template <int GPT, bool TWO, int GAP, int DELAY, int REPOLL, typename Fail, typename F>
__device__ __forceinline__ void poll_granules(const u64* base, const int (&off)[GPT], const bool (&val)[GPT], unsigned tag,
                                              Fail&& fail, F&& use) {
  auto cur = [&](const u64 (&x)[GPT]) {
    bool ok = true;
#pragma unroll
    for (int u = 0; u < GPT; ++u) ok &= !val[u] || (unsigned)(x[u] >> 32) == tag;
    return ok;
  };
  auto probe = [&](u64 (&x)[GPT]) {
#pragma unroll
    for (int u = 0; u < GPT; ++u) x[u] = gload(base + (val[u] ? off[u] : 0));
  };
  if constexpr (DELAY > 0) __builtin_amdgcn_s_sleep(DELAY);
  if constexpr (TWO) {
    u64 a[GPT], b[GPT];
    probe(a);
    __builtin_amdgcn_s_sleep(GAP);
    probe(b);
    for (unsigned spin = 0;; spin += 2) {
      if (cur(a) || fail(spin)) {
        use(a);
        break;
      }
      probe(a);
      if (cur(b)) {
        use(b);
        break;
      }
      probe(b);
    }
  } else {
    u64 g[GPT];
    probe(g);
    for (unsigned spin = 0; !cur(g) && !fail(spin); ++spin) {
      __builtin_amdgcn_s_sleep(REPOLL);
#pragma unroll
      for (int u = 0; u < GPT; ++u)
        if (val[u] && (unsigned)(g[u] >> 32) != tag) g[u] = gload(base + off[u]);
    }
    use(g);
  }
}

// poll_granules over granule PAIRS: one 16-B sc1 load per pair (granules 2i, 2i + 1: their tags in
// words 1 and 3), pair offsets in granules (even).  Same protocol and vmcnt discipline as
// poll_granules (one probe, stale pairs re-polled); use(x) gets the u32x4 of every pair.
// Tearing: correctness needs each naturally aligned 8-B half of a 16-B sc1 load (and of a producer's
// 16-B sc1 store of two granules) to be seen whole, never a fresh tag beside a stale value.  The HIP /
// HSA memory model promises that only for aligned atomics of <= 8 B; on gfx950 under ROCm 7.2 16-B
// sc1 accesses are observed untorn at 8-B halves, not as an architectural guarantee
// (/opt/skills/guides/MI355X_MICROARCH.md, inter-workgroup visibility: "R2's granule ... also for 16-B
// sc1 halves").  The guard is the data: the 125-frame bf16 fixtures (tests/test_long_gpu.py) and the
// determinism checks (tests/test_dec_frame_gpu.py) run every frame through these polls, and a torn
// read would put a stale partial into a sum and change codes or logits.
template <int GPP, int DELAY, int REPOLL, typename Fail, typename F>
__device__ __forceinline__ void poll_pairs(const u64* base, int bytes, const int (&off)[GPP], unsigned tag, Fail&& fail, F&& use) {
  auto cur1 = [&](const u32x4_t& x) { return x.y == tag && x.w == tag; };
  if constexpr (DELAY > 0) __builtin_amdgcn_s_sleep(DELAY);
  u32x4_t g[GPP];
#pragma unroll
  for (int u = 0; u < GPP; ++u) g[u] = sc1_load16(base, off[u] * 8, bytes);
  for (unsigned spin = 0;; ++spin) {
    bool ok = true;
#pragma unroll
    for (int u = 0; u < GPP; ++u) ok &= cur1(g[u]);
    if (ok || fail(spin)) break;
    __builtin_amdgcn_s_sleep(REPOLL);
#pragma unroll
    for (int u = 0; u < GPP; ++u)
      if (!cur1(g[u])) g[u] = sc1_load16(base, off[u] * 8, bytes);
  }
  use(g);
}

// ---- int4 (MLX affine, group 64; common.h layout) weight chunks for the persistent kernels
// 4-B raw buffer load (an int4 group's {scale, bias} word), descriptor as bload
template <int AUX = 0>
__device__ __forceinline__ unsigned bload4(const void* base, int voff, int soff) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, AUX);
}
// One 16-B chunk of 32 nibbles (a half group: word i holds elements 8i .. 8i + 7, byte b elements 8i + 2b
// (low nibble) and 8i + 2b + 1) against 32 consecutive fp32 activations x (LDS), with that half group's
// affine word sb and activation sum hs: scale * sum_j q_j x_j + bias * sum_j x_j (the int4 GEMV's
// per-half-group arithmetic, q4_kernels.hip gemv_q4_kernel).
__device__ __forceinline__ float q4dot32(const u32x4_t w, const float* x, unsigned sb, float hs) {
  float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const unsigned u = w[i], lo = u & 0x0F0F0F0Fu, hi = (u >> 4) & 0x0F0F0F0Fu;
    const float4 a = *reinterpret_cast<const float4*>(x + 8 * i), b = *reinterpret_cast<const float4*>(x + 8 * i + 4);
    d0 = fmaf((float)(lo & 0xFFu), a.x, d0);
    d1 = fmaf((float)(hi & 0xFFu), a.y, d1);
    d2 = fmaf((float)((lo >> 8) & 0xFFu), a.z, d2);
    d3 = fmaf((float)((hi >> 8) & 0xFFu), a.w, d3);
    d0 = fmaf((float)((lo >> 16) & 0xFFu), b.x, d0);
    d1 = fmaf((float)((hi >> 16) & 0xFFu), b.y, d1);
    d2 = fmaf((float)(lo >> 24), b.z, d2);
    d3 = fmaf((float)(hi >> 24), b.w, d3);
  }
  return fmaf(bf16_lo(sb), (d0 + d1) + (d2 + d3), bf16_hi(sb) * hs);
}
// 8 nibbles of one word (elements j < 8, low nibble of byte b = element 2b) against x[0..7]
__device__ __forceinline__ float q4dot8(unsigned u, const float* x) {
  const unsigned lo = u & 0x0F0F0F0Fu, hi = (u >> 4) & 0x0F0F0F0Fu;
  const float4 a = *reinterpret_cast<const float4*>(x), b = *reinterpret_cast<const float4*>(x + 4);
  float s = (float)(lo & 0xFFu) * a.x;
  s = fmaf((float)(hi & 0xFFu), a.y, s);
  s = fmaf((float)((lo >> 8) & 0xFFu), a.z, s);
  s = fmaf((float)((hi >> 8) & 0xFFu), a.w, s);
  s = fmaf((float)((lo >> 16) & 0xFFu), b.x, s);
  s = fmaf((float)((hi >> 16) & 0xFFu), b.y, s);
  s = fmaf((float)(lo >> 24), b.z, s);
  s = fmaf((float)(hi >> 24), b.w, s);
  return s;
}
// Padded LDS layout of an int4 kernel's activation row: each 32-element half group 36 floats apart, so
// the 64 lanes' 16-B reads of their own half groups fall on distinct banks (gemv_q4_kernel's layout)
__device__ __forceinline__ int q4p(int k) { return (k >> 5) * 36 + (k & 31); }
// sums of lanes 0-31 and of lanes 32-63 (wave_sum's DPP row reductions, rows combined per half)
__device__ __forceinline__ float2 half_sums(float v) {
  v += dpp_f<0x128>(v);
  v += dpp_f<0x124>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0xB1>(v);
  return make_float2(lane_f(v, 0) + lane_f(v, 16), lane_f(v, 32) + lane_f(v, 48));
}

// threadIdx.x through an opaque move: lane-dependent addresses derived from it inside the frame loop
// are recomputed per iteration instead of being hoisted out of the loop and held (spilled) for the
// whole frame.
__device__ __forceinline__ int opaque_tid() {
  int t;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
  return t;
}

}  // namespace handoff
