// Shared device helpers for the CSM / Mimi HIP kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CSM_WAVE 64

typedef uint16_t bf16_t;  // raw bf16 bits; weights are stored as bf16 or f32

__device__ __forceinline__ float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ float bf16_to_f32(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// Load 8 consecutive weights starting at p (16-B aligned for bf16, 32-B for f32) as floats.
template <typename WT> struct W8;
template <> struct W8<bf16_t> {
  __device__ __forceinline__ static void load(const bf16_t* p, float (&w)[8]) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    w[0] = bf16_lo(u.x); w[1] = bf16_hi(u.x); w[2] = bf16_lo(u.y); w[3] = bf16_hi(u.y);
    w[4] = bf16_lo(u.z); w[5] = bf16_hi(u.z); w[6] = bf16_lo(u.w); w[7] = bf16_hi(u.w);
  }
  // streamed-once weights: non-temporal 16-B load (does not displace re-read lines in L2/MALL)
  __device__ __forceinline__ static void load_nt(const bf16_t* p, float (&w)[8]) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 u = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    w[0] = bf16_lo(u.x); w[1] = bf16_hi(u.x); w[2] = bf16_lo(u.y); w[3] = bf16_hi(u.y);
    w[4] = bf16_lo(u.z); w[5] = bf16_hi(u.z); w[6] = bf16_lo(u.w); w[7] = bf16_hi(u.w);
  }
};
template <> struct W8<float> {
  __device__ __forceinline__ static void load(const float* p, float (&w)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
  }
  __device__ __forceinline__ static void load_nt(const float* p, float (&w)[8]) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    const f32x4 a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    const f32x4 b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 4));
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
  }
};

// 8 consecutive weights held raw in VGPRs (loaded early, converted at use): 16 B bf16 / 32 B f32.
template <typename WT> struct Raw8;
template <> struct Raw8<bf16_t> {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 u;
  template <bool NT> __device__ __forceinline__ void load(const bf16_t* p) {
    if constexpr (NT) u = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else u = *reinterpret_cast<const u32x4*>(p);
  }
  __device__ __forceinline__ void get(float (&w)[8]) const {
    w[0] = bf16_lo(u.x); w[1] = bf16_hi(u.x); w[2] = bf16_lo(u.y); w[3] = bf16_hi(u.y);
    w[4] = bf16_lo(u.z); w[5] = bf16_hi(u.z); w[6] = bf16_lo(u.w); w[7] = bf16_hi(u.w);
  }
};
template <> struct Raw8<float> {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  f32x4 a, b;
  template <bool NT> __device__ __forceinline__ void load(const float* p) {
    if constexpr (NT) {
      a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
      b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 4));
    } else {
      a = *reinterpret_cast<const f32x4*>(p);
      b = *reinterpret_cast<const f32x4*>(p + 4);
    }
  }
  __device__ __forceinline__ void get(float (&w)[8]) const {
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
  }
};

template <typename WT> __device__ __forceinline__ float ld1(const WT* p);
template <> __device__ __forceinline__ float ld1<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld1<bf16_t>(const bf16_t* p) { return bf16_to_f32(*p); }

template <typename T> __device__ __forceinline__ T st_cast(float v);
template <> __device__ __forceinline__ float st_cast<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t st_cast<bf16_t>(float v) {
  uint32_t u = __float_as_uint(v);
  u = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;  // RNE (inputs are finite)
  return (bf16_t)u;
}

// Wave reductions without LDS round trips: each row of 16 lanes reduced by DPP (rotations by 8
// and 4, then quad swaps), the four row results combined from lanes 0 / 16 / 32 / 48 by readlane in
// a fixed order -- every lane returns the same value (all 64 lanes must be active).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float lane_f(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0x128>(v);  // row_ror:8
  v += dpp_f<0x124>(v);  // row_ror:4
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_f<0x128>(v));
  v = fmaxf(v, dpp_f<0x124>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0xB1>(v));
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float gelu_tanh_f(float x) {
  const float c = 0.7978845608028654f;  // sqrt(2/pi)
  return 0.5f * x * (1.0f + tanhf(c * (x + 0.044715f * x * x * x)));
}
__device__ __forceinline__ float gelu_erf_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.7071067811865476f)); }
__device__ __forceinline__ float elu_f(float x) { return x > 0.f ? x : expm1f(x); }

// Row -> (utterance, position) map shared by the projection epilogues and attention.
//   b(m)   = b_off + m / T
//   pos(m) = (pos_arr ? pos_arr[b(m)] : 0) + pos_const + m % T
struct RowMap {
  int T;
  int b_off;
  const int* pos_arr;
  int pos_const;
  // ragged batched prefill: per-row utterance and position tables (device), overriding the above
  const int* row_b = nullptr;
  const int* row_pos = nullptr;
  // prompt-prefill attention (attn_prefill_kernel): runs of <= 64 rows of one utterance at consecutive
  // positions, {first row, rows} (device; null: attn_block per row)
  const int2* tiles = nullptr;
  int ntiles = 0;
  __device__ __forceinline__ int b(int m) const { return row_b ? row_b[m] : b_off + m / T; }
  __device__ __forceinline__ int pos(int m) const {
    if (row_pos) return row_pos[m];
    const int bb = b(m);
    return (pos_arr ? pos_arr[bb] : 0) + pos_const + m % T;
  }
};

// splitmix64 -- the sampler's counter-based RNG (restated in oracle/csm_oracle.py:gumbel_u)
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// ---------------------------------------------------------------------------- int4 (MLX affine, g64)
// Device layout of a quantized [N][K] matrix (one allocation): nibbles [N][K/2] (element k of a row in
// byte k/2, low nibble for even k -- MLX's uint32 packing read as bytes), then per group of 64 a
// uint32 {lo16 = scale bf16, hi16 = bias bf16} [N][K/64].  w_hat = scale * q + bias.
constexpr int Q4_GROUP = 64;
__host__ __device__ __forceinline__ size_t q4_bytes(size_t N, size_t K) { return N * K / 2 + N * (K / Q4_GROUP) * 4; }
__host__ __device__ __forceinline__ size_t q4_sb_offset(size_t N, size_t K) { return N * K / 2; }

// 8 dequantized weights of row r starting at k (k % 8 == 0) of a quantized matrix with N rows
__device__ __forceinline__ void q4_load8(const uint8_t* base, size_t N, int K, size_t r, int k, float (&w)[8]) {
  const uint32_t q = *reinterpret_cast<const uint32_t*>(base + r * (K / 2) + k / 2);
  const uint32_t sb = reinterpret_cast<const uint32_t*>(base + q4_sb_offset(N, K))[r * (K / Q4_GROUP) + k / Q4_GROUP];
  const float s = bf16_lo(sb), b = bf16_hi(sb);
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = fmaf(s, (float)((q >> (4 * j)) & 15u), b);
}
