// Split activations ("XS"): the A operand of the streaming matrix-core GEMM (gemm_xs.hip) for the
// batched depth decoder, written once by whichever kernel produces a row block and read by every
// block of the consuming projection straight into MFMA registers (no LDS staging, no per-block split).
//
// An fp32 activation x is held as three bf16 parts x = hi + mid + lo (all 24 significant bits;
// each part times a bf16 weight is exact in fp32, so three v_mfma_f32_32x32x16_bf16 per K-step give
// the fp32 product exactly -- the arithmetic of gemm_wide_kernel, gemm_kernels.hip).  The operand is
// stored in MFMA fragment order: with kk = k % 64, h = kk / 32, s = (kk % 32) / 8, j = kk % 8 and
// lane = m % 32 + 32 h, lane (r, h) of step s holds the 8 values of its v_mfma_f32_32x32x16_bf16 A
// fragment (the same in-stage K permutation as the fragment-tiled weight copy, gemm_retile) -- as
// fp32 (XS_F32, split by the consumer) or as the three parts (below).  A producer applies the consumer's RMSNorm weight
// before splitting (x * nw) and publishes per-row partial sums of squares of the un-normed x; the
// consumer scales by rsqrt(sum / K + eps) after the dot product.
#pragma once
#include "common.h"

namespace xs {

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// XS_F32 (default): the producer writes the fp32 value itself in fragment order and the consumer
// splits it into the three bf16 parts in registers (split_frag, the same split3 and packing as the
// producer-side split, so the MFMA operands and results are bit-identical).  4 bytes per element
// instead of 6: the streaming GEMM's per-CU operand intake -- what bounds it (profiles/
// r04_lab_gemm_xs_ablation.txt: the loop with no data moved is still most of the launch) -- drops by
// a third on the activation side.  Element (m, k) lives at
//   [m / 32][k / 64][s][half][lane] x 16 B, float (kk % 4) of the lane's 16 B, half = (kk % 8) / 4,
// so each of a consumer's two loads per (row tile, step) is one contiguous KB per wave.
// XS_F32 0: the three parts stored by the producer ([m / 32][k / 64][part][s][lane] x 16 B, below).
#ifndef XS_F32
#define XS_F32 1
#endif
constexpr int XS_EB = XS_F32 ? 4 : 6;  // bytes per element
constexpr int XS_PART = 4 * 64 * 16;   // (XS_F32 0) bytes between the parts of one element

// byte offset of element (m, k) (XS_F32 0: of its part 0)
__host__ __device__ __forceinline__ size_t off(int K, int m, int k) {
  const int nks = K >> 6, kk = k & 63;
  const int lane = (m & 31) + 32 * (kk >> 5);
  if constexpr (XS_F32 != 0)
    return (((((size_t)(m >> 5) * nks + (k >> 6)) * 4 + ((kk >> 3) & 3)) * 2 + ((kk >> 2) & 1)) * 64 + lane) * 16 + (kk & 3) * 4;
  return ((((size_t)(m >> 5) * nks + (k >> 6)) * 3 * 4 + ((kk >> 3) & 3)) * 64 + lane) * 16 + (kk & 7) * 2;
}
__host__ __device__ __forceinline__ size_t bytes(int M, int K) { return (size_t)((M + 31) / 32) * 32 * K * XS_EB; }

// x -> hi, mid, lo by truncation (hi = x with its low 16 bits cleared, mid the same of the exact
// remainder, lo the rest: <= 8 significant bits): x = hi + mid + lo exactly; returned as bf16 bits.
__device__ __forceinline__ void split3(float v, uint32_t& h, uint32_t& m, uint32_t& l) {
  const uint32_t u = __float_as_uint(v);
  h = u & 0xFFFF0000u;
  const float r = v - __uint_as_float(h);
  m = __float_as_uint(r) & 0xFFFF0000u;
  l = __float_as_uint(r - __uint_as_float(m));
}

// eight fp32 (k .. k+7 of one lane's fragment: a = floats 0-3, b = 4-7) -> the three bf16x8 parts
__device__ __forceinline__ void split_frag(const u32x4_t& a, const u32x4_t& b, u32x4_t (&part)[3]) {
  uint32_t h[8], md[8], l[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    split3(__uint_as_float(a[q]), h[q], md[q], l[q]);
    split3(__uint_as_float(b[q]), h[4 + q], md[4 + q], l[4 + q]);
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    part[0][d] = __builtin_amdgcn_perm(h[2 * d + 1], h[2 * d], 0x07060302u);
    part[1][d] = __builtin_amdgcn_perm(md[2 * d + 1], md[2 * d], 0x07060302u);
    part[2][d] = __builtin_amdgcn_perm(l[2 * d + 1], l[2 * d], 0x07060302u);
  }
}

// four consecutive columns k .. k+3 (k % 4 == 0) of row m: one 16-B store (XS_F32) / one 8-byte
// store per part
__device__ __forceinline__ void store4(void* base, int K, int m, int k, const float (&v)[4]) {
  uint8_t* p = reinterpret_cast<uint8_t*>(base) + off(K, m, k);
  if constexpr (XS_F32 != 0) {
    *reinterpret_cast<u32x4_t*>(p) = u32x4_t{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
    return;
  }
  uint32_t h[4], md[4], l[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) split3(v[q], h[q], md[q], l[q]);
  *reinterpret_cast<u32x2_t*>(p) =
      u32x2_t{__builtin_amdgcn_perm(h[1], h[0], 0x07060302u), __builtin_amdgcn_perm(h[3], h[2], 0x07060302u)};
  *reinterpret_cast<u32x2_t*>(p + XS_PART) =
      u32x2_t{__builtin_amdgcn_perm(md[1], md[0], 0x07060302u), __builtin_amdgcn_perm(md[3], md[2], 0x07060302u)};
  *reinterpret_cast<u32x2_t*>(p + 2 * XS_PART) =
      u32x2_t{__builtin_amdgcn_perm(l[1], l[0], 0x07060302u), __builtin_amdgcn_perm(l[3], l[2], 0x07060302u)};
}

// eight consecutive columns k .. k+7 (k % 8 == 0) of row m: two 16-B stores (XS_F32) / one lane's
// whole 16-B fragment per part
__device__ __forceinline__ void store8(void* base, int K, int m, int k, const float (&v)[8]) {
  if constexpr (XS_F32 != 0) {
    store4(base, K, m, k, {v[0], v[1], v[2], v[3]});
    store4(base, K, m, k + 4, {v[4], v[5], v[6], v[7]});
    return;
  }
  uint32_t h[8], md[8], l[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) split3(v[q], h[q], md[q], l[q]);
  uint8_t* p = reinterpret_cast<uint8_t*>(base) + off(K, m, k);
  *reinterpret_cast<u32x4_t*>(p) = u32x4_t{__builtin_amdgcn_perm(h[1], h[0], 0x07060302u), __builtin_amdgcn_perm(h[3], h[2], 0x07060302u),
                                          __builtin_amdgcn_perm(h[5], h[4], 0x07060302u), __builtin_amdgcn_perm(h[7], h[6], 0x07060302u)};
  *reinterpret_cast<u32x4_t*>(p + XS_PART) =
      u32x4_t{__builtin_amdgcn_perm(md[1], md[0], 0x07060302u), __builtin_amdgcn_perm(md[3], md[2], 0x07060302u),
              __builtin_amdgcn_perm(md[5], md[4], 0x07060302u), __builtin_amdgcn_perm(md[7], md[6], 0x07060302u)};
  *reinterpret_cast<u32x4_t*>(p + 2 * XS_PART) =
      u32x4_t{__builtin_amdgcn_perm(l[1], l[0], 0x07060302u), __builtin_amdgcn_perm(l[3], l[2], 0x07060302u),
              __builtin_amdgcn_perm(l[5], l[4], 0x07060302u), __builtin_amdgcn_perm(l[7], l[6], 0x07060302u)};
}

// one element (a 4-byte store / a 2-byte store per part)
__device__ __forceinline__ void store1(void* base, int K, int m, int k, float v) {
  if constexpr (XS_F32 != 0) {
    *reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(base) + off(K, m, k)) = v;
    return;
  }
  uint32_t h, md, l;
  split3(v, h, md, l);
  uint16_t* p = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(base) + off(K, m, k));
  p[0] = (uint16_t)(h >> 16);
  p[XS_PART / 2] = (uint16_t)(md >> 16);
  p[XS_PART] = (uint16_t)(l >> 16);
}

// int4 consumers (MLX affine, w = scale * q + bias per group of 64 k) need the group sums
// X_g = sum_{k in g} a[m][k] of the split rows (the bias term): producers also publish half-group
// sums hs[k / 32][HS_ROWS] (32 columns, summed in column order), the consumer adds the two halves.
constexpr int HS_ROWS = 64;

// one uint32 of MLX int4 nibbles (k = 8s .. 8s+7, low nibble first) -> 8 exact bf16 (u32x4 of pairs).
// The even / odd nibbles' bytes are interleaved by v_perm and decoded as fp8 e4m3: a byte q in 0..15 is
// q x 2^-9 there exactly (exponent field q >> 3 = 0 (subnormal) or 1, mantissa q & 7: (q & 7) / 8 x 2^-6
// and (1 + (q & 7) / 8) x 2^-6), and v_cvt_scalef32_pk_bf16_fp8 with the power-of-two scale 2^9 returns q
// itself -- 9 vector ops a word instead of 15 (8 v_cvt_f32_ubyte + 4 v_perm + masks).  Q4_FP8=0: the
// byte -> float path (lab A/B).
#ifndef Q4_FP8
#define Q4_FP8 1
#endif
__device__ __forceinline__ u32x4_t q4_word_bf16(uint32_t u) {
  const uint32_t a = u & 0x0F0F0F0Fu, b = (u >> 4) & 0x0F0F0F0Fu;
  u32x4_t o;
  if constexpr (Q4_FP8 != 0) {
    typedef __bf16 v2bf16_t __attribute__((ext_vector_type(2)));
    const uint32_t x0 = __builtin_amdgcn_perm(b, a, 0x05010400u);  // {a0, b0, a1, b1}
    const uint32_t x1 = __builtin_amdgcn_perm(b, a, 0x07030602u);  // {a2, b2, a3, b3}
    o[0] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(x0, 512.0f, false));
    o[1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(x0, 512.0f, true));
    o[2] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(x1, 512.0f, false));
    o[3] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(x1, 512.0f, true));
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t fa = __float_as_uint((float)((a >> (8 * i)) & 0xFFu));
      const uint32_t fb = __float_as_uint((float)((b >> (8 * i)) & 0xFFu));
      o[i] = __builtin_amdgcn_perm(fb, fa, 0x07060302u);  // {hi16(fa), hi16(fb)}
    }
  }
  return o;
}

}  // namespace xs
