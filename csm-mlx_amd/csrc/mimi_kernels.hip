// Mimi codec kernels for gfx950: SEANet causal convs / transposed convs as fp32 implicit GEMMs,
// codec-transformer pieces (LayerNorm, RoPE + KV append, linear), split-RVQ gather / encode.
//
// Reference: moshi_mlx Mimi as called by /root/reference/csm_mlx/tokenizers.py:61-85 (encode),
// :148-150 (decode) and generation.py:249-256 (decode_step); restated in oracle/mimi_oracle.py.
// Everything stays fp32 (waveform parity target: 1e-4 RMS).
#include "mimi_kernels.h"

// ============================================================================ tiled GEMM core
// out(i, j) = sum_kk A(i, kk) * B(kk, j); 64 x 64 tile, K-step 16, 4x4 outputs per thread.
// Problems supply a(), b(), store(); B_KCONTIG selects the B-tile load mapping (consecutive kk
// per thread when B's memory is contiguous along kk, else consecutive j).
// SPLIT: blockIdx.z = z * ks + slice; the block sums K range [slice * KD / ks, (slice + 1) * KD / ks)
// (whole 16-steps) and writes its raw tile to slab[slice][z][i][j]; splitk_reduce_kernel adds the slices
// in order and runs the problem's epilogue.
template <class P, bool SPLIT>
__global__ __launch_bounds__(256) void gemm64_kernel(P p, int ks, float* slab, int Z) {
  __shared__ __attribute__((aligned(16))) float As[16][68];
  __shared__ __attribute__((aligned(16))) float Bs[16][68];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  const int z = SPLIT ? (int)blockIdx.z / ks : (int)blockIdx.z, sl = SPLIT ? (int)blockIdx.z % ks : 0;
  const int KD = p.kdim();
  int kb = 0, ke = KD;
  if constexpr (SPLIT) {
    const int nst = (KD + 15) / 16;
    kb = (nst * sl / ks) * 16;
    ke = min(KD, (nst * (sl + 1) / ks) * 16);
  }
  float acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = 0.f;
  // the next K tile is fetched into registers while the current one is multiplied (one tile of
  // prefetch hides the global-load latency that a load -> sync -> compute loop exposes per step)
  float va[4], vb[4];
  auto fetch = [&](int k0) {
    {
      const int i = tid >> 2, kq = (tid & 3) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        va[e] = (i0 + i < p.M && k0 + kq + e < ke) ? p.a(z, i0 + i, k0 + kq + e) : 0.f;
    }
    if constexpr (P::B_KCONTIG) {
      const int j = tid >> 2, kq = (tid & 3) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        vb[e] = (j0 + j < p.N && k0 + kq + e < ke) ? p.b(z, k0 + kq + e, j0 + j) : 0.f;
    } else {
      const int kk = tid >> 4, jb = (tid & 15) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        vb[e] = (k0 + kk < ke && j0 + jb + e < p.N) ? p.b(z, k0 + kk, j0 + jb + e) : 0.f;
    }
  };
  fetch(kb);
  for (int k0 = kb; k0 < ke; k0 += 16) {
    {
      const int i = tid >> 2, kq = (tid & 3) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) As[kq + e][i] = va[e];
    }
    if constexpr (P::B_KCONTIG) {
      const int j = tid >> 2, kq = (tid & 3) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) Bs[kq + e][j] = vb[e];
    } else {
      const int kk = tid >> 4, jb = (tid & 15) * 4;
      *reinterpret_cast<float4*>(&Bs[kk][jb]) = make_float4(vb[0], vb[1], vb[2], vb[3]);
    }
    __syncthreads();
    if (k0 + 16 < ke) fetch(k0 + 16);
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const float4 a = *reinterpret_cast<const float4*>(&As[kk][ty * 4]);
      const float4 b = *reinterpret_cast<const float4*>(&Bs[kk][tx * 4]);
      const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(av[r], bv[c], acc[r][c]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int i = i0 + ty * 4 + r, j = j0 + tx * 4 + c;
      if (i < p.M && j < p.N) {
        if constexpr (SPLIT) slab[(((size_t)sl * Z + z) * p.M + i) * p.N + j] = acc[r][c];
        else p.store(z, i, j, acc[r][c]);
      }
    }
}

// Four consecutive floats at p as one 16-B load when p is 16-B aligned (else four 4-B loads): the
// same values either way, fewer load instructions for the tile staging.
__device__ __forceinline__ void ld4(const float* p, float (&v)[4]) {
  if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
    const float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = p[e];
  }
}

// The same tile on the matrix cores: v_mfma_f32_32x32x2_f32 (fp32 operands, fp32 accumulation; each
// instruction adds its two products in k order with a rounding after each, as the fmaf chain above --
// MI355X_MICROARCH.md, f32-input MFMA "exact f32 (= fmaf chain, bitwise)"), so every output is the
// same fmaf chain over kk in order and the results equal gemm64_kernel's bit for bit.  Wave w owns
// the 32 x 32 quadrant (w >> 1, w & 1): per K-step 8 MFMAs, operands one LDS dword per lane (lane
// (r, h): A(i0 + 32 qi + r, k0 + 2t + h), B(k0 + 2t + h, j0 + 32 qj + r)); accumulator register q of
// lane (r, h) holds output row 8 (q >> 2) + 4 h + (q & 3) of the quadrant, column r.  The im2col
// staging (fetch) is unchanged: its VALU work for the next K-step runs beside the MFMAs.
template <class P, bool SPLIT>
__global__ __launch_bounds__(256) void gemm64_mf_kernel(P p, int ks, float* slab, int Z) {
  typedef float f32x16_t __attribute__((ext_vector_type(16)));
  __shared__ __attribute__((aligned(16))) float As[16][68];
  __shared__ __attribute__((aligned(16))) float Bs[16][68];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, qi = wave >> 1, qj = wave & 1;
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  const int z = SPLIT ? (int)blockIdx.z / ks : (int)blockIdx.z, sl = SPLIT ? (int)blockIdx.z % ks : 0;
  const int KD = p.kdim();
  int kb = 0, ke = KD;
  if constexpr (SPLIT) {
    const int nst = (KD + 15) / 16;
    kb = (nst * sl / ks) * 16;
    ke = min(KD, (nst * (sl + 1) / ks) * 16);
  }
  f32x16_t acc = {};
  float va[4], vb[4];
  // B staged along kk (runs of taps) for the linears and the strided convs, along the output steps
  // otherwise
  const bool bk = P::B_KCONTIG || p.kcontig();
  // (whole runs of four inside the tile take the problem's 4-wide loads: A along kk, B along kk
  // or along the output steps; the values are those of the per-element accessors)
  auto fetch = [&](int k0) {
    {
      const int i = tid >> 2, kq = (tid & 3) * 4;
      if (i0 + i < p.M && k0 + kq + 3 < ke) {
        ld4(p.aptr(z, i0 + i, k0 + kq), va);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          va[e] = (i0 + i < p.M && k0 + kq + e < ke) ? p.a(z, i0 + i, k0 + kq + e) : 0.f;
      }
    }
    if (bk) {
      const int j = tid >> 2, kq = (tid & 3) * 4;
      if (!(j0 + j < p.N && k0 + kq + 3 < ke && p.b4k(z, k0 + kq, j0 + j, vb))) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          vb[e] = (j0 + j < p.N && k0 + kq + e < ke) ? p.b(z, k0 + kq + e, j0 + j) : 0.f;
      }
    } else {
      const int kk = tid >> 4, jb = (tid & 15) * 4;
      if (!(k0 + kk < ke && j0 + jb + 3 < p.N && p.b4(z, k0 + kk, j0 + jb, vb))) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          vb[e] = (k0 + kk < ke && j0 + jb + e < p.N) ? p.b(z, k0 + kk, j0 + jb + e) : 0.f;
      }
    }
  };
  fetch(kb);
  const int r = lane & 31, h = lane >> 5;
  for (int k0 = kb; k0 < ke; k0 += 16) {
    {
      const int i = tid >> 2, kq = (tid & 3) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) As[kq + e][i] = va[e];
    }
    if (bk) {
      const int j = tid >> 2, kq = (tid & 3) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) Bs[kq + e][j] = vb[e];
    } else {
      const int kk = tid >> 4, jb = (tid & 15) * 4;
      *reinterpret_cast<float4*>(&Bs[kk][jb]) = make_float4(vb[0], vb[1], vb[2], vb[3]);
    }
    __syncthreads();
    if (k0 + 16 < ke) fetch(k0 + 16);
#pragma unroll
    for (int t = 0; t < 8; ++t)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[2 * t + h][32 * qi + r], Bs[2 * t + h][32 * qj + r], acc, 0, 0, 0);
    __syncthreads();
  }
  // the epilogue's loads (bias, residual, accumulated-onto values) issued four rows at a time before
  // their stores (which they could alias as far as the compiler knows): 4 memory round trips per tile
  // instead of 16
  if constexpr (SPLIT) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = i0 + 32 * qi + 8 * (q >> 2) + 4 * h + (q & 3), j = j0 + 32 * qj + r;
      if (i < p.M && j < p.N) slab[(((size_t)sl * Z + z) * p.M + i) * p.N + j] = acc[q];
    }
  } else {
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // four rows at a time (registers: occupancy of the main loop)
      float2 e[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + 32 * qi + 8 * g + 4 * h + u, j = j0 + 32 * qj + r;
        e[u] = (i < p.M && j < p.N) ? p.pre(z, i, j) : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + 32 * qi + 8 * g + 4 * h + u, j = j0 + 32 * qj + r;
        if (i < p.M && j < p.N) p.post(z, i, j, acc[4 * g + u], e[u]);
      }
    }
  }
}

// Wide problems (>= 256 columns: whole-utterance encode / decode convs, the codec transformer's
// linears): BM x 128 tiles, each wave a (BM / WM) x (128 / WN) block of 32 x 32 MFMA tiles (BM 128:
// 2 x 2 tiles per wave, one A and one B LDS dword per two MFMAs instead of per one; BM 32 / 64 for the
// 32- / 64-channel convs, which the 64-row tile ran half / fully padded or on one tile row).  Same
// K-steps and slices as gemm64_mf_kernel, each output one accumulator fed k in order: bit-identical.
// LDS rows are BM + 32 (or BM when BM % 64 == 32) floats apart, so the two k rows an MFMA operand read
// touches (lanes h = 0 / 1) land on disjoint halves of the 64 banks.
template <class P, bool SPLIT, int BM>
__global__ __launch_bounds__(256) void gemm128_mf_kernel(P p, int ks, float* slab, int Z) {
  typedef float f32x16_t __attribute__((ext_vector_type(16)));
  constexpr int BN = 128, WM = BM >= 64 ? 2 : 1, WN = 4 / WM, TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int SA = BM % 64 ? BM : BM + 32, SB = BN + 32;
  constexpr int NA = BM >= 64 ? BM / 64 : 1;  // A groups of four per thread
  __shared__ __attribute__((aligned(16))) float As[16][SA];
  __shared__ __attribute__((aligned(16))) float Bs[16][SB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave / WN, wn = wave % WN;
  const int i0 = blockIdx.y * BM, j0 = blockIdx.x * BN;
  const int z = SPLIT ? (int)blockIdx.z / ks : (int)blockIdx.z, sl = SPLIT ? (int)blockIdx.z % ks : 0;
  const int KD = p.kdim();
  int kb = 0, ke = KD;
  if constexpr (SPLIT) {
    const int nst = (KD + 15) / 16;
    kb = (nst * sl / ks) * 16;
    ke = min(KD, (nst * (sl + 1) / ks) * 16);
  }
  f32x16_t acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x16_t{};
  float va[NA][4], vb[2][4];
  const bool bk = P::B_KCONTIG || p.kcontig();
  const bool a_on = BM >= 64 || tid < BM * 4;
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int i = u * 64 + (tid >> 2), kq = (tid & 3) * 4;
      if (a_on && i0 + i < p.M && k0 + kq + 3 < ke) {
        ld4(p.aptr(z, i0 + i, k0 + kq), va[u]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          va[u][e] = (a_on && i0 + i < p.M && k0 + kq + e < ke) ? p.a(z, i0 + i, k0 + kq + e) : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int g = tid + 256 * u;
      if (bk) {
        const int j = g >> 2, kq = (g & 3) * 4;
        if (!(j0 + j < p.N && k0 + kq + 3 < ke && p.b4k(z, k0 + kq, j0 + j, vb[u]))) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            vb[u][e] = (j0 + j < p.N && k0 + kq + e < ke) ? p.b(z, k0 + kq + e, j0 + j) : 0.f;
        }
      } else {
        const int kk = g >> 5, jb = (g & 31) * 4;
        if (!(k0 + kk < ke && j0 + jb + 3 < p.N && p.b4(z, k0 + kk, j0 + jb, vb[u]))) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            vb[u][e] = (k0 + kk < ke && j0 + jb + e < p.N) ? p.b(z, k0 + kk, j0 + jb + e) : 0.f;
        }
      }
    }
  };
  fetch(kb);
  const int r = lane & 31, h = lane >> 5;
  const int ra = wm * (BM / WM) + r, rb = wn * (BN / WN) + r;
  for (int k0 = kb; k0 < ke; k0 += 16) {
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int i = u * 64 + (tid >> 2), kq = (tid & 3) * 4;
      if (a_on)
#pragma unroll
        for (int e = 0; e < 4; ++e) As[kq + e][i] = va[u][e];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int g = tid + 256 * u;
      if (bk) {
        const int j = g >> 2, kq = (g & 3) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) Bs[kq + e][j] = vb[u][e];
      } else {
        const int kk = g >> 5, jb = (g & 31) * 4;
        *reinterpret_cast<float4*>(&Bs[kk][jb]) = make_float4(vb[u][0], vb[u][1], vb[u][2], vb[u][3]);
      }
    }
    __syncthreads();
    if (k0 + 16 < ke) fetch(k0 + 16);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float a[TM], b[TN];
#pragma unroll
      for (int x = 0; x < TM; ++x) a[x] = As[2 * t + h][ra + 32 * x];
#pragma unroll
      for (int y = 0; y < TN; ++y) b[y] = Bs[2 * t + h][rb + 32 * y];
#pragma unroll
      for (int x = 0; x < TM; ++x)
#pragma unroll
        for (int y = 0; y < TN; ++y) acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[x], b[y], acc[x][y], 0, 0, 0);
    }
    __syncthreads();
  }
  // per 32 x 32 tile, four rows at a time: their epilogue loads, then their stores (as gemm64_mf_kernel)
#pragma unroll
  for (int x = 0; x < TM; ++x)
#pragma unroll
    for (int y = 0; y < TN; ++y) {
      const int ib = i0 + wm * (BM / WM) + 32 * x + 4 * h, j = j0 + wn * (BN / WN) + 32 * y + r;
      if constexpr (SPLIT) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int i = ib + 8 * (q >> 2) + (q & 3);
          if (i < p.M && j < p.N) slab[(((size_t)sl * Z + z) * p.M + i) * p.N + j] = acc[x][y][q];
        }
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float2 e[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int i = ib + 8 * g + u;
            e[u] = (i < p.M && j < p.N) ? p.pre(z, i, j) : make_float2(0.f, 0.f);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int i = ib + 8 * g + u;
            if (i < p.M && j < p.N) p.post(z, i, j, acc[x][y][4 * g + u], e[u]);
          }
        }
      }
    }
}

// CSM_MIMI_WIDE=0: every codec GEMM on the 64 x 64 tile (A/B); else launches of >= CSM_MIMI_WIDE_N columns
// (default 256) and >= 192 wide blocks (fewer left CUs idle: a 4096-column decode conv ran 620 us on 128
// blocks against 324 on 512 64-tiles), except 1-tap convs, take gemm128_mf_kernel
// (profiles/r04_ab_mimi_wide.txt)
static int mimi_wide_n() {
  static const int v = [] {
    const char* e = getenv("CSM_MIMI_WIDE");
    if (e && atoi(e) == 0) return 1 << 30;
    const char* n = getenv("CSM_MIMI_WIDE_N");
    return n ? atoi(n) : 256;
  }();
  return v;
}

// CSM_MIMI_MFMA=0: the VALU tile (A/B)
static bool mimi_mfma() {
  static const bool v = [] { const char* e = getenv("CSM_MIMI_MFMA"); return !e || atoi(e) != 0; }();
  return v;
}

// the split-K slices of every output, added in slice order, then the problem's epilogue
template <class P>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(P p, const float* slab, int ks, int Z) {
  const size_t tot = (size_t)Z * p.M * p.N;
  for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < tot; e += (size_t)gridDim.x * 256) {
    float v = slab[e];
    for (int s = 1; s < ks; ++s) v += slab[(size_t)s * tot + e];
    const int j = (int)(e % p.N);
    const size_t r = e / p.N;
    p.store((int)(r / p.M), (int)(r % p.M), j, v);
  }
}

// Split-K slices for a launch whose grid would hold `blocks` 64 x 64 tiles (counted on the batch-folded
// column space, so a folded and an unfolded launch of the same conv split alike -- same sums): slices
// double while the grid stays <= CSM_MIMI_KS_BLOCKS (default 512; 0 = never split) and every slice keeps
// >= 64 of the K dimension.  The streaming decode_step's first conv (1024 x 64 outputs, K 3584) ran on
// 16 blocks for 500 us (profiles/r04_prof_config3_per_frame.txt).
static int mimi_splitk(int KD, int blocks, size_t slab_per_slice) {
  static const int target = [] { const char* e = getenv("CSM_MIMI_KS_BLOCKS"); return e ? atoi(e) : 512; }();
  int ks = 1;
  while (blocks * ks * 2 <= target && KD / (ks * 2) >= 64 && ks < 32 && slab_per_slice * ks * 2 <= MIMI_KS_WS_FLOATS) ks *= 2;
  return ks;
}

template <class P, int BM>
static void launch_wide(const P& pr, dim3 grid, int ks, float* ws, hipStream_t st) {
  const int Z = (int)grid.z;
  const dim3 g((pr.N + 127) / 128, (pr.M + BM - 1) / BM, grid.z);
  if (ks <= 1 || !ws) {
    hipLaunchKernelGGL((gemm128_mf_kernel<P, false, BM>), g, dim3(256), 0, st, pr, 1, nullptr, Z);
    return;
  }
  hipLaunchKernelGGL((gemm128_mf_kernel<P, true, BM>), dim3(g.x, g.y, g.z * ks), dim3(256), 0, st, pr, ks, ws, Z);
  const size_t tot = (size_t)Z * pr.M * pr.N;
  const int rb = (int)std::min<size_t>(2048, (tot + 255) / 256);
  hipLaunchKernelGGL(splitk_reduce_kernel<P>, dim3(rb), dim3(256), 0, st, pr, ws, ks, Z);
}

// grid: the 64 x 64 tile grid (its block count also sized the split-K slices, so a wide launch splits
// exactly as the 64-tile one would: same sums)
template <class P>
static void launch_gemm64(const P& pr, dim3 grid, int ks, float* ws, hipStream_t st) {
  const bool mf = mimi_mfma();
  const size_t wblocks = (size_t)((pr.N + 127) / 128) * ((pr.M + (pr.M <= 32 ? 31 : pr.M <= 64 ? 63 : 127)) /
                                                          (pr.M <= 32 ? 32 : pr.M <= 64 ? 64 : 128)) * grid.z;
  if (mf && pr.wide_ok() && pr.N >= mimi_wide_n() && wblocks >= 192) {
    if (pr.M <= 32) launch_wide<P, 32>(pr, grid, ks, ws, st);
    else if (pr.M <= 64) launch_wide<P, 64>(pr, grid, ks, ws, st);
    else launch_wide<P, 128>(pr, grid, ks, ws, st);
    return;
  }
  if (ks <= 1 || !ws) {
    if (mf) hipLaunchKernelGGL((gemm64_mf_kernel<P, false>), grid, dim3(256), 0, st, pr, 1, nullptr, (int)grid.z);
    else hipLaunchKernelGGL((gemm64_kernel<P, false>), grid, dim3(256), 0, st, pr, 1, nullptr, (int)grid.z);
    return;
  }
  const int Z = (int)grid.z;
  const dim3 g2(grid.x, grid.y, grid.z * ks);
  if (mf) hipLaunchKernelGGL((gemm64_mf_kernel<P, true>), g2, dim3(256), 0, st, pr, ks, ws, Z);
  else hipLaunchKernelGGL((gemm64_kernel<P, true>), g2, dim3(256), 0, st, pr, ks, ws, Z);
  const size_t tot = (size_t)Z * pr.M * pr.N;
  const int rb = (int)std::min<size_t>(2048, (tot + 255) / 256);
  hipLaunchKernelGGL(splitk_reduce_kernel<P>, dim3(rb), dim3(256), 0, st, pr, ws, ks, Z);
}

// ---------------------------------------------------------------------------- causal conv1d
// Few output steps per utterance (streaming decode_step: 2-16 per frame) leave most columns of a
// 64-wide time tile empty while every (utterance, Cout tile) block still reads its whole weight
// panel, so below 64 steps the batch is folded into the columns (fold = Tout: column = b * Tout + t,
// grid.z = 1).  Each output's summation order is unchanged (bit-identical results).
struct ConvProblem {
  ConvParams c;
  int M, N;
  int fold;  // > 0: columns are (utterance, step) pairs of `fold` steps each
  static constexpr bool B_KCONTIG = false;
  __device__ int kdim() const { return c.Cin * c.k; }
  __device__ float a(int, int co, int kk) const { return c.w[(size_t)co * c.Cin * c.k + kk]; }
  __device__ const float* aptr(int, int co, int kk) const { return c.w + (size_t)co * c.Cin * c.k + kk; }
  // strided convs (the encoder's downsampling): B staged along the taps -- consecutive kk of one input
  // channel are consecutive input samples
  __device__ bool kcontig() const { return c.stride > 1 && c.dil == 1 && !fold; }
  // 1-tap convs (K = Cin, memory-bound, mostly with a residual) ran faster on the 64 x 64 tile
  bool wide_ok() const { return c.k > 1; }
  __device__ bool b4k(int z, int kk0, int t, float (&v)[4]) const {
    const int ci = kk0 / c.k, j = kk0 - ci * c.k;
    const int u = t * c.stride + j - c.pad_l;
    if (j + 3 >= c.k || u < 0 || u + 3 >= c.Tin) return false;
    ld4(c.x + (size_t)z * c.x_bstride + (size_t)ci * c.x_cstride + c.x_off + u, v);
    if (c.elu_in)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = elu_f(v[e]);
    return true;
  }
  // steps t0 .. t0 + 3 of one utterance at stride 1, all inside the input: one 4-wide load
  __device__ bool b4(int z, int kk, int t0, float (&v)[4]) const {
    if (c.stride != 1) return false;
    if (fold) {
      z = t0 / fold;
      t0 -= z * fold;
      if (t0 + 3 >= fold) return false;
    }
    const int ci = kk / c.k, j = kk - ci * c.k;
    const int u = t0 + j * c.dil - c.pad_l;
    if (u < 0 || u + 3 >= c.Tin) return false;
    ld4(c.x + (size_t)z * c.x_bstride + (size_t)ci * c.x_cstride + c.x_off + u, v);
    if (c.elu_in)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = elu_f(v[e]);
    return true;
  }
  __device__ float b(int z, int kk, int t) const {
    if (fold) {
      z = t / fold;
      t -= z * fold;
    }
    const int ci = kk / c.k, j = kk - ci * c.k;
    int u = t * c.stride + j * c.dil - c.pad_l;
    if (u < 0 || u >= c.Tin) {
      if (!c.replicate) return 0.f;
      u = u < 0 ? 0 : c.Tin - 1;
    }
    const float v = c.x[(size_t)z * c.x_bstride + (size_t)ci * c.x_cstride + c.x_off + u];
    return c.elu_in ? elu_f(v) : v;
  }
  // epilogue operands (bias, residual), loaded by a tile for all its outputs before its first store
  __device__ float2 pre(int z, int co, int t) const {
    if (fold) {
      z = t / fold;
      t -= z * fold;
    }
    return make_float2(c.bias ? c.bias[co] : 0.f,
                       c.resid ? c.resid[(size_t)z * c.r_bstride + (size_t)co * c.r_cstride + c.r_off + t] : 0.f);
  }
  __device__ void post(int z, int co, int t, float v, float2 e) const {
    if (fold) {
      z = t / fold;
      t -= z * fold;
    }
    if (c.bias) v += e.x;
    if (c.resid) v += e.y;
    const size_t o = (size_t)z * c.y_bstride + (size_t)co * c.y_cstride + c.y_off + t;
    if (c.y2) c.y2[o] = elu_f(v);
    c.y[o] = c.elu_out ? elu_f(v) : v;
  }
  __device__ void store(int z, int co, int t, float v) const { post(z, co, t, v, pre(z, co, t)); }
};

// CSM_MIMI_CONV_FOLD=0: no batch folding (A/B).  Measured: config 3 (B = 32 streaming decode_step)
// 2932 -> 3253 frames/s (profiles/r03_ab_mimi.txt)
static bool conv_fold_enabled() {
  static const bool v = [] { const char* e = getenv("CSM_MIMI_CONV_FOLD"); return !e || atoi(e) != 0; }();
  return v;
}

void launch_conv1d(const ConvParams& p, hipStream_t st) {
  const bool fold = p.Tout < 64 && p.B > 1 && conv_fold_enabled();
  ConvProblem pr{p, p.Cout, fold ? p.B * p.Tout : p.Tout, fold ? p.Tout : 0};
  dim3 grid((pr.N + 63) / 64, (p.Cout + 63) / 64, fold ? 1 : p.B);
  const int ks = mimi_splitk(p.Cin * p.k, ((p.B * p.Tout + 63) / 64) * ((p.Cout + 63) / 64), (size_t)p.B * p.Tout * p.Cout);
  launch_gemm64(pr, grid, ks, p.ks_ws, st);
}

// ---------------------------------------------------------------------------- transposed conv (k = 2s)
// fold > 0: columns are (utterance, input) pairs of `fold` inputs each, grid.z = the s phases
struct ConvTrProblem {
  ConvTrParams c;
  int M, N;
  int fold;
  static constexpr bool B_KCONTIG = false;
  __device__ int kdim() const { return c.Cin * 2; }
  __device__ float a(int z, int co, int kk) const {
    const int r = z % c.s;
    return c.wt[((size_t)r * c.Cout + co) * c.Cin * 2 + kk];
  }
  __device__ const float* aptr(int z, int co, int kk) const { return c.wt + ((size_t)(z % c.s) * c.Cout + co) * c.Cin * 2 + kk; }
  __device__ bool kcontig() const { return false; }
  bool wide_ok() const { return true; }
  __device__ bool b4k(int, int, int, float (&)[4]) const { return false; }
  // inputs i0 .. i0 + 3 of one utterance, all at or after the first: one 4-wide load
  __device__ bool b4(int z, int kk, int i0, float (&v)[4]) const {
    int bb = z / c.s;
    if (fold) {
      bb = i0 / fold;
      i0 -= bb * fold;
      if (i0 + 3 >= fold) return false;
    }
    const int ci = kk >> 1, e = kk & 1;
    const int ti = c.t_in0 + i0 - e;
    if (ti < 0) return false;
    ld4(c.x + (size_t)bb * c.x_bstride + (size_t)ci * c.x_cstride + c.x_off + ti, v);
    if (c.elu_in)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = elu_f(v[q]);
    return true;
  }
  __device__ float b(int z, int kk, int i) const {
    int bb = z / c.s;
    if (fold) {
      bb = i / fold;
      i -= bb * fold;
    }
    const int ci = kk >> 1, e = kk & 1;
    const int ti = c.t_in0 + i - e;
    if (ti < 0) return 0.f;
    const float v = c.x[(size_t)bb * c.x_bstride + (size_t)ci * c.x_cstride + c.x_off + ti];
    return c.elu_in ? elu_f(v) : v;
  }
  __device__ float2 pre(int, int co, int) const { return make_float2(c.bias ? c.bias[co] : 0.f, 0.f); }
  __device__ void post(int z, int co, int i, float v, float2 e) const {
    int bb = z / c.s;
    const int r = z % c.s;
    if (fold) {
      bb = i / fold;
      i -= bb * fold;
    }
    if (c.bias) v += e.x;
    c.y[(size_t)bb * c.y_bstride + (size_t)co * c.y_cstride + c.y_off + (size_t)i * c.s + r] = v;
  }
  __device__ void store(int z, int co, int i, float v) const { post(z, co, i, v, pre(z, co, i)); }
};

void launch_convtr(const ConvTrParams& p, hipStream_t st) {
  const bool fold = p.n_in < 64 && p.B > 1 && conv_fold_enabled();
  ConvTrProblem pr{p, p.Cout, fold ? p.B * p.n_in : p.n_in, fold ? p.n_in : 0};
  dim3 grid((pr.N + 63) / 64, (p.Cout + 63) / 64, fold ? p.s : p.B * p.s);
  const int ks = mimi_splitk(p.Cin * 2, ((p.B * p.n_in + 63) / 64) * ((p.Cout + 63) / 64) * p.s,
                             (size_t)p.B * p.n_in * p.s * p.Cout);
  launch_gemm64(pr, grid, ks, p.ks_ws, st);
}

// ---------------------------------------------------------------------------- linear (rows x W^T)
struct LinProblem {
  LinParams c;
  int M, N;  // M = output features (weight rows), N = activation rows
  static constexpr bool B_KCONTIG = true;
  __device__ int kdim() const { return c.K; }
  __device__ float a(int, int n, int kk) const { return c.W[(size_t)n * c.K + kk]; }
  __device__ float b(int, int kk, int m) const { return c.x[(size_t)m * c.xs + kk]; }
  __device__ const float* aptr(int, int n, int kk) const { return c.W + (size_t)n * c.K + kk; }
  __device__ bool kcontig() const { return true; }
  bool wide_ok() const { return true; }
  __device__ bool b4k(int, int kk0, int m, float (&v)[4]) const {
    ld4(c.x + (size_t)m * c.xs + kk0, v);
    return true;
  }
  __device__ bool b4(int, int, int, float (&)[4]) const { return false; }
  __device__ float* optr(int n, int m) const {
    if (c.conv_T) {  // conv layout out[b][n][t], m = b*T + t
      const int bb = m / c.conv_T, t = m % c.conv_T;
      return c.out + (size_t)bb * c.conv_bstride + (size_t)n * c.conv_T + t;
    }
    return c.out + (size_t)m * c.os + n;
  }
  // (the value accumulated onto, the layer scale)
  __device__ float2 pre(int, int n, int m) const {
    if (c.conv_T) return make_float2(c.accumulate ? *optr(n, m) : 0.f, 0.f);
    if (c.epi == EPI_ADD) return make_float2(*optr(n, m), c.scale ? c.scale[n] : 0.f);
    return make_float2(0.f, 0.f);
  }
  __device__ void post(int, int n, int m, float v, float2 e) const {
    float* o = optr(n, m);
    if (c.conv_T) {
      *o = c.accumulate ? e.x + v : v;
      return;
    }
    switch (c.epi) {
      case EPI_GELU:
        *o = c.gelu_erf ? gelu_erf_f(v) : gelu_tanh_f(v);
        break;
      case EPI_ADD:
        *o = e.x + (c.scale ? e.y * v : v);
        break;
      default:
        *o = v;
    }
  }
  __device__ void store(int z, int n, int m, float v) const { post(z, n, m, v, pre(z, n, m)); }
};

// Few rows (streaming decode_step: one row per utterance): gemm64's 64 x 64 tiles leave most of the
// chip idle (8-32 blocks), so row-major linears of <= 32 rows go through the decode GEMV instead
// (fp32 weights, same epilogues: y = gelu(v) / out += scale * v).  Measured: config 3 (B = 32
// decode_step) 2083 -> 2123 frames/s; at 125 rows (one-shot decode of a 10 s utterance) neutral, and
// 16 rows per weight pass was slower (2001).  Round 3: the codec transformer's rows at B = 32 are 64
// (two 25 Hz steps per frame), where gemm64 left the N = 512 outputs on 8 workgroups: cutoff 64,
// config 3 2932 -> 3076 frames/s (profiles/r03_ab_mimi.txt).  Round 4: above 16 rows the tiled GEMM
// with split-K (mimi_splitk: 64-512 blocks instead of 8-32) -- the 64-row linears took 40-68 us on the
// GEMV, which re-reads the weights for every 4-row pass (profiles/r04_prof_config3_per_frame.txt).
// CSM_MIMI_GEMV_M sets the largest row count on the GEMV (0 = never).
static int mimi_gemv_rows() {
  static const int v = [] { const char* e = getenv("CSM_MIMI_GEMV_M"); return e ? atoi(e) : 16; }();
  return v;
}

void launch_linear(const LinParams& p, hipStream_t st) {
  if (!p.conv_T && p.M <= mimi_gemv_rows() && p.N % 8 == 0 && p.K % 8 == 0 &&
      p.N % gemv_rows_per_block(p.N, p.K, p.M) == 0 && gemv_rows_per_block(p.N, p.K, p.M) % 2 == 0) {
    GemvParams g{};
    g.W = p.W; g.N = p.N; g.K = p.K; g.x = p.x; g.xs = p.xs; g.M = p.M; g.out = p.out; g.os = p.os;
    g.scale = p.scale; g.gelu_erf = p.gelu_erf;
    launch_gemv(g, WDT_F32, p.epi, 0, st, 3);  // tag 3: default cache policy
    return;
  }
  LinProblem pr{p, p.N, p.M};
  dim3 grid((p.M + 63) / 64, (p.N + 63) / 64, 1);
  const int ks = mimi_splitk(p.K, (int)(grid.x * grid.y), (size_t)p.M * p.N);
  launch_gemm64(pr, grid, ks, p.ks_ws, st);
}

// ============================================================================ LayerNorm rows
// mlx fast.layer_norm: (x - mean) / sqrt(var + eps) * w + b, two-pass in fp32.
__global__ __launch_bounds__(256) void layernorm_rows_kernel(const float* x, int D, const float* w, const float* b,
                                                              float eps, float* out) {
  __shared__ float red[4];
  const int m = blockIdx.x, tid = threadIdx.x;
  const float* xr = x + (size_t)m * D;
  float s = 0.f;
  for (int d = tid; d < D; d += 256) s += xr[d];
  s = wave_sum(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  const float mean = (red[0] + red[1] + red[2] + red[3]) / (float)D;
  __syncthreads();
  float v = 0.f;
  for (int d = tid; d < D; d += 256) {
    const float t = xr[d] - mean;
    v += t * t;
  }
  v = wave_sum(v);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  const float rstd = 1.f / sqrtf((red[0] + red[1] + red[2] + red[3]) / (float)D + eps);
  for (int d = tid; d < D; d += 256) out[(size_t)m * D + d] = (xr[d] - mean) * rstd * w[d] + b[d];
}

void launch_layernorm_rows(const float* x, int D, const float* w, const float* b, float eps, float* out, int M,
                           hipStream_t st) {
  hipLaunchKernelGGL(layernorm_rows_kernel, dim3(M), dim3(256), 0, st, x, D, w, b, eps, out);
}

// ============================================================================ layout transposes
__global__ void conv_to_rows_kernel(const float* x, int C, int T, int x_bstride, int x_cstride, int x_off,
                                    float* rows) {
  const int b = blockIdx.z, t = blockIdx.x * 64 + (threadIdx.x & 63);
  const int c = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (t < T && c < C) rows[((size_t)b * T + t) * C + c] = x[(size_t)b * x_bstride + (size_t)c * x_cstride + x_off + t];
}
void launch_conv_to_rows(const float* x, int B, int C, int T, int x_bstride, int x_cstride, int x_off, float* rows,
                         hipStream_t st) {
  hipLaunchKernelGGL(conv_to_rows_kernel, dim3((T + 63) / 64, (C + 3) / 4, B), dim3(256), 0, st, x, C, T, x_bstride,
                     x_cstride, x_off, rows);
}
__global__ void rows_to_conv_kernel(const float* rows, int C, int T, float* y, int y_bstride, int y_cstride,
                                    int y_off) {
  const int b = blockIdx.z, t = blockIdx.x * 64 + (threadIdx.x & 63);
  const int c = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (t < T && c < C) y[(size_t)b * y_bstride + (size_t)c * y_cstride + y_off + t] = rows[((size_t)b * T + t) * C + c];
}
void launch_rows_to_conv(const float* rows, int B, int C, int T, float* y, int y_bstride, int y_cstride, int y_off,
                         hipStream_t st) {
  hipLaunchKernelGGL(rows_to_conv_kernel, dim3((T + 63) / 64, (C + 3) / 4, B), dim3(256), 0, st, rows, C, T, y,
                     y_bstride, y_cstride, y_off);
}

// ============================================================================ RoPE + KV append
// moshi_mlx nn.RoPE(traditional=True): rotate (x[2i], x[2i+1]) of q and k per head.
__global__ void rope_append_kernel(const float* qkv, int M, int D, int H, int hd, const float* rope, RowMap rm,
                                   float* qout, float* kc, float* vc, int S_cap) {
  const int m = blockIdx.x;
  const int b = rm.b(m), pos = rm.pos(m);
  const float* row = qkv + (size_t)m * 3 * D;
  for (int pi = threadIdx.x; pi < D / 2; pi += blockDim.x) {
    const int n = pi * 2, h = n / hd, d = n % hd;
    const float2 cs = *reinterpret_cast<const float2*>(rope + ((size_t)pos * (hd / 2) + d / 2) * 2);
    const float q0 = row[n], q1 = row[n + 1];
    const float k0 = row[D + n], k1 = row[D + n + 1];
    qout[(size_t)m * D + n] = q0 * cs.x - q1 * cs.y;
    qout[(size_t)m * D + n + 1] = q0 * cs.y + q1 * cs.x;
    const size_t ci = (((size_t)b * H + h) * S_cap + pos) * hd + d;
    kc[ci] = k0 * cs.x - k1 * cs.y;
    kc[ci + 1] = k0 * cs.y + k1 * cs.x;
    vc[ci] = row[2 * D + n];
    vc[ci + 1] = row[2 * D + n + 1];
  }
}
void launch_rope_append(const float* qkv, int M, int D, int H, int hd, const float* rope, RowMap rm, float* qout,
                        float* kc, float* vc, int S_cap, hipStream_t st) {
  hipLaunchKernelGGL(rope_append_kernel, dim3(M), dim3(256), 0, st, qkv, M, D, H, hd, rope, rm, qout, kc, vc, S_cap);
}

// ============================================================================ depthwise upsample
__global__ void upsample_dw_kernel(const float* x, int C, int x_bstride, int x_cstride, int x_off, const float* w,
                                   int s, int t_in0, int n_in, float* y, int y_bstride, int y_cstride, int y_off) {
  const int b = blockIdx.z, c = blockIdx.y;
  const int o = blockIdx.x * blockDim.x + threadIdx.x;  // output index within the produced range
  if (o >= n_in * s) return;
  const int i = o / s, r = o % s, ti = t_in0 + i;
  const float* xr = x + (size_t)b * x_bstride + (size_t)c * x_cstride + x_off;
  float v = xr[ti] * w[(size_t)c * 2 * s + r];
  if (ti - 1 >= 0) v += xr[ti - 1] * w[(size_t)c * 2 * s + r + s];
  y[(size_t)b * y_bstride + (size_t)c * y_cstride + y_off + o] = v;
}
void launch_upsample_dw(const float* x, int B, int C, int x_bstride, int x_cstride, int x_off, const float* w, int s,
                        int t_in0, int n_in, float* y, int y_bstride, int y_cstride, int y_off, hipStream_t st) {
  hipLaunchKernelGGL(upsample_dw_kernel, dim3((n_in * s + 255) / 256, C, B), dim3(256), 0, st, x, C, x_bstride,
                     x_cstride, x_off, w, s, t_in0, n_in, y, y_bstride, y_cstride, y_off);
}

// ============================================================================ RVQ
// decode gather: the codebook rows are summed in codebook order with plain fp32 adds, exactly as
// the restated ResidualVectorQuantizer.decode accumulates them.  Ids >= bins (2048..2050, valid
// CSM outputs but outside the Mimi codebook) are clamped to bins-1.
__global__ void rvq_gather_kernel(const int* codes, int layout, int B, int F, int n_q, int k0, int k1,
                                  const float* cb, int bins, int cd, float* q) {
  const int m = blockIdx.x;  // b*F + f
  const int b = m / F, f = m % F;
  for (int d = threadIdx.x; d < cd; d += blockDim.x) {
    float acc = 0.f;
    for (int k = k0; k < k1; ++k) {
      int c = layout == 0 ? codes[((size_t)b * n_q + k) * F + f] : codes[((size_t)f * B + b) * n_q + k];
      c = min(max(c, 0), bins - 1);
      acc = acc + cb[((size_t)k * bins + c) * cd + d];
    }
    q[(size_t)m * cd + d] = acc;
  }
}
void launch_rvq_gather(const int* codes, int layout, int B, int F, int n_q, int k0, int k1, const float* cb, int bins,
                       int cd, float* q, hipStream_t st) {
  hipLaunchKernelGGL(rvq_gather_kernel, dim3(B * F), dim3(256), 0, st, codes, layout, B, F, n_q, k0, k1, cb, bins, cd,
                     q);
}

// encode: one block per latent row; residual in LDS; per codebook every thread scores bins/256
// codes as c2half - r.c (moshi_mlx EuclideanCodebook.encode), first-minimum arg-min.
__global__ __launch_bounds__(256) void rvq_encode_kernel(float* r, int T, int cd, const float* cb,
                                                         const float* c2half, int bins, int k0, int k1, int n_q,
                                                         int* codes) {
  __shared__ __attribute__((aligned(16))) float rs[1024];
  __shared__ float sv[4];
  __shared__ int si[4];
  const int m = blockIdx.x, tid = threadIdx.x;
  const int b = m / T, t = m % T;
  for (int d = tid; d < cd; d += 256) rs[d] = r[(size_t)m * cd + d];
  __syncthreads();
  for (int k = k0; k < k1; ++k) {
    const float* cbk = cb + (size_t)k * bins * cd;
    float best = INFINITY;
    int bi = 0x7fffffff;
    for (int c = tid; c < bins; c += 256) {
      const float4* cr = reinterpret_cast<const float4*>(cbk + (size_t)c * cd);
      const float4* rr = reinterpret_cast<const float4*>(rs);
      float dot = 0.f;
      for (int d4 = 0; d4 < cd / 4; ++d4) {
        const float4 a = cr[d4], x = rr[d4];
        dot = fmaf(a.x, x.x, dot);
        dot = fmaf(a.y, x.y, dot);
        dot = fmaf(a.z, x.z, dot);
        dot = fmaf(a.w, x.w, dot);
      }
      const float dist = c2half[(size_t)k * bins + c] - dot;
      if (dist < best) {
        best = dist;
        bi = c;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov < best || (ov == best && oi < bi)) {
        best = ov;
        bi = oi;
      }
    }
    if ((tid & 63) == 0) {
      sv[tid >> 6] = best;
      si[tid >> 6] = bi;
    }
    __syncthreads();
    float bv = sv[0];
    int bidx = si[0];
    for (int w = 1; w < 4; ++w)
      if (sv[w] < bv || (sv[w] == bv && si[w] < bidx)) {
        bv = sv[w];
        bidx = si[w];
      }
    bidx = min(max(bidx, 0), bins - 1);
    if (tid == 0) codes[((size_t)b * n_q + k) * T + t] = bidx;
    for (int d = tid; d < cd; d += 256) rs[d] = rs[d] - cbk[(size_t)bidx * cd + d];
    __syncthreads();
  }
  for (int d = tid; d < cd; d += 256) r[(size_t)m * cd + d] = rs[d];
}

// Tiled encode for many rows: a block owns 16 latent rows (wave w: rows 4w..4w+3) and streams each
// codebook through LDS in [32 dims][256 codes] tiles shared by all its rows -- the codebook is read
// once per block instead of once per row.  Lane l of a wave scores codes 4l..4l+3 of every tile
// against the wave's 4 rows (16 fp32 accumulators: one 16-B code read and one 16-B residual read
// per 16 FMAs); the residuals sit transposed ([dim][row]) in LDS.  Every (row, code) dot is one
// fmaf chain over the dims in order -- rvq_encode_kernel's arithmetic, so codes and residuals are
// identical; the arg-min keeps the first minimum.
constexpr int RVQ_RB = 16, RVQ_CC = 256, RVQ_DC = 32, RVQ_CDMAX = 512;
__global__ __launch_bounds__(256) void rvq_encode_tiled_kernel(float* r, int M, int T, int cd, const float* cb,
                                                               const float* c2half, int bins, int k0, int k1,
                                                               int n_q, int* codes) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) float rsT[RVQ_CDMAX][RVQ_RB];   // residuals [dim][row]
  __shared__ __attribute__((aligned(16))) float ct[RVQ_DC][RVQ_CC];       // codebook tile [dim][code]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * RVQ_RB;
  for (int e = tid; e < RVQ_RB * cd; e += 256) {
    const int i = e / cd, d = e % cd;
    rsT[d][i] = r[(size_t)min(m0 + i, M - 1) * cd + d];
  }
  __syncthreads();
  for (int k = k0; k < k1; ++k) {
    const float* cbk = cb + (size_t)k * bins * cd;
    float best[4];
    int bi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      best[i] = INFINITY;
      bi[i] = 0x7fffffff;
    }
    for (int c0 = 0; c0 < bins; c0 += RVQ_CC) {
      float acc[4][4];  // [row][code]
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
      for (int d0 = 0; d0 < cd; d0 += RVQ_DC) {
        const int dn = min(RVQ_DC, cd - d0);
        __syncthreads();  // previous tile consumed
        for (int e = tid; e < RVQ_CC * RVQ_DC; e += 256) {  // coalesced along dims
          const int cc = e / RVQ_DC, dd = e % RVQ_DC;
          const int c = c0 + cc;
          ct[dd][cc] = (c < bins && dd < dn) ? cbk[(size_t)c * cd + d0 + dd] : 0.f;
        }
        __syncthreads();
        for (int dd = 0; dd < dn; ++dd) {
          const f4 a = *reinterpret_cast<const f4*>(&ct[dd][4 * lane]);
          const f4 x = *reinterpret_cast<const f4*>(&rsT[d0 + dd][4 * wave]);
          const float av[4] = {a.x, a.y, a.z, a.w}, xv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[j], xv[i], acc[i][j]);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = c0 + 4 * lane + j;
        if (c < bins) {
          const float c2 = c2half[(size_t)k * bins + c];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float dist = c2 - acc[i][j];
            if (dist < best[i]) {  // codes visited in increasing order: first minimum kept
              best[i] = dist;
              bi[i] = c;
            }
          }
        }
      }
    }
    // per row: first minimum over the wave's lanes, then the wave updates its rows' residuals
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float bv = best[i];
      int bx = bi[i];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bx, o, 64);
        if (ov < bv || (ov == bv && oi < bx)) {
          bv = ov;
          bx = oi;
        }
      }
      bx = min(max(bx, 0), bins - 1);
      const int m = m0 + 4 * wave + i;
      if (lane == 0 && m < M) codes[((size_t)(m / T) * n_q + k) * T + m % T] = bx;
      for (int d = lane; d < cd; d += 64) rsT[d][4 * wave + i] = rsT[d][4 * wave + i] - cbk[(size_t)bx * cd + d];
    }
  }
  __syncthreads();
  for (int e = tid; e < RVQ_RB * cd; e += 256) {
    const int i = e / cd, d = e % cd;
    if (m0 + i < M) r[(size_t)(m0 + i) * cd + d] = rsT[d][i];
  }
}

// Split-RVQ encode as one distance GEMM per codebook (config 5's context encode: 4032 latent rows x 31
// codebooks per 64 segments; rvq_encode_tiled_kernel streamed every codebook through every 16-row
// block, 15 ms per launch).  Launch k: block (code tile ct of 256, row tile of 64) first finishes codebook
// k-1 for its rows -- arg-min over the 8 code-tile partials of k-1 (first minimum), residual r_k = r_{k-1}
// - c_{k-1}[idx] into LDS (every code tile of a row tile computes the same r_k; tile 0 writes it and the
// code) -- then scores its 256 codes against the 64 rows: the (row, code) dots are fmaf chains over the
// dims in order with the code operand first, rvq_encode_kernel's arithmetic, so codes and residuals are
// bit-identical to it; the codebook arrives dims-major (cbT [k][dim][code], built at load) in 32-dim
// LDS chunks, double-buffered.  A partial (dist key, code) per (row, code tile) goes to part_cur.
constexpr int RQ_R = 64, RQ_C = 256, RQ_D = 32, RQ_CDMAX = 256;
__device__ __forceinline__ unsigned long long rq_key(float dist, int c) {
  return ((unsigned long long)f2key(dist) << 32) | (unsigned)c;  // min = smallest dist, then smallest code
}

struct RvqStep {
  const float* r_in;                 // [M][cd] residual r_{k-1} (or the input latent when part_prev is null)
  float* r_out;                      // [M][cd] r_k for the next launch
  const unsigned long long* part_prev;  // [M][nct] partials of codebook k-1, null at the first codebook
  unsigned long long* part_cur;      // [M][nct] partials of codebook k (null: finishing pass only)
  const float* cb_prev;              // codebook k-1 [bins][cd]
  const float* cbT;                  // codebook k dims-major [cd][bins]
  const float* c2half;               // [bins] of codebook k
  int* codes;                        // [B][n_q][T]
  int M, T, cd, bins, nct, k, n_q;
};

// MF: the scores on the fp32 matrix cores (v_mfma_f32_32x32x2_f32: each (row, code) dot the same
// k-ordered fmaf chain, the product's operand order immaterial -- bit-identical codes).  Wave w scores
// codes 64 w .. 64 w + 63 of the tile against all 64 rows (2 x 2 tiles of 32 x 32); odd dims of r_k and
// of the codebook chunk are stored with the 32-column halves swapped, so the two k rows an operand read
// touches (lanes h = 0 / 1) sit on disjoint LDS bank halves.
template <bool MF>
__global__ __launch_bounds__(256) void rvq_step_kernel(RvqStep p) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) float rsT[RQ_CDMAX][RQ_R];      // r_k [dim][row]
  __shared__ __attribute__((aligned(16))) float Bs[2][RQ_D][RQ_C];        // codebook chunk [dim][code]
  __shared__ int sidx[RQ_R];
  __shared__ unsigned long long wred[MF ? 4 : 1][RQ_R];
  const int tid = threadIdx.x, ct = blockIdx.x, m0 = blockIdx.y * RQ_R;
  auto sw = [](int d) { return MF ? (d & 1) * 32 : 0; };  // column swizzle of dim d's row
  const int cd = p.cd;
  // (1) finish codebook k-1 for the 64 rows
  if (tid < RQ_R) {
    int idx = -1;
    const int m = min(m0 + tid, p.M - 1);
    if (p.part_prev) {
      unsigned long long best = ~0ull;
      for (int j = 0; j < p.nct; ++j) best = min(best, p.part_prev[(size_t)m * p.nct + j]);
      idx = min(max((int)(unsigned)(best & 0xffffffffu), 0), p.bins - 1);
      if (ct == 0 && m0 + tid < p.M) p.codes[((size_t)(m / p.T) * p.n_q + (p.k - 1)) * p.T + m % p.T] = idx;
    }
    sidx[tid] = idx;
  }
  __syncthreads();
  for (int e = tid; e < RQ_R * cd; e += 256) {
    const int i = e / cd, d = e % cd, m = min(m0 + i, p.M - 1);
    float v = p.r_in[(size_t)m * cd + d];
    if (sidx[i] >= 0) v = v - p.cb_prev[(size_t)sidx[i] * cd + d];
    rsT[d][i ^ sw(d)] = v;
    if (ct == 0 && m0 + i < p.M) p.r_out[(size_t)m * cd + d] = v;
  }
  if (!p.part_cur) return;  // finishing pass (after the last codebook)
  // (2) distances of this tile's 256 codes: thread (ty, tx) -> rows 8 ty .. +8, codes 8 tx .. +8
  const int tx = tid & 31, ty = tid >> 5, c0 = ct * RQ_C;
  auto load = [&](int buf, int d0) {
    for (int e = tid; e < RQ_D * RQ_C / 4; e += 256) {
      const int dd = e / (RQ_C / 4), c4 = (e % (RQ_C / 4)) * 4;
      *reinterpret_cast<f4*>(&Bs[buf][dd][c4 ^ sw(dd)]) = *reinterpret_cast<const f4*>(p.cbT + (size_t)(d0 + dd) * p.bins + c0 + c4);
    }
  };
  const int nch = cd / RQ_D;
  if constexpr (MF) {
    typedef float f32x16_t __attribute__((ext_vector_type(16)));
    const int lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    f32x16_t acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[x][y] = f32x16_t{};
    load(0, 0);
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
      const int buf = ch & 1;
      if (ch + 1 < nch) load(buf ^ 1, (ch + 1) * RQ_D);
#pragma unroll 4
      for (int t = 0; t < RQ_D / 2; ++t) {
        const int dd = 2 * t + h, d = ch * RQ_D + dd;  // (RQ_D even: d and dd share their parity)
        float a[2], b[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) a[x] = rsT[d][(32 * x + r) ^ sw(d)];
#pragma unroll
        for (int y = 0; y < 2; ++y) b[y] = Bs[buf][dd][(64 * wave + 32 * y + r) ^ sw(dd)];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y) acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(b[y], a[x], acc[x][y], 0, 0, 0);
      }
      __syncthreads();
    }
    // acc[x][y][q]: code 64 wave + 32 y + 8 (q >> 2) + 4 h + (q & 3), row 32 x + r (B operand = rows)
    float c2[2][16];
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int q = 0; q < 16; ++q) c2[y][q] = p.c2half[c0 + 64 * wave + 32 * y + 8 * (q >> 2) + 4 * h + (q & 3)];
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      unsigned long long best = ~0ull;
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int q = 0; q < 16; ++q)
          best = min(best, rq_key(c2[y][q] - acc[x][y][q], c0 + 64 * wave + 32 * y + 8 * (q >> 2) + 4 * h + (q & 3)));
      best = min(best, (unsigned long long)__shfl_xor(best, 32, 64));  // the other half's codes of this row
      if (h == 0) wred[wave][32 * x + r] = best;
    }
    __syncthreads();
    if (tid < RQ_R) {
      const unsigned long long best = min(min(wred[0][tid], wred[1][tid]), min(wred[2][tid], wred[3][tid]));
      if (m0 + tid < p.M) p.part_cur[(size_t)(m0 + tid) * p.nct + ct] = best;
    }
    return;
  }
  float acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
  load(0, 0);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < nch) load(buf ^ 1, (ch + 1) * RQ_D);
#pragma unroll 4
    for (int dd = 0; dd < RQ_D; ++dd) {
      const int d = ch * RQ_D + dd;
      const f4 r0 = *reinterpret_cast<const f4*>(&rsT[d][8 * ty]);
      const f4 r1 = *reinterpret_cast<const f4*>(&rsT[d][8 * ty + 4]);
      const f4 b0 = *reinterpret_cast<const f4*>(&Bs[buf][dd][8 * tx]);
      const f4 b1 = *reinterpret_cast<const f4*>(&Bs[buf][dd][8 * tx + 4]);
      const float rv[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
      const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = fmaf(bv[j], rv[i], acc[i][j]);
    }
    __syncthreads();
  }
  // (3) per row: first minimum over the tile's codes (keys: dist, then code)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    unsigned long long best = ~0ull;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + 8 * tx + j;
      best = min(best, rq_key(p.c2half[c] - acc[i][j], c));
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) best = min(best, (unsigned long long)__shfl_xor(best, o, 32));
    const int m = m0 + 8 * ty + i;
    if (tx == 0 && m < p.M) p.part_cur[(size_t)m * p.nct + ct] = best;
  }
}

// CSM_RVQ_MFMA=0: the VALU scoring tile (A/B)
static bool rvq_mfma() {
  static const bool v = [] { const char* e = getenv("CSM_RVQ_MFMA"); return !e || atoi(e) != 0; }();
  return v;
}

bool rvq_gemm_eligible(int cd, int bins) { return cd % RQ_D == 0 && cd <= RQ_CDMAX && bins % RQ_C == 0; }
size_t rvq_gemm_parts(int M, int bins) { return (size_t)M * (bins / RQ_C); }

void launch_rvq_encode_gemm(float* r, int M, int T, int cd, const float* cb, const float* cbT, const float* c2half,
                            int bins, int k0, int k1, int n_q, int* codes, float* rbuf, unsigned long long* pbuf,
                            hipStream_t st) {
  const int nct = bins / RQ_C;
  const size_t pn = (size_t)M * nct;
  RvqStep s{};
  s.M = M; s.T = T; s.cd = cd; s.bins = bins; s.nct = nct; s.n_q = n_q; s.codes = codes;
  const dim3 grid(nct, (M + RQ_R - 1) / RQ_R);
  for (int k = k0; k <= k1; ++k) {
    const int i = k - k0;
    s.k = k;
    s.r_in = i == 0 ? r : rbuf + (size_t)(i & 1) * M * cd;
    s.r_out = k == k1 ? r : rbuf + (size_t)((i + 1) & 1) * M * cd;   // the finishing pass writes r_{k1} back
    s.part_prev = i == 0 ? nullptr : pbuf + (size_t)((i - 1) & 1) * pn;
    s.part_cur = k == k1 ? nullptr : pbuf + (size_t)(i & 1) * pn;
    s.cb_prev = k > k0 ? cb + (size_t)(k - 1) * bins * cd : nullptr;
    s.cbT = k < k1 ? cbT + (size_t)k * bins * cd : nullptr;
    s.c2half = k < k1 ? c2half + (size_t)k * bins : nullptr;
    // the finishing pass needs only code tile 0 (it writes the codes and r); it computes no distances
    if (rvq_mfma()) hipLaunchKernelGGL(rvq_step_kernel<true>, k == k1 ? dim3(1, grid.y) : grid, dim3(256), 0, st, s);
    else hipLaunchKernelGGL(rvq_step_kernel<false>, k == k1 ? dim3(1, grid.y) : grid, dim3(256), 0, st, s);
  }
}

void launch_rvq_encode(float* r, int M, int T, int cd, const float* cb, const float* c2half, int bins, int k0, int k1,
                       int n_q, int* codes, hipStream_t st) {
  const char* env = getenv("CSM_RVQ_TILED");  // read per call (encode is never graph-captured): A/B tests
  const int mode = env ? atoi(env) : 1;
  if (mode && cd <= RVQ_CDMAX && M >= 1024) {  // tiled once there are >= 64 blocks of 16 rows
    hipLaunchKernelGGL(rvq_encode_tiled_kernel, dim3((M + RVQ_RB - 1) / RVQ_RB), dim3(256), 0, st, r, M, T, cd, cb,
                       c2half, bins, k0, k1, n_q, codes);
    return;
  }
  hipLaunchKernelGGL(rvq_encode_kernel, dim3(M), dim3(256), 0, st, r, T, cd, cb, c2half, bins, k0, k1, n_q, codes);
}

// ============================================================================ window copy
__global__ void copy_window_kernel(const float* src, int src_bstride, int src_cstride, int src_off, float* dst,
                                   int dst_bstride, int dst_cstride, int dst_off, int len) {
  const int b = blockIdx.z, c = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < len)
    dst[(size_t)b * dst_bstride + (size_t)c * dst_cstride + dst_off + i] =
        src[(size_t)b * src_bstride + (size_t)c * src_cstride + src_off + i];
}
void launch_copy_window(const float* src, int B, int C, int src_bstride, int src_cstride, int src_off, float* dst,
                        int dst_bstride, int dst_cstride, int dst_off, int len, hipStream_t st) {
  if (len <= 0) return;
  hipLaunchKernelGGL(copy_window_kernel, dim3((len + 255) / 256, C, B), dim3(256), 0, st, src, src_bstride,
                     src_cstride, src_off, dst, dst_bstride, dst_cstride, dst_off, len);
}
