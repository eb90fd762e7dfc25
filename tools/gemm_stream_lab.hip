// Lab microbenchmark (not part of the library): a streaming MFMA GEMM for the batched decode shapes
// y[m][n] = sum_k A[m][k] W[n][k] at M = 32 / 64 batch rows, where the activations arrive already split
// into the three exact bf16 parts (hi, mid, lo) in MFMA fragment order -- no LDS staging, no
// per-stage barrier, no VALU split in the main loop -- against the current gemm_wide structure's
// cost.  Weights in the engine's fragment-tiled copy (gemm_retile layout).  Prints us per launch.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_stream_lab.hip -o tools/gemm_stream_lab
//   tools/gemm_stream_lab
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int KC = 64;  // K per stage

// A fragments: [mtile][kst][part 3][s 4][lane 64] x 16 B;  W fragments: [tile32][kst][s 4][lane 64] x 16 B
// Block: WAVES waves over one K slice (split evenly), RTW 32-row weight tiles per wave (the same tiles for
// every wave), MT batch tiles.  Waves' partial sums are added in a fixed order through LDS.
template <int RTW, int MT, int WAVES, int PD>
__global__ __launch_bounds__(64 * WAVES) void gemm_stream(const u32x4_t* __restrict__ W, const u32x4_t* __restrict__ A,
                                                          float* __restrict__ out, int N, int K, int ks) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nks = K / KC, nt32 = N / 32;
  const int t0 = blockIdx.x * RTW;           // first 32-row weight tile
  const int kslice = blockIdx.y, nst = nks / ks, st0 = kslice * nst;
  const int wst = nst / WAVES, ws0 = st0 + wave * wst;  // this wave's stages
  f32x16_t acc[MT][RTW];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < RTW; ++i) acc[t][i] = f32x16_t{};
  struct St { u32x4_t w[RTW][4]; u32x4_t a[MT][3][4]; };
  auto load = [&](int st, St& g) {
#pragma unroll
    for (int i = 0; i < RTW; ++i)
#pragma unroll
      for (int s = 0; s < 4; ++s) g.w[i][s] = W[(((size_t)(t0 + i) * nks + st) * 4 + s) * 64 + lane];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int s = 0; s < 4; ++s) g.a[t][p][s] = A[((((size_t)t * nks + st) * 3 + p) * 4 + s) * 64 + lane];
  };
  // ring of PD stages, loads straight-line (a clamped stage index past the end re-reads the last
  // stage: no branch around a load, so the compiler's vmcnt counts stay exact)
  St g[PD];
#pragma unroll
  for (int d = 0; d < PD; ++d) load(ws0 + min(d, wst - 1), g[d]);
  asm volatile("" ::: "memory");  // keep the ring's loads where they are issued (no sinking to their use)
  for (int j0 = 0; j0 < wst; j0 += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      const St& c = g[d];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int i = 0; i < RTW; ++i)
              acc[t][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, c.a[t][p][s]),
                                                                   __builtin_bit_cast(bf16x8_t, c.w[i][s]), acc[t][i], 0, 0, 0);
      load(ws0 + min(j0 + d + PD, wst - 1), g[d]);
      asm volatile("" ::: "memory");
    }
  }
  // fixed-order cross-wave sum through LDS: [wave][t][i][j][lane]
  __shared__ float red[WAVES > 1 ? (WAVES - 1) : 1][MT * RTW * 16][64];
  if (WAVES > 1) {
    if (wave > 0)
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int i = 0; i < RTW; ++i)
#pragma unroll
          for (int j = 0; j < 16; ++j) red[wave - 1][(t * RTW + i) * 16 + j][lane] = acc[t][i][j];
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int w = 1; w < WAVES; ++w)
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int i = 0; i < RTW; ++i)
#pragma unroll
          for (int j = 0; j < 16; ++j) acc[t][i][j] += red[w - 1][(t * RTW + i) * 16 + j][lane];
  }
  // C[row (j&3) + 8(j>>2) + 4h][col r]: batch row, weight row
  const int r = lane & 31, h = lane >> 5;
  float* o = out + (size_t)kslice * MT * 32 * N;
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < RTW; ++i)
#pragma unroll
      for (int j = 0; j < 16; ++j) o[(size_t)(32 * t + (j & 3) + 8 * (j >> 2) + 4 * h) * N + 32 * (t0 + i) + r] = acc[t][i][j];
  (void)nt32;
}

// reference: fp32 from the same fragments
__global__ void ref_kernel(const unsigned short* W, const unsigned short* A, float* out, int N, int K, int M) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  const int nks = K / KC;
  auto bf = [](unsigned short u) { return __uint_as_float((unsigned)u << 16); };
  float s = 0.f;
  for (int k = 0; k < K; ++k) {
    const int kst = k / KC, kk = k % KC, hh = kk / 32, ss = (kk % 32) / 8, jj = kk % 8;
    const int lane_w = (n % 32) + 32 * hh, lane_a = (m % 32) + 32 * hh, t = m / 32;
    const float w = bf(W[((((size_t)(n / 32) * nks + kst) * 4 + ss) * 64 + lane_w) * 8 + jj]);
    float a = 0.f;
    for (int p = 0; p < 3; ++p) a += bf(A[(((((size_t)t * nks + kst) * 3 + p) * 4 + ss) * 64 + lane_a) * 8 + jj]);
    s += w * a;
  }
  out[(size_t)m * N + n] = s;
}

template <int RTW, int MT, int WAVES, int PD = 2>
void run(const char* name, int N, int K, int ks, int nlay) {
  const int M = 32 * MT;
  const size_t wbytes = (size_t)N * K * 2, abytes = (size_t)M * K * 6;
  std::vector<void*> Ws(nlay);
  std::vector<unsigned short> h(wbytes / 2);
  srand(1);
  for (auto& v : h) v = (unsigned short)(0x3c00 + (rand() & 0x3ff) - 0x200) ^ ((rand() & 1) << 15);
  for (auto& p : Ws) { CK(hipMalloc(&p, wbytes)); CK(hipMemcpy(p, h.data(), wbytes, hipMemcpyHostToDevice)); }
  std::vector<unsigned short> ha(abytes / 2);
  for (auto& v : ha) v = (unsigned short)(0x3f00 + (rand() & 0xff)) ^ ((rand() & 1) << 15);
  void* A;
  CK(hipMalloc(&A, abytes));
  CK(hipMemcpy(A, ha.data(), abytes, hipMemcpyHostToDevice));
  float *out, *ref;
  CK(hipMalloc(&out, (size_t)ks * M * N * 4));
  CK(hipMalloc(&ref, (size_t)M * N * 4));
  const dim3 grid(N / (32 * RTW), ks);
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((gemm_stream<RTW, MT, WAVES, PD>), grid, dim3(64 * WAVES), 0, 0, (const u32x4_t*)Ws[i % nlay], (const u32x4_t*)A, out, N, K, ks);
  CK(hipDeviceSynchronize());
  // check
  hipLaunchKernelGGL(ref_kernel, dim3((N + 255) / 256, M), dim3(256), 0, 0, (const unsigned short*)Ws[2 % nlay], (const unsigned short*)A, ref, N, K, M);
  CK(hipDeviceSynchronize());
  std::vector<float> ho((size_t)ks * M * N), hr((size_t)M * N);
  CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), ref, hr.size() * 4, hipMemcpyDeviceToHost));
  double maxe = 0, maxr = 0;
  for (size_t i = 0; i < hr.size(); ++i) {
    double s = 0;
    for (int k = 0; k < ks; ++k) s += ho[(size_t)k * M * N + i];
    maxe = std::max(maxe, std::fabs(s - hr[i]));
    maxr = std::max(maxr, (double)std::fabs(hr[i]));
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int iters = 200;
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((gemm_stream<RTW, MT, WAVES, PD>), grid, dim3(64 * WAVES), 0, 0, (const u32x4_t*)Ws[i % nlay], (const u32x4_t*)A, out, N, K, ks);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1000.0 / iters;
  printf("%-10s M=%2d N=%5d K=%5d RTW=%d WAVES=%d ks=%2d blocks=%4d  %7.2f us  W %6.0f GB/s  err %.1e\n", name, M, N, K, RTW,
         WAVES, ks, grid.x * grid.y, us, wbytes / us / 1e3, maxe / maxr);
  for (auto p : Ws) CK(hipFree(p));
  CK(hipFree(A));
  CK(hipFree(out));
  CK(hipFree(ref));
}

int main() {
  // (wst must be a multiple of PD: stages per wave = K / 64 / ks / WAVES)
  run<2, 1, 4, 1>("gate_up", 16384, 1024, 1, 4);
  run<2, 1, 4, 2>("gate_up", 16384, 1024, 1, 4);
  run<2, 1, 4, 4>("gate_up", 16384, 1024, 1, 4);
  run<2, 1, 2, 4>("gate_up", 16384, 1024, 1, 4);
  run<2, 1, 2, 8>("gate_up", 16384, 1024, 1, 4);
  run<2, 1, 1, 8>("gate_up", 16384, 1024, 1, 4);
  run<4, 1, 4, 2>("gate_up", 16384, 1024, 2, 4);
  run<2, 1, 4, 2>("down", 1024, 8192, 16, 4);
  run<2, 1, 2, 4>("down", 1024, 8192, 16, 4);
  run<2, 1, 1, 8>("down", 1024, 8192, 16, 4);
  run<1, 1, 4, 1>("qkv", 1536, 1024, 4, 4);
  run<1, 1, 2, 1>("o", 1024, 1024, 8, 4);
  return 0;
}
