// Mimi codec kernels (SEANet convs, codec transformer pieces, split RVQ) -- parameter blocks.
#pragma once
#include "csm_kernels.h"

// Split-K scratch of the codec GEMMs (one per codec, mimi_create): partial tiles of up to 512 blocks of
// 64 x 64 (launches with fewer than 512 blocks split K until they reach it: the streaming decode_step's
// short-time, wide-channel convs and its 64-row transformer linears), summed in slice order by a
// second kernel that runs the problem's epilogue.  Null: no split.
constexpr size_t MIMI_KS_WS_FLOATS = (size_t)512 * 64 * 64;

// Causal Conv1d as implicit GEMM: y[b][co][t] = bias[co] + sum_{ci,j} w[co][ci][j] * act(xv(b,ci,t*stride+j*dil-pad_l))
// xv outside [0, Tin) is 0 (constant pad) or the edge sample (replicate pad); act = ELU when elu_in.
struct ConvParams {
  const float* x;
  int Cin, Tin, x_bstride, x_off;  // x_off: index of sample 0 inside each channel row
  int x_cstride;                   // elements between channels
  const float* w;                  // [Cout][Cin][k]
  const float* bias;               // [Cout] or null
  int Cout, k, stride, dil, pad_l, replicate, elu_in;
  float* y;
  int Tout, y_bstride, y_cstride, y_off;
  const float* resid;              // optional, same layout as y (added after bias)
  int r_bstride, r_cstride, r_off;
  int B;
  float* ks_ws;                    // split-K scratch (MIMI_KS_WS_FLOATS) or null
  // ELU of the output for a consumer that would apply it on every load (the encoder's ELU-input convs:
  // each input read k x ceil(Cout / tile) times): elu_out stores ELU(y) in place of y, y2 (same layout
  // as y) receives ELU(y) beside it.  ELU(v) of the stored v is what the consumer computed: bit-identical.
  int elu_out;
  float* y2;
};

// ConvTranspose1d with k = 2*s (every Mimi transposed conv): per output phase r = t % s,
// y[b][co][(ti - t_in0)*s + r] = bias + sum_ci sum_e wt[r][co][ci][e] * act(x[b][ci][ti - e]), ti - e >= 0
struct ConvTrParams {
  const float* x;
  int Cin, Tin, x_bstride, x_cstride, x_off;
  const float* wt;                 // [s][Cout][Cin][2]
  const float* bias;
  int Cout, s, elu_in;
  int t_in0, n_in;                 // produce outputs of inputs [t_in0, t_in0 + n_in)
  float* y;
  int y_bstride, y_cstride, y_off;
  int B;
  float* ks_ws;                    // split-K scratch (MIMI_KS_WS_FLOATS) or null
};

// Row-major linear: out[m][n] = epi( sum_k x[m][k] * W[n][k] )
struct LinParams {
  const float* x;
  int M, K, xs;
  const float* W;   // [N][K] f32
  int N;
  float* out;
  int os;
  int epi;          // EPI_STORE / EPI_ADD / EPI_GELU
  const float* scale;
  int gelu_erf;
  // optional transposed store into a conv-layout tensor: out[b][n][t] with m = b*T + t
  int conv_T;       // 0 = row-major store
  int conv_bstride;
  int accumulate;   // conv store: add into existing values
  float* ks_ws;     // split-K scratch (MIMI_KS_WS_FLOATS) or null
};

void launch_conv1d(const ConvParams& p, hipStream_t st);
void launch_convtr(const ConvTrParams& p, hipStream_t st);
void launch_linear(const LinParams& p, hipStream_t st);
void launch_layernorm_rows(const float* x, int D, const float* w, const float* b, float eps, float* out, int M,
                           hipStream_t st);
// conv layout [B][C][T] (+offset) <-> rows [B*T][C]
void launch_conv_to_rows(const float* x, int B, int C, int T, int x_bstride, int x_cstride, int x_off, float* rows,
                         hipStream_t st);
void launch_rows_to_conv(const float* rows, int B, int C, int T, float* y, int y_bstride, int y_cstride, int y_off,
                         hipStream_t st);
// Mimi RoPE (interleaved, table) on q and k of a fused qkv row buffer [M][3D]; q -> qout [M][D],
// k/v -> caches [B][H][S_cap][hd] at pos(m)
void launch_rope_append(const float* qkv, int M, int D, int H, int hd, const float* rope, RowMap rm, float* qout,
                        float* kc, float* vc, int S_cap, hipStream_t st);
// depthwise ConvTranspose k=2s (upsample): y[b][c][(ti-t_in0)*s + r] = x[ti]*w[c][r] + x[ti-1]*w[c][r+s]
void launch_upsample_dw(const float* x, int B, int C, int x_bstride, int x_cstride, int x_off, const float* w, int s,
                        int t_in0, int n_in, float* y, int y_bstride, int y_cstride, int y_off, hipStream_t st);
// RVQ decode gather: q[m][cd] = sum_{k in [k0,k1)} cb[k][code(m,k)]  with codes [B][n_q][F] (layout 0)
// or engine history [F][B][n_q] (layout 1); m = b*F + f
void launch_rvq_gather(const int* codes, int layout, int B, int F, int n_q, int k0, int k1, const float* cb, int bins,
                       int cd, float* q, hipStream_t st);
// RVQ encode: r[m][cd] residual (in place); for k in [k0,k1): idx = argmin(c2half - r.c), r -= c[idx];
// codes[b][k][t] for m = b*T + t
void launch_rvq_encode(float* r, int M, int T, int cd, const float* cb, const float* c2half, int bins, int k0, int k1,
                       int n_q, int* codes, hipStream_t st);
// The same as one distance GEMM launch per codebook (+ a finishing pass): cbT = codebooks dims-major
// [n_q][cd][bins]; rbuf = 2 x [M][cd] floats, pbuf = 2 x rvq_gemm_parts(M, bins) partials of scratch.
// Codes and the final residual bit-identical to launch_rvq_encode's.
bool rvq_gemm_eligible(int cd, int bins);
size_t rvq_gemm_parts(int M, int bins);
void launch_rvq_encode_gemm(float* r, int M, int T, int cd, const float* cb, const float* cbT, const float* c2half,
                            int bins, int k0, int k1, int n_q, int* codes, float* rbuf, unsigned long long* pbuf,
                            hipStream_t st);
// copy a [B][C][len] window: dst[b][c][i] = src[b][c][src_off + i]
void launch_copy_window(const float* src, int B, int C, int src_bstride, int src_cstride, int src_off, float* dst,
                        int dst_bstride, int dst_cstride, int dst_off, int len, hipStream_t st);
