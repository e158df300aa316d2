// Skinny-M GEMM for KV-cache decode steps: C[M][N] = A[M][K] . W[K][N], M <= 32 tokens, bf16 in / bf16 out.
//
// hipBLASLt picks MT16x32 tiles for M = 32, which launch ~128 workgroups for a 2048-wide projection and stream the
// weight at ~435 GB/s (profiles/r1h_decode_kv.md). The op is weight-bandwidth bound (M FMAs per weight element), so
// this kernel is laid out for HBM streaming: every weight element is read exactly once per 16-row M tile with 16-byte
// loads, the K range is split over blocks so a 2048x2048 weight launches 256+ blocks, and the fp32 partials
// (KS x M x N, 1/8 of the weight bytes at KS = 4) are summed by a second pass that writes bf16.
//
// Block = 256 threads: tx = t % 8 owns 8 contiguous columns (one uint4 of a weight row), ky = t / 8 (32 k-lanes)
// walks the block's K range with stride 32. A's [16][KR] tile is staged in LDS as fp32 (reads are broadcasts).
// Reduction over the 32 k-lanes: xor-shuffles over the 8 k-lanes inside a wave, then LDS across the 4 waves.
#include "common.h"

namespace {

constexpr int SK_MT = 16;    // M rows per tile
constexpr int SK_KR = 512;   // K rows per block
constexpr int SK_NB = 64;    // columns per block

__global__ __launch_bounds__(256) void skinny_partial_kernel(const bf16_t* __restrict__ A, int lda,
                                                             const bf16_t* __restrict__ W, int ldw,
                                                             float* __restrict__ ws, int M, int N, int K) {
  __shared__ float xs[SK_MT][SK_KR];
  __shared__ float red[4][8][SK_MT * 8 + 1];
  const int t = threadIdx.x, tx = t & 7, ky = t >> 3, lane = t & 63, w = t >> 6;
  const int n0 = blockIdx.x * SK_NB + tx * 8;
  const int kb = blockIdx.y * SK_KR;
  const int m0 = blockIdx.z * SK_MT;
  const int kr = min(SK_KR, K - kb);
  for (int i = t; i < SK_MT * SK_KR; i += 256) {
    const int m = i / SK_KR, k = i % SK_KR;
    xs[m][k] = (m0 + m < M && k < kr) ? bf2f(A[(long long)(m0 + m) * lda + kb + k]) : 0.f;
  }
  __syncthreads();
  float acc[SK_MT][8];
#pragma unroll
  for (int m = 0; m < SK_MT; ++m)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[m][j] = 0.f;
  const bool colok = n0 < N;
#pragma unroll 4
  for (int k = ky; k < kr; k += 32) {
    uint4 u = make_uint4(0, 0, 0, 0);
    if (colok) u = *reinterpret_cast<const uint4*>(W + (long long)(kb + k) * ldw + n0);
    const uint32_t p[4] = {u.x, u.y, u.z, u.w};
    float wv[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) { wv[2 * j] = bf2f(p[j] & 0xffff); wv[2 * j + 1] = bf2f(p[j] >> 16); }
#pragma unroll
    for (int m = 0; m < SK_MT; ++m) {
      const float xv = xs[m][k];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[m][j] = fmaf(xv, wv[j], acc[m][j]);
    }
  }
  // lanes with the same tx inside a wave differ in bits 3..5 of the lane id
#pragma unroll
  for (int m = 0; m < SK_MT; ++m)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = acc[m][j];
      v += __shfl_xor(v, 8);
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      acc[m][j] = v;
    }
  if (lane < 8) {
#pragma unroll
    for (int m = 0; m < SK_MT; ++m)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[w][lane][m * 8 + j] = acc[m][j];
  }
  __syncthreads();
  // 256 threads write the block's [16][64] partial: thread -> (m, column)
  for (int i = t; i < SK_MT * SK_NB; i += 256) {
    const int m = i / SK_NB, c = i % SK_NB, g = c / 8, j = c % 8;
    const int n = blockIdx.x * SK_NB + c;
    if (m0 + m < M && n < N) {
      const float v = red[0][g][m * 8 + j] + red[1][g][m * 8 + j] + red[2][g][m * 8 + j] + red[3][g][m * 8 + j];
      ws[((long long)blockIdx.y * M + m0 + m) * N + n] = v;
    }
  }
}

__global__ __launch_bounds__(256) void skinny_combine_kernel(const float* __restrict__ ws, bf16_t* __restrict__ C,
                                                             int ldc, int M, int N, int KS) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)M * N) return;
  const int m = (int)(i / N), n = (int)(i % N);
  float s = 0.f;
  for (int k = 0; k < KS; ++k) s += ws[(long long)k * M * N + i];
  C[(long long)m * ldc + n] = f2bf(s);
}

}  // namespace

// ws: fp32 [ceil(K / 512)][M][N]
OBST_API int obst_skinny_gemm(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M, int N, int K,
                              float* ws, hipStream_t st) {
  if (M <= 0 || M > 2 * SK_MT || N <= 0 || K <= 0 || N % 8 || ldw % 8 || lda < K || ldw < N || ldc < N) return -1;
  if (((uintptr_t)W) & 15) return -2;
  const int KS = (K + SK_KR - 1) / SK_KR;
  hipLaunchKernelGGL(skinny_partial_kernel, dim3((N + SK_NB - 1) / SK_NB, KS, (M + SK_MT - 1) / SK_MT), dim3(256), 0,
                     st, (const bf16_t*)A, lda, (const bf16_t*)W, ldw, ws, M, N, K);
  const long long total = (long long)M * N;
  hipLaunchKernelGGL(skinny_combine_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, ws, (bf16_t*)C,
                     ldc, M, N, KS);
  return (int)hipGetLastError();
}
