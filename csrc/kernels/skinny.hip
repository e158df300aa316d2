// Skinny-M GEMM for KV-cache decode steps: C[M][N] = A[M][K] . W[K][N] for M <= 32 tokens, bf16 in / bf16 out,
// on v_mfma_f32_16x16x32_bf16 with the weight read ONCE for all M rows.
//
// The op is weight-bandwidth bound (M = 32 FMAs per weight element). The weight comes in as the framework's cached
// K-contiguous copy Wt[N][K] (ParamStore.transposed), so both MFMA operands load straight from global memory into
// registers with 16-byte loads and no LDS staging (cdna_hip_programming.md §5, 'GEMV / M <= 16 decode weights':
// operand streamed once, loads straight to VGPRs, deep unroll):
//   MFMA A = Wt tile: lane l holds Wt[n0 + (l & 15)][k + 8 (l >> 4) .. +8]   (16 rows x 64 contiguous bytes)
//   MFMA B = A^T    : lane l holds A[t0 + (l & 15)][k + 8 (l >> 4) .. +8]    (tokens t0 = 0 and 16: two MFMAs)
//   D[n][t]         : lane l holds rows n0 + 4 (l >> 4) + i, column t0 + (l & 15) -> C[t][n .. n+3] (8-byte store)
// Block = 4 waves on one 16-column tile of C; wave w takes the 32-deep k-steps s = w, w + 4, ... of the block's K
// range (4 steps per unrolled iteration: 4 weight + 8 activation loads in flight per lane), the 4 wave sums are
// added through LDS in wave order. KSPLIT > 1 splits K over blocks (grid.y) into fp32 partial slabs that a second
// kernel adds in slab order: the result is deterministic either way.
#include "common.h"

namespace {

constexpr int SK_NT = 16;     // C columns (weight rows of Wt) per block
constexpr int SK_W = 4;       // waves per block
constexpr int SK_U = 4;       // k-steps (of 32) per unrolled iteration

__device__ __forceinline__ bf16x8_t ld8(const bf16_t* p) {
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p));
}

__global__ __launch_bounds__(SK_W * 64) void skinny_mfma_kernel(const bf16_t* __restrict__ A, int lda,
                                                                const bf16_t* __restrict__ Wt, int ldw,
                                                                bf16_t* __restrict__ C, int ldc,
                                                                float* __restrict__ ws, int M, int N, int K,
                                                                int kchunk) {
  if (__builtin_amdgcn_wavefrontsize() != 64) __builtin_trap();   // fragment maps below are wave64 maps
  __shared__ float red[SK_W][64][8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int n0 = blockIdx.x * SK_NT;
  const int kb = blockIdx.y * kchunk, ke = min(K, kb + kchunk);
  const bf16_t* wrow = Wt + (long long)(n0 + r) * ldw + 8 * q;
  const bool t0ok = r < M, t1ok = r + 16 < M;
  const bf16_t* a0 = A + (long long)(t0ok ? r : 0) * lda + 8 * q;
  const bf16_t* a1 = A + (long long)(t1ok ? r + 16 : 0) * lda + 8 * q;
  const bf16x8_t zero = __builtin_bit_cast(bf16x8_t, make_uint4(0, 0, 0, 0));
  f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const int nsteps = (ke - kb) / 32;
  int s = w;
  for (; s + (SK_U - 1) * SK_W < nsteps; s += SK_U * SK_W) {
    bf16x8_t wf[SK_U], x0[SK_U], x1[SK_U];
#pragma unroll
    for (int u = 0; u < SK_U; ++u) {
      const int k = kb + (s + u * SK_W) * 32;
      wf[u] = ld8(wrow + k);
      x0[u] = t0ok ? ld8(a0 + k) : zero;
      x1[u] = t1ok ? ld8(a1 + k) : zero;
    }
#pragma unroll
    for (int u = 0; u < SK_U; ++u) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[u], x0[u], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[u], x1[u], acc1, 0, 0, 0);
    }
  }
  for (; s < nsteps; s += SK_W) {
    const int k = kb + s * 32;
    const bf16x8_t wf = ld8(wrow + k);
    const bf16x8_t x0 = t0ok ? ld8(a0 + k) : zero, x1 = t1ok ? ld8(a1 + k) : zero;
    acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, x0, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, x1, acc1, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) { red[w][lane][i] = acc0[i]; red[w][lane][4 + i] = acc1[i]; }
  __syncthreads();
  if (w != 0) return;
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = red[0][lane][i] + red[1][lane][i] + red[2][lane][i] + red[3][lane][i];
  const int n = n0 + 4 * q;                 // this lane's 4 consecutive columns
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int t = r + 16 * h;
    if (t >= M) continue;
    const float* vv = v + 4 * h;
    if (ws) {
      *reinterpret_cast<float4*>(ws + ((long long)blockIdx.y * M + t) * N + n) = make_float4(vv[0], vv[1], vv[2], vv[3]);
    } else {
      const uint2 o = make_uint2(pack_bf16x2(vv[0], vv[1]), pack_bf16x2(vv[2], vv[3]));
      *reinterpret_cast<uint2*>(C + (long long)t * ldc + n) = o;
    }
  }
}

// C[t][n] = sum over slabs s (in order) of ws[s][t][n]
__global__ __launch_bounds__(256) void skinny_combine_kernel(const float* __restrict__ ws, bf16_t* __restrict__ C,
                                                             int ldc, int M, int N, int KS) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)M * N) return;
  const int m = (int)(i / N), n = (int)(i % N);
  float s = 0.f;
  for (int k = 0; k < KS; ++k) s += ws[(long long)k * M * N + i];
  C[(long long)m * ldc + n] = f2bf(s);
}

int ksplit_for(int M, int N, int K) {
  // enough blocks to put a block on most CUs (256), each block still streaming >= 256 k per wave-step range
  const int tiles = N / SK_NT;
  int ks = 1;
  while (tiles * ks < 256 && K / (ks * 2) >= 1024 && ks < 8) ks *= 2;
  return ks;
}

}  // namespace

// floats of fp32 workspace obst_skinny_gemm needs (0: single pass)
OBST_API long long obst_skinny_ws(int M, int N, int K) {
  const int ks = ksplit_for(M, N, K);
  return ks > 1 ? (long long)ks * M * N : 0;
}

// A [M][K] (lda), Wt [N][K] (ldw: the K-contiguous weight copy), C [M][N] (ldc); M <= 32, N % 16 == 0, K % 32 == 0,
// 16-byte aligned A / Wt rows; ws: obst_skinny_ws(M, N, K) floats (or null when that is 0)
OBST_API int obst_skinny_gemm(const void* A, int lda, const void* Wt, int ldw, void* C, int ldc, int M, int N, int K,
                              float* ws, hipStream_t st) {
  if (M <= 0 || M > 32 || N <= 0 || K <= 0 || N % SK_NT || K % 32 || lda % 8 || ldw % 8 || ldc % 4 || lda < K ||
      ldw < K || ldc < N)
    return -1;
  if ((((uintptr_t)A) | ((uintptr_t)Wt)) & 15 || ((uintptr_t)C) & 7) return -2;
  const int ks = ksplit_for(M, N, K);
  if (ks > 1 && !ws) return -3;
  const int kchunk = (K / 32 + ks - 1) / ks * 32;
  hipLaunchKernelGGL(skinny_mfma_kernel, dim3(N / SK_NT, ks), dim3(SK_W * 64), 0, st, (const bf16_t*)A, lda,
                     (const bf16_t*)Wt, ldw, (bf16_t*)C, ldc, ks > 1 ? ws : nullptr, M, N, K, kchunk);
  if (ks > 1) {
    const long long total = (long long)M * N;
    hipLaunchKernelGGL(skinny_combine_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, ws,
                       (bf16_t*)C, ldc, M, N, ks);
  }
  return (int)hipGetLastError();
}
