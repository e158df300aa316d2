// Skinny-M GEMM for KV-cache decode steps: C[M][N] = epilogue(A[M][K] . W[K][N]) for M <= 32 tokens, bf16 in /
// bf16 out, on v_mfma_f32_16x16x32_bf16 with the weight read ONCE for all M rows (reference decode loop:
// src/run/inference.py:76-97 -- every projection of a decode step is one of these).
//
// The op is weight-bandwidth bound (M = 32 FMAs per weight element): a 32 x 2048 x 4096 product streams 16 MiB of
// weight, ~2.7 us at 6 TB/s. What bounds a naive kernel is the bytes in flight (Little's law: ~6 TB/s x ~2-3 us of
// loaded-chip latency = ~15 MiB), so every wave issues ALL its weight loads of a batch before its first MFMA:
//   block = 8 waves on 16 columns of C (16 rows of the K-contiguous weight copy Wt[N][K]); wave w takes a contiguous
//   run of 32-deep k-steps, in batches of NS = 8 steps: 8 weight loads (16 B per lane, 16 rows x 64 B each) and 16
//   activation loads (L2-resident, shared by every block) are in flight before the 16 MFMAs of the batch.
//   Split-K over blocks (grid.y) brings the grid to >= 256 blocks for the narrow shapes; its fp32 slabs are summed in
//   slab order by a second kernel (deterministic).
//   MFMA A = Wt tile: lane l holds Wt[n0 + (l & 15)][k + 8 (l >> 4) .. +8]
//   MFMA B = A^T    : lane l holds A[t0 + (l & 15)][k + 8 (l >> 4) .. +8]    (tokens t0 = 0 and 16: two MFMAs)
//   D[n][t]         : lane l holds rows n0 + 4 (l >> 4) + i, column t0 + (l & 15)
// Loads are raw buffer loads: rows t >= M and the steps past a wave's range read at an offset past the resource
// (returned as zeros, no branch around the load). The 8 waves' partial sums meet in LDS; the epilogue (alpha,
// residual R, pre-activation Zout, activation) runs on 4 consecutive columns per thread with 8-byte stores.
#include "common.h"

namespace {

constexpr int SK_NT = 16;     // C columns (weight rows of Wt) per block
constexpr int SK_W = 8;       // waves per block
constexpr int SK_NS = 8;      // k-steps (of 32) per wave and batch: all their loads in flight before the MFMAs
constexpr unsigned SK_OOR = 0x80000000u;   // a buffer offset past any resource: the load returns zeros

typedef __attribute__((ext_vector_type(4))) unsigned v4u32s_t;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t sk_rsrc(const void* base, long long nbytes) {
  const int n = (int)(unsigned)(nbytes <= 0 ? 0ull : nbytes >= 0x7fffffffll ? 0x7fffffffull : (unsigned long long)nbytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, n, 0x00020000);
}

__device__ __forceinline__ bf16x8_t sk_ld(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

// v = act(alpha * acc + R); Zout <- alpha * acc + R (pre-activation), 4 consecutive columns
__device__ __forceinline__ void sk_epilogue(float (&v)[4], long long idx, const bf16_t* R, bf16_t* Zout, bf16_t* C,
                                            float alpha, int act) {
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] *= alpha;
  if (R) {
    const uint2 r = *reinterpret_cast<const uint2*>(R + idx);
    v[0] += bf2f(r.x & 0xffff); v[1] += bf2f(r.x >> 16); v[2] += bf2f(r.y & 0xffff); v[3] += bf2f(r.y >> 16);
  }
  if (Zout) *reinterpret_cast<uint2*>(Zout + idx) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
  if (act) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = act_fwd(act, v[i]);
  }
  *reinterpret_cast<uint2*>(C + idx) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
}

__global__ __launch_bounds__(SK_W * 64) void skinny_mfma_kernel(const bf16_t* __restrict__ A, int lda,
                                                                const bf16_t* __restrict__ Wt, int ldw,
                                                                bf16_t* __restrict__ C, int ldc,
                                                                float* __restrict__ ws, const bf16_t* R,
                                                                bf16_t* Zout, float alpha, int act, int M, int N,
                                                                int K, int kchunk) {
  if (__builtin_amdgcn_wavefrontsize() != 64) __builtin_trap();   // fragment maps below are wave64 maps
  __shared__ f32x4_t red[SK_W][2][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int n0 = blockIdx.x * SK_NT;
  const int kb = blockIdx.y * kchunk, ke = min(K, kb + kchunk);
  const int nsteps = (ke - kb) / 32;
  const int per = (nsteps + SK_W - 1) / SK_W;                // this wave's k-steps: [s0, s1)
  const int s0 = min(w * per, nsteps), s1 = min(s0 + per, nsteps);
  const __amdgpu_buffer_rsrc_t rw = sk_rsrc(Wt, ((long long)(N - 1) * ldw + K) * 2);
  const __amdgpu_buffer_rsrc_t ra = sk_rsrc(A, ((long long)(M - 1) * lda + K) * 2);   // rows >= M: past the end
  const unsigned wbase = (unsigned)(((long long)(n0 + r) * ldw + kb + 8 * q) * 2);
  const unsigned a0base = (unsigned)(((long long)r * lda + kb + 8 * q) * 2);
  const unsigned a1base = (unsigned)(((long long)(r + 16) * lda + kb + 8 * q) * 2);
  f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int b = s0; b < s1; b += SK_NS) {
    bf16x8_t wf[SK_NS], x0[SK_NS], x1[SK_NS];
#pragma unroll
    for (int u = 0; u < SK_NS; ++u) {   // every weight load of the batch first
      const bool ok = b + u < s1;
      wf[u] = sk_ld(rw, ok ? wbase + (b + u) * 64 : SK_OOR);
    }
#pragma unroll
    for (int u = 0; u < SK_NS; ++u) {
      const bool ok = b + u < s1;
      x0[u] = sk_ld(ra, ok ? a0base + (b + u) * 64 : SK_OOR);
      x1[u] = sk_ld(ra, ok ? a1base + (b + u) * 64 : SK_OOR);
    }
#pragma unroll
    for (int u = 0; u < SK_NS; ++u) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[u], x0[u], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[u], x1[u], acc1, 0, 0, 0);
    }
  }
  red[w][0][lane] = acc0;
  red[w][1][lane] = acc1;
  __syncthreads();
  if (threadIdx.x >= 128) return;
  // thread (h, L): tokens t = (L & 15) + 16 h, columns n0 + 4 (L >> 4) .. +3, summed over the waves in order
  const int L = threadIdx.x & 63, h = threadIdx.x >> 6;
  f32x4_t s = red[0][h][L];
#pragma unroll
  for (int i = 1; i < SK_W; ++i) s += red[i][h][L];
  const int t = (L & 15) + 16 * h, n = n0 + 4 * (L >> 4);
  if (t >= M) return;
  if (ws) {
    *reinterpret_cast<f32x4_t*>(ws + ((long long)blockIdx.y * M + t) * N + n) = s;
  } else {
    float v[4] = {s[0], s[1], s[2], s[3]};
    sk_epilogue(v, (long long)t * ldc + n, R, Zout, C, alpha, act);
  }
}

// C[t][n..n+3] = epilogue(sum over slabs s (in order) of ws[s][t][n..n+3])
__global__ __launch_bounds__(256) void skinny_combine_kernel(const float* __restrict__ ws, bf16_t* __restrict__ C,
                                                             int ldc, const bf16_t* R, bf16_t* Zout, float alpha,
                                                             int act, int M, int N, int KS) {
  const long long i4 = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i4 * 4 >= (long long)M * N) return;
  const int m = (int)(i4 * 4 / N), n = (int)(i4 * 4 % N);
  f32x4_t s = *reinterpret_cast<const f32x4_t*>(ws + i4 * 4);
  for (int k = 1; k < KS; ++k) s += *reinterpret_cast<const f32x4_t*>(ws + (long long)k * M * N + i4 * 4);
  float v[4] = {s[0], s[1], s[2], s[3]};
  sk_epilogue(v, (long long)m * ldc + n, R, Zout, C, alpha, act);
}

int ksplit_for(int M, int N, int K) {
  // >= 256 blocks (one per CU) for the narrow shapes while every wave keeps >= 2 k-steps
  const int tiles = N / SK_NT;
  int ks = 1;
  while (tiles * ks < 256 && (K / 32) / (ks * 2) >= 2 * SK_W && ks < 16) ks *= 2;
  return ks;
}

}  // namespace

// floats of fp32 workspace obst_skinny_gemm needs (0: single pass)
OBST_API long long obst_skinny_ws(int M, int N, int K) {
  const int ks = ksplit_for(M, N, K);
  return ks > 1 ? (long long)ks * M * N : 0;
}

// A [M][K] (lda), Wt [N][K] (ldw: the K-contiguous weight copy), C [M][N] (ldc); M <= 32, N % 16 == 0, K % 32 == 0,
// 16-byte aligned A / Wt rows; ws: obst_skinny_ws(M, N, K) floats (or null when that is 0). Epilogue:
// C = act(alpha * A.W + R), Zout = alpha * A.W + R (R / Zout: bf16 in C's layout, or null; act: ACT_*).
OBST_API int obst_skinny_gemm(const void* A, int lda, const void* Wt, int ldw, void* C, int ldc, int M, int N, int K,
                              float* ws, const void* R, void* Zout, float alpha, int act, hipStream_t st) {
  if (M <= 0 || M > 32 || N <= 0 || K <= 0 || N % SK_NT || K % 32 || lda % 8 || ldw % 8 || ldc % 4 || lda < K ||
      ldw < K || ldc < N || act < 0 || act > ACT_EXP)
    return -1;
  if ((((uintptr_t)A) | ((uintptr_t)Wt)) & 15 || (((uintptr_t)C) | (uintptr_t)R | (uintptr_t)Zout) & 7) return -2;
  if (((long long)(N - 1) * ldw + K) * 2 >= 0x7fffffffll || ((long long)(M - 1) * lda + K) * 2 >= 0x7fffffffll)
    return -4;   // 32-bit buffer offsets
  const int ks = ksplit_for(M, N, K);
  if (ks > 1 && !ws) return -3;
  const int kchunk = (K / 32 + ks - 1) / ks * 32;
  hipLaunchKernelGGL(skinny_mfma_kernel, dim3(N / SK_NT, ks), dim3(SK_W * 64), 0, st, (const bf16_t*)A, lda,
                     (const bf16_t*)Wt, ldw, (bf16_t*)C, ldc, ks > 1 ? ws : nullptr, (const bf16_t*)R, (bf16_t*)Zout,
                     alpha, act, M, N, K, kchunk);
  if (ks > 1) {
    const long long total4 = (long long)M * N / 4;
    hipLaunchKernelGGL(skinny_combine_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, st, ws,
                       (bf16_t*)C, ldc, (const bf16_t*)R, (bf16_t*)Zout, alpha, act, M, N, ks);
  }
  return (int)hipGetLastError();
}
