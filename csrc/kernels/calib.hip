// Same-process calibration kernels for the perf gate (tools/kbench.py): a bare bf16 MFMA loop -- what the chip's
// matrix pipes deliver on random operands at the clock it holds right now -- so kernel floors can be stated as
// box-independent ratios (MI355X_MICROARCH.md 'DVFS give-back': devices differ by up to 12 % on an MFMA loop).
#include "common.h"

#pragma clang diagnostic ignored "-Winline-asm"

namespace {

__device__ __forceinline__ float calib_rand(unsigned x) {
  x *= 2654435761u;
  x ^= x >> 13;
  x *= 0x5bd1e995u;
  x ^= x >> 15;
  return ((x & 0xffffff) / 8388608.0f - 1.0f) * 0.125f;   // uniform [-1/8, 1/8)
}

// 2048 blocks of 4 waves (the dispatcher does not promise one 256-thread block per CU: with exactly 256 blocks some
// CUs got two and the loop measured 0.8 PF/s), 8 independent accumulators of v_mfma_f32_16x16x32_bf16 on random
// register operands; the result is stored only when it equals an impossible value (kept live, never written)
__global__ __launch_bounds__(256) void calib_mfma_kernel(float* out, int iters, unsigned seed) {
  const unsigned t = blockIdx.x * 256u + threadIdx.x;
  bf16x8_t a[2], b[4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) a[i][e] = (__bf16)calib_rand(seed ^ (t * 64u + i * 8u + e));
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) b[i][e] = (__bf16)calib_rand(~seed ^ (t * 64u + i * 8u + e));
  f32x4_t acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // accumulators pinned to AGPRs by tied asm operands (as builtins the allocator rotated them through VGPR copies
  // every iteration), 32 MFMAs per trip
  for (int it = 0; it < iters; it += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(a[j & 1]), "v"(b[j >> 1]));
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3]), "+a"(acc[4]),
               "+a"(acc[5]), "+a"(acc[6]), "+a"(acc[7]));
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  if (s == 1.2345e38f) out[t] = s;
}

}  // namespace

constexpr int CALIB_BLOCKS = 2048;

// FLOPs of one obst_calib_mfma call: CALIB_BLOCKS blocks x 4 waves x iters x 8 MFMAs x 16 x 16 x 32 x 2
OBST_API double obst_calib_mfma_flops(int iters) { return (double)CALIB_BLOCKS * 4 * iters * 8 * 16384.0; }

OBST_API int obst_calib_mfma(float* out, int iters, hipStream_t st) {
  if (iters <= 0 || !out) return -1;
  hipLaunchKernelGGL(calib_mfma_kernel, dim3(CALIB_BLOCKS), dim3(256), 0, st, out, iters, 0x9e3779b9u);
  return (int)hipGetLastError();
}
