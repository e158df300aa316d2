// MFMA issue rate by operand placement: v_mfma_f32_32x32x16_bf16 chains with the accumulator in VGPRs or AGPRs and
// the B operand in VGPRs or AGPRs (one wave per SIMD, 4 accumulators interleaved). Build:
//   hipcc --offload-arch=gfx950 -O3 -o bin/mfma_operand_bench tools/lab/mfma_operand_bench.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t cvt_pk(float lo, float hi) {
  uint32_t r;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

template <int MODE>   // 0: acc v, B v; 1: acc v, B a; 2: acc a, B v; 3: acc a, B a
__global__ __launch_bounds__(256, 1) void k(float* out, int iters) {
  f32x16 acc[4];
  for (int j = 0; j < 4; ++j) acc[j] = f32x16{};
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(threadIdx.x * 0.001f + j); b[j] = (__bf16)(j * 0.5f); }
  if (MODE & 1) asm volatile("; b->agpr" : "=a"(b) : "0"(b));
  if (MODE & 2)
    for (int j = 0; j < 4; ++j) asm volatile("; acc->agpr" : "=a"(acc[j]) : "0"(acc[j]));
  asm volatile("s_nop 4");
  uint32_t pk[4][4];
  float fv[8];
  for (int j = 0; j < 8; ++j) fv[j] = threadIdx.x * 0.01f + j;
  for (int g = 0; g < 4; ++g)
    for (int j = 0; j < 4; ++j) pk[g][j] = 0x3f803f80u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (MODE == 0) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc[j]) : "v"(a), "v"(b));
        if (MODE == 1) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc[j]) : "v"(a), "a"(b));
        if (MODE == 2) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(a), "v"(b));
        if (MODE == 3) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(a), "a"(b));
        if (MODE == 4) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc[j & 1]) : "v"(a), "a"(b));
        if (MODE == 5) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc[0]) : "v"(a), "a"(b));
        if (MODE == 6) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc[0]) : "v"(a), "v"(b));
        if (MODE == 7) {   // the PV pattern: B packed by VALU two MFMAs ahead, 4 AGPR accumulators
          const int g = (r * 4 + j) >> 2;
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(a), "v"(__builtin_bit_cast(bf16x8, pk[g & 3])));
          if (j < 2) {
            pk[(g + 1) & 3][2 * j] = cvt_pk(fv[4 * j], fv[4 * j + 1]);
            pk[(g + 1) & 3][2 * j + 1] = cvt_pk(fv[4 * j + 2], fv[4 * j + 3]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4");
  float s = 0.f;
  for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][15];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
void run(float* out, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 2048;
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double fl = 5.0 * blocks * 4 * (double)iters * 32 * 32768;
  const char* names[8] = {"acc v, B v, 4 chains", "acc v, B a, 4 chains", "acc a, B v, 4 chains", "acc a, B a, 4 chains",
                          "acc v, B a, 2 chains", "acc v, B a, 1 chain", "acc a, B v, 1 chain",
                          "acc a, 4 chains, B packed by VALU 2 MFMAs ahead"};
  printf("mode %d (%s): %.1f TF/s\n", MODE, names[MODE], fl / ms / 1e9);
}

int main() {
  float* out;
  hipMalloc(&out, 2048 * 256 * 4);
  const int iters = 200;
  for (int rep = 0; rep < 2; ++rep) {
    run<0>(out, iters);
    run<1>(out, iters);
    run<2>(out, iters);
    run<3>(out, iters);
    run<4>(out, iters);
    run<5>(out, iters);
    run<6>(out, iters);
    run<7>(out, iters);
  }
  hipFree(out);
  return 0;
}
