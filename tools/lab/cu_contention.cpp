// How much does a persistent GEMM lose when another kernel holds some CUs (as RCCL's all-reduce kernels do while
// the DP gradient sync overlaps the backward GEMMs at N > 1)? One 131072 x 4096 x 2048 bf16 product through
// obst_gemm (gemm4w, or hipBLASLt with OBST_GEMM_LT=1), alone and with a "hog" kernel of H blocks spinning for T us
// launched just before it on a second stream.
//
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/kernels tools/lab/cu_contention.cpp -o bin/cu_contention \
//            -Lhomebrewnlp_mtf_amd -l:_kernels.so -Wl,-rpath,'$ORIGIN/../homebrewnlp_mtf_amd'
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gemm_desc.h"

extern "C" int obst_gemm(const ObstGemmDesc* d, hipStream_t stream);

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                                   \
    }                                                                            \
  } while (0)

// one wave per block, spinning on the 100 MHz real-time counter for `ticks` (every wave reaches the exit)
__global__ __launch_bounds__(64) void hog(unsigned long long ticks, int* sink) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int x = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x += threadIdx.x;
  if (x == -1) sink[0] = x;
}

int main() {
  const int M = 131072, N = 4096, K = 2048;
  void *A, *B, *C;
  int* sink;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 2));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(A, 0, (size_t)M * K * 2));
  CK(hipMemset(B, 0, (size_t)N * K * 2));
  ObstGemmDesc d;
  memset(&d, 0, sizeof(d));
  d.A = A; d.B = B; d.C = C;
  d.lda = K; d.ldb = K; d.ldc = N;
  d.M = M; d.N = N; d.K = K; d.batch1 = d.batch2 = 1;
  d.alpha = 1.f;
  hipStream_t s0, s1;
  CK(hipStreamCreate(&s0));
  CK(hipStreamCreate(&s1));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) if (obst_gemm(&d, s0)) return 3;
  CK(hipDeviceSynchronize());
  const int hogs[] = {0, 16, 32, 64};
  const double us_hog[] = {200.0, 800.0};
  for (double us : us_hog)
    for (int h : hogs) {
      float best = 1e30f, sum = 0.f;
      const int reps = 5;
      for (int r = 0; r < reps; ++r) {
        CK(hipDeviceSynchronize());
        if (h > 0) hipLaunchKernelGGL(hog, dim3(h), dim3(64), 0, s1, (unsigned long long)(us * 100.0), sink);
        CK(hipEventRecord(e0, s0));
        if (obst_gemm(&d, s0)) return 3;
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        sum += ms;
      }
      CK(hipDeviceSynchronize());
      printf("hog %3d blocks x %6.0f us: gemm %8.1f us (best %8.1f)\n", h, us, 1e3 * sum / reps, 1e3 * best);
    }
  return 0;
}
