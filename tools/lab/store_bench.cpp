// Store-path microbenchmark: how fast can one workgroup (4 waves) write a 256 x 256 bf16 tile (128 KiB) with
// 16-byte-per-lane buffer stores, by lane -> address pattern? (gemm4w's epilogue issues its 32 stores per wave in
// ~9.4k clocks whatever the grid size: tools/lab/g4w_sched.cpp stamps.)
//
//   P0 fragment: lane (ml = lane & 15, gq = lane >> 4) -> row ml, 16-byte chunk gq (+ 4 per pp): 16 rows x 64 B
//   P1 rows:     lane -> row lane / 16, chunk lane % 16: 4 rows x 256 B per instruction
//   P2 linear:   1 KiB contiguous per instruction
//   + the same with the compiler's global_store (no inline asm, no pads)
//
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lab/store_bench.cpp -o bin/store_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                                   \
    }                                                                            \
  } while (0)

typedef __attribute__((ext_vector_type(4))) int i32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned v4u32_t;

__device__ __forceinline__ i32x4_t rsrc(const void* base, unsigned n) {
  const unsigned long long a = (unsigned long long)base;
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32));
  r[2] = __builtin_amdgcn_readfirstlane((int)n);
  r[3] = 0x00020000;
  return r;
}

// MODE 0..2: asm buffer stores of pattern P0..P2; MODE 3..5: plain C++ stores (global_store) of the same patterns
template <int MODE>
__global__ __launch_bounds__(256, 1) void store_tile(char* out, int ldc_bytes, int tiles_per_block,
                                                     unsigned long long* clk) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int pat = MODE % 3;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < tiles_per_block; ++t) {
    char* tile = out + ((size_t)blockIdx.x * tiles_per_block + t) * 256 * (size_t)ldc_bytes;
    // this wave's 128 x 128 bf16 quadrant: 128 rows x 256 B
    char* q = tile + (size_t)(wm * 128) * ldc_bytes + wn * 256;
    const i32x4_t rs = rsrc(q, 0x7fffffff);
    v4u32_t v = {(unsigned)lane, (unsigned)t, 1u, 2u};
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      int off;
      if (pat == 0) {   // fragment row s/4 (16 rows), pair pp = s%4
        const int i = s >> 2, pp = s & 3, ml = lane & 15, gq = lane >> 4;
        off = (i * 16 + ml) * ldc_bytes + (pp * 4 + gq) * 16;
      } else if (pat == 1) {   // 4 rows x 256 B
        off = (s * 4 + (lane >> 4)) * ldc_bytes + (lane & 15) * 16;
      } else {   // 1 KiB contiguous: row s*4 + lane/16 of a 4-row block, but rows 256 B apart (packed)
        off = (s * 4 + (lane >> 4)) * ldc_bytes + (lane & 15) * 16;   // same rows as P1 when ldc = 256
      }
      v[2] = s;
      if (MODE < 3) {
        asm volatile("s_nop 4\n\tbuffer_store_dwordx4 %0, %1, %2, 0 offen\n\ts_nop 4" ::"v"(v), "v"(off), "s"(rs)
                     : "memory");
      } else {
        *reinterpret_cast<v4u32_t*>(q + off) = v;
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int MODE>
static void run(const char* name, char* out, int ldc_bytes, int blocks, int tpb, unsigned long long* dclk) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(store_tile<MODE>, dim3(blocks), dim3(256), 0, 0, out, ldc_bytes, tpb, dclk);
  CK(hipEventRecord(e0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(store_tile<MODE>, dim3(blocks), dim3(256), 0, 0, out, ldc_bytes, tpb, dclk);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[256];
  CK(hipMemcpy(h, dclk, sizeof(unsigned long long) * (blocks < 256 ? blocks : 256), hipMemcpyDeviceToHost));
  double avg = 0;
  for (int i = 0; i < (blocks < 256 ? blocks : 256); ++i) avg += (double)h[i];
  avg /= (blocks < 256 ? blocks : 256);
  const double bytes = (double)blocks * tpb * 256.0 * 512.0;
  printf("%-28s ldc %6d B  blocks %4d  tiles/block %3d: %8.1f clk per tile (block-side), %7.1f GB/s\n", name,
         ldc_bytes, blocks, tpb, avg / tpb, bytes / (ms / reps * 1e-3) / 1e9);
}

int main() {
  char* out;
  const size_t cap = (size_t)4 << 30;
  CK(hipMalloc(&out, cap));
  unsigned long long* dclk;
  CK(hipMalloc(&dclk, 256 * 8));
  const int ldcs[] = {512, 1024, 8192, 100608};
  for (int ldc : ldcs) {
    for (int blocks : {1, 8, 256}) {
      int tpb = 8;
      while ((size_t)blocks * tpb * 256 * (size_t)ldc > cap && tpb > 1) tpb /= 2;
      if ((size_t)blocks * tpb * 256 * (size_t)ldc > cap) continue;
      run<0>("asm fragment (16r x 64B)", out, ldc, blocks, tpb, dclk);
      run<1>("asm rows (4r x 256B)", out, ldc, blocks, tpb, dclk);
      run<3>("c++ fragment", out, ldc, blocks, tpb, dclk);
      run<4>("c++ rows", out, ldc, blocks, tpb, dclk);
    }
  }
  CK(hipFree(out));
  return 0;
}
