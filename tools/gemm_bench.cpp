// GEMM harness for the training step's shapes: hipBLASLt vs the MFMA kernels of _kernels.so, same random bf16
// operands, interleaved rounds in one process (cdna guide §5.4 rule 24), plus an element-wise comparison of every
// path against hipBLASLt and a small-shape fp32 CPU check of every layout.
//
//   build: hipcc -O2 --offload-arch=gfx950 tools/gemm_bench.cpp -o build/gemm_bench \
//            -Lhomebrewnlp_mtf_amd -l:_kernels.so -Wl,-rpath,'$ORIGIN/../homebrewnlp_mtf_amd' \
//            tools/lab/blaslt.cpp -lhipblaslt
//   run:   build/gemm_bench [rounds] [reps] [shape-filter substring]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../csrc/kernels/gemm_desc.h"

extern "C" int obst_gemm(const ObstGemmDesc* d, hipStream_t stream);
extern "C" int obst_blaslt_set(int on);
int obst_blaslt_gemm(const ObstGemmDesc* d, hipStream_t stream);   // tools/lab/blaslt.cpp (linked in)
extern "C" long long obst_gemm4w_calls();
extern "C" void obst_gemm4w_stamps(unsigned long long* dev);

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

__global__ void fill_kernel(uint16_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    const float f = ((x & 0xffffff) / 8388608.0f) - 1.0f;   // uniform [-1, 1)
    uint32_t u = __float_as_uint(f);
    p[i] = (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
  }
}

struct Shape {
  int M, N, K, a_t, b_t, f32;
  const char* what;
};

// mode: 0 hipBLASLt (tools/lab/blaslt.cpp), else the framework's dispatch (gemm4w)
static int run(const Shape& s, const void* A, const void* B, void* C, int mode, hipStream_t st) {
  obst_blaslt_set(mode == 0);
  ObstGemmDesc d;
  memset(&d, 0, sizeof(d));
  d.A = A; d.B = B; d.C = C;
  d.lda = s.a_t == 0 ? s.K : s.M;
  d.ldb = s.b_t == 0 ? s.K : s.N;
  d.ldc = s.N;
  d.M = s.M; d.N = s.N; d.K = s.K; d.batch1 = d.batch2 = 1;
  d.a_t = s.a_t; d.b_t = s.b_t; d.out_f32 = s.f32;
  d.alpha = 1.f; d.beta = 0.f;
  return mode == 0 ? obst_blaslt_gemm(&d, st) : obst_gemm(&d, st);
}

static void host_check(hipStream_t st, int K) {
  // fp32 CPU reference of every layout at a small ragged shape, both output types, all three paths
  const int M = 520, N = 264;
  std::vector<uint16_t> ha((size_t)M * K), hb((size_t)N * K);
  for (size_t i = 0; i < ha.size(); ++i) ha[i] = f2bf((float)((i * 7919 % 2003) / 1001.5 - 1.0));
  for (size_t i = 0; i < hb.size(); ++i) hb[i] = f2bf((float)((i * 104729 % 1999) / 999.5 - 1.0));
  uint16_t *dA, *dB;
  void* dC;
  CK(hipMalloc(&dA, ha.size() * 2));
  CK(hipMalloc(&dB, hb.size() * 2));
  CK(hipMalloc(&dC, (size_t)M * N * 4));
  CK(hipMemcpy(dA, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
  for (int at = 0; at < 2; ++at)
    for (int bt = 0; bt < 2; ++bt)
      for (int f32 = 0; f32 < 2; ++f32) {
        std::vector<float> ref((size_t)M * N);
        for (int m = 0; m < M; ++m)
          for (int n = 0; n < N; ++n) {
            double acc = 0;
            for (int k = 0; k < K; ++k) {
              const float a = bf2f(at == 0 ? ha[(size_t)m * K + k] : ha[(size_t)k * M + m]);
              const float b = bf2f(bt == 0 ? hb[(size_t)n * K + k] : hb[(size_t)k * N + n]);
              acc += (double)a * b;
            }
            ref[(size_t)m * N + n] = (float)acc;
          }
        for (int mode = 0; mode < 3; ++mode) {
          Shape s{M, N, K, at, bt, f32, "check"};
          CK(hipMemset(dC, 0, (size_t)M * N * 4));
          const int r = run(s, dA, dB, dC, mode, st);
          CK(hipStreamSynchronize(st));
          std::vector<float> out((size_t)M * N);
          if (f32) {
            CK(hipMemcpy(out.data(), dC, out.size() * 4, hipMemcpyDeviceToHost));
          } else {
            std::vector<uint16_t> o16(out.size());
            CK(hipMemcpy(o16.data(), dC, o16.size() * 2, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < out.size(); ++i) out[i] = bf2f(o16[i]);
          }
          size_t bad = 0;
          double maxe = 0;
          for (size_t i = 0; i < out.size(); ++i) {
            const double e = fabs(out[i] - ref[i]);
            maxe = e > maxe ? e : maxe;
            if (e > 0.05 + 0.01 * fabs(ref[i])) ++bad;
          }
          printf("check K=%d a_t=%d b_t=%d f32=%d mode=%d rc=%d: %zu bad, max err %.4g\n", K, at, bt, f32, mode, r, bad,
                 maxe);
        }
      }
  CK(hipFree(dA));
  CK(hipFree(dB));
  CK(hipFree(dC));
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const int rounds = argc > 1 ? atoi(argv[1]) : 3;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const char* filt = argc > 3 ? argv[3] : "";
  hipStream_t st;
  CK(hipStreamCreate(&st));
  if (!getenv("SKIP_CHECK"))
    for (int K : {64, 192, 576}) host_check(st, K);
  const Shape shapes[] = {
      {131072, 4096, 2048, 0, 0, 0, "fwd d->2d (qkv/ffn-in)"},
      {131072, 2048, 4096, 0, 0, 0, "fwd 2d->d / dgrad"},
      {131072, 6144, 4096, 0, 0, 0, "fwd kqv 2d->6d"},
      {131072, 4096, 6144, 0, 0, 0, "dgrad 6d->2d"},
      {131072, 50304, 2048, 0, 0, 0, "logits"},
      {131072, 2048, 50304, 0, 0, 0, "logits dgrad"},
      {4096, 2048, 131072, 0, 1, 1, "wgrad 01 4096x2048"},
      {2048, 4096, 131072, 0, 1, 1, "wgrad 01 2048x4096"},
      {4096, 2048, 131072, 1, 0, 1, "wgrad 10 4096x2048"},
      {4096, 2048, 131072, 1, 1, 1, "wgrad 11 4096x2048"},
      {2048, 4096, 131072, 1, 1, 1, "wgrad 11 2048x4096"},
      {2048, 6144, 131072, 1, 1, 1, "wgrad 11 2048x6144"},
      {131072, 2048, 4096, 0, 1, 0, "dgrad on stored [K][N] weights"},
      {2048, 50304, 131072, 0, 1, 1, "wgrad logits"},
      {8192, 8192, 8192, 0, 0, 0, "8192^3"},
  };
  for (const Shape& s : shapes) {
    char name[160];
    snprintf(name, sizeof(name), "%dx%dx%d a%d b%d %s %s", s.M, s.N, s.K, s.a_t, s.b_t, s.f32 ? "f32" : "bf16", s.what);
    if (*filt && !strstr(name, filt)) continue;
    const size_t na = (size_t)s.M * s.K, nb = (size_t)s.N * s.K, nc = (size_t)s.M * s.N;
    uint16_t *A, *B;
    void *C0, *C1;
    CK(hipMalloc(&A, na * 2));
    CK(hipMalloc(&B, nb * 2));
    CK(hipMalloc(&C0, nc * (s.f32 ? 4 : 2)));
    CK(hipMalloc(&C1, nc * (s.f32 ? 4 : 2)));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, A, na, 1234u);
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, B, nb, 987u);
    // correctness of each path against hipBLASLt on the full shape
    int rc0 = run(s, A, B, C0, 0, st);
    for (int mode = 1; mode < 3; ++mode) {
      CK(hipMemsetAsync(C1, 0, nc * (s.f32 ? 4 : 2), st));
      const long long c4 = obst_gemm4w_calls();
      int rc = run(s, A, B, C1, mode, st);
      CK(hipStreamSynchronize(st));
      const bool took4w = obst_gemm4w_calls() > c4;
      // compare on the host, strided sample of rows
      size_t bad = 0, cnt = 0;
      double maxe = 0, maxr = 0;
      const int step = s.M > 4096 ? 97 : 1;
      std::vector<uint32_t> r0(s.N), r1(s.N);
      for (int m = 0; m < s.M; m += step) {
        const size_t off = (size_t)m * s.N * (s.f32 ? 4 : 2);
        CK(hipMemcpy(r0.data(), (char*)C0 + off, (size_t)s.N * (s.f32 ? 4 : 2), hipMemcpyDeviceToHost));
        CK(hipMemcpy(r1.data(), (char*)C1 + off, (size_t)s.N * (s.f32 ? 4 : 2), hipMemcpyDeviceToHost));
        for (int n = 0; n < s.N; ++n) {
          float x, y;
          if (s.f32) {
            memcpy(&x, &r0[n], 4);
            memcpy(&y, &r1[n], 4);
          } else {
            x = bf2f(((uint16_t*)r0.data())[n]);
            y = bf2f(((uint16_t*)r1.data())[n]);
          }
          const double e = fabs((double)x - y);
          maxe = e > maxe ? e : maxe;
          maxr = fabs(x) > maxr ? fabs(x) : maxr;
          if (e > 0.02 * sqrt(s.K / 64.0) + 0.01 * fabs(x)) ++bad;
          ++cnt;
        }
      }
      printf("%-58s mode %d rc %d (lt rc %d)%s: %zu/%zu bad, max err %.4g (max |ref| %.4g)\n", name, mode, rc, rc0,
             mode == 2 && !took4w ? " [4w NOT taken]" : "", bad, cnt, maxe, maxr);
    }
    // interleaved timing
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    double best[3] = {1e30, 1e30, 1e30}, sum[3] = {0, 0, 0};
    for (int r = 0; r < rounds; ++r)
      for (int mode = 0; mode < 3; ++mode) {
        run(s, A, B, C1, mode, st);   // warm (plans, workspaces)
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < reps; ++i) run(s, A, B, C1, mode, st);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double t = ms / reps;
        best[mode] = t < best[mode] ? t : best[mode];
        sum[mode] += t;
      }
    const double fl = 2.0 * s.M * s.N * (double)s.K;
    if (getenv("STAMPS")) {   // per-block phase breakdown of one gemm4w launch (shader clocks / real time)
      const long long nblk = 256;   // persistent: one block per CU
      unsigned long long* ds;
      CK(hipMalloc(&ds, nblk * 64));
      CK(hipMemset(ds, 0, nblk * 64));
      obst_gemm4w_stamps(ds);
      run(s, A, B, C1, 2, st);
      CK(hipStreamSynchronize(st));
      obst_gemm4w_stamps(nullptr);
      std::vector<unsigned long long> h(nblk * 8);
      CK(hipMemcpy(h.data(), ds, nblk * 64, hipMemcpyDeviceToHost));
      double pro = 0, s2 = 0, loop = 0, epi = 0, span_rt = 0, tiles = 0;
      unsigned long long rt_min = ~0ull, rt_max = 0;
      long long nb = 0;
      for (long long b = 0; b < nblk; ++b) {   // [start, first landed, loop clocks, epilogue clocks, xcc, rt0, rt1, tiles]
        const unsigned long long* t = &h[b * 8];
        if (!t[6]) continue;
        ++nb;
        pro += (double)t[0];   // PROF build: clocks at sync 1 (lgkmcnt + barrier), sync 2 in t[1]
        s2 += (double)t[1];
        loop += (double)t[2];
        epi += (double)t[3];
        tiles += (double)t[7];
        span_rt += (double)(t[6] - t[5]);
        rt_min = t[5] < rt_min ? t[5] : rt_min;
        rt_max = t[6] > rt_max ? t[6] : rt_max;
      }
      printf("%-58s stamps: %lld blocks, %.1f tiles/block, per tile clocks: loop %.0f (sync1 %.0f, sync2 %.0f) "
             "epilogue %.0f; mean block %.1f us, launch span %.1f us, busy %.3f\n",
             name, nb, tiles / nb, loop / tiles, pro / tiles, s2 / tiles, epi / tiles, span_rt / nb / 100.0,
             (rt_max - rt_min) / 100.0, span_rt / nb / (double)(rt_max - rt_min));
      CK(hipFree(ds));
    }
    printf("%-58s TF/s best (mean): hipBLASLt %.0f (%.0f)  phase %.0f (%.0f)  4w %.0f (%.0f)   4w/lt %.3f\n", name,
           fl / best[0] / 1e9, fl / (sum[0] / rounds) / 1e9, fl / best[1] / 1e9, fl / (sum[1] / rounds) / 1e9,
           fl / best[2] / 1e9, fl / (sum[2] / rounds) / 1e9, best[0] / best[2]);
    fflush(stdout);
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C0));
    CK(hipFree(C1));
  }
  return 0;
}
