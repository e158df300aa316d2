// gemm4w schedule variants (csrc/kernels/gemm4w.h template knobs SCH / STG / CPA / CPB) against hipBLASLt, one
// process, interleaved rounds on the same random operands (cdna guide §5.4 rule 24), outputs checked against the
// library's on a strided sample of rows.
//
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/kernels tools/lab/g4w_sched.cpp -o bin/g4w_sched \
//            -Lhomebrewnlp_mtf_amd -l:_kernels.so -Wl,-rpath,'$ORIGIN/../homebrewnlp_mtf_amd' \
//            tools/lab/blaslt.cpp -lhipblaslt
//   run:   bin/g4w_sched [rounds] [reps] [shape filter]
#include "gemm4w.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "gemm_desc.h"

extern "C" int obst_gemm(const ObstGemmDesc* d, hipStream_t stream);
extern "C" int obst_blaslt_set(int on);
int obst_blaslt_gemm(const ObstGemmDesc* d, hipStream_t stream);   // tools/lab/blaslt.cpp (linked in)
extern "C" int obst_gemm4w_set(int on);

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

static float h_bf2f(uint16_t h) {
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

template <int A_T, int B_T, bool F32, int SCH, bool STG, int CPA, int CPB, int OPT, bool PROF = false>
hipError_t launch_v(GemmArgs a, hipStream_t st) {
  a.tiles_m = (a.M + 255) / 256;
  a.tiles_n = (a.N + 255) / 256;
  a.nbatch = a.ksplit;
  const long long tiles = (long long)a.tiles_m * a.tiles_n * a.nbatch;
  const int grid = (int)(tiles >= 256 ? 256 : ((tiles + 7) / 8) * 8);
  const size_t lds = 2 * Q_STAGE + 32768;
  auto k = gemm4w_kernel<A_T, B_T, F32, PROF, 4, SCH, STG, CPA, CPB, OPT>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, st, a);
  return hipGetLastError();
}

struct Shape {
  int M, N, K, a_t, b_t, f32;
  const char* what;
};
typedef hipError_t (*Launch)(GemmArgs, hipStream_t);
struct Variant {
  const char* name;
  Launch l00b, l01b, l00b_prof, l11f;
};

#define V(NAME, SCH, STG, CPA, CPB, OPT)                                                             \
  Variant {                                                                                          \
    NAME, launch_v<0, 0, false, SCH, STG, CPA, CPB, OPT>, launch_v<0, 1, false, SCH, STG, CPA, CPB, OPT>, \
        launch_v<0, 0, false, SCH, STG, CPA, CPB, OPT, true>, launch_v<1, 1, true, SCH, STG, CPA, CPB, OPT> \
  }
static const Variant variants[] = {
    V("sch1 tlay", 1, false, 0, 0, 0),
    V("sch1 tlay stag", 1, false, 0, 0, 2),
    V("sch1 tlay relax", 1, false, 0, 0, 1),
    V("sch1 tlay late", 1, false, 0, 0, 4),
};
constexpr int NV = sizeof(variants) / sizeof(variants[0]);

static GemmArgs args_of(const Shape& s, const void* A, const void* B, void* C) {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C;
  a.lda = s.a_t == 0 ? s.K : s.M;
  a.ldb = s.b_t == 0 ? s.K : s.N;
  a.ldc = s.N;
  a.M = s.M; a.N = s.N; a.K = s.K; a.nb2 = 1;
  a.alpha = 1.f; a.beta = 0.f; a.ksplit = 1;
  return a;
}

static bool wanted(int v) {   // G4W_ONLY=0,2: run only these variants
  const char* e = getenv("G4W_ONLY");
  if (!e || !*e) return true;
  std::string l = std::string(",") + e + ",";
  return l.find("," + std::to_string(v) + ",") != std::string::npos;
}

static Launch pick(const Variant& v, const Shape& s) {
  if (s.a_t == 0 && s.b_t == 0 && !s.f32) return v.l00b;
  if (s.a_t == 0 && s.b_t == 1 && !s.f32) return v.l01b;
  if (s.a_t == 1 && s.b_t == 1 && s.f32) return v.l11f;
  return nullptr;
}

static int run_lt(const Shape& s, const void* A, const void* B, void* C, hipStream_t st) {
  obst_blaslt_set(1);
  ObstGemmDesc d;
  memset(&d, 0, sizeof(d));
  d.A = A; d.B = B; d.C = C;
  d.lda = s.a_t == 0 ? s.K : s.M;
  d.ldb = s.b_t == 0 ? s.K : s.N;
  d.ldc = s.N;
  d.M = s.M; d.N = s.N; d.K = s.K; d.batch1 = d.batch2 = 1;
  d.a_t = s.a_t; d.b_t = s.b_t; d.out_f32 = s.f32;
  d.alpha = 1.f; d.beta = 0.f;
  return obst_blaslt_gemm(&d, st);
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const char* filt = argc > 3 ? argv[3] : "";
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const Shape shapes[] = {
      {131072, 4096, 2048, 0, 0, 0, "fwd d->2d"},
      {131072, 2048, 4096, 0, 0, 0, "fwd 2d->d"},
      {131072, 6144, 2048, 0, 0, 0, "fwd qkv"},
      {131072, 50304, 2048, 0, 0, 0, "logits"},
      {8192, 8192, 8192, 0, 0, 0, "8192^3"},
      {131072, 2048, 4096, 0, 1, 0, "dgrad [K][N] weights"},
      {2048, 8192, 131072, 1, 1, 1, "wgrad d x 4d"},
      {512, 512, 2048, 0, 0, 0, "few tiles (4)"},
      {2048, 1024, 2048, 0, 0, 0, "few tiles (32)"},
      {131072, 4096, 128, 0, 0, 0, "K sweep 128"},
      {131072, 4096, 512, 0, 0, 0, "K sweep 512"},
  };
  for (const Shape& s : shapes) {
    char name[160];
    snprintf(name, sizeof(name), "%dx%dx%d a%d b%d %s %s", s.M, s.N, s.K, s.a_t, s.b_t, s.f32 ? "f32" : "bf16", s.what);
    if (*filt && !strstr(name, filt)) continue;
    const size_t na = (size_t)s.M * s.K, nb = (size_t)s.N * s.K, nc = (size_t)s.M * s.N, es = s.f32 ? 4 : 2;
    uint16_t *A, *B;
    void *C0, *C1;
    CK(hipMalloc(&A, na * 2));
    CK(hipMalloc(&B, nb * 2));
    CK(hipMalloc(&C0, nc * es));
    CK(hipMalloc(&C1, nc * es));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, A, na, 1234u);
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, B, nb, 987u);
    const int rc0 = run_lt(s, A, B, C0, st);
    CK(hipStreamSynchronize(st));
    const GemmArgs a = args_of(s, A, B, C1);
    for (int v = 0; v < NV; ++v) {
      Launch l = pick(variants[v], s);
      if (!l || !wanted(v) || getenv("SKIP_CHECK")) continue;
      CK(hipMemsetAsync(C1, 0, nc * es, st));
      CK(l(a, st));
      CK(hipStreamSynchronize(st));
      size_t bad = 0, cnt = 0;
      double maxe = 0;
      const int step = s.M > 4096 ? 97 : 7;
      std::vector<uint8_t> r0(s.N * es), r1(s.N * es);
      for (int m = 0; m < s.M; m += step) {
        CK(hipMemcpy(r0.data(), (char*)C0 + (size_t)m * s.N * es, s.N * es, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r1.data(), (char*)C1 + (size_t)m * s.N * es, s.N * es, hipMemcpyDeviceToHost));
        for (int n = 0; n < s.N; ++n) {
          float x, y;
          if (s.f32) {
            memcpy(&x, &r0[n * 4], 4);
            memcpy(&y, &r1[n * 4], 4);
          } else {
            x = h_bf2f(((uint16_t*)r0.data())[n]);
            y = h_bf2f(((uint16_t*)r1.data())[n]);
          }
          const double e = fabs((double)x - y);
          maxe = e > maxe ? e : maxe;
          if (!(e <= 0.02 * sqrt(s.K / 64.0) + 0.01 * fabs(x))) ++bad;
          ++cnt;
        }
      }
      printf("%-44s %-16s lt rc %d: %zu/%zu bad, max err %.4g\n", name, variants[v].name, rc0, bad, cnt, maxe);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<double>> t(NV + 1);
    for (int r = 0; r < rounds; ++r)
      for (int v = 0; v <= NV; ++v) {
        Launch l = v < NV ? pick(variants[v], s) : nullptr;
        if (v < NV && (!l || !wanted(v))) continue;
        auto go = [&]() { if (v < NV) (void)l(a, st); else run_lt(s, A, B, C1, st); };
        go();
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < reps; ++i) go();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[v].push_back(ms / reps);
      }
    const double fl = 2.0 * s.M * s.N * (double)s.K;
    std::vector<double> lt = t[NV];
    std::sort(lt.begin(), lt.end());
    const double lt_med = lt[lt.size() / 2];
    for (int v = 0; v <= NV; ++v) {
      if (t[v].empty()) continue;
      std::vector<double> x = t[v];
      std::sort(x.begin(), x.end());
      const double med = x[x.size() / 2], best = x[0];
      printf("%-44s %-16s median %8.1f us  best %8.1f us  %6.0f TF/s  vs lt %.3f\n", name,
             v < NV ? variants[v].name : "hipBLASLt", med * 1e3, best * 1e3, fl / med / 1e9, lt_med / med);
    }
    if (getenv("STAMPS") && s.a_t == 0 && s.b_t == 0 && !s.f32) {
      // per-block [sync1 clocks (lgkmcnt + barrier waits), sync2 clocks (vmcnt + barrier waits), loop clocks,
      // epilogue clocks, xcc, realtime start, realtime end, tiles] of one PROF-build launch per variant
      unsigned long long* ds;
      CK(hipMalloc(&ds, 256 * 64));
      for (int v = 0; v < NV; ++v) {
        if (!wanted(v)) continue;
        GemmArgs b = a;
        b.stamps = ds;
        for (int w = 0; w < 3; ++w) CK(variants[v].l00b_prof(b, st));   // warm clocks
        CK(hipMemset(ds, 0, 256 * 64));
        CK(variants[v].l00b_prof(b, st));
        CK(hipStreamSynchronize(st));
        std::vector<unsigned long long> h(256 * 8);
        CK(hipMemcpy(h.data(), ds, 256 * 64, hipMemcpyDeviceToHost));
        double s1 = 0, s2 = 0, loop = 0, epi = 0, tiles = 0, rt = 0, iss = 0;
        int nb = 0;
        for (int i = 0; i < 256; ++i) {
          const unsigned long long* t = &h[i * 8];
          if (!t[6]) continue;
          ++nb;
          s1 += t[0]; s2 += t[1]; loop += t[2]; epi += t[3]; iss += t[4]; tiles += t[7]; rt += (double)(t[6] - t[5]);
        }
        const double nkt = s.K / 64.0;
        printf("%-44s %-16s stamps: per K-tile loop %.0f clk (sync1 %.0f, sync2 %.0f), epilogue %.0f clk/tile, "
               "(stores issued after %.0f), clock %.2f GHz\n", name, variants[v].name, loop / tiles / nkt, s1 / tiles / nkt,
               s2 / tiles / nkt, epi / tiles, iss / tiles, (loop + epi) / (rt / 100.0) / 1e3 / nb * nb);
      }
      CK(hipFree(ds));
    }
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C0));
    CK(hipFree(C1));
  }
  return 0;
}
