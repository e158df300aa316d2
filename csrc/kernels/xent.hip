// K10: fused softmax cross-entropy + z-loss + accuracy over the vocabulary row
// (reference src/mtf_wrapper.py:64-71, src/model/__init__.py:183-187):
//   loss = -mean(logit_y - logZ) + z_loss * mean(logZ^2);  acc = mean(argmax == y)
// Forward: one 256-thread block per row, one pass of 16-byte bf16 loads with an online (max, sum-exp) per lane,
// wave64 shuffles + LDS to combine; writes per-row logZ, loss and hit. Backward recomputes p from logZ and writes
// d logits = g * (p - onehot + 2 z logZ p) in place (bf16). Columns >= V (vocab padded to a multiple of 256
// for the GEMM) are ignored in the forward and get zero gradient.
#include "common.h"

namespace {
constexpr int NTH = 256;

__global__ __launch_bounds__(NTH) void xent_fwd_kernel(const bf16_t* __restrict__ L, const int* __restrict__ tgt,
                                                       float* __restrict__ lse_out, float* __restrict__ loss_out,
                                                       float* __restrict__ hit_out, int V, int Vp, float zl) {
  __shared__ float sm[4], ss[4], sv[4];
  __shared__ int si[4];
  const long long row = blockIdx.x;
  const bf16_t* x = L + row * Vp;
  const int y = tgt[row];
  float m = -INFINITY, s = 0.f, best = -INFINITY;
  int bi = 0x7fffffff;
  for (int c = threadIdx.x * 8; c < V; c += NTH * 8) {
    uint4 u = *reinterpret_cast<const uint4*>(x + c);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
    float f[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) { f[2 * j] = bf2f(w[j] & 0xffff); f[2 * j + 1] = bf2f(w[j] >> 16); }
    float lm = m;
#pragma unroll
    for (int j = 0; j < 8; ++j) if (c + j < V) lm = fmaxf(lm, f[j]);
    s *= __expf(m - lm);
    m = lm;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (c + j < V) {
        s += __expf(f[j] - m);
        if (f[j] > best) { best = f[j]; bi = c + j; }
      }
  }
  // wave combine
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    const float b2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    const float mn = fmaxf(m, m2);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
    m = mn;
    if (b2 > best || (b2 == best && i2 < bi)) { best = b2; bi = i2; }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[w] = m; ss[w] = s; sv[w] = best; si[w] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], Ssum = 0.f, B = sv[0];
    int I = si[0];
    for (int k = 1; k < 4; ++k) M = fmaxf(M, sm[k]);
    for (int k = 0; k < 4; ++k) Ssum += ss[k] * __expf(sm[k] - M);
    for (int k = 1; k < 4; ++k) if (sv[k] > B || (sv[k] == B && si[k] < I)) { B = sv[k]; I = si[k]; }
    const float lse = M + __logf(Ssum);
    const float ly = (y >= 0 && y < V) ? bf2f(x[y]) : 0.f;
    lse_out[row] = lse;
    loss_out[row] = -(ly - lse) + zl * lse * lse;
    hit_out[row] = (I == y) ? 1.f : 0.f;
  }
}

__global__ __launch_bounds__(NTH) void xent_bwd_kernel(const bf16_t* __restrict__ L, const int* __restrict__ tgt,
                                                       const float* __restrict__ lse_in, bf16_t* __restrict__ G,
                                                       const float* __restrict__ gscale_ptr, float gscale, int V,
                                                       int Vp, float zl) {
  const long long row = blockIdx.x;
  const bf16_t* x = L + row * Vp;
  bf16_t* gx = G + row * Vp;
  const int y = tgt[row];
  const float lse = lse_in[row];
  const float g = gscale * (gscale_ptr ? gscale_ptr[0] : 1.f);
  const float zf = 1.f + 2.f * zl * lse;
  for (int c = threadIdx.x * 8; c < Vp; c += NTH * 8) {
    uint4 u = *reinterpret_cast<const uint4*>(x + c);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
    float f[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) { f[2 * j] = bf2f(w[j] & 0xffff); f[2 * j + 1] = bf2f(w[j] >> 16); }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = c + j;
      float d = 0.f;
      if (col < V) {
        const float p = __expf(f[j] - lse);
        d = g * (p * zf - (col == y ? 1.f : 0.f));
      }
      f[j] = d;
    }
    *reinterpret_cast<uint4*>(gx + c) = make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]),
                                                   pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7]));
  }
}
}  // namespace

OBST_API int obst_xent_fwd(const void* L, const int* tgt, float* lse, float* loss, float* hit, long long rows, int V,
                           int Vp, float zl, hipStream_t st) {
  if (Vp % 8 || V > Vp || rows <= 0) return -1;
  hipLaunchKernelGGL(xent_fwd_kernel, dim3((unsigned)rows), dim3(NTH), 0, st, (const bf16_t*)L, tgt, lse, loss, hit, V,
                     Vp, zl);
  return (int)hipGetLastError();
}

OBST_API int obst_xent_bwd(const void* L, const int* tgt, const float* lse, void* G, const float* gscale_ptr,
                           float gscale, long long rows, int V, int Vp, float zl, hipStream_t st) {
  if (Vp % 8 || V > Vp || rows <= 0) return -1;
  hipLaunchKernelGGL(xent_bwd_kernel, dim3((unsigned)rows), dim3(NTH), 0, st, (const bf16_t*)L, tgt, lse, (bf16_t*)G,
                     gscale_ptr, gscale, V, Vp, zl);
  return (int)hipGetLastError();
}
