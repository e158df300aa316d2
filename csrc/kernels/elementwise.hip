// K06/K07/K08/K09/K13 and small memory-bound helpers. Every kernel moves bf16 as 16-byte vectors (8 elements
// per lane, Guideline 13) with a grid-stride loop capped at 256 CUs x 8 blocks (Guideline 11).
//  * activations fwd/bwd (src/model/activation.py: relu, sigmoid, tanh, gelu, lecun_tanh, silu, mish, softsign, exp)
//  * residual add, rezero (x * g), dropout (counter-based hash RNG, keep-mask recomputed in backward)
//  * embedding gather (K08, src/model/embedding.py:91-125) and scatter-add gradient (K09) into the fp32 grad buffer
//  * cumsum / cummean along the sequence (K13, src/model/spatial.py:26-39) and its reverse-cumsum gradient
#include "common.h"
#include <stdlib.h>

namespace {

constexpr int NTH = 256;

// Streaming elementwise launches: one 16-byte vector per thread, grid = all of them (the dispatcher keeps every CU
// full; a grid-stride loop over 2048 blocks left one load in flight per lane, ~40 KiB per CU): gelu forward on
// [131072][4096] 508 -> 429 us, backward 747 -> 553 us, residual add 348 -> 268 us (6.0 TB/s). OBST_EW_CAP caps the
// block count again (A/B knob).
inline long long ew_cap() {
  static long long v = -1;
  if (v < 0) {
    const char* e = getenv("OBST_EW_CAP");
    v = e ? atoll(e) : (1ll << 30);
  }
  return v;
}

inline int grid_ew(long long n_vec) {
  long long g = (n_vec + NTH - 1) / NTH;
  const long long cap = ew_cap();
  return (int)(g < cap ? (g < 1 ? 1 : g) : cap);
}

inline int grid_for(long long n_vec) {
  long long g = (n_vec + NTH - 1) / NTH;
  return (int)(g < 2048 ? (g < 1 ? 1 : g) : 2048);
}

__device__ __forceinline__ void unpack8(const uint4& u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) { f[2 * j] = bf2f(w[j] & 0xffff); f[2 * j + 1] = bf2f(w[j] >> 16); }
}

__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7]));
}

// op: 0 act fwd (y=act(x)), 1 act bwd (y = dy * act'(x)), 2 add (y = x + z), 3 mul scalar tensor (y = x * s[0]),
//     4 dropout fwd/bwd (y = x * keep(i) / keep_prob), 5 axpby (y = alpha*x + beta*z), 6 mul (y = x*z)
// OP / ACT as template parameters (-1: taken from the runtime arguments) so the hot instances -- gelu forward and
// backward, residual add -- carry no per-element dispatch
template <int OP, int ACT>
__global__ __launch_bounds__(NTH) void ew_kernel(int op_rt, int act_rt, const bf16_t* __restrict__ X,
                                                 const bf16_t* __restrict__ Z, bf16_t* __restrict__ Y, long long nvec,
                                                 const float* __restrict__ sptr, float alpha, float beta,
                                                 unsigned long long seed, float keep) {
  const int op = OP >= 0 ? OP : op_rt;
  const int act = ACT >= 0 ? ACT : act_rt;
  for (long long v = (long long)blockIdx.x * NTH + threadIdx.x; v < nvec; v += (long long)gridDim.x * NTH) {
    float x[8], z[8];
    unpack8(reinterpret_cast<const uint4*>(X)[v], x);
    if (op == 1 || op == 2 || op == 5 || op == 6) unpack8(reinterpret_cast<const uint4*>(Z)[v], z);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float r;
      switch (op) {
        case 0: r = act_fwd(act, x[j]); break;
        case 1: r = z[j] * act_grad(act, x[j]); break;  // X = saved input, Z = dy
        case 2: r = x[j] + z[j]; break;
        case 3: r = x[j] * sptr[0]; break;
        case 4: {
          unsigned long long h = (unsigned long long)(v * 8 + j) * 0x9E3779B97F4A7C15ull ^ seed;
          h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull; h ^= h >> 33;
          const float u = (float)(h >> 40) * (1.f / 16777216.f);
          r = u < keep ? x[j] / keep : 0.f;
          break;
        }
        case 5: r = alpha * x[j] + beta * z[j]; break;
        case 6: r = x[j] * z[j]; break;
        default: r = x[j];
      }
      x[j] = r;
    }
    reinterpret_cast<uint4*>(Y)[v] = pack8(x);
  }
}

// sum of x*dy over all elements (rezero gradient: d g = sum(x * dy)): one partial per block into part[blockIdx.x],
// then dot_fold_kernel adds the partials to out[0] in block order (bitwise reproducible, no float atomics)
__global__ __launch_bounds__(NTH) void dot_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ DY,
                                                  float* __restrict__ part, long long nvec) {
  __shared__ float red[4];
  float acc = 0.f;
  for (long long v = (long long)blockIdx.x * NTH + threadIdx.x; v < nvec; v += (long long)gridDim.x * NTH) {
    float x[8], d[8];
    unpack8(reinterpret_cast<const uint4*>(X)[v], x);
    unpack8(reinterpret_cast<const uint4*>(DY)[v], d);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += x[j] * d[j];
  }
  acc = block_sum<4>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// out[0] += sum of part[0..n) in a fixed order (one block: strided per-thread sums, then the block tree)
__global__ __launch_bounds__(NTH) void dot_fold_kernel(const float* __restrict__ part, int n, float* __restrict__ out) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += NTH) acc += part[i];
  acc = block_sum<4>(acc, red);
  if (threadIdx.x == 0) out[0] += acc;
}

// out[t, :] = E[idx[t], :]   (E bf16 [V, F], F % 8 == 0)
__global__ __launch_bounds__(NTH) void gather_kernel(const int* __restrict__ idx, const bf16_t* __restrict__ E,
                                                     bf16_t* __restrict__ out, long long T, int F, int V) {
  const int vpr = F / 8;
  const long long n = T * vpr;
  for (long long v = (long long)blockIdx.x * NTH + threadIdx.x; v < n; v += (long long)gridDim.x * NTH) {
    const long long t = v / vpr;
    const int c = v % vpr;
    int r = idx[t];
    r = r < 0 ? 0 : (r >= V ? V - 1 : r);
    reinterpret_cast<uint4*>(out)[v] = reinterpret_cast<const uint4*>(E + (long long)r * F)[c];
  }
}

// dE[idx[t], :] += dy[t, :]   (fp32 atomics; each wave-instruction covers 256 contiguous bytes of one row)
__global__ __launch_bounds__(NTH) void scatter_add_kernel(const int* __restrict__ idx, const bf16_t* __restrict__ DY,
                                                          float* __restrict__ dE, long long T, int F, int V) {
  const long long n = T * F;
  for (long long e = (long long)blockIdx.x * NTH + threadIdx.x; e < n; e += (long long)gridDim.x * NTH) {
    const long long t = e / F;
    const int c = e % F;
    int r = idx[t];
    r = r < 0 ? 0 : (r >= V ? V - 1 : r);
    atomicAdd(dE + (long long)r * F + c, bf2f(DY[e]));
  }
}

// Deterministic embedding gradient: the token ids are sorted (stable) on the host side's stream, so the rows
// that add into one table row form a segment of the sorted order. One block per sorted position; the block that
// starts a segment sums the segment's dy rows in sorted order (8 columns per lane, 16-byte loads) and adds the sum
// to its table row -- every row is owned by one block, so the result is bitwise reproducible (no float atomics).
__global__ __launch_bounds__(NTH) void scatter_sorted_kernel(const int* __restrict__ sidx,
                                                             const long long* __restrict__ perm,
                                                             const bf16_t* __restrict__ DY, float* __restrict__ dE,
                                                             long long T, int F) {
  const long long i = blockIdx.x;
  const int r = sidx[i];
  if (i > 0 && sidx[i - 1] == r) return;
  long long j = i + 1;
  while (j < T && sidx[j] == r) ++j;
  float* row = dE + (long long)r * F;
  for (int c0 = threadIdx.x * 8; c0 < F; c0 += NTH * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (long long k = i; k < j; ++k) {
      float d[8];
      unpack8(*reinterpret_cast<const uint4*>(DY + perm[k] * F + c0), d);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += d[e];
    }
    float4* o = reinterpret_cast<float4*>(row + c0);
    float4 a = o[0], b = o[1];
    a.x += acc[0]; a.y += acc[1]; a.z += acc[2]; a.w += acc[3];
    b.x += acc[4]; b.y += acc[5]; b.z += acc[6]; b.w += acc[7];
    o[0] = a;
    o[1] = b;
  }
}

// Chunked form of the same (bounded work per block under skewed ids -- a padding id can own tens of thousands of
// rows): the sorted order is cut into fixed chunks of SC_CH positions. A run of equal ids that lies inside one chunk
// is summed and added to its table row by that chunk's block. A run that crosses a chunk boundary leaves one partial
// row per chunk it touches: "head" (the chunk's first run, continued from before) or "tail" (the chunk's last run,
// continuing after); the fold block of the chunk where the run starts adds its tail and the following heads in chunk
// order. Every sum has a fixed order: bitwise reproducible. scale (optional, per ORIGINAL row): dy[r] * scale[r].
constexpr int SC_CH = 64;

__device__ __forceinline__ void sc_row(const bf16_t* DY, const float* scale, long long r, int F, int c0, float (&acc)[8]) {
  float d[8];
  unpack8(*reinterpret_cast<const uint4*>(DY + r * F + c0), d);
  const float sv = scale ? scale[r] : 1.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] += d[e] * sv;
}

__device__ __forceinline__ void sc_add(float* dst, int c0, const float (&acc)[8]) {
  float4* o = reinterpret_cast<float4*>(dst + c0);
  float4 a = o[0], b = o[1];
  a.x += acc[0]; a.y += acc[1]; a.z += acc[2]; a.w += acc[3];
  b.x += acc[4]; b.y += acc[5]; b.z += acc[6]; b.w += acc[7];
  o[0] = a;
  o[1] = b;
}

__device__ __forceinline__ void sc_put(float* dst, int c0, const float (&acc)[8]) {
  reinterpret_cast<float4*>(dst + c0)[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
  reinterpret_cast<float4*>(dst + c0)[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
}

// ws: head [nchunk][F] then tail [nchunk][F]
__global__ __launch_bounds__(NTH) void scatter_chunk_kernel(const int* __restrict__ sidx, const long long* __restrict__ perm,
                                                            const bf16_t* __restrict__ DY, const float* __restrict__ scale,
                                                            float* __restrict__ dE, float* __restrict__ ws, long long T,
                                                            int F) {
  const long long c = blockIdx.x, nchunk = gridDim.x;
  const long long p0 = c * SC_CH, p1 = p0 + SC_CH < T ? p0 + SC_CH : T;
  const bool from_prev = p0 > 0 && sidx[p0 - 1] == sidx[p0];
  const bool to_next = p1 < T && sidx[p1] == sidx[p1 - 1];
  float* head = ws + c * F;
  float* tail = ws + (nchunk + c) * F;
  for (int c0 = threadIdx.x * 8; c0 < F; c0 += NTH * 8) {
    long long i = p0;
    while (i < p1) {
      const int key = sidx[i];
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      long long j = i;
      for (; j < p1 && sidx[j] == key; ++j) sc_row(DY, scale, perm[j], F, c0, acc);
      const bool first = i == p0 && from_prev, last = j == p1 && to_next;
      if (first) sc_put(head, c0, acc);            // continued run (also when it spans the whole chunk)
      else if (last) sc_put(tail, c0, acc);        // run starting here, continuing after
      else sc_add(dE + (long long)key * F, c0, acc);
      i = j;
    }
  }
}

__global__ __launch_bounds__(NTH) void scatter_fold_kernel(const int* __restrict__ sidx, float* __restrict__ dE,
                                                           const float* __restrict__ ws, long long T, int F) {
  const long long c = blockIdx.x, nchunk = gridDim.x;
  const long long p0 = c * SC_CH, p1 = p0 + SC_CH < T ? p0 + SC_CH : T;
  if (!(p1 < T && sidx[p1] == sidx[p1 - 1])) return;                  // the chunk's last run ends here
  const int key = sidx[p1 - 1];
  if (p0 > 0 && sidx[p0 - 1] == key && sidx[p0] == key) return;       // the run started in an earlier chunk
  for (int c0 = threadIdx.x * 8; c0 < F; c0 += NTH * 8) {
    float acc[8];
    const float4 a = reinterpret_cast<const float4*>(ws + (nchunk + c) * F + c0)[0];
    const float4 b = reinterpret_cast<const float4*>(ws + (nchunk + c) * F + c0)[1];
    acc[0] = a.x; acc[1] = a.y; acc[2] = a.z; acc[3] = a.w; acc[4] = b.x; acc[5] = b.y; acc[6] = b.z; acc[7] = b.w;
    for (long long k = c + 1; k < nchunk; ++k) {
      const float4 x = reinterpret_cast<const float4*>(ws + k * F + c0)[0];
      const float4 y = reinterpret_cast<const float4*>(ws + k * F + c0)[1];
      acc[0] += x.x; acc[1] += x.y; acc[2] += x.z; acc[3] += x.w; acc[4] += y.x; acc[5] += y.y; acc[6] += y.z;
      acc[7] += y.w;
      const long long q1 = (k + 1) * SC_CH < T ? (k + 1) * SC_CH : T;
      if (sidx[q1 - 1] != key || q1 == T || sidx[q1] != key) break;    // the run ends inside chunk k
    }
    sc_add(dE + (long long)key * F, c0, acc);
  }
}

// cumulative sum over the sequence axis of x viewed as [outer, S, inner]; reverse for the gradient; cummean
// divides by (position + 1) (backward of cummean = reverse-cumsum of dy / (pos+1)).
__global__ __launch_bounds__(NTH) void cumsum_kernel(const bf16_t* __restrict__ X, bf16_t* __restrict__ Y,
                                                     long long outer, int S, long long inner, int reverse, int mean,
                                                     int grad) {
  const long long n = outer * inner;
  for (long long e = (long long)blockIdx.x * NTH + threadIdx.x; e < n; e += (long long)gridDim.x * NTH) {
    const long long o = e / inner, in = e % inner;
    const bf16_t* x = X + o * S * inner + in;
    bf16_t* y = Y + o * S * inner + in;
    float acc = 0.f;
    for (int s = 0; s < S; ++s) {
      const int p = reverse ? S - 1 - s : s;
      float v = bf2f(x[(long long)p * inner]);
      if (mean && grad) v /= (float)(p + 1);
      acc += v;
      float out = acc;
      if (mean && !grad) out /= (float)(p + 1);
      y[(long long)p * inner] = f2bf(out);
    }
  }
}

__global__ __launch_bounds__(NTH) void cast_f32_bf16_kernel(const float* __restrict__ X, bf16_t* __restrict__ Y,
                                                            long long n) {
  for (long long v = (long long)blockIdx.x * NTH + threadIdx.x; v * 4 < n; v += (long long)gridDim.x * NTH) {
    if (v * 4 + 3 < n) {
      float4 f = reinterpret_cast<const float4*>(X)[v];
      reinterpret_cast<uint2*>(Y)[v] = make_uint2(pack_bf16x2(f.x, f.y), pack_bf16x2(f.z, f.w));
    } else {
      for (long long j = v * 4; j < n; ++j) Y[j] = f2bf(X[j]);
    }
  }
}

// y(fp32) = x(bf16): the reversible body's fp32 streams out of its bf16 input
__global__ __launch_bounds__(NTH) void cast_bf16_f32_kernel(const bf16_t* __restrict__ X, float* __restrict__ Y,
                                                            long long nvec) {
  for (long long v = (long long)blockIdx.x * NTH + threadIdx.x; v < nvec; v += (long long)gridDim.x * NTH) {
    float r[8];
    unpack8(reinterpret_cast<const uint4*>(X)[v], r);
    reinterpret_cast<float4*>(Y)[2 * v] = make_float4(r[0], r[1], r[2], r[3]);
    reinterpret_cast<float4*>(Y)[2 * v + 1] = make_float4(r[4], r[5], r[6], r[7]);
  }
}

// y(bf16) = x1(fp32) + x2(fp32) in one pass: the reversible body's output (y1 + y2) and the embedding's gradient out of
// it (g1 + g2), instead of an fp32 add plus a cast (18 -> 10 bytes per element)
__global__ __launch_bounds__(NTH) void add2_f32_bf16_kernel(const float* __restrict__ X1, const float* __restrict__ X2,
                                                            bf16_t* __restrict__ Y, long long n) {
  for (long long v = (long long)blockIdx.x * NTH + threadIdx.x; v * 4 < n; v += (long long)gridDim.x * NTH) {
    if (v * 4 + 3 < n) {
      const float4 a = reinterpret_cast<const float4*>(X1)[v], b = reinterpret_cast<const float4*>(X2)[v];
      reinterpret_cast<uint2*>(Y)[v] = make_uint2(pack_bf16x2(a.x + b.x, a.y + b.y), pack_bf16x2(a.z + b.z, a.w + b.w));
    } else {
      for (long long j = v * 4; j < n; ++j) Y[j] = f2bf(X1[j] + X2[j]);
    }
  }
}

// y(fp32) = alpha * x(fp32) + beta * z(bf16); optional bf16 copy of y (the reversible bodies' residual streams)
__global__ __launch_bounds__(NTH) void mix_f32_kernel(const float* __restrict__ X, const bf16_t* __restrict__ Z,
                                                      float* __restrict__ Y, bf16_t* __restrict__ Yb, long long nvec,
                                                      float alpha, float beta) {
  for (long long v = (long long)blockIdx.x * NTH + threadIdx.x; v < nvec; v += (long long)gridDim.x * NTH) {
    float z[8];
    unpack8(reinterpret_cast<const uint4*>(Z)[v], z);
    const float4 a = reinterpret_cast<const float4*>(X)[2 * v], b = reinterpret_cast<const float4*>(X)[2 * v + 1];
    float r[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = alpha * r[j] + beta * z[j];
    reinterpret_cast<float4*>(Y)[2 * v] = make_float4(r[0], r[1], r[2], r[3]);
    reinterpret_cast<float4*>(Y)[2 * v + 1] = make_float4(r[4], r[5], r[6], r[7]);
    if (Yb) reinterpret_cast<uint4*>(Yb)[v] = pack8(r);
  }
}

}  // namespace

OBST_API int obst_mix_f32(const float* X, const void* Z, float* Y, void* Yb, long long n, float alpha, float beta,
                          hipStream_t st) {
  if (n % 8) return -1;
  if ((((uintptr_t)X) | ((uintptr_t)Y) | ((uintptr_t)Z) | ((uintptr_t)Yb)) & 15) return -2;
  hipLaunchKernelGGL(mix_f32_kernel, dim3(grid_ew(n / 8)), dim3(NTH), 0, st, X, (const bf16_t*)Z, Y, (bf16_t*)Yb,
                     n / 8, alpha, beta);
  return (int)hipGetLastError();
}

struct ObstEwDesc {
  const void* X; const void* Z; void* Y; const float* sptr;
  long long n; int op; int act; float alpha; float beta; unsigned long long seed; float keep;
};

OBST_API int obst_elementwise(const ObstEwDesc* d, hipStream_t st) {
  if (d->n % 8) return -1;
  if ((((uintptr_t)d->X) | ((uintptr_t)d->Y) | ((uintptr_t)d->Z)) & 15) return -2;
  const long long nvec = d->n / 8;
  auto k = ew_kernel<-1, -1>;
  if (d->act == ACT_GELU && d->op == 0) k = ew_kernel<0, ACT_GELU>;
  else if (d->act == ACT_GELU && d->op == 1) k = ew_kernel<1, ACT_GELU>;
  else if (d->act == ACT_RELU && d->op == 0) k = ew_kernel<0, ACT_RELU>;   // bottleneck linears (ctx32_mixer)
  else if (d->act == ACT_RELU && d->op == 1) k = ew_kernel<1, ACT_RELU>;
  else if (d->op == 2) k = ew_kernel<2, 0>;
  else if (d->op == 5) k = ew_kernel<5, 0>;                                  // axpby (MomentumNet / RevNet)
  hipLaunchKernelGGL(k, dim3(grid_ew(nvec)), dim3(NTH), 0, st, d->op, d->act, (const bf16_t*)d->X,
                     (const bf16_t*)d->Z, (bf16_t*)d->Y, nvec, d->sptr, d->alpha, d->beta, d->seed, d->keep);
  return (int)hipGetLastError();
}

// part: obst_dot_parts(n) floats of workspace
OBST_API int obst_dot_parts(long long n) { return grid_for(n / 8); }

OBST_API int obst_dot(const void* X, const void* DY, float* out, float* part, long long n, hipStream_t st) {
  if (n % 8) return -1;
  const int g = grid_for(n / 8);
  hipLaunchKernelGGL(dot_kernel, dim3(g), dim3(NTH), 0, st, (const bf16_t*)X, (const bf16_t*)DY, part, n / 8);
  hipLaunchKernelGGL(dot_fold_kernel, dim3(1), dim3(NTH), 0, st, part, g, out);
  return (int)hipGetLastError();
}

OBST_API int obst_gather(const int* idx, const void* E, void* out, long long T, int F, int V, hipStream_t st) {
  if (F % 8) return -1;
  hipLaunchKernelGGL(gather_kernel, dim3(grid_ew(T * F / 8)), dim3(NTH), 0, st, idx, (const bf16_t*)E, (bf16_t*)out,
                     T, F, V);
  return (int)hipGetLastError();
}

OBST_API int obst_scatter_add(const int* idx, const void* DY, float* dE, long long T, int F, int V, hipStream_t st) {
  hipLaunchKernelGGL(scatter_add_kernel, dim3(grid_for(T * F)), dim3(NTH), 0, st, idx, (const bf16_t*)DY, dE, T, F, V);
  return (int)hipGetLastError();
}

// sidx: token ids sorted ascending (already clamped to [0, V)); perm: their positions (int64, stable order)
OBST_API int obst_scatter_add_sorted(const int* sidx, const long long* perm, const void* DY, float* dE, long long T,
                                     int F, hipStream_t st) {
  if (F % 8 || T <= 0) return -1;
  if ((((uintptr_t)DY) | ((uintptr_t)dE)) & 15) return -2;
  hipLaunchKernelGGL(scatter_sorted_kernel, dim3((unsigned)T), dim3(NTH), 0, st, sidx, perm, (const bf16_t*)DY, dE,
                     T, F);
  return (int)hipGetLastError();
}

// workspace floats of obst_scatter_add_chunked
OBST_API long long obst_scatter_ws(long long T, int F) { return 2 * ((T + SC_CH - 1) / SC_CH) * (long long)F; }

// dE[sidx[i]] += DY[perm[i]] (* scale[perm[i]]) over the stable-sorted ids sidx, deterministic, bounded per block
OBST_API int obst_scatter_add_chunked(const int* sidx, const long long* perm, const void* DY, const float* scale,
                                      float* dE, long long T, int F, float* ws, hipStream_t st) {
  if (F % 8 || T <= 0 || !ws) return -1;
  if ((((uintptr_t)DY) | ((uintptr_t)dE) | ((uintptr_t)ws)) & 15) return -2;
  const unsigned nchunk = (unsigned)((T + SC_CH - 1) / SC_CH);
  hipLaunchKernelGGL(scatter_chunk_kernel, dim3(nchunk), dim3(NTH), 0, st, sidx, perm, (const bf16_t*)DY, scale, dE, ws,
                     T, F);
  hipLaunchKernelGGL(scatter_fold_kernel, dim3(nchunk), dim3(NTH), 0, st, sidx, dE, ws, T, F);
  return (int)hipGetLastError();
}

OBST_API int obst_cumsum(const void* X, void* Y, long long outer, int S, long long inner, int reverse, int mean,
                         int grad, hipStream_t st) {
  hipLaunchKernelGGL(cumsum_kernel, dim3(grid_for(outer * inner)), dim3(NTH), 0, st, (const bf16_t*)X, (bf16_t*)Y,
                     outer, S, inner, reverse, mean, grad);
  return (int)hipGetLastError();
}

OBST_API int obst_add2_f32_bf16(const float* X1, const float* X2, void* Y, long long n, hipStream_t st) {
  hipLaunchKernelGGL(add2_f32_bf16_kernel, dim3(grid_ew((n + 3) / 4)), dim3(NTH), 0, st, X1, X2, (bf16_t*)Y, n);
  return (int)hipGetLastError();
}

OBST_API int obst_cast_f32_bf16(const float* X, void* Y, long long n, hipStream_t st) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_ew((n + 3) / 4)), dim3(NTH), 0, st, X, (bf16_t*)Y, n);
  return (int)hipGetLastError();
}

OBST_API int obst_cast_bf16_f32(const void* X, float* Y, long long n, hipStream_t st) {
  if (n % 8) return -1;
  if ((((uintptr_t)X) | ((uintptr_t)Y)) & 15) return -2;
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_ew(n / 8)), dim3(NTH), 0, st, (const bf16_t*)X, Y, n / 8);
  return (int)hipGetLastError();
}

namespace {
// split-K fold of the weight-gradient GEMM (blaslt.cpp): C[m][n] = beta * C[m][n] + sum_j W[j][m][n], slabs summed in
// index order (deterministic); 4 fp32 per lane, N % 4 == 0
__global__ __launch_bounds__(NTH) void splitk_fold_kernel(const float* __restrict__ W, float* __restrict__ C, int M,
                                                          int N, long long ldc, int s, float beta) {
  const long long n4 = (long long)M * (N / 4), slab = (long long)M * N;
  for (long long v = (long long)blockIdx.x * NTH + threadIdx.x; v < n4; v += (long long)gridDim.x * NTH) {
    const long long e = v * 4, m = e / N, n = e % N;
    float4 acc = reinterpret_cast<const float4*>(W)[v];
    for (int j = 1; j < s; ++j) {
      const float4 w = reinterpret_cast<const float4*>(W + j * slab)[v];
      acc.x += w.x; acc.y += w.y; acc.z += w.z; acc.w += w.w;
    }
    float4* c = reinterpret_cast<float4*>(C + m * ldc + n);
    if (beta != 0.f) {
      const float4 o = *c;
      acc.x += beta * o.x; acc.y += beta * o.y; acc.z += beta * o.z; acc.w += beta * o.w;
    }
    *c = acc;
  }
}
}  // namespace

OBST_API int obst_splitk_fold(const float* W, float* C, int M, int N, long long ldc, int s, float beta, hipStream_t st) {
  if (N % 4 || ldc % 4 || s < 1) return -1;
  if ((((uintptr_t)W) | ((uintptr_t)C)) & 15) return -2;
  hipLaunchKernelGGL(splitk_fold_kernel, dim3(grid_ew((long long)M * N / 4)), dim3(NTH), 0, st, W, C, M, N, ldc, s,
                     beta);
  return (int)hipGetLastError();
}
