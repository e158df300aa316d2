// Kernels for the block-grammar ops off the GPT-Neo hot path, each one pass over HBM:
//  K07 glu gate: y = a * sigmoid(g) and both input gradients in one pass (ref src/model/basic.py:47-57)
//  K14 product-key memory (ref src/model/basic.py:93-115): per sub-key axis top-1 + the softmax probability of the
//      winner (value = product over axes), combined index; value-weighted gather from the [P, heads, f] table and
//      its backward (scatter-add into the fp32 gradient, d value = <dy, row>)
//  K15 dense soft mixture of experts (ref src/model/basic.py:37-44): the expert contraction of the [T, N, E] expert
//      GEMM output with the expert softmax computed in the same kernel (and the softmax Jacobian in the backward)
//  K16 sum over one axis (sum_heads, ref basic.py:77-78)
//  K21 Gumbel-argmax sampling with the token write (ref src/run/inference.py:87-97), counter-hash RNG
//  K24 frame unpack (uint8 or bit-folded ints -> bf16 / 255, ref src/model/__init__.py:37-55) and the masked
//      L1 video loss with its gradient (ref src/model/__init__.py:187-199)
//  serving: single-query attention over a KV cache (incremental decoding; the reference recomputes the context)
#include "common.h"

namespace {

constexpr int NTH = 256;
constexpr int NW = NTH / 64;

inline int grid_for(long long n) {
  long long g = (n + NTH - 1) / NTH;
  return (int)(g < 2048 ? (g < 1 ? 1 : g) : 2048);
}

inline int grid_rows(long long rows, int per_block) {
  long long g = (rows + per_block - 1) / per_block;
  return (int)(g < 4096 ? (g < 1 ? 1 : g) : 4096);
}

__device__ __forceinline__ void unpack8(const uint4& u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) { f[2 * j] = bf2f(w[j] & 0xffff); f[2 * j + 1] = bf2f(w[j] >> 16); }
}

__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7]));
}

// splitmix64 finaliser over a counter (the dropout kernel's generator): 24-bit uniforms strictly inside (0, 1)
__device__ __forceinline__ float hash_uniform(unsigned long long i, unsigned long long seed) {
  unsigned long long h = i * 0x9E3779B97F4A7C15ull ^ seed;
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull; h ^= h >> 33;
  return ((float)(h >> 40) + 0.5f) * (1.f / 16777216.f);
}

// (value, index) arg-max across the wave; ties -> smallest index
__device__ __forceinline__ void wave_argmax(float& m, int& mi) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oi = __shfl_xor(mi, o, 64);
    if (om > m || (om == m && oi < mi)) { m = om; mi = oi; }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// K07: DY == nullptr -> Y = A * s(G); otherwise Y = dA = DY * s, DG = DY * A * s (1 - s)
__global__ __launch_bounds__(NTH) void glu_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ G,
                                                  const bf16_t* __restrict__ DY, bf16_t* __restrict__ Y,
                                                  bf16_t* __restrict__ DG, long long nvec) {
  for (long long v = (long long)blockIdx.x * NTH + threadIdx.x; v < nvec; v += (long long)gridDim.x * NTH) {
    float a[8], g[8];
    unpack8(reinterpret_cast<const uint4*>(A)[v], a);
    unpack8(reinterpret_cast<const uint4*>(G)[v], g);
    if (DY == nullptr) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] *= sigmoidf_(g[j]);
      reinterpret_cast<uint4*>(Y)[v] = pack8(a);
    } else {
      float d[8];
      unpack8(reinterpret_cast<const uint4*>(DY)[v], d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float s = sigmoidf_(g[j]);
        g[j] = d[j] * a[j] * s * (1.f - s);
        a[j] = d[j] * s;
      }
      reinterpret_cast<uint4*>(Y)[v] = pack8(a);
      reinterpret_cast<uint4*>(DG)[v] = pack8(g);
    }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// K14 forward: X [R][A][F] (normalised assignment logits). One wave per row r:
//   per axis a: m_a = max_f x, i_a = first arg-max, s_a = sum_f exp(x - m_a)
//   val[r] = prod_a 1 / s_a (= prod_a softmax_a(i_a), the reference's exp-normalised top-1 product)
//   idx[r] = sum_a i_a * F^a; (m_a, s_a, i_a) are kept for the backward
__global__ __launch_bounds__(NTH) void pkm_top1_kernel(const bf16_t* __restrict__ X, int* __restrict__ idx,
                                                       float* __restrict__ val, float* __restrict__ st,
                                                       int* __restrict__ aidx, long long R, int A, int F) {
  const int lane = threadIdx.x & 63;
  for (long long r = (long long)blockIdx.x * NW + (threadIdx.x >> 6); r < R; r += (long long)gridDim.x * NW) {
    long long comb = 0, mult = 1;
    float v = 1.f;
    for (int a = 0; a < A; ++a) {
      const bf16_t* x = X + (r * A + a) * F;
      float m = -INFINITY;
      int mi = F;
      for (int f = lane; f < F; f += 64) {
        const float t = bf2f(x[f]);
        if (t > m) { m = t; mi = f; }
      }
      wave_argmax(m, mi);
      if (mi >= F) mi = 0;           // all -inf / NaN row: index 0 (the gather clamps anyway)
      float s = 0.f;
      for (int f = lane; f < F; f += 64) s += __expf(bf2f(x[f]) - m);
      s = wave_sum(s);
      v /= s;
      comb += (long long)mi * mult;
      mult *= F;
      if (lane == 0) {
        st[(r * A + a) * 2] = m;
        st[(r * A + a) * 2 + 1] = s;
        aidx[r * A + a] = mi;
      }
    }
    if (lane == 0) { idx[r] = (int)comb; val[r] = v; }
  }
}

// K14 backward of val: dX[r][a][f] = dval[r] * val[r] * (delta(f, i_a) - exp(x - m_a) / s_a)
__global__ __launch_bounds__(NTH) void pkm_top1_bwd_kernel(const bf16_t* __restrict__ X, const float* __restrict__ val,
                                                           const float* __restrict__ dval,
                                                           const float* __restrict__ st, const int* __restrict__ aidx,
                                                           bf16_t* __restrict__ DX, long long R, int A, int F) {
  const int lane = threadIdx.x & 63;
  for (long long r = (long long)blockIdx.x * NW + (threadIdx.x >> 6); r < R; r += (long long)gridDim.x * NW) {
    const float g = dval[r] * val[r];
    for (int a = 0; a < A; ++a) {
      const long long o = (r * A + a) * F;
      const float m = st[(r * A + a) * 2], inv = 1.f / st[(r * A + a) * 2 + 1];
      const int ia = aidx[r * A + a];
      for (int f = lane; f < F; f += 64) {
        const float p = __expf(bf2f(X[o + f]) - m) * inv;
        DX[o + f] = f2bf(g * ((f == ia ? 1.f : 0.f) - p));
      }
    }
  }
}

// K14 value gather: out[r][:] = table[idx[r] * H + r % H][:] * val[r]   (table [P][H][Fk], Fk % 8 == 0)
__global__ __launch_bounds__(NTH) void pkm_gather_kernel(const int* __restrict__ idx, const float* __restrict__ val,
                                                         const bf16_t* __restrict__ table, bf16_t* __restrict__ out,
                                                         long long R, int H, int Fk, int P) {
  const int vpr = Fk / 8;
  const long long n = R * vpr;
  for (long long v = (long long)blockIdx.x * NTH + threadIdx.x; v < n; v += (long long)gridDim.x * NTH) {
    const long long r = v / vpr;
    const int c = (int)(v % vpr);
    int p = idx[r];
    p = p < 0 ? 0 : (p >= P ? P - 1 : p);
    float t[8];
    unpack8(reinterpret_cast<const uint4*>(table + ((long long)p * H + r % H) * Fk)[c], t);
    const float s = val[r];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] *= s;
    reinterpret_cast<uint4*>(out)[v] = pack8(t);
  }
}

// K14 gather backward, one wave per row: dval[r] = <dy[r], table row>; dtable row += dy[r] * val[r] (fp32 atomics)
__global__ __launch_bounds__(NTH) void pkm_gather_bwd_kernel(const int* __restrict__ idx, const float* __restrict__ val,
                                                             const bf16_t* __restrict__ table,
                                                             const bf16_t* __restrict__ DY, float* __restrict__ dtable,
                                                             float* __restrict__ dval, long long R, int H, int Fk, int P) {
  const int lane = threadIdx.x & 63;
  for (long long r = (long long)blockIdx.x * NW + (threadIdx.x >> 6); r < R; r += (long long)gridDim.x * NW) {
    int p = idx[r];
    p = p < 0 ? 0 : (p >= P ? P - 1 : p);
    const long long row = ((long long)p * H + r % H) * Fk;
    const float s = val[r];
    float acc = 0.f;
    for (int f = lane; f < Fk; f += 64) {
      const float d = bf2f(DY[r * Fk + f]);
      acc += d * bf2f(table[row + f]);
      if (dtable) atomicAdd(dtable + row + f, d * s);   // null: dtable by the deterministic sorted scatter
    }
    acc = wave_sum(acc);
    if (lane == 0) dval[r] = acc;
  }
}

// ---------------------------------------------------------------------------------------------------------------
// K15 mixture-of-experts combine. U [T][N][E] = x · W (one plain GEMM over the expert-major weight [K][N][E]),
// Lg [T][E] gate logits. Per token (one block): p = softmax(Lg[t]) (kept in P for the backward),
// Y[t][n] = sum_e U[t][n][e] p[e]. E/8 lanes share one n (E % 8 == 0, E/8 a power of two <= 64).
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = red[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) t = fmaxf(t, red[i]);
  return t;
}

__global__ __launch_bounds__(NTH) void moe_fwd_kernel(const bf16_t* __restrict__ U, const bf16_t* __restrict__ Lg,
                                                      float* __restrict__ P, bf16_t* __restrict__ Y, long long T, int N,
                                                      int E) {
  __shared__ float p_s[512];
  __shared__ float red[NW];
  const int tid = threadIdx.x, lpr = E >> 3, c = tid & (lpr - 1);
  for (long long t = blockIdx.x; t < T; t += gridDim.x) {
    float mx = -INFINITY;
    for (int e = tid; e < E; e += NTH) mx = fmaxf(mx, bf2f(Lg[t * E + e]));
    mx = block_max(mx, red);
    float sum = 0.f;
    for (int e = tid; e < E; e += NTH) {
      const float q = __expf(bf2f(Lg[t * E + e]) - mx);
      p_s[e] = q;
      sum += q;
    }
    const float inv = 1.f / block_sum<NW>(sum, red);   // its barriers publish p_s
    for (int e = tid; e < E; e += NTH) P[t * E + e] = p_s[e] * inv;
    float pc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) pc[j] = p_s[c * 8 + j] * inv;
    for (int n = tid / lpr; n < N; n += NTH / lpr) {
      float u[8];
      unpack8(*reinterpret_cast<const uint4*>(U + (t * N + n) * E + c * 8), u);
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += u[j] * pc[j];
      for (int o = lpr >> 1; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (c == 0) Y[t * N + n] = f2bf(acc);
    }
    __syncthreads();   // p_s is rewritten by the next token
  }
}

// K15 backward: dU[t][n][e] = dy[t][n] p[e]; dp[e] = sum_n dy[t][n] U[t][n][e]; dLg = p (dp - <p, dp>)
__global__ __launch_bounds__(NTH) void moe_bwd_kernel(const bf16_t* __restrict__ DY, const bf16_t* __restrict__ U,
                                                      const float* __restrict__ P, bf16_t* __restrict__ DU,
                                                      bf16_t* __restrict__ DLg, long long T, int N, int E) {
  __shared__ float dp_s[512];
  __shared__ float dpp[NTH * 8];   // [row group][E] partial dp sums, added in row-group order (no LDS atomics)
  __shared__ float red[NW];
  const int tid = threadIdx.x, lpr = E >> 3, c = tid & (lpr - 1), rg = tid / lpr, nrg = NTH / lpr;
  for (long long t = blockIdx.x; t < T; t += gridDim.x) {
    for (int e = tid; e < E; e += NTH) dp_s[e] = 0.f;
    float pc[8], dp[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { pc[j] = P[t * E + c * 8 + j]; dp[j] = 0.f; }
    __syncthreads();
    for (int n = tid / lpr; n < N; n += NTH / lpr) {
      const float d = bf2f(DY[t * N + n]);
      float u[8], g[8];
      const long long o = (t * N + n) * E + c * 8;
      unpack8(*reinterpret_cast<const uint4*>(U + o), u);
#pragma unroll
      for (int j = 0; j < 8; ++j) { dp[j] += d * u[j]; g[j] = d * pc[j]; }
      *reinterpret_cast<uint4*>(DU + o) = pack8(g);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) dpp[rg * E + c * 8 + j] = dp[j];
    __syncthreads();
    for (int e = tid; e < E; e += NTH) {
      float v = 0.f;
      for (int r = 0; r < nrg; ++r) v += dpp[r * E + e];
      dp_s[e] = v;
    }
    __syncthreads();
    float s = 0.f;
    for (int e = tid; e < E; e += NTH) s += P[t * E + e] * dp_s[e];
    s = block_sum<NW>(s, red);
    for (int e = tid; e < E; e += NTH) DLg[t * E + e] = f2bf(P[t * E + e] * (dp_s[e] - s));
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------------------------
// K16: y[o][i] = sum_h x[o][h][i]   (inner % 8 == 0, fp32 accumulation)
// K12 axial positional embedding (reference embedding.py 'axial'): the [n_0 x ... x n_{k-1}, F] table is the
// product of k factor tables [n_m][F] broadcast over the other axes, out[i_0 .. i_{k-1}][f] = prod_m T_m[i_m][f].
struct AxialArgs {
  const bf16_t* t[4];
  float* g[4];   // backward: fp32 factor gradients
  int n[4];
  int k, F;
};

__global__ __launch_bounds__(NTH) void axial_fwd_kernel(AxialArgs a, bf16_t* __restrict__ out, long long total) {
  const long long e = (long long)blockIdx.x * NTH + threadIdx.x;
  if (e >= total) return;
  const int f = (int)(e % a.F);
  long long r = e / a.F;
  float v = 1.f;
  for (int m = a.k - 1; m >= 0; --m) {   // the last factor is the fastest-varying position axis
    const int i = (int)(r % a.n[m]);
    r /= a.n[m];
    v *= bf2f(a.t[m][(long long)i * a.F + f]);
  }
  out[e] = f2bf(v);
}

// dT_m[i][f] = sum over the other axes (row-major order, fp32) of g[..i..][f] * prod_{m' != m} T_m'[i_m'][f]:
// one thread per (i, f) of factor m -- a fixed summation order, no atomics
__global__ __launch_bounds__(NTH) void axial_bwd_kernel(AxialArgs a, const bf16_t* __restrict__ gout, int m) {
  const long long e = (long long)blockIdx.x * NTH + threadIdx.x;
  if (e >= (long long)a.n[m] * a.F) return;
  const int f = (int)(e % a.F), im = (int)(e / a.F);
  long long others = 1;
  for (int j = 0; j < a.k; ++j)
    if (j != m) others *= a.n[j];
  float acc = 0.f;
  for (long long o = 0; o < others; ++o) {
    long long r = o, pos = 0, stride = 1;
    float prod = 1.f;
    for (int j = a.k - 1; j >= 0; --j) {   // compose the flat position with index im on axis m
      int i;
      if (j == m) {
        i = im;
      } else {
        i = (int)(r % a.n[j]);
        r /= a.n[j];
        prod *= bf2f(a.t[j][(long long)i * a.F + f]);
      }
      pos += (long long)i * stride;
      stride *= a.n[j];
    }
    acc += bf2f(gout[pos * a.F + f]) * prod;
  }
  a.g[m][e] = acc;
}

__global__ __launch_bounds__(NTH) void sum_axis_kernel(const bf16_t* __restrict__ X, bf16_t* __restrict__ Y,
                                                       long long outer, int H, long long inner) {
  const long long iv = inner / 8, n = outer * iv;
  for (long long v = (long long)blockIdx.x * NTH + threadIdx.x; v < n; v += (long long)gridDim.x * NTH) {
    const long long o = v / iv, i = v % iv;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int h = 0; h < H; ++h) {
      float x[8];
      unpack8(reinterpret_cast<const uint4*>(X + (o * H + h) * inner)[i], x);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += x[j];
    }
    reinterpret_cast<uint4*>(Y + o * inner)[i] = pack8(acc);
  }
}

// ---------------------------------------------------------------------------------------------------------------
// K21: one block per logits row r = b * Pt + j (Pt = token patch): arg-max of logit - T_b log(-log u) with
// u = hash(seed, r * V + v); the winner goes to X[b][min(pos_b, S-1)][j] when pos_b < end_b and to pred[r].
__global__ __launch_bounds__(NTH) void sample_kernel(const float* __restrict__ L, long long rows, int V, int Pt,
                                                     const float* __restrict__ temp, const long long* __restrict__ pos,
                                                     const long long* __restrict__ end, int* __restrict__ X, int S,
                                                     int* __restrict__ pred, unsigned long long seed) {
  __shared__ float rm[NW];
  __shared__ int ri[NW];
  for (long long r = blockIdx.x; r < rows; r += gridDim.x) {
    const long long b = r / Pt;
    const float T = temp[b];
    float m = -INFINITY;
    int mi = V;
    for (int v = threadIdx.x; v < V; v += NTH) {
      float l = L[r * V + v];
      if (T != 0.f) l -= T * logf(-logf(hash_uniform((unsigned long long)(r * V + v), seed)));
      if (l > m) { m = l; mi = v; }
    }
    wave_argmax(m, mi);
    if ((threadIdx.x & 63) == 0) { rm[threadIdx.x >> 6] = m; ri[threadIdx.x >> 6] = mi; }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < NW; ++w)
        if (rm[w] > m || (rm[w] == m && ri[w] < mi)) { m = rm[w]; mi = ri[w]; }
      if (mi >= V) mi = 0;
      if (pred) pred[r] = mi;
      if (X && pos[b] < end[b]) {
        const long long w = pos[b] < S - 1 ? pos[b] : S - 1;
        X[(b * S + w) * Pt + r % Pt] = mi;
      }
    }
    __syncthreads();
  }
}

// Split variant for decode-sized batches (rows << CUs): NB blocks per row each reduce a contiguous slice of the
// vocabulary to one (value, index) pair in `ws`; sample_final_kernel picks each row's winner (ties -> smallest
// index, so the split changes nothing but the parallelism: 32 rows x 50304 logits took 55 us on 32 blocks).
__global__ __launch_bounds__(NTH) void sample_part_kernel(const float* __restrict__ L, long long rows, int V, int Pt,
                                                          int NB, const float* __restrict__ temp,
                                                          unsigned long long seed, float2* __restrict__ ws) {
  __shared__ float rm[NW];
  __shared__ int ri[NW];
  const long long r = blockIdx.x / NB;
  const int part = blockIdx.x % NB;
  if (r >= rows) return;
  const int chunk = (V + NB - 1) / NB;
  const int v0 = part * chunk, v1 = min(V, v0 + chunk);
  const float T = temp[r / Pt];
  float m = -INFINITY;
  int mi = V;
  for (int v = v0 + threadIdx.x; v < v1; v += NTH) {
    float l = L[r * V + v];
    if (T != 0.f) l -= T * logf(-logf(hash_uniform((unsigned long long)(r * V + v), seed)));
    if (l > m) { m = l; mi = v; }
  }
  wave_argmax(m, mi);
  if ((threadIdx.x & 63) == 0) { rm[threadIdx.x >> 6] = m; ri[threadIdx.x >> 6] = mi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < NW; ++w)
      if (rm[w] > m || (rm[w] == m && ri[w] < mi)) { m = rm[w]; mi = ri[w]; }
    ws[r * NB + part] = make_float2(m, __int_as_float(mi));
  }
}

__global__ __launch_bounds__(NTH) void sample_final_kernel(long long rows, int V, int Pt, int NB,
                                                           const float2* __restrict__ ws,
                                                           const long long* __restrict__ pos,
                                                           const long long* __restrict__ end, int* __restrict__ X,
                                                           int S, int* __restrict__ pred) {
  const long long r = (long long)blockIdx.x * NTH + threadIdx.x;
  if (r >= rows) return;
  float m = -INFINITY;
  int mi = V;
  for (int k = 0; k < NB; ++k) {   // parts in vocabulary order: a tie keeps the earlier (smaller) index
    const float2 e = ws[r * NB + k];
    const int ei = __float_as_int(e.y);
    if (e.x > m || (e.x == m && ei < mi)) { m = e.x; mi = ei; }
  }
  if (mi >= V) mi = 0;
  if (pred) pred[r] = mi;
  const long long b = r / Pt;
  if (X && pos[b] < end[b]) {
    const long long w = pos[b] < S - 1 ? pos[b] : S - 1;
    X[(b * S + w) * Pt + r % Pt] = mi;
  }
}

// ---------------------------------------------------------------------------------------------------------------
// K24 frame unpack: V [rows][C] (uint8 or int32) -> Y [rows][C * folds] bf16,
// Y[r][i * C + c] = ((V[r][c] / base^i) % base) / 255   (folds == 1: V / 255)
template <typename TIn>
__global__ __launch_bounds__(NTH) void frames_kernel(const TIn* __restrict__ V, bf16_t* __restrict__ Y, long long rows,
                                                     int C, int folds, int base) {
  const long long n = rows * C * folds;
  for (long long e = (long long)blockIdx.x * NTH + threadIdx.x; e < n; e += (long long)gridDim.x * NTH) {
    const long long r = e / ((long long)C * folds);
    const int k = (int)(e % ((long long)C * folds)), i = k / C, c = k % C;
    long long v = (long long)V[r * C + c];
    for (int f = 0; f < i; ++f) v /= base;
    if (folds > 1) v %= base;
    Y[e] = f2bf((float)v / 255.f);
  }
}

// K24 masked L1: d = (F - G) * m[e / inner]; loss += |d| (one atomic per block); with DF: DF = sign(d) m * g
// where g = gscale (* gptr[0])
__global__ __launch_bounds__(NTH) void l1_kernel(const bf16_t* __restrict__ Fo, const bf16_t* __restrict__ G,
                                                 const float* __restrict__ M, long long inner, long long n,
                                                 float* __restrict__ loss, bf16_t* __restrict__ DF,
                                                 const float* __restrict__ gptr, float gscale) {
  __shared__ float red[NW];
  const float g = gscale * (gptr ? gptr[0] : 1.f);
  float acc = 0.f;
  for (long long e = (long long)blockIdx.x * NTH + threadIdx.x; e < n; e += (long long)gridDim.x * NTH) {
    const float m = M ? M[e / inner] : 1.f;
    const float d = (bf2f(Fo[e]) - bf2f(G[e])) * m;
    if (DF) DF[e] = f2bf(d > 0.f ? m * g : (d < 0.f ? -m * g : 0.f));
    else acc += fabsf(d);
  }
  if (!DF) {
    acc = block_sum<NW>(acc, red);
    if (threadIdx.x == 0) atomicAdd(loss, acc);
  }
}

// ---------------------------------------------------------------------------------------------------------------
// KV-cache decode attention (serving): one new query per (b, h) against the cached keys / values of that row,
// o[b][h] = softmax_j(scale q.K[b][j][h], j < len[b]) . V[b][j][h]. Q/O are [B][H][D], the caches [B][S][H][D]
// (token-major, the layout the k/v linears write). Block = (b, h), 4 waves stride over the keys 4 at a time (4
// independent dot-product reductions in flight per wave), lanes over the head dim (2 elements per lane, D <= 128,
// 256-byte coalesced rows), online softmax per wave, the 4 partial states merged through LDS.
__global__ __launch_bounds__(NTH) void decode_attn_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ Kn,
                                                          const bf16_t* __restrict__ Vn, bf16_t* __restrict__ K,
                                                          bf16_t* __restrict__ V, bf16_t* __restrict__ O,
                                                          const long long* __restrict__ pos, int S, int H, int D,
                                                          float scale) {
  __shared__ float sm[NW], sl[NW];
  __shared__ float sacc[NW][128];
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e0 = 2 * lane;
  const bool act = e0 < D;
  const long long P = pos[b];                            // the new token's position: keys [0, P]
  long long L = P + 1;
  L = L < 0 ? 0 : (L > S ? S : L);
  float q0 = 0.f, q1 = 0.f;
  uint32_t kn = 0, vn = 0;
  if (act) {
    const uint32_t u = *reinterpret_cast<const uint32_t*>(Q + (long long)bh * D + e0);
    q0 = bf2f(u & 0xffff) * scale;
    q1 = bf2f(u >> 16) * scale;
    kn = *reinterpret_cast<const uint32_t*>(Kn + (long long)bh * D + e0);
    vn = *reinterpret_cast<const uint32_t*>(Vn + (long long)bh * D + e0);
  }
  const long long rs = (long long)H * D;                 // cache row stride
  bf16_t* Kb = K + (long long)b * S * rs + (long long)h * D + e0;
  bf16_t* Vb = V + (long long)b * S * rs + (long long)h * D + e0;
  if (w == 0 && act && P >= 0 && P < S) {                // append the new key / value (read below from registers)
    *reinterpret_cast<uint32_t*>(Kb + P * rs) = kn;
    *reinterpret_cast<uint32_t*>(Vb + P * rs) = vn;
  }
  float m = -INFINITY, l = 0.f, a0 = 0.f, a1 = 0.f;
  for (long long j0 = 4 * w; j0 < L; j0 += 4 * NW) {
    float s[4];
    uint32_t vv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long j = j0 + u;
      uint32_t kk = 0;
      vv[u] = 0;
      if (act && j < L) {
        const bool cur = j == P;
        kk = cur ? kn : *reinterpret_cast<const uint32_t*>(Kb + j * rs);
        vv[u] = cur ? vn : *reinterpret_cast<const uint32_t*>(Vb + j * rs);
      }
      s[u] = q0 * bf2f(kk & 0xffff) + q1 * bf2f(kk >> 16);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) s[u] = wave_sum(s[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (j0 + u >= L) continue;                           // wave-uniform
      const float mn = fmaxf(m, s[u]);
      const float c = __expf(m - mn), p = __expf(s[u] - mn);
      l = l * c + p;
      a0 = a0 * c + p * bf2f(vv[u] & 0xffff);
      a1 = a1 * c + p * bf2f(vv[u] >> 16);
      m = mn;
    }
  }
  if (lane == 0) { sm[w] = m; sl[w] = l; }
  if (act) { sacc[w][e0] = a0; sacc[w][e0 + 1] = a1; }
  __syncthreads();
  if (w == 0 && act) {
    float M = sm[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) M = fmaxf(M, sm[i]);
    float Lt = 0.f, o0 = 0.f, o1 = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const float c = sm[i] == -INFINITY ? 0.f : __expf(sm[i] - M);
      Lt += sl[i] * c;
      o0 += sacc[i][e0] * c;
      o1 += sacc[i][e0 + 1] * c;
    }
    const float inv = Lt > 0.f ? 1.f / Lt : 0.f;
    *reinterpret_cast<uint32_t*>(O + (long long)bh * D + e0) = pack_bf16x2(o0 * inv, o1 * inv);
  }
}

// Split-K ("flash-decoding") variant for D % 8 == 0: grid (nsplit, B * H), block = 4 waves. A wave holds 4 keys at
// a time, 16 lanes per key row with one 16-byte load each (8 dims per lane, D <= 128), so a score needs a 4-step
// xor reduction inside the 16-lane group instead of 6 steps over the wave; 4 such groups are unrolled, i.e. 8
// 16-byte K/V loads per lane are in flight. Each of the 16 (wave, group) states runs its own online softmax; the
// block merges them through LDS and either writes the output (one split) or its unnormalised partial
// (m, l, acc[D]) for decode_combine_kernel.
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(NTH) void decode_attn_split_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ Kn, const bf16_t* __restrict__ Vn,
    bf16_t* __restrict__ K, bf16_t* __restrict__ V, bf16_t* __restrict__ O, float* __restrict__ part,
    const long long* __restrict__ pos, int S, int H, int D, float scale, int chunk) {
  __shared__ float sm[16], sl[16];
  __shared__ float sacc[16][128];
  const int sp = blockIdx.x, nsplit = gridDim.x, bh = blockIdx.y, b = bh / H, h = bh % H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, e0 = 8 * (lane & 15);
  const bool act = e0 < D;
  const long long P = pos[b];
  long long L = P + 1;
  L = L < 0 ? 0 : (L > S ? S : L);
  const long long jb = (long long)sp * chunk, je = jb + chunk < L ? jb + chunk : L;
  float q[8];
  uint4 kn = make_uint4(0, 0, 0, 0), vn = make_uint4(0, 0, 0, 0);
  if (act) {
    unpack8(*reinterpret_cast<const uint4*>(Q + (long long)bh * D + e0), q);
    kn = *reinterpret_cast<const uint4*>(Kn + (long long)bh * D + e0);
    vn = *reinterpret_cast<const uint4*>(Vn + (long long)bh * D + e0);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] *= scale;
  const long long rs = (long long)H * D;
  bf16_t* Kb = K + (long long)b * S * rs + (long long)h * D + e0;
  bf16_t* Vb = V + (long long)b * S * rs + (long long)h * D + e0;
  if (sp == 0 && w == 0 && g == 0 && act && P >= 0 && P < S) {   // append; read back below from registers
    *reinterpret_cast<uint4*>(Kb + P * rs) = kn;
    *reinterpret_cast<uint4*>(Vb + P * rs) = vn;
  }
  float m = -INFINITY, l = 0.f, acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  // lanes past D read column 0 of their row (values unused); rows past the split's end re-read its last row
  const bf16_t* Kr = act ? Kb : Kb - e0;
  const bf16_t* Vr = act ? Vb : Vb - e0;
  for (long long j0 = jb; j0 < je; j0 += 64) {
    float s[4];
    uint4 kk[4], vv[4];
    // all 8 K / V row loads of the step issued before any is used: unconditional loads on clamped rows (a load
    // under `if (j < je)` compiled to load + vmcnt(0), one row in flight per lane at a time)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long j = j0 + w * 16 + u * 4 + g, jc = j < je ? j : je - 1;
      kk[u] = *reinterpret_cast<const uint4*>(Kr + jc * rs);
      vv[u] = *reinterpret_cast<const uint4*>(Vr + jc * rs);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long j = j0 + w * 16 + u * 4 + g;
      const bool ok = act && j < je, cur = j == P;   // the new token's row: from registers (appended above)
      kk[u] = !ok ? make_uint4(0, 0, 0, 0) : (cur ? kn : kk[u]);
      vv[u] = !ok ? make_uint4(0, 0, 0, 0) : (cur ? vn : vv[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float kf[8];
      unpack8(kk[u], kf);
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) d += q[i] * kf[i];
      s[u] = d;
    }
    float mx = m;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s[u] = group16_sum(s[u]);
      if (j0 + w * 16 + u * 4 + g >= je) s[u] = -INFINITY;
      mx = fmaxf(mx, s[u]);
    }
    if (mx == -INFINITY) continue;
    const float c = __expf(m - mx);
    l *= c;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] *= c;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float p = __expf(s[u] - mx);
      float vf[8];
      unpack8(vv[u], vf);
      l += p;
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += p * vf[i];
    }
    m = mx;
  }
  const int st = w * 4 + g;
  if ((lane & 15) == 0) { sm[st] = m; sl[st] = l; }
  if (act) {
#pragma unroll
    for (int i = 0; i < 8; ++i) sacc[st][e0 + i] = acc[i];
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < D) {
    float M = sm[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) M = fmaxf(M, sm[i]);
    float Lt = 0.f, o = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float c = sm[i] == -INFINITY ? 0.f : __expf(sm[i] - M);
      Lt += sl[i] * c;
      o += sacc[i][t] * c;
    }
    if (nsplit == 1) {
      O[(long long)bh * D + t] = f2bf(Lt > 0.f ? o / Lt : 0.f);
    } else {
      float* pp = part + ((long long)bh * nsplit + sp) * (D + 2);
      pp[2 + t] = o;
      if (t == 0) { pp[0] = M; pp[1] = Lt; }
    }
  }
}

// merges the nsplit partials of one (b, h): grid B * H, one thread per head dim
__global__ __launch_bounds__(128) void decode_combine_kernel(const float* __restrict__ part, bf16_t* __restrict__ O,
                                                            int D, int nsplit) {
  const int bh = blockIdx.x, t = threadIdx.x;
  if (t >= D) return;
  const float* pp = part + (long long)bh * nsplit * (D + 2);
  float M = -INFINITY;
  for (int i = 0; i < nsplit; ++i) M = fmaxf(M, pp[i * (D + 2)]);
  float Lt = 0.f, o = 0.f;
  for (int i = 0; i < nsplit; ++i) {
    const float mi = pp[i * (D + 2)];
    const float c = mi == -INFINITY ? 0.f : __expf(mi - M);
    Lt += pp[i * (D + 2) + 1] * c;
    o += pp[i * (D + 2) + 2 + t] * c;
  }
  O[(long long)bh * D + t] = f2bf(Lt > 0.f ? o / Lt : 0.f);
}

inline bool aligned16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

}  // namespace

OBST_API int obst_glu(const void* A, const void* G, const void* DY, void* Y, void* DG, long long n, hipStream_t st) {
  if (n % 8) return -1;
  if (!aligned16(A) || !aligned16(G) || !aligned16(DY) || !aligned16(Y) || !aligned16(DG)) return -2;
  if (DY && !DG) return -3;
  hipLaunchKernelGGL(glu_kernel, dim3(grid_for(n / 8)), dim3(NTH), 0, st, (const bf16_t*)A, (const bf16_t*)G,
                     (const bf16_t*)DY, (bf16_t*)Y, (bf16_t*)DG, n / 8);
  return (int)hipGetLastError();
}

OBST_API int obst_pkm_top1(const void* X, int* idx, float* val, float* stats, int* aidx, long long R, int A, int F,
                           hipStream_t st) {
  if (R <= 0 || A <= 0 || F <= 0) return -1;
  double p = 1.0;
  for (int a = 0; a < A; ++a) p *= F;
  if (p >= 2147483647.0) return -2;   // combined index is int32
  hipLaunchKernelGGL(pkm_top1_kernel, dim3(grid_rows(R, NW)), dim3(NTH), 0, st, (const bf16_t*)X, idx, val, stats,
                     aidx, R, A, F);
  return (int)hipGetLastError();
}

OBST_API int obst_pkm_top1_bwd(const void* X, const float* val, const float* dval, const float* stats,
                               const int* aidx, void* DX, long long R, int A, int F, hipStream_t st) {
  if (R <= 0 || A <= 0 || F <= 0) return -1;
  hipLaunchKernelGGL(pkm_top1_bwd_kernel, dim3(grid_rows(R, NW)), dim3(NTH), 0, st, (const bf16_t*)X, val, dval,
                     stats, aidx, (bf16_t*)DX, R, A, F);
  return (int)hipGetLastError();
}

OBST_API int obst_pkm_gather(const int* idx, const float* val, const void* table, void* out, long long R, int H,
                             int Fk, int P, hipStream_t st) {
  if (Fk % 8 || H <= 0 || P <= 0) return -1;
  if (!aligned16(table) || !aligned16(out)) return -2;
  hipLaunchKernelGGL(pkm_gather_kernel, dim3(grid_for(R * Fk / 8)), dim3(NTH), 0, st, idx, val,
                     (const bf16_t*)table, (bf16_t*)out, R, H, Fk, P);
  return (int)hipGetLastError();
}

OBST_API int obst_pkm_gather_bwd(const int* idx, const float* val, const void* table, const void* DY, float* dtable,
                                 float* dval, long long R, int H, int Fk, int P, hipStream_t st) {
  if (H <= 0 || P <= 0 || Fk <= 0) return -1;
  hipLaunchKernelGGL(pkm_gather_bwd_kernel, dim3(grid_rows(R, NW)), dim3(NTH), 0, st, idx, val, (const bf16_t*)table,
                     (const bf16_t*)DY, dtable, dval, R, H, Fk, P);
  return (int)hipGetLastError();
}

// E: multiple of 8 with E/8 a power of two <= 64 (8 <= E <= 512)
static bool moe_ok(int E) { const int l = E >> 3; return E % 8 == 0 && l >= 1 && l <= 64 && (l & (l - 1)) == 0; }

OBST_API int obst_moe_fwd(const void* U, const void* Lg, float* P, void* Y, long long T, int N, int E,
                          hipStream_t st) {
  if (!moe_ok(E) || N <= 0 || T <= 0) return -1;
  if (!aligned16(U)) return -2;
  const int g = (int)(T < 8192 ? T : 8192);
  hipLaunchKernelGGL(moe_fwd_kernel, dim3(g), dim3(NTH), 0, st, (const bf16_t*)U, (const bf16_t*)Lg, P, (bf16_t*)Y,
                     T, N, E);
  return (int)hipGetLastError();
}

OBST_API int obst_moe_bwd(const void* DY, const void* U, const float* P, void* DU, void* DLg, long long T, int N,
                          int E, hipStream_t st) {
  if (!moe_ok(E) || N <= 0 || T <= 0) return -1;
  if (!aligned16(U) || !aligned16(DU)) return -2;
  const int g = (int)(T < 8192 ? T : 8192);
  hipLaunchKernelGGL(moe_bwd_kernel, dim3(g), dim3(NTH), 0, st, (const bf16_t*)DY, (const bf16_t*)U, P, (bf16_t*)DU,
                     (bf16_t*)DLg, T, N, E);
  return (int)hipGetLastError();
}

OBST_API int obst_sum_axis(const void* X, void* Y, long long outer, int H, long long inner, hipStream_t st) {
  if (inner % 8 || H <= 0) return -1;
  if (!aligned16(X) || !aligned16(Y)) return -2;
  hipLaunchKernelGGL(sum_axis_kernel, dim3(grid_for(outer * inner / 8)), dim3(NTH), 0, st, (const bf16_t*)X,
                     (bf16_t*)Y, outer, H, inner);
  return (int)hipGetLastError();
}

// blocks per row of the split sampler (1: the single-kernel path): enough blocks to cover the CUs when rows are few
OBST_API int obst_sample_parts(long long rows, int V) {
  if (rows <= 0 || rows >= 256 || V < 4 * 1024) return 1;
  const long long want = (512 + rows - 1) / rows;
  const long long cap = V / 2048;
  return (int)(want < cap ? (want < 16 ? want : 16) : (cap < 16 ? cap : 16));
}

// ws: obst_sample_parts(rows, V) * rows float2 pairs when that is > 1 (else unused)
OBST_API int obst_sample(const float* L, long long rows, int V, int Pt, const float* temp, const long long* pos,
                         const long long* end, int* X, int S, int* pred, unsigned long long seed, void* ws,
                         hipStream_t st) {
  if (rows <= 0 || V <= 0 || Pt <= 0 || (X && (!pos || !end || S <= 0))) return -1;
  const int nb = obst_sample_parts(rows, V);
  if (nb > 1 && ws) {
    hipLaunchKernelGGL(sample_part_kernel, dim3((unsigned)(rows * nb)), dim3(NTH), 0, st, L, rows, V, Pt, nb, temp,
                       seed, (float2*)ws);
    hipLaunchKernelGGL(sample_final_kernel, dim3((unsigned)((rows + NTH - 1) / NTH)), dim3(NTH), 0, st, rows, V, Pt,
                       nb, (const float2*)ws, pos, end, X, S, pred);
    return (int)hipGetLastError();
  }
  const int g = (int)(rows < 16384 ? rows : 16384);
  hipLaunchKernelGGL(sample_kernel, dim3(g), dim3(NTH), 0, st, L, rows, V, Pt, temp, pos, end, X, S, pred, seed);
  return (int)hipGetLastError();
}

// in_bytes: 1 (uint8) or 4 (int32)
OBST_API int obst_frames(const void* V, int in_bytes, void* Y, long long rows, int C, int folds, int base,
                         hipStream_t st) {
  if (rows <= 0 || C <= 0 || folds <= 0 || base <= 1) return -1;
  const dim3 grid(grid_for(rows * C * folds));
  if (in_bytes == 1)
    hipLaunchKernelGGL(frames_kernel<uint8_t>, grid, dim3(NTH), 0, st, (const uint8_t*)V, (bf16_t*)Y, rows, C, folds,
                       base);
  else if (in_bytes == 4)
    hipLaunchKernelGGL(frames_kernel<int>, grid, dim3(NTH), 0, st, (const int*)V, (bf16_t*)Y, rows, C, folds, base);
  else
    return -2;
  return (int)hipGetLastError();
}

// DF == nullptr: loss[0] += sum |(F - G) m|; otherwise DF = sign((F - G) m) m gscale (* gptr[0])
OBST_API int obst_l1(const void* Fo, const void* G, const float* M, long long inner, long long n, float* loss,
                     void* DF, const float* gptr, float gscale, hipStream_t st) {
  if (n <= 0 || inner <= 0 || (!DF && !loss)) return -1;
  hipLaunchKernelGGL(l1_kernel, dim3(grid_for(n)), dim3(NTH), 0, st, (const bf16_t*)Fo, (const bf16_t*)G, M, inner, n,
                     loss, (bf16_t*)DF, gptr, gscale);
  return (int)hipGetLastError();
}

// Q, Kn, Vn, O [B][H][D] (the new token's q / k / v and the output); K, V caches [B][S][H][D] receive Kn / Vn at
// pos[b]; row b attends over keys [0, pos[b]]. D even, <= 128. With D % 8 == 0, 16-byte aligned operands and a
// workspace of B * H * nsplit * (D + 2) floats the split-K kernel runs (nsplit key chunks per (b, h) + a combine)
OBST_API int obst_decode_attn(const void* Q, const void* Kn, const void* Vn, void* K, void* V, void* O,
                              const long long* pos, int B, int S, int H, int D, float scale, int nsplit, float* ws,
                              hipStream_t st) {
  if (B <= 0 || S <= 0 || H <= 0 || D <= 0 || D > 128 || D % 2) return -1;
  if ((((uintptr_t)Q) | ((uintptr_t)Kn) | ((uintptr_t)Vn) | ((uintptr_t)K) | ((uintptr_t)V) | ((uintptr_t)O)) & 3)
    return -2;
  if (D % 8 == 0 && nsplit >= 1 && aligned16(Q) && aligned16(Kn) && aligned16(Vn) && aligned16(K) &&
      aligned16(V) && (nsplit == 1 || ws != nullptr)) {
    const int chunk = (S + nsplit - 1) / nsplit;
    hipLaunchKernelGGL(decode_attn_split_kernel, dim3(nsplit, B * H), dim3(NTH), 0, st, (const bf16_t*)Q,
                       (const bf16_t*)Kn, (const bf16_t*)Vn, (bf16_t*)K, (bf16_t*)V, (bf16_t*)O, ws, pos, S, H, D,
                       scale, chunk);
    if (nsplit > 1)
      hipLaunchKernelGGL(decode_combine_kernel, dim3(B * H), dim3(128), 0, st, (const float*)ws, (bf16_t*)O, D,
                         nsplit);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(decode_attn_kernel, dim3(B * H), dim3(NTH), 0, st, (const bf16_t*)Q, (const bf16_t*)Kn,
                     (const bf16_t*)Vn, (bf16_t*)K, (bf16_t*)V, (bf16_t*)O, pos, S, H, D, scale);
  return (int)hipGetLastError();
}

// K12: tables t[0..k-1] ([n_m][F] bf16, k <= 4) -> out [prod n_m][F] bf16
OBST_API int obst_axial_fwd(const void* const* t, const int* n, int k, int F, void* out, hipStream_t st) {
  if (k < 1 || k > 4 || F <= 0) return -1;
  AxialArgs a{};
  long long total = F;
  for (int m = 0; m < k; ++m) {
    if (n[m] <= 0) return -1;
    a.t[m] = (const bf16_t*)t[m];
    a.n[m] = n[m];
    total *= n[m];
  }
  a.k = k;
  a.F = F;
  hipLaunchKernelGGL(axial_fwd_kernel, dim3((unsigned)((total + NTH - 1) / NTH)), dim3(NTH), 0, st, a, (bf16_t*)out,
                     total);
  return (int)hipGetLastError();
}

// gout [prod n_m][F] bf16 -> g[m] [n_m][F] fp32 for every factor
OBST_API int obst_axial_bwd(const void* const* t, const int* n, int k, int F, const void* gout, float* const* g,
                            hipStream_t st) {
  if (k < 1 || k > 4 || F <= 0) return -1;
  AxialArgs a{};
  for (int m = 0; m < k; ++m) {
    if (n[m] <= 0) return -1;
    a.t[m] = (const bf16_t*)t[m];
    a.g[m] = g[m];
    a.n[m] = n[m];
  }
  a.k = k;
  a.F = F;
  for (int m = 0; m < k; ++m)
    hipLaunchKernelGGL(axial_bwd_kernel, dim3((unsigned)(((long long)n[m] * F + NTH - 1) / NTH)), dim3(NTH), 0, st, a,
                       (const bf16_t*)gout, m);
  return (int)hipGetLastError();
}
