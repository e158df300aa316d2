// K20: fused multi-tensor optimizer step over the flat parameter / gradient buffers.
//
// The reference builds one update graph per variable from a '-'-separated chain, e.g.
// "adaptive_clip:0.003-sm3-momentum:0.9:1:1-learning_rate" (src/optimizer/__init__.py:31-66,
// src/optimizer/optimizers.py). Here the chain is compiled (python side) into segments of stage opcodes; each
// segment is ONE launch over every tensor at once (a chunk table maps blocks to tensors), with per-tensor
// statistics (sum x^2, sum x, sum w^2, sum w) accumulated by a preceding pass and turned into per-tensor factors by a
// one-thread-per-tensor scalar kernel. Stateful stages (SM3 accumulators, momentum, Adam, NovoGrad, Adafactor
// factors) update their state in the same pass that consumes it. The last segment applies the rezero LR
// multiplier, the "large tensor" weight decay (added after the learning rate, quirk A4), `w -= update`, and writes
// the bf16 compute copy -- no separate cast pass.
#include "common.h"

namespace {
constexpr int NTH = 256;
constexpr int MAXST = 8;

enum Op : int {
  OP_NONE = 0, OP_ADAPTIVE_CLIP, OP_L2_CLIP, OP_GLOBAL_L2_CLIP, OP_VALUE_CLIP, OP_GRAD_CENTRAL, OP_WEIGHT_CENTRAL,
  OP_SM3, OP_MOMENTUM, OP_ADAM, OP_NOVOGRAD, OP_LR, OP_ADAFACTOR, OP_ADAFACTOR_CLIP, OP_SCALE
};

struct Stage { int op; float a, b, c; };

struct OptTensor {
  long long off, n;
  int ndim, flags;            // flags: 1 = weight decay eligible, 2 = rezero, 4 = TP-sharded
  int dims[4];
  long long sm3_off[4];       // per-dim accumulator offsets (into the SM3 buffer)
  long long fac_off;          // adafactor: row accumulators at fac_off, cols at fac_off + rows
  int fac_rows, fac_cols;
};

struct Chunk { int t; int pad; long long start, len; };

struct ApplyArgs {
  const OptTensor* tensors; const Chunk* chunks;
  const float* grad;          // raw gradient (segment 0) ...
  const float* uin;           // ... or the previous segment's output
  float* uout;                // intermediate output (null in the final segment)
  float* master; bf16_t* compute;
  float* stats;               // [T][8]: 0 sum x^2, 1 sum x (this segment's output, if emit_stats), 2 sum w^2, 3 sum w
  const float* fac;           // [T][8] factors for reduction stages
  float* sstate;              // [T][4] scalar state (0-dim tensors' adam m/v, novograd p2)
  float* mom; float* adam_m; float* adam_v;
  const float* sm3_old; float* sm3_new;
  const float* af_old; float* af_rows_sum; float* af_cols_sum;   // adafactor
  Stage st[MAXST]; int nst;
  int final_seg, emit_stats, emit_factored;
  float lr, wd, rezero_mult, grad_scale, beta1, beta2, step_count;
  const float* dyn;           // device [lr, step_count] (graph replay: the host values change every step) or null
  float* part; int part_base; // emit_stats: block b stores (sum x^2, sum x) at part[(part_base + b) * 4 + 0/1]
};

__device__ __forceinline__ float lr_of(const ApplyArgs& a) { return a.dyn ? a.dyn[0] : a.lr; }
__device__ __forceinline__ float step_of(const ApplyArgs& a) { return a.dyn ? a.dyn[1] : a.step_count; }

__device__ __forceinline__ float opt_rsqrt(float x) { return 1.f / fmaxf(sqrtf(x), 1e-5f); }

__device__ __forceinline__ void atomic_max_nonneg(float* addr, float v) {
  atomicMax(reinterpret_cast<int*>(addr), __float_as_int(v));   // valid for v >= 0 (IEEE ordering of non-negatives)
}

// SM3 accumulator max (and Adafactor row/col sums) per chunk: every dim whose index takes few enough values inside
// the chunk is reduced in an LDS window and flushed with one global atomic per slot; leading-dim updates are first
// max-reduced across the wave when all its lanes share the index (the common case: a wave's 256 elements lie in one
// row), so LDS atomics do not serialise on one address.
constexpr int NTA = 512;          // apply threads (16 waves per CU at 2 blocks)
constexpr int WIN_LEAD = 1024;    // LDS slots per leading dim
constexpr int WIN_LAST = 16384;   // LDS slots for the contiguous trailing dim (>= any chunk's distinct indices)

struct Windows {
  int lo[4], cnt[4];              // cnt = 0: window unusable -> global atomics
};

__device__ __forceinline__ float* win_slot(float* lead, float* last, int d, int ndim) {
  return d == ndim - 1 ? last : lead + d * WIN_LEAD;
}

__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// V consecutive elements of one tensor, starting at tensor-relative element e (multi-index idx of e; for V > 1 the
// trailing dim is a multiple of V so all V share the leading indices)
template <int V>
__device__ __forceinline__ void apply_elems(const ApplyArgs& a, const OptTensor& T, const float* F, int tix, int e,
                                            const int (&idx)[4], bool sm3_on, const Windows& W, float* wlead,
                                            float* wlast, bool af, long long af_r0, bool af_rows_win,
                                            bool af_cols_win, float deb1, float deb2, float& s1, float& s2) {
  const long long gi = T.off + e;
  float g[V], w[V];
  if (V == 4) {
    const float4 gv = a.uin ? *reinterpret_cast<const float4*>(a.uin + gi) : *reinterpret_cast<const float4*>(a.grad + gi);
    const float4 wv = *reinterpret_cast<const float4*>(a.master + gi);
    g[0] = gv.x; g[1] = gv.y; g[2] = gv.z; g[3] = gv.w;
    w[0] = wv.x; w[1] = wv.y; w[2] = wv.z; w[3] = wv.w;
    if (!a.uin) {
#pragma unroll
      for (int j = 0; j < V; ++j) g[j] *= a.grad_scale;
    }
  } else {
    g[0] = a.uin ? a.uin[gi] : a.grad[gi] * a.grad_scale;
    w[0] = a.master[gi];
  }
  const int last = T.ndim - 1;
  for (int s = 0; s < a.nst; ++s) {
    const Stage S = a.st[s];
    switch (S.op) {
      case OP_ADAPTIVE_CLIP: case OP_L2_CLIP: case OP_GLOBAL_L2_CLIP: case OP_ADAFACTOR_CLIP: case OP_SCALE:
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] *= F[0];
        break;
      case OP_VALUE_CLIP:
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] = fmaxf(fminf(g[j], S.a), -S.a);
        break;
      case OP_GRAD_CENTRAL:
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] -= F[0];
        break;
      case OP_WEIGHT_CENTRAL:
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] += F[1];
        break;
      case OP_SM3: {
        if (T.ndim == 0) goto scalar_adam;
        float lead = 3.4e38f;
        for (int d = 0; d < last; ++d) lead = fminf(lead, a.sm3_old[T.sm3_off[d] + idx[d]]);
        float nu[V], numax = 0.f;
#pragma unroll
        for (int j = 0; j < V; ++j) {
          nu[j] = fminf(lead, a.sm3_old[T.sm3_off[last] + idx[last] + j]) + g[j] * g[j];
          numax = fmaxf(numax, nu[j]);
        }
        // leading dims: one value per vector
        for (int d = 0; d < last; ++d) {
          const int i0 = __shfl(idx[d], 0, 64);
          const bool uni = __builtin_amdgcn_ballot_w64(idx[d] != i0) == 0 &&
                           __builtin_amdgcn_ballot_w64(1) == ~0ull;
          float v = numax;
          if (uni) v = wave_max_f(v);
          if (!uni || (threadIdx.x & 63) == 0) {
            if (W.cnt[d]) {
              int slot = idx[d] - W.lo[d];
              if (slot < 0) slot += T.dims[d];
              atomicMax(reinterpret_cast<int*>(wlead + d * WIN_LEAD + slot), __float_as_int(v));
            } else {
              atomic_max_nonneg(a.sm3_new + T.sm3_off[d] + idx[d], v);
            }
          }
        }
        // trailing dim: V distinct slots
#pragma unroll
        for (int j = 0; j < V; ++j) {
          if (W.cnt[last]) {
            int slot = idx[last] + j - W.lo[last];
            if (slot < 0) slot += T.dims[last];
            atomicMax(reinterpret_cast<int*>(wlast + slot), __float_as_int(nu[j]));
          } else {
            atomic_max_nonneg(a.sm3_new + T.sm3_off[last] + idx[last] + j, nu[j]);
          }
          g[j] *= opt_rsqrt(nu[j]);
        }
        break;
      }
      case OP_MOMENTUM: {
        float m[V];
        if (V == 4) {
          const float4 mv = *reinterpret_cast<const float4*>(a.mom + gi);
          m[0] = mv.x; m[1] = mv.y; m[2] = mv.z; m[3] = mv.w;
        } else {
          m[0] = a.mom[gi];
        }
#pragma unroll
        for (int j = 0; j < V; ++j) {
          m[j] = S.a * m[j] + g[j] * S.b;
          g[j] = S.c != 0.f ? g[j] + S.a * m[j] : m[j];
        }
        if (V == 4) *reinterpret_cast<float4*>(a.mom + gi) = make_float4(m[0], m[1], m[2], m[3]);
        else a.mom[gi] = m[0];
        break;
      }
      case OP_ADAM: {
        if (T.ndim == 0) goto scalar_adam;
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float v = a.adam_v[gi + j] * a.beta2 + g[j] * g[j] * (1.f - a.beta2);
          const float m = a.adam_m[gi + j] * a.beta1 + g[j] * (1.f - a.beta1);
          a.adam_v[gi + j] = v; a.adam_m[gi + j] = m;
          g[j] = opt_rsqrt(v * deb2) * m * deb1;
        }
        break;
      }
      case OP_NOVOGRAD: {
        if (T.ndim == 0) goto scalar_adam;
        // F[2] = rsqrt-term of the OLD p2, F[3] = rsqrt-term of the debiased NEW p2 (scalar kernel)
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float p1 = a.beta1 * a.mom[gi + j] + g[j] * F[2];
          a.mom[gi + j] = p1;
          g[j] = a.beta1 * p1 + g[j] * F[3];
        }
        break;
      }
      case OP_ADAFACTOR: {
#pragma unroll
        for (int j = 0; j < V; ++j) {
          if (T.fac_rows == 0) {  // unfactored (<= 1-D): per-element second moment in adam_v
            const float v = a.adam_v[gi + j] * F[4] + (g[j] * g[j] + 1e-30f) * (1.f - F[4]);
            a.adam_v[gi + j] = v;
            g[j] = g[j] * rsqrtf(v);
          } else {
            const int rr = (e + j) / T.fac_cols, cc = (e + j) % T.fac_cols;
            const float R = a.af_old[T.fac_off + rr], C = a.af_old[T.fac_off + T.fac_rows + cc];
            const float vhat = R * C * F[5];       // F[5] = 1 / mean(R)
            g[j] = g[j] * rsqrtf(fmaxf(vhat, 1e-30f));
          }
        }
        break;
      }
      case OP_LR:
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] *= lr_of(a);
        break;
      default: break;
    }
    continue;
  scalar_adam: {   // 0-dim tensors (always the scalar path, V == 1)
      float* ss = a.sstate + tix * 4;
      const float v = ss[1] * a.beta2 + g[0] * g[0] * (1.f - a.beta2);
      const float m = ss[0] * a.beta1 + g[0] * (1.f - a.beta1);
      ss[1] = v; ss[0] = m;
      g[0] = opt_rsqrt(v * deb2) * m * deb1;
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) {
    if (a.emit_stats) { s2 += g[j] * g[j]; s1 += g[j]; }
  }
  if (a.final_seg) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      if (T.flags & 2) g[j] *= a.rezero_mult;
      if ((T.flags & 1) && a.wd > 0.f) g[j] += w[j] * lr_of(a) * a.wd;
      w[j] -= g[j];
    }
    if (V == 4) {
      *reinterpret_cast<float4*>(a.master + gi) = make_float4(w[0], w[1], w[2], w[3]);
      if (a.compute)
        *reinterpret_cast<uint2*>(a.compute + gi) = make_uint2(pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3]));
    } else {
      a.master[gi] = w[0];
      if (a.compute) a.compute[gi] = f2bf(w[0]);
    }
  } else if (a.uout) {   // null: a statistics-only segment (graft's probe of its inner stage)
    if (V == 4) *reinterpret_cast<float4*>(a.uout + gi) = make_float4(g[0], g[1], g[2], g[3]);
    else a.uout[gi] = g[0];
  }
}

__global__ __launch_bounds__(NTA) void opt_apply_kernel(ApplyArgs a) {
  const Chunk ck = a.chunks[blockIdx.x];
  const OptTensor T = a.tensors[ck.t];
  const float* F = a.fac + ck.t * 8;
  float s2 = 0.f, s1 = 0.f;
  __shared__ float wlead[3 * WIN_LEAD];
  __shared__ float wlast[WIN_LAST];
  Windows W;
  for (int d = 0; d < 4; ++d) W.lo[d] = W.cnt[d] = 0;
  bool sm3_on = false;
  for (int s = 0; s < a.nst; ++s) sm3_on |= a.st[s].op == OP_SM3;
  sm3_on &= T.ndim > 0;
  const int start = (int)ck.start, len = (int)ck.len;
  if (sm3_on) {
    int stride = 1;
    for (int d = T.ndim - 1; d >= 0; --d) {
      const int span = (len - 1) / stride + 2;
      const int cnt = span < T.dims[d] ? span : T.dims[d];
      W.lo[d] = (start / stride) % T.dims[d];
      W.cnt[d] = cnt <= (d == T.ndim - 1 ? WIN_LAST : WIN_LEAD) ? cnt : 0;
      stride *= T.dims[d];
      float* wb = win_slot(wlead, wlast, d, T.ndim);
      for (int i = threadIdx.x; i < W.cnt[d]; i += NTA) wb[i] = 0.f;
    }
  }
  // Adafactor's factored statistics of this segment's output are NOT accumulated here: opt_factored_kernel reads
  // them back from uout in a fixed order (float atomics made the step nondeterministic)
  const bool af = false;
  const long long af_r0 = 0;
  const bool af_rows_win = false, af_cols_win = false;
  __syncthreads();
  const float deb1 = 1.f / (1.f - powf(a.beta1, step_of(a)));
  const float deb2 = 1.f / (1.f - powf(a.beta2, step_of(a)));
  const bool vec = T.ndim > 0 && (T.off & 3) == 0 && (start & 3) == 0 && (len & 3) == 0 &&
                   (T.dims[T.ndim - 1] & 3) == 0 && (!af || (T.fac_cols & 3) == 0);
  const int V = vec ? 4 : 1;
  for (int e = start + threadIdx.x * V; e < start + len; e += NTA * V) {
    int idx[4] = {0, 0, 0, 0};
    {
      int r = e;
      for (int d = T.ndim - 1; d >= 0; --d) { idx[d] = r % T.dims[d]; r /= T.dims[d]; }
    }
    if (vec) apply_elems<4>(a, T, F, ck.t, e, idx, sm3_on, W, wlead, wlast, af, af_r0, af_rows_win, af_cols_win, deb1,
                            deb2, s1, s2);
    else apply_elems<1>(a, T, F, ck.t, e, idx, sm3_on, W, wlead, wlast, af, af_r0, af_rows_win, af_cols_win, deb1,
                        deb2, s1, s2);
  }
  if (sm3_on) {
    __syncthreads();
    for (int d = 0; d < T.ndim; ++d) {
      const float* wb = win_slot(wlead, wlast, d, T.ndim);
      for (int i = threadIdx.x; i < W.cnt[d]; i += NTA) {
        const float v = wb[i];
        if (v > 0.f) {
          int j = W.lo[d] + i;
          if (j >= T.dims[d]) j -= T.dims[d];
          atomic_max_nonneg(a.sm3_new + T.sm3_off[d] + j, v);
        }
      }
    }
  }
  if (a.emit_stats) {
    __shared__ float red[8];
    s2 = block_sum<8>(s2, red);
    s1 = block_sum<8>(s1, red);
    if (threadIdx.x == 0) {
      a.part[(a.part_base + blockIdx.x) * 4 + 0] = s2;
      a.part[(a.part_base + blockIdx.x) * 4 + 1] = s1;
    }
  }
}


// ---------------------------------------------------------------------------------------------------------------
// Row-tiled apply for every chain without Adafactor (the shipped SM3 chain among them). A tensor is viewed as
// [rows][C] (C = trailing dim); a chunk is a tile of whole rows x a column range (<= RW_COLS). Each thread owns the
// same columns in every row, so:
//   * no per-element multi-index arithmetic: the leading-dim indices are derived once per row;
//   * the SM3 trailing-dim max is a thread-private running max in LDS (no atomics), flushed with one global atomic
//     per column per chunk; the leading-dim max is one wave reduction + one global atomic per wave per row.
// (The generic opt_apply_kernel above derived a 4-D index per element and reduced through LDS atomics: ~620 VALU
// instructions per 4 elements, measured with rocprofv3 --pmc.)
constexpr int RW_NT = 256;
constexpr int RW_COLS = 8192;

struct RChunk { int t, row0, nrows, col0, ncols, vec; };

// the segment's stage program on V consecutive elements of one row (gi: flat index; acc_last: the trailing-dim SM3
// accumulators of those V columns; lead: min over the row's leading-dim accumulators). tm: running trailing-dim max
// of these columns, rmax: running max of this lane's part of the row.
template <int V, int PROG>
__device__ __forceinline__ void row_program(const ApplyArgs& a, const float* F, long long gi, const float* acc_last,
                                            float lead, float (&g)[V], const float (&w)[V], float (&tm)[V],
                                            float& rmax, float deb1, float deb2) {
  if (PROG == 1) {   // the shipped chain, stages fixed at compile time: [norm clip] - sm3 - momentum - learning_rate
    const Stage M = a.st[2];
    const float lr = lr_of(a);
    float al[V], m[V];
    if (V == 4) {
      const float4 v = *reinterpret_cast<const float4*>(acc_last);
      const float4 mv = *reinterpret_cast<const float4*>(a.mom + gi);
      al[0] = v.x; al[1] = v.y; al[2] = v.z; al[3] = v.w;
      m[0] = mv.x; m[1] = mv.y; m[2] = mv.z; m[3] = mv.w;
    } else {
      al[0] = acc_last[0];
      m[0] = a.mom[gi];
    }
#pragma unroll
    for (int j = 0; j < V; ++j) {
      g[j] *= F[0];
      const float nu = fminf(lead, al[j]) + g[j] * g[j];
      tm[j] = fmaxf(tm[j], nu);
      rmax = fmaxf(rmax, nu);
      g[j] *= opt_rsqrt(nu);
      m[j] = M.a * m[j] + g[j] * M.b;
      g[j] = (M.c != 0.f ? g[j] + M.a * m[j] : m[j]) * lr;
    }
    if (V == 4) *reinterpret_cast<float4*>(a.mom + gi) = make_float4(m[0], m[1], m[2], m[3]);
    else a.mom[gi] = m[0];
    return;
  }
      for (int s = 0; s < a.nst; ++s) {
    const Stage S = a.st[s];
    switch (S.op) {
      case OP_ADAPTIVE_CLIP: case OP_L2_CLIP: case OP_GLOBAL_L2_CLIP: case OP_SCALE:
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] *= F[0];
        break;
      case OP_VALUE_CLIP:
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] = fmaxf(fminf(g[j], S.a), -S.a);
        break;
      case OP_GRAD_CENTRAL:
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] -= F[0];
        break;
      case OP_WEIGHT_CENTRAL:
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] += F[1];
        break;
      case OP_SM3: {
        float al[V];
        if (V == 4) {
          const float4 v = *reinterpret_cast<const float4*>(acc_last);
          al[0] = v.x; al[1] = v.y; al[2] = v.z; al[3] = v.w;
        } else {
          al[0] = acc_last[0];
        }
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float nu = fminf(lead, al[j]) + g[j] * g[j];
          tm[j] = fmaxf(tm[j], nu);
          rmax = fmaxf(rmax, nu);
          g[j] *= opt_rsqrt(nu);
        }
        break;
      }
      case OP_MOMENTUM: {
        float m[V];
        if (V == 4) {
          const float4 mv = *reinterpret_cast<const float4*>(a.mom + gi);
          m[0] = mv.x; m[1] = mv.y; m[2] = mv.z; m[3] = mv.w;
        } else {
          m[0] = a.mom[gi];
        }
#pragma unroll
        for (int j = 0; j < V; ++j) {
          m[j] = S.a * m[j] + g[j] * S.b;
          g[j] = S.c != 0.f ? g[j] + S.a * m[j] : m[j];
        }
        if (V == 4) *reinterpret_cast<float4*>(a.mom + gi) = make_float4(m[0], m[1], m[2], m[3]);
        else a.mom[gi] = m[0];
        break;
      }
      case OP_ADAM:
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float v = a.adam_v[gi + j] * a.beta2 + g[j] * g[j] * (1.f - a.beta2);
          const float m = a.adam_m[gi + j] * a.beta1 + g[j] * (1.f - a.beta1);
          a.adam_v[gi + j] = v; a.adam_m[gi + j] = m;
          g[j] = opt_rsqrt(v * deb2) * m * deb1;
        }
        break;
      case OP_NOVOGRAD:
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float p1 = a.beta1 * a.mom[gi + j] + g[j] * F[2];
          a.mom[gi + j] = p1;
          g[j] = a.beta1 * p1 + g[j] * F[3];
        }
        break;
      case OP_LR:
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] *= lr_of(a);
        break;
      default: break;
    }
  }
}

// segment output for V elements: statistics, then either the final weight update (+ bf16 compute copy) or the
// intermediate update buffer
template <int V>
__device__ __forceinline__ void finish_elems(const ApplyArgs& a, const OptTensor& T, long long gi, float (&g)[V],
                                             float (&w)[V], float& s1, float& s2) {
      if (a.emit_stats) {
#pragma unroll
    for (int j = 0; j < V; ++j) { s2 += g[j] * g[j]; s1 += g[j]; }
  }
  if (a.final_seg) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      if (T.flags & 2) g[j] *= a.rezero_mult;
      if ((T.flags & 1) && a.wd > 0.f) g[j] += w[j] * lr_of(a) * a.wd;
      w[j] -= g[j];
    }
    if (V == 4) {
      *reinterpret_cast<float4*>(a.master + gi) = make_float4(w[0], w[1], w[2], w[3]);
      if (a.compute)
        *reinterpret_cast<uint2*>(a.compute + gi) = make_uint2(pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3]));
    } else {
      a.master[gi] = w[0];
      if (a.compute) a.compute[gi] = f2bf(w[0]);
    }
  } else if (a.uout) {   // null: a statistics-only segment (graft's probe of its inner stage)
    if (V == 4) *reinterpret_cast<float4*>(a.uout + gi) = make_float4(g[0], g[1], g[2], g[3]);
    else a.uout[gi] = g[0];
  }
    }

// exact n / d for 0 <= n < 2^31 from a precomputed m = floor((2^32 - 1) / d) + 1 (d >= 2): the estimate is floor(n/d)
// or one more
__device__ __forceinline__ int fast_div(int n, int d, unsigned m) {
  if (d == 1) return n;
  int q = (int)__umulhi((unsigned)n, m);
  if (q * d > n) --q;
  return q;
}

// narrow rows (C / V lanes per row, a power of two <= 64): the block covers RW_NT * V / C whole rows per iteration,
// each lane keeps the same V columns in every iteration (register running max of the trailing-dim accumulator),
// the row max is a shuffle reduction over the row's lanes
template <int V, int PROG>
__device__ __forceinline__ void rows_packed(const ApplyArgs& a, const OptTensor& T, const float* F, const RChunk& ck,
                                            float* tmax, bool sm3_on, float deb1, float deb2, float& s1, float& s2) {
  const int tid = threadIdx.x;
  const int last = T.ndim - 1;
  const int C = T.dims[last];
  const int lpr = C / V;
  const int rpi = RW_NT / lpr;
  const int sub = tid / lpr, col = (tid % lpr) * V;
  const float* acc_last = a.sm3_old + T.sm3_off[last] + col;
  unsigned mg[3] = {0u, 0u, 0u};
  for (int d = 0; d < last && d < 3; ++d) mg[d] = T.dims[d] > 1 ? 0xFFFFFFFFu / (unsigned)T.dims[d] + 1u : 0u;
  float tm[V];
#pragma unroll
  for (int j = 0; j < V; ++j) tm[j] = 0.f;
  for (int r0 = 0; r0 < ck.nrows; r0 += rpi) {
    const int rr = r0 + sub;
    const bool ok = rr < ck.nrows;
    const int row = ck.row0 + rr;
    float lead = 3.4e38f;
    int lidx[3] = {0, 0, 0};
    if (sm3_on && ok) {
      int r = row;
      for (int d = last - 1; d >= 0; --d) {
        const int q = fast_div(r, T.dims[d], mg[d]);
        lidx[d] = r - q * T.dims[d];
        r = q;
        lead = fminf(lead, a.sm3_old[T.sm3_off[d] + lidx[d]]);
      }
    }
    float rmax = 0.f;
    if (ok) {
      const long long gi = T.off + (long long)row * C + col;
      float g[V], w[V];
      if (V == 4) {
        const float4 gv = a.uin ? *reinterpret_cast<const float4*>(a.uin + gi) : *reinterpret_cast<const float4*>(a.grad + gi);
        const float4 wv = *reinterpret_cast<const float4*>(a.master + gi);
        g[0] = gv.x; g[1] = gv.y; g[2] = gv.z; g[3] = gv.w;
        w[0] = wv.x; w[1] = wv.y; w[2] = wv.z; w[3] = wv.w;
      } else {
        g[0] = a.uin ? a.uin[gi] : a.grad[gi];
        w[0] = a.master[gi];
      }
      if (!a.uin) {
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] *= a.grad_scale;
      }
      row_program<V, PROG>(a, F, gi, acc_last, lead, g, w, tm, rmax, deb1, deb2);
      finish_elems<V>(a, T, gi, g, w, s1, s2);
    }
    if (sm3_on && last > 0) {
      for (int o = lpr / 2; o > 0; o >>= 1) rmax = fmaxf(rmax, __shfl_xor(rmax, o, 64));
      if (ok && (tid % lpr) == 0 && rmax > 0.f)
        for (int d = 0; d < last; ++d) atomic_max_nonneg(a.sm3_new + T.sm3_off[d] + lidx[d], rmax);
    }
  }
  if (sm3_on) {   // combine the rpi lanes that share each column, then one global atomic per column
    for (int i = tid; i < C; i += RW_NT) tmax[i] = 0.f;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < V; ++j)
      if (tm[j] > 0.f) atomicMax(reinterpret_cast<int*>(tmax + col + j), __float_as_int(tm[j]));
    __syncthreads();
    for (int i = tid; i < C; i += RW_NT)
      if (tmax[i] > 0.f) atomic_max_nonneg(a.sm3_new + T.sm3_off[last] + i, tmax[i]);
  }
}

template <int V, int PROG>
__device__ __forceinline__ void rows_body(const ApplyArgs& a, const OptTensor& T, const float* F, const RChunk& ck,
                                          float* tmax, bool sm3_on, float deb1, float deb2, float& s1, float& s2) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int last = T.ndim - 1;
  const int C = T.dims[last];
  const float* acc_last = a.sm3_old + T.sm3_off[last] + ck.col0;
  if (sm3_on)
    for (int c = tid * V; c < ck.ncols; c += RW_NT * V)
#pragma unroll
      for (int j = 0; j < V; ++j) tmax[c + j] = 0.f;
  for (int rr = 0; rr < ck.nrows; ++rr) {
    const int row = ck.row0 + rr;
    float lead = 3.4e38f;
    int lidx[3] = {0, 0, 0};
    if (sm3_on) {
      int r = row;
      for (int d = last - 1; d >= 0; --d) {
        lidx[d] = r % T.dims[d];
        r /= T.dims[d];
        lead = fminf(lead, a.sm3_old[T.sm3_off[d] + lidx[d]]);
      }
    }
    float rmax = 0.f;
    const long long rbase = T.off + (long long)row * C + ck.col0;
    int c0 = tid * V;
    if (PROG == 1 && V == 4 && sm3_on && a.final_seg && !a.uin && !a.emit_stats) {
      // the shipped chain on float4 rows, two column groups per pass with every load of both issued before any
      // store: the generic loop below issues one group's loads only after the previous group's stores (the
      // compiler cannot prove master / mom / compute apart), one round trip per 1024 columns
      const Stage M = a.st[2];
      const float lr = lr_of(a), cl = F[0];
      for (; c0 + RW_NT * V < ck.ncols; c0 += 2 * RW_NT * V) {
        const int cc[2] = {c0, c0 + RW_NT * V};
        float4 gv[2], wv[2], mv[2], av[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const long long gi = rbase + cc[u];
          gv[u] = *reinterpret_cast<const float4*>(a.grad + gi);
          wv[u] = *reinterpret_cast<const float4*>(a.master + gi);
          mv[u] = *reinterpret_cast<const float4*>(a.mom + gi);
          av[u] = *reinterpret_cast<const float4*>(acc_last + cc[u]);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const long long gi = rbase + cc[u];
          float g[4] = {gv[u].x, gv[u].y, gv[u].z, gv[u].w}, w[4] = {wv[u].x, wv[u].y, wv[u].z, wv[u].w};
          float m[4] = {mv[u].x, mv[u].y, mv[u].z, mv[u].w}, al[4] = {av[u].x, av[u].y, av[u].z, av[u].w};
          float tm[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            tm[j] = tmax[cc[u] + j];
            g[j] *= a.grad_scale;   // same operation order as the generic path: bit-identical updates
            g[j] *= cl;
            const float nu = fminf(lead, al[j]) + g[j] * g[j];
            tm[j] = fmaxf(tm[j], nu);
            rmax = fmaxf(rmax, nu);
            g[j] *= opt_rsqrt(nu);
            m[j] = M.a * m[j] + g[j] * M.b;
            g[j] = (M.c != 0.f ? g[j] + M.a * m[j] : m[j]) * lr;
            if (T.flags & 2) g[j] *= a.rezero_mult;
            if ((T.flags & 1) && a.wd > 0.f) g[j] += w[j] * lr * a.wd;
            w[j] -= g[j];
            tmax[cc[u] + j] = tm[j];
          }
          *reinterpret_cast<float4*>(a.mom + gi) = make_float4(m[0], m[1], m[2], m[3]);
          *reinterpret_cast<float4*>(a.master + gi) = make_float4(w[0], w[1], w[2], w[3]);
          if (a.compute)
            *reinterpret_cast<uint2*>(a.compute + gi) = make_uint2(pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3]));
        }
      }
    }
    for (int c = c0; c < ck.ncols; c += RW_NT * V) {
      const long long gi = rbase + c;
      float g[V], w[V];
      if (V == 4) {
        const float4 gv = a.uin ? *reinterpret_cast<const float4*>(a.uin + gi) : *reinterpret_cast<const float4*>(a.grad + gi);
        const float4 wv = *reinterpret_cast<const float4*>(a.master + gi);
        g[0] = gv.x; g[1] = gv.y; g[2] = gv.z; g[3] = gv.w;
        w[0] = wv.x; w[1] = wv.y; w[2] = wv.z; w[3] = wv.w;
      } else {
        g[0] = a.uin ? a.uin[gi] : a.grad[gi];
        w[0] = a.master[gi];
      }
      if (!a.uin) {
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] *= a.grad_scale;
      }
      float tmx[V];
#pragma unroll
      for (int j = 0; j < V; ++j) tmx[j] = sm3_on ? tmax[c + j] : 0.f;
      row_program<V, PROG>(a, F, gi, acc_last + c, lead, g, w, tmx, rmax, deb1, deb2);
      if (sm3_on) {
#pragma unroll
        for (int j = 0; j < V; ++j) tmax[c + j] = tmx[j];
      }
      finish_elems<V>(a, T, gi, g, w, s1, s2);
    }
    if (sm3_on && last > 0) {
      rmax = wave_max_f(rmax);
      if (lane == 0 && rmax > 0.f)
        for (int d = 0; d < last; ++d) atomic_max_nonneg(a.sm3_new + T.sm3_off[d] + lidx[d], rmax);
    }
  }
  if (sm3_on)
    for (int c = tid * V; c < ck.ncols; c += RW_NT * V)
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float v = tmax[c + j];
        if (v > 0.f) atomic_max_nonneg(a.sm3_new + T.sm3_off[last] + ck.col0 + c + j, v);
      }
}

template <int PROG>
__global__ __launch_bounds__(RW_NT) void opt_rows_kernel(ApplyArgs a, const RChunk* chunks) {
  __shared__ float tmax[RW_COLS];
  const RChunk ck = chunks[blockIdx.x];
  const OptTensor T = a.tensors[ck.t];
  const float* F = a.fac + ck.t * 8;
  bool sm3_on = false;
  for (int s = 0; s < a.nst; ++s) sm3_on |= a.st[s].op == OP_SM3;
  const float deb1 = 1.f / (1.f - powf(a.beta1, step_of(a)));
  const float deb2 = 1.f / (1.f - powf(a.beta2, step_of(a)));
  float s1 = 0.f, s2 = 0.f;
  // vec bit 0: float4 (offset and C multiples of 4); bit 1: narrow rows (C / V lanes per row, power of two <= 64)
  if (ck.vec & 2) {
    if (ck.vec & 1) rows_packed<4, PROG>(a, T, F, ck, tmax, sm3_on, deb1, deb2, s1, s2);
    else rows_packed<1, PROG>(a, T, F, ck, tmax, sm3_on, deb1, deb2, s1, s2);
  } else {
    if (ck.vec & 1) rows_body<4, PROG>(a, T, F, ck, tmax, sm3_on, deb1, deb2, s1, s2);
    else rows_body<1, PROG>(a, T, F, ck, tmax, sm3_on, deb1, deb2, s1, s2);
  }
  if (a.emit_stats) {
    __shared__ float red[4];
    s2 = block_sum<4>(s2, red);
    s1 = block_sum<4>(s1, red);
    if (threadIdx.x == 0) {
      a.part[(a.part_base + blockIdx.x) * 4 + 0] = s2;
      a.part[(a.part_base + blockIdx.x) * 4 + 1] = s1;
    }
  }
}

// pass 0: sum g^2, sum g of the (scaled) raw gradient, sum w^2, sum w of the weights (float4 when aligned), one
// partial per chunk into part[chunk][4]; opt_fold_kernel sums each tensor's chunks in chunk order (no atomics)
__global__ __launch_bounds__(NTH) void opt_stats_kernel(const OptTensor* tensors, const Chunk* chunks,
                                                        const float* grad, const float* master, float* part,
                                                        float grad_scale) {
  const Chunk ck = chunks[blockIdx.x];
  const OptTensor T = tensors[ck.t];
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  const long long base = T.off + ck.start;
  if ((base & 3) == 0 && (ck.len & 3) == 0) {
    const float4* g4 = reinterpret_cast<const float4*>(grad + base);
    const float4* w4 = reinterpret_cast<const float4*>(master + base);
    for (long long v = threadIdx.x; v < ck.len / 4; v += NTH) {
      const float4 g = g4[v], w = w4[v];
      const float gx = g.x * grad_scale, gy = g.y * grad_scale, gz = g.z * grad_scale, gw = g.w * grad_scale;
      a0 += gx * gx + gy * gy + gz * gz + gw * gw; a1 += gx + gy + gz + gw;
      a2 += w.x * w.x + w.y * w.y + w.z * w.z + w.w * w.w; a3 += w.x + w.y + w.z + w.w;
    }
  } else {
    for (long long e = threadIdx.x; e < ck.len; e += NTH) {
      const float g = grad[base + e] * grad_scale, w = master[base + e];
      a0 += g * g; a1 += g; a2 += w * w; a3 += w;
    }
  }
  __shared__ float red[4];
  a0 = block_sum<4>(a0, red); a1 = block_sum<4>(a1, red); a2 = block_sum<4>(a2, red); a3 = block_sum<4>(a3, red);
  if (threadIdx.x == 0)
    *reinterpret_cast<float4*>(part + (long long)blockIdx.x * 4) = make_float4(a0, a1, a2, a3);
}

// stats[t][j] = sum over the tensor's partial rows part[first .. first + count)[j] (j < ncols), in row order: one
// wave per tensor, lane-strided sums combined by the (deterministic) butterfly
__global__ __launch_bounds__(NTH) void opt_fold_kernel(const int* __restrict__ ranges, int ntensors,
                                                       const float* __restrict__ part, float* __restrict__ stats,
                                                       int ncols) {
  const int t = blockIdx.x * (NTH / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (t >= ntensors) return;
  const int first = ranges[2 * t], count = ranges[2 * t + 1];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int i = lane; i < count; i += 64) {
    const float4 v = *reinterpret_cast<const float4*>(part + (long long)(first + i) * 4);
    acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
  }
  for (int j = 0; j < ncols; ++j) {
    const float v = wave_sum(acc[j]);
    if (lane == 0) stats[t * 8 + j] = v;
  }
}

// per-tensor factors for the reduction stage that opens the next segment. One thread per tensor; the global
// L2 norm is reduced by a single block first (ntensors is small: hundreds).
__global__ __launch_bounds__(NTH) void opt_scalar_kernel(const OptTensor* tensors, int ntensors, const float* stats,
                                                         float* fac, float* sstate, float* af_state,
                                                         const float* af_rows_sum, const float* af_cols_sum, Stage st,
                                                         float beta1, float beta2, float step_count, int tp_size,
                                                         const float* dyn) {
  if (dyn) step_count = dyn[1];
  __shared__ float red[4];
  float gl = 0.f;
  for (int t = threadIdx.x; t < ntensors; t += NTH) gl += stats[t * 8 + 0];
  gl = block_sum<4>(gl, red);
  for (int t = threadIdx.x; t < ntensors; t += NTH) {
    const OptTensor T = tensors[t];
    const float* s = stats + t * 8;
    float* f = fac + t * 8;
    const float n = (float)T.n;
    switch (st.op) {
      case OP_ADAPTIVE_CLIP: {
        const float gn = fminf(rsqrtf(s[0]), 1e6f);
        const float wn = fmaxf(sqrtf(s[2]), 1e-3f);
        f[0] = fminf(wn * gn * st.a, 1.f);
        break;
      }
      case OP_L2_CLIP: f[0] = st.a * rsqrtf(fmaxf(s[0], 1.f / (st.a * st.a))); break;
      case OP_GLOBAL_L2_CLIP: f[0] = st.a * rsqrtf(fmaxf(gl, 1.f / (st.a * st.a))); break;
      case OP_GRAD_CENTRAL: f[0] = s[1] / (n * ((T.flags & 4) ? tp_size : 1)); break;
      case OP_WEIGHT_CENTRAL: f[1] = s[3] / (n * ((T.flags & 4) ? tp_size : 1)); break;
      case OP_NOVOGRAD: {
        float* ss = sstate + t * 4;
        const float p2_old = ss[2];
        const float p2_new = p2_old * beta2 + s[0] * (1.f - beta2);
        ss[2] = p2_new;
        f[2] = 1.f / fmaxf(sqrtf(p2_old), 1e-5f);
        const float deb2 = 1.f / (1.f - powf(beta2, step_count));
        f[3] = 1.f / fmaxf(sqrtf(p2_new * deb2), 1e-5f);
        break;
      }
      case OP_ADAFACTOR: {
        // decay rate 1 - step^-0.8 (Shazeer & Stern 2018, eq. in section 7.2), fixed-beta variant if st.a > 0.
        // Under TP the sums are of the full tensor (TP-reduced by the caller) and the counts global: flags 8 = the
        // rows (leading dims) are head-sharded, 16 = the columns (last dim) are. f[6] = sum of the row factors
        // (partial when rows are sharded: the caller reduces it and recomputes f[5] = f[7] / f[6]).
        const float b2 = st.a > 0.f ? st.a : 1.f - powf(step_count, -0.8f);
        f[4] = b2;
        if (T.fac_rows > 0) {
          const float rows_g = (float)T.fac_rows * ((T.flags & 8) ? tp_size : 1);
          const float cols_g = (float)T.fac_cols * ((T.flags & 16) ? tp_size : 1);
          float msum = 0.f;
          for (int r = 0; r < T.fac_rows; ++r) {
            float* R = af_state + T.fac_off + r;
            *R = *R * b2 + (af_rows_sum[T.fac_off + r] / cols_g + 1e-30f) * (1.f - b2);
            msum += *R;
          }
          for (int c = 0; c < T.fac_cols; ++c) {
            float* C = af_state + T.fac_off + T.fac_rows + c;
            *C = *C * b2 + (af_cols_sum[T.fac_off + T.fac_rows + c] / rows_g + 1e-30f) * (1.f - b2);
          }
          f[5] = rows_g / fmaxf(msum, 1e-30f);
          f[6] = msum;
          f[7] = rows_g;
        }
        break;
      }
      case OP_ADAFACTOR_CLIP: {
        const float rms = sqrtf(s[0] / (n * ((T.flags & 4) ? tp_size : 1)));
        f[0] = 1.f / fmaxf(1.f, rms / (st.a > 0.f ? st.a : 1.f));
        break;
      }
      default: break;
    }
  }
}
// ---------------------------------------------------------------------------------------------------------------
// Adafactor's factored statistics of a segment output u (Shazeer & Stern 2018), deterministic: a tensor is viewed as
// [R rows][C cols]; a work item is a tile of <= 64 rows x <= 1024 columns. Its 4 waves take every 4th row; a lane
// owns the 16 columns c0 + lane + 64 k. Per row the lane's squares are summed in k order and reduced across the
// wave by a fixed butterfly: one partial row sum per (column chunk, row) into rowpart. Column partials are summed
// over the wave's rows in order, then over the 4 waves in wave order: one partial column sum per (row tile, col)
// into colpart. opt_factored_fold adds the partials in index order. No float atomics: bitwise reproducible.
struct FChunk { int t, row0, nrows, col0, ncols, rt, cc, pad; long long cp_off, rp_off; };
struct FFold { int t, kind, start, len; long long off; int nparts, pad; };   // kind 0: rows, 1: cols

__global__ __launch_bounds__(256) void opt_factored_kernel(const OptTensor* __restrict__ tensors,
                                                           const FChunk* __restrict__ chunks,
                                                           const float* __restrict__ u, float* __restrict__ colpart,
                                                           float* __restrict__ rowpart) {
  __shared__ float cacc[4][1024];
  const FChunk ck = chunks[blockIdx.x];
  const OptTensor T = tensors[ck.t];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* base = u + T.off;
  float cs[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) cs[k] = 0.f;
  for (int r = w; r < ck.nrows; r += 4) {
    const float* row = base + (long long)(ck.row0 + r) * T.fac_cols + ck.col0;
    float x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int c = lane + 64 * k;
      x[k] = c < ck.ncols ? row[c] : 0.f;
    }
    float rs = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float q = x[k] * x[k];
      rs += q;
      cs[k] += q;
    }
    rs = wave_sum(rs);
    if (lane == 0) rowpart[ck.rp_off + (long long)ck.cc * T.fac_rows + ck.row0 + r] = rs;
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) cacc[w][lane + 64 * k] = cs[k];
  __syncthreads();
  for (int c = threadIdx.x; c < ck.ncols; c += 256)
    colpart[ck.cp_off + (long long)ck.rt * T.fac_cols + ck.col0 + c] =
        ((cacc[0][c] + cacc[1][c]) + cacc[2][c]) + cacc[3][c];
}

// af_rows_sum / af_cols_sum (at each tensor's fac_off) = the partials added in index order
__global__ __launch_bounds__(256) void opt_factored_fold_kernel(const OptTensor* __restrict__ tensors,
                                                                const FFold* __restrict__ folds,
                                                                const float* __restrict__ colpart,
                                                                const float* __restrict__ rowpart,
                                                                float* __restrict__ af_sums) {
  const FFold f = folds[blockIdx.x];
  const OptTensor T = tensors[f.t];
  const int i = f.start + (int)threadIdx.x;
  if (threadIdx.x >= (unsigned)f.len) return;
  float s = 0.f;
  if (f.kind == 0) {
    for (int p = 0; p < f.nparts; ++p) s += rowpart[f.off + (long long)p * T.fac_rows + i];
    af_sums[T.fac_off + i] = s;
  } else {
    for (int p = 0; p < f.nparts; ++p) s += colpart[f.off + (long long)p * T.fac_cols + i];
    af_sums[T.fac_off + T.fac_rows + i] = s;
  }
}
}  // namespace

struct ObstOptDesc {
  const void* tensors; const void* chunks; int ntensors; int nchunks;
  const float* grad; const float* uin; float* uout; float* master; void* compute;
  float* stats; float* fac; float* sstate; float* mom; float* adam_m; float* adam_v;
  const float* sm3_old; float* sm3_new; float* af_state; float* af_rows_sum; float* af_cols_sum;
  int stages[MAXST * 4];   // (op, a, b, c) with a/b/c as float bit patterns
  int nst; int final_seg; int emit_stats; int emit_factored;
  float lr, wd, rezero_mult, grad_scale, beta1, beta2, step_count;
  int tp_size;
  const float* dyn;        // device [lr, step_count] or null (then lr / step_count above)
  float* part;             // per-block partial statistics ([blocks][4] floats), folded by obst_opt_fold
  int part_base;           // emit_stats of obst_opt_apply: first partial row of this launch's blocks
};

static_assert(sizeof(OptTensor) == 88, "OptTensor layout is mirrored in python (optim/fused.py)");
static_assert(sizeof(Chunk) == 24, "Chunk layout is mirrored in python (optim/fused.py)");
static_assert(sizeof(RChunk) == 24, "RChunk layout is mirrored in python (optim/fused.py)");
static_assert(sizeof(FChunk) == 48 && sizeof(FFold) == 32, "FChunk / FFold layouts are mirrored in optim/fused.py");

OBST_API int obst_opt_stats(const ObstOptDesc* d, hipStream_t s) {
  if (!d->part) return -1;
  hipLaunchKernelGGL(opt_stats_kernel, dim3(d->nchunks), dim3(NTH), 0, s, (const OptTensor*)d->tensors,
                     (const Chunk*)d->chunks, d->grad, d->master, d->part, d->grad_scale);
  return (int)hipGetLastError();
}

// ranges: int32 [ntensors][2] = (first partial row, count) of each tensor
OBST_API int obst_opt_fold(const ObstOptDesc* d, const int* ranges, int ncols, hipStream_t s) {
  if (!d->part || ncols < 1 || ncols > 4) return -1;
  hipLaunchKernelGGL(opt_fold_kernel, dim3((unsigned)((d->ntensors + 3) / 4)), dim3(NTH), 0, s, ranges,
                     d->ntensors, d->part, d->stats, ncols);
  return (int)hipGetLastError();
}

OBST_API int obst_opt_scalar(const ObstOptDesc* d, hipStream_t s) {
  Stage st;
  st.op = d->stages[0];
  st.a = __builtin_bit_cast(float, d->stages[1]);
  st.b = __builtin_bit_cast(float, d->stages[2]);
  st.c = __builtin_bit_cast(float, d->stages[3]);
  hipLaunchKernelGGL(opt_scalar_kernel, dim3(1), dim3(NTH), 0, s, (const OptTensor*)d->tensors, d->ntensors, d->stats,
                     d->fac, d->sstate, d->af_state, d->af_rows_sum, d->af_cols_sum, st, d->beta1, d->beta2,
                     d->step_count, d->tp_size, d->dyn);
  return (int)hipGetLastError();
}

static ApplyArgs apply_args(const ObstOptDesc* d) {
  ApplyArgs a;
  a.tensors = (const OptTensor*)d->tensors; a.chunks = (const Chunk*)d->chunks;
  a.grad = d->grad; a.uin = d->uin; a.uout = d->uout; a.master = d->master; a.compute = (bf16_t*)d->compute;
  a.stats = d->stats; a.fac = d->fac; a.sstate = d->sstate; a.mom = d->mom; a.adam_m = d->adam_m;
  a.adam_v = d->adam_v; a.sm3_old = d->sm3_old; a.sm3_new = d->sm3_new; a.af_old = d->af_state;
  a.af_rows_sum = d->af_rows_sum; a.af_cols_sum = d->af_cols_sum;
  for (int i = 0; i < d->nst; ++i) {
    a.st[i].op = d->stages[4 * i];
    a.st[i].a = __builtin_bit_cast(float, d->stages[4 * i + 1]);
    a.st[i].b = __builtin_bit_cast(float, d->stages[4 * i + 2]);
    a.st[i].c = __builtin_bit_cast(float, d->stages[4 * i + 3]);
  }
  a.nst = d->nst; a.final_seg = d->final_seg; a.emit_stats = d->emit_stats; a.emit_factored = d->emit_factored;
  a.lr = d->lr; a.wd = d->wd; a.rezero_mult = d->rezero_mult; a.grad_scale = d->grad_scale;
  a.beta1 = d->beta1; a.beta2 = d->beta2; a.step_count = d->step_count; a.dyn = d->dyn;
  a.part = d->part; a.part_base = d->part_base;
  return a;
}

OBST_API int obst_opt_apply(const ObstOptDesc* d, hipStream_t s) {
  if (d->nst > MAXST) return -1;
  if (d->emit_stats && !d->part) return -3;
  if (d->nchunks <= 0) return 0;
  hipLaunchKernelGGL(opt_apply_kernel, dim3(d->nchunks), dim3(NTA), 0, s, apply_args(d));
  return (int)hipGetLastError();
}

// row-tiled apply (no Adafactor stages, no factored-stat emission); rchunks: RChunk[nrchunks]
OBST_API int obst_opt_apply_rows(const ObstOptDesc* d, const void* rchunks, int nrchunks, hipStream_t s) {
  if (d->nst > MAXST || d->emit_factored) return -1;
  if (d->emit_stats && !d->part) return -3;
  for (int i = 0; i < d->nst; ++i)
    if (d->stages[4 * i] == OP_ADAFACTOR || d->stages[4 * i] == OP_ADAFACTOR_CLIP) return -2;
  if (nrchunks <= 0) return 0;
  const int* st = d->stages;
  const bool shipped = d->nst == 4 && d->final_seg && !d->emit_stats && !d->uin &&
                       (st[0] == OP_ADAPTIVE_CLIP || st[0] == OP_L2_CLIP || st[0] == OP_GLOBAL_L2_CLIP ||
                        st[0] == OP_SCALE) &&
                       st[4] == OP_SM3 && st[8] == OP_MOMENTUM && st[12] == OP_LR;
  if (shipped)
    hipLaunchKernelGGL(opt_rows_kernel<1>, dim3(nrchunks), dim3(RW_NT), 0, s, apply_args(d), (const RChunk*)rchunks);
  else
    hipLaunchKernelGGL(opt_rows_kernel<0>, dim3(nrchunks), dim3(RW_NT), 0, s, apply_args(d), (const RChunk*)rchunks);
  return (int)hipGetLastError();
}

// deterministic Adafactor row / column sums of u (the segment output) into d->af_rows_sum (= af_cols_sum buffer)
OBST_API int obst_opt_factored(const ObstOptDesc* d, const float* u, const void* fchunks, int nfchunks,
                               const void* folds, int nfolds, float* colpart, float* rowpart, hipStream_t s) {
  if (nfchunks <= 0) return 0;
  hipLaunchKernelGGL(opt_factored_kernel, dim3(nfchunks), dim3(256), 0, s, (const OptTensor*)d->tensors,
                     (const FChunk*)fchunks, u, colpart, rowpart);
  hipLaunchKernelGGL(opt_factored_fold_kernel, dim3(nfolds), dim3(256), 0, s, (const OptTensor*)d->tensors,
                     (const FFold*)folds, colpart, rowpart, d->af_rows_sum);
  return (int)hipGetLastError();
}
