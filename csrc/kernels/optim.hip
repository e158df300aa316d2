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
};

__device__ __forceinline__ float opt_rsqrt(float x) { return 1.f / fmaxf(sqrtf(x), 1e-5f); }

__device__ __forceinline__ void atomic_max_nonneg(float* addr, float v) {
  atomicMax(reinterpret_cast<int*>(addr), __float_as_int(v));   // valid for v >= 0 (IEEE ordering of non-negatives)
}

constexpr int SM3_WIN = 1024;  // per-dim LDS window of accumulator slots reduced inside the block

__global__ __launch_bounds__(NTH) void opt_apply_kernel(ApplyArgs a) {
  const Chunk ck = a.chunks[blockIdx.x];
  const OptTensor T = a.tensors[ck.t];
  const float* F = a.fac + ck.t * 8;
  float s2 = 0.f, s1 = 0.f;
  // SM3 accumulator max: dims whose index takes few values inside this chunk (leading dims) are max-reduced in
  // LDS and flushed with one global atomic per slot; dims with many distinct indices (the contiguous trailing
  // dim) go straight to global atomics, whose addresses are then all different (no contention).
  __shared__ float sm3_lds[4][SM3_WIN];
  int win_lo[4] = {0, 0, 0, 0}, win_cnt[4] = {0, 0, 0, 0};
  bool has_sm3 = false;
  for (int s = 0; s < a.nst; ++s) has_sm3 |= a.st[s].op == OP_SM3;
  has_sm3 &= T.ndim > 0;
  if (has_sm3) {
    long long stride = 1;
    for (int d = T.ndim - 1; d >= 0; --d) {
      const long long span = (ck.len - 1) / stride + 2;
      const int cnt = (int)(span < T.dims[d] ? span : T.dims[d]);
      win_lo[d] = (int)((ck.start / stride) % T.dims[d]);
      win_cnt[d] = cnt <= SM3_WIN ? cnt : 0;
      stride *= T.dims[d];
    }
    for (int d = 0; d < 4; ++d)
      for (int i = threadIdx.x; i < SM3_WIN; i += NTH) sm3_lds[d][i] = 0.f;
    __syncthreads();
  }
  // adafactor row/column sums of g^2: same LDS-window treatment (rows of this chunk, and all columns when few)
  const bool af = a.emit_factored && T.fac_rows > 0;
  const long long af_r0 = af ? ck.start / T.fac_cols : 0;
  const bool af_rows_win = af && ((ck.start + ck.len - 1) / T.fac_cols - af_r0 + 1) <= SM3_WIN;
  const bool af_cols_win = af && T.fac_cols <= SM3_WIN;
  if (af) {
    for (int d = 0; d < 2; ++d)
      for (int i = threadIdx.x; i < SM3_WIN; i += NTH) sm3_lds[d][i] = 0.f;
    __syncthreads();
  }
  const float deb1 = 1.f / (1.f - powf(a.beta1, a.step_count));
  const float deb2 = 1.f / (1.f - powf(a.beta2, a.step_count));
  for (long long e = ck.start + threadIdx.x; e < ck.start + ck.len; e += NTH) {
    const long long gi = T.off + e;
    float g = a.uin ? a.uin[gi] : a.grad[gi] * a.grad_scale;
    const float w = a.master[gi];
    // multi-index for SM3 / adafactor
    int idx[4] = {0, 0, 0, 0};
    {
      long long r = e;
      for (int d = T.ndim - 1; d >= 0; --d) { idx[d] = (int)(r % T.dims[d]); r /= T.dims[d]; }
    }
    for (int s = 0; s < a.nst; ++s) {
      const Stage S = a.st[s];
      switch (S.op) {
        case OP_ADAPTIVE_CLIP: case OP_L2_CLIP: case OP_GLOBAL_L2_CLIP: case OP_ADAFACTOR_CLIP: case OP_SCALE:
          g *= F[0]; break;
        case OP_VALUE_CLIP: g = fmaxf(fminf(g, S.a), -S.a); break;
        case OP_GRAD_CENTRAL: g -= F[0]; break;
        case OP_WEIGHT_CENTRAL: g += F[1]; break;
        case OP_SM3: {
          if (T.ndim == 0) goto scalar_adam;
          float nu = a.sm3_old[T.sm3_off[0] + idx[0]];
          for (int d = 1; d < T.ndim; ++d) nu = fminf(nu, a.sm3_old[T.sm3_off[d] + idx[d]]);
          nu += g * g;
          for (int d = 0; d < T.ndim; ++d) {
            if (win_cnt[d]) {
              int slot = idx[d] - win_lo[d];
              if (slot < 0) slot += T.dims[d];
              atomicMax(reinterpret_cast<int*>(&sm3_lds[d][slot]), __float_as_int(nu));
            } else {
              atomic_max_nonneg(a.sm3_new + T.sm3_off[d] + idx[d], nu);
            }
          }
          g *= opt_rsqrt(nu);
          break;
        }
        case OP_MOMENTUM: {
          const float st = S.a * a.mom[gi] + g * S.b;
          a.mom[gi] = st;
          g = S.c != 0.f ? g + S.a * st : st;
          break;
        }
        case OP_ADAM: {
          if (T.ndim == 0) goto scalar_adam;
          const float v = a.adam_v[gi] * a.beta2 + g * g * (1.f - a.beta2);
          const float m = a.adam_m[gi] * a.beta1 + g * (1.f - a.beta1);
          a.adam_v[gi] = v; a.adam_m[gi] = m;
          g = opt_rsqrt(v * deb2) * m * deb1;
          break;
        }
        case OP_NOVOGRAD: {
          if (T.ndim == 0) goto scalar_adam;
          // F[2] = rsqrt-term of the OLD p2, F[3] = rsqrt-term of the debiased NEW p2 (scalar kernel)
          const float p1 = a.beta1 * a.mom[gi] + g * F[2];
          a.mom[gi] = p1;
          g = a.beta1 * p1 + g * F[3];
          break;
        }
        case OP_ADAFACTOR: {
          if (T.fac_rows == 0) {  // unfactored (<= 1-D): per-element second moment in adam_v
            const float v = a.adam_v[gi] * F[4] + (g * g + 1e-30f) * (1.f - F[4]);
            a.adam_v[gi] = v;
            g = g * rsqrtf(v);
          } else {
            const long long inner = T.fac_cols;
            const long long rr = e / inner, cc = e % inner;
            const float R = a.af_old[T.fac_off + rr], C = a.af_old[T.fac_off + T.fac_rows + cc];
            const float vhat = R * C * F[5];       // F[5] = 1 / mean(R)
            g = g * rsqrtf(fmaxf(vhat, 1e-30f));
          }
          break;
        }
        case OP_LR: g *= a.lr; break;
        default: break;
      }
      continue;
    scalar_adam: {
        float* ss = a.sstate + ck.t * 4;
        const float v = ss[1] * a.beta2 + g * g * (1.f - a.beta2);
        const float m = ss[0] * a.beta1 + g * (1.f - a.beta1);
        ss[1] = v; ss[0] = m;
        g = opt_rsqrt(v * deb2) * m * deb1;
      }
    }
    if (a.emit_stats) { s2 += g * g; s1 += g; }
    if (a.emit_factored && T.fac_rows > 0) {
      const long long inner = T.fac_cols;
      const float v = g * g + 1e-30f;
      const long long r = e / inner, c = e % inner;
      if (af_rows_win) atomicAdd(&sm3_lds[0][r - af_r0], v);
      else atomicAdd(a.af_rows_sum + T.fac_off + r, v);
      if (af_cols_win) atomicAdd(&sm3_lds[1][c], v);
      else atomicAdd(a.af_cols_sum + T.fac_off + T.fac_rows + c, v);
    }
    if (a.final_seg) {
      if (T.flags & 2) g *= a.rezero_mult;
      if ((T.flags & 1) && a.wd > 0.f) g += w * a.lr * a.wd;
      const float nw = w - g;
      a.master[gi] = nw;
      if (a.compute) a.compute[gi] = f2bf(nw);
    } else {
      a.uout[gi] = g;
    }
  }
  if (has_sm3) {
    __syncthreads();
    for (int d = 0; d < T.ndim; ++d) {
      for (int i = threadIdx.x; i < win_cnt[d]; i += NTH) {
        const float v = sm3_lds[d][i];
        if (v > 0.f) {
          int j = win_lo[d] + i;
          if (j >= T.dims[d]) j -= T.dims[d];
          atomic_max_nonneg(a.sm3_new + T.sm3_off[d] + j, v);
        }
      }
    }
  }
  if (af) {
    __syncthreads();
    if (af_rows_win) {
      const int nr = (int)((ck.start + ck.len - 1) / T.fac_cols - af_r0 + 1);
      for (int i = threadIdx.x; i < nr; i += NTH) atomicAdd(a.af_rows_sum + T.fac_off + af_r0 + i, sm3_lds[0][i]);
    }
    if (af_cols_win)
      for (int i = threadIdx.x; i < T.fac_cols; i += NTH)
        atomicAdd(a.af_cols_sum + T.fac_off + T.fac_rows + i, sm3_lds[1][i]);
  }
  if (a.emit_stats) {
    __shared__ float red[4];
    s2 = block_sum<4>(s2, red);
    s1 = block_sum<4>(s1, red);
    if (threadIdx.x == 0) { atomicAdd(a.stats + ck.t * 8 + 0, s2); atomicAdd(a.stats + ck.t * 8 + 1, s1); }
  }
}

// pass 0: sum g^2, sum g of the (scaled) raw gradient, sum w^2, sum w of the weights
__global__ __launch_bounds__(NTH) void opt_stats_kernel(const OptTensor* tensors, const Chunk* chunks,
                                                        const float* grad, const float* master, float* stats,
                                                        float grad_scale) {
  const Chunk ck = chunks[blockIdx.x];
  const OptTensor T = tensors[ck.t];
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  for (long long e = ck.start + threadIdx.x; e < ck.start + ck.len; e += NTH) {
    const float g = grad[T.off + e] * grad_scale, w = master[T.off + e];
    a0 += g * g; a1 += g; a2 += w * w; a3 += w;
  }
  __shared__ float red[4];
  a0 = block_sum<4>(a0, red); a1 = block_sum<4>(a1, red); a2 = block_sum<4>(a2, red); a3 = block_sum<4>(a3, red);
  if (threadIdx.x == 0) {
    float* s = stats + ck.t * 8;
    atomicAdd(s + 0, a0); atomicAdd(s + 1, a1); atomicAdd(s + 2, a2); atomicAdd(s + 3, a3);
  }
}

// per-tensor factors for the reduction stage that opens the next segment. One thread per tensor; the global
// L2 norm is reduced by a single block first (ntensors is small: hundreds).
__global__ __launch_bounds__(NTH) void opt_scalar_kernel(const OptTensor* tensors, int ntensors, const float* stats,
                                                         float* fac, float* sstate, float* af_state,
                                                         const float* af_rows_sum, const float* af_cols_sum, Stage st,
                                                         float beta1, float beta2, float step_count, int tp_size) {
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
        // decay rate 1 - step^-0.8 (Shazeer & Stern 2018, eq. in section 7.2), fixed-beta variant if st.a > 0
        const float b2 = st.a > 0.f ? st.a : 1.f - powf(step_count, -0.8f);
        f[4] = b2;
        if (T.fac_rows > 0) {
          float msum = 0.f;
          for (int r = 0; r < T.fac_rows; ++r) {
            float* R = af_state + T.fac_off + r;
            *R = *R * b2 + (af_rows_sum[T.fac_off + r] / T.fac_cols) * (1.f - b2);
            msum += *R;
          }
          for (int c = 0; c < T.fac_cols; ++c) {
            float* C = af_state + T.fac_off + T.fac_rows + c;
            *C = *C * b2 + (af_cols_sum[T.fac_off + T.fac_rows + c] / T.fac_rows) * (1.f - b2);
          }
          f[5] = T.fac_rows / fmaxf(msum, 1e-30f);
        }
        break;
      }
      case OP_ADAFACTOR_CLIP: {
        const float rms = sqrtf(s[0] / n);
        f[0] = 1.f / fmaxf(1.f, rms / (st.a > 0.f ? st.a : 1.f));
        break;
      }
      default: break;
    }
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
};

static_assert(sizeof(OptTensor) == 88, "OptTensor layout is mirrored in python (optim/fused.py)");
static_assert(sizeof(Chunk) == 24, "Chunk layout is mirrored in python (optim/fused.py)");

OBST_API int obst_opt_stats(const ObstOptDesc* d, hipStream_t s) {
  hipLaunchKernelGGL(opt_stats_kernel, dim3(d->nchunks), dim3(NTH), 0, s, (const OptTensor*)d->tensors,
                     (const Chunk*)d->chunks, d->grad, d->master, d->stats, d->grad_scale);
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
                     d->step_count, d->tp_size);
  return (int)hipGetLastError();
}

OBST_API int obst_opt_apply(const ObstOptDesc* d, hipStream_t s) {
  if (d->nst > MAXST) return -1;
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
  a.beta1 = d->beta1; a.beta2 = d->beta2; a.step_count = d->step_count;
  hipLaunchKernelGGL(opt_apply_kernel, dim3(d->nchunks), dim3(NTH), 0, s, a);
  return (int)hipGetLastError();
}
