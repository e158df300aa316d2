// K05: the reference `norm` layer (src/model/normalization.py:22-34):
//   x -= mean(x);  x *= rsqrt(mean(x^2) + 1e-5);  x *= scale;  x += shift
// statistics over the trailing F elements of each row (F = features, or features_per_head for `group`, where
// rows are (token, head) pairs and the [heads, F] scale/shift is indexed by row % groups).
// One wave per row, the row held in registers (16-byte bf16 vector loads, Guideline 13), two-pass statistics,
// fp32 math. Backward: dx = rstd * (dxh - mean(dxh) - xh * mean(dxh * xh)); scale/shift gradients are summed per
// lane group in registers, stored as per-block (groups == 1) or per-lane-group partial slabs, and folded into the
// fp32 gradient buffer by norm_fold_kernel in a fixed order -- no float atomics, so the gradients (and with them the
// whole training step) are bitwise reproducible run to run and between eager and hipGraph replay.
// A split "row statistics" path (partial sums -> all-reduce over the TP group -> apply) serves the non-group
// norm when `heads` is split across ranks (collective X05).
#include "common.h"

#include <mutex>
#include <unordered_map>

namespace {

constexpr int NTH = 256;

// one-chunk rows (F <= 8 x lanes per row: ctx32_mixer's 256- and 512-wide head groups): forward rows in flight per lane
// group, backward rows in flight and blocks per CU (the backward's grid: one resident wave of blocks)
#ifndef NORM_FWD_U1
#define NORM_FWD_U1 1
#endif
#ifndef NORM_FWD_U64
#define NORM_FWD_U64 2
#endif
#ifndef NORM_BWD_U1
#define NORM_BWD_U1 4
#endif
#ifndef NORM_BWD_BPC1
#define NORM_BWD_BPC1 2
#endif
// the one-chunk backward (norm_bwd1_kernel): blocks per CU (its grid: one resident wave of them); 0 turns it off
#ifndef NORM_BWD1_BPC
#define NORM_BWD1_BPC 4
#endif

// LPR lanes per row (64 for F > 256; 32 / 16 / 8 for short rows so a wave covers 64/LPR rows at once),
// NCH chunks of LPR*8 elements per row
// row sums by DPP (quad permutes, half-row / row mirrors) and the gfx950 row swaps (v_permlane16/32_swap) instead of
// one ds_bpermute round trip through the LDS unit per step: every step adds a lane's value to its partner's in both
// lanes' order-independent form (a + b == b + a), so every lane of the row ends with the same bits
#ifndef NORM_DPP
#define NORM_DPP 1
#endif
// forward grid: 1 one resident wave of blocks (occupancy x CUs), 0 the fixed 2048-block grid of rounds 1-5 (1 measured
// 1.5 % slower at GPT-Neo-1.3B's 2048-wide rows and equal elsewhere, profiles/r6s/norm_ab9.jsonl)
#ifndef NORM_FWD_RESIDENT
#define NORM_FWD_RESIDENT 0
#endif
// forward streaming hints: bit 0 nontemporal row loads, bit 1 nontemporal output stores
#ifndef NORM_NT
#define NORM_NT 0
#endif
// whole-wave rows (64 lanes): 1 the two row swaps, 0 ds_bpermute, 2 row broadcasts + readlane
#ifndef NORM_DPP64
#define NORM_DPP64 1
#endif
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
template <int LPR, bool DPP = (NORM_DPP != 0)>
__device__ __forceinline__ float row_sum(float v) {
  if constexpr (DPP) {
    static_assert(LPR >= 8 && LPR <= 64, "rows of 8 to 64 lanes");
    v += dpp_mov<0xB1>(v);    // quad_perm [1, 0, 3, 2]: lane ^ 1
    v += dpp_mov<0x4E>(v);    // quad_perm [2, 3, 0, 1]: lane ^ 2
    v += dpp_mov<0x141>(v);   // row_half_mirror: the other quad of the 8-lane half
    if constexpr (LPR >= 16) v += dpp_mov<0x140>(v);   // row_mirror: the other half of the 16-lane row
    if constexpr (LPR == 64 && NORM_DPP64 == 0) {   // the ds_bpermute steps for the whole wave
      v += __shfl_xor(v, 16, 64);
      return v + __shfl_xor(v, 32, 64);
    }
    if constexpr (LPR == 64 && NORM_DPP64 == 2) {
      // whole wave: row 1 += row 0 and row 3 += row 2 (row_bcast:15), rows 2, 3 += row 1 (row_bcast:31), lane 63
      // broadcast through an SGPR
      v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142, 0xa, 0xf, false));
      v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x143, 0xc, 0xf, false));
      return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
    }
    if constexpr (LPR >= 32) {   // lane ^ 16
      const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
      v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    if constexpr (LPR >= 64) {   // lane ^ 32
      const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
      v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    return v;
  } else {
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  }
}

template <int LPR>
__device__ __forceinline__ float sub_sum(float v) {   // across the row-groups of a wave (same column)
#pragma unroll
  for (int o = LPR; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// 8 consecutive fp32 parameters (scale / shift) as two 16-byte loads (col % 8 == 0, F % 8 == 0)
__device__ __forceinline__ void load8f(const float* p, float (&o)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

template <int NCH, int LPR>
__device__ __forceinline__ void load_raw(const bf16_t* x, int F, int sl, bool ok, uint4 (&u)[NCH]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * LPR * 8 + sl * 8;
    if constexpr (NORM_NT & 1) {
      typedef unsigned v4u __attribute__((ext_vector_type(4)));
      const v4u t = (ok && col < F) ? __builtin_nontemporal_load(reinterpret_cast<const v4u*>(x + col)) : v4u{0u, 0u, 0u, 0u};
      u[c] = make_uint4(t[0], t[1], t[2], t[3]);
    } else {
      u[c] = (ok && col < F) ? *reinterpret_cast<const uint4*>(x + col) : make_uint4(0, 0, 0, 0);
    }
  }
}

// unconditional 16-byte loads of a row whose pointer the caller has clamped to a valid row; lanes past F re-read
// column 0 (their values are never used). No branch around the loads, so the compiler need not wait for each one
// before the join (a conditional load compiled to load + vmcnt(0) per chunk)
template <int NCH, int LPR>
__device__ __forceinline__ void load_rawc(const bf16_t* x, int F, int sl, uint4 (&u)[NCH]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * LPR * 8 + sl * 8;
    u[c] = *reinterpret_cast<const uint4*>(x + (col < F ? col : 0));
  }
}

__device__ __forceinline__ void unpack8(const uint4& u, float (&v)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[2 * j] = bf2f(w[j] & 0xffff); v[2 * j + 1] = bf2f(w[j] >> 16); }
}

template <int NCH>
__device__ __forceinline__ void unpack_row(const uint4 (&u)[NCH], float (&v)[NCH][8]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const uint32_t w[4] = {u[c].x, u[c].y, u[c].z, u[c].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[c][2 * j] = bf2f(w[j] & 0xffff); v[c][2 * j + 1] = bf2f(w[j] >> 16); }
  }
}

template <int NCH, int LPR>
__device__ __forceinline__ void load_row(const bf16_t* x, int F, int sl, bool ok, float (&v)[NCH][8]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * LPR * 8 + sl * 8;
    if (ok && col < F) {
      uint4 u = *reinterpret_cast<const uint4*>(x + col);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[c][2 * j] = bf2f(w[j] & 0xffff); v[c][2 * j + 1] = bf2f(w[j] >> 16); }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
  }
}

// The host sizes the grid so that the rows of one lane group (row, row + nw, ...) all belong to one parameter group
// (nw % groups == 0): scale / shift are loaded into registers once, not re-fetched per row (with 256-wide group rows
// the per-row parameter loads were 4x the row's own bytes)
// ACT: a following activation layer fused (Y = act(z)); its own instantiation, the plain kernel keeps its registers
template <int NCH, int LPR, int AK>   // AK: 0 plain, > 0 that activation (compile-time), -1 the runtime `act`
__device__ __forceinline__ void norm_fwd_body(const bf16_t* __restrict__ X, const float* __restrict__ scale,
                                              const float* __restrict__ shift, bf16_t* __restrict__ Y,
                                              float* __restrict__ rstd_out, long long rows, int F,
                                              int groups, float eps, const float* __restrict__ ext_stats,
                                              int act) {
  constexpr int RPW = 64 / LPR;
  // rows in flight per lane group (F 2048: 2-4 measured 2 % slower than 1; one-chunk rows: 2 at 64 lanes per row,
  // 1930 -> 1750 us at ctx32_mixer's 512-wide groups, but 1010 -> 1250 us at 32 lanes, 256-wide)
  constexpr int U = NCH == 1 ? (LPR == 64 ? NORM_FWD_U64 : NORM_FWD_U1) : 1;
  const int lane = threadIdx.x & 63, sub = lane / LPR, sl = lane % LPR;
  const long long nw = (long long)gridDim.x * 4 * RPW;
  long long r0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  float sc[NCH][8], sh[NCH][8];
  {
    const long long poff = (long long)((r0 + sub) % groups) * F;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * LPR * 8 + sl * 8;
      if (scale && col < F) load8f(scale + poff + col, sc[c]);
      if (shift && col < F) load8f(shift + poff + col, sh[c]);
    }
  }
  uint4 nxt[U][NCH];
#pragma unroll
  for (int u = 0; u < U; ++u) load_raw<NCH, LPR>(X + (r0 + u * nw + sub) * F, F, sl, r0 + u * nw + sub < rows, nxt[u]);
  for (; r0 < rows; r0 += U * nw) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = r0 + u * nw + sub;
      const bool ok = row < rows;
      float v[NCH][8];
      unpack_row<NCH>(nxt[u], v);
      load_raw<NCH, LPR>(X + (row + U * nw) * F, F, sl, row + U * nw < rows, nxt[u]);
      float mean, rstd;
      if (ext_stats) {  // [rows, 2] = (mean, rstd) computed over the full (TP-gathered) feature set
        mean = ok ? ext_stats[2 * row] : 0.f;
        rstd = ok ? ext_stats[2 * row + 1] : 0.f;
      } else {
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
          for (int j = 0; j < 8; ++j) s += v[c][j];
        mean = row_sum<LPR>(s) / F;
        float q = 0.f;
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int col = c * LPR * 8 + sl * 8 + j;
            const float d = col < F ? v[c][j] - mean : 0.f;
            q += d * d;
          }
        rstd = rsqrtf(row_sum<LPR>(q) / F + eps);
      }
      if (!ok) continue;
      if (rstd_out && sl == 0) *reinterpret_cast<float2*>(rstd_out + 2 * row) = make_float2(mean, rstd);
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = c * LPR * 8 + sl * 8;
        if (col >= F) continue;
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float y0 = (v[c][2 * j] - mean) * rstd, y1 = (v[c][2 * j + 1] - mean) * rstd;
          if (scale) { y0 *= sc[c][2 * j]; y1 *= sc[c][2 * j + 1]; }
          if (shift) { y0 += sh[c][2 * j]; y1 += sh[c][2 * j + 1]; }
          if constexpr (AK != 0) {   // the following activation layer
            y0 = act_fwd(AK > 0 ? AK : act, y0);
            y1 = act_fwd(AK > 0 ? AK : act, y1);
          }
          o[j] = pack_bf16x2(y0, y1);
        }
        if constexpr (NORM_NT & 2) {
          typedef unsigned v4u __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(v4u{o[0], o[1], o[2], o[3]}, reinterpret_cast<v4u*>(Y + row * F + col));
        } else {
          *reinterpret_cast<uint4*>(Y + row * F + col) = make_uint4(o[0], o[1], o[2], o[3]);
        }
      }
    }
  }
}

#define NORM_FWD_PARAMS                                                                                       \
  const bf16_t *__restrict__ X, const float *__restrict__ scale, const float *__restrict__ shift,             \
      bf16_t *__restrict__ Y, float *__restrict__ rstd_out, long long rows, int F, int groups, float eps,     \
      const float *__restrict__ ext_stats, int act
template <int NCH, int LPR>
__global__ __launch_bounds__(NTH) void norm_fwd_kernel(NORM_FWD_PARAMS) {
  norm_fwd_body<NCH, LPR, 0>(X, scale, shift, Y, rstd_out, rows, F, groups, eps, ext_stats, act);
}
template <int NCH, int LPR>
__global__ __launch_bounds__(NTH) void norm_fwd_act_kernel(NORM_FWD_PARAMS) {
  norm_fwd_body<NCH, LPR, -1>(X, scale, shift, Y, rstd_out, rows, F, groups, eps, ext_stats, act);
}
template <int NCH, int LPR>
__global__ __launch_bounds__(NTH) void norm_fwd_gelu_kernel(NORM_FWD_PARAMS) {
  norm_fwd_body<NCH, LPR, ACT_GELU>(X, scale, shift, Y, rstd_out, rows, F, groups, eps, ext_stats, act);
}

// row partial sums for the TP path: out[row] = (sum x, sum x^2) over this rank's slice
__global__ __launch_bounds__(NTH) void norm_partial_kernel(const bf16_t* __restrict__ X, float* __restrict__ out,
                                                           long long rows, int F) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float s = 0.f, q = 0.f;
  for (int col = lane * 2; col < F; col += 128) {
    uint32_t u = *reinterpret_cast<const uint32_t*>(X + row * F + col);
    const float a = bf2f(u & 0xffff), b = bf2f(u >> 16);
    s += a + b;
    q += a * a + b * b;
  }
  s = wave_sum(s);
  q = wave_sum(q);
  if (lane == 0) { out[2 * row] = s; out[2 * row + 1] = q; }
}

// the scale values of chunk c for a backward row: hoisted registers (narrow rows), the LDS copy (wide rows, one
// group) or global memory
template <int NCH, int LPR, bool HOIST>
__device__ __forceinline__ void scale8(int c, int sl, int F, bool ok, long long poff, const float* __restrict__ scale,
                                       bool sc_lds, const float* sc_s, const float (&hsc)[HOIST ? NCH : 1][8],
                                       float (&gsc)[8]) {
  const int col0 = c * LPR * 8 + sl * 8;
  if (HOIST) {
#pragma unroll
    for (int j = 0; j < 8; ++j) gsc[j] = hsc[HOIST ? c : 0][j];
  } else if (sc_lds) {
    if (col0 < F) {
      const float4 a4 = *reinterpret_cast<const float4*>(sc_s + col0);
      const float4 b4 = *reinterpret_cast<const float4*>(sc_s + col0 + 4);
      gsc[0] = a4.x; gsc[1] = a4.y; gsc[2] = a4.z; gsc[3] = a4.w;
      gsc[4] = b4.x; gsc[5] = b4.y; gsc[6] = b4.z; gsc[7] = b4.w;
    }
  } else if (scale && ok && col0 < F) {
    load8f(scale + poff + col0, gsc);
  }
}

// dy of a norm whose output went through a fused activation: dy * act'(z), z = xh * scale + shift recomputed
template <int LPR, int AK, bool HSH>
__device__ __forceinline__ void act_dy8(int c, int sl, int F, bool ok, long long poff, const float* __restrict__ scale,
                                        const float* __restrict__ shift, int act, float mean, float rstd,
                                        const float (&gsc)[8], const float (&hsh)[8], const float (&x)[8],
                                        float (&dy)[8]) {
  const int col0 = c * LPR * 8 + sl * 8;
  float b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (HSH) {
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = hsh[j];
  } else {
    if (shift && ok && col0 < F) load8f(shift + poff + col0, b);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float z = (x[j] - mean) * rstd * (scale ? gsc[j] : 1.f) + b[j];
    dy[j] *= act_grad(AK > 0 ? AK : act, z);
  }
}

// backward. stats = (mean, rstd) per row. If `partial_out` is set, only writes per-row partial
// (sum dxh, sum dxh*xh) for the TP all-reduce and returns (phase 1); with `ext_dsum` (phase 2) uses them.
// Parameter gradients: per-lane register sums; the host sizes the grid so that (rows per grid step) % groups == 0,
// so every lane only ever sees rows of one group (row % groups is fixed along the grid-stride loop).
// Wide rows (NCH >= 8: F > 2048 at 64 lanes per row) run one block per CU with 512 VGPRs: the 8 x NCH parameter-
// gradient sums per lane plus a double-buffered row do not fit the 256 of two blocks per CU. At F = 2048 (NCH 4) two
// blocks per CU fit without spills once the residual gradient is loaded for the current row (not a row ahead) and
// the output pairs are packed with the scalar conversions (pk2 below): 411 us per call at 131072 x 2048 against
// 596 us with one block per CU and 833 us with the ~60 VGPRs the vector-convert pack spilled.
template <int NCH>
constexpr int bwd_blocks_per_cu() { return NCH >= 8 ? 1 : NCH == 1 ? NORM_BWD_BPC1 : 2; }

// two floats -> packed bf16 pair through two scalar conversions: the vector convert (common.h pack_bf16x2) costs
// this kernel ~60 VGPRs of spills at F = 2048 (register allocation around the v_cvt_pk_bf16_f32 pairs)
__device__ __forceinline__ uint32_t pk2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// F32R: the RevNet stream form (fp32 gradient R32 added, dx written in fp32 to DX32 and as its bf16 copy to DX) --
// its own instantiation, so the plain kernel keeps its register budget
// ACTF: the norm's output went through a fused activation (forward Y = act(z), z = xh * scale + shift): dy is taken
// through act'(z) first, z recomputed from the row statistics and the parameters (its own instantiation)
template <int NCH, int LPR, bool F32R, int AK>   // AK: 0 plain, > 0 that fused activation, -1 the runtime `act`
__device__ __forceinline__ void norm_bwd_body(const bf16_t* __restrict__ X, const bf16_t* __restrict__ DY,
                                                       const float* __restrict__ scale, const float* __restrict__ stats,
                                                       bf16_t* __restrict__ DX, float* __restrict__ dscale,
                                                       float* __restrict__ dshift, long long rows, int F, int groups,
                                                       int Ffull, float* __restrict__ partial_out,
                                                       const float* __restrict__ ext_dsum,
                                                       const bf16_t* __restrict__ R, float* __restrict__ ws,
                                                       const float* __restrict__ R32, float* __restrict__ DX32,
                                                       const float* __restrict__ shift, int act, int in_relu) {
  constexpr int RPW = 64 / LPR;
  constexpr bool ACTF = AK != 0;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red_s = reinterpret_cast<float*>(smem);           // [4 waves][F] dscale partials, then dshift
  // wide rows, one parameter group: scale staged once in LDS behind the reduction scratch (row reads by ds_read)
  float* sc_s = red_s + 8 * LPR * 8;
  const bool sc_lds = NCH > 2 && scale != nullptr && groups == 1;
  if (sc_lds) {
    for (int i = threadIdx.x * 4; i < F; i += NTH * 4)
      *reinterpret_cast<float4*>(sc_s + i) = *reinterpret_cast<const float4*>(scale + i);
    __syncthreads();
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, sub = lane / LPR, sl = lane % LPR;
  const bool want_param = (dscale || dshift) && partial_out == nullptr;
  float gs[NCH][8], gb[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) gs[c][j] = gb[c][j] = 0.f;
  const long long nw = (long long)gridDim.x * 4 * RPW;
  const long long first = ((long long)blockIdx.x * 4 + w) * RPW + sub;
  constexpr int U = NCH == 1 ? NORM_BWD_U1 : NCH == 2 ? 2 : 1;   // rows per lane group in flight
  // next rows (x, dy, the residual gradient and the row statistics) in flight while this one is processed
  uint4 nx[U][NCH], nd[U][NCH];
  float2 nst[U];
  const long long rbase = ((long long)blockIdx.x * 4 + w) * RPW + sub;
  // narrow rows: the lane group's scale is loaded once (all its rows are of group rbase % groups)
  constexpr bool HOIST = NCH <= 2;
  float hsc[HOIST ? NCH : 1][8];
  if (HOIST && scale) {
#pragma unroll
    for (int c = 0; c < (HOIST ? NCH : 1); ++c) {
      const int col0 = c * LPR * 8 + sl * 8;
      if (col0 < F) load8f(scale + (long long)(rbase % groups) * F + col0, hsc[c]);
    }
  }
  // the fused activation's shift, hoisted the same way (narrow rows)
  constexpr bool HSH = ACTF && HOIST;
  float hsh[HSH ? NCH : 1][8];
  if constexpr (HSH) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int j = 0; j < 8; ++j) hsh[c][j] = 0.f;
      const int col0 = c * LPR * 8 + sl * 8;
      if (shift && col0 < F) load8f(shift + (long long)(rbase % groups) * F + col0, hsh[c]);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long row = rbase + u * nw, rc = row < rows ? row : rows - 1;
    load_rawc<NCH, LPR>(X + rc * F, F, sl, nx[u]);
    load_rawc<NCH, LPR>(DY + rc * F, F, sl, nd[u]);
    nst[u] = *reinterpret_cast<const float2*>(stats + 2 * rc);
  }
  for (long long r0 = rbase - sub; r0 < rows; r0 += U * nw) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
    const long long row = r0 + u * nw + sub;
    const bool ok = row < rows;
    const long long nrow = row + U * nw, nrc = nrow < rows ? nrow : rows - 1;
    // this row stays packed (bf16) and is unpacked once per pass: the float copies of x and dy held across both
    // passes pushed the kernel to 255 VGPRs, and the register reuse then forced a vmcnt(0) behind every next-row load
    uint4 cx[NCH], cd[NCH], cr[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      cx[c] = nx[u][c];
      cd[c] = nd[u][c];
    }
    // the residual gradient is only read in the second pass: loaded for this row here (its latency hides under the
    // first pass and the row reductions) instead of a row ahead -- 16 fewer live VGPRs at F = 2048, where the
    // parameter-gradient sums already hold 64 (a row-ahead copy spilled ~60 VGPRs and doubled the kernel's time)
    if (R) load_rawc<NCH, LPR>(R + (ok ? row : rows - 1) * F, F, sl, cr);
    load_rawc<NCH, LPR>(X + nrc * F, F, sl, nx[u]);
    load_rawc<NCH, LPR>(DY + nrc * F, F, sl, nd[u]);
    const float mean = ok ? nst[u].x : 0.f, rstd = ok ? nst[u].y : 0.f;
    nst[u] = *reinterpret_cast<const float2*>(stats + 2 * nrc);
    const long long poff = (long long)(row % groups) * F;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      float gsc[8], x[8], dy[8];
      scale8<NCH, LPR, HOIST>(c, sl, F, ok, poff, scale, sc_lds, sc_s, hsc, gsc);
      unpack8(cx[c], x);
      unpack8(cd[c], dy);
      if constexpr (ACTF) {
        if (AK > 0 || act) {
          // dy through act'(z) once: pass 2 reads the product back from cd (bf16, as the separate pass stored it)
          act_dy8<LPR, AK, HSH>(c, sl, F, ok, poff, scale, shift, act, mean, rstd, gsc, hsh[HSH ? c : 0], x, dy);
          cd[c] = make_uint4(pk2(dy[0], dy[1]), pk2(dy[2], dy[3]), pk2(dy[4], dy[5]), pk2(dy[6], dy[7]));
        }
      }
      const int col0 = c * LPR * 8 + sl * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = col0 + j;
        if (ok && col < F) {
          const float xh = (x[j] - mean) * rstd;
          const float g = scale ? gsc[j] : 1.f;
          const float dxh = dy[j] * g;
          s1 += dxh;
          s2 += dxh * xh;
          if (want_param) { gs[c][j] += dy[j] * xh; gb[c][j] += dy[j]; }
        }
      }
    }
    s1 = row_sum<LPR, false>(s1);
    s2 = row_sum<LPR, false>(s2);
    if (!ok) continue;
    if (partial_out) {
      if (sl == 0) { partial_out[2 * row] = s1; partial_out[2 * row + 1] = s2; }
      continue;
    }
    if (ext_dsum) { s1 = ext_dsum[2 * row]; s2 = ext_dsum[2 * row + 1]; }
    const float m1 = s1 / Ffull, m2 = s2 / Ffull;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * LPR * 8 + sl * 8;
      if (col >= F) continue;
      float gsc[8], x[8], dy[8];
      scale8<NCH, LPR, HOIST>(c, sl, F, ok, poff, scale, sc_lds, sc_s, hsc, gsc);
      unpack8(cx[c], x);
      unpack8(cd[c], dy);
      float r[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if constexpr (F32R) {   // the RevNet stream gradient (fp32): dx in fp32 to DX32, its bf16 copy to DX
        const float4 ra = reinterpret_cast<const float4*>(R32 + row * F + col)[0];
        const float4 rb = reinterpret_cast<const float4*>(R32 + row * F + col)[1];
        r[0] = ra.x; r[1] = ra.y; r[2] = ra.z; r[3] = ra.w; r[4] = rb.x; r[5] = rb.y; r[6] = rb.z; r[7] = rb.w;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float g = scale ? gsc[j] : 1.f;
          const float xh = (x[j] - mean) * rstd;
          v[j] = rstd * (dy[j] * g - m1 - xh * m2) + r[j];
        }
        *reinterpret_cast<uint4*>(DX + row * F + col) =
            make_uint4(pk2(v[0], v[1]), pk2(v[2], v[3]), pk2(v[4], v[5]), pk2(v[6], v[7]));
        reinterpret_cast<float4*>(DX32 + row * F + col)[0] = make_float4(v[0], v[1], v[2], v[3]);
        reinterpret_cast<float4*>(DX32 + row * F + col)[1] = make_float4(v[4], v[5], v[6], v[7]);
        continue;
      }
      if (R) unpack8(cr[c], r);   // the block's residual-input gradient, summed here instead of in a separate pass
      uint32_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int j0 = 2 * j, j1 = 2 * j + 1;
        const float g0 = scale ? gsc[j0] : 1.f, g1 = scale ? gsc[j1] : 1.f;
        const float xh0 = (x[j0] - mean) * rstd, xh1 = (x[j1] - mean) * rstd;
        const float d0 = dy[j0] * g0, d1 = dy[j1] * g1;
        float v0 = rstd * (d0 - m1 - xh0 * m2) + r[j0], v1 = rstd * (d1 - m1 - xh1 * m2) + r[j1];
        if constexpr (ACTF) {
          if (in_relu) {   // the norm's input was relu(z): dz = dx * [x > 0] (the producing GEMM skips its pass)
            v0 = x[j0] > 0.f ? v0 : 0.f;
            v1 = x[j1] > 0.f ? v1 : 0.f;
          }
        }
        o[j] = pk2(v0, v1);
      }
      *reinterpret_cast<uint4*>(DX + row * F + col) = make_uint4(o[0], o[1], o[2], o[3]);
    }
    }
  }
  if (want_param && groups > 1) {
    // lane group `first` (its rows are first, first + nw, ... -- all of group first % groups) stores its partial
    // sums as row `first` of the [nw][2F] slab (lane groups without rows store zeros)
    float* wr = ws + first * 2 * F;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * LPR * 8 + sl * 8;
      if (col < F) {
        *reinterpret_cast<float4*>(wr + col) = make_float4(gs[c][0], gs[c][1], gs[c][2], gs[c][3]);
        *reinterpret_cast<float4*>(wr + col + 4) = make_float4(gs[c][4], gs[c][5], gs[c][6], gs[c][7]);
        *reinterpret_cast<float4*>(wr + F + col) = make_float4(gb[c][0], gb[c][1], gb[c][2], gb[c][3]);
        *reinterpret_cast<float4*>(wr + F + col + 4) = make_float4(gb[c][4], gb[c][5], gb[c][6], gb[c][7]);
      }
    }
  }
  if (want_param && groups == 1) {
    // fold the row-groups of the wave, then per chunk reduce the 4 waves through LDS ([2][4][LPR*8] floats) and
    // store the block's partial sums as row blockIdx.x of the [grid][2F] slab
    constexpr int CW = LPR * 8;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = sub_sum<LPR>(gs[c][j]), b = sub_sum<LPR>(gb[c][j]);
        if (sub == 0) { red_s[w * CW + sl * 8 + j] = a; red_s[(4 + w) * CW + sl * 8 + j] = b; }
      }
      __syncthreads();
      for (int k = threadIdx.x; k < CW; k += NTH) {
        const int col = c * CW + k;
        if (col < F) {
          const float a = red_s[k] + red_s[CW + k] + red_s[2 * CW + k] + red_s[3 * CW + k];
          const float b = red_s[4 * CW + k] + red_s[5 * CW + k] + red_s[6 * CW + k] + red_s[7 * CW + k];
          ws[(long long)blockIdx.x * 2 * F + col] = a;
          ws[(long long)blockIdx.x * 2 * F + F + col] = b;
        }
      }
      __syncthreads();
    }
  }
}

#define NORM_BWD_PARAMS                                                                                          \
  const bf16_t *__restrict__ X, const bf16_t *__restrict__ DY, const float *__restrict__ scale,                \
      const float *__restrict__ stats, bf16_t *__restrict__ DX, float *__restrict__ dscale,                    \
      float *__restrict__ dshift, long long rows, int F, int groups, int Ffull, float *__restrict__ partial_out, \
      const float *__restrict__ ext_dsum, const bf16_t *__restrict__ R, float *__restrict__ ws,               \
      const float *__restrict__ R32, float *__restrict__ DX32, const float *__restrict__ shift, int act, int in_relu
#define NORM_BWD_ARGS \
  X, DY, scale, stats, DX, dscale, dshift, rows, F, groups, Ffull, partial_out, ext_dsum, R, ws, R32, DX32, shift, act, \
      in_relu

template <int NCH, int LPR>
__global__ __launch_bounds__(NTH, bwd_blocks_per_cu<NCH>()) void norm_bwd_kernel(NORM_BWD_PARAMS) {
  norm_bwd_body<NCH, LPR, false, 0>(NORM_BWD_ARGS);
}

template <int NCH, int LPR>
__global__ __launch_bounds__(NTH, bwd_blocks_per_cu<NCH>()) void norm_bwd32_kernel(NORM_BWD_PARAMS) {
  norm_bwd_body<NCH, LPR, true, 0>(NORM_BWD_ARGS);
}

template <int NCH, int LPR>
__global__ __launch_bounds__(NTH, bwd_blocks_per_cu<NCH>()) void norm_bwd_act_kernel(NORM_BWD_PARAMS) {
  norm_bwd_body<NCH, LPR, false, -1>(NORM_BWD_ARGS);
}

template <int NCH, int LPR>
__global__ __launch_bounds__(NTH, bwd_blocks_per_cu<NCH>()) void norm_bwd_gelu_kernel(NORM_BWD_PARAMS) {
  norm_bwd_body<NCH, LPR, false, ACT_GELU>(NORM_BWD_ARGS);
}

// One-chunk rows (F <= 8 x LPR: ctx32_mixer's 256-wide head groups and 512-wide bottleneck groups), the plain, bf16
// residual, fused-activation and input-relu forms of the backward without the TP / fp32-stream paths: each lane holds
// 8 columns of one row; the next row's x, dy and statistics are in flight while this one is processed, the residual
// gradient is loaded for this row ahead of the first pass. The general body held 100-130 VGPRs at one chunk (64-bit
// address pairs of its generic paths): two waves per SIMD, too few to cover the gelu form's VALU and the loads (3.4
// TB/s). This one fits four blocks per CU. Parameter gradients: per-lane-group partial slabs (row `first` of a [lane
// groups][2F] slab, every group count, groups == 1 too), folded in order by norm_fold_kernel.
// AK: 0 plain, ACT_GELU, -1 the runtime `act`
template <int LPR, int AK>
__global__ __launch_bounds__(NTH, NORM_BWD1_BPC) void norm_bwd1_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ DY, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ stats, bf16_t* __restrict__ DX,
    const bf16_t* __restrict__ R, float* __restrict__ ws, long long rows, int F, int groups, int act, int in_relu) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, sub = lane / LPR, sl = lane % LPR;
  const int col = sl * 8;
  const bool colok = col < F;
  const int ccol = colok ? col : 0;   // lanes past F re-read column 0 (their values are never used)
  const long long nw = (long long)gridDim.x * 4 * RPW;
  const long long first = ((long long)blockIdx.x * 4 + w) * RPW + sub;
  const long long poff = (first % groups) * F + ccol;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = 1.f; sh[j] = 0.f; }
  if (scale) load8f(scale + poff, sc);
  if (AK != 0 && shift) load8f(shift + poff, sh);
  float gs[8], gb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) gs[j] = gb[j] = 0.f;
  const float inv_f = 1.f / (float)F;
  long long row = first;
  long long rc = row < rows ? row : rows - 1;
  uint4 nx = *reinterpret_cast<const uint4*>(X + rc * F + ccol);
  uint4 nd = *reinterpret_cast<const uint4*>(DY + rc * F + ccol);
  float2 nst = *reinterpret_cast<const float2*>(stats + 2 * rc);
#pragma nounroll
  for (; row < rows; row += nw) {
    const uint4 cx = nx, cd = nd;
    const float mean = nst.x, rstd = nst.y;
    uint4 cr = make_uint4(0u, 0u, 0u, 0u);
    if (R) cr = *reinterpret_cast<const uint4*>(R + row * F + ccol);
    const long long nrow = row + nw, nrc = nrow < rows ? nrow : rows - 1;
    nx = *reinterpret_cast<const uint4*>(X + nrc * F + ccol);
    nd = *reinterpret_cast<const uint4*>(DY + nrc * F + ccol);
    nst = *reinterpret_cast<const float2*>(stats + 2 * nrc);
    float x[8], dy[8], xh[8];
    unpack8(cx, x);
    unpack8(cd, dy);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xh[j] = (x[j] - mean) * rstd;
      if constexpr (AK != 0) {
        if (AK > 0 || act) dy[j] *= act_grad(AK > 0 ? AK : act, __builtin_fmaf(xh[j], sc[j], sh[j]));
      }
      const float dxh = dy[j] * sc[j];
      s1 += dxh;
      s2 += dxh * xh[j];
      gs[j] += dy[j] * xh[j];
      gb[j] += dy[j];
    }
    if (!colok) s1 = s2 = 0.f;
    // (the activation forms keep the ds_bpermute steps: DPP measured 2-5 % slower there, 3-7 % faster elsewhere)
    s1 = row_sum<LPR, NORM_DPP != 0 && AK == 0>(s1) * inv_f;
    s2 = row_sum<LPR, NORM_DPP != 0 && AK == 0>(s2) * inv_f;
    float r[8];
    unpack8(cr, r);
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int j0 = 2 * j, j1 = 2 * j + 1;
      float v0 = rstd * (dy[j0] * sc[j0] - s1 - xh[j0] * s2) + r[j0];
      float v1 = rstd * (dy[j1] * sc[j1] - s1 - xh[j1] * s2) + r[j1];
      if (AK != 0 && in_relu) {   // the norm's input was relu(z): dz = dx * [x > 0]
        v0 = x[j0] > 0.f ? v0 : 0.f;
        v1 = x[j1] > 0.f ? v1 : 0.f;
      }
      o[j] = pk2(v0, v1);
    }
    if (colok) *reinterpret_cast<uint4*>(DX + row * F + col) = make_uint4(o[0], o[1], o[2], o[3]);
  }
  if (ws && colok) {
    // lanes of groups past the last row hold zeros; a lane group that saw a row past `rows` summed nothing for it
    // (its loop exited), so every slab row is exactly its lane group's sum
    float* wr = ws + first * 2 * F;
    *reinterpret_cast<float4*>(wr + col) = make_float4(gs[0], gs[1], gs[2], gs[3]);
    *reinterpret_cast<float4*>(wr + col + 4) = make_float4(gs[4], gs[5], gs[6], gs[7]);
    *reinterpret_cast<float4*>(wr + F + col) = make_float4(gb[0], gb[1], gb[2], gb[3]);
    *reinterpret_cast<float4*>(wr + F + col + 4) = make_float4(gb[4], gb[5], gb[6], gb[7]);
  }
}

// deterministic fold of the parameter-gradient slab: out[g][f] += sum over partial rows p = g, g + period, ... (in
// order) of ws[p][which * F + f] for the scale (which 0) and shift (which 1) halves. Block = 32 output columns x 8
// segments of the partial rows; the 8 segment sums are added in segment order.
__global__ __launch_bounds__(NTH) void norm_fold_kernel(const float* __restrict__ ws, long long nparts, int period,
                                                        int F, int groups, float* __restrict__ dscale,
                                                        float* __restrict__ dshift) {
  __shared__ float red[8][32];
  const int c = threadIdx.x & 31, seg = threadIdx.x >> 5;
  const long long o = (long long)blockIdx.x * 32 + c;
  const long long nout = 2LL * groups * F;
  float acc = 0.f;
  int which = 0, g = 0, f = 0;
  if (o < nout) {
    which = (int)(o / ((long long)groups * F));
    const int rem = (int)(o % ((long long)groups * F));
    g = rem / F;
    f = rem % F;
    const long long K = nparts > g ? (nparts - g + period - 1) / period : 0;   // partial rows of this group
    const long long k0 = K * seg / 8, k1 = K * (seg + 1) / 8;
    const float* src = ws + (long long)which * F + f + (long long)g * 2 * F;
    const long long step = (long long)period * 2 * F;
    long long k = k0;
    for (; k + 4 <= k1; k += 4) {   // four loads in flight, added in k order
      const float v0 = src[k * step], v1 = src[(k + 1) * step], v2 = src[(k + 2) * step], v3 = src[(k + 3) * step];
      acc += v0;
      acc += v1;
      acc += v2;
      acc += v3;
    }
    for (; k < k1; ++k) acc += src[k * step];
  }
  red[seg][c] = acc;
  __syncthreads();
  if (seg == 0 && o < nout) {
    float s = red[0][c];
#pragma unroll
    for (int i = 1; i < 8; ++i) s += red[i][c];
    float* dst = which ? dshift : dscale;
    if (dst) dst[(long long)g * F + f] += s;
  }
}

}  // namespace

struct ObstNormDesc {
  const void* X; const float* scale; const float* shift; void* Y; float* stats;
  const void* DY; void* DX; float* dscale; float* dshift;
  float* partial; const float* ext;   // TP path
  long long rows; int F; int groups; int Ffull; float eps;
  const void* R;                      // backward: gradient added to DX (residual input of the block) or null
  float* ws;                          // backward with parameter gradients: obst_norm_bwd_ws(desc) floats
  const float* R32;                   // backward: fp32 gradient added to DX (the RevNet stream gradient) or null
  float* DX32;                        // backward with R32: DX in fp32 (DX then holds its bf16 copy)
  int act;                            // a following activation fused: forward Y = act(norm), backward dy *= act'(z)
  int in_relu;                        // backward: the input was relu(z) of the producing GEMM, dx *= [x > 0]
};

#define NORM_DISPATCH_L(KERNEL, LPR, GRID, LDSB, ...)                                               \
  do {                                                                                              \
    const int nch = (d->F + LPR * 8 - 1) / (LPR * 8);                                               \
    if (nch <= 1) hipLaunchKernelGGL((KERNEL<1, LPR>), GRID, dim3(NTH), LDSB, st, __VA_ARGS__);     \
    else if (nch <= 2) hipLaunchKernelGGL((KERNEL<2, LPR>), GRID, dim3(NTH), LDSB, st, __VA_ARGS__);\
    else if (nch <= 4) hipLaunchKernelGGL((KERNEL<4, LPR>), GRID, dim3(NTH), LDSB, st, __VA_ARGS__);\
    else if (nch <= 8) hipLaunchKernelGGL((KERNEL<8, LPR>), GRID, dim3(NTH), LDSB, st, __VA_ARGS__);\
    else if (nch <= 16) hipLaunchKernelGGL((KERNEL<16, LPR>), GRID, dim3(NTH), LDSB, st, __VA_ARGS__);\
    else return -2;                                                                                 \
  } while (0)

static int lanes_per_row(int F) { return F <= 64 ? 8 : F <= 128 ? 16 : F <= 256 ? 32 : 64; }

// the forward's lanes per row: NORM_FWD_NARROW halves them for 128 < F <= 512 (two 16-byte chunks per lane and row)
#ifndef NORM_FWD_NARROW
#define NORM_FWD_NARROW 0
#endif
static int fwd_lanes_per_row(int F) {
  return (NORM_FWD_NARROW && F > 128 && F <= 512) ? lanes_per_row(F) / 2 : lanes_per_row(F);
}

#define NORM_DISPATCH(KERNEL, GRID, LDSB, ...) NORM_DISPATCH_F(lanes_per_row, KERNEL, GRID, LDSB, __VA_ARGS__)
#define NORM_DISPATCH_F(LPRF, KERNEL, GRID, LDSB, ...)                                              \
  do {                                                                                              \
    switch (LPRF(d->F)) {                                                                           \
      case 8: NORM_DISPATCH_L(KERNEL, 8, GRID, LDSB, __VA_ARGS__); break;                           \
      case 16: NORM_DISPATCH_L(KERNEL, 16, GRID, LDSB, __VA_ARGS__); break;                         \
      case 32: NORM_DISPATCH_L(KERNEL, 32, GRID, LDSB, __VA_ARGS__); break;                         \
      default: NORM_DISPATCH_L(KERNEL, 64, GRID, LDSB, __VA_ARGS__); break;                         \
    }                                                                                               \
  } while (0)

static int group_aligned(int grid, int groups, int F, int lpr) {
  // rows per grid step (4 waves x 64/LPR rows per block) must be a multiple of groups
  if (groups <= 1) return grid;
  int a = groups, b = 4 * (64 / lpr);
  while (b) { const int t = a % b; a = b; b = t; }
  const int q = groups / a;                 // blocks per group period
  return grid < q ? q : grid / q * q;
}

// The forward's grid (NORM_FWD_RESIDENT): one resident wave of blocks (the occupancy of that instantiation x the CUs)
// or the fixed 2048 blocks, grid-striding over the rows.
static int resident_blocks(const void* fn) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> cache;
  static int ncu = 0;
  std::lock_guard<std::mutex> lk(mu);
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || ncu <= 0)
      ncu = 256;
  }
  auto it = cache.find(fn);
  if (it != cache.end()) return it->second;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, NTH, 0) != hipSuccess || per_cu <= 0) per_cu = 8;
  return cache[fn] = per_cu * ncu;
}

template <int LPR, typename K>
static void fwd_launch(K kern, const ObstNormDesc* d, hipStream_t st) {
  const long long need = (d->rows + 4 * (64 / LPR) - 1) / (4 * (64 / LPR));
  const int cap = NORM_FWD_RESIDENT ? resident_blocks(reinterpret_cast<const void*>(kern)) : 2048;
  const int grid = group_aligned((int)(need < cap ? need : cap), d->groups, d->F, LPR);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NTH), 0, st, (const bf16_t*)d->X, d->scale, d->shift, (bf16_t*)d->Y,
                     d->stats, d->rows, d->F, d->groups, d->eps, d->ext, d->act);
}

#define NORM_FWD_L(KERNEL, LPR)                                                         \
  do {                                                                                  \
    const int nch = (d->F + LPR * 8 - 1) / (LPR * 8);                                   \
    if (nch <= 1) fwd_launch<LPR>(KERNEL<1, LPR>, d, st);                               \
    else if (nch <= 2) fwd_launch<LPR>(KERNEL<2, LPR>, d, st);                          \
    else if (nch <= 4) fwd_launch<LPR>(KERNEL<4, LPR>, d, st);                          \
    else if (nch <= 8) fwd_launch<LPR>(KERNEL<8, LPR>, d, st);                          \
    else if (nch <= 16) fwd_launch<LPR>(KERNEL<16, LPR>, d, st);                        \
    else return -2;                                                                     \
  } while (0)
#define NORM_FWD_DISPATCH(KERNEL)                                                       \
  do {                                                                                  \
    switch (fwd_lanes_per_row(d->F)) {                                                  \
      case 8: NORM_FWD_L(KERNEL, 8); break;                                             \
      case 16: NORM_FWD_L(KERNEL, 16); break;                                           \
      case 32: NORM_FWD_L(KERNEL, 32); break;                                           \
      default: NORM_FWD_L(KERNEL, 64); break;                                           \
    }                                                                                   \
  } while (0)

OBST_API int obst_norm_fwd(const ObstNormDesc* d, hipStream_t st) {
  if (d->F % 8 || d->rows <= 0) return -1;
  if (d->act == ACT_GELU) NORM_FWD_DISPATCH(norm_fwd_gelu_kernel);
  else if (d->act) NORM_FWD_DISPATCH(norm_fwd_act_kernel);
  else NORM_FWD_DISPATCH(norm_fwd_kernel);
  return (int)hipGetLastError();
}

OBST_API int obst_norm_partial(const ObstNormDesc* d, hipStream_t st) {
  if (d->F % 2 || d->rows <= 0) return -1;
  hipLaunchKernelGGL(norm_partial_kernel, dim3((unsigned)((d->rows + 3) / 4)), dim3(NTH), 0, st, (const bf16_t*)d->X,
                     d->partial, d->rows, d->F);
  return (int)hipGetLastError();
}

// the one-chunk backward serves the row (F <= 8 x lanes per row), plain / bf16-residual / activation forms
static bool norm_bwd_one_chunk(const ObstNormDesc* d) {
  return NORM_BWD1_BPC > 0 && d->F <= 8 * lanes_per_row(d->F) && !d->partial && !d->ext && !d->R32 && !d->DX32;
}

static int norm_bwd_grid(const ObstNormDesc* d) {
  // one resident wave of blocks (2 blocks of 4 waves per CU; wide rows: 1, bwd_blocks_per_cu; the one-chunk kernel:
  // NORM_BWD1_BPC) grid-strides over the rows; more blocks only grow the parameter-gradient slab that
  // norm_fold_kernel reads back (2048 blocks: 103 us)
  const int lpr = lanes_per_row(d->F);
  const int nch = (d->F + lpr * 8 - 1) / (lpr * 8);
  const int cap = norm_bwd_one_chunk(d) ? 256 * (NORM_BWD1_BPC > 0 ? NORM_BWD1_BPC : 1)
                  : nch > 4 ? 256 : nch == 1 ? 256 * NORM_BWD_BPC1 : 512;
  long long g = (d->rows + 15) / 16;
  int grid = (int)(g < cap ? (g < 1 ? 1 : g) : cap);
  if (d->groups > 1) {   // rows per grid step (4 waves x 64/LPR rows per block) must be a multiple of groups
    int a = d->groups, b = 4 * (64 / lanes_per_row(d->F));
    while (b) { const int t = a % b; a = b; b = t; }
    const int q = d->groups / a;                 // blocks per group period
    grid = grid < q ? q : grid / q * q;
  }
  return grid;
}

static bool norm_bwd_params(const ObstNormDesc* d) { return (d->dscale || d->dshift) && !d->partial; }

// rows of the parameter-gradient slab: one per lane group (grouped rows, and every one-chunk launch), else one per
// block
static long long norm_bwd_parts(const ObstNormDesc* d) {
  const long long grid = norm_bwd_grid(d);
  return (d->groups > 1 || norm_bwd_one_chunk(d)) ? grid * 4 * (64 / lanes_per_row(d->F)) : grid;
}

// floats of the parameter-gradient slab obst_norm_bwd needs in desc->ws (0: no parameter gradients)
OBST_API long long obst_norm_bwd_ws(const ObstNormDesc* d) {
  if (!norm_bwd_params(d) || d->F <= 0 || d->rows <= 0) return 0;
  return norm_bwd_parts(d) * 2 * d->F;
}

OBST_API int obst_norm_bwd(const ObstNormDesc* d, hipStream_t st) {
  if (d->F % 8 || d->rows <= 0) return -1;
  if ((d->R && d->R32) || (d->DX32 && !d->R32) || ((d->act || d->in_relu) && d->R32)) return -4;
  const bool params = norm_bwd_params(d);
  if (params && !d->ws) return -3;
  // reduction scratch [8][LPR*8] floats (<= 16 KiB), plus the staged scale ([F] floats) for wide rows
  const int nch = (d->F + lanes_per_row(d->F) * 8 - 1) / (lanes_per_row(d->F) * 8);
  const size_t lds = (size_t)8 * lanes_per_row(d->F) * 8 * 4 + (nch > 2 && d->scale && d->groups == 1 ? d->F * 4 : 0);
  const int grid = norm_bwd_grid(d);
#define NORM_BWD_LAUNCH(KERNEL)                                                                                  \
  NORM_DISPATCH(KERNEL, dim3(grid), lds, (const bf16_t*)d->X, (const bf16_t*)d->DY, d->scale, d->stats,           \
                (bf16_t*)d->DX, d->dscale, d->dshift, d->rows, d->F, d->groups, d->Ffull, d->partial, d->ext,   \
                (const bf16_t*)d->R, d->ws, d->R32, d->DX32, d->shift, d->act, d->in_relu)
  if (norm_bwd_one_chunk(d)) {
#define NORM_BWD1_LAUNCH(AK)                                                                                     \
  do {                                                                                                          \
    const dim3 gr(grid), bl(NTH);                                                                               \
    float* ws = params ? d->ws : nullptr;                                                                       \
    switch (lanes_per_row(d->F)) {                                                                              \
      case 8: hipLaunchKernelGGL((norm_bwd1_kernel<8, AK>), gr, bl, 0, st, NORM_BWD1_ARGS); break;             \
      case 16: hipLaunchKernelGGL((norm_bwd1_kernel<16, AK>), gr, bl, 0, st, NORM_BWD1_ARGS); break;           \
      case 32: hipLaunchKernelGGL((norm_bwd1_kernel<32, AK>), gr, bl, 0, st, NORM_BWD1_ARGS); break;           \
      default: hipLaunchKernelGGL((norm_bwd1_kernel<64, AK>), gr, bl, 0, st, NORM_BWD1_ARGS); break;           \
    }                                                                                                           \
  } while (0)
#define NORM_BWD1_ARGS                                                                                           \
  (const bf16_t*)d->X, (const bf16_t*)d->DY, d->scale, d->shift, d->stats, (bf16_t*)d->DX, (const bf16_t*)d->R, \
      ws, d->rows, d->F, d->groups, d->act, d->in_relu
    if (d->act == ACT_GELU) NORM_BWD1_LAUNCH(ACT_GELU);
    else if (d->act || d->in_relu) NORM_BWD1_LAUNCH(-1);
    else NORM_BWD1_LAUNCH(0);
#undef NORM_BWD1_LAUNCH
#undef NORM_BWD1_ARGS
  } else if (d->R32) NORM_BWD_LAUNCH(norm_bwd32_kernel);
  else if (d->act == ACT_GELU) NORM_BWD_LAUNCH(norm_bwd_gelu_kernel);
  else if (d->act || d->in_relu) NORM_BWD_LAUNCH(norm_bwd_act_kernel);
  else NORM_BWD_LAUNCH(norm_bwd_kernel);
#undef NORM_BWD_LAUNCH
  if (params) {
    const long long parts = norm_bwd_parts(d);
    const long long nout = 2LL * d->groups * d->F;
    // a lane group's rows are p, p + nw, ... so partial row p belongs to group p % groups (nw % groups == 0)
    hipLaunchKernelGGL(norm_fold_kernel, dim3((unsigned)((nout + 31) / 32)), dim3(NTH), 0, st, d->ws, parts,
                       d->groups > 1 ? d->groups : 1, d->F, d->groups, d->dscale, d->dshift);
  }
  return (int)hipGetLastError();
}
