// K04 variants: the reference's dot-product attention with learned per-head maps (src/model/spatial.py:54-81)
// that the main flash kernels (attention.hip) do not take -- an additive map on the logits before the softmax
// ('biased_softmax'), a multiplicative map on the probabilities after it ('scale_attention_map'), or both -- on
// token-major [B, S, H, D] q / k / v, without any [B, H, S, S] tensor:
//
//   s_qk = scale q.k + b_qk (keys <= query when causal),  m_q / l_q its running max / exp-sum,
//   o_q  = sum_k c_qk e^{s_qk - m_q} v_k / l_q,   lse_q = m_q + log l_q          (c = 1 without a scale map)
//
// Backward (P_qk = e^{s_qk - lse_q}; delta_q = do_q . o_q = sum_k P_qk c_qk (do_q . v_k)):
//   dv_k = sum_q P_qk c_qk do_q,  dP_qk = do_q . v_k,  ds_qk = P_qk (c_qk dP_qk - delta_q),
//   dq = scale sum_k ds_qk k_k,  dk = scale sum_q ds_qk q_q,  db = sum_batch ds,  dc = sum_batch P dP.
//
// Kernels: forward and dq (+ delta) per (64-query block, head, batch); dk/dv per (64-key block, head, batch
// slice) walking its batches and query blocks in a fixed order, so the map gradients (sums over the batch)
// accumulate in place by plain read-modify-write of the workgroup's own key columns -- no atomics; batch slices
// > 1 write separate partial maps that map_fold_kernel sums in slice order (deterministic).
//
// MFMA layout (v_mfma_f32_16x16x32_bf16; C: lane holds column lane & 15, rows 4 (lane >> 4) + r): the query-major
// kernels compute the score tile transposed (rows = keys, columns = queries), so each lane owns one query and the
// softmax statistics are lane-local (two xor-shuffles across the 4 lane groups). The probability registers feed the
// next MFMA's B operand directly under a permuted contraction order -- slots 0-3 = rows 4g..4g+3 of one 16-row
// tile, slots 4-7 = the same rows of the next -- and the matching A operand is read from the same row-major LDS
// image by the CDNA4 transposing read ds_read_b64_tr_b16 with that permutation (frag_tr): every tile is staged
// once, row-major. The key-major dk/dv kernel does the same with queries and keys swapped.
#include "common.h"

#include <stdlib.h>

namespace {

constexpr int TQ = 64;    // queries per workgroup (16 per wave)
constexpr int TK = 64;    // keys per tile
constexpr int PADR = 8;   // row pad of the row-major images [64][D + PADR] (16-B fragment reads conflict-free)

struct MapArgs {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  const bf16_t* o;
  const bf16_t* dO;
  bf16_t* out;
  bf16_t* dq;
  bf16_t* dk;
  bf16_t* dv;
  const float* bias;   // [H][S][S] or null
  const float* cmap;   // [H][S][S] or null
  float* dbias;        // [bsplit][H][S][S] (zero-initialised) or null
  float* dcmap;
  float* lse;          // [B][H][S]
  float* delta;
  int B, S, H, bsplit;
  float scale;
  int causal;
};

__device__ __forceinline__ uint4 ld16(const bf16_t* p, bool ok) {
  return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0u, 0u, 0u, 0u);
}

// register staging of one 64-row tile (D / 32 16-byte pieces per thread): the next tile's global loads are issued
// before the current tile's MFMAs and written to LDS behind the next barrier, so their latency hides under compute
template <int D>
struct Rows {
  uint4 v[D / 32];
};
template <int D>
__device__ __forceinline__ void load_rows(Rows<D>& r, const bf16_t* g, long long ld, int r0, int S, int tid) {
  constexpr int CH = D / 8;
#pragma unroll
  for (int i = 0; i < D / 32; ++i) {
    const int c = tid + 256 * i, row = c / CH, cc = c - row * CH;
    r.v[i] = ld16(g + (long long)(r0 + row) * ld + cc * 8, r0 + row < S);
  }
}
// full tiles (r0 + 64 <= S): the per-thread 32-bit offsets of its D / 32 pieces, computed once, on a uniform tile
// base (global_load with an SGPR base and a VGPR offset: no 64-bit address VALU and no exec-masked branch per load)
template <int D>
__device__ __forceinline__ void row_offsets(int (&off)[D / 32], int ld, int tid) {
  constexpr int CH = D / 8;
#pragma unroll
  for (int i = 0; i < D / 32; ++i) {
    const int c = tid + 256 * i, row = c / CH, cc = c - row * CH;
    off[i] = row * ld + cc * 8;
  }
}
template <int D>
__device__ __forceinline__ void load_tile(Rows<D>& r, const bf16_t* g, long long ld, int r0, int S, int tid,
                                          const int (&off)[D / 32]) {
  if (r0 + 64 <= S) {
    const bf16_t* gt = g + (long long)r0 * ld;
#pragma unroll
    for (int i = 0; i < D / 32; ++i) r.v[i] = *reinterpret_cast<const uint4*>(gt + off[i]);
  } else {
    load_rows<D>(r, g, ld, r0, S, tid);
  }
}
template <int D>
__device__ __forceinline__ void store_rows(bf16_t* img, const Rows<D>& r, int tid) {
  constexpr int CH = D / 8;
#pragma unroll
  for (int i = 0; i < D / 32; ++i) {
    const int c = tid + 256 * i, row = c / CH, cc = c - row * CH;
    *reinterpret_cast<uint4*>(img + row * (D + PADR) + cc * 8) = r.v[i];
  }
}

// map values of keys key0 .. key0 + 3 on one query row (16-byte load when in range; zero past S)
// (per-lane conditions: the compiler emits exec-masked branches around each load -- callers take map4_full, one
// plain 16-byte load, on full tiles of a row length divisible by 4, a uniform condition)
__device__ __forceinline__ f32x4_t map4_full(const float* row, int key0) {
  return *reinterpret_cast<const f32x4_t*>(row + key0);
}
__device__ __forceinline__ f32x4_t map4(const float* row, int key0, int S) {
  if ((S & 3) == 0 && key0 + 3 < S) return *reinterpret_cast<const f32x4_t*>(row + key0);
  f32x4_t v;
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = key0 + r < S ? row[key0 + r] : 0.f;
  return v;
}

// operand of 16 rows (rb + lane & 15) x 32 contraction elements (kk * 32 + 8 g ..) from a row-major image
template <int RS>
__device__ __forceinline__ bf16x8_t frag_rm(const bf16_t* img, int rb, int kk, int lane) {
  return *reinterpret_cast<const bf16x8_t*>(img + (rb + (lane & 15)) * RS + kk * 32 + 8 * (lane >> 4));
}
// A operand [m = mb + (lane & 15)][k slots of chunk c] from a ROW-MAJOR image [k][m] (row stride RS elements) by
// the transposing read: per 16-lane group, lane 4q+p addresses row q of a 4-row block at columns 4p..4p+3 and lane i
// receives column i of the 4 rows (cdna guide T10). Slots 0-3 = rows 32c + 4g .. +3, slots 4-7 = rows 32c + 16 + 4g ..
// (g = lane >> 4): the permutation frag_acc gives the matching B operand. Called with EXEC all ones only.
template <int RS>
__device__ __forceinline__ bf16x8_t frag_tr(const bf16_t* img, int mb, int c, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const bf16_t* p0 = img + (32 * c + 4 * g + (i >> 2)) * RS + mb + 4 * (i & 3);
  const s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, p0));
  const s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, p0 + 16 * RS));
  const s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}
// B operand from two accumulator tiles in C layout (same slot permutation as frag_tr)
__device__ __forceinline__ bf16x8_t frag_acc(const f32x4_t& t0, const f32x4_t& t1) {
  return __builtin_bit_cast(bf16x8_t, make_uint4(pack_bf16x2(t0[0], t0[1]), pack_bf16x2(t0[2], t0[3]),
                                                 pack_bf16x2(t1[0], t1[1]), pack_bf16x2(t1[2], t1[3])));
}
__device__ __forceinline__ f32x4_t mfma(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------------------------------------------
// HB / HC: a bias / scale map is present (separate instantiations: a runtime-null map load in a branch made the
// compiler's wait at its use a vmcnt(0), which also waited for the next tile's K / V prefetch -- every tile paid a
// full memory round trip, with or without a map). The next tile's map values are prefetched with its K / V rows.
template <int D, bool HB, bool HC>
__global__ __launch_bounds__(256) void attn_map_fwd_kernel(MapArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t kimg[64 * (D + PADR)];
  __shared__ __attribute__((aligned(16))) bf16_t vimg[64 * (D + PADR)];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int S = a.S, nqb = (S + TQ - 1) / TQ;
  const int qb = nqb - 1 - (int)blockIdx.x;   // longest causal rows first
  const int h = blockIdx.y, b = blockIdx.z;
  const long long ld = (long long)a.H * D;
  const long long base = (long long)b * S * ld + (long long)h * D;
  const int myq = qb * TQ + w * 16 + (lane & 15);
  const bool qok = myq < S;
  bf16x8_t qf[D / 32];
#pragma unroll
  for (int kk = 0; kk < D / 32; ++kk)
    qf[kk] = __builtin_bit_cast(bf16x8_t, ld16(a.q + base + (long long)myq * ld + kk * 32 + 8 * g, qok));
  f32x4_t acc[D / 16];
#pragma unroll
  for (int i = 0; i < D / 16; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const long long mrow = ((long long)h * S + (qok ? myq : 0)) * S;
  float m = -INFINITY, l = 0.f;
  const int nkt = a.causal ? qb + 1 : (S + TK - 1) / TK;
  Rows<D> nk, nv;
  int roff[D / 32];
  row_offsets<D>(roff, (int)ld, tid);
  f32x4_t nb[4], nc[4];
  auto fetch = [&](int k0) {
    if ((S & 3) == 0 && k0 + TK <= S) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        if constexpr (HB) nb[kb] = map4_full(a.bias + mrow, k0 + kb * 16 + 4 * g);
        if constexpr (HC) nc[kb] = map4_full(a.cmap + mrow, k0 + kb * 16 + 4 * g);
      }
    } else {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        if constexpr (HB) nb[kb] = map4(a.bias + mrow, k0 + kb * 16 + 4 * g, S);
        if constexpr (HC) nc[kb] = map4(a.cmap + mrow, k0 + kb * 16 + 4 * g, S);
      }
    }
    load_tile<D>(nk, a.k + base, ld, k0, S, tid, roff);
    load_tile<D>(nv, a.v + base, ld, k0, S, tid, roff);
  };
  fetch(0);
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * TK;
    __syncthreads();
    store_rows<D>(kimg, nk, tid);
    store_rows<D>(vimg, nv, tid);
    f32x4_t bv[4], cv[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      if constexpr (HB) bv[kb] = nb[kb];
      if constexpr (HC) cv[kb] = nc[kb];
    }
    __syncthreads();
    if (kt + 1 < nkt) fetch(k0 + TK);
    f32x4_t s[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s[kb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < D / 32; ++kk) s[kb] = mfma(frag_rm<D + PADR>(kimg, kb * 16, kk, lane), qf[kk], s[kb]);
    }
    // masks only on the diagonal tile and the tile past S (uniform branch)
    const bool edge = (a.causal && kt == nkt - 1) || k0 + TK > S;
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = s[kb][r] * a.scale;
        if constexpr (HB) x += bv[kb][r];
        s[kb][r] = x;
      }
    if (edge) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + kb * 16 + 4 * g + r;
          if (!(key < S && (!a.causal || key <= myq))) s[kb][r] = -INFINITY;
        }
    }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[kb][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);   // finite: key k0 <= every query of a visited tile
    const float al = __expf(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf(s[kb][r] - mn);
        rs += p;
        s[kb][r] = HC ? p * cv[kb][r] : p;
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l = l * al + rs;
    // the output rescale only when some lane's max moved (exact; after the first tiles it rarely does): the
    // accumulators live in AGPRs, and every rescale moved all of them through VGPRs and back
    if (__any(mn > m)) {
#pragma unroll
      for (int i = 0; i < D / 16; ++i) acc[i] *= al;
    }
    m = mn;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const bf16x8_t pb = frag_acc(s[2 * c], s[2 * c + 1]);
#pragma unroll
      for (int i = 0; i < D / 16; ++i) acc[i] = mfma(frag_tr<D + PADR>(vimg, i * 16, c, lane), pb, acc[i]);
    }
  }
  if (qok) {
    const float inv = 1.f / l;
    bf16_t* orow = a.out + base + (long long)myq * ld + 4 * g;
#pragma unroll
    for (int i = 0; i < D / 16; ++i)
      *reinterpret_cast<uint2*>(orow + i * 16) =
          make_uint2(pack_bf16x2(acc[i][0] * inv, acc[i][1] * inv), pack_bf16x2(acc[i][2] * inv, acc[i][3] * inv));
    if (g == 0) a.lse[((long long)b * a.H + h) * S + myq] = m + __logf(l);
  }
}

// ------------------------------------------------------------------------------------------------------------------
// dq per (query block, head, batch); writes delta_q = do_q . o_q first (the dk/dv kernel reads it)
template <int D, bool HB, bool HC>
__global__ __launch_bounds__(256) void attn_map_dq_kernel(MapArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t kimg[64 * (D + PADR)];
  __shared__ __attribute__((aligned(16))) bf16_t vimg[64 * (D + PADR)];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int S = a.S, nqb = (S + TQ - 1) / TQ;
  const int qb = nqb - 1 - (int)blockIdx.x;
  const int h = blockIdx.y, b = blockIdx.z;
  const long long ld = (long long)a.H * D;
  const long long base = (long long)b * S * ld + (long long)h * D;
  const int myq = qb * TQ + w * 16 + (lane & 15);
  const bool qok = myq < S;
  bf16x8_t qf[D / 32], df[D / 32];
  float dl = 0.f;
#pragma unroll
  for (int kk = 0; kk < D / 32; ++kk) {
    const long long off = base + (long long)myq * ld + kk * 32 + 8 * g;
    qf[kk] = __builtin_bit_cast(bf16x8_t, ld16(a.q + off, qok));
    const uint4 dv4 = ld16(a.dO + off, qok), ov4 = ld16(a.o + off, qok);
    df[kk] = __builtin_bit_cast(bf16x8_t, dv4);
    const uint32_t dw[4] = {dv4.x, dv4.y, dv4.z, dv4.w}, ow[4] = {ov4.x, ov4.y, ov4.z, ov4.w};
#pragma unroll
    for (int t = 0; t < 4; ++t)
      dl += bf2f((bf16_t)(dw[t] & 0xffff)) * bf2f((bf16_t)(ow[t] & 0xffff)) +
            bf2f((bf16_t)(dw[t] >> 16)) * bf2f((bf16_t)(ow[t] >> 16));
  }
  dl += __shfl_xor(dl, 16, 64);
  dl += __shfl_xor(dl, 32, 64);
  const long long srow = ((long long)b * a.H + h) * S;
  const float lse = qok ? a.lse[srow + myq] : 0.f;
  if (qok && g == 0) a.delta[srow + myq] = dl;
  const long long mrow = ((long long)h * S + (qok ? myq : 0)) * S;
  f32x4_t acc[D / 16];
#pragma unroll
  for (int i = 0; i < D / 16; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int nkt = a.causal ? qb + 1 : (S + TK - 1) / TK;
  Rows<D> nk, nv;
  int roff[D / 32];
  row_offsets<D>(roff, (int)ld, tid);
  f32x4_t nb[4], nc[4];
  auto fetch = [&](int k0) {
    if ((S & 3) == 0 && k0 + TK <= S) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        if constexpr (HB) nb[kb] = map4_full(a.bias + mrow, k0 + kb * 16 + 4 * g);
        if constexpr (HC) nc[kb] = map4_full(a.cmap + mrow, k0 + kb * 16 + 4 * g);
      }
    } else {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        if constexpr (HB) nb[kb] = map4(a.bias + mrow, k0 + kb * 16 + 4 * g, S);
        if constexpr (HC) nc[kb] = map4(a.cmap + mrow, k0 + kb * 16 + 4 * g, S);
      }
    }
    load_tile<D>(nk, a.k + base, ld, k0, S, tid, roff);
    load_tile<D>(nv, a.v + base, ld, k0, S, tid, roff);
  };
  fetch(0);
  for (int kti = 0; kti < nkt; ++kti) {
    const int k0 = kti * TK;
    __syncthreads();
    store_rows<D>(kimg, nk, tid);
    store_rows<D>(vimg, nv, tid);
    f32x4_t bv[4], cv[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      if constexpr (HB) bv[kb] = nb[kb];
      if constexpr (HC) cv[kb] = nc[kb];
    }
    __syncthreads();
    if (kti + 1 < nkt) fetch(k0 + TK);
    f32x4_t s[4], dp[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s[kb] = dp[kb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < D / 32; ++kk) {
        s[kb] = mfma(frag_rm<D + PADR>(kimg, kb * 16, kk, lane), qf[kk], s[kb]);
        dp[kb] = mfma(frag_rm<D + PADR>(vimg, kb * 16, kk, lane), df[kk], dp[kb]);
      }
    }
    // (rows of queries past S hold zero q / dO and lse 0: finite p, ds = 0; their dq is not stored)
    const bool edge = (a.causal && kti == nkt - 1) || k0 + TK > S;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int key0 = k0 + kb * 16 + 4 * g;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = key0 + r;
        float x = s[kb][r] * a.scale - lse;
        if constexpr (HB) x += bv[kb][r];
        float p = __expf(x);
        if (edge && !(key < S && (!a.causal || key <= myq))) p = 0.f;
        const float c = HC ? cv[kb][r] : 1.f;
        s[kb][r] = p * (c * dp[kb][r] - dl);
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const bf16x8_t sb = frag_acc(s[2 * c], s[2 * c + 1]);
#pragma unroll
      for (int i = 0; i < D / 16; ++i) acc[i] = mfma(frag_tr<D + PADR>(kimg, i * 16, c, lane), sb, acc[i]);
    }
  }
  if (qok) {
    bf16_t* row = a.dq + base + (long long)myq * ld + 4 * g;
    const float sc = a.scale;
#pragma unroll
    for (int i = 0; i < D / 16; ++i)
      *reinterpret_cast<uint2*>(row + i * 16) =
          make_uint2(pack_bf16x2(acc[i][0] * sc, acc[i][1] * sc), pack_bf16x2(acc[i][2] * sc, acc[i][3] * sc));
  }
}

// ------------------------------------------------------------------------------------------------------------------
// dk / dv per (key block, head, batch slice); map gradients accumulated in place over the slice's batches
template <int D, bool HB, bool HC>
__global__ __launch_bounds__(256) void attn_map_dkv_kernel(MapArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t qimg[64 * (D + PADR)];
  __shared__ __attribute__((aligned(16))) bf16_t dimg[64 * (D + PADR)];
  __shared__ float lse_s[TQ], dl_s[TQ];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int S = a.S, nqb = (S + TQ - 1) / TQ;
  const int kbk = blockIdx.x, h = blockIdx.y, slice = blockIdx.z;
  const long long ld = (long long)a.H * D;
  const int myk = kbk * TK + w * 16 + (lane & 15);
  const bool kok = myk < S;
  const bool kedge = (kbk + 1) * TK > S;
  const int bper = (a.B + a.bsplit - 1) / a.bsplit;
  const int b0 = slice * bper, b1 = min(a.B, b0 + bper);
  const long long mbase = (long long)h * S * S;
  const long long pbase = (long long)slice * a.H * S * S + mbase;   // this slice's partial map gradients
  const int qb_first = a.causal ? kbk : 0;                            // query blocks holding a query >= a key here
  int roff[D / 32];
  row_offsets<D>(roff, (int)ld, tid);
  for (int b = b0; b < b1; ++b) {
    const long long base = (long long)b * S * ld + (long long)h * D;
    const long long srow = ((long long)b * a.H + h) * S;
    bf16x8_t kf[D / 32], vf[D / 32];
#pragma unroll
    for (int kk = 0; kk < D / 32; ++kk) {
      const long long off = base + (long long)myk * ld + kk * 32 + 8 * g;
      kf[kk] = __builtin_bit_cast(bf16x8_t, ld16(a.k + off, kok));
      vf[kk] = __builtin_bit_cast(bf16x8_t, ld16(a.v + off, kok));
    }
    f32x4_t dk[D / 16], dv[D / 16];
#pragma unroll
    for (int i = 0; i < D / 16; ++i) dk[i] = dv[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    Rows<D> nq, nd;
    float nl = 0.f, ndl = 0.f;
    // the next tile's q / dO rows, statistics, map values and running map-gradient sums, one tile ahead (clamped
    // addresses, unconditional loads: a load under a branch made its use wait for every younger load)
    f32x4_t nbv[4], ncv[4], nob[4], noc[4];
    auto fetch = [&](int qbn) {
      const int qn = qbn * TQ;
#pragma unroll
      for (int qi = 0; qi < 4; ++qi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qq = qn + qi * 16 + 4 * g + r;
          const bool inb = kok && qq < S;
          const long long mi = (long long)(inb ? qq : 0) * S + (kok ? myk : 0);
          if constexpr (HB) {
            const float x = a.bias[mbase + mi], y = a.dbias[pbase + mi];
            nbv[qi][r] = inb ? x : 0.f;
            nob[qi][r] = inb ? y : 0.f;
          }
          if constexpr (HC) {
            const float x = a.cmap[mbase + mi], y = a.dcmap[pbase + mi];
            ncv[qi][r] = inb ? x : 1.f;
            noc[qi][r] = inb ? y : 0.f;
          }
        }
      load_tile<D>(nq, a.q + base, ld, qn, S, tid, roff);
      load_tile<D>(nd, a.dO + base, ld, qn, S, tid, roff);
      if (tid < TQ) {
        const bool ok = qn + tid < S;
        const long long i = srow + (ok ? qn + tid : 0);
        const float x = a.lse[i], y = a.delta[i];
        nl = ok ? x : 0.f;
        ndl = ok ? y : 0.f;
      }
    };
    if (qb_first < nqb) fetch(qb_first);
    for (int qb = qb_first; qb < nqb; ++qb) {
      const int q0 = qb * TQ;
      f32x4_t bv[4], cv[4], ob[4], oc[4];
#pragma unroll
      for (int qi = 0; qi < 4; ++qi) {
        if constexpr (HB) {
          bv[qi] = nbv[qi];
          ob[qi] = nob[qi];
        }
        if constexpr (HC) {
          cv[qi] = ncv[qi];
          oc[qi] = noc[qi];
        }
      }
      __syncthreads();
      store_rows<D>(qimg, nq, tid);
      store_rows<D>(dimg, nd, tid);
      if (tid < TQ) {
        lse_s[tid] = nl;
        dl_s[tid] = ndl;
      }
      __syncthreads();
      if (qb + 1 < nqb) fetch(qb + 1);
      // S / dP tiles [queries][keys]: lane holds key myk, queries q0 + qi * 16 + 4 g + r
      f32x4_t s[4], dp[4];
#pragma unroll
      for (int qi = 0; qi < 4; ++qi) {
        s[qi] = dp[qi] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < D / 32; ++kk) {
          s[qi] = mfma(frag_rm<D + PADR>(qimg, qi * 16, kk, lane), kf[kk], s[qi]);
          dp[qi] = mfma(frag_rm<D + PADR>(dimg, qi * 16, kk, lane), vf[kk], dp[qi]);
        }
      }
      const bool edge = kedge || (a.causal && qb == kbk) || q0 + TQ > S;   // uniform: masks only here
#pragma unroll
      for (int qi = 0; qi < 4; ++qi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = qi * 16 + 4 * g + r, qq = q0 + ql;
          const bool inb = !edge || (kok && qq < S);
          const bool ok = !edge || (inb && (!a.causal || myk <= qq));
          const long long mi = (long long)qq * S + myk;
          const float c = HC ? cv[qi][r] : 1.f;
          float x = s[qi][r] * a.scale - lse_s[ql];
          if constexpr (HB) x += bv[qi][r];
          const float e = __expf(x);
          const float p = ok ? e : 0.f;
          const float ds = p * (c * dp[qi][r] - dl_s[ql]);
          if (inb) {
            if constexpr (HB) a.dbias[pbase + mi] = ob[qi][r] + ds;
            if constexpr (HC) a.dcmap[pbase + mi] = oc[qi][r] + p * dp[qi][r];
          }
          s[qi][r] = p * c;
          dp[qi][r] = ds;
        }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const bf16x8_t pb = frag_acc(s[2 * c], s[2 * c + 1]);
        const bf16x8_t sb = frag_acc(dp[2 * c], dp[2 * c + 1]);
#pragma unroll
        for (int i = 0; i < D / 16; ++i) {
          dv[i] = mfma(frag_tr<D + PADR>(dimg, i * 16, c, lane), pb, dv[i]);
          dk[i] = mfma(frag_tr<D + PADR>(qimg, i * 16, c, lane), sb, dk[i]);
        }
      }
    }
    if (kok) {
      const long long off = base + (long long)myk * ld + 4 * g;
      const float sc = a.scale;
#pragma unroll
      for (int i = 0; i < D / 16; ++i) {
        *reinterpret_cast<uint2*>(a.dk + off + i * 16) =
            make_uint2(pack_bf16x2(dk[i][0] * sc, dk[i][1] * sc), pack_bf16x2(dk[i][2] * sc, dk[i][3] * sc));
        *reinterpret_cast<uint2*>(a.dv + off + i * 16) =
            make_uint2(pack_bf16x2(dv[i][0], dv[i][1]), pack_bf16x2(dv[i][2], dv[i][3]));
      }
    }
  }
}

// out[i] = sum over slices s (in order) of part[s][i]
__global__ __launch_bounds__(256) void map_fold_kernel(const float* part, float* out, long long n, int slices) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float v = 0.f;
  for (int s = 0; s < slices; ++s) v += part[s * n + i];
  out[i] = v;
}

template <int D, bool HB, bool HC>
hipError_t launch_fwd(const MapArgs& a, hipStream_t st) {
  const int nqb = (a.S + TQ - 1) / TQ;
  hipLaunchKernelGGL((attn_map_fwd_kernel<D, HB, HC>), dim3(nqb, a.H, a.B), dim3(256), 0, st, a);
  return hipGetLastError();
}
template <int D, bool HB, bool HC>
hipError_t launch_bwd(const MapArgs& a, hipStream_t st) {
  const int nqb = (a.S + TQ - 1) / TQ;
  hipLaunchKernelGGL((attn_map_dq_kernel<D, HB, HC>), dim3(nqb, a.H, a.B), dim3(256), 0, st, a);
  hipLaunchKernelGGL((attn_map_dkv_kernel<D, HB, HC>), dim3(nqb, a.H, a.bsplit), dim3(256), 0, st, a);
  return hipGetLastError();
}
// the map-presence instantiations of one head dim
template <int D>
hipError_t launch_fwd_d(const MapArgs& a, hipStream_t st) {
  if (a.bias) return a.cmap ? launch_fwd<D, true, true>(a, st) : launch_fwd<D, true, false>(a, st);
  return a.cmap ? launch_fwd<D, false, true>(a, st) : launch_fwd<D, false, false>(a, st);
}
template <int D>
hipError_t launch_bwd_d(const MapArgs& a, hipStream_t st) {
  if (a.bias) return a.cmap ? launch_bwd<D, true, true>(a, st) : launch_bwd<D, true, false>(a, st);
  return a.cmap ? launch_bwd<D, false, true>(a, st) : launch_bwd<D, false, false>(a, st);
}

}  // namespace

struct ObstMapDesc {
  const void *Q, *K, *V, *O, *dO;
  void *Out, *dQ, *dK, *dV;
  const void *bias, *cmap;
  void *dbias, *dcmap, *dbias_out, *dcmap_out;   // partial maps [bsplit][H][S][S] and the folded [H][S][S]
  void *LSE, *delta;
  int B, S, H, D, bsplit;
  float scale;
  int causal;
};

// batch slices of the dk/dv kernel: enough workgroups for 4 per CU, at most 4 partial maps
static int map_wg_target() {   // OBST_MAP_WG: dk/dv workgroups to aim for (A/B)
  static int v = [] { const char* e = getenv("OBST_MAP_WG"); return e ? atoi(e) : 1024; }();
  return v;
}
static int map_max_split() {   // OBST_MAP_SPLIT: most partial maps
  static int v = [] { const char* e = getenv("OBST_MAP_SPLIT"); return e ? atoi(e) : 4; }();
  return v;
}
OBST_API int obst_attn_map_bsplit(int B, int S, int H) {
  const long long wg = (long long)((S + TK - 1) / TK) * H;
  long long s = (map_wg_target() + wg - 1) / wg;
  if (s > map_max_split()) s = map_max_split();
  if (s > B) s = B;
  return (int)(s < 1 ? 1 : s);
}

static int fill(MapArgs& a, const ObstMapDesc* d) {
  if (d->B <= 0 || d->S <= 0 || d->H <= 0 || d->bsplit <= 0) return -1;
  a.q = (const bf16_t*)d->Q; a.k = (const bf16_t*)d->K; a.v = (const bf16_t*)d->V;
  a.o = (const bf16_t*)d->O; a.dO = (const bf16_t*)d->dO;
  a.out = (bf16_t*)d->Out; a.dq = (bf16_t*)d->dQ; a.dk = (bf16_t*)d->dK; a.dv = (bf16_t*)d->dV;
  a.bias = (const float*)d->bias; a.cmap = (const float*)d->cmap;
  a.dbias = (float*)d->dbias; a.dcmap = (float*)d->dcmap;
  a.lse = (float*)d->LSE; a.delta = (float*)d->delta;
  a.B = d->B; a.S = d->S; a.H = d->H; a.bsplit = d->bsplit; a.scale = d->scale; a.causal = d->causal;
  return 0;
}

OBST_API int obst_attn_map_fwd(const ObstMapDesc* d, hipStream_t st) {
  MapArgs a;
  if (fill(a, d) != 0) return -1;
  hipError_t e;
  switch (d->D) {
    case 32: e = launch_fwd_d<32>(a, st); break;
    case 64: e = launch_fwd_d<64>(a, st); break;
    case 96: e = launch_fwd_d<96>(a, st); break;
    case 128: e = launch_fwd_d<128>(a, st); break;
    default: return -2;
  }
  return (int)e;
}

OBST_API int obst_attn_map_bwd(const ObstMapDesc* d, hipStream_t st) {
  MapArgs a;
  if (fill(a, d) != 0) return -1;
  if ((a.bias && !a.dbias) || (a.cmap && !a.dcmap)) return -3;   // a present map always gets its gradient
  hipError_t e;
  switch (d->D) {
    case 32: e = launch_bwd_d<32>(a, st); break;
    case 64: e = launch_bwd_d<64>(a, st); break;
    case 96: e = launch_bwd_d<96>(a, st); break;
    case 128: e = launch_bwd_d<128>(a, st); break;
    default: return -2;
  }
  if (e != hipSuccess) return (int)e;
  const long long n = (long long)d->H * d->S * d->S;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (d->dbias && d->dbias_out && d->dbias_out != d->dbias)
    hipLaunchKernelGGL(map_fold_kernel, grid, dim3(256), 0, st, (const float*)d->dbias, (float*)d->dbias_out, n, d->bsplit);
  if (d->dcmap && d->dcmap_out && d->dcmap_out != d->dcmap)
    hipLaunchKernelGGL(map_fold_kernel, grid, dim3(256), 0, st, (const float*)d->dcmap, (float*)d->dcmap_out, n, d->bsplit);
  return (int)hipGetLastError();
}
