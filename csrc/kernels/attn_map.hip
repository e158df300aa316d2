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
template <int D>
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
  load_rows<D>(nk, a.k + base, ld, 0, S, tid);
  load_rows<D>(nv, a.v + base, ld, 0, S, tid);
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * TK;
    __syncthreads();
    store_rows<D>(kimg, nk, tid);
    store_rows<D>(vimg, nv, tid);
    __syncthreads();
    if (kt + 1 < nkt) {
      load_rows<D>(nk, a.k + base, ld, k0 + TK, S, tid);
      load_rows<D>(nv, a.v + base, ld, k0 + TK, S, tid);
    }
    f32x4_t s[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s[kb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < D / 32; ++kk) s[kb] = mfma(frag_rm<D + PADR>(kimg, kb * 16, kk, lane), qf[kk], s[kb]);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const f32x4_t bv = a.bias != nullptr ? map4(a.bias + mrow, k0 + kb * 16 + 4 * g, S) : f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + kb * 16 + 4 * g + r;
        const bool ok = key < S && (!a.causal || key <= myq);
        const float x = ok ? s[kb][r] * a.scale + bv[r] : -INFINITY;
        s[kb][r] = x;
        mx = fmaxf(mx, x);
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);   // finite: key k0 <= every query of a visited tile
    const float al = __expf(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const f32x4_t cv = a.cmap != nullptr ? map4(a.cmap + mrow, k0 + kb * 16 + 4 * g, S) : f32x4_t{1.f, 1.f, 1.f, 1.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf(s[kb][r] - mn);
        rs += p;
        s[kb][r] = p * cv[r];
      }
    }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l = l * al + rs;
    m = mn;
#pragma unroll
    for (int i = 0; i < D / 16; ++i) acc[i] *= al;
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
template <int D>
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
  load_rows<D>(nk, a.k + base, ld, 0, S, tid);
  load_rows<D>(nv, a.v + base, ld, 0, S, tid);
  for (int kti = 0; kti < nkt; ++kti) {
    const int k0 = kti * TK;
    __syncthreads();
    store_rows<D>(kimg, nk, tid);
    store_rows<D>(vimg, nv, tid);
    __syncthreads();
    if (kti + 1 < nkt) {
      load_rows<D>(nk, a.k + base, ld, k0 + TK, S, tid);
      load_rows<D>(nv, a.v + base, ld, k0 + TK, S, tid);
    }
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
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int key0 = k0 + kb * 16 + 4 * g;
      const f32x4_t bv = a.bias != nullptr ? map4(a.bias + mrow, key0, S) : f32x4_t{0.f, 0.f, 0.f, 0.f};
      const f32x4_t cv = a.cmap != nullptr ? map4(a.cmap + mrow, key0, S) : f32x4_t{1.f, 1.f, 1.f, 1.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = key0 + r;
        const bool ok = qok && key < S && (!a.causal || key <= myq);
        const float p = ok ? __expf(s[kb][r] * a.scale + bv[r] - lse) : 0.f;
        s[kb][r] = p * (cv[r] * dp[kb][r] - dl);
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
template <int D>
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
  const int bper = (a.B + a.bsplit - 1) / a.bsplit;
  const int b0 = slice * bper, b1 = min(a.B, b0 + bper);
  const long long mbase = (long long)h * S * S;
  const long long pbase = (long long)slice * a.H * S * S + mbase;   // this slice's partial map gradients
  const int qb_first = a.causal ? kbk : 0;                            // query blocks holding a query >= a key here
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
    auto fetch = [&](int qbn) {
      const int qn = qbn * TQ;
      load_rows<D>(nq, a.q + base, ld, qn, S, tid);
      load_rows<D>(nd, a.dO + base, ld, qn, S, tid);
      if (tid < TQ) {
        const bool ok = qn + tid < S;
        nl = ok ? a.lse[srow + qn + tid] : 0.f;
        ndl = ok ? a.delta[srow + qn + tid] : 0.f;
      }
    };
    if (qb_first < nqb) fetch(qb_first);
    for (int qb = qb_first; qb < nqb; ++qb) {
      const int q0 = qb * TQ;
      // this tile's map values and the running map-gradient sums, loaded before the staging and the score MFMAs so
      // their latency hides under them (issued at their use, every read-modify-write paid a full memory round trip)
      f32x4_t bv[4], cv[4], ob[4], oc[4];
#pragma unroll
      for (int qi = 0; qi < 4; ++qi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qq = q0 + qi * 16 + 4 * g + r;
          const bool inb = kok && qq < S;
          const long long mi = (long long)(inb ? qq : 0) * S + (kok ? myk : 0);
          bv[qi][r] = a.bias != nullptr && inb ? a.bias[mbase + mi] : 0.f;
          cv[qi][r] = a.cmap != nullptr && inb ? a.cmap[mbase + mi] : 1.f;
          ob[qi][r] = a.dbias != nullptr && inb ? a.dbias[pbase + mi] : 0.f;
          oc[qi][r] = a.dcmap != nullptr && inb ? a.dcmap[pbase + mi] : 0.f;
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
#pragma unroll
      for (int qi = 0; qi < 4; ++qi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = qi * 16 + 4 * g + r, qq = q0 + ql;
          const bool inb = kok && qq < S;
          const bool ok = inb && (!a.causal || myk <= qq);
          const long long mi = (long long)qq * S + myk;
          const float c = cv[qi][r];
          const float p = ok ? __expf(s[qi][r] * a.scale + bv[qi][r] - lse_s[ql]) : 0.f;
          const float ds = p * (c * dp[qi][r] - dl_s[ql]);
          if (inb) {
            if (a.dbias != nullptr) a.dbias[pbase + mi] = ob[qi][r] + ds;
            if (a.dcmap != nullptr) a.dcmap[pbase + mi] = oc[qi][r] + p * dp[qi][r];
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

template <int D>
hipError_t launch_fwd(const MapArgs& a, hipStream_t st) {
  const int nqb = (a.S + TQ - 1) / TQ;
  hipLaunchKernelGGL(attn_map_fwd_kernel<D>, dim3(nqb, a.H, a.B), dim3(256), 0, st, a);
  return hipGetLastError();
}
template <int D>
hipError_t launch_bwd(const MapArgs& a, hipStream_t st) {
  const int nqb = (a.S + TQ - 1) / TQ;
  hipLaunchKernelGGL(attn_map_dq_kernel<D>, dim3(nqb, a.H, a.B), dim3(256), 0, st, a);
  hipLaunchKernelGGL(attn_map_dkv_kernel<D>, dim3(nqb, a.H, a.bsplit), dim3(256), 0, st, a);
  return hipGetLastError();
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
OBST_API int obst_attn_map_bsplit(int B, int S, int H) {
  const long long wg = (long long)((S + TK - 1) / TK) * H;
  long long s = (1024 + wg - 1) / wg;
  if (s > 4) s = 4;
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
    case 32: e = launch_fwd<32>(a, st); break;
    case 64: e = launch_fwd<64>(a, st); break;
    case 96: e = launch_fwd<96>(a, st); break;
    case 128: e = launch_fwd<128>(a, st); break;
    default: return -2;
  }
  return (int)e;
}

OBST_API int obst_attn_map_bwd(const ObstMapDesc* d, hipStream_t st) {
  MapArgs a;
  if (fill(a, d) != 0) return -1;
  hipError_t e;
  switch (d->D) {
    case 32: e = launch_bwd<32>(a, st); break;
    case 64: e = launch_bwd<64>(a, st); break;
    case 96: e = launch_bwd<96>(a, st); break;
    case 128: e = launch_bwd<128>(a, st); break;
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
