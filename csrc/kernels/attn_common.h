// Shared device helpers of the attention kernels (attention.hip; the lab's attn_fwd64.hip): LDS image swizzles,
// LDS-DMA staging, fragment offsets, the XCD-aware block map, the kernel argument block. Included inside an
// anonymous namespace by each translation unit.
#pragma once
#include "common.h"
#include <stdlib.h>
#include <type_traits>

namespace {

constexpr int NTH = 256;  // 4 waves

template <int D>
struct Geo {
  static constexpr int CPR = D / 8;        // 16-byte chunks per row
  static constexpr int DS = D / 32;        // k-steps over the head dim
  static constexpr int DT = D / 16;        // 16-wide d tiles
  static constexpr int ROWB = D * 2;       // bytes per row
};

// one XOR-swizzle per head dim, used for every tile (row reads via ds_read_b128 and transposed reads via
// ds_read_b64_tr_b16); layout (b) of cdna_hip_programming.md T10 for D=128.
template <int D>
__device__ __forceinline__ int swz(int row) {
  if (D == 128) return ((row & 3) << 2) | ((row >> 2) & 3);
  if (D == 64) return ((row >> 1) & 3) << 1 | ((row >> 3) & 1);
  return (row >> 2) & 3;
}

template <int D>
__device__ __forceinline__ int lds_off(int row, int chunk) {
  return row * Geo<D>::ROWB + ((chunk ^ swz<D>(row)) << 4);
}

// swizzle of the images the 16x16x32 kernels (dQ, dK/dV, forward v1) stage and read. D = 128: chunk ^= (row & 7) << 1.
// Their row read (lanes 0-15 rows r..r+15 of chunk c, lanes 16-31 chunk c+1) meets the ds_read_b128 lane groups
// {0-3,12-15,20-27} / {4-11,16-19,28-31}: rows {0-3,12-15} of c with rows 4-11 of c+1 -- (row & 7) << 1 is one-to-one
// on each of those row sets and leaves bit 0 to the chunk, so the 16 slots of a group are distinct. Their transposed
// read (one 32-lane half = rows r..r+7, chunks c, c+1) gets 8 distinct bit-1..3 values and the chunk bit: also
// conflict-free. The (row&3)<<2 | (row>>2)&3 swizzle of the 32x32x16 kernels is 2-way on both reads here
// (cdna_hip_programming.md T10: SQ_LDS_BANK_CONFLICT 138M per dK/dV launch, profiles/r1e_pmc_attn_dkv16.txt).
template <int D>
__device__ __forceinline__ int swz16(int row) {
  if (D == 128) return (row & 7) << 1;
  return swz<D>(row);
}

template <int D>
__device__ __forceinline__ int lds_off16(int row, int chunk) {
  return row * Geo<D>::ROWB + ((chunk ^ swz16<D>(row)) << 4);
}

// stage ROWS x D bf16 rows (token-major, row stride ld) into an LDS image with direct global->LDS DMA
// (global_load_lds_dwordx4 from inline asm, one 1 KiB piece per wave-instruction, lane-linear in LDS; the consumer
// waits with vm_wait<0>() before the publishing barrier -- the builtin made the compiler put vmcnt(0) in front of
// every LDS read, so the next tile's DMA could never overlap the current tile's MFMAs): the per-lane SOURCE chunk is
// pre-swizzled so the image matches lds_off(). Rows >= nvalid are clamped to the last valid row (masked later).
template <int D, int ROWS, int NW = 4>
__device__ __forceinline__ void stage_rows(char* lds, const bf16_t* g, long long ld, int nvalid, int tid) {
  constexpr int CPR = Geo<D>::CPR;
  constexpr int PIECES = ROWS * CPR * 16 / 1024;   // 1 KiB pieces in the image
  static_assert(ROWS * CPR % 64 == 0, "the image must be whole 1 KiB pieces");
  const int wave = tid >> 6, lane = tid & 63;
  const int last = nvalid - 1;
#pragma unroll
  for (int i = 0; i < (PIECES + NW - 1) / NW; ++i) {
    const int j = wave + NW * i;
    if (PIECES % NW == 0 || j < PIECES) {
      // chunk j*64 + lane of the row-major image (D = 96: 12 chunks per row, so a piece straddles rows)
      const int row = (j * 64 + lane) / CPR;
      const int p = (j * 64 + lane) % CPR;
      const int c = p ^ swz16<D>(row);
      const int srow = row < last ? row : last;
      glds16_asm(g + srow * ld + c * 8, lds + j * 1024);
    }
  }
}

// Full-tile form of stage_rows for D = 128, 64 rows, 4 waves: piece j = wave + 4i covers rows 4j .. 4j + 3, so a
// lane's source offset inside the tile depends only on its lane and on j & 1 (the swizzle (row & 7) << 1 of row
// 4j + (lane >> 4)). The two 32-bit lane offsets are computed once per kernel (lane_off16_128); per piece the address
// is a wave-uniform base + 4j rows (scalar) + that offset, instead of stage_rows' per-chunk 64-bit row arithmetic
// (~150 VALU per chunk per wave in the dK/dV kernel, whose loop is VALU-issue bound).
__device__ __forceinline__ void lane_off16_128(unsigned (&off)[2], long long ld, int lane) {
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int row = 4 * e + (lane >> 4);   // row & 7 of piece j with j & 1 == e
    off[e] = (unsigned)((lane >> 4) * (int)ld + (((lane & 15) ^ swz16<128>(row)) << 3)) * 2u;
  }
}

template <int ROWS = 64>   // 64- or 32-row tile: ROWS / 16 pieces per wave
__device__ __forceinline__ void stage_full16_128(char* lds, const bf16_t* g, long long ld, const unsigned (&off)[2],
                                                 int wave) {
  const char* gb = reinterpret_cast<const char*>(g);
#pragma unroll
  for (int i = 0; i < ROWS / 16; ++i) {
    const int j = wave + 4 * i;
    glds16_asm(gb + (long long)(4 * j) * ld * 2 + off[j & 1], lds + j * 1024);
  }
}

// 4-byte values (lse / delta rows) for `n` <= 64 consecutive queries: one 256-B piece from wave 0
__device__ __forceinline__ void stage_f32(char* lds, const float* g, int n, int nvalid, int tid) {
  if (tid >= 0 && tid < 64) {   // one wave, all lanes (n <= 64: lanes past n re-read the last value)
    const int q = min(min(tid, n - 1), nvalid - 1);
    glds4_asm(g + q, lds);
  }
}

// row fragment: lane holds X[row0 + (lane&15)][d = ds*32 + 8*(lane>>4) + 0..7]
template <int D>
__device__ __forceinline__ bf16x8_t row_frag(const char* lds, int row0, int ds, int lane) {
  const int r = row0 + (lane & 15);
  return *reinterpret_cast<const bf16x8_t*>(lds + lds_off16<D>(r, ds * 4 + (lane >> 4)));
}

// transposed fragment over 32 rows starting at row0: lane (g, i) holds X[row0 + perm(g, jj)][d0 + i],
// perm(g, jj) = (jj >> 2) * 16 + 4g + (jj & 3)
template <int D>
__device__ __forceinline__ bf16x8_t tr_frag(const char* lds, int row0, int d0, int lane) {
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
  const int col = d0 + 4 * pp;
  const int c = col >> 3;
  const int r0 = row0 + 4 * g + q, r1 = r0 + 16;
  const int o0 = r0 * Geo<D>::ROWB + ((c ^ swz16<D>(r0)) << 4) + ((pp & 1) << 3);
  const int o1 = r1 * Geo<D>::ROWB + ((c ^ swz16<D>(r1)) << 4) + ((pp & 1) << 3);
  s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, lds + o0));
  s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, lds + o1));
  s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// pack two 16x16 fp32 accumulator tiles (k-halves) into one bf16x8 B-operand with the perm() k order
__device__ __forceinline__ bf16x8_t pack_p(const f32x4_t& a, const f32x4_t& b) {
  s16x8_t v;
  v[0] = (short)f2bf(a[0]); v[1] = (short)f2bf(a[1]); v[2] = (short)f2bf(a[2]); v[3] = (short)f2bf(a[3]);
  v[4] = (short)f2bf(b[0]); v[5] = (short)f2bf(b[1]); v[6] = (short)f2bf(b[2]); v[7] = (short)f2bf(b[3]);
  return __builtin_bit_cast(bf16x8_t, v);
}

__device__ __forceinline__ bf16x8_t load_frag_g(const bf16_t* p, bool ok) {
  if (!ok) return __builtin_bit_cast(bf16x8_t, s16x8_t{0, 0, 0, 0, 0, 0, 0, 0});
  return *reinterpret_cast<const bf16x8_t*>(p);
}

// XCD-aware block coordinates for a 1-D grid of nx * (B*H) blocks (T1): the bijective XCD remap puts consecutive
// logical blocks -- the nx blocks of one (b, h), which all stream the same K/V (forward, dQ) or Q/dO (dK/dV) -- on
// the same XCD, so those re-reads hit that XCD's L2 instead of MALL/HBM.
__device__ __forceinline__ void attn_block(int nx, int& bx, int& bh) {
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  bx = L % nx;
  bh = L / nx;
}

// bias_order: the map-hooked kernels (BIAS) take (b, h) = (bh % B, bh / B) instead of (bh / H, bh % H), so the
// consecutive logical blocks one XCD runs are the batches of one head, which read the same [S][S] map rows: the map
// is fetched from HBM about once per head and re-read from L2 / MALL, instead of once per (batch, head)

constexpr float LOG2E = 1.4426950408889634f;
constexpr float NEG_BIG = -1e30f;

struct AttnArgs {
  const bf16_t *Q, *K, *V, *O, *dO;
  bf16_t *Oout, *dQ, *dK, *dV;
  float *LSE, *delta;
  int B, S, H;
  long long ld;   // token stride (elements) of Q, K, V and dQ, dK, dV: H*D, or 3*H*D for the interleaved k|q|v layout
  long long ld_o; // token stride of O and dO (H*D)
  float scale;
  int causal;
  int prio;       // s_setprio(1) around the MFMA clusters: bit 0 dK/dV kernel (default on: -2 %), bit 1 dQ (+1 %: off)
  const bf16_t* Res;   // forward, optional: Sum = bf16(O) + Res, the block's residual add (O's layout, row stride ld_o)
  bf16_t* Sum;
  const float* bias;   // optional (obst_attn_fwd_bias / obst_attn_bwd_bias): [H][S][S] fp32 added to the scaled logits
  float* dbias;        // backward with bias: per-batch partial map gradients [B][H][S][S] (dS of the dK/dV kernel)
};

// the forward epilogue's 4-element store of O (and, with a residual, of O + residual from the rounded O values)
__device__ __forceinline__ void store_o4(const AttnArgs& a, long long off, float v0, float v1, float v2, float v3) {
  const uint2 ov = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
  *reinterpret_cast<uint2*>(a.Oout + off) = ov;
  if (a.Sum) {
    const uint2 r = *reinterpret_cast<const uint2*>(a.Res + off);
    *reinterpret_cast<uint2*>(a.Sum + off) =
        make_uint2(pack_bf16x2(bf2f(ov.x & 0xffff) + bf2f(r.x & 0xffff), bf2f(ov.x >> 16) + bf2f(r.x >> 16)),
                   pack_bf16x2(bf2f(ov.y & 0xffff) + bf2f(r.y & 0xffff), bf2f(ov.y >> 16) + bf2f(r.y >> 16)));
  }
}

// Epilogue staging of a wave's [rows][128] bf16 output tile held in 16x16 accumulator layout (lane i = row within a
// 16-row group, g = lane >> 4: d = dt*16 + 4g + [0, 4)), so the global stores go out as whole 256-byte rows, 16-byte
// per lane, instead of 8-byte pieces at row stride. Image: row r, 16-byte chunk c at (c ^ (r & 7)), 8-byte half at
// hf ^ ((r >> 3) & 1): the 16 lanes of a ds_write_b64 group (16 rows, one chunk, one half) hit 16 distinct slots.
__device__ __forceinline__ void epi_put(char* so, int row, int dt, int g, const f32x4_t& v, float sc) {
  const int c = 2 * dt + (g >> 1), hf = g & 1;
  *reinterpret_cast<uint2*>(so + row * 256 + ((c ^ (row & 7)) << 4) + ((hf ^ ((row >> 3) & 1)) << 3)) =
      make_uint2(pack_bf16x2(v[0] * sc, v[1] * sc), pack_bf16x2(v[2] * sc, v[3] * sc));
}

// 16-byte chunk c (elements 8c..8c+7) of row rr of the staged image, in logical order
__device__ __forceinline__ uint4 epi_get(const char* so, int rr, int c) {
  const uint4 v = *reinterpret_cast<const uint4*>(so + rr * 256 + ((c ^ (rr & 7)) << 4));
  return ((rr >> 3) & 1) ? make_uint4(v.z, v.w, v.x, v.y) : v;
}

// ----------------------------------------------------------------------------------------------------------------
// raw v_exp_f32 (2^x): no denormal range fix-up (exp2f adds a compare + 2 ldexp per call); -inf -> 0
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// The running max only moves when a row's max grew by more than 2^RESCALE_TH (P stays <= 2^8 in bf16, l and O in
// fp32), so the O rescale -- 64 multiplies per tile at D=128 -- runs on a few early tiles instead of every tile.
constexpr float RESCALE_TH = 8.f;

typedef __attribute__((ext_vector_type(16))) float f32x16_t;

__device__ __forceinline__ float xh_max(float v) {   // max over lanes l and l^32
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

__device__ __forceinline__ float xh_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ bf16x8_t pack8(const f32x16_t& a, int off) {
  s16x8_t v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (short)f2bf(a[off + j]);
  return __builtin_bit_cast(bf16x8_t, v);
}

// per-lane LDS byte offsets of the fragments, tile-relative (row n of K for k-step ks; Vᵀ rows r0 / r0 + 8 for d-tile
// dt). The swizzle depends on row & 15 only, so every 16-row shift of a fragment is a constant (immediate) offset.
struct Frag32 {
  int k[8];
  int v[4][2];
};

__device__ __forceinline__ void frag32_offsets(Frag32& f, int lane) {
  const int h = lane >> 5, n = lane & 31, hi = (lane >> 4) & 1, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) f.k[ks] = lds_off<128>(n, ks * 2 + h);
  const int r0 = 4 * h + q, r1 = r0 + 8;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int c = (dt * 32 + hi * 16 + 4 * pp) >> 3;
    f.v[dt][0] = r0 * 256 + ((c ^ swz<128>(r0)) << 4) + ((pp & 1) << 3);
    f.v[dt][1] = r1 * 256 + ((c ^ swz<128>(r1)) << 4) + ((pp & 1) << 3);
  }
}

__device__ __forceinline__ bf16x8_t tr_pair(const char* lds, int o0, int o1) {
  const s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, lds + o0));
  const s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, lds + o1));
  const s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// LDS-DMA of a full 64-row tile: wave-uniform global base + 32-bit per-lane byte offsets computed once (soff), so
// the loads take the saddr + voffset form and the LDS base (M0) is scalar
template <int NP, int NW = 4>   // NP pieces per wave: 4 for a 64-row tile, 2 for 32 rows (NW = 4 waves)
__device__ __forceinline__ void stage_full64(char* lds, const bf16_t* g, const unsigned (&soff)[NP], int w) {
  const char* gb = reinterpret_cast<const char*>(g);
#pragma unroll
  for (int i = 0; i < NP; ++i) glds16_asm(gb + soff[i], lds + (w + NW * i) * 1024);
}

// stage_rows with the asm DMA (ragged last tile: rows >= nvalid clamped to the last valid row)
template <int NP, int NW = 4>
__device__ __forceinline__ void stage_rows64_asm(char* lds, const bf16_t* g, long long ld, int nvalid, int w,
                                                 int lane) {
  const int last = nvalid - 1;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int j = w + NW * i;
    const int row = j * 4 + (lane >> 4);
    const int c = (lane & 15) ^ swz<128>(row);
    const int srow = row < last ? row : last;
    glds16_asm(g + srow * ld + c * 8, lds + j * 1024);
  }
}

}  // namespace

