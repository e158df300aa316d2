// K04: flash attention (causal / full) for gfx950 with v_mfma_f32_16x16x32_bf16.
// Reference semantics (src/model/spatial.py:44-81): logits = q·kᵀ·scale (scale is a runtime argument: the
// reference uses attention-dim length^-0.5, quirk A1), causal mask by -inf (ref adds -2e38), max-subtracted
// softmax, ·v. Tensors are token-major [B, S, H, D] (row stride H*D) -- the layout the q/k/v linears write --
// so no transposes are needed around the kernel. LSE/delta are fp32 [B, H, S].
//
// Orientation (cdna_hip_programming.md §3 "accumulator tile as the next MFMA's operand", Appendix B attention):
//  * forward and dQ kernels compute Sᵀ = K·Qᵀ, so a lane owns one query column (lane&15) and 16 keys of a
//    64-key block: the softmax row max/sum is 15 local ops + 2 xor-shuffles, and the rescale of Oᵀ is lane-uniform.
//  * the P / dS accumulators feed the next MFMA directly as B operand (bf16-packed in registers) with a permuted
//    k order; the matching A operand (V or K, [key][d] in LDS) is read with ds_read_b64_tr_b16 (T10).
//  * the dK/dV kernel computes S = Q·Kᵀ (key on the lane) so dVᵀ += dOᵀ·P and dKᵀ += Qᵀ·dS reuse the registers.
// dQ is produced by its own kernel (recomputing S and dP) instead of fp32 atomics: at S=2048 the atomic dQ sum
// would move ~16x the dQ bytes through the ~1.3 TB/s atomic path (Guideline 12).
#include "common.h"
#include <stdlib.h>
#include <type_traits>

#include "attn_common.h"

namespace {


// one 64-key tile of the forward for a wave's 32 queries. MASK: diagonal / ragged tiles (causal + bounds), branch
// free; unmasked tiles carry no mask arithmetic at all.
template <int D, bool MASK>
__device__ __forceinline__ void fwd_tile(const char* sK, const char* sV, const bf16x8_t (&qf)[2][Geo<D>::DS],
                                         f32x4_t (&o)[Geo<D>::DT][2], float (&m)[2], float (&l)[2], int k0, int qw,
                                         int S, int causal, float c2, int lane) {
  using G = Geo<D>;
  const int g = lane >> 4, i = lane & 15;
  f32x4_t s[2][4];
  {
    bf16x8_t kf[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) kf[kt] = row_frag<D>(sK, kt * 16, 0, lane);
#pragma unroll
    for (int ds = 0; ds < G::DS; ++ds) {
      bf16x8_t kn[4];
      if (ds + 1 < G::DS) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) kn[kt] = row_frag<D>(sK, kt * 16, ds + 1, lane);
      }
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          s[qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt], qf[qt][ds],
                                                              ds == 0 ? f32x4_t{0.f, 0.f, 0.f, 0.f} : s[qt][kt], 0, 0, 0);
      if (ds + 1 < G::DS) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) kf[kt] = kn[kt];
      }
    }
  }
  bf16x8_t pf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = qw + qt * 16 + i;
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        if (MASK) {
          const int key = k0 + kt * 16 + 4 * g + v;
          const bool dead = key >= S || (causal && key > q);
          s[qt][kt][v] = dead ? -INFINITY : s[qt][kt][v];
        }
        mx = fmaxf(mx, s[qt][kt][v]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float ms = mx * c2;                       // row max in the scaled log2 domain (c2 > 0)
    const bool bump = ms > m[qt] + RESCALE_TH;
    if (__builtin_amdgcn_ballot_w64(bump)) {        // wave-uniform: rare after the first tile
      const float mn = bump ? ms : m[qt];
      const float alpha = fexp2(m[qt] - mn);
      l[qt] *= alpha;
#pragma unroll
      for (int dt = 0; dt < G::DT; ++dt) o[dt][qt] *= alpha;
      m[qt] = mn;
    }
    const float nm = -m[qt];
    float rs = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float p = fexp2(__builtin_fmaf(s[qt][kt][v], c2, nm));
        s[qt][kt][v] = p;
        rs += p;
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l[qt] += rs;
    pf[qt][0] = pack_p(s[qt][0], s[qt][1]);
    pf[qt][1] = pack_p(s[qt][2], s[qt][3]);
  }
#pragma unroll
  for (int dt = 0; dt < G::DT; ++dt) {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      bf16x8_t vf = tr_frag<D>(sV, st * 32, dt * 16, lane);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
        o[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qt][st], o[dt][qt], 0, 0, 0);
    }
  }
}

// forward: block = 128 queries of one (b, h); wave w owns queries q0 + 32w + [0, 32). K/V tiles of 64 keys are
// double-buffered in LDS and filled by LDS-DMA one tile ahead; one barrier per tile.
template <int D>
__global__ __launch_bounds__(NTH, 2) void attn_fwd_kernel(AttnArgs a) {
  using G = Geo<D>;
  constexpr int TILE = 64 * G::ROWB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, i = lane & 15;
  const int nx = (a.S + 127) / 128;
  int bx, bh;
  attn_block(nx, bx, bh);
  const int b = bh / a.H, h = bh % a.H;
  // heaviest causal blocks first: the tail of the grid then fills with short blocks
  const int qblk = (a.causal ? (nx - 1 - bx) : bx) * 128;
  const int qw = qblk + w * 32;
  const bf16_t* Qb = a.Q + (long long)b * a.S * a.ld + h * D;
  const bf16_t* Kb = a.K + (long long)b * a.S * a.ld + h * D;
  const bf16_t* Vb = a.V + (long long)b * a.S * a.ld + h * D;

  const int kend = a.causal ? min(a.S, qblk + 128) : a.S;
  const int nkb = (kend + 63) / 64;
  stage_rows<D, 64>(smem, Kb, a.ld, a.S, tid);
  stage_rows<D, 64>(smem + TILE, Vb, a.ld, a.S, tid);

  bf16x8_t qf[2][G::DS];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = qw + qt * 16 + i;
#pragma unroll
    for (int ds = 0; ds < G::DS; ++ds) qf[qt][ds] = load_frag_g(Qb + (long long)q * a.ld + ds * 32 + 8 * g, q < a.S);
  }
  f32x4_t o[G::DT][2];
#pragma unroll
  for (int dt = 0; dt < G::DT; ++dt) o[dt][0] = o[dt][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m[2] = {NEG_BIG, NEG_BIG}, l[2] = {0.f, 0.f};
  const float c2 = a.scale * LOG2E;
  vm_wait<0>();   // staged tiles (asm LDS-DMA: the compiler does not track them) have landed
  __syncthreads();

  for (int kb = 0; kb < nkb; ++kb) {
    const int k0 = kb * 64;
    const char* sK = smem + (kb & 1) * 2 * TILE;
    const char* sV = sK + TILE;
    if (kb + 1 < nkb) {
      char* nxt = smem + ((kb + 1) & 1) * 2 * TILE;
      stage_rows<D, 64>(nxt, Kb + (long long)(k0 + 64) * a.ld, a.ld, a.S - k0 - 64, tid);
      stage_rows<D, 64>(nxt + TILE, Vb + (long long)(k0 + 64) * a.ld, a.ld, a.S - k0 - 64, tid);
    }
    if (!(a.causal && k0 > qw + 31)) {  // wave-uniform: skip blocks entirely in this wave's future
      const bool need_mask = (a.causal && k0 + 63 > qw) || k0 + 64 > a.S;
      if (need_mask) fwd_tile<D, true>(sK, sV, qf, o, m, l, k0, qw, a.S, a.causal, c2, lane);
      else fwd_tile<D, false>(sK, sV, qf, o, m, l, k0, qw, a.S, a.causal, c2, lane);
    }
    vm_wait<0>();   // staged tiles (asm LDS-DMA: the compiler does not track them) have landed
    __syncthreads();
  }
  // epilogue: lane holds O[q = qw + qt*16 + i][d = dt*16 + 4g + v]
  const long long ob = (long long)b * a.S * a.ld_o + h * D;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = qw + qt * 16 + i;
    if (q >= a.S) continue;
    const float inv = 1.f / l[qt];
#pragma unroll
    for (int dt = 0; dt < G::DT; ++dt) {
      const int d = dt * 16 + 4 * g;
      store_o4(a, ob + (long long)q * a.ld_o + d, o[dt][qt][0] * inv, o[dt][qt][1] * inv, o[dt][qt][2] * inv,
               o[dt][qt][3] * inv);
    }
    if (g == 0) a.LSE[((long long)b * a.H + h) * a.S + q] = (m[qt] + __log2f(l[qt])) / LOG2E;
  }
}

// ----------------------------------------------------------------------------------------------------------------
// delta[b,h,q] = sum_d dO * O
template <int D>
__global__ __launch_bounds__(NTH) void attn_delta_kernel(AttnArgs a) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);  // row = (b*S + q)*H + h
  const long long nrows = (long long)a.B * a.S * a.H;
  if (row >= nrows) return;
  const int h = row % a.H;
  const long long bq = row / a.H;
  const int q = bq % a.S, b = bq / a.S;
  const bf16_t* o = a.O + bq * a.ld_o + h * D;
  const bf16_t* d = a.dO + bq * a.ld_o + h * D;
  float acc = 0.f;
  for (int j = lane * 2; j < D; j += 128) {
    uint32_t ov = *reinterpret_cast<const uint32_t*>(o + j);
    uint32_t dv = *reinterpret_cast<const uint32_t*>(d + j);
    acc += bf2f(ov & 0xffff) * bf2f(dv & 0xffff) + bf2f(ov >> 16) * bf2f(dv >> 16);
  }
  acc = wave_sum(acc);
  if (lane == 0) a.delta[((long long)b * a.H + h) * a.S + q] = acc;
}

// dK/dV read-ahead: score loop (DKV_SPF) and update loop (DKV_UPF). Both on exceed the 256 VGPRs of two waves per
// SIMD (a spilled LDS address whose reload's vmcnt(0) waits for the next chunk's DMA). DKV_SPF=0 DKV_UPF=1 cuts the
// MFMAs behind lgkmcnt(0) from 21 to 10 of 128 and measured the same (3120 / 3088 vs 3086 / 3119 us,
// profiles/r3_attn_bwd_ab.md): the partner wave hides that latency; the kernel is bound elsewhere
#ifndef DKV_FAST_STAGE
#define DKV_FAST_STAGE 1   // dK/dV full-tile staging from precomputed lane offsets
#endif
#ifndef DKV_SPF
#define DKV_SPF 2
#endif
#ifndef DKV_UPF
#define DKV_UPF 0
#endif
#ifndef DKV_PF
#define DKV_PF 2   // score-loop fragment prefetch distance of dq_tile / dkv_chunk (0: the plain loops)
#endif

// backward map hook (biased_softmax): 1 loads a tile's map values after its score MFMAs instead of before them (their
// registers are then not live across the MFMA loop of the kernels that already use all 256 VGPRs)
#ifndef BIAS_LATE
#define BIAS_LATE 1
#endif

// one 64-key tile of the dQ kernel for a wave's 32 queries (two 32-key halves: P needs only the stored LSE, so no
// state crosses the halves). dP starts from -delta (the accumulator init), so dS = P * dP.
// BIAS (biased_softmax): bq = this lane's query row (qt = 0) of the [H][S][S] map; its 4 keys per 16-key sub-tile are
// one 16-byte load, issued before the score MFMAs and added to the scaled logits after them
template <int D, bool MASK, int HALVES = 2, bool BIAS = false>
__device__ __forceinline__ void dq_tile(const char* sK, const char* sV, const bf16x8_t (&qf)[2][Geo<D>::DS],
                                        const bf16x8_t (&df)[2][Geo<D>::DS], const float (&lse2)[2],
                                        const float (&dlt)[2], f32x4_t (&acc)[Geo<D>::DT][2], int k0, int qw, int S,
                                        int causal, float c2, int lane, int prio = 0, const float* bq = nullptr) {
  using G = Geo<D>;
  const int g = lane >> 4, i = lane & 15;
#pragma unroll
  for (int st = 0; st < HALVES; ++st) {
    f32x4_t sc[2][2], dp[2][2], bv[2][2];
    auto load_bias = [&]() {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          bv[qt][kk] = *reinterpret_cast<const f32x4_t*>(bq + (long long)qt * 16 * S + k0 + (2 * st + kk) * 16 + 4 * g);
    };
    if constexpr (BIAS && !BIAS_LATE) load_bias();
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        sc[qt][kk] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        dp[qt][kk] = f32x4_t{-dlt[qt], -dlt[qt], -dlt[qt], -dlt[qt]};
      }
    if (prio) __builtin_amdgcn_s_setprio(1);
    if constexpr (DKV_PF > 0 && HALVES == 1) {   // fenced prefetch as in dkv_chunk, steps t = ds * 2 + kk (the
      // two-half 64-key tile variants spill with it)
      constexpr int NB = DKV_PF + 1, NT = G::DS * 2;
      bf16x8_t kf[NB], vf[NB];
      auto ld = [&](int t) {
        kf[t % NB] = row_frag<D>(sK, (2 * st + (t & 1)) * 16, t >> 1, lane);
        vf[t % NB] = row_frag<D>(sV, (2 * st + (t & 1)) * 16, t >> 1, lane);
      };
#pragma unroll
      for (int t = 0; t < DKV_PF; ++t) ld(t);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (t + DKV_PF < NT) ld(t + DKV_PF);
        __builtin_amdgcn_sched_barrier(0);
        const int ds = t >> 1, kk = t & 1;
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          sc[qt][kk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[t % NB], qf[qt][ds], sc[qt][kk], 0, 0, 0);
          dp[qt][kk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[t % NB], df[qt][ds], dp[qt][kk], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
    for (int ds = 0; ds < G::DS; ++ds) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int kt = 2 * st + kk;
        bf16x8_t kf = row_frag<D>(sK, kt * 16, ds, lane);
        bf16x8_t vf = row_frag<D>(sV, kt * 16, ds, lane);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          sc[qt][kk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qt][ds], sc[qt][kk], 0, 0, 0);
          dp[qt][kk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, df[qt][ds], dp[qt][kk], 0, 0, 0);
        }
      }
    }
    }
    if (prio) __builtin_amdgcn_s_setprio(0);
    if constexpr (BIAS && BIAS_LATE) load_bias();
    bf16x8_t sf[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int q = qw + qt * 16 + i;
      const float nl = -lse2[qt];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          float x = __builtin_fmaf(sc[qt][kk][v], c2, nl);
          if constexpr (BIAS) x = __builtin_fmaf(bv[qt][kk][v], LOG2E, x);
          float p = fexp2(x);
          if (MASK) {
            const int key = k0 + (2 * st + kk) * 16 + 4 * g + v;
            p = (key >= S || (causal && key > q)) ? 0.f : p;
          }
          sc[qt][kk][v] = p * dp[qt][kk][v];
        }
      sf[qt] = pack_p(sc[qt][0], sc[qt][1]);
    }
    if (prio) __builtin_amdgcn_s_setprio(1);
    if constexpr (DKV_PF > 0 && HALVES == 1) {
      constexpr int NB = DKV_PF + 1;
      bf16x8_t kt[NB];
#pragma unroll
      for (int dt = 0; dt < DKV_PF; ++dt) kt[dt % NB] = tr_frag<D>(sK, st * 32, dt * 16, lane);
#pragma unroll
      for (int dt = 0; dt < G::DT; ++dt) {
        if (dt + DKV_PF < G::DT) kt[(dt + DKV_PF) % NB] = tr_frag<D>(sK, st * 32, (dt + DKV_PF) * 16, lane);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          acc[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kt[dt % NB], sf[qt], acc[dt][qt], 0, 0, 0);
      }
    } else {
#pragma unroll
    for (int dt = 0; dt < G::DT; ++dt) {
      bf16x8_t kf = tr_frag<D>(sK, st * 32, dt * 16, lane);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
        acc[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, sf[qt], acc[dt][qt], 0, 0, 0);
    }
    }
    if (prio) __builtin_amdgcn_s_setprio(0);
  }
}

// ----------------------------------------------------------------------------------------------------------------
// dQ: block = NW x 32 queries; recompute Sᵀ, Pᵀ, dPᵀ = V·dOᵀ, dSᵀ, dQᵀ += Kᵀ·dSᵀ. K/V tiles in an NS-deep LDS ring
// filled by LDS-DMA NS - 1 tiles ahead (NW = 8, NS = 3: one block per CU, every wave's DMA share of a tile is 4
// pieces, a tile has two tiles' time to land instead of one).
template <int D, int NW = 4, int NS = 2, int KT = 64, bool BIAS = false>
__global__ __launch_bounds__(NW * 64, 2) void attn_bwd_dq_kernel(AttnArgs a) {
  using G = Geo<D>;
  constexpr int TILE = KT * G::ROWB;                   // KT keys per K / V tile (64, or 32 in a 4-deep ring)
  constexpr int QB = 32 * NW;                          // queries per block
  constexpr int PPW = 2 * (TILE / 1024) / NW;          // LDS-DMA pieces per wave per stage (K + V)
  static_assert(NS == 2 || (2 * (TILE / 1024)) % NW == 0, "counted waits need an even piece split");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, i = lane & 15;
  const int nx = (a.S + QB - 1) / QB;
  int bx, bh;
  attn_block(nx, bx, bh);
  const int b = BIAS ? bh % a.B : bh / a.H, h = BIAS ? bh / a.B : bh % a.H;   // BIAS: batch-major (bias_order)
  const int qblk = (a.causal ? (nx - 1 - bx) : bx) * QB;  // heaviest first
  const int qw = qblk + w * 32;
  const long long base = (long long)b * a.S * a.ld + h * D;
  const long long base_o = (long long)b * a.S * a.ld_o + h * D;
  const int kend = a.causal ? min(a.S, qblk + QB) : a.S;
  const int nkb = (kend + KT - 1) / KT;
  // full K / V tiles from per-lane offsets computed once (see stage_full16_128); ragged ones through stage_rows
  constexpr bool FAST = D == 128 && (KT == 32 || KT == 64) && NW == 4 && DKV_FAST_STAGE;
  unsigned offk[2] = {0u, 0u};
  const int wu = __builtin_amdgcn_readfirstlane(w);
  if (FAST) lane_off16_128(offk, a.ld, lane);
  auto stage_kv = [&](char* dst, int kn) {
    kn = __builtin_amdgcn_readfirstlane(kn);
    if (FAST && (kn + 1) * KT <= a.S) {
      stage_full16_128<KT>(dst, a.K + base + (long long)kn * KT * a.ld, a.ld, offk, wu);
      stage_full16_128<KT>(dst + TILE, a.V + base + (long long)kn * KT * a.ld, a.ld, offk, wu);
    } else {
      stage_rows<D, KT, NW>(dst, a.K + base + (long long)kn * KT * a.ld, a.ld, a.S - kn * KT, tid);
      stage_rows<D, KT, NW>(dst + TILE, a.V + base + (long long)kn * KT * a.ld, a.ld, a.S - kn * KT, tid);
    }
  };
#pragma unroll
  for (int st = 0; st < NS - 1; ++st)
    if (st < nkb) stage_kv(smem + st * 2 * TILE, st);

  bf16x8_t qf[2][G::DS], df[2][G::DS];
  float lse2[2], dlt[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = qw + qt * 16 + i;
    const bool ok = q < a.S;
#pragma unroll
    for (int ds = 0; ds < G::DS; ++ds) {
      qf[qt][ds] = load_frag_g(a.Q + base + (long long)q * a.ld + ds * 32 + 8 * g, ok);
      df[qt][ds] = load_frag_g(a.dO + base_o + (long long)q * a.ld_o + ds * 32 + 8 * g, ok);
    }
    const long long si = ((long long)b * a.H + h) * a.S + (ok ? q : 0);
    lse2[qt] = a.LSE[si] * LOG2E;
    // delta = rowsum(dO * O), fused here (the dK/dV kernel runs after this one and reads it back): this lane holds
    // d = ds*32 + 8g + [0, 8) of query q; the 4 lanes g = 0..3 of the query are i, i+16, i+32, i+48
    float part = 0.f;
#pragma unroll
    for (int ds = 0; ds < G::DS; ++ds) {
      const bf16x8_t of = load_frag_g(a.O + base_o + (long long)q * a.ld_o + ds * 32 + 8 * g, ok);
#pragma unroll
      for (int j = 0; j < 8; ++j) part += (float)of[j] * (float)df[qt][ds][j];
    }
    part += __shfl_xor(part, 16, 64);
    part += __shfl_xor(part, 32, 64);
    dlt[qt] = part;
    if (ok && g == 0) a.delta[si] = part;
  }
  f32x4_t acc[G::DT][2];
#pragma unroll
  for (int dt = 0; dt < G::DT; ++dt) acc[dt][0] = acc[dt][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const float c2 = a.scale * LOG2E;
  const float* bq = BIAS ? a.bias + ((long long)h * a.S + qw + i) * a.S : nullptr;
  vm_wait<0>();   // staged tiles (asm LDS-DMA: the compiler does not track them) have landed
  __syncthreads();
  // key tiles in two branch-free runs: unmasked, then masked (the causal diagonal band of the whole block, and a ragged
  // last tile). A per-tile branch merged the dQ accumulators of its two arms (v_mov per tile); a tile past a wave's
  // queries contributes exactly zero under the mask, and the block waits for its slowest wave at every barrier anyway
  const int kbm = a.causal ? min(nkb, (qblk + 1) / KT) : ((nkb * KT > a.S) ? nkb - 1 : nkb);
  auto tile = [&](int kb, auto mk) {
    constexpr bool MK = decltype(mk)::value;
    const int k0 = kb * KT;
    const char* sK = smem + (kb % NS) * 2 * TILE;
    const char* sV = sK + TILE;
    const int kn = kb + NS - 1;   // tile issued now; its slot was last read in iteration kb - 1 (behind a barrier)
    if (kn < nkb) stage_kv(smem + (kn % NS) * 2 * TILE, kn);
    dq_tile<D, MK, KT / 32, BIAS>(sK, sV, qf, df, lse2, dlt, acc, k0, qw, a.S, a.causal, c2, lane, a.prio & 2, bq);
    // tile kb + 1 must have landed; tiles kb + 2 .. kb + NS - 2 may stay in flight across the barrier (counted
    // wait: the only vector-memory ops of this loop are the DMA pieces, PPW per wave per tile)
    const int ahead = min(NS - 2, nkb - 2 - kb);
    if (NS >= 4 && ahead >= 2) vm_wait<2 * PPW>();
    else if (NS >= 3 && ahead >= 1) vm_wait<PPW>();
    else vm_wait<0>();
    __syncthreads();
  };
  if (a.prio & 8) {   // A/B (OBST_ATTN_PRIO bit 3): the per-tile masked-or-not branch of rounds 1-3
    for (int kb = 0; kb < nkb; ++kb) {
      const int k0 = kb * KT;
      if ((a.causal && k0 + KT - 1 > qw) || k0 + KT > a.S) tile(kb, std::true_type{});
      else tile(kb, std::false_type{});
    }
  } else {
    for (int kb = 0; kb < kbm; ++kb) tile(kb, std::false_type{});
    for (int kb = kbm; kb < nkb; ++kb) tile(kb, std::true_type{});
  }
  if constexpr (D == 128 && NW * 32 * 256 <= NS * 2 * TILE) {   // dQ through LDS as whole rows (epi_put)
    char* so = smem + w * 32 * 256;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int dt = 0; dt < G::DT; ++dt) epi_put(so, qt * 16 + i, dt, g, acc[dt][qt], a.scale);
    __syncthreads();
    const int c = lane & 15;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int rr = it * 4 + (lane >> 4), q = qw + rr;
      const uint4 v = epi_get(so, rr, c);
      if (q < a.S) *reinterpret_cast<uint4*>(a.dQ + base + (long long)q * a.ld + c * 8) = v;
    }
  } else {
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = qw + qt * 16 + i;
    if (q >= a.S) continue;
#pragma unroll
    for (int dt = 0; dt < G::DT; ++dt) {
      const int d = dt * 16 + 4 * g;
      const float sc = a.scale;
      *reinterpret_cast<uint2*>(a.dQ + base + (long long)q * a.ld + d) =
          make_uint2(pack_bf16x2(acc[dt][qt][0] * sc, acc[dt][qt][1] * sc), pack_bf16x2(acc[dt][qt][2] * sc, acc[dt][qt][3] * sc));
    }
  }
  }
}

// one 64-query chunk of the dK/dV kernel for a wave's KG groups of 16 keys (key on the lane: S = Q·Kᵀ, P and dS feed
// dVᵀ and dKᵀ as B operands straight from the accumulators). dP starts from -delta[q] (read from LDS as one f32x4 per
// tile). Every Q / dO fragment read from LDS feeds KG MFMAs: with KG = 2 the LDS bytes per MFMA halve (at KG = 1 the
// 104 LDS reads of a chunk take ~2300 LDS cycles per CU against ~2050 MFMA cycles per SIMD: LDS-bound).
// BIAS (biased_softmax, KG = 1): bcol / dcol = this head's [S][S] map and this batch's partial map gradient (uniform
// bases, 32-bit per-lane offsets q * S + key). The 16 map values of a chunk (queries 4g + v of each 16-query tile) are loaded before the score MFMAs;
// dS is stored to dcol for every query of the chunk (masked entries as 0) -- the dK/dV kernel visits every (query,
// key) pair of the causal triangle exactly once per batch, so the partial maps need no zeroing or accumulation
template <int D, bool MASK, int KG, int NQT = 4, bool BIAS = false>
__device__ __forceinline__ void dkv_chunk(const char* sQ, const char* sD, const float* sL, const float* sDl,
                                          const bf16x8_t (&kf)[KG][Geo<D>::DS], const bf16x8_t (&vf)[KG][Geo<D>::DS],
                                          f32x4_t (&dk)[KG][Geo<D>::DT], f32x4_t (&dv)[KG][Geo<D>::DT], int q0,
                                          int key, int S, int causal, float c2, int lane, int prio,
                                          const float* bcol = nullptr, float* dcol = nullptr) {
  using G = Geo<D>;
  static_assert(!BIAS || KG == 1, "the map hook covers one 16-key group per wave");
  const int g = lane >> 4;
  f32x4_t sc[KG][NQT], dp[KG][NQT];
  float bv[BIAS ? NQT : 1][4];
  // buffer accesses: one lane offset for the whole kernel ((4g S + key) * 4 bytes) plus a uniform SGPR offset per
  // (tile, row) -- no per-access 64-bit address registers in a kernel already at 256 VGPRs
  const int voff = (4 * g * S + key) * 4;
  const int nrec = S * S * 4;
  auto load_bias = [&]() {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bcol), 0, nrec, 0x00020000);
#pragma unroll
    for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        bv[qt][v] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, (q0 + qt * 16 + v) * S * 4, 0));
  };
  if constexpr (BIAS && !BIAS_LATE) load_bias();
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt) {
    const float4 dl = *reinterpret_cast<const float4*>(sDl + qt * 16 + 4 * g);
#pragma unroll
    for (int j = 0; j < KG; ++j) {
      sc[j][qt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      dp[j][qt] = f32x4_t{-dl.x, -dl.y, -dl.z, -dl.w};
    }
  }
  if (prio) __builtin_amdgcn_s_setprio(1);
  if constexpr (DKV_SPF > 0) {
    // flat step sequence t = ds * NQT + qt, Q / dO fragments read SPF steps ahead behind scheduling fences
    constexpr int SPF = DKV_SPF;
    constexpr int NB = SPF + 1, NT = G::DS * NQT;
    bf16x8_t qa[NB], da[NB];
    auto ld = [&](int t) {
      qa[t % NB] = row_frag<D>(sQ, (t % NQT) * 16, t / NQT, lane);
      da[t % NB] = row_frag<D>(sD, (t % NQT) * 16, t / NQT, lane);
    };
#pragma unroll
    for (int t = 0; t < SPF; ++t) ld(t);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (t + SPF < NT) ld(t + SPF);
      __builtin_amdgcn_sched_barrier(0);
      const int ds = t / NQT, qt = t % NQT;
#pragma unroll
      for (int j = 0; j < KG; ++j) {
        sc[j][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[t % NB], kf[j][ds], sc[j][qt], 0, 0, 0);
        dp[j][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da[t % NB], vf[j][ds], dp[j][qt], 0, 0, 0);
      }
    }
  } else {
#pragma unroll
  for (int ds = 0; ds < G::DS; ++ds) {
#pragma unroll
    for (int qt = 0; qt < NQT; ++qt) {
      bf16x8_t qa = row_frag<D>(sQ, qt * 16, ds, lane);
      bf16x8_t da = row_frag<D>(sD, qt * 16, ds, lane);
#pragma unroll
      for (int j = 0; j < KG; ++j) {
        sc[j][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[j][ds], sc[j][qt], 0, 0, 0);
        dp[j][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, vf[j][ds], dp[j][qt], 0, 0, 0);
      }
    }
  }
  }
  if (prio) __builtin_amdgcn_s_setprio(0);
  if constexpr (BIAS && BIAS_LATE) load_bias();
  // sc[j][qt][v] = S[q = q0 + qt*16 + 4g + v][key + 16 j]
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt) {
    const float4 lv = *reinterpret_cast<const float4*>(sL + qt * 16 + 4 * g);
    const float nl[4] = {-lv.x * LOG2E, -lv.y * LOG2E, -lv.z * LOG2E, -lv.w * LOG2E};
#pragma unroll
    for (int j = 0; j < KG; ++j)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float x = __builtin_fmaf(sc[j][qt][v], c2, nl[v]);
        if constexpr (BIAS) x = __builtin_fmaf(bv[qt][v], LOG2E, x);
        float pv = fexp2(x);
        if (MASK) {
          const int q = q0 + qt * 16 + 4 * g + v, kj = key + 16 * j;
          pv = (q >= S || kj >= S || (causal && kj > q)) ? 0.f : pv;
        }
        sc[j][qt][v] = pv;
        dp[j][qt][v] = pv * dp[j][qt][v];
        if constexpr (BIAS) {
          // a plain store: the raw_buffer_store builtin with per-row SGPR offsets compiled to one value stored to all
          // four rows of a lane (ROCm 7.2 clang; the loads above are unaffected -- checked in the device assembly)
          char* row = reinterpret_cast<char*>(dcol + (long long)(q0 + qt * 16 + v) * S);
          *reinterpret_cast<float*>(row + (unsigned)voff) = dp[j][qt][v];
        }
      }
  }
  if (prio) __builtin_amdgcn_s_setprio(1);
  if constexpr (DKV_UPF > 0) {   // update steps t = st * DT + dt, transposed operands UPF steps ahead
    constexpr int UPF = DKV_UPF;
    constexpr int NB = UPF + 1, NT = NQT / 2 * G::DT;
    bf16x8_t dot[NB], qtr[NB], pb[KG], sb[KG];
    auto ld = [&](int t) {
      dot[t % NB] = tr_frag<D>(sD, (t / G::DT) * 32, (t % G::DT) * 16, lane);
      qtr[t % NB] = tr_frag<D>(sQ, (t / G::DT) * 32, (t % G::DT) * 16, lane);
    };
#pragma unroll
    for (int t = 0; t < UPF; ++t) ld(t);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int st = t / G::DT, dt = t % G::DT;
      if (t + UPF < NT) ld(t + UPF);
      if (dt == 0)
#pragma unroll
        for (int j = 0; j < KG; ++j) {
          pb[j] = pack_p(sc[j][2 * st], sc[j][2 * st + 1]);
          sb[j] = pack_p(dp[j][2 * st], dp[j][2 * st + 1]);
        }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < KG; ++j) {
        dv[j][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dot[t % NB], pb[j], dv[j][dt], 0, 0, 0);
        dk[j][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qtr[t % NB], sb[j], dk[j][dt], 0, 0, 0);
      }
    }
    if (prio) __builtin_amdgcn_s_setprio(0);
    return;
  }
#pragma unroll
  for (int st = 0; st < NQT / 2; ++st) {
    bf16x8_t pb[KG], sb[KG];
#pragma unroll
    for (int j = 0; j < KG; ++j) {
      pb[j] = pack_p(sc[j][2 * st], sc[j][2 * st + 1]);
      sb[j] = pack_p(dp[j][2 * st], dp[j][2 * st + 1]);
    }
#pragma unroll
    for (int dt = 0; dt < G::DT; ++dt) {
      bf16x8_t dot = tr_frag<D>(sD, st * 32, dt * 16, lane);
      bf16x8_t qtr = tr_frag<D>(sQ, st * 32, dt * 16, lane);
#pragma unroll
      for (int j = 0; j < KG; ++j) {
        dv[j][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dot, pb[j], dv[j][dt], 0, 0, 0);
        dk[j][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qtr, sb[j], dk[j][dt], 0, 0, 0);
      }
    }
  }
  if (prio) __builtin_amdgcn_s_setprio(0);
}

// ----------------------------------------------------------------------------------------------------------------
// dK/dV: block = NW x KG x 16 keys; wave w owns keys k0 + 16 KG w + [0, 16 KG). Loop over 64-query chunks (Q, dO, lse,
// delta) in an NS-deep LDS ring filled by LDS-DMA NS - 1 chunks ahead. KG = 2 holds ~300 registers: one wave per SIMD.
template <int D, int NW = 4, int NS = 2, int KG = 1, int QC = 64, bool BIAS = false>
__global__ __launch_bounds__(NW * 64, KG == 1 ? 2 : 1) void attn_bwd_dkv_kernel(AttnArgs a) {
  using G = Geo<D>;
  constexpr int TILE = QC * G::ROWB;
  constexpr int STAGE = 2 * TILE + 2 * 256;   // Q, dO, lse[64], delta[64]
  constexpr int KW = 16 * KG;                 // keys per wave
  constexpr int KB = KW * NW;                 // keys per block
  constexpr int PPW = 2 * (TILE / 1024) / NW; // Q + dO pieces per wave per stage (+1 on waves 0 / 1: lse / delta)
  static_assert(NS == 2 || (2 * (TILE / 1024)) % NW == 0, "counted waits need an even piece split");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, i = lane & 15;
  int bx, bh;
  attn_block((a.S + KB - 1) / KB, bx, bh);
  const int b = BIAS ? bh % a.B : bh / a.H, h = BIAS ? bh / a.B : bh % a.H;   // BIAS: batch-major (bias_order)
  const int kblk = bx * KB;
  const int kw = kblk + w * KW;
  const long long base = (long long)b * a.S * a.ld + h * D;
  const long long base_o = (long long)b * a.S * a.ld_o + h * D;
  const long long sbase = ((long long)b * a.H + h) * a.S;
  const int qstart = a.causal ? (kblk / QC) * QC : 0;
  const int nqc = (a.S - qstart + QC - 1) / QC;

  constexpr bool FAST = D == 128 && QC == 64 && NW == 4 && DKV_FAST_STAGE;
  unsigned offq[2] = {0u, 0u}, offo[2] = {0u, 0u};
  const int wu = __builtin_amdgcn_readfirstlane(w);
  if (FAST) {
    lane_off16_128(offq, a.ld, lane);
    lane_off16_128(offo, a.ld_o, lane);
  }
  auto stage = [&](char* st, int q0) {
    q0 = __builtin_amdgcn_readfirstlane(q0);
    if (FAST && q0 + QC <= a.S) {
      stage_full16_128(st, a.Q + base + (long long)q0 * a.ld, a.ld, offq, wu);
      stage_full16_128(st + TILE, a.dO + base_o + (long long)q0 * a.ld_o, a.ld_o, offo, wu);
    } else {
      stage_rows<D, QC, NW>(st, a.Q + base + (long long)q0 * a.ld, a.ld, a.S - q0, tid);
      stage_rows<D, QC, NW>(st + TILE, a.dO + base_o + (long long)q0 * a.ld_o, a.ld_o, a.S - q0, tid);
    }
    if (NW == 4) {   // wave 0 stages both
      stage_f32(st + 2 * TILE, a.LSE + sbase + q0, QC, a.S - q0, tid);
      stage_f32(st + 2 * TILE + 256, a.delta + sbase + q0, QC, a.S - q0, tid);
    } else {         // wave 0: lse, wave 1: delta (one extra piece each)
      stage_f32(st + 2 * TILE, a.LSE + sbase + q0, QC, a.S - q0, tid);
      stage_f32(st + 2 * TILE + 256, a.delta + sbase + q0, QC, a.S - q0, tid - 64);
    }
  };
#pragma unroll
  for (int c = 0; c < NS - 1; ++c)
    if (c < nqc) stage(smem + c * STAGE, qstart + c * QC);

  bf16x8_t kf[KG][G::DS], vf[KG][G::DS];
#pragma unroll
  for (int j = 0; j < KG; ++j) {
    const int key = kw + 16 * j + i;
    const bool ok = key < a.S;
#pragma unroll
    for (int ds = 0; ds < G::DS; ++ds) {
      kf[j][ds] = load_frag_g(a.K + base + (long long)key * a.ld + ds * 32 + 8 * g, ok);
      vf[j][ds] = load_frag_g(a.V + base + (long long)key * a.ld + ds * 32 + 8 * g, ok);
    }
  }
  f32x4_t dk[KG][G::DT], dv[KG][G::DT];
#pragma unroll
  for (int j = 0; j < KG; ++j)
#pragma unroll
    for (int dt = 0; dt < G::DT; ++dt) dk[j][dt] = dv[j][dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const float c2 = a.scale * LOG2E;
  const int key = kw + i;
  const float* bcol = BIAS ? a.bias + (long long)h * a.S * a.S : nullptr;
  float* dcol = BIAS ? a.dbias + ((long long)b * a.H + h) * a.S * a.S : nullptr;
  vm_wait<0>();   // staged tiles (asm LDS-DMA: the compiler does not track them) have landed
  __syncthreads();
  // Chunks in three branch-free runs: masked (causal diagonal band of the whole block, or every chunk when the block's
  // keys run past S), unmasked, masked (a ragged last chunk). A per-chunk masked / unmasked branch merged the dK / dV
  // accumulators of its two arms: 64 v_mov per chunk in a VALU-bound kernel (profiles/r3_attn_bwd_ab.md). A chunk
  // entirely before a wave's keys contributes exactly zero under the mask, so no per-wave skip either.
  const bool all_mask = kblk + KB > a.S;
  const int c_diag = a.causal ? min(nqc, (kblk + KB - 1 - qstart + QC - 1) / QC) : 0;
  const int cm1 = all_mask ? nqc : c_diag;
  const int cm2 = all_mask ? nqc : max(cm1, (qstart + nqc * QC > a.S) ? nqc - 1 : nqc);
  auto chunk = [&](int c, auto mk) {
    constexpr bool MK = decltype(mk)::value;
    const int q0 = qstart + c * QC;
    const char* sQ = smem + (c % NS) * STAGE;
    const char* sD = sQ + TILE;
    const float* sL = reinterpret_cast<const float*>(sQ + 2 * TILE);
    const float* sDl = sL + 64;
    const int cn = c + NS - 1;
    if (cn < nqc) stage(smem + (cn % NS) * STAGE, qstart + cn * QC);
    dkv_chunk<D, MK, KG, QC / 16, BIAS>(sQ, sD, sL, sDl, kf, vf, dk, dv, q0, key, a.S, a.causal, c2, lane,
                                        a.prio & 1, bcol, dcol);
    // chunk c + 1 must have landed; chunks c + 2 .. c + NS - 2 may stay in flight across the barrier. Per chunk a
    // wave issues PPW pieces, plus the lse / delta pieces: NW = 4 wave 0 issues both, NW = 8 waves 0 and 1 one each
    const int ahead = min(NS - 2, nqc - 2 - c);
    constexpr int X0 = NW == 4 ? 2 : 1;
    const bool extra = NW == 4 ? w == 0 : w < 2;
    if (NS >= 4 && ahead >= 2) {
      if (extra) vm_wait<2 * (PPW + X0)>();
      else vm_wait<2 * PPW>();
    } else if (NS >= 3 && ahead >= 1) {
      if (extra) vm_wait<PPW + X0>();
      else vm_wait<PPW>();
    } else {
      vm_wait<0>();
    }
    __syncthreads();
  };
  if (a.prio & 8) {   // A/B (OBST_ATTN_PRIO bit 3): the per-chunk masked-or-not branch of rounds 1-3
    for (int c = 0; c < nqc; ++c) {
      const int q0 = qstart + c * QC;
      if ((a.causal && q0 < kw + KW - 1) || q0 + QC > a.S || kw + KW > a.S) chunk(c, std::true_type{});
      else chunk(c, std::false_type{});
    }
  } else {
    for (int c = 0; c < cm1; ++c) chunk(c, std::true_type{});
    for (int c = cm1; c < cm2; ++c) chunk(c, std::false_type{});
    for (int c = cm2; c < nqc; ++c) chunk(c, std::true_type{});
  }
  if constexpr (D == 128 && NW * 2 * KW * 256 <= NS * STAGE) {   // dK, dV through LDS as whole rows (epi_put)
    char* sk = smem + w * 2 * KW * 256;
    char* sv = sk + KW * 256;
#pragma unroll
    for (int j = 0; j < KG; ++j)
#pragma unroll
      for (int dt = 0; dt < G::DT; ++dt) {
        epi_put(sk, 16 * j + i, dt, g, dk[j][dt], a.scale);
        epi_put(sv, 16 * j + i, dt, g, dv[j][dt], 1.f);
      }
    __syncthreads();
    const int c = lane & 15;
#pragma unroll
    for (int it = 0; it < KW / 4; ++it) {
      const int rr = it * 4 + (lane >> 4), kj = kw + rr;
      const uint4 vk = epi_get(sk, rr, c), vv = epi_get(sv, rr, c);
      if (kj < a.S) {
        *reinterpret_cast<uint4*>(a.dK + base + (long long)kj * a.ld + c * 8) = vk;
        *reinterpret_cast<uint4*>(a.dV + base + (long long)kj * a.ld + c * 8) = vv;
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < KG; ++j) {
    const int kj = key + 16 * j;
    if (kj < a.S) {
#pragma unroll
      for (int dt = 0; dt < G::DT; ++dt) {
        const int d = dt * 16 + 4 * g;
        const float sc = a.scale;
        *reinterpret_cast<uint2*>(a.dK + base + (long long)kj * a.ld + d) =
            make_uint2(pack_bf16x2(dk[j][dt][0] * sc, dk[j][dt][1] * sc), pack_bf16x2(dk[j][dt][2] * sc, dk[j][dt][3] * sc));
        *reinterpret_cast<uint2*>(a.dV + base + (long long)kj * a.ld + d) =
            make_uint2(pack_bf16x2(dv[j][dt][0], dv[j][dt][1]), pack_bf16x2(dv[j][dt][2], dv[j][dt][3]));
      }
    }
  }
}

// ================================================================================================================
// D = 128 forward with v_mfma_f32_32x32x16_bf16 (cdna_hip_programming.md Appendix B "Fused attention prefill").
// A 32x32x16 MFMA holds the SIMD's vector issue for 8 of its 32 cycles (16x16x32: 8 of 16), so the softmax VALU
// work of one wave fits in the MFMA gaps of its partner; the per-query row reductions shrink to 31 local ops + one
// v_permlane32_swap. Sᵀ = K·Qᵀ keeps the query on the lane: lane (h = lane>>5, n = lane&31) holds, for query n,
// keys 8a + 4h + b (register 4a + b) of every 32-key sub-tile. Those registers, bf16-packed 8 at a time, are the
// B operand of P·V directly (k-step s of a sub-tile = registers 8s..8s+7); the A operand Vᵀ is read from the same
// swizzled [key][d] LDS image with ds_read_b64_tr_b16 in that key order, so P never crosses lanes.
#ifndef FWD_KPF
#define FWD_KPF 2
#endif
#ifndef FWD_KPF_FENCE
#define FWD_KPF_FENCE 1
#endif

// one 64-key tile for a wave's 32 queries (query n = lane&31 is `q`); l is this lane's partial row sum
// BIAS (biased_softmax, ref src/model/spatial.py:65-66,74-75; 32-key tiles): bv holds this lane's 16 map values of
// the tile (keys 8a + 4h + b of its query row, loaded one tile ahead by the kernel), added to the scaled logits after
// the score MFMAs, so the softmax below runs on scale q.k + b (in log2 units)
template <bool MASK, int NKT = 2, bool BIAS = false>
__device__ __forceinline__ void fwd32_tile(const char* sK, const char* sV, const bf16x8_t (&qf)[8],
                                           f32x16_t (&o)[4], float& m, float& l, int k0, int q, int S, int causal,
                                           float c2, int lane, int prio, const f32x4_t (&bv)[4]) {
  static_assert(!BIAS || NKT == 1, "the map hook runs on 32-key tiles");
  const int h = lane >> 5;
  Frag32 fo;
  frag32_offsets(fo, lane);
  f32x16_t s[NKT];
  if (prio) __builtin_amdgcn_s_setprio(1);
  // the NKT score chains interleaved k-step by k-step, K fragments read FWD_KPF k-steps ahead of their MFMA: with
  // one chain at a time the compiler re-used one fragment register and every MFMA waited out a full LDS read
  constexpr int PF = FWD_KPF;
  bf16x8_t kf[PF + 1][NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) s[kt] = f32x16_t{};
#pragma unroll
  for (int ks = 0; ks < PF; ++ks)
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
      kf[ks][kt] = *reinterpret_cast<const bf16x8_t*>(sK + fo.k[ks] + kt * 32 * 256);
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    if (ks + PF < 8)
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
        kf[(ks + PF) % (PF + 1)][kt] = *reinterpret_cast<const bf16x8_t*>(sK + fo.k[ks + PF] + kt * 32 * 256);
    // fence: the scheduler would otherwise sink each read next to its MFMA (one fragment register, no prefetch)
    if (FWD_KPF_FENCE) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
      s[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[ks % (PF + 1)][kt], qf[ks], s[kt], 0, 0, 0);
  }
  if (prio) __builtin_amdgcn_s_setprio(0);
  if constexpr (BIAS) {   // logits in log2 units: scale q.k log2(e) + b log2(e); the softmax below then takes c2 = 1
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kt][r] = __builtin_fmaf(s[kt][r], c2, bv[kt * 4 + (r >> 2)][r & 3] * LOG2E);
    c2 = 1.f;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (MASK) {
        const int key = k0 + kt * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
        s[kt][r] = (key >= S || (causal && key > q)) ? -INFINITY : s[kt][r];
      }
      mx = fmaxf(mx, s[kt][r]);
    }
  mx = xh_max(mx);
  const float ms = mx * c2;
  const bool bump = ms > m + RESCALE_TH;
  if (__builtin_amdgcn_ballot_w64(bump)) {
    const float mn = bump ? ms : m;
    const float alpha = fexp2(m - mn);
    l *= alpha;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
    m = mn;
  }
  const float nm = -m;
  float rs = 0.f;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = fexp2(__builtin_fmaf(s[kt][r], c2, nm));
      s[kt][r] = p;
      rs += p;
    }
  l += rs;
  if (prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const bf16x8_t pf = pack8(s[kt], 8 * st);
      const int kb = (kt * 32 + 16 * st) * 256;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_pair(sV, fo.v[dt][0] + kb, fo.v[dt][1] + kb), pf, o[dt],
                                                        0, 0, 0);
    }
  if (prio) __builtin_amdgcn_s_setprio(0);
}

// forward epilogue through LDS (whole-row 16-byte stores); 0: per-lane 8-byte stores at row stride (A/B)
#ifndef FWD_EPI_LDS
#define FWD_EPI_LDS 1
#endif

// block = 128 queries of one (b, h), wave w owns 32; K/V 64-key tiles double-buffered by LDS-DMA, one barrier/tile;
// the tile loop is unrolled by two so both buffers' fragment addresses are immediates
// KT = 32: 32-key tiles in a 4-deep ring (the same 64 KiB), the next three tiles in flight instead of one
// NW = 8: 256 queries per block, one block per CU -- the K/V tiles each CU streams from L2 halve (A/B knob)
template <int KT = 64, int NW = 4, bool BIAS = false>
__global__ __launch_bounds__(NW * 64, 8 / NW) void attn_fwd32_kernel(AttnArgs a) {
  constexpr int D = 128;
  constexpr int TILE = KT * 256;
  constexpr int NS = KT == 64 ? 2 : 4;
  constexpr int NP = KT / 4 / NW;     // LDS-DMA pieces per wave per K (or V) tile
  constexpr int QB = 32 * NW;         // queries per block
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, n = lane & 31;
  const int nx = (a.S + QB - 1) / QB;
  int bx, bh;
  attn_block(nx, bx, bh);
  const int b = BIAS ? bh % a.B : bh / a.H, hd = BIAS ? bh / a.B : bh % a.H;   // BIAS: batch-major (bias_order)
  const int qblk = (a.causal ? (nx - 1 - bx) : bx) * QB;
  const int qw = qblk + w * 32;
  const int q = qw + n;
  const long long base = (long long)b * a.S * a.ld + hd * D;
  const bf16_t* Kb = a.K + base;
  const bf16_t* Vb = a.V + base;
  const int kend = a.causal ? min(a.S, qblk + QB) : a.S;
  const int nkb = (kend + KT - 1) / KT;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  unsigned soff[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int row = (wu + NW * i) * 4 + (lane >> 4);
    soff[i] = (unsigned)(row * (int)a.ld + (((lane & 15) ^ swz<128>(row)) << 3)) * 2u;
  }
  auto stage = [&](char* buf, int k0) {
    k0 = __builtin_amdgcn_readfirstlane(k0);
    if (k0 + KT <= a.S) {
      stage_full64<NP, NW>(buf, Kb + (long long)k0 * a.ld, soff, wu);
      stage_full64<NP, NW>(buf + TILE, Vb + (long long)k0 * a.ld, soff, wu);
    } else {
      stage_rows64_asm<NP, NW>(buf, Kb + (long long)k0 * a.ld, a.ld, a.S - k0, wu, lane);
      stage_rows64_asm<NP, NW>(buf + TILE, Vb + (long long)k0 * a.ld, a.ld, a.S - k0, wu, lane);
    }
  };
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nkb) stage(smem + t * 2 * TILE, t * KT);
  bf16x8_t qf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) qf[ks] = load_frag_g(a.Q + base + (long long)q * a.ld + ks * 16 + 8 * h, q < a.S);
  // consume Q here so the compiler's own vmcnt wait for it lands in the prologue, not in front of the first MFMA
  // of every tile (where it would also wait for the next tile's in-flight DMA)
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) asm volatile("" ::"v"(qf[ks]));
  f32x16_t o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x16_t{};
  float m = NEG_BIG, l = 0.f;
  const float c2 = a.scale * LOG2E;
  // BIAS: this lane's query row of the map (rows past S read the last row; their outputs are not stored). The 16
  // values of tile kb + 1 are loaded during tile kb by inline asm, ahead of that iteration's K/V DMA: a compiler-
  // visible load would get a vmcnt wait in front of its first use that also drains the K/V DMA issued after it (the
  // compiler does not count the asm LDS-DMA), i.e. every tile would wait for the tile three ahead to land. The
  // iteration's closing wait covers them instead (only the newer DMA of tile kb + 3 may stay in flight).
  const float* brow = BIAS ? a.bias + ((long long)hd * a.S + min(q, a.S - 1)) * a.S + 4 * h : nullptr;
  f32x4_t bcur[4], bnx[4];
  auto bias_load = [&](f32x4_t (&dst)[4], int k0) {
    if constexpr (BIAS) {
      const float* p = brow + k0;
      asm volatile(
          "global_load_dwordx4 %0, %4, off\n\t"
          "global_load_dwordx4 %1, %4, off offset:32\n\t"
          "global_load_dwordx4 %2, %4, off offset:64\n\t"
          "global_load_dwordx4 %3, %4, off offset:96"
          : "=&v"(dst[0]), "=&v"(dst[1]), "=&v"(dst[2]), "=&v"(dst[3])
          : "v"(p)
          : "memory");
    }
  };
  auto bias_pin = [&](f32x4_t (&r)[4]) {   // after the wait: the values are in place from here on
    if constexpr (BIAS) {
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(r[i]));
    }
  };
  if constexpr (BIAS) {
    static_assert(KT == 32 && NS == 4, "the map pipeline is laid out for the 32-key, 4-deep ring");
    bias_load(bcur, 0);   // (issued after the prologue's DMA: the wait below covers both)
  }
  vm_wait<0>();
  bias_pin(bcur);
  __syncthreads();
  // key tiles in two branch-free runs, unmasked then the block's masked band (as in the backward kernels): the
  // per-tile branch merged O, m and l of its two arms. Fully masked tiles of the lower waves add exactly nothing (the
  // first tile, key 0, makes every row's running max finite) and run while those waves would wait at the barrier.
  const int kbm = a.causal ? min(nkb, (qblk + 1) / KT) : ((nkb * KT > a.S) ? nkb - 1 : nkb);
  // the ring step of iteration kb: (BIAS: map values of tile kb + 1,) the DMA of tile kb + NS - 1, [the tile's work],
  // then the wait for tile kb + 1 (and its map values) and the barrier
  auto issue = [&](int kb) {
    bias_load(bnx, min(kb + 1, nkb - 1) * KT);
    const int kn = kb + NS - 1;   // its slot was last read in iteration kb - 1 (behind the barrier)
    if (kn < nkb) stage(smem + (kn % NS) * 2 * TILE, kn * KT);
  };
  auto retire = [&](int kb) {
    if constexpr (BIAS) {   // the map loads sit between tile kb + 2's DMA and tile kb + 3's: only the latter may stay
      if (kb + NS - 1 < nkb) vm_wait<2 * NP>();
      else vm_wait<0>();
      bias_pin(bnx);   // (ordered after the wait: the copy below cannot be hoisted above it)
#pragma unroll
      for (int i = 0; i < 4; ++i) bcur[i] = bnx[i];
    } else {
      // tile kb + 1 has landed; tiles kb + 2 .. kb + NS - 2 may stay in flight (2 NP pieces per wave per tile)
      const int ahead = min(NS - 2, nkb - 2 - kb);
      if (NS >= 4 && ahead >= 2) vm_wait<4 * NP>();
      else if (NS >= 3 && ahead >= 1) vm_wait<2 * NP>();
      else vm_wait<0>();
    }
    __syncthreads();
  };
  auto tile = [&](int kb, auto mk) {
    constexpr bool MK = decltype(mk)::value;
    const int k0 = kb * KT;
    const char* sK = smem + (kb % NS) * 2 * TILE;
    const char* sV = sK + TILE;
    issue(kb);
    fwd32_tile<MK, KT / 32, BIAS>(sK, sV, qf, o, m, l, k0, q, a.S, a.causal, c2, lane, a.prio & 4, bcur);
    retire(kb);
  };
  if (!(a.prio & 16)) {   // default: the per-tile branch with its skip of the tiles past a wave's queries (bit 4,
    // the branch-free runs, measured within 1 %: profiles/r4_attn_branchfree_ab.txt)
    for (int kb = 0; kb < nkb; ++kb) {
      const int k0 = kb * KT;
      if (a.causal && k0 > qw + 31) {   // nothing of this tile for this wave: keep the ring's staging and barrier
        issue(kb);
        retire(kb);
      } else if ((a.causal && k0 + KT - 1 > qw) || k0 + KT > a.S) {
        tile(kb, std::true_type{});
      } else {
        tile(kb, std::false_type{});
      }
    }
  } else {
    for (int kb = 0; kb < kbm; ++kb) tile(kb, std::false_type{});
    for (int kb = kbm; kb < nkb; ++kb) tile(kb, std::true_type{});
  }
  l = xh_sum(l);
  const float inv = 1.f / l;
  if (q < a.S && h == 0) a.LSE[((long long)b * a.H + hd) * a.S + q] = (m + __log2f(l)) / LOG2E;
  if (FWD_EPI_LDS && NW * 32 * 256 <= NS * 2 * TILE) {
    // O through LDS, stored as whole rows: the lane's 64 values are 16 pieces of 8 bytes at row stride (each store
    // instruction touched 32 rows); staged in the wave's 8 KiB of the (now idle) K/V ring and read back as 16-byte
    // chunks, 16 lanes per 256-byte row, every store instruction writes 4 whole rows (and the residual add reads them
    // the same way). Image: row n, 16-byte chunk c at (c ^ (n & 7)), 8-byte half h at h ^ ((n >> 3) & 1) -- the 16
    // lanes of a ds_write_b64 group (rows n..n+15, one c, one h) hit 16 distinct 8-byte slots of 128 bytes.
    char* so = smem + w * 32 * 256;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int c = dt * 4 + g4;
        const uint2 v = make_uint2(pack_bf16x2(o[dt][4 * g4] * inv, o[dt][4 * g4 + 1] * inv),
                                   pack_bf16x2(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv));
        *reinterpret_cast<uint2*>(so + n * 256 + ((c ^ (n & 7)) << 4) + ((h ^ ((n >> 3) & 1)) << 3)) = v;
      }
    __syncthreads();
    const int c = lane & 15;
    const long long obase = (long long)b * a.S * a.ld_o + hd * D + c * 8;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int rr = it * 4 + (lane >> 4), qr = qw + rr;
      uint4 v = *reinterpret_cast<const uint4*>(so + rr * 256 + ((c ^ (rr & 7)) << 4));
      if ((rr >> 3) & 1) v = make_uint4(v.z, v.w, v.x, v.y);
      if (qr < a.S) {
        const long long off = obase + (long long)qr * a.ld_o;
        *reinterpret_cast<uint4*>(a.Oout + off) = v;
        if (a.Sum) {
          const uint4 r = *reinterpret_cast<const uint4*>(a.Res + off);
          const uint32_t ov[4] = {v.x, v.y, v.z, v.w}, rv[4] = {r.x, r.y, r.z, r.w};
          uint32_t sv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            sv[j] = pack_bf16x2(bf2f(ov[j] & 0xffff) + bf2f(rv[j] & 0xffff), bf2f(ov[j] >> 16) + bf2f(rv[j] >> 16));
          *reinterpret_cast<uint4*>(a.Sum + off) = make_uint4(sv[0], sv[1], sv[2], sv[3]);
        }
      }
    }
  } else if (q < a.S) {
    const long long orow = (long long)b * a.S * a.ld_o + hd * D + (long long)q * a.ld_o;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = dt * 32 + 8 * g4 + 4 * h;
        store_o4(a, orow + d, o[dt][4 * g4] * inv, o[dt][4 * g4 + 1] * inv, o[dt][4 * g4 + 2] * inv,
                 o[dt][4 * g4 + 3] * inv);
      }
  }
}

// Dispatch. D = 128 (every shipped config) takes the 32x32x16 forward and the dQ kernel over 32-key tiles in a 4-deep
// LDS-DMA ring; other head sizes take the 16x16x32 forward. Alternatives measured slower and removed in round 6 (the
// numbers stay in git history and profiles/): the one-wave-per-SIMD forward attn_fwd64 (1.76 vs 1.42 ms,
// profiles/r5_attn_fwd64.md), 8-wave forward / backward blocks with 3-deep rings (5.86 / 5.68 / 5.61 vs 5.23 ms), the
// 32x32x16 dK/dV kernel (3.71 vs 3.01 ms, profiles/r3_attn_bwd_ab.md), two 16-key groups per dK/dV wave (6.27 vs
// 5.24 ms), the forward over 32-key tiles (1.47 vs 1.37 ms) and dK/dV over 32-query chunks (5.59 vs 4.98 ms).
template <int D>
int launch_fwd(const AttnArgs& a, hipStream_t st) {
  dim3 grid((a.S + 127) / 128 * a.B * a.H);
  if (D == 128)
    hipLaunchKernelGGL(attn_fwd32_kernel<64>, grid, dim3(NTH), 2 * 2 * 64 * 256, st, a);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<D>, grid, dim3(NTH), 4 * 64 * Geo<D>::ROWB, st, a);
  return (int)hipGetLastError();
}

template <int D>
int launch_bwd(const AttnArgs& a, hipStream_t st) {
  // dQ first: it also produces delta = rowsum(dO * O), which the dK/dV kernel reads
  hipLaunchKernelGGL((attn_bwd_dq_kernel<D, 4, 4, 32>), dim3((a.S + 127) / 128 * a.B * a.H), dim3(NTH),
                     4 * 2 * 32 * Geo<D>::ROWB, st, a);
  hipLaunchKernelGGL(attn_bwd_dkv_kernel<D>, dim3((a.S + 63) / 64 * a.B * a.H), dim3(NTH),
                     2 * (2 * 64 * Geo<D>::ROWB + 512), st, a);
  return (int)hipGetLastError();
}

// dbias[h][q][k] = sum over b (in order) of part[b][h][q][k]; 0 above the diagonal when causal (never written there)
__global__ __launch_bounds__(NTH) void bias_fold_kernel(const float* __restrict__ part, float* __restrict__ out, int B,
                                                        long long n, int S, int causal) {
  for (long long v = (long long)blockIdx.x * NTH + threadIdx.x; v * 4 < n; v += (long long)gridDim.x * NTH) {
    const long long e = v * 4;
    const int k = (int)(e % S), q = (int)((e / S) % S);
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    if (!causal || k <= q) {
      for (int b = 0; b < B; ++b) acc += *reinterpret_cast<const f32x4_t*>(part + b * n + e);
      if (causal) {
#pragma unroll
        for (int j = 1; j < 4; ++j) acc[j] = k + j > q ? 0.f : acc[j];
      }
    }
    *reinterpret_cast<f32x4_t*>(out + e) = acc;
  }
}

}  // namespace

struct ObstAttnDesc {
  const void *Q, *K, *V, *O, *dO;
  void *Oout, *dQ, *dK, *dV;
  float *LSE, *delta;
  int B, S, H, D;
  long long ld;
  float scale;
  int causal;
  long long ld_o;   // 0: same as ld
  const void* Res;  // forward: optional residual input, Sum = bf16(O) + Res (O's layout)
  void* Sum;
};

static bool fill(AttnArgs& a, const ObstAttnDesc* d) {
  a.Q = (const bf16_t*)d->Q; a.K = (const bf16_t*)d->K; a.V = (const bf16_t*)d->V;
  a.O = (const bf16_t*)d->O; a.dO = (const bf16_t*)d->dO;
  a.Oout = (bf16_t*)d->Oout; a.dQ = (bf16_t*)d->dQ; a.dK = (bf16_t*)d->dK; a.dV = (bf16_t*)d->dV;
  a.LSE = d->LSE; a.delta = d->delta;
  a.B = d->B; a.S = d->S; a.H = d->H; a.ld = d->ld; a.scale = d->scale; a.causal = d->causal;
  a.ld_o = d->ld_o ? d->ld_o : d->ld;
  a.Res = (const bf16_t*)d->Res; a.Sum = (bf16_t*)d->Sum;
  a.bias = nullptr;
  a.dbias = nullptr;
  if ((a.Res == nullptr) != (a.Sum == nullptr)) return false;
  static const int prio = [] { const char* e = getenv("OBST_ATTN_PRIO"); return e ? atoi(e) : 3; }();
  a.prio = prio;
  return d->B > 0 && d->S > 0 && d->H > 0 && d->ld % 8 == 0 && d->ld >= (long long)d->H * d->D &&
         a.ld_o % 8 == 0 && a.ld_o >= (long long)d->H * d->D;
}

OBST_API int obst_attn_fwd(const ObstAttnDesc* d, hipStream_t st) {
  AttnArgs a;
  if (!fill(a, d)) return -1;
  switch (d->D) {
    case 32: return launch_fwd<32>(a, st);
    case 64: return launch_fwd<64>(a, st);
    case 96: return launch_fwd<96>(a, st);
    case 128: return launch_fwd<128>(a, st);
    default: return -2;
  }
}

// biased_softmax forward on the flash schedule (D = 128, S % 128 == 0): attn_fwd32_kernel over 32-key tiles in a
// 4-deep ring (185 VGPRs: room for the 16 map values per lane and tile that the 64-key kernel's 239 do not leave),
// the [H][S][S] fp32 map added to the scaled logits. O and LSE as the map kernels of attn_map.hip write them, so
// their backward consumes this forward unchanged.
OBST_API int obst_attn_fwd_bias(const ObstAttnDesc* d, const float* bias, hipStream_t st) {
  AttnArgs a;
  if (!fill(a, d) || d->D != 128 || !bias || d->S % 128 || a.Sum) return -1;
  a.bias = bias;
  dim3 grid(d->S / 128 * d->B * d->H);
  hipLaunchKernelGGL((attn_fwd32_kernel<32, 4, true>), grid, dim3(NTH), 4 * 2 * 32 * 256, st, a);
  return (int)hipGetLastError();
}

// biased_softmax backward on the flash schedule (D = 128, S % 128 == 0): the dQ and dK/dV kernels with the map hook;
// the dK/dV kernel writes dS per batch into part ([B][H][S][S] fp32, no zeroing needed), bias_fold_kernel sums the
// batches in order into dbias ([H][S][S]) -- deterministic, no atomics
OBST_API int obst_attn_bwd_bias(const ObstAttnDesc* d, const float* bias, float* part, float* dbias, hipStream_t st) {
  AttnArgs a;
  if (!fill(a, d) || d->D != 128 || !bias || !part || !dbias || d->S % 128) return -1;
  a.bias = bias;
  a.dbias = part;
  hipLaunchKernelGGL((attn_bwd_dq_kernel<128, 4, 4, 32, true>), dim3(d->S / 128 * d->B * d->H), dim3(NTH),
                     4 * 2 * 32 * Geo<128>::ROWB, st, a);
  hipLaunchKernelGGL((attn_bwd_dkv_kernel<128, 4, 2, 1, 64, true>), dim3(d->S / 64 * d->B * d->H), dim3(NTH),
                     2 * (2 * 64 * Geo<128>::ROWB + 512), st, a);
  const long long n = (long long)d->H * d->S * d->S;
  const long long nv = n / 4;
  const unsigned g = (unsigned)(nv / NTH + 1 < 8192 ? nv / NTH + 1 : 8192);
  hipLaunchKernelGGL(bias_fold_kernel, dim3(g), dim3(NTH), 0, st, part, dbias, d->B, n, d->S, d->causal);
  return (int)hipGetLastError();
}

OBST_API int obst_attn_bwd(const ObstAttnDesc* d, hipStream_t st) {
  AttnArgs a;
  if (!fill(a, d)) return -1;
  switch (d->D) {
    case 32: return launch_bwd<32>(a, st);
    case 64: return launch_bwd<64>(a, st);
    case 96: return launch_bwd<96>(a, st);
    case 128: return launch_bwd<128>(a, st);
    default: return -2;
  }
}
