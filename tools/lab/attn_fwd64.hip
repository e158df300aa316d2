// LAB ONLY (round 6): moved out of the product -- slower than attn_fwd32_kernel (profiles/r5_attn_fwd64.md). It
// declared its launcher in attn_common.h; building it again needs that declaration back.
// D = 128 causal / full attention forward, one wave per SIMD, 64 queries per wave, the softmax software-pipelined
// beside the MFMAs (K04 forward, same contract as attn_fwd32_kernel in attention.hip: ref src/model/spatial.py:44-81).
//
// Why a second forward: attn_fwd32_kernel runs two waves per SIMD and leaves the overlap of one wave's softmax with
// the other's MFMAs to the hardware arbiter. Its softmax VALU per 64x64 score tile (64 fma + 64 v_exp + max, sums,
// packs) is about as long as the tile's MFMAs, and the two waves mostly serialise: 0.76 PF/s at B64 H16 S2048,
// ~38 % of the same-process MFMA calibration (profiles/kbench_floor.json). Here one wave owns 64 queries as two
// 32-query halves and runs them as a two-stage pipeline inside its own instruction stream; per 64-key tile j:
//   A: Sᵀ(half 0, j) = K(j)·Qᵀ     (16 MFMAs)  beside  P(half 1, j-1) = exp2(S·c2 - m)   (32 fma + 32 v_exp)
//   B: Oᵀ(half 1) += Vᵀ(j-1)·P     (16 MFMAs)  beside  row max of S(half 0, j), row sums of P(half 1), packs
//   C: Sᵀ(half 1, j) = K(j)·Qᵀ     (16 MFMAs)  beside  P(half 0, j)
//   D: Oᵀ(half 0) += Vᵀ(j)·P       (16 MFMAs)  beside  row max of S(half 1, j), row sums of P(half 0), packs
// so each 32-cycle MFMA gap carries 3-4 VALU instructions (MI355X_MICROARCH.md: <= 5 single-issue fillers hide per
// 32x32x16 gap at one wave per SIMD), placed in source order between sched_barrier fences.
//
// Registers: the scores must be VALU operands (AGPR copies alone would cost 128 issue cycles per half tile); the 128
// O accumulators and the 64 Q fragment registers are only MFMA operands. With the builtins the compiler puts either
// every MFMA result in AGPRs (one wave per SIMD) or every one in VGPRs (-amdgpu-mfma-vgpr-form), and then reloads the
// Q fragments from AGPR spill slots before each MFMA. So all MFMAs here are inline asm: Sᵀ accumulates in VGPRs
// ("+v"), Oᵀ in AGPRs ("+a") and the Q fragments are AGPR sources ("a"), leaving ~200 VGPRs. The asm MFMAs are
// invisible to the compiler's hazard recognizer, so the code keeps their hazards by construction: a chain's first
// MFMA takes the constant 0 as SrcC, the packed P operand (a VALU result) is written >= 2 instructions before its
// MFMA (s_nop 1 where the schedule cannot show it), VALU reads of fresh scores come >= 2 MFMAs after their last
// write or behind s_nop padding, and every VALU access to O (rescale, epilogue) is padded the same way.
//
// The block stages 64-key K/V tiles through a 4-deep LDS-DMA ring; a wave's tiles are [0, nu) unmasked, at most one
// masked tile (the causal diagonal or the ragged tail: its row max taken with the mask) and idle ones (staging and
// barrier only). The wave's pipeline drains one step after its last tile, so the block runs nkb + 1 steps.
#include "attn_common.h"

namespace {

#ifndef FWD64_KPF
#define FWD64_KPF 2   // K fragments read this many k-steps ahead of their MFMA
#endif
#ifndef FWD64_NS
#define FWD64_NS 4    // LDS ring slots of 64-key K/V tiles (32 KiB each): NS - 3 tiles in flight past the next one
#endif
#ifndef FWD64_VPF
#define FWD64_VPF 2   // Vᵀ fragments read this many MFMAs ahead
#endif

#define FENCE() __builtin_amdgcn_sched_barrier(0)

// timing-only ablations (wrong results): 1 no exp, 2 no max/sum, 4 no per-step barrier, 8 no fences, 16 no K/V
// staging after the prologue, 32 fragments read from LDS once per phase (the MFMAs reuse them), 64 per-block cycle
// stamps (prologue, steps, epilogue, step count) written over LSE[4 * block ..]
#ifndef FWD64_DBG
#define FWD64_DBG 0
#endif

// Oᵀ tile += Vᵀ·P with the accumulator pinned in AGPRs (NOP: 2 wait states for a P packed just before)
template <bool NOP = false>
__device__ __forceinline__ void mfma_o(f32x16_t& acc, const bf16x8_t& a, const bf16x8_t& b) {
  if (NOP) asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// Sᵀ tile (+)= K·Qᵀ: accumulator in VGPRs, the Q fragment an AGPR source; FIRST: SrcC = 0 (a fresh chain)
template <bool FIRST>
__device__ __forceinline__ void mfma_s(f32x16_t& acc, const bf16x8_t& a, const bf16x8_t& b) {
  if (FIRST) asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(b));
  else asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
}

// padding before a VALU read of an asm-MFMA result (XDL 16-pass write -> VALU read: 18 wait states on gfx940+)
__device__ __forceinline__ void o_settle() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" ::: "memory"); }

// max(a, b, c) in one v_max3_f32: the scores are asm outputs, so fmaxf would first canonicalize each (v_max x, x)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// A / C: (QK) Sᵀ of one half from the K tile, beside (EX) P = exp2(S·c2 - m) of the other half in place
template <bool QK, bool EX>
__device__ __forceinline__ void f64_qk(const char* sK, const bf16x8_t (&qf)[8], f32x16_t (&sn)[2], f32x16_t (&se)[2],
                                       float nm, float c2, const Frag32& fo) {
  constexpr int PF = FWD64_KPF;
  bf16x8_t kf[PF + 1][2];
  if (QK) {
#pragma unroll
    for (int ks = 0; ks < PF; ++ks)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) kf[ks][kt] = *reinterpret_cast<const bf16x8_t*>(sK + fo.k[ks] + kt * 32 * 256);
  }
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      if (QK) {
        if (ks + PF < 8 && !(FWD64_DBG & 32))
          kf[(ks + PF) % (PF + 1)][kt] = *reinterpret_cast<const bf16x8_t*>(sK + fo.k[ks + PF] + kt * 32 * 256);
        if ((FWD64_DBG & 32) && ks >= PF) kf[ks % (PF + 1)][kt] = kf[kt % PF][kt];
        if (ks == 0) mfma_s<true>(sn[kt], kf[0][kt], qf[0]);
        else mfma_s<false>(sn[kt], kf[ks % (PF + 1)][kt], qf[ks]);
      }
      if (EX)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int e = ks * 4 + kt * 2 + i;
          if (FWD64_DBG & 1) se[e >> 4][e & 15] = __builtin_fmaf(se[e >> 4][e & 15], c2, nm);
          else se[e >> 4][e & 15] = fexp2(__builtin_fmaf(se[e >> 4][e & 15], c2, nm));
        }
      if (QK && !(FWD64_DBG & 8)) FENCE();   // source order = issue order (the asm MFMAs' hazards are kept by that order)
    }
  }
}

// 8 P values (key sub-tile kt, k-step st: registers 8 st .. 8 st + 7) as one bf16x8 B operand, two dwords at a time
__device__ __forceinline__ void pack_half(const f32x16_t& p, int st, uint32_t (&d)[4], int part) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = 8 * st + 2 * (2 * part + j);
    d[2 * part + j] = pack_bf16x2(p[r], p[r + 1]);
  }
}

// B / D: (PV) Oᵀ += Vᵀ·P of one half with its row sums, beside (MX) the row max of the other half's fresh scores.
// The 16 MFMAs run as one flat sequence (i = 4 (2 kt + st) + dt) with the Vᵀ fragments read FWD64_VPF MFMAs ahead and
// the next group's P packed during the three MFMAs before it is needed.
template <bool PV, bool MX>
__device__ __forceinline__ void f64_pv(const char* sV, const f32x16_t (&p)[2], f32x16_t (&o)[4], float& rs,
                                       const f32x16_t (&sm)[2], float& mx, const Frag32& fo) {
  constexpr int PF = FWD64_VPF;
  auto vread = [&](int i) {
    const int i4 = i >> 2, dt = i & 3, kb = ((i4 >> 1) * 32 + 16 * (i4 & 1)) * 256;
    return tr_pair(sV, fo.v[dt][0] + kb, fo.v[dt][1] + kb);
  };
  bf16x8_t vf[PF + 1];
  uint32_t pk[4][4];   // the four 8-key groups' packed P (fully unrolled: no moves between them)
  if (PV) {
#pragma unroll
    for (int i = 0; i < PF; ++i) vf[i] = vread(i);
    pack_half(p[0], 0, pk[0], 0);
    pack_half(p[0], 0, pk[0], 1);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (PV) {
      if (i + PF < 16 && !(FWD64_DBG & 32)) vf[(i + PF) % (PF + 1)] = vread(i + PF);
      if ((FWD64_DBG & 32) && i >= PF) vf[i % (PF + 1)] = vf[i % PF];
      if (i == 0) mfma_o<true>(o[0], vf[0], __builtin_bit_cast(bf16x8_t, pk[0]));
      else mfma_o(o[i & 3], vf[i % (PF + 1)], __builtin_bit_cast(bf16x8_t, pk[i >> 2]));
      const int g = (i >> 2) + 1;   // the next 8-key group: packed beside this group's MFMAs 0 and 1
      if (g < 4 && (i & 3) < 2) pack_half(p[g >> 1], g & 1, pk[g], i & 3);
      if (!(FWD64_DBG & 2)) rs += p[i >> 3][2 * (i & 7)] + p[i >> 3][2 * (i & 7) + 1];
    }
    if (MX && !(FWD64_DBG & 2)) mx = max3f(mx, sm[i >> 3][2 * (i & 7)], sm[i >> 3][2 * (i & 7) + 1]);
    if (PV && !(FWD64_DBG & 8)) FENCE();
  }
}

// row max of one half's scores of a masked tile (the causal diagonal or the ragged tail); masked scores become -inf
__device__ __forceinline__ void f64_masked_max(f32x16_t (&s)[2], float& mx, int k0, int q, int S, int causal,
                                               int lane) {
  const int h = lane >> 5;
  o_settle();   // right behind the scores' MFMAs (or a PV phase)
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = k0 + kt * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
      const float v = (key >= S || (causal && key > q)) ? -INFINITY : s[kt][r];
      s[kt][r] = v;
      mx = fmaxf(mx, v);
    }
}

// one half's running max moves (lazily, by more than 2^RESCALE_TH) to its fresh row max
__device__ __forceinline__ void f64_rescale(float mx, float& m, float& l, f32x16_t (&o)[4], float c2) {
  const float ms = xh_max(mx) * c2;
  const bool bump = ms > m + RESCALE_TH;
  if (__builtin_amdgcn_ballot_w64(bump)) {
    o_settle();   // (also keeps the branch: speculated, the multiply of O would run on every tile)
    const float mn = bump ? ms : m;
    const float alpha = fexp2(m - mn);
    l *= alpha;
    // O *= alpha one AGPR at a time inside asm: as plain C++ the compiler copies all of O to VGPRs ahead of the
    // branch on every tile (live-range split of the "+a" accumulators)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float t;
        asm volatile("v_accvgpr_read_b32 %1, %0\n\ts_nop 0\n\tv_mul_f32 %1, %1, %2\n\tv_accvgpr_write_b32 %0, %1"
                     : "+a"(o[dt][r]), "=&v"(t) : "v"(alpha));
      }
    m = mn;
    asm volatile("s_nop 2" ::: "memory");   // VALU write of O -> MFMA read as SrcC
  }
}

__global__ __launch_bounds__(256, 1) void attn_fwd64_kernel(AttnArgs a) {
  constexpr int D = 128, KT = 64, NS = FWD64_NS, NW = 4, NP = 4, QB = 256;
  constexpr int AH = NS - 2;       // tiles staged ahead: step j stages tile j + AH into the slot of tile j - 2
  static_assert(NS == 4 || NS == 5, "ring of 4 (128 KiB) or 5 (160 KiB) tiles");
  constexpr int TILE = KT * 256;   // bytes of one 64-key K (or V) tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, n = lane & 31;
  const long long t0 = (FWD64_DBG & 64) ? (long long)__builtin_readcyclecounter() : 0;
  long long t1 = 0, t2 = 0;
  const int nx = (a.S + QB - 1) / QB;
  int bx, bh;
  attn_block(nx, bx, bh);
  const int b = bh / a.H, hd = bh % a.H;
  const int qblk = (a.causal ? (nx - 1 - bx) : bx) * QB;   // heaviest causal blocks first
  const int qw = qblk + w * 64;
  const long long base = (long long)b * a.S * a.ld + hd * D;
  const bf16_t* Kb = a.K + base;
  const bf16_t* Vb = a.V + base;
  const int kend = a.causal ? min(a.S, qblk + QB) : a.S;
  const int nkb = (kend + KT - 1) / KT;
  // this wave's tiles: [0, nu) unmasked, then at most one masked tile; last = its final tile (-1: none)
  const int full = a.S / KT;
  int nu, last;
  if (qw >= a.S) {
    nu = 0; last = -1;
  } else if (a.causal) {
    nu = min(qw / KT, full); last = qw / KT;    // qw is a multiple of 64: the diagonal tile is always masked
  } else {
    nu = full; last = nkb - 1;
  }
  nu = __builtin_amdgcn_readfirstlane(nu);
  last = __builtin_amdgcn_readfirstlane(last);
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int q0 = qw + n, q1 = qw + 32 + n;
  unsigned soff[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int row = (wu + NW * i) * 4 + (lane >> 4);
    soff[i] = (unsigned)(row * (int)a.ld + (((lane & 15) ^ swz<128>(row)) << 3)) * 2u;
  }
  auto stage = [&](int t) {
    char* buf = smem + (t % NS) * 2 * TILE;
    const int k0 = __builtin_amdgcn_readfirstlane(t * KT);
    if (k0 + KT <= a.S) {
      stage_full64<NP, NW>(buf, Kb + (long long)k0 * a.ld, soff, wu);
      stage_full64<NP, NW>(buf + TILE, Vb + (long long)k0 * a.ld, soff, wu);
    } else {
      stage_rows64_asm<NP, NW>(buf, Kb + (long long)k0 * a.ld, a.ld, a.S - k0, wu, lane);
      stage_rows64_asm<NP, NW>(buf + TILE, Vb + (long long)k0 * a.ld, a.ld, a.S - k0, wu, lane);
    }
  };
  // vmcnt wait leaving the y youngest tiles' DMA pieces (2 NP each) in flight (y < NS - 2)
  auto wait_younger = [&](int y) {
    if (NS >= 5 && y >= 2) vm_wait<(NS >= 5 ? 4 : 2) * NP>();
    else if (y >= 1) vm_wait<2 * NP>();
    else vm_wait<0>();
  };
  stage(0);
  bf16x8_t qf[2][8];
  {
    // rows past S read row S - 1: their scores and O are never stored and do not touch the valid query columns
    const long long r0 = min(q0, a.S - 1), r1 = min(q1, a.S - 1);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      qf[0][ks] = *reinterpret_cast<const bf16x8_t*>(a.Q + base + r0 * a.ld + ks * 16 + 8 * h);
      qf[1][ks] = *reinterpret_cast<const bf16x8_t*>(a.Q + base + r1 * a.ld + ks * 16 + 8 * h);
    }
  }
#pragma unroll
  for (int t = 1; t < AH; ++t)
    if (t < nkb) stage(t);
  // tile 0 and Q have landed once at most the younger tiles' 2 NP pieces each are in flight
  wait_younger(min(AH, nkb) - 1);
  // the Q fragments move to AGPRs once (tied no-op asm: the copy is the compiler's) and stay there as MFMA sources
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) asm volatile("; Q -> AGPR" : "=a"(qf[qa][ks]) : "0"(qf[qa][ks]));
  asm volatile("s_nop 2" ::: "memory");   // VALU write of an AGPR -> MFMA source read
  __syncthreads();
  Frag32 fo;
  frag32_offsets(fo, lane);
  f32x16_t o0[4], o1[4], s0[2], s1[2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o0[dt] = o1[dt] = f32x16_t{};
  float m0 = NEG_BIG, m1 = NEG_BIG, l0 = 0.f, l1 = 0.f;
  const float c2 = a.scale * LOG2E;
  if (FWD64_DBG & 64) t1 = (long long)__builtin_readcyclecounter();
  auto sync = [&](int j) {   // tile j + 1 (read by step j + 1) has landed; tiles j + 2 .. j + AH may stay in flight
    wait_younger(max(0, min(j + AH, nkb - 1) - (j + 1)));
    if (!(FWD64_DBG & 4)) __syncthreads();
  };
  // step j: stage tile j + AH (into the slot of tile j - 2); A/B finish half 1 of tile j - 1 beside half 0 of tile
  // j, C/D run half 1 of tile j beside the rest of half 0; wait for tile j + 1, barrier. The steps of a wave: 0 (no
  // half 1 to finish), the steady ones [1, nu), the masked tile, the drain (last + 1) and idle ones -- each a loop or
  // branch of its own so the steady loop carries no role tests.
  int j = 0;
  if (last >= 0) {
    {   // step 0: scores of half 0 of tile 0, then C/D of tile 0
      if (AH < nkb) stage(AH);
      float mx0 = -INFINITY, mx1 = -INFINITY, rs0 = 0.f, rs1 = 0.f;
      f64_qk<true, false>(smem, qf[0], s0, s1, 0.f, c2, fo);
      o_settle();
      if (nu > 0) f64_pv<false, true>(smem + TILE, s1, o1, rs1, s0, mx0, fo);
      else f64_masked_max(s0, mx0, 0, q0, a.S, a.causal, lane);
      f64_rescale(mx0, m0, l0, o0, c2);
      f64_qk<true, true>(smem, qf[1], s1, s0, -m0, c2, fo);
      if (nu > 0) {
        f64_pv<true, true>(smem + TILE, s0, o0, rs0, s1, mx1, fo);
      } else {
        f64_pv<true, false>(smem + TILE, s0, o0, rs0, s1, mx1, fo);
        f64_masked_max(s1, mx1, 0, q1, a.S, a.causal, lane);
      }
      l0 += rs0;
      f64_rescale(mx1, m1, l1, o1, c2);
      sync(j);
      ++j;
    }
    for (; j < nu; ++j) {   // steady steps: tile j unmasked, half 1 of tile j - 1 pending
      if (j + AH < nkb && !(FWD64_DBG & 16)) stage(j + AH);
      const char* sK = smem + (j % NS) * 2 * TILE;
      const char* sVp = smem + ((j + NS - 1) % NS) * 2 * TILE + TILE;
      float mx0 = -INFINITY, mx1 = -INFINITY, rs0 = 0.f, rs1 = 0.f;
      f64_qk<true, true>(sK, qf[0], s0, s1, -m1, c2, fo);
      f64_pv<true, true>(sVp, s1, o1, rs1, s0, mx0, fo);
      l1 += rs1;
      f64_rescale(mx0, m0, l0, o0, c2);
      f64_qk<true, true>(sK, qf[1], s1, s0, -m0, c2, fo);
      f64_pv<true, true>(sK + TILE, s0, o0, rs0, s1, mx1, fo);
      l0 += rs0;
      f64_rescale(mx1, m1, l1, o1, c2);
      sync(j);
    }
    if (j == last) {   // the masked tile (j >= 1 here)
      if (j + AH < nkb && !(FWD64_DBG & 16)) stage(j + AH);
      const char* sK = smem + (j % NS) * 2 * TILE;
      const char* sVp = smem + ((j + NS - 1) % NS) * 2 * TILE + TILE;
      float mx0 = -INFINITY, mx1 = -INFINITY, rs0 = 0.f, rs1 = 0.f;
      f64_qk<true, true>(sK, qf[0], s0, s1, -m1, c2, fo);
      f64_pv<true, false>(sVp, s1, o1, rs1, s0, mx0, fo);
      f64_masked_max(s0, mx0, j * KT, q0, a.S, a.causal, lane);
      l1 += rs1;
      f64_rescale(mx0, m0, l0, o0, c2);
      f64_qk<true, true>(sK, qf[1], s1, s0, -m0, c2, fo);
      f64_pv<true, false>(sK + TILE, s0, o0, rs0, s1, mx1, fo);
      f64_masked_max(s1, mx1, j * KT, q1, a.S, a.causal, lane);
      l0 += rs0;
      f64_rescale(mx1, m1, l1, o1, c2);
      sync(j);
      ++j;
    }
    {   // drain: half 1 of the last tile
      if (j + AH < nkb && !(FWD64_DBG & 16)) stage(j + AH);
      const char* sVp = smem + ((j + NS - 1) % NS) * 2 * TILE + TILE;
      float rs1 = 0.f, mx0 = 0.f;
      f64_qk<false, true>(smem, qf[0], s0, s1, -m1, c2, fo);
      f64_pv<true, false>(sVp, s1, o1, rs1, s0, mx0, fo);
      l1 += rs1;
      sync(j);
      ++j;
    }
  }
  for (; j <= nkb; ++j) {   // idle steps: the block's staging and barriers
    if (j + AH < nkb && !(FWD64_DBG & 16)) stage(j + AH);
    sync(j);
  }
  o_settle();
  if (FWD64_DBG & 64) t2 = (long long)__builtin_readcyclecounter();
  // epilogue: O = Oᵀ/l through LDS as whole 256-byte rows (the ring is idle after the last barrier)
  const float lt0 = xh_sum(l0), lt1 = xh_sum(l1);
  const float inv[2] = {1.f / lt0, 1.f / lt1};
  if (h == 0) {
    const long long lb = ((long long)b * a.H + hd) * a.S;
    if (q0 < a.S) a.LSE[lb + q0] = (m0 + __log2f(lt0)) / LOG2E;
    if (q1 < a.S) a.LSE[lb + q1] = (m1 + __log2f(lt1)) / LOG2E;
  }
  char* so = smem + w * 64 * 256;
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x16_t& ov = qa ? o1[dt] : o0[dt];
        const int c = dt * 4 + g4, rr = 32 * qa + n;
        const uint2 v = make_uint2(pack_bf16x2(ov[4 * g4] * inv[qa], ov[4 * g4 + 1] * inv[qa]),
                                   pack_bf16x2(ov[4 * g4 + 2] * inv[qa], ov[4 * g4 + 3] * inv[qa]));
        *reinterpret_cast<uint2*>(so + rr * 256 + ((c ^ (rr & 7)) << 4) + ((h ^ ((rr >> 3) & 1)) << 3)) = v;
      }
  __syncthreads();
  const int c = lane & 15;
  const long long obase = (long long)b * a.S * a.ld_o + hd * D + c * 8;
#pragma unroll
  for (int it = 0; it < 16; ++it) {
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
        for (int jj = 0; jj < 4; ++jj)
          sv[jj] = pack_bf16x2(bf2f(ov[jj] & 0xffff) + bf2f(rv[jj] & 0xffff), bf2f(ov[jj] >> 16) + bf2f(rv[jj] >> 16));
        *reinterpret_cast<uint4*>(a.Sum + off) = make_uint4(sv[0], sv[1], sv[2], sv[3]);
      }
    }
  }
  if ((FWD64_DBG & 64) && tid == 0) {
    const long long t3 = (long long)__builtin_readcyclecounter();
    float* st = a.LSE + 4 * (long long)blockIdx.x;
    st[0] = (float)(t1 - t0);
    st[1] = (float)(t2 - t1);
    st[2] = (float)(t3 - t2);
    st[3] = (float)(nkb + 1);
  }
}

}  // namespace

int attn_fwd64_launch(const void* args, hipStream_t st) {
  const AttnArgs& a = *static_cast<const AttnArgs*>(args);
  hipLaunchKernelGGL(attn_fwd64_kernel, dim3((a.S + 255) / 256 * a.B * a.H), dim3(256), FWD64_NS * 2 * 64 * 256, st, a);
  return (int)hipGetLastError();
}
