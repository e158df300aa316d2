// K01/K02 main GEMM, ping-pong form: two waves per SIMD, 256x256 block tile, 64 x 128 of C per wave.
//
// Reference einsum sites as gemm4w.h (src/model/backend.py:108-110, basic.py:33-126). Why a second form: with one
// wave per SIMD (gemm4w) the wave that feeds the matrix pipe also issues the LDS-DMAs and the fragment reads, and
// the ~50-60 cycles each LDS-DMA holds the issuing wave cost ~800 cycles of a 2,048-cycle K-tile
// (profiles/r3_gemm4w_bounds.md). Here the two waves of a SIMD take turns: while one runs a 32-MFMA "compute"
// phase, its partner runs a "load" phase (fragment reads for its next compute phase + 4 LDS-DMA pieces), and a
// workgroup barrier separates the phases (MI355X_MICROARCH.md, "Two waves per SIMD").
//
//  * 8 waves: group 0 = waves 0-3, group 1 = waves 4-7 (one wave of each group per SIMD). Wave w owns rows
//    64 (w & 3) .. +63 and columns 128 (w >> 2) .. +127 of the tile: 4 x 8 accumulators of v_mfma_f32_16x16x32_bf16
//    (128 AGPRs), one BK = 32 substep of fragments (4 A + 8 B = 48 VGPRs, single-buffered: a wave reads the
//    fragments of its next compute phase in its load phase).
//  * Each group runs the same program, L C L C ... per 64-deep K-tile (L = load substep k, C = compute it); group 1
//    starts one barrier later, so in every phase one group computes and the other loads.
//  * LDS: a ring of 4 slots, one per 32-deep half K-tile ("half" t.k): [A image 16 KiB | B image 16 KiB], 128 KiB.
//    Half (t, k) lives in slot (2 t + k) & 3. K-contiguous images are [256 rows][32 k] (64-B rows, 16-B chunk c of
//    row r at chunk c ^ fa(r): conflict-free ds_read_b128 fragment reads); the B image stores tile column
//    8 m + j of each 128-column half at row 16 j + m, so the row-layout (TLAY) B fragment j is 16 consecutive rows.
//    Transposed images ([K][rows] operands) are two [32 k][128 rows] halves read with ds_read_b64_tr_b16.
//  * LDS-DMA: group 0 stages A, group 1 stages B; a wave issues 4 pieces (1 KiB each) per load phase. L(t, k0)
//    issues half (t+1, k1), L(t, k1) issues (t+2, k0) -- the slot whose readers all finished two phases earlier.
//    Every load phase ends with vmcnt(8) (the pieces issued two load phases before have landed: the ring's lead is
//    ~3 phases) + lgkmcnt(0) + barrier. The DMA cursor runs across tile boundaries like gemm4w's.
//  * Epilogue: in the first load phase of the next tile (the partner group computes meanwhile), straight from the
//    accumulators; its S stores sit in the vmcnt queue, so the first K-tile of every tile waits vmcnt(8 + S) (and
//    the prologue issues S stores into an empty resource so the first tile sees the same queue). The first compute
//    phase of a tile writes the accumulators with C = 0 (no zeroing pass).
#pragma once
#include "gemm4w.h"

namespace {

constexpr int G8_SLOT = 32768;   // one ring slot: A + B image of a 32-deep half K-tile
constexpr int G8_OP = 16384;     // one operand image
constexpr int G8_HALF = 8192;    // one [32 k][128 rows] half of a transposed image

__device__ __forceinline__ int g8_fa(int r) { return (-(r >> 2)) & 3; }

// per-lane source offsets (bytes from a half K-tile's base) of the 4 LDS-DMA pieces wave wq of a group stages of one
// operand. T = 0: piece P = LDS rows 16 P .. +15 x 64 B (B image: LDS row 16 j + m of a 128-row half holds tile row
// 8 m + j); T = 1: piece P = k-rows 4 (P & 7) .. +3 of half P >> 3.
template <int T, bool BIMG>
__device__ __forceinline__ void g8_piece_offsets(int (&vo)[4], long long ld, int wq, int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int P = 4 * wq + q;
    if (T == 0) {
      const int lrow = 16 * P + (lane >> 2);
      const int grow = BIMG ? (lrow & ~127) + 8 * (lrow & 15) + ((lrow >> 4) & 7) : lrow;
      const int c = (lane & 3) ^ g8_fa(lrow);
      vo[q] = (int)(grow * ld * 2) + c * 16;
    } else {
      const int h = P >> 3, kr = (P & 7) * 4 + (lane >> 4);
      const int c = (lane & 15) ^ kswz(kr);
      vo[q] = (int)(kr * ld * 2) + (h * 128 + c * 8) * 2;
    }
  }
}

// A fragment (16 rows from rbase) of a half K-tile image
template <int T>
__device__ __forceinline__ bf16x8_t g8_frag_a(const char* img, int rbase, int lane) {
  if constexpr (T == 0) {
    const int r = rbase + (lane & 15), c = lane >> 4;
    return *reinterpret_cast<const bf16x8_t*>(img + r * 64 + ((c ^ g8_fa(r)) << 4));
  } else {
    return read_frag<1>(img + (rbase >> 7) * G8_HALF, rbase & 127, 0, lane);
  }
}

// B fragment j of the 128 columns at nbase. T = 0 (TLAY): operand column l = tile column nbase + 8 l + j (the MFMA
// takes A first; a lane's accumulators hold 4 rows x 8 consecutive columns). T = 1: gemm4w's paired-column order
// (frag_b), MFMA B first.
template <int T>
__device__ __forceinline__ bf16x8_t g8_frag_b(const char* img, int nbase, int j, int lane) {
  if constexpr (T == 0) {
    const int r = nbase + 16 * j + (lane & 15), c = lane >> 4;
    return *reinterpret_cast<const bf16x8_t*>(img + r * 64 + ((c ^ g8_fa(r)) << 4));
  } else {
    const int base = nbase + 32 * (j >> 1) + 4 * (j & 1);
    const char* h = img + (base >> 7) * G8_HALF;
    const int gg = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
    const int col = (base & 127) + 8 * pp;
    const int c = col >> 3;
    const int k0 = 8 * gg + q, k1 = k0 + 4;
    const int off0 = k0 * 256 + ((c ^ kswz(k0)) << 4) + ((col & 4) << 1);
    const int off1 = k1 * 256 + ((c ^ kswz(k1)) << 4) + ((col & 4) << 1);
    s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, h + off0));
    s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, h + off1));
    s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// dma16o with 5 wait states in front: the first piece of a group reads a resource that v_readfirstlane may have
// written right before it (VALU -> SGPR -> VMEM needs five; tools/sgpr_hazard.py)
#define OBST_DMA16P(BITS)                                                                                          \
  asm volatile("s_nop 4\n\ts_add_u32 m0, %2, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen" BITS " lds" ::"v"(voff), \
               "s"(rs), "s"(sbase), "n"(OFF)                                                                      \
               : "memory", "m0")
template <int CP, int OFF>
__device__ __forceinline__ void dma16p(const i32x4_t& rs, int voff, unsigned sbase) {
  if constexpr (CP == 0) OBST_DMA16P("");
  else if constexpr (CP == 1) OBST_DMA16P(" sc0");
  else if constexpr (CP == 2) OBST_DMA16P(" sc1");
  else if constexpr (CP == 3) OBST_DMA16P(" sc0 sc1");
  else OBST_DMA16P(" nt");
}
#undef OBST_DMA16P
// the first MFMA of a tile: C = A.B (source C = 0), accumulator register kept in place ("+a")
__device__ __forceinline__ void mfma_zero(f32x4_t& c, const bf16x8_t& a, const bf16x8_t& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "+a"(c) : "v"(a), "v"(b));
}
#pragma clang diagnostic pop

// a buffer resource whose words are forced into SGPRs (v_readfirstlane; a no-op for values already scalar): under
// SGPR pressure the allocator kept epilogue pointers in VGPRs ("illegal VGPR to SGPR copy" at the store)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_brsrc_u(const void* base, long long nbytes) {
  const unsigned long long a = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane(
      (int)(unsigned)(nbytes <= 0 ? 0ull : nbytes >= 0xffffffffll ? 0xffffffffull : (unsigned long long)nbytes));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo), 0, n,
                                           0x00020000);
}

__device__ __forceinline__ void pad_redefine48(f32x4_t (&acc)[4][8]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(acc[0][0]), "+a"(acc[0][1]), "+a"(acc[0][2]), "+a"(acc[0][3]),
               "+a"(acc[0][4]), "+a"(acc[0][5]), "+a"(acc[0][6]), "+a"(acc[0][7]));
#pragma unroll
  for (int i = 1; i < 4; ++i)
    asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]), "+a"(acc[i][4]),
                 "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
}

#ifndef G8W_OPT
#define G8W_OPT 1
#endif
// OPT bits (tools/lab/g8w_ab.cpp):
//   1 PRIO: group 1 (the second-dispatched half, the arbitration loser) runs at s_setprio 1 for the whole kernel
//   2 DMAFIRST: a load phase issues its LDS-DMA pieces before its fragment reads
//   4 CPRIO: s_setprio 1 around every compute phase
template <int A_T, int B_T, bool OUT_F32, bool PROF, int OPT = G8W_OPT, int CPA = 0, int CPB = 0>
__global__ __launch_bounds__(512, 2) void gemm8w_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  constexpr bool PRIO = (OPT & 1) != 0, DMAFIRST = (OPT & 2) != 0, CPRIO = (OPT & 4) != 0;
  constexpr int S = 32;                  // direct-epilogue stores per wave, every variant (see epilogue_v)
  constexpr int VF = 8 + S;              // vmcnt of the first K-tile's load phases
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wq = wave & 3;
  const int wm = wq, wn = grp;

  const long long total = (long long)p.tiles_m * p.tiles_n * p.nbatch;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;
  const long long Q = total >> 3, Rm = total & 7;
  const bool cyc = p.tri != 0;
  const long long start = cyc ? 0 : xcd < Rm ? xcd * (Q + 1) : Rm * (Q + 1) + (xcd - Rm) * Q;
  const long long len = cyc ? total : Q + (xcd < Rm ? 1 : 0);
  const long long first = cyc ? blockIdx.x : slot;
  const long long stride = cyc ? gridDim.x : nslot;
  const int ntiles = (int)(len > first ? (len - first + stride - 1) / stride : 0);
  if (ntiles == 0) return;
  auto logical = [&](int r) { return start + first + (long long)r * stride; };

  // LDS-DMA: group 0 stages the A images, group 1 the B images (wave-uniform choice)
  int vo[4];
  if (grp == 0) g8_piece_offsets<A_T, false>(vo, p.lda, wq, lane);
  else g8_piece_offsets<B_T, true>(vo, p.ldb, wq, lane);
  const bool opa = grp == 0;
  const long long ldo = opa ? p.lda : p.ldb;
  const bool tro = opa ? A_T != 0 : B_T != 0;
  const unsigned long long step = tro ? 128ull * (unsigned long long)ldo : 128ull;   // one 64-deep K-tile
  const unsigned long long koff = tro ? 64ull * (unsigned long long)ldo : 64ull;    // its second half
  const unsigned lds0 = lds_u32(smem);
  auto sbase_of = [&](int s) -> unsigned {
    return __builtin_amdgcn_readfirstlane(lds0 + s * G8_SLOT + grp * G8_OP + wq * 4096);
  };

  int d_rnd = 0, d_kt = 0, d_nk = 0;
  unsigned long long cur, rem;
  auto cursor_tile = [&](const Tile4& T) {
    d_nk = T.nk;
    cur = opa ? (unsigned long long)T.a : (unsigned long long)T.b;
    rem = opa ? (unsigned long long)T.arem : (unsigned long long)T.brem;
  };
  cursor_tile(decode4<A_T, B_T>(p, logical(0)));
  // (readfirstlane: a no-op on values the allocator keeps in SGPRs; it turns an "illegal VGPR to SGPR copy" into a
  // v_readfirstlane when SGPR pressure moved one to a VGPR -- tools/sgpr_hazard.py checks the DMA behind it)
  auto rsrc_of = [](unsigned long long base, unsigned long long rm) {
    i32x4_t r;
    r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)base);
    r[1] = __builtin_amdgcn_readfirstlane((int)(unsigned)(base >> 32));
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(rm >> 32));
    r[2] = hi ? -1 : __builtin_amdgcn_readfirstlane((int)(unsigned)rm);
    r[3] = 0x00020000;
    return r;
  };
  auto advance = [&]() {
    if (d_kt + 1 < d_nk) {
      ++d_kt;
      cur += step;
      rem -= step;
    } else if (d_rnd + 1 < ntiles) {
      asm volatile("");
      ++d_rnd;
      d_kt = 0;
      cursor_tile(decode4<A_T, B_T>(p, logical(d_rnd)));
    }
  };
  // this wave's 4 pieces of half `half` of the cursor's K-tile into ring slot s
  auto dma = [&](int half, int s) __attribute__((always_inline)) {
    const unsigned long long o = half ? koff : 0ull;
    const i32x4_t rs = rsrc_of(cur + o, rem - o);
    const unsigned sb = sbase_of(s);
    if (CPA == CPB || opa) {
      static_for<4>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        if constexpr (q == 0) dma16p<CPA, 0>(rs, vo[q], sb);
        else dma16o<CPA, q * 1024>(rs, vo[q], sb);
      });
    } else {
      static_for<4>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        if constexpr (q == 0) dma16p<CPB, 0>(rs, vo[q], sb);
        else dma16o<CPB, q * 1024>(rs, vo[q], sb);
      });
    }
  };

  f32x4_t acc[4][8];
  bf16x8_t af[4], bfr[8];
  auto read_frags = [&](int s) __attribute__((always_inline)) {
    const char* img = smem + s * G8_SLOT;
    static_for<4>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      af[i] = g8_frag_a<A_T>(img, wm * 64 + 16 * i, lane);
    });
    static_for<8>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      bfr[j] = g8_frag_b<B_T>(img + G8_OP, wn * 128, j, lane);
    });
  };
  auto lphase = [&](int rs, int ds, int half, auto vwc) __attribute__((always_inline)) {
    constexpr int VW = decltype(vwc)::value;
    if constexpr (DMAFIRST) {
      dma(half, ds);
      fence();
      read_frags(rs);
    } else {
      read_frags(rs);
      fence();
      dma(half, ds);
    }
    fence();
    vm_wait<VW>();
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this phase's fragments are in registers (and the compiler
                                          // learns it), and every wave is done reading the slot before the barrier
    __builtin_amdgcn_s_barrier();
    fence();
  };
  auto cphase = [&](auto zc) __attribute__((always_inline)) {
    constexpr bool ZERO = decltype(zc)::value;
    if constexpr (CPRIO) __builtin_amdgcn_s_setprio(1);
    static_for<32>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      constexpr int i = q & 3, j = q >> 2;
      if constexpr (B_T == 0) {
        if constexpr (ZERO) mfma_zero(acc[i][j], af[i], bfr[j]);
        else mfma_acc(acc[i][j], af[i], bfr[j]);
      } else {
        if constexpr (ZERO) mfma_zero(acc[i][j], bfr[j], af[i]);
        else mfma_acc(acc[i][j], bfr[j], af[i]);
      }
    });
    fence();
    if constexpr (CPRIO) {
      if (PRIO && grp == 1) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
    __builtin_amdgcn_s_barrier();
    fence();
  };

  // Direct epilogue of one tile from the accumulators. Every variant leaves EXACTLY S stores in the vmcnt queue (the
  // first K-tile's counted waits assume S ops younger than the awaited pieces): stores of masked columns go to an
  // offset past the resource (dropped by the range check, still counted), plain bf16 products pad with 16 such
  // stores, and the side-input loads (R, Zin, beta * C) are compiler-visible -- the compiler waits for them before
  // their use, so none is left outstanding. Rows past M fall outside the resource.
  //   EX: residual R and / or beta * C (fp32);  AC: 0 none, 1 activation forward (+ Zout pre-activation), 2 backward
  //   (C = v * act'(Zin)); ACTK: the activation (gelu / relu)
  auto epilogue_v = [&](const Tile4& ct, auto exc, auto acc_, auto actk) __attribute__((always_inline)) {
    constexpr bool EX = decltype(exc)::value;
    constexpr int AC = decltype(acc_)::value;
    constexpr int ACTK = decltype(actk)::value;
    const bool ws_out = OUT_F32 && p.ksplit > 1;
    const long long ldc = ws_out ? p.N : p.ldc;
    constexpr int ES = OUT_F32 ? 4 : 2;
    char* cbase = ws_out ? reinterpret_cast<char*>(p.ws + (long long)ct.wsi * p.M * p.N)
                         : reinterpret_cast<char*>(p.C) + ct.coff * ES;
    const long long corg = ((long long)ct.m0 * ldc + ct.n0) * ES;
    const long long cext = ((long long)(p.M - ct.m0 - 1) * ldc + (p.N - ct.n0)) * ES;
    const __amdgpu_buffer_rsrc_t rc = make_brsrc_u(cbase + corg, cext);
    const __amdgpu_buffer_rsrc_t rr =
        make_brsrc_u(p.R ? reinterpret_cast<const char*>(p.R) + ct.coff * ES + corg : cbase + corg, cext);
    const __amdgpu_buffer_rsrc_t rz = make_brsrc_u(
        (AC == 1 && p.Zout) ? reinterpret_cast<const char*>(p.Zout) + ct.coff * 2 + corg
                            : (AC == 2 ? reinterpret_cast<const char*>(p.Zin) + ct.coff * 2 + corg : cbase + corg),
        (AC == 1 && !p.Zout) ? 0 : cext);   // no Zout: its stores go nowhere (still counted)
    const float alpha = p.alpha, beta = ws_out ? 0.f : p.beta;
    const int ldcs = __builtin_amdgcn_readfirstlane((int)ldc);
    const int ml = lane & 15, gq = lane >> 4;
    // per-lane origin of the 8 consecutive columns of store (i, u): row ro(i, u), column offset
    //   B_T == 0 (TLAY): u = r, row 16 i + 4 gq + r, columns 8 ml .. +7 (acc[i][0..7][r])
    //   B_T == 1: u = pp, row 16 i + ml, columns 32 pp + 8 gq .. +7 (acc[i][2 pp][0..3], acc[i][2 pp + 1][0..3])
    const int row0 = B_T == 0 ? wm * 64 + 4 * gq : wm * 64 + ml;
    const int col0 = B_T == 0 ? wn * 128 + 8 * ml : wn * 128 + 8 * gq;
    // one 8-column row segment (i, u) at a time: the VGPR half of two waves per SIMD is 128 registers (the
    // accumulators take the 128 AGPRs), so the side inputs, the arithmetic and the stores stay segment-local
    static_for<16>([&](auto sc) {
      constexpr int i = decltype(sc)::value >> 2, u = decltype(sc)::value & 3;
      const int row = row0 + 16 * i + (B_T == 0 ? u : 0);
      const int col = col0 + (B_T == 0 ? 0 : 32 * u);
      const int off = ct.n0 + col < p.N ? (row * ldcs + col) * ES : (int)0x80000000u;
      float x[8];
      static_for<8>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (B_T == 0) x[j] = alpha * acc[i][j][u];
        else x[j] = alpha * acc[i][2 * u + (j >> 2)][j & 3];
      });
      if constexpr (OUT_F32) {
        if constexpr (EX) {
          if (p.R) {
            const f32x4_t r0 = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0));
            const f32x4_t r1 = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rr, off + 16, 0, 0));
            static_for<4>([&](auto tc) {
              constexpr int t = decltype(tc)::value;
              x[t] += r0[t];
              x[4 + t] += r1[t];
            });
          }
          if (beta != 0.f) {
            const f32x4_t c0 = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rc, off, 0, 0));
            const f32x4_t c1 = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rc, off + 16, 0, 0));
            static_for<4>([&](auto tc) {
              constexpr int t = decltype(tc)::value;
              x[t] += beta * c0[t];
              x[4 + t] += beta * c1[t];
            });
          }
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, f32x4_t{x[0], x[1], x[2], x[3]}), rc, off, 0,
                                               0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, f32x4_t{x[4], x[5], x[6], x[7]}), rc,
                                               off + 16, 0, 0);
      } else {
        if constexpr (EX) {
          const v4u32_t rv = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
          static_for<4>([&](auto tc) {
            constexpr int t = decltype(tc)::value;
            x[2 * t] += bf2f(rv[t] & 0xffff);
            x[2 * t + 1] += bf2f(rv[t] >> 16);
          });
        }
        if constexpr (AC == 1) {
          const v4u32_t zo = v4u32_t{pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]), pack_bf16x2(x[4], x[5]),
                                     pack_bf16x2(x[6], x[7])};
          __builtin_amdgcn_raw_buffer_store_b128(zo, rz, off, 0, 0);
          static_for<8>([&](auto tc) { x[decltype(tc)::value] = act_fwd(ACTK, x[decltype(tc)::value]); });
        } else if constexpr (AC == 2) {
          const v4u32_t zv = __builtin_amdgcn_raw_buffer_load_b128(rz, off, 0, 0);
          static_for<4>([&](auto tc) {
            constexpr int t = decltype(tc)::value;
            x[2 * t] *= act_grad(ACTK, bf2f(zv[t] & 0xffff));
            x[2 * t + 1] *= act_grad(ACTK, bf2f(zv[t] >> 16));
          });
        }
        const v4u32_t o = v4u32_t{pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]), pack_bf16x2(x[4], x[5]),
                                  pack_bf16x2(x[6], x[7])};
        __builtin_amdgcn_raw_buffer_store_b128(o, rc, off, 0, 0);
        if constexpr (AC != 1) __builtin_amdgcn_raw_buffer_store_b128(o, rc, (int)0x80000000u, 0, 0);   // count pad
      }
      if constexpr ((decltype(sc)::value & 3) == 3) fence();
    });
  };
  auto epilogue = [&](const Tile4& ct) __attribute__((always_inline)) {
    fence();
    pad_redefine48(acc);
    fence();
    using F0 = std::false_type;
    using T0 = std::true_type;
    using A0 = std::integral_constant<int, 0>;
    using A1 = std::integral_constant<int, 1>;
    using A2 = std::integral_constant<int, 2>;
    using KG = std::integral_constant<int, ACT_GELU>;
    using KR = std::integral_constant<int, ACT_RELU>;
    const bool ex = (OUT_F32 && p.ksplit <= 1 && p.beta != 0.f) || p.R != nullptr;
    if constexpr (OUT_F32) {
      if (ex) epilogue_v(ct, T0{}, A0{}, KG{});
      else epilogue_v(ct, F0{}, A0{}, KG{});
    } else {
      // (the dispatcher sends an activation here only without a residual: gemm8w_supported)
      if (p.act == ACT_GELU) {
        if (p.mode == 1) epilogue_v(ct, F0{}, A2{}, KG{});
        else epilogue_v(ct, F0{}, A1{}, KG{});
      } else if (p.act == ACT_RELU) {
        if (p.mode == 1) epilogue_v(ct, F0{}, A2{}, KR{});
        else epilogue_v(ct, F0{}, A1{}, KR{});
      } else if (ex) {
        epilogue_v(ct, T0{}, A0{}, KG{});
      } else {
        epilogue_v(ct, F0{}, A0{}, KG{});
      }
    }
    fence();
  };

  const bool stamp = PROF && p.stamps != nullptr && tid == 0;
  const long long sbase = (long long)blockIdx.x * 8;
  unsigned long long t0 = 0, tep = 0, ep_clk = 0;
  if (stamp) t0 = __builtin_amdgcn_s_memtime();

  // prologue: halves (0, k0), (0, k1), (1, k0) into slots 0, 1, 2
  dma(0, 0);
  dma(1, 1);
  advance();
  dma(0, 2);
  vm_wait<8>();
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_s_waitcnt(0xc07f);
  {   // S stores into an empty resource (dropped, but counted): the first tile's queue matches the later tiles'
    const __amdgpu_buffer_rsrc_t nul = make_brsrc(p.C, 0);
    static_for<S>([&](auto) { __builtin_amdgcn_raw_buffer_store_b128(v4u32_t{0u, 0u, 0u, 0u}, nul, 0, 0, 0); });
  }
  if constexpr (PRIO) {
    if (grp == 1) __builtin_amdgcn_s_setprio(1);
  }
  if (grp == 1) __builtin_amdgcn_s_barrier();   // group 1 runs one phase behind
  fence();

  using T_ = std::true_type;
  using F_ = std::false_type;
  using VFc = std::integral_constant<int, VF>;
  using V8c = std::integral_constant<int, 8>;
  int pos = 0;
  Tile4 prev;
  for (int rnd = 0; rnd < ntiles; ++rnd) {
    const Tile4 ct = decode4<A_T, B_T>(p, logical(rnd));
    // first K-tile: the previous tile's epilogue rides in the first load phase, the first compute phase zeroes
    if (rnd > 0) {
      if (stamp) tep = __builtin_amdgcn_s_memtime();
      epilogue(prev);
      if (stamp) ep_clk += __builtin_amdgcn_s_memtime() - tep;
    }
    fence();
    lphase((2 * pos) & 3, (2 * pos + 3) & 3, 1, VFc{});
    cphase(T_{});
    advance();
    lphase((2 * pos + 1) & 3, (2 * pos) & 3, 0, VFc{});
    cphase(F_{});
    ++pos;
    for (int t = 1; t < ct.nk; ++t, ++pos) {
      lphase((2 * pos) & 3, (2 * pos + 3) & 3, 1, V8c{});
      cphase(F_{});
      advance();
      lphase((2 * pos + 1) & 3, (2 * pos) & 3, 0, V8c{});
      cphase(F_{});
    }
    prev = ct;
  }
  epilogue(prev);
  if (grp == 0) __builtin_amdgcn_s_barrier();   // matches group 1's extra barrier at the start
  vm_wait<0>();   // the last re-staged halves must land before the LDS is released
  if (stamp) {
    p.stamps[sbase + 0] = __builtin_amdgcn_s_memtime() - t0;
    p.stamps[sbase + 1] = ep_clk;
    p.stamps[sbase + 7] = ntiles;
  }
}

template <int A_T, int B_T, bool F32>
hipError_t launch8w(GemmArgs a, int batch, hipStream_t stream) {
  a.tiles_m = (a.M + 255) / 256;
  a.tiles_n = (a.N + 255) / 256;
  a.nbatch = batch * a.ksplit;
  const long long tiles = (long long)a.tiles_m * a.tiles_n * a.nbatch;
  const int grid = (int)(tiles >= 256 ? 256 : ((tiles + 7) / 8) * 8);
  const size_t lds = 4 * G8_SLOT;   // 128 KiB ring
  auto k = a.stamps ? gemm8w_kernel<A_T, B_T, F32, true> : gemm8w_kernel<A_T, B_T, F32, false>;
  static bool attr[2] = {false, false};
  if (!attr[a.stamps != nullptr]) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr[a.stamps != nullptr] = true;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(512), lds, stream, a);
  return hipGetLastError();
}

}  // namespace

// one operand-layout pair per translation unit (gemm8w_<a_t><b_t>.hip)
#define OBST_GEMM8W_TU(AT, BT)                                                                                      \
  hipError_t gemm8w_launch_##AT##BT(const gemmk::GemmArgs* a, int out_f32, int batch, hipStream_t stream) {      \
    return out_f32 ? launch8w<AT, BT, true>(*a, batch, stream) : launch8w<AT, BT, false>(*a, batch, stream);    \
  }
