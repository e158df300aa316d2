// K01/K02 main GEMM: one wave per SIMD, 256x256x64 block tile, 128x128 of C per wave.
//
// Every plain product of the training step -- forward projections, data gradients, fp32 weight gradients, the
// logits GEMM -- runs here (reference einsum sites: src/model/backend.py:108-110, basic.py:33-126,
// spatial.py:45-81). Design (CDNA4, gfx950):
//
//  * 4 waves (2 M x 2 N), each owning a 128 x 128 quarter of the 256 x 256 tile: 8 x 8 accumulators of
//    v_mfma_f32_16x16x32_bf16 = 256 fp32 registers per lane (the AGPR half of the unified register file). One
//    wave per SIMD: the wave itself keeps the matrix pipe fed, so every non-MFMA instruction of the K loop is
//    placed in the MFMA stream's free issue slots (an MFMA leaves 8 of its 16 cycles for other issue).
//  * A K-tile (BK = 64) is two k-substeps of 32. Fragments of substep 0 and substep 1 live in separate registers
//    (2 x 128 VGPRs), so the LDS image of tile t is dead as soon as its substep-1 fragments are read -- after 16
//    of the tile's 128 MFMAs. From then on the same LDS stage receives tile t+2 by LDS-DMA (buffer_load ... lds,
//    16 B per lane, 1 KiB per wave-instruction, source address = SGPR resource + one constant per-lane offset).
//    Two LDS stages of 64 KiB. Default schedule (SCH 1, the K-loop structure of the vendor library's 256x256x64 gfx950 kernel
//    as read from its code object, profiles/r4_gemm_sched.md): per-operand barrier pairs -- A / B image of stage s
//    free (lgkmcnt(0) + barrier), then DMA bursts into it; A / B of tile t+1 landed (counted vmcnt + barrier), then
//    its substep-0 fragments are read under the last MFMAs of tile t. SCH 0 is the round-3 two-barrier schedule.
//    The instruction order is pinned with sched_barrier(0) fences; the compiler only allocates registers and
//    counts lgkmcnt for the fragment reads. Out-of-range prefetches (t+2 >= nk) re-read the last tile into the
//    stage nobody reads any more, so the loop has no branches.
//  * K-contiguous operands ([rows][K]) are staged as [256 rows][64 k] images (128-B rows, chunk ^= (row>>1)&7:
//    conflict-free ds_read_b128 fragment reads); row-contiguous operands ([K][rows]) as two [64 k][128 rows]
//    halves (256-B rows, chunk ^= kswz(k)) read with the CDNA4 transposing ds_read_b64_tr_b16. The swizzle lives
//    in the per-lane SOURCE address (LDS-DMA writes lane-linearly).
//  * Accumulator layout. K-contiguous B (TLAY, the default for it): the MFMA takes the A fragment first and B
//    fragment j reads tile columns 8 l + j, so a lane holds 4 rows x 8 consecutive columns and every epilogue store
//    instruction writes 4 rows x 256 B (the store path takes ~4x longer for 16 rows x 64 B, store_bench.cpp).
//    Transposed B: mfma(B, A) with paired column permutation, each lane 8 consecutive columns of one row.
//  * Epilogues: direct from the accumulators for plain products, gelu / relu forward (+ pre-activation output) and
//    backward, residual, fp32 accumulate and split-K slabs (batched too); the rest through a wave-private LDS region
//    and the shared epilogue_store of gemm_kern.h.
//  * Hand-written buffer ops lead with s_nop 4: the resource SGPRs may come straight from a VALU write (spill
//    reloads), which the compiler's hazard recognizer does not pad for inline asm (tools/sgpr_hazard.py).
#pragma once
#include "common.h"
#include "gemm_kern.h"
#include <utility>

// G4W_EXP (diagnostic builds of tools/gemm_bench only, never the library): bit 0 drops the K loop's LDS-DMAs, bit 1
// its fragment reads, bit 2 its two barriers -- which resource bounds the loop (outputs are garbage); bit 3 drops the
// direct epilogue's stores (what the epilogue costs without them), bit 4 sends every product through the LDS-path
// epilogue
#ifndef G4W_EXP
#define G4W_EXP 0
#endif

namespace {

typedef __attribute__((ext_vector_type(4))) int i32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned v4u32_t;
typedef __attribute__((ext_vector_type(2))) unsigned v2u32_t;

constexpr int Q_OP = 256 * 64 * 2;   // one operand image of a K-tile: 32 KiB
constexpr int Q_STAGE = 2 * Q_OP;    // A + B: 64 KiB; two stages

__device__ __forceinline__ unsigned lds_u32(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// raw buffer resource over [base, base + nbytes): stride 0; loads at offsets >= nbytes return zeros (edge tiles)
__device__ __forceinline__ i32x4_t make_rsrc(const void* base, long long nbytes) {
  const unsigned long long a = (unsigned long long)base;
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32));
  r[2] = __builtin_amdgcn_readfirstlane(
      (int)(unsigned)(nbytes <= 0 ? 0ull : nbytes >= 0xffffffffll ? 0xffffffffull : (unsigned long long)nbytes));
  r[3] = 0x00020000;
  return r;
}

// the same resource as the compiler's buffer type (epilogue loads / stores through the raw_buffer builtins)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_brsrc(const void* base, long long nbytes) {
  const int n = (int)(unsigned)(nbytes <= 0 ? 0ull : nbytes >= 0xffffffffll ? 0xffffffffull : (unsigned long long)nbytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, n, 0x00020000);
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// LDS-DMA of 16 B per lane into the 1 KiB at LDS address m0 (lane-linear). In inline asm so the compiler neither
// drains it with a vmcnt(0) before later LDS reads nor reorders it: every consumer waits with an explicit counted
// vmcnt before the barrier that publishes the stage. One wait state between the M0 write and the LDS-DMA.
// CP: cache-policy bits of the load (0 none, 1 sc0, 2 sc1, 3 sc0 sc1, 4 nt) -- an operand staged once per CU gains
// nothing from the CU's L1.
// Inline asm is opaque to the compiler's hazard recognizer: a VMEM instruction reading an SGPR that a VALU op wrote
// (v_readfirstlane of make_rsrc, v_readlane of an SGPR spill reload) needs five wait states, which the compiler only
// inserts in front of its own VMEM instructions. The prologue form (once per block) leads with s_nop 4; the K-loop
// form (dma16o) reads SALU-computed resources and is checked by tools/sgpr_hazard.py (tests/test_asm_hazards.py).
template <int CP = 0>
__device__ __forceinline__ void dma16(const i32x4_t& rs, int voff, unsigned m0) {
  const unsigned m = __builtin_amdgcn_readfirstlane(m0);
  if constexpr (CP == 0)
    asm volatile("s_nop 4\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "s"(m)
                 : "memory", "m0");
  else if constexpr (CP == 1)
    asm volatile("s_nop 4\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen sc0 lds" ::"v"(voff), "s"(rs),
                 "s"(m)
                 : "memory", "m0");
  else if constexpr (CP == 2)
    asm volatile("s_nop 4\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen sc1 lds" ::"v"(voff), "s"(rs),
                 "s"(m)
                 : "memory", "m0");
  else if constexpr (CP == 3)
    asm volatile("s_nop 4\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen sc0 sc1 lds" ::"v"(voff),
                 "s"(rs), "s"(m)
                 : "memory", "m0");
  else
    asm volatile("s_nop 4\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen nt lds" ::"v"(voff), "s"(rs),
                 "s"(m)
                 : "memory", "m0");
}
// the same with m0 = stage base (SGPR) + OFF in one SALU op (the K loop's form: no temporary, no s_mov)
#define OBST_DMA16O(BITS)                                                                                          \
  asm volatile("s_add_u32 m0, %2, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen" BITS " lds" ::"v"(voff),   \
               "s"(rs), "s"(sbase), "n"(OFF)                                                                      \
               : "memory", "m0")
template <int CP, int OFF>
__device__ __forceinline__ void dma16o(const i32x4_t& rs, int voff, unsigned sbase) {
  if constexpr (CP == 0) OBST_DMA16O("");
  else if constexpr (CP == 1) OBST_DMA16O(" sc0");
  else if constexpr (CP == 2) OBST_DMA16O(" sc1");
  else if constexpr (CP == 3) OBST_DMA16O(" sc0 sc1");
  else OBST_DMA16O(" nt");
}
#undef OBST_DMA16O
// C += A.B on one 16x16x32 bf16 tile, accumulator pinned to AGPRs: as a builtin, the register allocator re-assigned
// the 64 loop-carried accumulators every iteration and copied them back through VGPRs at the back edge (512
// registers, spills); a tied "+a" operand keeps each one in place. Hazards the compiler cannot see inside the asm
// are padded by hand where the accumulators are initialised and read back (s_nop, fenced).
__device__ __forceinline__ void mfma_acc(f32x4_t& c, const bf16x8_t& a, const bf16x8_t& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
// 16-byte buffer store of v at voff + IMM (range-checked: past num_records it is dropped), padded on both sides.
// Behind: a store of more than 8 bytes reads its data VGPRs after issue and the next VALU op may rewrite them (the
// compiler pads that only for its own stores). In front: the resource SGPRs may come straight from a VALU write --
// under SGPR pressure the compiler reloads spilled resource words with v_readlane 2-4 instructions before the store,
// and the store then read a stale base: the illegal-address faults of round 4 in a small batched gelu epilogue
// (test_gemm_batched_epilogues; found with tools/sgpr_hazard.py on the device assembly).
// SC: cache-policy bits of the store (0 none, 1 sc0, 2 sc1, 3 sc0 sc1, 4 nt)
#define OBST_ST16(BITS)                                                                                           \
  asm volatile("s_nop 4\n\tbuffer_store_dwordx4 %0, %1, %2, 0 offen offset:%3" BITS "\n\ts_nop 4" ::"v"(v), "v"(voff), \
               "s"(rs), "n"(IMM)                                                                                   \
               : "memory")
template <int IMM, int SC = 0, typename V>
__device__ __forceinline__ void store16_padded(const V& v, int voff, const i32x4_t& rs,
                                               std::integral_constant<int, IMM>) {
  if constexpr ((G4W_EXP & 8) != 0) return;   // diagnostic: an epilogue without its stores
  if constexpr (SC == 0) OBST_ST16("");
  else if constexpr (SC == 1) OBST_ST16(" sc0");
  else if constexpr (SC == 2) OBST_ST16(" sc1");
  else if constexpr (SC == 3) OBST_ST16(" sc0 sc1");
  else OBST_ST16(" nt");
}
// the same without a memory clobber: LDS reads / writes of the epilogue may move across it (data dependences
// still order it after the LDS read that produces its value)
#define OBST_ST16NC(BITS)                                                                                      \
  asm volatile("s_nop 4\n\tbuffer_store_dwordx4 %0, %1, %2, 0 offen" BITS "\n\ts_nop 4" ::"v"(v), "v"(voff), \
               "s"(rs))
template <int SC = 0, typename V>
__device__ __forceinline__ void store16_nc(const V& v, int voff, const i32x4_t& rs_) {
  if constexpr ((G4W_EXP & 8) != 0) return;
  // uniform by construction, but in the activation epilogues the register allocator had the resource in VGPRs
  // ("illegal VGPR to SGPR copy"): read it back into SGPRs (a no-op copy when it is already scalar; the s_nop 4 in
  // front of the store covers the VALU-write -> VMEM-read hazard otherwise)
  i32x4_t rs;
  rs[0] = __builtin_amdgcn_readfirstlane(rs_[0]);
  rs[1] = __builtin_amdgcn_readfirstlane(rs_[1]);
  rs[2] = __builtin_amdgcn_readfirstlane(rs_[2]);
  rs[3] = __builtin_amdgcn_readfirstlane(rs_[3]);
  if constexpr (SC == 0) OBST_ST16NC("");
  else if constexpr (SC == 1) OBST_ST16NC(" sc0");
  else if constexpr (SC == 2) OBST_ST16NC(" sc1");
  else if constexpr (SC == 3) OBST_ST16NC(" sc0 sc1");
  else OBST_ST16NC(" nt");
}
#undef OBST_ST16NC
#undef OBST_ST16
#pragma clang diagnostic pop

__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }
// 16-byte buffer load straight into an accumulator's AGPRs, invisible to the compiler's wait model: the caller waits
// with an explicit counted vmcnt and then agpr_opaque()s the value before reading it (emit_zpipe)
// emit_tpipe's side-row schedule: row i (i < 4) issues rows 2i + 1 and 2i + 2 (row 3: row 7) after forming its
// outputs, then its 4 stores; row k waits until only the ops issued after its side rows are pending:
//   k 1: R2 S0 | 2: S0 R3 R4 S1 | 3: R4 S1 R5 R6 S2 | 4: S1 R5 R6 S2 R7 S3 | 5: R6 S2 R7 S3 S4 | 6: S2 R7 S3 S4 S5 |
//   7: S3 S4 S5 S6   (4 ops each)
template <int K>
__device__ __forceinline__ void tpipe_wait() {
  static_assert(K >= 1 && K <= 7, "rows 1..7");
  if constexpr (K == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (K == 2 || K == 7) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (K == 4) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
}
// emit_zpipe's schedule (8 loads R per row, 12 stores S): row k waits until only the ops issued after its rows are
// pending -- k 1: S0 | 2: R3 S1 | 3: S1 R4 S2 | 4: S2 R5 S3 | 5: S3 R6 S4 | 6: S4 R7 S5 | 7: S5 S6
template <int K>
__device__ __forceinline__ void zpipe_wait() {
  static_assert(K >= 1 && K <= 7, "rows 1..7");
  if constexpr (K == 1) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (K == 2) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
  else if constexpr (K == 7) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
}
template <int IMM>
__device__ __forceinline__ void load16_agpr(f32x4_t& dst, int voff, const i32x4_t& rs_) {
  i32x4_t rs;   // uniform by construction; read back into SGPRs as store16_nc does (the caller's s_nop covers the hazard)
  rs[0] = __builtin_amdgcn_readfirstlane(rs_[0]);
  rs[1] = __builtin_amdgcn_readfirstlane(rs_[1]);
  rs[2] = __builtin_amdgcn_readfirstlane(rs_[2]);
  rs[3] = __builtin_amdgcn_readfirstlane(rs_[3]);
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3" : "=a"(dst) : "v"(voff), "s"(rs), "n"(IMM) : "memory");
}
// makes c an asm-produced AGPR value (no later rematerialisation of what it was computed from)
__device__ __forceinline__ void agpr_opaque(f32x4_t& c) { asm volatile("" : "+a"(c)); }

// 24 wait states after the last MFMA, then every accumulator redefined by asm (8 per statement, in order)
__device__ __forceinline__ void pad_redefine(f32x4_t (&acc)[8][8]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(acc[0][0]), "+a"(acc[0][1]), "+a"(acc[0][2]), "+a"(acc[0][3]),
               "+a"(acc[0][4]), "+a"(acc[0][5]), "+a"(acc[0][6]), "+a"(acc[0][7]));
#pragma unroll
  for (int i = 1; i < 8; ++i)
    asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]), "+a"(acc[i][4]),
                 "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
}
__device__ __forceinline__ void pad_redefine(f32x4_t (&acc)[8][4]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(acc[0][0]), "+a"(acc[0][1]), "+a"(acc[0][2]), "+a"(acc[0][3]));
#pragma unroll
  for (int i = 1; i < 8; ++i) asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]));
}

// compile-time loop: f(std::integral_constant<int, 0>) ... f(<N-1>) -- the K-loop body is 128 MFMA slots, past
// what #pragma unroll expands, and every register array must stay statically indexed
template <typename F, int... Qs>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Qs...>) {
  (f(std::integral_constant<int, Qs>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// chunk swizzle of a K-contiguous B image: frag_b reads rows {0-3, 8-11, 16-19, 24-27} + base per lane group, on
// which the A images' (row >> 1) & 7 is 2-way bank-conflicted (67 M conflict cycles per 131072x4096x2048 launch);
// row bits 1, 3 and 4 give the 16 lanes of every ds_read_b128 group distinct bank quads (profiles/r3_gemm4w_bounds.md)
__device__ __forceinline__ int bswz(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1) | (((r >> 4) & 1) << 2); }
// TLAY (row-layout accumulators, see frag_b): the 16 lanes of a fragment read rows j, 8 + j, ..., 120 + j -- row bits
// 3..5 give each group of 8 lanes distinct 16-byte chunks of its bank half
__device__ __forceinline__ int bswz2(int r) { return (r >> 3) & 7; }

// per-lane source offsets (bytes, relative to a K-tile's base) of the 8 LDS-DMA pieces this wave stages for one
// operand -- the same for every tile (edges are handled by the resource's num_records). T = 0: [rows][K] operand,
// piece P = 8 rows of 128 B (BI: the B image's swizzle); T = 1: [K][rows] operand, piece P = 4 k-rows x 128 columns
// of half P >> 4.
template <int T, bool BI = false, int PPW = 8, bool TL = false>
__device__ __forceinline__ void piece_offsets(int (&vo)[PPW], long long ld, int wave, int lane) {
#pragma unroll
  for (int q = 0; q < PPW; ++q) {
    const int P = wave * PPW + q;
    if (T == 0) {
      const int row = P * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (BI ? (TL ? bswz2(row) : bswz(row)) : ((row >> 1) & 7));
      vo[q] = (int)(row * ld * 2) + c * 16;
    } else {
      const int h = P >> 4, kr = (P & 15) * 4 + (lane >> 4);
      const int c = (lane & 15) ^ kswz(kr);
      vo[q] = (int)(kr * ld * 2) + (h * 128 + c * 8) * 2;
    }
  }
}

// fragment (16 rows/cols starting at rbase within the 256 of the tile) of k-substep kk from an operand image
template <int T>
__device__ __forceinline__ bf16x8_t frag(const char* img, int rbase, int kk, int lane) {
  if (T == 0) return read_frag<0>(img, rbase, kk, lane);
  return read_frag<1>(img + (rbase >> 7) * (Q_OP / 2), rbase & 127, kk, lane);
}

// B (output-column) fragment j of a wave's 128 columns at nbase, with the columns permuted inside each pair of
// fragments: fragment 2p + h, operand row r reads tile column nbase + 32p + 8 (r >> 2) + 4h + (r & 3). The MFMA
// puts operand rows 4g .. 4g+3 into lane row g's four accumulator registers, so after the pair each lane holds 8
// CONSECUTIVE output columns nbase + 32p + 8g .. +7 (fragment 2p: +0..3, 2p+1: +4..7) and the epilogue stores
// 16 bytes per lane without any cross-lane exchange. K-contiguous image: any row order is a gather of rows; the
// transposed image: each lane of a ds_read_b64_tr_b16 group addresses its own 4-column chunk.
//
// TL (K-contiguous B only): fragment j, operand column l reads tile column nbase + 8 l + j, and the MFMA takes the A
// fragment first. A lane's accumulators then hold rows 4g .. 4g+3 of its row block, and over the 8 fragments the 8
// CONSECUTIVE columns nbase + 8 l .. +7: lanes 0..15 of a store instruction write 256 contiguous bytes of one row
// (bf16; 4 rows per instruction) -- the row-contiguous pattern the store path takes ~4x faster than 64-byte pieces
// of 16 rows (tools/lab/store_bench.cpp). (The transposed image cannot: a ds_read_b64_tr_b16 group hands each lane
// 4 consecutive columns of one fragment.)
template <int T, bool TL = false>
__device__ __forceinline__ bf16x8_t frag_b(const char* img, int nbase, int j, int kk, int lane) {
  if constexpr (TL && T == 0) {
    const int r = nbase + 8 * (lane & 15) + j;
    const int c = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8_t*>(img + r * 128 + ((c ^ bswz2(r)) << 4));
  }
  const int base = nbase + 32 * (j >> 1) + 4 * (j & 1);
  if (T == 0) {
    const int r = base + 8 * ((lane & 15) >> 2) + (lane & 3);
    const int c = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8_t*>(img + r * 128 + ((c ^ bswz(r)) << 4));
  } else {
    const char* h = img + (base >> 7) * (Q_OP / 2);
    const int gg = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
    const int col = (base & 127) + 8 * pp;          // this lane's 4-column chunk (8-byte half j & 1 of a 16-B chunk)
    const int c = col >> 3;
    const int k0 = kk * 32 + 8 * gg + q, k1 = k0 + 4;
    const int off0 = k0 * 256 + ((c ^ kswz(k0)) << 4) + ((col & 4) << 1);
    const int off1 = k1 * 256 + ((c ^ kswz(k1)) << 4) + ((col & 4) << 1);
    s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, h + off0));
    s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, h + off1));
    s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}

// one output tile of the launch: operand bases at its first K-tile, the bytes left in each operand from there
// (the resource bound that zero-fills rows / columns past the edge), output origin
struct Tile4 {
  const char* a;
  const char* b;
  long long arem, brem;
  long long coff;
  int m0, n0, split, wsi;
  int nk;   // K-tiles of this tile (the K range of a triangular A, see decode4)
};

// split contraction index (GemmArgs::kin > 0, K-contiguous operands): contraction index k lives at element
// (k / kin) * sk + k % kin of a row -- the token mixer's weight gradient contracts over (batch, feature) pairs of a
// [B, S, H, F] tensor in place (kin = F, sk = S * H * F). Whole 64-deep K-tiles lie inside one kin block, and every
// split-K slab starts on a block boundary (obst_gemm), so a slab's first element is split * kin_bps * sk -- no
// runtime division (which the compiler would run in VGPRs and then feed to the SGPR-only asm operands).
template <bool KIN>
__device__ __forceinline__ long long kin_map(long long k, int split, const GemmArgs& p, long long sk) {
  return KIN ? (long long)split * p.kin_bps * sk : k;
}

// output tiles of a launch: tri 3 (only C[m][n], n <= m, receives the product; M == N) walks the lower-triangle tiles
// (the diagonal included) of every batch
__host__ __device__ __forceinline__ long long tiles_total(const GemmArgs& p) {
  const long long per = p.tri == 3 ? (long long)p.tiles_m * (p.tiles_m + 1) / 2 : (long long)p.tiles_m * p.tiles_n;
  return per * p.nbatch;
}

template <int A_T, int B_T, bool KIN = false>
__device__ __forceinline__ Tile4 decode4(const GemmArgs& p, long long L64) {
  // unsigned 32-bit index arithmetic (a launch has < 2^31 tiles): the 64-bit divisions were ~170 SALU ops on the
  // MFMA stream's critical path at every tile switch
  const unsigned L = (unsigned)L64;
  Tile4 T;
  int tm, tn;
  unsigned ybat;
  if (KIN && p.tri == 3) {
    // (the split-index instantiation only: the causal mixer weight gradient)
    // lower-triangle tiles of each batch, row by row: tile row tm holds tm + 1 tiles (tn <= tm); all of equal work
    const unsigned per = (unsigned)(p.tiles_m * (p.tiles_m + 1) / 2);
    unsigned bid = L % per;
    ybat = L / per;
    tm = 0;
    while (bid > (unsigned)tm) {   // at most tiles_m steps, once per tile switch
      bid -= (unsigned)tm + 1;
      ++tm;
    }
    tn = (int)bid;
  } else if (p.tri == 0) {
    const unsigned ntile = (unsigned)(p.tiles_m * p.tiles_n);
    const int bid = (int)(L % ntile);
    ybat = L / ntile;
    const int GROUP = 4;   // tile rows per N sweep: neighbouring CUs of an XCD share A panels and B panels
    const int per_group = GROUP * p.tiles_n;
    const int first_m = (bid / per_group) * GROUP;
    const int gsz = min(p.tiles_m - first_m, GROUP);
    tm = first_m + (bid % per_group) % gsz;
    tn = (bid % per_group) / gsz;
  } else if (p.tri_group == 0) {
    // triangular A (tri 1: A[m][k] = 0 for k > m, tri 2: for k < m): tile rows in order of decreasing K range,
    // the slowest index, so every round of the block-cyclic walk (logical4) holds tiles of equal work
    const unsigned per_row = (unsigned)p.tiles_n * (unsigned)p.nbatch;
    const int tmr = (int)(L / per_row);
    const unsigned rest = L % per_row;
    ybat = rest / (unsigned)p.tiles_n;
    tn = (int)(rest % (unsigned)p.tiles_n);
    tm = p.tri == 1 ? p.tiles_m - 1 - tmr : tmr;
  } else {
    // grouped order (tri_group G > 0): batches in groups of G, and inside a group the tile rows heaviest first with
    // the batch next -- the B operand of one batch (the token mixer's x[b, :, h, :]) is re-read by its tile rows
    // within one group's span instead of one whole sweep over the batch apart (L2 / MALL reuse). G a multiple of 8
    // keeps the XCD interleave (tile x + 8 j on XCD x) on the batches of one residue class.
    const unsigned G = (unsigned)p.tri_group, tmn = (unsigned)p.tiles_m, tnn = (unsigned)p.tiles_n;
    const unsigned block = tmn * G * tnn;
    const unsigned yg = L / block, r = L - yg * block;
    const unsigned left = (unsigned)p.nbatch - yg * G;
    const unsigned gsz = left < G ? left : G;   // (the last group may be short)
    const unsigned tmr = r / (gsz * tnn), r2 = r - tmr * (gsz * tnn);
    ybat = yg * G + r2 / tnn;
    tn = (int)(r2 % tnn);
    tm = p.tri == 1 ? p.tiles_m - 1 - (int)tmr : (int)tmr;
  }
  T.m0 = tm * 256;
  T.n0 = tn * 256;
  T.split = (int)(ybat % (unsigned)p.ksplit);   // split-K slab: ws [batch][split][M][N] (fold: splitk_reduce)
  const unsigned bidx = ybat / (unsigned)p.ksplit;
  T.wsi = (int)ybat;
  const long long b1 = bidx / (unsigned)p.nb2, b2 = bidx % (unsigned)p.nb2;
  long long kbeg = (long long)T.split * (p.K / p.ksplit);
  T.nk = p.K / p.ksplit / 64;
  if (p.tri == 1) {            // k < min(K, m0 + 256)
    T.nk = min(p.K, T.m0 + 256) / 64;
  } else if (p.tri == 2) {     // k >= m0
    kbeg = T.m0;
    T.nk = (p.K - T.m0) / 64;
  }
  const bf16_t* A = p.A + b1 * p.a_s1 + b2 * p.a_s2;
  const bf16_t* B = p.B + b1 * p.b_s1 + b2 * p.b_s2;
  // extent of each operand (elements from its batch base): [M][lda] rows / [K][lda] k-rows; with a split
  // contraction index (K-contiguous only) a row spans (K / kin - 1) * sk + kin elements
  const long long kext_a = KIN ? (long long)(p.kin_bps * p.ksplit - 1) * p.a_sk + p.kin : p.K;   // K / kin blocks
  const long long kext_b = KIN ? (long long)(p.kin_bps * p.ksplit - 1) * p.b_sk + p.kin : p.K;
  const long long aext = A_T == 0 ? (long long)(p.M - 1) * p.lda + kext_a : (long long)(p.K - 1) * p.lda + p.M;
  const long long bext = B_T == 0 ? (long long)(p.N - 1) * p.ldb + kext_b : (long long)(p.K - 1) * p.ldb + p.N;
  const long long aoff = A_T == 0 ? (long long)T.m0 * p.lda + kin_map<KIN>(kbeg, T.split, p, p.a_sk) : kbeg * p.lda + T.m0;
  const long long boff = B_T == 0 ? (long long)T.n0 * p.ldb + kin_map<KIN>(kbeg, T.split, p, p.b_sk) : kbeg * p.ldb + T.n0;
  T.a = reinterpret_cast<const char*>(A + aoff);
  T.b = reinterpret_cast<const char*>(B + boff);
  T.arem = (aext - aoff) * 2;
  T.brem = (bext - boff) * 2;
  T.coff = b1 * p.c_s1 + b2 * p.c_s2;
  return T;
}

// Persistent kernel: one block per CU walks its tiles; the LDS-DMA stream runs two K-tiles ahead of the MFMAs
// ACROSS tile boundaries (positions of a flat (tile, K-tile) sequence), so the next tile's first two K-tiles are
// in LDS when the current tile's epilogue is done, and its first fragments are read under the current tile's
// last MFMAs. XCD x owns a contiguous run of logical tiles, dealt to its CUs in rounds.
// NWV = 8 (G8W): two waves per SIMD, each owning 128 x 64 of C (8 x 4 accumulators, 128 AGPRs), 4 LDS-DMA pieces
// per operand and K-tile per wave and a 64-slot MFMA stream -- a wave's DMA issue cost (~60 cycles per piece, one
// wave per SIMD: nothing covers it) is hidden by its SIMD partner's MFMAs.
// Schedule SCH = 1 ("split", the K-loop structure of the library's 256x256x64 gfx950 kernel as read from its code
// object, profiles/r4_gemm_sched.md): one K-tile = 128 MFMA slots q, four barriers, each operand on its own pair:
//   q 1..15   substep-1 A fragments of this K-tile          q 20  lgkmcnt(0) + barrier: stage's A image free
//   q 22..58  A LDS-DMA pieces of position pos+2 (8)        q 24..42 substep-1 B fragments
//   q 50      lgkmcnt(0) + barrier: stage's B image free     q 61..124 B LDS-DMA pieces (8)
//   q 67      vmcnt(18) + barrier: A of pos+1 landed         q 69..83 substep-0 A fragments of pos+1
//   q 104     vmcnt(15) + barrier: B of pos+1 landed         q 106..120 substep-0 B fragments of pos+1
// vmcnt(18) at q 67 = B(pos+1) 8 + this K-tile's 8 A + 2 B pieces; vmcnt(15) at q 104 = 8 A + 7 B pieces.
// STG: waves on odd SIMDs run the same stream with every read / DMA one slot later (barriers fixed), so the four
// SIMDs' LDS-DMA issue and fragment reads do not hit the TA and LDS in the same cycles.
namespace g4s {
constexpr int A1[8] = {1, 3, 5, 7, 9, 11, 13, 15};
constexpr int B1[8] = {24, 27, 30, 33, 36, 38, 40, 42};
constexpr int DA[8] = {22, 25, 28, 31, 34, 52, 55, 58};
constexpr int DB[8] = {61, 64, 85, 87, 89, 95, 99, 124};
// SCH = 2 ("burst"): each operand's 8 pieces back to back (one per 2 MFMAs) right behind the barrier that frees it
constexpr int DA2[8] = {22, 24, 26, 28, 30, 32, 34, 36};
constexpr int DB2[8] = {52, 54, 56, 58, 60, 62, 64, 66};
constexpr int A0N[8] = {69, 71, 73, 75, 77, 79, 81, 83};
constexpr int B0N[8] = {106, 108, 110, 112, 114, 116, 118, 120};
constexpr int SETUP = 18, BAR_A = 20, BAR_B = 50, WA = 67, WB = 104, VA = 18, VB = 15;
constexpr int idx(const int (&a)[8], int q) {
  for (int i = 0; i < 8; ++i)
    if (a[i] == q) return i;
  return -1;
}
}  // namespace g4s

#ifndef G4W_SCH
#define G4W_SCH 1   // the split schedule (profiles/r4_gemm_sched.md): 1-5 % over SCH 0 on every measured shape
#endif
#ifndef G4W_STG
#define G4W_STG 0
#endif
#ifndef G4W_CPA
#define G4W_CPA 0   // 3 / 1: sc0 sc1 on the A stream, sc0 on B (as the library's kernel; within 0.3 %)
#endif
#ifndef G4W_CPB
#define G4W_CPB 0
#endif

#ifndef G4W_OPT
#define G4W_OPT 0   // 4: LATE (row layout: epilogue 8.6k -> 6.5k clocks, +0.5-1 % per shape in the lab, but the
                    // step measured 137.2k vs 138.8k tokens/s: off); 1: RELAX
#endif
// the stream-update epilogue with the next fragment row's residual loads ahead of this row's stores (emit_zpipe);
// 0: the plain per-row loads
#ifndef G4W_ZPIPE
#define G4W_ZPIPE 1
#endif
#ifndef G4W_TPM
#define G4W_TPM 3   // bit 0 residual, bit 1 gelu', bit 2 relu' (with all three the kernel hits "illegal VGPR to SGPR copy")
#endif
// the fp32 + bf16-copy (RevNet stream update) instantiation's options: its epilogue moves 10 bytes per output
#ifndef G4W_ZCP_OPT
#define G4W_ZCP_OPT G4W_OPT
#endif
// OPT bits (schedule options under A/B, tools/lab/g4w_sched.cpp):
//   1 RELAX: the first K-tile of every tile is a separate (peeled) copy whose waits count the previous tile's
//     direct-epilogue stores out (S = 32 bf16 / 64 fp32 stores per wave) instead of waiting for their write
//     acknowledgements; the prologue issues S stores to an empty buffer resource (dropped by the hardware, but
//     counted) so the first tile's first K-tile sees the same queue, and every epilogue that issues a different
//     number of stores (edge tiles, activations, residuals, the LDS path) drains vmcnt at its end
//   2 STAGGER: blocks start (slot & 7) / 8 of a tile apart (s_sleep), so the CUs' epilogue store bursts do not
//     coincide on the fabric
template <int A_T, int B_T, bool OUT_F32, bool PROF, int NWV = 4, int SCH = G4W_SCH, bool STG = (G4W_STG != 0),
          int CPA = G4W_CPA, int CPB = G4W_CPB, int OPT = G4W_OPT, bool KINT = false, bool ZCP = false,
          bool QUE = false>
__global__ __launch_bounds__(64 * NWV, 1) void gemm4w_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  constexpr bool RELAX = (OPT & 1) != 0, STAGGER = (OPT & 2) != 0, LATE = (OPT & 4) != 0;
  // split contraction index (+ tri 3): its own instantiation, so the plain kernel carries none of it
  constexpr bool KIN = KINT && A_T == 0 && B_T == 0;
  constexpr int SC = (OPT >> 3) & 7;   // cache policy of the direct epilogue's C stores
  constexpr bool ROWS = (OPT & 64) != 0;   // plain products: C rows staged through LDS, row-contiguous stores
  // TLAY: row-layout accumulators for K-contiguous B (frag_b): row-contiguous epilogue stores without data movement
  constexpr bool TLAY = B_T == 0 && NWV == 4 && (OPT & 256) == 0 && !ROWS;
  // fp32 output + its bf16 copy in Zout (the fused RevNet stream update): its own instantiation as well
  constexpr bool ZCOPY = ZCP && OUT_F32 && !ROWS;
  // dynamic tile queue (its own instantiation): a block's first tile is dealt statically, every later one is taken
  // from its XCD's counter (p.queue[xcd], zeroed before the launch) -- a block that starts late or runs slower
  // because another kernel (RCCL's collectives at N > 1) holds CUs beside it simply takes fewer tiles. Wave 0
  // dequeues the NEXT tile at the start of the current tile's first K-tile (one returning vector atomic), the
  // K-tile's own vmcnt wait retires it, wave 0 passes it through LDS before that K-tile's barrier; the DMA cursor
  // needs it by the end of K-tile nk - 3 (the host enables the queue only when every tile has nk >= 3: dense
  // products and the triangular token-mixer products, whose tiles are dequeued in decreasing-work order).
  constexpr bool QUEUE = QUE && !RELAX && !LATE && !KINT && !STG;

  static_assert(!(RELAX && LATE), "RELAX peels the first K-tile, LATE the last: not both");
  static_assert(SCH == 0 || NWV == 4, "the split schedule is laid out for one wave per SIMD");
  constexpr int WN = NWV == 4 ? 128 : 64;    // output columns per wave
  constexpr int JB = WN / 16;                // B fragments per substep
  constexpr int PPW = 32 / NWV;              // LDS-DMA pieces per operand, K-tile and wave
  constexpr int QS = 16 * JB;                // MFMA slots per K-tile
  constexpr int NR = 8 + JB;                 // fragment reads per substep
  constexpr int QB1 = NWV == 4 ? 25 : 14;    // barrier 1
  constexpr int QA0 = NWV == 4 ? 26 : 15, QB0 = NWV == 4 ? 66 : 31, DQ = NWV == 4 ? 5 : 4;   // DMA slots
  constexpr int QW = NWV == 4 ? 107 : 50;    // barrier 2
  constexpr int VA = SCH == 2 ? 24 : g4s::VA, VB = SCH == 2 ? 16 : g4s::VB;   // pieces younger than the awaited
  constexpr int SE = RELAX ? (OUT_F32 ? 64 : 32) : 0;   // stores of a plain direct epilogue per wave (RELAX)
  constexpr int VAF = VA + SE > 63 ? 63 : VA + SE, VBF = VB + SE > 63 ? 63 : VB + SE;
  constexpr int V0F = 2 * PPW + SE > 63 ? 63 : 2 * PPW + SE;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = NWV == 4 ? wave >> 1 : wave & 1, wn = NWV == 4 ? wave & 1 : wave >> 1;

  const long long total = KIN ? tiles_total(p) : (long long)p.tiles_m * p.tiles_n * p.nbatch;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;
  const long long Q = total >> 3, Rm = total & 7;
  // XCD x owns a run of logical tiles, its local index j -> tile gidx(j), walked by its blocks from slot (static
  // deal: j = slot, slot + nslot, ...; the queue: the first tile static, then j = nslot + dequeued index).
  // dense: a contiguous run (L2 sharing of A / B panels); triangular A: tiles x, x + 8, x + 16, ... -- decode4
  // orders the tiles by decreasing work, so every XCD takes its tiles heaviest first and the 8 XCDs get equal work
  // (the batch index runs fastest: XCD x keeps the heads of one residue class in its L2); tri 3: tiles of equal
  // work, dense walk
  const bool cyc = KIN ? (p.tri == 1 || p.tri == 2) : p.tri != 0;
  const long long start = cyc ? 0 : xcd < Rm ? xcd * (Q + 1) : Rm * (Q + 1) + (xcd - Rm) * Q;
  const long long len = cyc ? (total > xcd ? (total - xcd + 7) >> 3 : 0) : Q + (xcd < Rm ? 1 : 0);
  auto gidx = [&](long long j) { return cyc ? xcd + 8 * j : start + j; };
  const int ntiles = (int)(len > slot ? (len - slot + nslot - 1) / nslot : 0);   // statically dealt tiles
  if (ntiles == 0) return;   // (a small launch: the grid is rounded up to the 8 XCDs)
  auto logical = [&](int r) { return gidx(slot + (long long)r * nslot); };
  const long long astep = A_T == 0 ? 128 : 128 * p.lda;
  const long long bstep = B_T == 0 ? 128 : 128 * p.ldb;

  int voa[PPW], vob[PPW];
  piece_offsets<A_T, false, PPW>(voa, p.lda, wave, lane);
  piece_offsets<B_T, true, PPW, TLAY>(vob, p.ldb, wave, lane);
  const unsigned lds0 = lds_u32(smem);
  // this wave's PPW pieces of an operand image are contiguous: PPW KiB at (wave * PPW KiB)
  auto stage_a = [&](int s) -> unsigned { return lds0 + s * Q_STAGE + wave * PPW * 1024; };
  auto stage_b = [&](int s) -> unsigned { return lds0 + s * Q_STAGE + Q_OP + wave * PPW * 1024; };
  // SIMD of this wave (HW_ID bits 5:4): the stagger's parity
  const int simd_odd = STG ? (__builtin_amdgcn_s_getreg((4 << 0) | (4 << 6) | (0 << 11)) & 1) : 0;

  // DMA cursor: (tile round, K-tile) of the next position to stage; past the last tile it re-stages the last
  // position into the stage nobody reads any more
  // (the cursor's operand bases and bytes left advance by one K step in SALU adds; the resource clamps the bytes
  // left with a 32-bit select -- a K-tile's setup was ~30 VALU/SALU ops of 64-bit signed compares at one slot)
  int d_rnd = 0, d_kt = 0, d_nk = 0, d_kin = 0;   // d_kin: K-tiles left in the cursor's kin block
  unsigned long long cur_a, cur_b, rem_a, rem_b;
  // split contraction index: at a kin-block boundary the cursor also jumps over the rest of the outer stride
  // (only the K-contiguous pair can carry a split contraction index: obst_gemm; the other layouts compile it out)
  const int kin_tiles = KIN ? p.kin >> 6 : 0;
  auto cursor_tile = [&](const Tile4& T) {
    d_nk = T.nk;
    d_kin = kin_tiles;   // (slabs start on kin-block boundaries)
    cur_a = (unsigned long long)T.a;
    cur_b = (unsigned long long)T.b;
    rem_a = (unsigned long long)T.arem;   // > 0 at every position the cursor visits
    rem_b = (unsigned long long)T.brem;
  };
  cursor_tile(decode4<A_T, B_T, KIN>(p, logical(0)));
  auto rsrc_of = [](unsigned long long base, unsigned long long rem) {
    i32x4_t r;
    r[0] = (int)(unsigned)base;
    r[1] = (int)(unsigned)(base >> 32);
    unsigned hi = (unsigned)(rem >> 32);
    asm volatile("" : "+s"(hi));   // an opaque SGPR: the clamp stays a 32-bit SALU select (not a VALU 64-bit compare)
    r[2] = hi ? -1 : (int)(unsigned)rem;
    r[3] = 0x00020000;
    return r;
  };
  // QUEUE: the next tile (-1: none); static deal: tile 1 of the slot (q_next only steers the queue path)
  long long q_next = -1;
  unsigned q_ret = 0;
  const unsigned q_slot = lds0 + 2 * Q_STAGE + 32768 - 16;   // LDS address: the end of the epilogue region
  auto q_issue = [&]() {   // wave 0, lane 0: take the next index of this XCD's queue (returning vector atomic)
    if (wave == 0 && lane == 0) {
      unsigned* qp = p.queue + xcd;
      asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(q_ret) : "v"(qp), "v"(1u) : "memory");
    }
  };
  auto q_pin = [&]() { asm volatile("" : "+v"(q_ret)); };
  // after the K-tile's vmcnt wait: the returned index into LDS before its barrier (asm LDS ops: the compiler would
  // address a cast pointer generically, and a flat store waits for vmcnt(0), i.e. for every DMA in flight)
  auto q_publish = [&]() {
    if (wave == 0 && lane == 0) asm volatile("ds_write_b32 %0, %1" ::"v"(q_slot), "v"(q_ret) : "memory");
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the write is done before the barrier
  };
  auto q_take = [&]() {   // every wave: dynamic index i -> tile nslot + i of the XCD's range (the static tiles first)
    unsigned v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(q_slot) : "memory");
    const long long i = (long long)__builtin_amdgcn_readfirstlane(v);
    q_next = nslot + i < len ? gidx(nslot + i) : -1;
  };
  i32x4_t ra, rb;
  auto dma_setup = [&]() {   // resources of the cursor's K-tile
    ra = rsrc_of(cur_a, rem_a);
    rb = rsrc_of(cur_b, rem_b);
  };
  auto dma_advance = [&]() {
    if (d_kt + 1 < d_nk) {
      ++d_kt;
      cur_a += astep;
      rem_a -= astep;
      cur_b += bstep;
      rem_b -= bstep;
      if (KIN && --d_kin == 0) {   // (uniform; p.kin == 0 for every product but the mixer weight gradient)
        d_kin = kin_tiles;
        const unsigned long long ajump = (unsigned long long)(p.a_sk - p.kin) * 2;
        const unsigned long long bjump = (unsigned long long)(p.b_sk - p.kin) * 2;
        cur_a += ajump;
        rem_a -= ajump;
        cur_b += bjump;
        rem_b -= bjump;
      }
    } else if (QUEUE ? q_next >= 0 : d_rnd + 1 < ntiles) {
      // once per tile: the volatile asm keeps the compiler from if-converting the decode into every K-tile
      asm volatile("");
      ++d_rnd;
      d_kt = 0;
      cursor_tile(decode4<A_T, B_T, KIN>(p, QUEUE ? q_next : logical(d_rnd)));
    }
  };

  f32x4_t acc[8][JB];
  bf16x8_t a0[8], b0[JB], a1[8], b1f[JB];

  // read order of a substep's 16 fragments: A0, B0, A1..A7, B1..B7 (the order the MFMA stream consumes them)
  auto read_sub = [&](int s, auto kkc, auto rc, bf16x8_t (&af)[8], bf16x8_t (&bf)[JB]) {
    constexpr int kk = decltype(kkc)::value, r = decltype(rc)::value;
    const char* ia = smem + s * Q_STAGE;
    const char* ib = smem + s * Q_STAGE + Q_OP;
    if constexpr (r == 0) af[0] = frag<A_T>(ia, wm * 128, kk, lane);
    else if constexpr (r == 1) bf[0] = frag_b<B_T, TLAY>(ib, wn * WN, 0, kk, lane);
    else if constexpr (r < 9) af[r - 1] = frag<A_T>(ia, wm * 128 + (r - 1) * 16, kk, lane);
    else bf[r - 8] = frag_b<B_T, TLAY>(ib, wn * WN, r - 8, kk, lane);
  };
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;

  // diagnostic timestamps (GemmArgs::stamps, null in production): per block [start, first tile landed, summed
  // loop clocks, summed epilogue clocks], the XCC id, [start, end] in 100 MHz real time, tiles
  const bool stamp = p.stamps != nullptr && tid == 0;
  const long long sbase = (long long)blockIdx.x * 8;
  unsigned long long loop_clk = 0, epi_clk = 0, tmark = 0, sync1 = 0, sync2 = 0, tw = 0, epi_issue = 0;
  if (stamp) {
    p.stamps[sbase] = __builtin_amdgcn_s_memtime();
    p.stamps[sbase + 4] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));   // HW_REG_XCC_ID[3:0]
    p.stamps[sbase + 5] = __builtin_amdgcn_s_memrealtime();
    p.stamps[sbase + 7] = ntiles;
  }

  // the whole tile walk, its event stream shifted by SH slots on odd SIMDs (STG): two copies of the kernel body
  // that meet only after the last tile (a branch per K-tile put a phi over the 256 accumulators: spills)
  auto body = [&](auto shc) {
    constexpr int SH = decltype(shc)::value;
    if constexpr (STAGGER) {   // ~1/8 of a 2048-deep tile per slot step
      for (int d = 0; d < 3 * (slot & 7); ++d) __builtin_amdgcn_s_sleep(64);
    }
    // prologue: positions 0 and 1 into stages 0 and 1, wait for position 0, read its substep-0 fragments
    dma_setup();
  #pragma unroll
    for (int q = 0; q < PPW; ++q) dma16<CPA>(ra, voa[q], stage_a(0) + q * 1024);
  #pragma unroll
    for (int q = 0; q < PPW; ++q) dma16<CPB>(rb, vob[q], stage_b(0) + q * 1024);
    dma_advance();
    dma_setup();
  #pragma unroll
    for (int q = 0; q < PPW; ++q) dma16<CPA>(ra, voa[q], stage_a(1) + q * 1024);
  #pragma unroll
    for (int q = 0; q < PPW; ++q) dma16<CPB>(rb, vob[q], stage_b(1) + q * 1024);
    dma_advance();
    if constexpr (RELAX) {   // SE stores into an empty resource: dropped, but counted like an epilogue's
      const i32x4_t nul = make_rsrc(p.C, 0);
      static_for<SE>([&](auto) {
        store16_padded(v4u32_t{0u, 0u, 0u, 0u}, 0, nul, std::integral_constant<int, 0>{});
      });
      vm_wait<V0F>();
    } else {
      vm_wait<2 * PPW>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);   // nothing (kernel-argument loads) pending in lgkmcnt at the loop entry
    if (stamp) p.stamps[sbase + 1] = __builtin_amdgcn_s_memtime();
    fence();
    if constexpr (!LATE) static_for<NR>([&](auto rc) { read_sub(0, K0{}, rc, a0, b0); fence(); });   // loop order

    int pos = 0;   // flat position of the K-tile being multiplied (its stage is pos & 1)
    long long q_cur = logical(0);   // QUEUE: the tile being multiplied
    for (int rnd = 0; QUEUE ? q_cur >= 0 : rnd < ntiles; ++rnd) {
      const Tile4 ct = decode4<A_T, B_T, KIN>(p, QUEUE ? q_cur : logical(rnd));
      // Accumulator zeroing (VALU writes of AGPRs) -> first MFMA reading them needs wait states the compiler cannot
      // see through the asm MFMAs; the empty "+a" asms pin the zeros before the pad (no rematerialisation past it)
  #pragma unroll
      for (int i = 0; i < 8; ++i)
  #pragma unroll
        for (int j = 0; j < JB; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      static_for<8 * JB>([&](auto c) { agpr_opaque(acc[decltype(c)::value / JB][decltype(c)::value % JB]); });
      asm volatile("s_nop 4" ::: "memory");
      fence();
      // LATE: this tile's first substep-0 fragments are read here, not by the previous tile's last K-tile (whose
      // 64 fragment VGPRs then stayed live through the epilogue: spills, and each reload waited on vmcnt)
      if constexpr (LATE) static_for<NR>([&](auto rc) { read_sub(pos & 1, K0{}, rc, a0, b0); fence(); });
      if (stamp) tmark = __builtin_amdgcn_s_memtime();

      // one K-tile (position pos in stage s), its event stream shifted by SH slots (the stagger)
      // The waits count the pieces younger than the awaited ones in the steady state. At the first K-tile of a
      // tile the previous tile's epilogue stores sit in between, so the same count also waits for the older stores
      // -- issued ~60 MFMAs earlier, they have retired by then; a relaxed count for that K-tile needs a runtime
      // branch at every wait or a second copy of the K-tile, and the copy's phi over the 256 accumulators spills.
      auto ktile = [&](auto fc, auto lc, int s, auto hc) {
        constexpr bool QH = decltype(hc)::value && QUEUE;   // this K-tile publishes the dequeued index
        constexpr bool FIRST = decltype(fc)::value && RELAX;
        constexpr bool NEXT0 = !(decltype(lc)::value && LATE);   // read pos+1's substep-0 fragments in this K-tile
        const unsigned sa = stage_a(s), sb = stage_b(s);
        static_for<QS>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          constexpr int sub = q / (8 * JB), j = (q % (8 * JB)) / 8, i = q & 7;
          if constexpr (TLAY) {   // A first: row-layout accumulators (frag_b)
            if constexpr (sub == 0) mfma_acc(acc[i][j], a0[i], b0[j]);
            else mfma_acc(acc[i][j], a1[i], b1f[j]);
          } else {
            if constexpr (sub == 0) mfma_acc(acc[i][j], b0[j], a0[i]);
            else mfma_acc(acc[i][j], b1f[j], a1[i]);
          }
          if constexpr (SCH == 0) {
            if constexpr (q < NR && !(G4W_EXP & 2)) read_sub(s, K1{}, qc, a1, b1f);   // substep-1 fragments of pos
            if constexpr (q == NR) dma_setup();                                 // resources of position pos + 2
            if constexpr (q == QB1) {                                           // stage s fully read by every wave
              if constexpr (PROF) tw = __builtin_amdgcn_s_memtime();
              __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0) as a builtin: the compiler's wait model learns the
              if constexpr (!(G4W_EXP & 4)) __builtin_amdgcn_s_barrier();   // substep-1 reads are done
              if constexpr (PROF) sync1 += __builtin_amdgcn_s_memtime() - tw;
            }
            if constexpr (!(G4W_EXP & 1) && q >= QA0 + SH && q < QA0 + SH + DQ * PPW && (q - QA0 - SH) % DQ == 0)
              dma16o<CPA, (q - QA0 - SH) / DQ * 1024>(ra, voa[(q - QA0 - SH) / DQ], sa);
            if constexpr (!(G4W_EXP & 1) && q >= QB0 + SH && q < QB0 + SH + DQ * PPW && (q - QB0 - SH) % DQ == 0)
              dma16o<CPB, (q - QB0 - SH) / DQ * 1024>(rb, vob[(q - QB0 - SH) / DQ], sb);
            if constexpr (q == QW) {                                            // position pos+1 landed in stage s^1
              // first K-tile of a tile: the previous tile's epilogue stores sit between that position's DMAs and
              // this iteration's; count them out instead of waiting for every store (direct epilogue: 32 bf16 /
              // 64 fp32)
              if constexpr (PROF) tw = __builtin_amdgcn_s_memtime();
              if constexpr (FIRST) vm_wait<V0F>();
              else vm_wait<2 * PPW>();
              if constexpr (QH) q_publish();   // the dequeued index (retired by the wait above) to every wave
              if constexpr (!(G4W_EXP & 4)) __builtin_amdgcn_s_barrier();
              if constexpr (PROF) sync2 += __builtin_amdgcn_s_memtime() - tw;
            }
            if constexpr (NEXT0 && q > QW && q <= QW + NR && !(G4W_EXP & 2))   // substep-0 fragments of pos+1
              read_sub(s ^ 1, K0{}, std::integral_constant<int, q - QW - 1>{}, a0, b0);
          } else {
            const char* ia = smem + s * Q_STAGE;
            const char* ib = ia + Q_OP;
            constexpr int ra1 = g4s::idx(g4s::A1, q - SH), rb1 = g4s::idx(g4s::B1, q - SH);
            constexpr int da = g4s::idx(SCH == 2 ? g4s::DA2 : g4s::DA, q - SH);
            constexpr int db = g4s::idx(SCH == 2 ? g4s::DB2 : g4s::DB, q - SH);
            constexpr int ra0 = g4s::idx(g4s::A0N, q - SH), rb0 = g4s::idx(g4s::B0N, q - SH);
            if constexpr (ra1 >= 0) a1[ra1] = frag<A_T>(ia, wm * 128 + ra1 * 16, 1, lane);
            if constexpr (rb1 >= 0) b1f[rb1] = frag_b<B_T, TLAY>(ib, wn * WN, rb1, 1, lane);
            if constexpr (q == g4s::SETUP) dma_setup();
            if constexpr (q == g4s::BAR_A || q == g4s::BAR_B) {   // every wave done reading this stage's A / B image
              if constexpr (PROF) tw = __builtin_amdgcn_s_memtime();
              __builtin_amdgcn_s_waitcnt(0xc07f);
              __builtin_amdgcn_s_barrier();
              if constexpr (PROF) sync1 += __builtin_amdgcn_s_memtime() - tw;
            }
            if constexpr (!(G4W_EXP & 1) && da >= 0) dma16o<CPA, (da < 0 ? 0 : da) * 1024>(ra, voa[da], sa);
            if constexpr (!(G4W_EXP & 1) && db >= 0) dma16o<CPB, (db < 0 ? 0 : db) * 1024>(rb, vob[db], sb);
            if constexpr (q == g4s::WA || q == g4s::WB) {   // A / B image of position pos+1 landed in stage s^1
              if constexpr (PROF) tw = __builtin_amdgcn_s_memtime();
              if constexpr (FIRST) vm_wait<q == g4s::WA ? VAF : VBF>();
              else vm_wait<q == g4s::WA ? VA : VB>();
              // the atomic was issued before every DMA of this K-tile: at WB at most VB (< the K-tile's own pieces
              // issued so far) are younger, so it has retired
              if constexpr (QH && q == g4s::WB) q_publish();
              __builtin_amdgcn_s_barrier();
              if constexpr (PROF) sync2 += __builtin_amdgcn_s_memtime() - tw;
            }
            if constexpr (NEXT0 && ra0 >= 0)
              a0[ra0] = frag<A_T>(smem + (s ^ 1) * Q_STAGE, wm * 128 + ra0 * 16, 0, lane);
            if constexpr (NEXT0 && rb0 >= 0)
              b0[rb0] = frag_b<B_T, TLAY>(smem + (s ^ 1) * Q_STAGE + Q_OP, wn * WN, rb0, 0, lane);
          }
          fence();
          // the dequeue's destination register has no hardware interlock: until the wait at WB retires the atomic,
          // the empty asm at every slot keeps the value where the atomic writes it (no copy or spill reads it early)
          if constexpr (QH && q < g4s::WB) q_pin();
        });
      };

      using T_ = std::true_type;
      using F_ = std::false_type;
      if constexpr (RELAX) {   // the first K-tile peeled (sequential copies: no phi over the accumulators)
        ktile(T_{}, F_{}, pos & 1, F_{});
        dma_advance();
        ++pos;
        for (int t = 1; t < ct.nk; ++t, ++pos) {
          ktile(F_{}, F_{}, pos & 1, F_{});
          dma_advance();
        }
      } else if constexpr (LATE) {   // the last K-tile peeled
        for (int t = 0; t < ct.nk - 1; ++t, ++pos) {
          ktile(F_{}, F_{}, pos & 1, F_{});
          dma_advance();
        }
        ktile(F_{}, T_{}, pos & 1, F_{});
        dma_advance();
        ++pos;
      } else if constexpr (QUEUE) {
        q_issue();   // the first K-tile peeled: it carries the dequeue (no runtime branch inside the MFMA stream)
        ktile(F_{}, F_{}, pos & 1, T_{});
        q_take();
        dma_advance();
        ++pos;
        for (int t = 1; t < ct.nk; ++t, ++pos) {
          ktile(F_{}, F_{}, pos & 1, F_{});
          dma_advance();
        }
      } else {
        for (int t = 0; t < ct.nk; ++t, ++pos) {
          ktile(F_{}, F_{}, pos & 1, F_{});
          dma_advance();
        }
      }
      // last MFMA -> accumulator reads: the pad redefines every accumulator ("+a"), so the register allocator's
      // AGPR -> VGPR copies for the epilogue (which fences do not bind) can only read them after it
      fence();
      pad_redefine(acc);
      fence();
      if (stamp) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        loop_clk += now - tmark;
        tmark = now;
      }

      // gelu / relu GEMMs (bf16, no residual) take the direct epilogue too: forward with the pre-activation kept in
      // Zout, backward C = acc * act'(Zin); each variant's activation is straight-line code (no per-value switch).
      // (relu through the LDS-path epilogue was 768 us per 65536 x 4096 x 256 product of ctx32_mixer: 179 TF/s)
      // (relu on the row-layout path only: with both activations the fragment-layout copies hit the compiler's
      // "illegal VGPR to SGPR copy")
      const bool gelu_direct = !OUT_F32 && (p.act == ACT_GELU || (TLAY && p.act == ACT_RELU)) && p.R == nullptr &&
                               ((p.mode == 0) || (p.mode == 1 && p.Zin != nullptr));
      // fp32 products with Zout (its bf16 copy, the fused RevNet stream update) take the direct path
      const bool zcopy_direct = ZCOPY && p.act == 0 && p.mode == 0 && p.ksplit == 1;
      if (!(G4W_EXP & 16) && ((p.act == 0 && p.mode == 0 && p.Zout == nullptr) || gelu_direct || zcopy_direct)) {
        // Direct epilogue (every plain product): each lane owns C[m][n..n+3] of 64 fragments and writes it with one
        // buffer store from the accumulators (bf16: 8 B, fp32: 16 B); one per-lane offset, the fragment row in the
        // SGPR offset, the fragment column in the instruction's immediate; rows past M fall outside the resource
        // (dropped), columns past N are masked on the last tile column only.
        const bool ws_out = OUT_F32 && p.ksplit > 1;
        const long long ldc = ws_out ? p.N : p.ldc;
        constexpr int ES = OUT_F32 ? 4 : 2;
        // split-K partials: slab (batch, split) = ybat of the tile (decode4: ybat = batch * ksplit + split)
        char* cbase = ws_out ? reinterpret_cast<char*>(p.ws + (long long)ct.wsi * p.M * p.N)
                             : reinterpret_cast<char*>(p.C) + ct.coff * ES;
        const long long corg = ((long long)ct.m0 * ldc + ct.n0) * ES;
        const long long cext = ((long long)(p.M - ct.m0 - 1) * ldc + (p.N - ct.n0)) * ES;   // bytes to C's end
        const __amdgpu_buffer_rsrc_t rc = make_brsrc(cbase + corg, cext);
        const i32x4_t rc4 = make_rsrc(cbase + corg, cext);
        const __amdgpu_buffer_rsrc_t rr = make_brsrc(p.R ? reinterpret_cast<const char*>(p.R) + ct.coff * ES + corg : cbase, cext);
        const int ml = lane & 15, gq = lane >> 4;
        const float alpha = p.alpha, beta = ws_out ? 0.f : p.beta;

        // ROWS / TLAY mask columns per lane at run time in one copy of each variant
        const bool edge = !ROWS && !TLAY && ct.n0 + wn * WN + WN > p.N;
        const bool extra = (OUT_F32 && beta != 0.f) || (p.R != nullptr && !ws_out);
        // fragment pair (2p, 2p+1) = 8 consecutive columns per lane (frag_b): 16 B (bf16) / 2 x 16 B (fp32) stores,
        // 32 / 64 per wave (64 bf16 stores with the 32 LDS-DMAs in flight overflowed the 63-entry vmcnt)
        // leading dimension through an opaque SGPR: the per-lane offsets below are then computed here, per tile
        // (a few VALU ops) -- hoisted out of the tile loop they stayed live across the K loop, spilled to scratch,
        // and every reload's vmcnt wait also waited for the next tile's in-flight LDS-DMAs
        int ldcs = (int)ldc;
        asm volatile("" : "+s"(ldcs));
        const int voff = ((wm * 128 + ml) * ldcs + wn * WN + 8 * gq) * ES;
        const int nbase = ct.n0 + wn * WN + 8 * gq;
        // Zout / Zin share C's leading dimension and batch offset (bf16)
        // (fp32 C, row layout: Zout is the output's bf16 copy, C's geometry at 2 bytes per element)
        constexpr bool ZC = ZCOPY;
        const i32x4_t rz4 = make_rsrc(p.Zout ? reinterpret_cast<const char*>(p.Zout) + ct.coff * 2 + (ZC ? corg / 2 : corg)
                                             : cbase,
                                      ZC ? cext / 2 : cext);
        const __amdgpu_buffer_rsrc_t rzi =
            make_brsrc(p.Zin ? reinterpret_cast<const char*>(p.Zin) + ct.coff * 2 + corg : cbase, cext);
        const bool zout = p.Zout != nullptr;
        // AC: 0 no activation, 1 gelu forward (+ Zout), 2 gelu backward (Zin)
        auto emit = [&](auto exc, auto edc, auto acc_) {
          constexpr bool EX = decltype(exc)::value, ED = decltype(edc)::value;
          constexpr int AC_ = decltype(acc_)::value;
          // AC_: 1 / 2 gelu forward / backward, 3 / 4 relu forward / backward -> AC (1 forward, 2 backward) + ACTK
          constexpr int AC = AC_ == 0 ? 0 : (AC_ == 1 || AC_ == 3) ? 1 : 2;
          constexpr int ACTK = AC_ >= 3 ? ACT_RELU : ACT_GELU;
          if constexpr (TLAY) {
            // row-layout accumulators (frag_b): lane (ml, gq) holds rows 16 i + 4 gq + r (r = 0..3) of the wave's
            // block at columns 8 ml .. +7 (acc[i][0..7][r]); every store / side load covers 4 rows x 256 B (bf16) or
            // 4 rows x 2 x 16 B per 32-byte chunk (fp32)
            const int vt = ((wm * 128 + 4 * gq) * ldcs + wn * WN + 8 * ml) * ES;
            const bool colok = ct.n0 + wn * WN + 8 * ml < p.N;
            static_for<8>([&](auto ic) {
              constexpr int i = decltype(ic)::value;
              int vro[4];
              v4u32_t side[4], side2[4], cl0[4], cl1[4];
              static_for<4>([&](auto rk) {   // side inputs of the 4 rows first
                constexpr int r = decltype(rk)::value;
                vro[r] = vt + (16 * i + r) * ES * ldcs;
                if constexpr (AC == 2) side[r] = __builtin_amdgcn_raw_buffer_load_b128(rzi, vro[r], 0, 0);
                if constexpr (EX) {
                  side[r] = __builtin_amdgcn_raw_buffer_load_b128(rr, vro[r], 0, 0);
                  if constexpr (OUT_F32) {
                    side2[r] = __builtin_amdgcn_raw_buffer_load_b128(rr, vro[r] + 16, 0, 0);
                    if (beta != 0.f) {
                      cl0[r] = __builtin_amdgcn_raw_buffer_load_b128(rc, vro[r], 0, 0);
                      cl1[r] = __builtin_amdgcn_raw_buffer_load_b128(rc, vro[r] + 16, 0, 0);
                    }
                  }
                }
              });
              v4u32_t o0[4], o1[4], zo[4];
              static_for<4>([&](auto rk) {
                constexpr int r = decltype(rk)::value;
                float x[8];
                static_for<8>([&](auto jc) {
                  constexpr int j = decltype(jc)::value;
                  x[j] = alpha * acc[i][j][r];
                });
                if constexpr (OUT_F32) {
                  if constexpr (EX) {
                    const f32x4_t ra = __builtin_bit_cast(f32x4_t, side[r]), rb = __builtin_bit_cast(f32x4_t, side2[r]);
                    if (beta != 0.f) {
                      const f32x4_t ca = __builtin_bit_cast(f32x4_t, cl0[r]), cb = __builtin_bit_cast(f32x4_t, cl1[r]);
                      static_for<4>([&](auto tc) {
                        constexpr int t = decltype(tc)::value;
                        x[t] += beta * ca[t];
                        x[4 + t] += beta * cb[t];
                      });
                    }
                    if (p.R) {
                      static_for<4>([&](auto tc) {
                        constexpr int t = decltype(tc)::value;
                        x[t] += ra[t];
                        x[4 + t] += rb[t];
                      });
                    }
                  }
                  o0[r] = __builtin_bit_cast(v4u32_t, f32x4_t{x[0], x[1], x[2], x[3]});
                  o1[r] = __builtin_bit_cast(v4u32_t, f32x4_t{x[4], x[5], x[6], x[7]});
                  if constexpr (ZCOPY)
                    zo[r] = v4u32_t{pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]), pack_bf16x2(x[4], x[5]),
                                    pack_bf16x2(x[6], x[7])};
                } else {
                  if constexpr (EX) {
                    static_for<4>([&](auto tc) {
                      constexpr int t = decltype(tc)::value;
                      x[2 * t] += bf2f(side[r][t] & 0xffff);
                      x[2 * t + 1] += bf2f(side[r][t] >> 16);
                    });
                  }
                  if constexpr (AC == 1) {
                    zo[r] = v4u32_t{pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]), pack_bf16x2(x[4], x[5]),
                                    pack_bf16x2(x[6], x[7])};
                    static_for<8>([&](auto tc) { x[decltype(tc)::value] = act_fwd(ACTK, x[decltype(tc)::value]); });
                  } else if constexpr (AC == 2) {
                    static_for<4>([&](auto tc) {
                      constexpr int t = decltype(tc)::value;
                      x[2 * t] *= act_grad(ACTK, bf2f(side[r][t] & 0xffff));
                      x[2 * t + 1] *= act_grad(ACTK, bf2f(side[r][t] >> 16));
                    });
                  }
                  o0[r] = v4u32_t{pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]), pack_bf16x2(x[4], x[5]),
                                  pack_bf16x2(x[6], x[7])};
                }
              });
              static_for<4>([&](auto rk) {   // then every store (no activation code between them)
                constexpr int r = decltype(rk)::value;
                if constexpr (AC == 1) {
                  if (zout && colok) store16_nc<SC>(zo[r], vro[r], rz4);
                }
                if (colok) {
                  store16_nc<SC>(o0[r], vro[r], rc4);
                  if constexpr (OUT_F32) {
                    store16_nc<SC>(o1[r], vro[r] + 16, rc4);
                    if constexpr (ZCOPY) {
                      if (zout) store16_nc<SC>(zo[r], vro[r] >> 1, rz4);   // the bf16 copy (2 of C's 4 bytes)
                    }
                  }
                }
              });
              fence();
            });
            if constexpr (PROF) {
              if (stamp) epi_issue += __builtin_amdgcn_s_memtime() - tmark;
            }
            if constexpr (EX || AC == 2 || (RELAX && (ED || AC != 0))) __builtin_amdgcn_s_waitcnt(0x0f70);
            return;
          }
          if constexpr (ROWS) {
            // ROWS: a lane's accumulators hold one row's 16-byte column chunk each, so a direct store instruction
            // writes 64-byte pieces of 16 rows; the store path takes ~4x longer for that pattern than for whole row
            // segments (tools/lab/store_bench.cpp: 8.3k vs 2.2k clocks per 256 x 256 bf16 tile and CU). Staged
            // through the wave's LDS region, each store instruction writes 4 (bf16) / 2 (fp32) rows of 256 / 512 B,
            // and the epilogue's side inputs (residual, Zin, C for beta) are read in the same row layout.
            // bf16: alpha * acc staged as bf16 (the output precision) in two 4 KiB buffers, the next fragment row
            // written while this one is read back; fp32: one 8 KiB buffer.
            constexpr int CPR = WN * ES / 16;   // 16-byte chunks per row of the wave's tile: 16 (bf16) / 32 (fp32)
            constexpr int RPI = 64 / CPR;       // rows per store instruction
            constexpr int NRD = 16 / RPI;       // store instructions per fragment row
            char* epb = smem + 2 * Q_STAGE + wave * 16 * WN * 4;
            const int rr0 = lane / CPR, cc = lane % CPR;
            const int vb = ((wm * 128 + rr0) * ldcs + wn * WN + cc * (16 / ES)) * ES;
            const bool colok = ct.n0 + wn * WN + cc * (16 / ES) < p.N;   // (every tile: one ROWS copy per variant)
            auto write_row = [&](auto ic, char* buf) {
              constexpr int i = decltype(ic)::value;
              if constexpr (OUT_F32) {
                static_for<JB>([&](auto jc) {
                  constexpr int j = decltype(jc)::value;
                  const int c4 = 8 * (j >> 1) + 2 * gq + (j & 1);   // frag_b column order, 16-byte units
                  *reinterpret_cast<f32x4_t*>(buf + ml * (CPR * 16) + ((c4 ^ ml) & (CPR - 1)) * 16) =
                      alpha * acc[i][j];
                });
              } else {
                static_for<JB / 2>([&](auto pc) {
                  constexpr int pp = decltype(pc)::value;
                  const f32x4_t va = alpha * acc[i][2 * pp], vb2 = alpha * acc[i][2 * pp + 1];
                  *reinterpret_cast<v4u32_t*>(buf + ml * (CPR * 16) + (((pp * 4 + gq) ^ ml) & (CPR - 1)) * 16) =
                      v4u32_t{pack_bf16x2(va[0], va[1]), pack_bf16x2(va[2], va[3]), pack_bf16x2(vb2[0], vb2[1]),
                              pack_bf16x2(vb2[2], vb2[3])};
                });
              }
            };
            auto unpack8 = [](const v4u32_t& o, float (&x)[8]) {
              static_for<4>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                x[2 * t] = bf2f(o[t] & 0xffff);
                x[2 * t + 1] = bf2f(o[t] >> 16);
              });
            };
            auto read_store_row = [&](auto ic, const char* buf) {
              constexpr int i = decltype(ic)::value;
              v4u32_t v[NRD], side[NRD], cold[NRD];
              int vro[NRD];
              static_for<NRD>([&](auto rk) {   // every read first: one LDS latency per fragment row
                constexpr int r = decltype(rk)::value;
                const int R = r * RPI + rr0;
                vro[r] = vb + (i * 16 + r * RPI) * ES * ldcs;
                v[r] = *reinterpret_cast<const v4u32_t*>(buf + R * (CPR * 16) + ((cc ^ R) & (CPR - 1)) * 16);
                if constexpr (AC == 2) side[r] = __builtin_amdgcn_raw_buffer_load_b128(rzi, vro[r], 0, 0);
                if constexpr (EX) {
                  side[r] = __builtin_amdgcn_raw_buffer_load_b128(rr, vro[r], 0, 0);
                  if constexpr (OUT_F32) cold[r] = __builtin_amdgcn_raw_buffer_load_b128(rc, vro[r], 0, 0);
                }
              });
              // the outputs first, then every store (activation code between the stores moved the resource
              // operands into VGPRs: "illegal VGPR to SGPR copy")
              v4u32_t out[NRD];
              static_for<NRD>([&](auto rk) {
                constexpr int r = decltype(rk)::value;
                if constexpr (AC == 0 && !EX) {
                  out[r] = v[r];
                } else if constexpr (OUT_F32) {   // EX: beta * C (+ R), fp32
                  f32x4_t x = __builtin_bit_cast(f32x4_t, v[r]);
                  if (beta != 0.f) x += beta * __builtin_bit_cast(f32x4_t, cold[r]);
                  if (p.R) x += __builtin_bit_cast(f32x4_t, side[r]);
                  out[r] = __builtin_bit_cast(v4u32_t, x);
                } else {
                  float x[8];
                  unpack8(v[r], x);
                  if constexpr (EX) {
                    float y[8];
                    unpack8(side[r], y);
                    static_for<8>([&](auto tc) { x[decltype(tc)::value] += y[decltype(tc)::value]; });
                  }
                  if constexpr (AC == 1) {
                    static_for<8>([&](auto tc) { x[decltype(tc)::value] = act_fwd(ACTK, x[decltype(tc)::value]); });
                  } else if constexpr (AC == 2) {
                    float z[8];
                    unpack8(side[r], z);
                    static_for<8>([&](auto tc) {
                      constexpr int t = decltype(tc)::value;
                      x[t] *= act_grad(ACTK, z[t]);
                    });
                  }
                  out[r] = v4u32_t{pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]), pack_bf16x2(x[4], x[5]),
                                   pack_bf16x2(x[6], x[7])};
                }
              });
              static_for<NRD>([&](auto rk) {
                constexpr int r = decltype(rk)::value;
                if constexpr (AC == 1) {
                  if (zout && colok) store16_nc<SC>(v[r], vro[r], rz4);   // the bf16 pre-activation
                }
                if (colok) store16_nc<SC>(out[r], vro[r], rc4);
              });
            };
            if constexpr (!OUT_F32) {
              char* const bufs[2] = {epb, epb + 16 * CPR * 16};
              write_row(std::integral_constant<int, 0>{}, bufs[0]);
              static_for<8>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                if constexpr (i + 1 < 8) write_row(std::integral_constant<int, i + 1>{}, bufs[(i + 1) & 1]);
                read_store_row(ic, bufs[i & 1]);
                fence();
              });
            } else {
              static_for<8>([&](auto ic) {
                write_row(ic, epb);
                read_store_row(ic, epb);
                fence();
              });
            }
            if constexpr (PROF) {
              if (stamp) epi_issue += __builtin_amdgcn_s_memtime() - tmark;
            }
            // loads into VGPRs (residual / Zin / C) retired here, as in the fragment-layout path below
            if constexpr (EX || AC == 2 || (RELAX && (ED || AC != 0))) __builtin_amdgcn_s_waitcnt(0x0f70);
            return;
          }
          // one fragment row at a time: with EX its residual / C loads are issued together and consumed after,
          // bounded by the fences (unbounded, the scheduler hoisted all 64 loads: 256 VGPRs, spills)
          static_for<8>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            // the fragment row goes into the VGPR offset: a raw buffer's range check covers the VGPR offset and
            // the immediate but not soffset, so rows past M (ragged M) must be in voff to be dropped
            const int vrow = voff + i * 16 * ES * ldcs;
            f32x4_t x[8];
            if constexpr (AC == 2) {
              static_for<JB / 2>([&](auto pc) {
                constexpr int pp = decltype(pc)::value;
                const v4u32_t o = __builtin_amdgcn_raw_buffer_load_b128(rzi, vrow + pp * 64, 0, 0);
                x[2 * pp] = f32x4_t{bf2f(o[0] & 0xffff), bf2f(o[0] >> 16), bf2f(o[1] & 0xffff), bf2f(o[1] >> 16)};
                x[2 * pp + 1] = f32x4_t{bf2f(o[2] & 0xffff), bf2f(o[2] >> 16), bf2f(o[3] & 0xffff), bf2f(o[3] >> 16)};
              });
            }
            if constexpr (EX) {
              static_for<JB / 2>([&](auto pc) {
                constexpr int pp = decltype(pc)::value;
                if constexpr (OUT_F32) {
                  x[2 * pp] = x[2 * pp + 1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
                  if (beta != 0.f) {
                    x[2 * pp] = beta * __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rc, vrow + pp * 128, 0, 0));
                    x[2 * pp + 1] = beta * __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rc, vrow + pp * 128 + 16, 0, 0));
                  }
                  if (p.R) {
                    x[2 * pp] += __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rr, vrow + pp * 128, 0, 0));
                    x[2 * pp + 1] += __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rr, vrow + pp * 128 + 16, 0, 0));
                  }
                } else {
                  const v4u32_t o = __builtin_amdgcn_raw_buffer_load_b128(rr, vrow + pp * 64, 0, 0);
                  x[2 * pp] = f32x4_t{bf2f(o[0] & 0xffff), bf2f(o[0] >> 16), bf2f(o[1] & 0xffff), bf2f(o[1] >> 16)};
                  x[2 * pp + 1] = f32x4_t{bf2f(o[2] & 0xffff), bf2f(o[2] >> 16), bf2f(o[3] & 0xffff), bf2f(o[3] >> 16)};
                }
              });
            }
            static_for<JB / 2>([&](auto pc) {
              constexpr int pp = decltype(pc)::value;
              if (ED && nbase + pp * 32 >= p.N) return;
              f32x4_t va = alpha * acc[i][2 * pp], vb = alpha * acc[i][2 * pp + 1];
              if constexpr (EX) {
                va += x[2 * pp];
                vb += x[2 * pp + 1];
              }
              if constexpr (AC == 1) {
                if (zout)
                  store16_padded(v4u32_t{pack_bf16x2(va[0], va[1]), pack_bf16x2(va[2], va[3]),
                                         pack_bf16x2(vb[0], vb[1]), pack_bf16x2(vb[2], vb[3])},
                                 vrow, rz4, std::integral_constant<int, pp * 64>{});
  #pragma unroll
                for (int t = 0; t < 4; ++t) {
                  va[t] = act_fwd(ACTK, va[t]);
                  vb[t] = act_fwd(ACTK, vb[t]);
                }
              } else if constexpr (AC == 2) {
  #pragma unroll
                for (int t = 0; t < 4; ++t) {
                  va[t] *= act_grad(ACTK, x[2 * pp][t]);
                  vb[t] *= act_grad(ACTK, x[2 * pp + 1][t]);
                }
              }
              if constexpr (OUT_F32) {
                store16_padded<pp * 128, SC>(va, vrow, rc4, std::integral_constant<int, pp * 128>{});
                store16_padded<pp * 128 + 16, SC>(vb, vrow, rc4, std::integral_constant<int, pp * 128 + 16>{});
                if (ZCOPY && zout)   // the bf16 copy: the same element offsets at 2 of C's 4 bytes
                  store16_padded<pp * 64, SC>(v4u32_t{pack_bf16x2(va[0], va[1]), pack_bf16x2(va[2], va[3]),
                                                      pack_bf16x2(vb[0], vb[1]), pack_bf16x2(vb[2], vb[3])},
                                             vrow >> 1, rz4, std::integral_constant<int, pp * 64>{});
              } else {
                // the same unpadded-hazard as the fp32 stores (garbage in ~1% of the bf16 outputs, measured)
                store16_padded<pp * 64, SC>(v4u32_t{pack_bf16x2(va[0], va[1]), pack_bf16x2(va[2], va[3]),
                                                    pack_bf16x2(vb[0], vb[1]), pack_bf16x2(vb[2], vb[3])},
                                           vrow, rc4, std::integral_constant<int, pp * 64>{});
              }
            });
            fence();
          });
          if constexpr (PROF) {
            if (stamp) epi_issue += __builtin_amdgcn_s_memtime() - tmark;   // every store of the direct path issued
          }
          // loads into VGPRs pending at the loop back edge make the compiler's wait model drain vmcnt (the in-flight
          // LDS-DMAs of the next tile included) at the top of every K-tile: retire them on this path. (Stores
          // skipped past N on an edge tile only shorten the queue the K loop's counted waits were derived for.)
          if constexpr (EX || AC == 2 || (RELAX && (ED || AC != 0))) __builtin_amdgcn_s_waitcnt(0x0f70);
        };
        // The RevNet stream update (fp32 C = R + alpha acc, its bf16 copy in Zout) with the residual loads of fragment
        // row i + 1 issued ahead of row i's stores. In the plain EX loop each row's residual loads were issued behind
        // the previous row's 12 stores and consumed at once: vmcnt completes in order, so every row waited for the
        // previous row's stores to be written AND for its own loads -- 8 serialized round trips per tile (the token
        // mixer's stream-update product ran 4.1 ms against 2.1 ms for the same product without the update). Here row
        // i + 1's loads go to acc[i]'s AGPRs (dead once row i's outputs are formed) by inline asm BEFORE row i's
        // stores, and row i + 1 waits with vmcnt(12): row i's stores may stay in flight. Row 0's loads are the
        // compiler's own. Full tiles only (edge tiles skip stores and would break the count).
        auto emit_zpipe = [&]() {
          const i32x4_t rr4 = make_rsrc(reinterpret_cast<const char*>(p.R) + ct.coff * ES + corg, cext);
          static_for<8>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const int vrow = voff + i * 16 * ES * ldcs;
            f32x4_t r[8];
            if constexpr (i == 0) {
              static_for<4>([&](auto pc) {
                constexpr int pp = decltype(pc)::value;
                r[2 * pp] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rr, vrow + pp * 128, 0, 0));
                r[2 * pp + 1] =
                    __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rr, vrow + pp * 128 + 16, 0, 0));
              });
            } else {
              zpipe_wait<i>();   // row i's residual landed; the ops issued after it may stay in flight
              constexpr int b = (i + 1) % 2;   // rows 1, 3, 5, 7 in acc[0], rows 2, 4, 6 in acc[1]
              static_for<8>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                agpr_opaque(acc[b][j]);   // the loaded values from here on
                r[j] = acc[b][j];
              });
            }
            static_for<8>([&](auto jc) {   // in place: no second set of 32 VGPRs (the queue's LDS slot spilled)
              constexpr int j = decltype(jc)::value;
              r[j] = alpha * acc[i][j] + r[j];
            });
            // two rows ahead: row 0 issues row 1 (acc[0]); row 1 rows 2 (acc[1]) and 3 (acc[0]); row i >= 2 row i + 2
            // into the buffer row i was read from
            auto issue = [&](auto kc, auto bc) {
              constexpr int k = decltype(kc)::value, bb = decltype(bc)::value;
              const int vk = voff + k * 16 * ES * ldcs;
              static_for<4>([&](auto pc) {
                constexpr int pp = decltype(pc)::value;
                load16_agpr<pp * 128>(acc[bb][2 * pp], vk, rr4);
                load16_agpr<pp * 128 + 16>(acc[bb][2 * pp + 1], vk, rr4);
              });
            };
            if constexpr (i == 0) {
              asm volatile("s_nop 4" ::: "memory");   // resource SGPRs possibly just written by VALU
              issue(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
            } else if constexpr (i == 1) {
              asm volatile("s_nop 4" ::: "memory");
              issue(std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{});
              issue(std::integral_constant<int, 3>{}, std::integral_constant<int, 0>{});
            } else if constexpr (i + 2 < 8) {
              asm volatile("s_nop 4" ::: "memory");
              issue(std::integral_constant<int, i + 2>{}, std::integral_constant<int, (i + 1) % 2>{});
            }
            static_for<4>([&](auto pc) {   // 12 stores per row (the count the next row's wait assumes)
              constexpr int pp = decltype(pc)::value;
              const f32x4_t va = r[2 * pp], vb = r[2 * pp + 1];
              store16_padded<pp * 128, SC>(va, vrow, rc4, std::integral_constant<int, pp * 128>{});
              store16_padded<pp * 128 + 16, SC>(vb, vrow, rc4, std::integral_constant<int, pp * 128 + 16>{});
              store16_padded<pp * 64, SC>(v4u32_t{pack_bf16x2(va[0], va[1]), pack_bf16x2(va[2], va[3]),
                                                  pack_bf16x2(vb[0], vb[1]), pack_bf16x2(vb[2], vb[3])},
                                          vrow >> 1, rz4, std::integral_constant<int, pp * 64>{});
            });
            fence();
          });
          if constexpr (PROF) {
            if (stamp) epi_issue += __builtin_amdgcn_s_memtime() - tmark;
          }
          // (no vmcnt drain: every asm load was waited for; the stores drain under the next tile's first K-tile)
        };
        // The same pipelining on the row-layout (TLAY) bf16 epilogues with one 16-byte side input per row: the
        // block output projections' residual (AC_ 0, R) and the activation backward of the FFN-in dgrad (AC_ 2 / 4,
        // gelu' / relu' of Zin). Measured on GPT-Neo-1.3B's shapes the side input cost +23 % (131072 x 2048 x 2048
        // + R) and +34 % (131072 x 8192 x 2048 with gelu', 3.22 -> 4.32 ms; tools/lab/epi_side_ab.py) -- 8 rows x
        // (the previous row's 4 stores + this row's loads) of exposed latency per tile. Row i + 1's side rows go to
        // acc[i][0..3] (consumed) ahead of row i's 4 stores; row i + 1 waits with vmcnt(4). Full tiles only.
        auto emit_tpipe = [&](auto acc_) {
          constexpr int AC_ = decltype(acc_)::value;
          constexpr bool ACT = AC_ != 0;
          constexpr int ACTK = AC_ >= 3 ? ACT_RELU : ACT_GELU;
          const char* sbase = ACT ? reinterpret_cast<const char*>(p.Zin) + ct.coff * 2 + corg
                                  : reinterpret_cast<const char*>(p.R) + ct.coff * ES + corg;
          const i32x4_t rs4 = make_rsrc(sbase, cext);
          const __amdgpu_buffer_rsrc_t rsb = ACT ? rzi : rr;
          const int vt = ((wm * 128 + 4 * gq) * ldcs + wn * WN + 8 * ml) * ES;
          static_for<8>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            int vro[4];
            v4u32_t side[4];
            static_for<4>([&](auto rk) {
              constexpr int r = decltype(rk)::value;
              vro[r] = vt + (16 * i + r) * ES * ldcs;
            });
            if constexpr (i == 0) {
              static_for<4>([&](auto rk) {
                constexpr int r = decltype(rk)::value;
                side[r] = __builtin_amdgcn_raw_buffer_load_b128(rsb, vro[r], 0, 0);
              });
            } else {
              // row i's side rows landed: the VMEM ops issued after them (TPIPE_W) may stay in flight
              tpipe_wait<i>();
              constexpr int lr = (i - 1) / 2, lj = (i & 1) ? 0 : 4;   // where row i's side rows were loaded
              static_for<4>([&](auto rk) {
                constexpr int r = decltype(rk)::value;
                agpr_opaque(acc[lr][lj + r]);
                side[r] = __builtin_bit_cast(v4u32_t, acc[lr][lj + r]);
              });
            }
            v4u32_t o0[4];
            static_for<4>([&](auto rk) {
              constexpr int r = decltype(rk)::value;
              float x[8];
              static_for<8>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                x[j] = alpha * acc[i][j][r];
              });
              static_for<4>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                const float lo = bf2f(side[r][t] & 0xffff), hi = bf2f(side[r][t] >> 16);
                if constexpr (ACT) {
                  x[2 * t] *= act_grad(ACTK, lo);
                  x[2 * t + 1] *= act_grad(ACTK, hi);
                } else {
                  x[2 * t] += lo;
                  x[2 * t + 1] += hi;
                }
              });
              o0[r] = v4u32_t{pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]), pack_bf16x2(x[4], x[5]),
                              pack_bf16x2(x[6], x[7])};
            });
            if constexpr (i < 4) {   // rows 2i + 1 (and 2i + 2) into acc[i][0..3] (and [4..7]): consumed
              constexpr int k0 = 2 * i + 1, nk = i < 3 ? 2 : 1;
              asm volatile("s_nop 4" ::: "memory");
              static_for<nk>([&](auto hc) {
                constexpr int h = decltype(hc)::value;
                static_for<4>([&](auto rk) {
                  constexpr int r = decltype(rk)::value;
                  load16_agpr<0>(acc[i][4 * h + r], vt + (16 * (k0 + h) + r) * ES * ldcs, rs4);
                });
              });
            }
            static_for<4>([&](auto rk) {   // 4 stores per row (the count the next row's wait assumes)
              constexpr int r = decltype(rk)::value;
              store16_nc<SC>(o0[r], vro[r], rc4);
            });
            fence();
          });
          if constexpr (PROF) {
            if (stamp) epi_issue += __builtin_amdgcn_s_memtime() - tmark;
          }
        };
        using A0 = std::integral_constant<int, 0>;
        const bool tfull = TLAY && G4W_ZPIPE != 0 && ct.n0 + 256 <= p.N;
        if constexpr (!OUT_F32) {
          if (gelu_direct && p.act == ACT_GELU) {
            using A1 = std::integral_constant<int, 1>;
            using A2 = std::integral_constant<int, 2>;
            if (p.mode == 1) {
              if constexpr (TLAY) {
                if ((G4W_TPM & 2) && tfull) emit_tpipe(A2{}); else emit(F_{}, F_{}, A2{});
              } else {
                if (edge) emit(F_{}, T_{}, A2{}); else emit(F_{}, F_{}, A2{});
              }
            } else {
              if (edge) emit(F_{}, T_{}, A1{}); else emit(F_{}, F_{}, A1{});
            }
          } else if (gelu_direct) {   // relu (TLAY only)
            if constexpr (TLAY) {
              using A3 = std::integral_constant<int, 3>;
              using A4 = std::integral_constant<int, 4>;
              if (p.mode == 1) {
                if ((G4W_TPM & 4) && tfull) emit_tpipe(A4{}); else emit(F_{}, F_{}, A4{});
              } else {
                emit(F_{}, F_{}, A3{});
              }
            }
          } else if (extra) {
            if constexpr (TLAY) {
              if ((G4W_TPM & 1) && tfull) emit_tpipe(A0{}); else emit(T_{}, F_{}, A0{});
            } else {
              if (edge) emit(T_{}, T_{}, A0{}); else emit(T_{}, F_{}, A0{});
            }
          } else {
            if (edge) emit(F_{}, T_{}, A0{}); else emit(F_{}, F_{}, A0{});
          }
        } else {
          if (extra) {
            if constexpr (ZCOPY && !TLAY && G4W_ZPIPE != 0) {
              if (!edge && beta == 0.f && zout && p.R != nullptr) emit_zpipe();
              else if (edge) emit(T_{}, T_{}, A0{});
              else emit(T_{}, F_{}, A0{});
            } else {
              if (edge) emit(T_{}, T_{}, A0{}); else emit(T_{}, F_{}, A0{});
            }
          } else {
            if (edge) emit(F_{}, T_{}, A0{}); else emit(F_{}, F_{}, A0{});
          }
        }
      } else {
        // Epilogue through a wave-private 8 KiB LDS region past the two stages (the stages already hold the next
        // tile's first two K-tiles): 8 rounds of 16 rows x 128 columns fp32, float4 columns XOR-swizzled by row
        // (conflict-free fragment writes). A round writes one fragment row of accumulators, then a compact runtime
        // loop reads 8 consecutive outputs per lane and applies epilogue_store8r (one activation switch per round)
        // with 16-byte global accesses; a fully unrolled per-fragment epilogue inlined the activation switch 64
        // times (~12k branches), instruction-cache bound and as long as the K loop at K = 2048.
        float* ep = reinterpret_cast<float*>(smem + 2 * Q_STAGE) + wave * 16 * WN;
        const float alpha = p.alpha;
        constexpr int LPR = WN / 8;   // lanes per 16-row x WN round row (8 outputs each)
        static_for<8>([&](auto rcc) {
          constexpr int r = decltype(rcc)::value;
          if constexpr (TLAY) {   // rows 4 gq + t, columns 8 ml .. +7 (acc[r][0..7][t])
            static_for<4>([&](auto tc) {
              constexpr int t = decltype(tc)::value;
              const int row = 4 * (lane >> 4) + t, c4 = 2 * (lane & 15);
              *reinterpret_cast<float4*>(ep + row * WN + ((c4 ^ (row & 7)) << 2)) =
                  make_float4(alpha * acc[r][0][t], alpha * acc[r][1][t], alpha * acc[r][2][t], alpha * acc[r][3][t]);
              *reinterpret_cast<float4*>(ep + row * WN + (((c4 + 1) ^ (row & 7)) << 2)) =
                  make_float4(alpha * acc[r][4][t], alpha * acc[r][5][t], alpha * acc[r][6][t], alpha * acc[r][7][t]);
            });
          } else {
            static_for<JB>([&](auto jc) {
              constexpr int j = decltype(jc)::value;
              const int row = lane & 15, c4 = 8 * (j >> 1) + 2 * (lane >> 4) + (j & 1);   // frag_b column order
              *reinterpret_cast<float4*>(ep + row * WN + ((c4 ^ (row & 7)) << 2)) =
                  make_float4(alpha * acc[r][j][0], alpha * acc[r][j][1], alpha * acc[r][j][2], alpha * acc[r][j][3]);
            });
          }
  #pragma unroll 1
          for (int it = 0; it < 16 * LPR / 64; ++it) {
            const int row = it * (64 / LPR) + lane / LPR, c4 = (lane % LPR) * 2;
            const float4 x0 = *reinterpret_cast<const float4*>(ep + row * WN + ((c4 ^ (row & 7)) << 2));
            const float4 x1 = *reinterpret_cast<const float4*>(ep + row * WN + (((c4 + 1) ^ (row & 7)) << 2));
            float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            const int m = ct.m0 + wm * 128 + r * 16 + row, n = ct.n0 + wn * WN + c4 * 4;
            if (m < p.M && n < p.N) epilogue_store8r<OUT_F32>(p, ct.coff + (long long)m * p.ldc + n, v);
          }
          fence();
        });
        __builtin_amdgcn_s_waitcnt(0x0f70);   // residual / spill reloads retired here (see emit)
      }
      fence();
      if (stamp) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        epi_clk += now - tmark;
      }
      if constexpr (QUEUE) q_cur = q_next;
    }
  };
  if constexpr (STG) {
    if (simd_odd) body(std::integral_constant<int, 1>{});
    else body(std::integral_constant<int, 0>{});
  } else {
    body(std::integral_constant<int, 0>{});
  }
  vm_wait<0>();   // the last re-staged positions must land before the LDS is released
  if (p.stamps != nullptr) {
    __syncthreads();
    if (stamp) {
      p.stamps[sbase + 2] = loop_clk;
      p.stamps[sbase + 3] = epi_clk;
      if (PROF) {   // the start / first-landed / XCC slots give way to the sync points' and store-issue clocks
        p.stamps[sbase + 0] = sync1;
        p.stamps[sbase + 1] = sync2;
        p.stamps[sbase + 4] = epi_issue;
      }
      p.stamps[sbase + 6] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

template <int A_T, int B_T, bool F32, int NWV = 4>
hipError_t launch4w(GemmArgs a, int batch, hipStream_t stream) {
  a.tiles_m = (a.M + 255) / 256;
  a.tiles_n = (a.N + 255) / 256;
  a.nbatch = batch * a.ksplit;
  const long long tiles = tiles_total(a);
  // one block per CU (32 per XCD); fewer for small launches, keeping a multiple of the 8 XCDs
  const int grid = (int)(tiles >= 256 ? 256 : ((tiles + 7) / 8) * 8);
  const size_t lds = 2 * Q_STAGE + 32768;   // 160 KiB: two stages + the epilogue regions (16 rows x 128 fp32 per SIMD)
  auto k = a.stamps ? gemm4w_kernel<A_T, B_T, F32, true, NWV> : gemm4w_kernel<A_T, B_T, F32, false, NWV>;
  int which = a.stamps != nullptr;
  if constexpr (A_T == 0 && B_T == 0) {
    if (a.kin) {   // the split contraction index (token-mixer weight gradient) has its own instantiation
      k = gemm4w_kernel<A_T, B_T, F32, false, NWV, G4W_SCH, (G4W_STG != 0), G4W_CPA, G4W_CPB, G4W_OPT, true>;
      which = 2;
    }
  }
  if constexpr (F32 && A_T == 0) {
    if (a.Zout) {   // fp32 output + bf16 copy (RevNet stream update: A is the activation or the mixer weight)
      k = gemm4w_kernel<A_T, B_T, F32, false, NWV, G4W_SCH, (G4W_STG != 0), G4W_CPA, G4W_CPB, G4W_ZCP_OPT, false,
                        true>;
      which = 3;
    }
  }
  if constexpr (!(F32 && A_T == 0)) {
    if (a.queue) {   // the dynamic tile queue (dense products, every tile >= 3 K-tiles: obst_gemm)
      k = gemm4w_kernel<A_T, B_T, F32, false, NWV, G4W_SCH, (G4W_STG != 0), G4W_CPA, G4W_CPB, G4W_OPT, false, false,
                        true>;
      which = 4;
    }
  } else {
    if (a.queue && !a.Zout) {
      k = gemm4w_kernel<A_T, B_T, F32, false, NWV, G4W_SCH, (G4W_STG != 0), G4W_CPA, G4W_CPB, G4W_OPT, false, false,
                        true>;
      which = 4;
    } else if (a.queue) {   // queued fp32 + bf16-copy products
      k = gemm4w_kernel<A_T, B_T, F32, false, NWV, G4W_SCH, (G4W_STG != 0), G4W_CPA, G4W_CPB, G4W_ZCP_OPT, false,
                        true, true>;
      which = 5;
    }
  }
  static bool attr[6] = {false, false, false, false, false, false};
  if (!attr[which]) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr[which] = true;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NWV), lds, stream, a);
  return hipGetLastError();
}

}  // namespace

// one operand-layout pair per translation unit (gemm4w_<a_t><b_t>.hip) so the instantiations compile in parallel
// (NWV = 8 builds and runs correctly but at 597 TF/s on 131072x4096x2048: with 128 AGPRs per wave the 96 fragment
// VGPRs leave too few registers and the K loop spills -- profiles/r3_gemm4w_bounds.md; only NWV = 4 is instantiated)
#define OBST_GEMM4W_TU(AT, BT)                                                                                      \
  hipError_t gemm4w_launch_##AT##BT(const gemmk::GemmArgs* a, int out_f32, int batch, hipStream_t stream) {      \
    return out_f32 ? launch4w<AT, BT, true>(*a, batch, stream) : launch4w<AT, BT, false>(*a, batch, stream);    \
  }
