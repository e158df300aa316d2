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
//    16 B per lane, 1 KiB per wave-instruction, source address = SGPR resource + one constant per-lane offset),
//    interleaved one piece per ~5 MFMAs. Two LDS stages of 64 KiB; two barriers per K-tile:
//      barrier 1 (after the substep-1 reads, lgkmcnt(0)): every wave is done reading stage s -> DMA into it;
//      barrier 2 (after a counted vmcnt(16): this tile's 16 DMAs stay in flight): tile t+1 has landed in stage
//      s^1 -> the substep-0 fragments of tile t+1 are read under the last 20 MFMAs of tile t.
//    The instruction order is pinned with sched_barrier(0) fences; the compiler only allocates registers and
//    counts lgkmcnt for the fragment reads. Out-of-range prefetches (t+2 >= nk) re-read the last tile into the
//    stage nobody reads any more, so the loop has no branches.
//  * K-contiguous operands ([rows][K]) are staged as [256 rows][64 k] images (128-B rows, chunk ^= (row>>1)&7:
//    conflict-free ds_read_b128 fragment reads); row-contiguous operands ([K][rows]) as two [64 k][128 rows]
//    halves (256-B rows, chunk ^= kswz(k)) read with the CDNA4 transposing ds_read_b64_tr_b16. The swizzle lives
//    in the per-lane SOURCE address (LDS-DMA writes lane-linearly).
//  * The MFMA is issued as mfma(B, A) so each lane ends with 4 consecutive output columns of one row; the
//    epilogue (alpha, beta, residual, activation with pre-activation output, activation backward, fp32 split-K
//    slabs) is the shared epilogue_store of gemm_kern.h.
#pragma once
#include "common.h"
#include "gemm_kern.h"
#include <utility>

namespace {

typedef __attribute__((ext_vector_type(4))) int i32x4_t;

constexpr int Q_OP = 256 * 64 * 2;   // one operand image of a K-tile: 32 KiB
constexpr int Q_STAGE = 2 * Q_OP;    // A + B: 64 KiB; two stages

__device__ __forceinline__ unsigned lds_u32(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// raw buffer resource over [base, base + 4 GiB): stride 0, no range check beyond num_records = 0xffffffff
__device__ __forceinline__ i32x4_t make_rsrc(const void* base) {
  const unsigned long long a = (unsigned long long)base;
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32));
  r[2] = -1;
  r[3] = 0x00020000;
  return r;
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// LDS-DMA of 16 B per lane into the 1 KiB at LDS address m0 (lane-linear). In inline asm so the compiler neither
// drains it with a vmcnt(0) before later LDS reads nor reorders it: every consumer waits with an explicit counted
// vmcnt before the barrier that publishes the stage.
__device__ __forceinline__ void dma16(const i32x4_t& rs, int voff, unsigned m0) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
               "s"(__builtin_amdgcn_readfirstlane(m0))
               : "memory", "m0");
}
// C += A.B on one 16x16x32 bf16 tile, accumulator pinned to AGPRs: as a builtin, the register allocator re-assigned
// the 64 loop-carried accumulators every iteration and copied them back through VGPRs at the back edge (512
// registers, spills); a tied "+a" operand keeps each one in place. Hazards the compiler cannot see inside the asm
// are padded by hand where the accumulators are initialised and read back (s_nop before / after the K loop).
__device__ __forceinline__ void mfma_acc(f32x4_t& c, const bf16x8_t& a, const bf16x8_t& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
#pragma clang diagnostic pop

__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }
// makes c an asm-produced AGPR value (no later rematerialisation of what it was computed from)
__device__ __forceinline__ void agpr_opaque(f32x4_t& c) { asm volatile("" : "+a"(c)); }

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

// per-lane source offsets (bytes, relative to the tile's K-tile base) of the 8 LDS-DMA pieces this wave stages
// for one operand. T = 0: [rows][K] operand, piece P = 8 rows; T = 1: [K][rows] operand, piece P = 4 k-rows x 128
// columns of half P >> 4. Rows / columns past the operand's edge are clamped (their results are never stored).
template <int T>
__device__ __forceinline__ void piece_offsets(int (&vo)[8], long long ld, int r0, int R, int wave, int lane) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int P = wave * 8 + q;
    if (T == 0) {
      const int row = P * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      const int rc = min(r0 + row, R - 1) - r0;
      vo[q] = (int)(rc * ld * 2) + c * 16;
    } else {
      const int h = P >> 4, kr = (P & 15) * 4 + (lane >> 4);
      const int c = (lane & 15) ^ kswz(kr);
      const int col = min(r0 + h * 128 + c * 8, R - 8) - r0;
      vo[q] = (int)(kr * ld * 2) + col * 2;
    }
  }
}

// fragment j (16 rows/cols starting at rbase within the 256 of the tile) of k-substep kk from an operand image
template <int T>
__device__ __forceinline__ bf16x8_t frag(const char* img, int rbase, int kk, int lane) {
  if (T == 0) return read_frag<0>(img, rbase, kk, lane);
  return read_frag<1>(img + (rbase >> 7) * (Q_OP / 2), rbase & 127, kk, lane);
}

template <int A_T, int B_T, bool OUT_F32>
__global__ __launch_bounds__(256, 1) void gemm4w_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware remap over the whole grid (tiles x batches x K-splits), then GROUP = 4 tile rows per N sweep
  int bid, ybat;
  {
    const int nx = gridDim.x;
    const long long nwg = (long long)nx * gridDim.y, lin = (long long)blockIdx.y * nx + blockIdx.x;
    const long long xcd = lin & 7, qq = nwg >> 3, r = nwg & 7;
    const long long lg = (xcd < r ? xcd * (qq + 1) : r * (qq + 1) + (xcd - r) * qq) + (lin >> 3);
    bid = (int)(lg % nx);
    ybat = (int)(lg / nx);
  }
  const int GROUP = 4;
  const int per_group = GROUP * p.tiles_n;
  const int first_m = (bid / per_group) * GROUP;
  const int gsz = min(p.tiles_m - first_m, GROUP);
  const int tm = first_m + (bid % per_group) % gsz;
  const int tn = (bid % per_group) / gsz;
  const int m0 = tm * 256, n0 = tn * 256;
  const int split = ybat % p.ksplit, bidx = ybat / p.ksplit;
  const int b1 = bidx / p.nb2, b2 = bidx % p.nb2;
  const int kspan = p.K / p.ksplit, kbeg = split * kspan;
  const int nk = kspan / 64;

  // K-tile bases: element pointer of (tile row/col 0, k = kbeg) and the per-K-tile step in bytes
  const char* abase = reinterpret_cast<const char*>(
      p.A + b1 * p.a_s1 + b2 * p.a_s2 + (A_T == 0 ? (long long)m0 * p.lda + kbeg : (long long)kbeg * p.lda + m0));
  const char* bbase = reinterpret_cast<const char*>(
      p.B + b1 * p.b_s1 + b2 * p.b_s2 + (B_T == 0 ? (long long)n0 * p.ldb + kbeg : (long long)kbeg * p.ldb + n0));
  const long long astep = A_T == 0 ? 128 : 128 * p.lda;
  const long long bstep = B_T == 0 ? 128 : 128 * p.ldb;

  int voa[8], vob[8];
  piece_offsets<A_T>(voa, p.lda, m0, p.M, wave, lane);
  piece_offsets<B_T>(vob, p.ldb, n0, p.N, wave, lane);
  const unsigned lds0 = lds_u32(smem);
  // this wave's 8 pieces of an operand image are contiguous: 8 KiB at (wave * 8 KiB)
  auto stage_a = [&](int s) -> unsigned { return lds0 + s * Q_STAGE + wave * 8192; };
  auto stage_b = [&](int s) -> unsigned { return lds0 + s * Q_STAGE + Q_OP + wave * 8192; };

  auto dma_a = [&](int t, int s, int q) {
    const int tc = min(t, nk - 1);
    dma16(make_rsrc(abase + tc * astep), voa[q], stage_a(s) + q * 1024);
  };
  auto dma_b = [&](int t, int s, int q) {
    const int tc = min(t, nk - 1);
    dma16(make_rsrc(bbase + tc * bstep), vob[q], stage_b(s) + q * 1024);
  };

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t a0[8], b0[8], a1[8], b1f[8];

  // read order of a substep's 16 fragments: A0, B0, A1..A7, B1..B7 (the order the MFMA stream consumes them)
  auto read_sub = [&](int s, auto kkc, auto rc, bf16x8_t (&af)[8], bf16x8_t (&bf)[8]) {
    constexpr int kk = decltype(kkc)::value, r = decltype(rc)::value;
    const char* ia = smem + s * Q_STAGE;
    const char* ib = smem + s * Q_STAGE + Q_OP;
    if constexpr (r == 0) af[0] = frag<A_T>(ia, wm * 128, kk, lane);
    else if constexpr (r == 1) bf[0] = frag<B_T>(ib, wn * 128, kk, lane);
    else if constexpr (r < 9) af[r - 1] = frag<A_T>(ia, wm * 128 + (r - 1) * 16, kk, lane);
    else bf[r - 8] = frag<B_T>(ib, wn * 128 + (r - 8) * 16, kk, lane);
  };
  // Accumulator zeroing (VALU writes of AGPRs) -> first MFMA reading them needs wait states the compiler cannot
  // see through the asm MFMAs. The zero constants would otherwise be rematerialised right in front of the loop,
  // past any pad: an empty "+a" asm per accumulator makes each a materialised value before the pad.
  static_for<64>([&](auto c) { agpr_opaque(acc[decltype(c)::value >> 3][decltype(c)::value & 7]); });
  asm volatile("s_nop 4" ::: "memory");
  fence();
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;

  // diagnostic timestamps (GemmArgs::stamps, null in production): per block [start, first tile landed, loop done,
  // epilogue done] in shader clocks, the XCC id, [start, end] in 100 MHz real time
  const bool stamp = p.stamps != nullptr && tid == 0;
  const long long sbase = ((long long)blockIdx.y * gridDim.x + blockIdx.x) * 8;
  if (stamp) {
    p.stamps[sbase] = __builtin_amdgcn_s_memtime();
    p.stamps[sbase + 4] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));   // HW_REG_XCC_ID[3:0]
    p.stamps[sbase + 5] = __builtin_amdgcn_s_memrealtime();
  }
  // prologue: tiles 0 and 1 into stages 0 and 1, wait for tile 0, read its substep-0 fragments
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_a(0, 0, q);
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_b(0, 0, q);
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_a(1, 1, q);
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_b(1, 1, q);
  vm_wait<16>();
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_s_waitcnt(0xc07f);   // nothing (kernel-argument loads) pending in lgkmcnt at the loop entry
  if (stamp) p.stamps[sbase + 1] = __builtin_amdgcn_s_memtime();
  fence();
  static_for<16>([&](auto rc) { read_sub(0, K0{}, rc, a0, b0); fence(); });   // same order as in the loop
  fence();

  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    static_for<128>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      constexpr int sub = q >> 6, j = (q >> 3) & 7, i = q & 7;
      if constexpr (sub == 0) mfma_acc(acc[i][j], b0[j], a0[i]);
      else mfma_acc(acc[i][j], b1f[j], a1[i]);
      if constexpr (q < 16) read_sub(s, K1{}, qc, a1, b1f);               // substep-1 fragments of tile t
      if constexpr (q == 25) {                                          // stage s fully read by every wave
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0) as a builtin: the compiler's wait model learns the
        __builtin_amdgcn_s_barrier();          // substep-1 reads are done (asm would leave it waiting for them again)
      }
      if constexpr (q >= 26 && q < 64 && (q - 26) % 5 == 0) dma_a(t + 2, s, (q - 26) / 5);
      if constexpr (q >= 66 && q < 106 && (q - 66) % 5 == 0) dma_b(t + 2, s, (q - 66) / 5);
      if constexpr (q == 107) {                                         // tile t+1 landed in stage s^1
        vm_wait<16>();
        __builtin_amdgcn_s_barrier();
      }
      if constexpr (q >= 108 && q < 124) read_sub(s ^ 1, K0{}, std::integral_constant<int, q - 108>{}, a0, b0);   // substep-0 fragments of tile t+1
      fence();
    });
  }
  fence();
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");   // last MFMA -> accumulator reads: the
  fence();                                                          // fences keep the reads below the pad
  vm_wait<0>();   // the over-range prefetches of the last two iterations must land before the LDS is reused
  if (stamp) p.stamps[sbase + 2] = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_s_barrier();   // ... by every wave: the epilogue below overwrites both stages
  fence();

  // Epilogue through LDS: per wave 4 rounds of 32 rows x 128 columns (fp32, rows padded to 132 floats:
  // conflict-free 16-byte fragment writes). Each round the wave writes two accumulator rows of fragments, then a
  // compact runtime loop reads 8 consecutive outputs per lane and applies epilogue_store8 with 16-byte global
  // accesses (a fully unrolled per-fragment epilogue inlined the activation switch 64 times: ~12k branches,
  // instruction-cache bound, as long as the K loop itself at K = 2048).
  constexpr int EP_LD = 132;
  float* ep = reinterpret_cast<float*>(smem) + wave * (32 * EP_LD);
  const long long coff = b1 * p.c_s1 + b2 * p.c_s2;
  const float alpha = p.alpha;
  static_for<4>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    static_for<16>([&](auto fc) {
      constexpr int f = decltype(fc)::value, i = 2 * r + (f >> 3), j = f & 7;
      const int row = (f >> 3) * 16 + (lane & 15), col = j * 16 + 4 * (lane >> 4);
      *reinterpret_cast<float4*>(ep + row * EP_LD + col) =
          make_float4(alpha * acc[i][j][0], alpha * acc[i][j][1], alpha * acc[i][j][2], alpha * acc[i][j][3]);
    });
#pragma unroll 1
    for (int it = 0; it < 8; ++it) {
      const int row = it * 4 + (lane >> 4), col = (lane & 15) * 8;
      const float4 x0 = *reinterpret_cast<const float4*>(ep + row * EP_LD + col);
      const float4 x1 = *reinterpret_cast<const float4*>(ep + row * EP_LD + col + 4);
      float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      const int m = m0 + wm * 128 + r * 32 + row, n = n0 + wn * 128 + col;
      if (m < p.M && n < p.N) {
        if (OUT_F32 && p.ksplit > 1) {
          float4* w = reinterpret_cast<float4*>(p.ws + (long long)split * p.M * p.N + (long long)m * p.N + n);
          w[0] = x0;
          w[1] = x1;
        } else {
          epilogue_store8<OUT_F32>(p, coff + (long long)m * p.ldc + n, v);
        }
      }
    }
  });
  if (p.stamps != nullptr) {
    __syncthreads();
    if (stamp) {
      p.stamps[sbase + 3] = __builtin_amdgcn_s_memtime();
      p.stamps[sbase + 6] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

template <int A_T, int B_T, bool F32>
hipError_t launch4w(GemmArgs a, int batch, hipStream_t stream) {
  a.tiles_m = (a.M + 255) / 256;
  a.tiles_n = (a.N + 255) / 256;
  dim3 grid(a.tiles_m * a.tiles_n, batch * a.ksplit);
  const size_t lds = 2 * Q_STAGE;
  auto k = gemm4w_kernel<A_T, B_T, F32>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(k, grid, dim3(256), lds, stream, a);
  return hipGetLastError();
}

}  // namespace

// one operand-layout pair per translation unit (gemm4w_<a_t><b_t>.hip) so the instantiations compile in parallel
#define OBST_GEMM4W_TU(AT, BT)                                                                                      \
  hipError_t gemm4w_launch_##AT##BT(const gemmk::GemmArgs* a, int out_f32, int batch, hipStream_t stream) {      \
    return out_f32 ? launch4w<AT, BT, true>(*a, batch, stream) : launch4w<AT, BT, false>(*a, batch, stream);    \
  }
