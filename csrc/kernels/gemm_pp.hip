// Persistent variant of the phase GEMM (see gemm.hip for the phase pipeline itself).
#include "common.h"
#include "gemm_kern.h"

namespace {

// ---------------------------------------------------------------------------------------------------------------
// Persistent phase kernel: the same 256x256 8-wave phase pipeline, but one block per CU walks a run of tiles, and a
// tile's epilogue stores overlap the NEXT tile's prologue loads (issued first) instead of leaving the CU idle
// through the HBM latency of every new tile -- on the token mixer's short triangular tiles (4-32 K-tiles of 64) a
// dense-to-triangular time ratio of 0.76 for 0.56 of the work put that fixed cost at several K-tiles per tile.
// Plain epilogue (alpha, tri 3 mask) on whole tiles only (M % 256 == N % 256 == 0), so every thread issues exactly 32
// stores per tile and the counted vmcnt waits of the next tile's first K-tile can step over them (vmcnt counts
// loads and stores in issue order on gfx9). XCD k owns a contiguous run of tiles (logical tile order as in
// gemm_ph_kernel: batches x M-groups, lower-triangular tiles longest first), dealt to its 32 CUs in rounds.
template <int A_T, int B_T, bool OUT_F32>
__global__ __launch_bounds__(NT2, 1) void gemm_pp_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int ntile = p.tiles_m * p.tiles_n;
  const long long total = (long long)ntile * p.nbatch;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;
  const long long Q = total >> 3, Rm = total & 7;
  const long long base = xcd < Rm ? xcd * (Q + 1) : Rm * (Q + 1) + (xcd - Rm) * Q;
  const long long len = Q + (xcd < Rm ? 1 : 0);

  struct Tile {
    const bf16_t* A;
    const bf16_t* B;
    long long coff;
    int m0, n0, nk;
  };
  auto decode = [&](long long L) {
    Tile T;
    const int bid = (int)(L % ntile), ybat = (int)(L / ntile);
    const int GROUP = 4;
    const int per_group = GROUP * p.tiles_n;
    const int first_m = (bid / per_group) * GROUP;
    const int gsz = min(p.tiles_m - first_m, GROUP);
    int tm = first_m + (bid % per_group) % gsz;
    const int tn = (bid % per_group) / gsz;
    if (p.tri == 1) tm = p.tiles_m - 1 - tm;
    T.m0 = tm * BM2;
    T.n0 = tn * BN2;
    const int b1 = ybat / p.nb2, b2 = ybat % p.nb2;
    int kspan = p.K, kbeg = 0;
    if (p.tri == 1) kspan = min(p.K, (T.m0 + BM2 + BK - 1) / BK * BK);
    if (p.tri == 2) { kbeg = min(T.m0 / BK * BK, p.K - BK); kspan = p.K - kbeg; }
    T.A = p.A + b1 * p.a_s1 + b2 * p.a_s2 + (A_T == 0 ? (long long)kbeg : (long long)kbeg * p.lda);
    T.B = p.B + b1 * p.b_s1 + b2 * p.b_s2 + (B_T == 0 ? (long long)kbeg : (long long)kbeg * p.ldb);
    T.nk = kspan / BK;
    T.coff = b1 * p.c_s1 + b2 * p.c_s2;
    return T;
  };
  auto slot_p = [&](int t, int pc) -> char* { return smem + ((t & 1) * 4 + pc) * PIECE; };
  auto stageA = [&](const Tile& T, int t, int q) {
    stage_piece<A_T, true>(slot_p(t, q), T.A, p.lda, T.m0, p.M, (long long)t * BK, q, wave, lane);
  };
  auto stageB = [&](const Tile& T, int t, int q) {
    stage_piece<B_T, false>(slot_p(t, 2 + q), T.B, p.ldb, T.n0, p.N, (long long)t * BK, q, wave, lane);
  };
  auto prologue = [&](const Tile& T) {   // the pieces phases -6..-1 would have staged
    stageA(T, 0, 0); stageB(T, 0, 0); stageB(T, 0, 1); stageA(T, 0, 1);
    if (T.nk > 1) { stageA(T, 1, 0); stageB(T, 1, 0); }
  };

  // round r of this XCD's run covers logical tiles base + r*nslot + [0, nslot); block `slot` takes the one at
  // offset (slot + r) % nslot, so with few tiles per batch (the token mixer's 8 M-tiles) a CU does not get the same
  // tile row -- the same K span under triangular operands -- in every round
  int rnd = 0;
  long long k = slot;
  if (k >= len) return;
  Tile cur = decode(base + k);
  prologue(cur);
  bool pend = false;   // the previous tile's 32 epilogue stores are still counted in vmcnt
  f32x4_t acc[8][4];
  bf16x8_t af[4][2], bq0[2][2], bq1[2][2];
  while (true) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int nk = cur.nk;
    if (nk <= 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (pend) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    if (wr == 1) bar();
    bar();
    for (int t = 0; t < nk; ++t) {
      const bool tail = t + 2 >= nk;
      const bool first = t == 0 && pend;
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        const int qm = (ph == 0 || ph == 1) ? 0 : 1;
        const int qn = (ph == 0 || ph == 3) ? 0 : 1;
        if (ph == 0) {
          const char* ib = slot_p(t, 2);
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) bq0[j][kk] = read_frag<B_T>(ib, wc * 32 + j * 16, kk, lane);
        }
        if (ph == 0 || ph == 2) {
          const char* ia = slot_p(t, qm);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) af[i][kk] = read_frag<A_T>(ia, wr * 64 + i * 16, kk, lane);
        }
        if (ph == 1) {
          const char* ib = slot_p(t, 3);
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) bq1[j][kk] = read_frag<B_T>(ib, wc * 32 + j * 16, kk, lane);
        }
        if (ph == 0 && t + 1 < nk) stageB(cur, t + 1, 1);
        if (ph == 1 && t + 1 < nk) stageA(cur, t + 1, 1);
        if (ph == 2 && t + 2 < nk) stageA(cur, t + 2, 0);
        if (ph == 3 && t + 2 < nk) stageB(cur, t + 2, 0);
        // t = 0 reads only prologue pieces, which are older than the previous tile's stores: step over them
        if (tail) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (first) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        bar();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
              const bf16x8_t bb = qn == 0 ? bq0[j][kk] : bq1[j][kk];
              acc[qm * 4 + i][qn * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb, af[i][kk],
                                                                                    acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
            }
        __builtin_amdgcn_s_setprio(0);
        bar();
      }
    }
    if (wr == 0) bar();
    // every LDS slot is free: the next tile's prologue goes out before this tile's stores
    const Tile done = cur;
    ++rnd;
    k = (long long)rnd * nslot + (slot + rnd) % nslot;
    const bool more = k < len;
    if (more) {
      cur = decode(base + k);
      prologue(cur);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = done.m0 + (i >> 2) * 128 + wr * 64 + (i & 3) * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = done.n0 + (j >> 1) * 128 + wc * 32 + (j & 1) * 16 + 4 * (lane >> 4);
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = p.alpha * acc[i][j][u];
        if (p.tri == 3) {
#pragma unroll
          for (int u = 0; u < 4; ++u) if (n + u > m) v[u] = 0.f;
        }
        const long long idx = done.coff + (long long)m * p.ldc + n;
        if (OUT_F32)
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.C) + idx) = make_float4(v[0], v[1], v[2], v[3]);
        else
          *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.C) + idx) =
              make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      }
    }
    if (!more) break;
    pend = true;
  }
}

template <int A_T, int B_T, bool F32>
hipError_t launch_pp(GemmArgs a, int batch, hipStream_t stream) {
  a.tiles_m = a.M / BM2;
  a.tiles_n = a.N / BN2;
  a.nbatch = batch;
  const size_t lds = 8 * PIECE;
  auto k = gemm_pp_kernel<A_T, B_T, F32>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(256), dim3(NT2), lds, stream, a);   // one block per CU, 32 per XCD
  return hipGetLastError();
}

}  // namespace

hipError_t gemm_pp_launch(const gemmk::GemmArgs* a, int a_t, int b_t, int out_f32, int batch, hipStream_t stream) {
#define OBST_GEMMPP_CASE(AT, BT, F) \
  if (a_t == AT && b_t == BT && (out_f32 != 0) == F) return launch_pp<AT, BT, F>(*a, batch, stream);
  OBST_GEMMPP_CASE(0, 0, false) OBST_GEMMPP_CASE(0, 1, false) OBST_GEMMPP_CASE(1, 0, false)
  OBST_GEMMPP_CASE(1, 1, false) OBST_GEMMPP_CASE(0, 0, true) OBST_GEMMPP_CASE(0, 1, true)
  OBST_GEMMPP_CASE(1, 0, true) OBST_GEMMPP_CASE(1, 1, true)
#undef OBST_GEMMPP_CASE
  return hipErrorInvalidValue;
}
