// K01/K02: bf16 MFMA GEMM for gfx950 with fused epilogues. One kernel template serves the forward (X·W),
// data-gradient (dY·Wᵀ) and weight-gradient (Xᵀ·dY) products of every linear in the block grammar
// (reference einsum sites: src/model/backend.py:108-110, basic.py:33-126, spatial.py:45-81), as a
// strided, two-level-batched GEMM (batch = heads for `group` linears, heads×batch for the token mixer).
//
//   C[m][n] = epilogue( alpha * sum_k A(m,k) * B(k,n) )
//   A_T = 0 : A stored [M][K] (K contiguous)      A_T = 1 : A stored [K][M] (M contiguous)
//   B_T = 0 : B stored [N][K] (K contiguous)      B_T = 1 : B stored [K][N] (N contiguous)
//
// Design (cdna_hip_programming.md §5): 128x128x64 block tile, 4 waves (2x2), each wave 64x64 = 4x4 tiles of
// v_mfma_f32_16x16x32_bf16; register-staged double-buffered LDS with ONE barrier per K-step (loads for tile k+1
// are issued before the MFMAs of tile k). K-contiguous operands are read with ds_read_b128 from an XOR-swizzled
// [rows][64] image (conflict-free: chunk ^= (row>>1)&7); M/N-contiguous operands are stored [64][128] as loaded
// (coalesced) and read through the CDNA4 hardware transpose ds_read_b64_tr_b16 with chunk ^= f(k) so both
// 16-lane groups of a half-wave hit distinct banks. The MFMA is issued as mfma(B, A) so each lane ends with 4
// consecutive output columns (8-byte bf16 / 16-byte fp32 stores). Block ids are remapped XCD-aware (T1) and
// grouped 8 tiles along M so blocks that share an XCD share A panels in its L2.
#include "common.h"
#include "gemm_desc.h"
#include "gemm_kern.h"
#include <stdlib.h>

namespace {


// --- staging: global -> registers -------------------------------------------------------------------------------
template <int T>
__device__ __forceinline__ void load_tile(uint4 (&reg)[4], const bf16_t* X, long long ld, int r0, int R, int k0,
                                          int K, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + i * NT;
    int row, col;
    bool ok;
    const bf16_t* g;
    if (T == 0) {  // [rows][K]
      row = q >> 3; col = (q & 7) * 8;
      ok = (r0 + row < R) && (k0 + col < K);
      g = X + (long long)(r0 + row) * ld + (k0 + col);
    } else {       // [K][rows]
      row = q >> 4; col = (q & 15) * 8;
      ok = (k0 + row < K) && (r0 + col < R);
      g = X + (long long)(k0 + row) * ld + (r0 + col);
    }
    reg[i] = ok ? *reinterpret_cast<const uint4*>(g) : make_uint4(0, 0, 0, 0);
  }
}

template <int T>
__device__ __forceinline__ void store_tile(char* lds, const uint4 (&reg)[4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + i * NT;
    int off;
    if (T == 0) {
      const int row = q >> 3, c = q & 7;
      off = row * 128 + ((c ^ ((row >> 1) & 7)) << 4);
    } else {
      const int k = q >> 4, c = q & 15;
      off = k * 256 + ((c ^ kswz(k)) << 4);
    }
    *reinterpret_cast<uint4*>(lds + off) = reg[i];
  }
}

template <int A_T, int B_T, bool OUT_F32>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // stage s: A image at smem + s*2*TILE_BYTES, B image right after it

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap (T1), then GROUP=8 ordering along M.
  int bid = blockIdx.x;
  {
    const int nwg = gridDim.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    bid = base + (bid >> 3);
  }
  const int GROUP = 8;
  const int per_group = GROUP * p.tiles_n;
  const int first_m = (bid / per_group) * GROUP;
  const int gsz = min(p.tiles_m - first_m, GROUP);
  const int tm = first_m + (bid % per_group) % gsz;
  const int tn = (bid % per_group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int b1 = blockIdx.y / p.nb2, b2 = blockIdx.y % p.nb2;
  const bf16_t* A = p.A + b1 * p.a_s1 + b2 * p.a_s2;
  const bf16_t* B = p.B + b1 * p.b_s1 + b2 * p.b_s2;

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  uint4 ra[4], rb[4];
  const int nk = (p.K + BK - 1) / BK;
  load_tile<A_T>(ra, A, p.lda, m0, p.M, 0, p.K, tid);
  load_tile<B_T>(rb, B, p.ldb, n0, p.N, 0, p.K, tid);
  store_tile<A_T>(smem, ra, tid);
  store_tile<B_T>(smem + TILE_BYTES, rb, tid);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int s = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      load_tile<A_T>(ra, A, p.lda, m0, p.M, (kt + 1) * BK, p.K, tid);
      load_tile<B_T>(rb, B, p.ldb, n0, p.N, (kt + 1) * BK, p.K, tid);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<A_T>(smem + s * 2 * TILE_BYTES, wm * 64 + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag<B_T>(smem + s * 2 * TILE_BYTES + TILE_BYTES, wn * 64 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_tile<A_T>(smem + (s ^ 1) * 2 * TILE_BYTES, ra, tid);
      store_tile<B_T>(smem + (s ^ 1) * 2 * TILE_BYTES + TILE_BYTES, rb, tid);
    }
    __syncthreads();
  }

  // ---- epilogue: lane holds C[m][n..n+3] for each (i, j) tile -----------------------------------------------------
  const long long coff = b1 * p.c_s1 + b2 * p.c_s2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
      if (n >= p.N) continue;
      const long long idx = coff + (long long)m * p.ldc + n;
      float v[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) v[t] = p.alpha * acc[i][j][t];
          if (p.tri == 3) {
#pragma unroll
            for (int t = 0; t < 4; ++t) if (n + t > m) v[t] = 0.f;
          }
      if (OUT_F32) {
        float* C = reinterpret_cast<float*>(p.C) + idx;
        if (p.beta != 0.f) {
          float4 o = *reinterpret_cast<const float4*>(C);
          v[0] += p.beta * o.x; v[1] += p.beta * o.y; v[2] += p.beta * o.z; v[3] += p.beta * o.w;
        }
        if (p.R) {
          float4 r = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.R) + idx);
          v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
        }
        if (p.act) {
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] = act_fwd(p.act, v[t]);
        }
        *reinterpret_cast<float4*>(C) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        if (p.mode == 1) {
          if (p.R) {
            uint2 r = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(p.R) + idx);
            v[0] += bf2f(r.x & 0xffff); v[1] += bf2f(r.x >> 16); v[2] += bf2f(r.y & 0xffff); v[3] += bf2f(r.y >> 16);
          }
          uint2 z = *reinterpret_cast<const uint2*>(p.Zin + idx);
          v[0] *= act_grad(p.act, bf2f(z.x & 0xffff)); v[1] *= act_grad(p.act, bf2f(z.x >> 16));
          v[2] *= act_grad(p.act, bf2f(z.y & 0xffff)); v[3] *= act_grad(p.act, bf2f(z.y >> 16));
        } else {
          if (p.R) {
            uint2 r = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(p.R) + idx);
            v[0] += bf2f(r.x & 0xffff); v[1] += bf2f(r.x >> 16); v[2] += bf2f(r.y & 0xffff); v[3] += bf2f(r.y >> 16);
          }
          if (p.Zout) {
            *reinterpret_cast<uint2*>(p.Zout + idx) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
          }
          if (p.act) {
#pragma unroll
            for (int t = 0; t < 4; ++t) v[t] = act_fwd(p.act, v[t]);
          }
        }
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.C) + idx) =
            make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      }
    }
  }
}

template <int A_T, int B_T, bool F32>
hipError_t launch(const GemmArgs& a, int batch, hipStream_t stream) {
  dim3 grid(a.tiles_m * a.tiles_n, batch);
  const size_t lds = 4 * TILE_BYTES;
  auto k = gemm_bf16_kernel<A_T, B_T, F32>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(k, grid, dim3(NT), lds, stream, a);
  return hipGetLastError();
}


// ================================================================================================================
// 256x256x64 tiles, 8 waves (2 M x 4 N, 128x64 per wave), staged by direct global->LDS DMA
// (global_load_lds_dwordx4: each wave-instruction writes 1 KiB of LDS lane-linearly). The XOR swizzle of the LDS
// image is applied to the per-lane SOURCE address (cdna guide §5.4 rule 21), the ds_read side applies the same
// XOR. Requires K % 64 == 0; rows/columns beyond M/N are clamped to valid memory (their results are never stored).

// ---------------------------------------------------------------------------------------------------------------
// Phase-pipelined 256x256 kernel (cdna_hip_programming.md §5 "256² 8-phase template", re-derived here).
// 8 waves = 2 (M) x 4 (N) groups; C is cut into quadrants (qm, qn) of 128 x 128, and wave (wr, wc) owns the
// 64 x 32 sub-block (wr, wc) of every quadrant (so its 128 x 64 of C are 2 x 2 sub-blocks 128 apart). A K-tile
// (BK = 64) is computed in 4 phases, one quadrant each, in the order (qm,qn) = (0,0) (0,1) (1,1) (1,0); fragments
// are loaded at the START of a phase: p0 A[qm=0] + B[qn=0], p1 B[qn=1], p2 A[qm=1], p3 nothing (B[qn=0] still in
// registers). LDS holds 8 "pieces" of 16 KiB: {A0, A1, B0, B1} x K-tile parity, A_q = rows q*128..+128 and
// B_q = columns q*128..+128 of the block tile -- contiguous, so an M/N-contiguous operand streams whole 256-B
// rows -- and a piece is dead as soon as its quadrant phase retired. Each phase stages ONE piece by LDS-DMA (2 x 16 B per thread), 4-6 phases ahead:
//   phase 4t+0: B1(t+1)   4t+1: A1(t+1)   4t+2: A0(t+2)   4t+3: B0(t+2)
// and waits with a COUNTED vmcnt(8) (4 pieces may stay in flight), never vmcnt(0) in the steady state.
// The two M wave groups run one barrier apart (group 1 takes an extra barrier up front) so one group's ds_reads
// and LDS-DMA issue overlap the other group's 16 MFMAs; each phase = reads, stage, wait, barrier, lgkmcnt(0),
// MFMAs (setprio 1), barrier. Derived hazard rules (intervals between barriers, stagger included):
//   RAW: a piece read in phase Q was waited for in phase <= Q-1 by every thread (vmcnt counts above);
//   WAR: a piece's slot is restaged >= 2 phases after its last read phase (A0: +2, B0: +3, B1: +3, A1: +3).
template <int A_T, int B_T, bool OUT_F32>
__global__ __launch_bounds__(NT2, 1) void gemm_ph_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  // XCD-aware remap over the WHOLE grid (tiles x batches): the hardware deals workgroups to the 8 XCDs round-robin
  // in linear order, so with few tiles per batch (token mixer: 8 M-tiles x 256 (b, h) batches) a per-row remap
  // pinned tile index x to XCD x for every batch -- with triangular operands one XCD got all the longest tiles
  // (8 K-tiles) and another all the shortest (1). Remapped linearly, each XCD owns a contiguous run of whole
  // batches, i.e. every tile shape in equal measure.
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
  int tm = first_m + (bid % per_group) % gsz;
  const int tn = (bid % per_group) / gsz;
  if (p.tri == 1) tm = p.tiles_m - 1 - tm;   // lower-triangular A: the longest K spans (largest m) dispatch first
  const int m0 = tm * BM2, n0 = tn * BN2;
  const int split = ybat % p.ksplit, bidx = ybat / p.ksplit;
  const int b1 = bidx / p.nb2, b2 = bidx % p.nb2;
  int kspan = p.K / p.ksplit, kbeg = split * kspan;
  if (p.tri == 1) kspan = min(p.K, (m0 + BM2 + BK - 1) / BK * BK);             // A[m][k] = 0 for k > m
  if (p.tri == 2) { kbeg = min(m0 / BK * BK, p.K - BK); kspan = p.K - kbeg; }   // A[m][k] = 0 for k < m
  if (p.tri == 3 && OUT_F32 && p.beta == 1.f && n0 > m0 + BM2 - 1) return;     // no output in this tile
  const bool ksp = p.kin > 0;   // split contraction index: tile offsets are mapped per tile (K-contiguous operands)
  const bf16_t* A = p.A + b1 * p.a_s1 + b2 * p.a_s2 +
                    (ksp ? 0LL : (A_T == 0 ? (long long)kbeg : (long long)kbeg * p.lda));
  const bf16_t* B = p.B + b1 * p.b_s1 + b2 * p.b_s2 +
                    (ksp ? 0LL : (B_T == 0 ? (long long)kbeg : (long long)kbeg * p.ldb));
  const int nk = kspan / BK;
  auto ktile = [&](int t, long long sk) -> long long {   // element offset of k-tile t (kin % BK == 0)
    if (!ksp) return (long long)t * BK;
    const int k = kbeg + t * BK;
    return (long long)(k / p.kin) * sk + (k % p.kin);
  };

  // piece slots: (parity * 4 + {A0, A1, B0, B1}) * 16 KiB
  auto slot = [&](int t, int pc) -> char* { return smem + ((t & 1) * 4 + pc) * PIECE; };
  auto stageA = [&](int t, int q) {
    stage_piece<A_T, true>(slot(t, q), A, p.lda, m0, p.M, ktile(t, p.a_sk), q, wave, lane);
  };
  auto stageB = [&](int t, int q) {
    stage_piece<B_T, false>(slot(t, 2 + q), B, p.ldb, n0, p.N, ktile(t, p.b_sk), q, wave, lane);
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // prologue: the pieces phases -6..-1 would have staged
  stageA(0, 0); stageB(0, 0); stageB(0, 1); stageA(0, 1);
  if (nk > 1) { stageA(1, 0); stageB(1, 0); asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
  else { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
  if (wr == 1) bar();
  bar();

  bf16x8_t af[4][2], bq0[2][2], bq1[2][2];
  for (int t = 0; t < nk; ++t) {
    const bool tail = t + 2 >= nk;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int qm = (ph == 0 || ph == 1) ? 0 : 1;
      const int qn = (ph == 0 || ph == 3) ? 0 : 1;
      // 1. fragments of this phase
      if (ph == 0) {
        const char* ib = slot(t, 2);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) bq0[j][kk] = read_frag<B_T>(ib, wc * 32 + j * 16, kk, lane);
      }
      if (ph == 0 || ph == 2) {
        const char* ia = slot(t, qm);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) af[i][kk] = read_frag<A_T>(ia, wr * 64 + i * 16, kk, lane);
      }
      if (ph == 1) {
        const char* ib = slot(t, 3);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) bq1[j][kk] = read_frag<B_T>(ib, wc * 32 + j * 16, kk, lane);
      }
      // 2. one piece of LDS-DMA
      if (ph == 0 && t + 1 < nk) stageB(t + 1, 1);
      if (ph == 1 && t + 1 < nk) stageA(t + 1, 1);
      if (ph == 2 && t + 2 < nk) stageA(t + 2, 0);
      if (ph == 3 && t + 2 < nk) stageB(t + 2, 0);
      // 3. counted wait, barrier, MFMAs, barrier
      if (tail) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

  const long long coff = b1 * p.c_s1 + b2 * p.c_s2;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + (i >> 2) * 128 + wr * 64 + (i & 3) * 16 + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + (j >> 1) * 128 + wc * 32 + (j & 1) * 16 + 4 * (lane >> 4);
      if (n >= p.N) continue;
      float v[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) v[t] = p.alpha * acc[i][j][t];
      if (p.tri == 3) {
#pragma unroll
        for (int t = 0; t < 4; ++t) if (n + t > m) v[t] = 0.f;
      }
      if (OUT_F32 && p.ksplit > 1) {
        *reinterpret_cast<float4*>(p.ws + (long long)split * p.M * p.N + (long long)m * p.N + n) =
            make_float4(v[0], v[1], v[2], v[3]);
      } else {
        epilogue_store<OUT_F32>(p, coff + (long long)m * p.ldc + n, v);
      }
    }
  }
}

// C[m][n] = beta * C[m][n] + sum_s ws[s][m][n]   (float4 per lane)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(float* __restrict__ C, const float* __restrict__ ws,
                                                             long long mn, long long ldc, int N, int ks, float beta) {
  const long long nv = mn / 4;
  for (long long v = (long long)blockIdx.x * 256 + threadIdx.x; v < nv; v += (long long)gridDim.x * 256) {
    const long long e = v * 4, m = e / N, n = e % N;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < ks; ++s) {
      const float4 w = reinterpret_cast<const float4*>(ws + s * mn)[v];
      acc.x += w.x; acc.y += w.y; acc.z += w.z; acc.w += w.w;
    }
    float4* c = reinterpret_cast<float4*>(C + m * ldc + n);
    if (beta != 0.f) {
      const float4 o = *c;
      acc.x += beta * o.x; acc.y += beta * o.y; acc.z += beta * o.z; acc.w += beta * o.w;
    }
    *c = acc;
  }
}

// batched split-K fold: C[b] (+ beta C[b]) = sum_s ws[b][s] for nb = nb1 x nb2 batches (C batch strides c_s1 / c_s2)
__global__ __launch_bounds__(256) void splitk_reduce_batched_kernel(float* __restrict__ C, const float* __restrict__ ws,
                                                                    long long mn, long long ldc, int N, int ks,
                                                                    float beta, int nb, int nb2, long long c_s1,
                                                                    long long c_s2) {
  const long long nv = mn / 4, tot = nv * nb;
  for (long long u = (long long)blockIdx.x * 256 + threadIdx.x; u < tot; u += (long long)gridDim.x * 256) {
    const long long b = u / nv, v = u % nv;
    const long long e = v * 4, m = e / N, n = e % N;
    const float* wb = ws + b * ks * mn;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < ks; ++s) {
      const float4 w = reinterpret_cast<const float4*>(wb + s * mn)[v];
      acc.x += w.x; acc.y += w.y; acc.z += w.z; acc.w += w.w;
    }
    float4* c = reinterpret_cast<float4*>(C + (b / nb2) * c_s1 + (b % nb2) * c_s2 + m * ldc + n);
    if (beta != 0.f) {
      const float4 o = *c;
      acc.x += beta * o.x; acc.y += beta * o.y; acc.z += beta * o.z; acc.w += beta * o.w;
    }
    *c = acc;
  }
}

float* splitk_workspace(size_t bytes) {
  static float* buf = nullptr;
  static size_t cap = 0;
  if (bytes > cap) {
    if (buf) (void)hipFree(buf);
    if (hipMalloc(&buf, bytes) != hipSuccess) { buf = nullptr; cap = 0; return nullptr; }
    cap = bytes;
  }
  return buf;
}

template <int A_T, int B_T, bool F32>
hipError_t launch_ph(GemmArgs a, int batch, hipStream_t stream) {
  a.tiles_m = (a.M + BM2 - 1) / BM2;
  a.tiles_n = (a.N + BN2 - 1) / BN2;
  dim3 grid(a.tiles_m * a.tiles_n, batch * a.ksplit);
  const size_t lds = 8 * PIECE;
  auto k = gemm_ph_kernel<A_T, B_T, F32>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(k, grid, dim3(NT2), lds, stream, a);
  if (F32 && a.ksplit > 1) {
    const long long mn = (long long)a.M * a.N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(2048), dim3(256), 0, stream, reinterpret_cast<float*>(a.C), a.ws,
                       mn, a.ldc, a.N, a.ksplit, a.beta);
  }
  return hipGetLastError();
}

}  // namespace

// OBST_GEMM_4W=0 keeps the plain products on the phase kernels (A/B); runtime switch obst_gemm4w_set
static int g_4w = -1;
static long long g_4w_calls = 0;
static int g4w_enabled() {
  if (g_4w < 0) {
    const char* e = getenv("OBST_GEMM_4W");
    g_4w = e ? atoi(e) : 1;
  }
  return g_4w;
}
OBST_API int obst_gemm4w_set(int on) {
  const int old = g4w_enabled();
  g_4w = on;
  return old;
}
OBST_API long long obst_gemm4w_calls() { return g_4w_calls; }

OBST_API int obst_gemm4w_enabled() { return g4w_enabled(); }
// diagnostics: device buffer of 5 u64 per block (gemm4w.h) filled by the following gemm4w launches; null: off
static unsigned long long* g_4w_stamps = nullptr;
OBST_API void obst_gemm4w_stamps(unsigned long long* dev) { g_4w_stamps = dev; }

static int getenv_big() {   // OBST_GEMM_BIG=0: only the 128x128 kernel (A/B, debugging)
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("OBST_GEMM_BIG");
    v = e ? (e[0] - '0') : 2;
    if (v == 1) v = 2;       // the former two-stage 256x256 kernel (superseded by the phase kernels, removed)
  }
  return v;
}


// Returns 0 on success, <0 on a host-side shape/alignment violation, >0 for a HIP error.
OBST_API int obst_gemm(const ObstGemmDesc* d, hipStream_t stream) {
  if (d->M <= 0 || d->N <= 0 || d->K <= 0 || d->batch1 <= 0 || d->batch2 <= 0) return -1;
  // 16-byte staging loads: the contiguous extent and every leading dimension must be multiples of 8 elements.
  if (d->K % 8 || d->N % 8) return -2;
  if (d->a_t == 1 && d->M % 8) return -3;
  if (d->lda % 8 || d->ldb % 8 || d->ldc % 8) return -4;
  if (((uintptr_t)d->A | (uintptr_t)d->B) & 15) return -5;
  if (((uintptr_t)d->C) & 15) return -6;
  {
    const int r = obst_blaslt_gemm_split(d, stream);
    if (r <= 0) return r;
  }
  GemmArgs a;
  a.A = (const bf16_t*)d->A; a.B = (const bf16_t*)d->B; a.C = d->C; a.R = d->R;
  a.Zout = (bf16_t*)d->Zout; a.Zin = (const bf16_t*)d->Zin;
  a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
  a.a_s1 = d->a_s1; a.a_s2 = d->a_s2; a.b_s1 = d->b_s1; a.b_s2 = d->b_s2; a.c_s1 = d->c_s1; a.c_s2 = d->c_s2;
  a.M = d->M; a.N = d->N; a.K = d->K; a.nb2 = d->batch2;
  a.tiles_m = (d->M + BM - 1) / BM; a.tiles_n = (d->N + BN - 1) / BN;
  a.alpha = d->alpha; a.beta = d->beta; a.act = d->act; a.mode = d->mode; a.tri = d->tri;
  a.kin = d->kin; a.a_sk = d->a_sk; a.b_sk = d->b_sk;
  a.stamps = g_4w_stamps;
  if (d->kin) {   // split contraction index: phase kernel, K-contiguous operands, whole 64-deep tiles per inner block
    if (d->kin < 0 || d->kin % 64 || d->K % d->kin || d->a_t || d->b_t || (d->tri == 1 || d->tri == 2) ||
        d->a_sk % 8 || d->b_sk % 8 || d->M < 256 || d->N < 256)
      return -9;
    a.ksplit = 1;
    a.ws = nullptr;
    const int batch = d->batch1 * d->batch2;
    hipError_t e = d->out_f32 ? launch_ph<0, 0, true>(a, batch, stream) : launch_ph<0, 0, false>(a, batch, stream);
    return e == hipSuccess ? 0 : (int)e;
  }
  if (d->tri < 0 || d->tri > 3 || ((d->tri == 1 || d->tri == 2) && d->M != d->K) || (d->tri == 3 && d->M != d->N))
    return -8;
  const int batch = d->batch1 * d->batch2;
  hipError_t e;
  // big-tile path: needs K % 64 == 0, M/N >= 256 and enough 256x256 tiles to fill the 256 CUs twice
  const long long big_tiles = (long long)((d->M + 255) / 256) * ((d->N + 255) / 256) * batch;
  const int impl = getenv_big();
  a.ksplit = 1;
  // split-K (fp32 accumulate-into-C GEMMs with few output tiles, i.e. the weight gradients): atomic-add epilogue
  static int ksplit_env = -1;
  if (ksplit_env < 0) {
    const char* e = getenv("OBST_GEMM_KSPLIT");
    ksplit_env = e ? atoi(e) : 1;
  }
  a.ws = nullptr;
  if (ksplit_env > 0 && impl >= 2 && big_tiles < 512 && d->tri == 0 && d->out_f32 && !d->R && !d->act && d->mode == 0 &&
      batch == 1 && d->M >= 256 && d->N >= 256 && d->N % 4 == 0) {
    int ks = 1;
    const long long want = 256LL * ksplit_env;   // blocks: one (or ksplit_env) per CU
    while (big_tiles * ks < want && d->K % (64 * ks * 2) == 0 && d->K / (ks * 2) >= 1024) ks *= 2;
    if (ks > 1) {
      a.ws = splitk_workspace((size_t)ks * d->M * d->N * sizeof(float));
      if (!a.ws) ks = 1;
    }
    a.ksplit = ks;
  }
  const bool big = impl > 0 && d->K % 64 == 0 && d->M >= 256 && d->N >= 256 &&
                   big_tiles * a.ksplit >= (a.ksplit > 1 ? 256 : 512) &&
                   (d->a_t == 0 || d->M % 8 == 0) && (d->b_t == 0 || d->N % 8 == 0);
  // one-wave-per-SIMD kernel (gemm4w.hip): every plain product and the triangular-A ones (tri 1 / 2: the token
  // mixer, K03 -- each output tile runs only its K range); not the split contraction index or tri 3
  if (g4w_enabled() && (d->tri == 0 || d->tri == 1 || d->tri == 2) && d->K % 64 == 0 &&
      (d->a_t == 0 || d->M % 8 == 0) && (d->b_t == 0 || d->N % 8 == 0)) {
    // split-K for fp32 products with few output tiles (the weight gradients): the persistent kernel runs
    // ceil(tiles * ks / 256) rounds of K / ks each; a split costs a deterministic fold over ks fp32 slabs. Pick the
    // ks of least modelled time (1.25 us per 64-deep K-tile of a tile, ~5 TB/s for the fold), workspace <= 1 GiB.
    int ks = 1;
    // batched products too (the per-head group-linear weight gradients: few tiles per batch); C batch strides must
    // keep 16-byte alignment for the fold. The folds index float4s of rows (m = e / N, e < M * N / 4): N and ldc
    // must be multiples of 4 (the entry checks already require 8; restated here so the fold's own contract is local)
    if (ksplit_env > 0 && big_tiles < 512 && d->out_f32 && !d->R && !d->act && d->mode == 0 && d->tri == 0 &&
        d->N % 4 == 0 && d->ldc % 4 == 0 &&
        (batch == 1 || (d->c_s1 % 4 == 0 && d->c_s2 % 4 == 0))) {
      const double per_k = 1.25 / 64.0;   // us per K element of one tile
      double best = 1e300;
      for (int c = 1; c <= 16; c *= 2) {
        if (d->K % (64 * c) || (c > 1 && d->K / c < 512) || (size_t)c * batch * d->M * d->N * 4 > (1ull << 30)) continue;
        const double rounds = (double)((big_tiles * c + 255) / 256);
        const double t = rounds * (d->K / c) * per_k +
                         (c > 1 ? (double)(c + (d->beta != 0.f ? 2 : 1)) * batch * d->M * d->N * 4.0 / 5e6 : 0.0);
        if (t < best * 0.98) { best = t; ks = c; }
      }
      if (ks > 1) {
        a.ws = splitk_workspace((size_t)ks * batch * d->M * d->N * sizeof(float));
        if (!a.ws) ks = 1;
      }
    }
    a.ksplit = ks;
    e = gemm4w_launch(&a, d->a_t, d->b_t, d->out_f32, batch, stream);
    if (e == hipSuccess && d->out_f32 && a.ksplit > 1) {
      const long long mn = (long long)a.M * a.N;
      if (batch == 1)
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3(2048), dim3(256), 0, stream, reinterpret_cast<float*>(a.C),
                           a.ws, mn, a.ldc, a.N, a.ksplit, a.beta);
      else
        hipLaunchKernelGGL(splitk_reduce_batched_kernel, dim3(2048), dim3(256), 0, stream,
                           reinterpret_cast<float*>(a.C), a.ws, mn, a.ldc, a.N, a.ksplit, a.beta, batch, a.nb2,
                           a.c_s1, a.c_s2);
      e = hipGetLastError();
    }
    ++g_4w_calls;
    return e == hipSuccess ? 0 : (int)e;
  }
  // persistent phase kernel: plain products on whole 256x256 tiles, at least two tiles per CU (OBST_GEMM_PP=0: off)
  static int pp_env = -1;
  if (pp_env < 0) {
    const char* e = getenv("OBST_GEMM_PP");
    pp_env = e ? atoi(e) : 1;
  }
  if (big && impl >= 2 && pp_env && a.ksplit == 1 && d->M % 256 == 0 && d->N % 256 == 0 && !d->R && !d->Zout &&
      !d->Zin && d->act == 0 && d->mode == 0 && (!d->out_f32 || d->beta == 0.f) && big_tiles >= 512) {
    e = gemm_pp_launch(&a, d->a_t, d->b_t, d->out_f32, batch, stream);
    return e == hipSuccess ? 0 : (int)e;
  }
  if (big) {
#define OBST_GEMM256_CASE(AT, BT, F)                                                             \
    if (d->a_t == AT && d->b_t == BT && (d->out_f32 != 0) == F) {                                \
      e = launch_ph<AT, BT, F>(a, batch, stream);                                              \
      return e == hipSuccess ? 0 : (int)e;                                                         \
    }
    OBST_GEMM256_CASE(0, 0, false) OBST_GEMM256_CASE(0, 1, false) OBST_GEMM256_CASE(1, 0, false)
    OBST_GEMM256_CASE(1, 1, false) OBST_GEMM256_CASE(0, 0, true) OBST_GEMM256_CASE(0, 1, true)
    OBST_GEMM256_CASE(1, 0, true) OBST_GEMM256_CASE(1, 1, true)
#undef OBST_GEMM256_CASE
  }
#define OBST_GEMM_CASE(AT, BT, F)                                   \
  if (d->a_t == AT && d->b_t == BT && (d->out_f32 != 0) == F) {    \
    e = launch<AT, BT, F>(a, batch, stream);                         \
    return e == hipSuccess ? 0 : (int)e;                             \
  }
  OBST_GEMM_CASE(0, 0, false) OBST_GEMM_CASE(0, 1, false) OBST_GEMM_CASE(1, 0, false) OBST_GEMM_CASE(1, 1, false)
  OBST_GEMM_CASE(0, 0, true) OBST_GEMM_CASE(0, 1, true) OBST_GEMM_CASE(1, 0, true) OBST_GEMM_CASE(1, 1, true)
#undef OBST_GEMM_CASE
  return -7;
}
