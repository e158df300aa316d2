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
        if (p.Zout)   // its bf16 copy
          *reinterpret_cast<uint2*>(p.Zout + idx) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
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


// tri 3 (only n <= m receives the product): the slabs of tiles above the diagonal were never written
__device__ __forceinline__ void tri3_mask(float4& acc, long long m, long long n, int tri3) {
  if (!tri3) return;
  acc.x = n > m ? 0.f : acc.x;
  acc.y = n + 1 > m ? 0.f : acc.y;
  acc.z = n + 2 > m ? 0.f : acc.z;
  acc.w = n + 3 > m ? 0.f : acc.w;
}

// C[m][n] = beta * C[m][n] + sum_s ws[s][m][n]   (float4 per lane)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(float* __restrict__ C, const float* __restrict__ ws,
                                                             long long mn, long long ldc, int N, int ks, float beta,
                                                             int tri3) {
  const long long nv = mn / 4;
  for (long long v = (long long)blockIdx.x * 256 + threadIdx.x; v < nv; v += (long long)gridDim.x * 256) {
    const long long e = v * 4, m = e / N, n = e % N;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < ks; ++s) {
      const float4 w = reinterpret_cast<const float4*>(ws + s * mn)[v];
      acc.x += w.x; acc.y += w.y; acc.z += w.z; acc.w += w.w;
    }
    tri3_mask(acc, m, n, tri3);
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
                                                                    long long c_s2, int tri3) {
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
    tri3_mask(acc, m, n, tri3);
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

}  // namespace

static long long g_4w_calls = 0, g_4w_queue_calls = 0;
OBST_API long long obst_gemm4w_calls() { return g_4w_calls; }
OBST_API long long obst_gemm4w_queue_calls() { return g_4w_queue_calls; }   // launches that took the tile queue
// diagnostics: device buffer of 8 u64 per block (gemm4w.h) filled by the following gemm4w launches; null: off
static unsigned long long* g_4w_stamps = nullptr;
OBST_API void obst_gemm4w_stamps(unsigned long long* dev) { g_4w_stamps = dev; }

// gemm4w dynamic tile queue (OBST_G4W_QUEUE, default 1): a ring of per-launch counter blocks (8 per-XCD counters
// each), zeroed on the launch's stream just before it -- in-flight launches on other streams (and the slots baked
// into a captured graph) keep their own block while the ring has not wrapped
static int g4w_queue_env() {
  static int v = [] { const char* e = getenv("OBST_G4W_QUEUE"); return e ? atoi(e) : 1; }();
  return v;
}
// OBST_G4W_TRI_GROUP (default: auto, below): work order of the triangular (token-mixer) products -- G > 0: batches in groups of
// G, the tile rows of a group heaviest first inside it (gemm4w.h decode4), so the B operand of a (batch, head) --
// x[b, :, h, :], re-read by each of its 8 tile rows -- stays in L2 / MALL between its reads; 0: tile rows slowest
// (each x re-read one whole sweep over the 2048 (batch, head) products later). ctx32_mixer at batch 256: 1862-1869
// vs 1934-1938 ms/step (G = 32: 1870; kbench's 32-batch mixer, which fits the MALL either way: equal;
// tools/lab/r6_tri_group.sh)
// Auto (unset): 8 when the B operands of the launch exceed 512 MiB (past the 256 MiB MALL), else 0 -- kbench's
// 32-batch mixer (268 MB of x) ran 3-5 % slower grouped
static int g_tri_group_force = -1;   // obst_gemm4w_tri_group (tests): >= 0 overrides the env / auto choice
OBST_API void obst_gemm4w_tri_group(int g) { g_tri_group_force = g; }
static int g4w_tri_group_env(long long b_bytes) {
  static int v = [] { const char* e = getenv("OBST_G4W_TRI_GROUP"); return e ? atoi(e) : -1; }();
  if (g_tri_group_force >= 0) return g_tri_group_force;
  if (v >= 0) return v;
  return b_bytes > (512ll << 20) ? 8 : 0;
}
static int g4w_queue_tri_env() {   // the triangular (token-mixer) products on the queue too (0: static walk)
  static int v = [] { const char* e = getenv("OBST_G4W_QUEUE_TRI"); return e ? atoi(e) : 1; }();
  return v;
}
static unsigned* g4w_queue_slot(hipStream_t stream) {
  constexpr int RING = 256;
  static unsigned* ring = nullptr;
  static int next = 0;
  if (!ring && hipMalloc(reinterpret_cast<void**>(&ring), RING * 8 * sizeof(unsigned)) != hipSuccess) {
    ring = nullptr;
    return nullptr;
  }
  unsigned* q = ring + (next++ % RING) * 8;
  if (hipMemsetAsync(q, 0, 8 * sizeof(unsigned), stream) != hipSuccess) return nullptr;
  return q;
}

// Every GEMM of the framework is one of two hand-written kernels: gemm4w (gemm4w.h: the one-wave-per-SIMD 256x256
// persistent kernel -- every product with K % 64 == 0, including the triangular token mixer (tri 1 / 2), the masked
// lower-triangle output (tri 3) and the split contraction index) and the 128x128 kernel above for what gemm4w does
// not take (K % 64 != 0, tri 3 with a transposed B or a fused activation, a transposed operand whose contiguous extent
// is not a multiple of 8). Decode-step products (M <= 32) go to skinny.hip from the Python dispatch.
// Returns 0 on success, <0 on a host-side shape/alignment violation, >0 for a HIP error.
OBST_API int obst_gemm(const ObstGemmDesc* d, hipStream_t stream) {
  if (d->M <= 0 || d->N <= 0 || d->K <= 0 || d->batch1 <= 0 || d->batch2 <= 0) return -1;
  // 16-byte staging loads: the contiguous extent and every leading dimension must be multiples of 8 elements.
  if (d->K % 8 || d->N % 8) return -2;
  if (d->a_t == 1 && d->M % 8) return -3;
  if (d->lda % 8 || d->ldb % 8 || d->ldc % 8) return -4;
  if (((uintptr_t)d->A | (uintptr_t)d->B) & 15) return -5;
  if (((uintptr_t)d->C) & 15) return -6;
  if (d->tri < 0 || d->tri > 3 || ((d->tri == 1 || d->tri == 2) && d->M != d->K) || (d->tri == 3 && d->M != d->N))
    return -8;
  GemmArgs a;
  a.A = (const bf16_t*)d->A; a.B = (const bf16_t*)d->B; a.C = d->C; a.R = d->R;
  a.Zout = (bf16_t*)d->Zout; a.Zin = (const bf16_t*)d->Zin;
  a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
  a.a_s1 = d->a_s1; a.a_s2 = d->a_s2; a.b_s1 = d->b_s1; a.b_s2 = d->b_s2; a.c_s1 = d->c_s1; a.c_s2 = d->c_s2;
  a.M = d->M; a.N = d->N; a.K = d->K; a.nb2 = d->batch2;
  a.tiles_m = (d->M + BM - 1) / BM; a.tiles_n = (d->N + BN - 1) / BN;
  a.alpha = d->alpha; a.beta = d->beta; a.act = d->act; a.mode = d->mode; a.tri = d->tri;
  a.kin = d->kin; a.a_sk = d->a_sk; a.b_sk = d->b_sk; a.kin_bps = 0;
  a.stamps = g_4w_stamps;
  a.queue = nullptr;
  a.tri_group = (d->tri == 1 || d->tri == 2)
                    ? g4w_tri_group_env((long long)d->batch1 * d->batch2 * d->K * d->N * 2) : 0;
  a.ksplit = 1;
  a.ws = nullptr;
  a.nbatch = 0;
  // split contraction index (the token mixer's weight gradient): K-contiguous operands, whole 64-deep K-tiles per
  // kin block, gemm4w only
  if (d->kin && (d->kin < 0 || d->kin % 64 || d->K % d->kin || d->a_t || d->b_t || d->tri == 1 || d->tri == 2 ||
                 d->a_sk % 8 || d->b_sk % 8))
    return -9;
  const int batch = d->batch1 * d->batch2;
  hipError_t e;
  // tri 3 on gemm4w (with a split contraction index: the causal mixer weight gradient, its own instantiation):
  // lower-triangle tiles only, always through the split-K slabs -- their fold masks the strictly upper elements of
  // the diagonal tiles (fp32 outputs)
  const bool tri3_ok = d->tri != 3 || (d->kin && d->out_f32 && d->act == 0 && d->mode == 0 && !d->R && !d->Zout &&
                                       d->K % 128 == 0 && d->N % 4 == 0 && d->ldc % 4 == 0 &&
                                       (batch == 1 || (d->c_s1 % 4 == 0 && d->c_s2 % 4 == 0)));
  // an fp32 output's bf16 copy (Zout) comes from gemm4w's direct epilogue (no activation, no split-K)
  const bool zcopy_ok = !(d->out_f32 && d->Zout) || (d->act == 0 && d->mode == 0 && d->a_t == 0);
  if (d->K % 64 == 0 && tri3_ok && zcopy_ok && (d->a_t == 0 || d->M % 8 == 0) && (d->b_t == 0 || d->N % 8 == 0)) {
    // split-K for fp32 products with few output tiles (the weight gradients): the persistent kernel runs
    // ceil(tiles * ks / 256) rounds of K / ks each; a split costs a deterministic fold over ks fp32 slabs. Pick the
    // ks of least modelled time (1.25 us per 64-deep K-tile of a tile, ~5 TB/s for the fold), workspace <= 1 GiB.
    const long long tm = (d->M + 255) / 256, tn = (d->N + 255) / 256;
    const long long big_tiles = (d->tri == 3 ? tm * (tm + 1) / 2 : tm * tn) * batch;
    int ks = 1;
    // batched products too (the per-head group-linear weight gradients: few tiles per batch); C batch strides must
    // keep 16-byte alignment for the fold. The folds index float4s of rows (m = e / N, e < M * N / 4): N and ldc
    // must be multiples of 4 (the entry checks already require 8; restated here so the fold's own contract is local)
    // (also long-K products with many tiles: the logits weight gradient, 8 x 197 tiles of 2048 K-tiles each, ran 7
    // rounds of which the last held 40 of 256 CUs -- split 4 ways it runs 25 rounds and one 0.4 GB fold)
    if ((big_tiles < 512 || d->tri == 3 || d->K >= 32768) && d->out_f32 && !d->R && !d->Zout && !d->act &&
        d->mode == 0 &&
        (d->tri == 0 || d->tri == 3) && d->N % 4 == 0 && d->ldc % 4 == 0 &&
        (batch == 1 || (d->c_s1 % 4 == 0 && d->c_s2 % 4 == 0))) {
      const double per_k = 1.25 / 64.0;   // us per K element of one tile
      double best = 1e300;
      for (int c = d->tri == 3 ? 2 : 1; c <= 16; c *= 2) {
        if (d->K % (64 * c) || (c > 2 && d->K / c < 512) || (size_t)c * batch * d->M * d->N * 4 > (2ull << 30) ||
            (d->kin && (d->K / c) % d->kin))   // split-K slabs of a split index start on kin-block boundaries
          continue;
        const double rounds = (double)((big_tiles * c + 255) / 256);
        const double t = rounds * (d->K / c) * per_k +
                         (c > 1 ? (double)(c + (d->beta != 0.f ? 2 : 1)) * batch * d->M * d->N * 4.0 / 5e6 : 0.0);
        if (t < best * 0.98) { best = t; ks = c; }
      }
      // (doubling ks so that one-tile-per-block products give the queue two items per block lost on the
      // GPT-Neo-1.3B step, 148.9-149.1k vs 150.2k tokens/s: removed in round 6, profiles/r5_summary.md)
      if (ks > 1) {
        a.ws = splitk_workspace((size_t)ks * batch * d->M * d->N * sizeof(float));
        if (!a.ws) ks = 1;
      }
    }
    if (d->tri == 3 && ks < 2) goto fallback;   // (no workspace: the 128x128 kernel masks in its epilogue)
    a.ksplit = ks;
    a.kin_bps = d->kin ? d->K / ks / d->kin : 0;
    // the queue: products whose every tile has >= 3 K-tiles (the next tile is dequeued in a tile's first K-tile
    // and the DMA cursor needs it by the end of K-tile nk - 3), more tiles than one per block, no stamps. Dense, or
    // triangular A (the token mixer, OBST_G4W_QUEUE_TRI): tri 1 tile rows span min(K, m0 + 256), tri 2 K - m0 --
    // the shortest is the first / last tile row
    const bool tri_nk3 = (d->tri == 1 && (d->K < 256 ? d->K : 256) >= 192) ||
                         (d->tri == 2 && d->K - (tm - 1) * 256 >= 192);
    if (g4w_queue_env() && (d->tri == 0 || (tri_nk3 && g4w_queue_tri_env())) && !d->kin && d->K / ks >= 192 &&
        !g_4w_stamps && tm * tn * batch * ks > 256)
      a.queue = g4w_queue_slot(stream);
    if (a.queue) ++g_4w_queue_calls;
    e = gemm4w_launch(&a, d->a_t, d->b_t, d->out_f32, batch, stream);
    if (e == hipSuccess && d->out_f32 && a.ksplit > 1) {
      const long long mn = (long long)a.M * a.N;
      if (batch == 1)
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3(2048), dim3(256), 0, stream, reinterpret_cast<float*>(a.C),
                           a.ws, mn, a.ldc, a.N, a.ksplit, a.beta, (int)(d->tri == 3));
      else
        hipLaunchKernelGGL(splitk_reduce_batched_kernel, dim3(2048), dim3(256), 0, stream,
                           reinterpret_cast<float*>(a.C), a.ws, mn, a.ldc, a.N, a.ksplit, a.beta, batch, a.nb2,
                           a.c_s1, a.c_s2, (int)(d->tri == 3));
      e = hipGetLastError();
    }
    ++g_4w_calls;
    return e == hipSuccess ? 0 : (int)e;
  }
fallback:
  if (d->kin) return -9;
  a.ksplit = 1;
  a.ws = nullptr;
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
