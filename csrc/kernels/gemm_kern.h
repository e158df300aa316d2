// Shared by the MFMA GEMM translation units (gemm.hip: the 128x128 kernel and the dispatcher; gemm4w*.hip: the
// one-wave-per-SIMD 256x256 kernel).
#pragma once
#include "common.h"

namespace gemmk {   // external linkage: gemm.hip hands a filled GemmArgs to gemm_pp.hip
struct GemmArgs {
  const bf16_t* A; const bf16_t* B; void* C;
  const void* R;          // residual added before the activation (same dtype/layout as C) or null
  bf16_t* Zout;           // bf16 C: pre-activation output; fp32 C: bf16 copy of the output (layout of C; gemm4w
                          // row-layout direct epilogue and the 128x128 kernel only) or null
  const bf16_t* Zin;      // saved pre-activation for the activation-backward epilogue (layout of C)
  long long lda, ldb, ldc;
  long long a_s1, a_s2, b_s1, b_s2, c_s1, c_s2;
  int M, N, K, nb2;
  int tiles_m, tiles_n;
  float alpha, beta;      // beta: fp32 output only, C = alpha*acc + beta*C_old (gradient accumulation)
  int act, mode;          // mode 0: out = act(alpha*acc + R); mode 1: out = (alpha*acc + R) * act'(Zin)
  int tri;                // 0 dense; 1 A lower-triangular (A[m][k] = 0 for k > m); 2 A upper-triangular (k < m);
                          // 3 only C[m][n] with n <= m is produced (strictly-upper outputs get no contribution)
  int ksplit;             // gemm4w: K split into ksplit slabs; partial tiles go to `ws` [batch][split][M][N]
  float* ws;              // split-K workspace (fp32), summed into C by splitk_reduce_kernel
  int kin;                // gemm4w: split contraction index, see ObstGemmDesc (0: plain K)
  long long a_sk, b_sk;
  int kin_bps;            // kin blocks per split-K slab (K / ksplit / kin; slabs start on block boundaries)
  int nbatch;             // gemm4w: batches x splits (the grid is one block per CU)
  unsigned long long* stamps;   // gemm4w diagnostics: per-block timestamps (null: off)
  unsigned* queue;        // gemm4w dynamic tile queue: 8 per-XCD counters zeroed before the launch (null: static)
  int tri_group;          // gemm4w tri 1 / 2: batches per tile-row group of the work order (0: tile rows slowest)
};
}  // namespace gemmk

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = 128 * 64 * 2;  // one operand tile, either image

using gemmk::GemmArgs;

__device__ __forceinline__ int kswz(int k) { return ((k & 3) << 1) | (((k >> 3) & 1) << 3); }

// --- LDS -> MFMA fragment (8 consecutive k of one row/col) -------------------------------------------------------
template <int T>
__device__ __forceinline__ bf16x8_t read_frag(const char* lds, int rbase, int kk, int lane) {
  if (T == 0) {
    const int r = rbase + (lane & 15);
    const int c = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8_t*>(lds + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
  } else {
    const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
    const int col = rbase + 4 * pp;
    const int c = col >> 3;
    const int k0 = kk * 32 + 8 * g + q;
    const int k1 = k0 + 4;
    const int off0 = k0 * 256 + ((c ^ kswz(k0)) << 4) + ((pp & 1) << 3);
    const int off1 = k1 * 256 + ((c ^ kswz(k1)) << 4) + ((pp & 1) << 3);
    s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, lds + off0));
    s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, lds + off1));
    s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}


// fused epilogue of one lane's 4 consecutive outputs C[m][n..n+3] at element index idx (layout of C)
template <bool OUT_F32>
__device__ __forceinline__ void epilogue_store(const GemmArgs& p, long long idx, float (&v)[4]) {
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
    if (p.R) {
      uint2 r = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(p.R) + idx);
      v[0] += bf2f(r.x & 0xffff); v[1] += bf2f(r.x >> 16); v[2] += bf2f(r.y & 0xffff); v[3] += bf2f(r.y >> 16);
    }
    if (p.mode == 1) {
      uint2 z = *reinterpret_cast<const uint2*>(p.Zin + idx);
      v[0] *= act_grad(p.act, bf2f(z.x & 0xffff)); v[1] *= act_grad(p.act, bf2f(z.x >> 16));
      v[2] *= act_grad(p.act, bf2f(z.y & 0xffff)); v[3] *= act_grad(p.act, bf2f(z.y >> 16));
    } else {
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

// the same epilogue for 8 consecutive outputs C[m][n..n+7] (16-byte loads / stores; n % 8 == 0, idx % 8 == 0)
template <bool OUT_F32>
__device__ __forceinline__ void epilogue_store8(const GemmArgs& p, long long idx, float (&v)[8]) {
  if (OUT_F32) {
    float* C = reinterpret_cast<float*>(p.C) + idx;
    if (p.beta != 0.f) {
      const float4 o0 = reinterpret_cast<const float4*>(C)[0], o1 = reinterpret_cast<const float4*>(C)[1];
      v[0] += p.beta * o0.x; v[1] += p.beta * o0.y; v[2] += p.beta * o0.z; v[3] += p.beta * o0.w;
      v[4] += p.beta * o1.x; v[5] += p.beta * o1.y; v[6] += p.beta * o1.z; v[7] += p.beta * o1.w;
    }
    if (p.R) {
      const float4* R = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.R) + idx);
      const float4 r0 = R[0], r1 = R[1];
      v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w; v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
    }
    if (p.act) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = act_fwd(p.act, v[t]);
    }
    reinterpret_cast<float4*>(C)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(C)[1] = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    if (p.R) {
      const uint4 r = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(p.R) + idx);
      const uint32_t rw[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) { v[2 * t] += bf2f(rw[t] & 0xffff); v[2 * t + 1] += bf2f(rw[t] >> 16); }
    }
    if (p.mode == 1) {
      const uint4 z = *reinterpret_cast<const uint4*>(p.Zin + idx);
      const uint32_t zw[4] = {z.x, z.y, z.z, z.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        v[2 * t] *= act_grad(p.act, bf2f(zw[t] & 0xffff));
        v[2 * t + 1] *= act_grad(p.act, bf2f(zw[t] >> 16));
      }
    } else {
      if (p.Zout)
        *reinterpret_cast<uint4*>(p.Zout + idx) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                                             pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
      if (p.act) {
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = act_fwd(p.act, v[t]);
      }
    }
    *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(p.C) + idx) =
        make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
  }
}

// activation of 8 values with ONE inlined switch: a rotation loop (v[0] transformed, the array shifted) keeps every
// register index static -- for epilogues instantiated many times per kernel (instruction-cache budget)
__device__ __forceinline__ void act8_fwd(int act, float (&v)[8]) {
#pragma unroll 1
  for (int t = 0; t < 8; ++t) {
    const float x = act_fwd(act, v[0]);
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4]; v[4] = v[5]; v[5] = v[6]; v[6] = v[7]; v[7] = x;
  }
}
__device__ __forceinline__ void act8_grad_mul(int act, float (&v)[8], float (&z)[8]) {
#pragma unroll 1
  for (int t = 0; t < 8; ++t) {
    const float x = v[0] * act_grad(act, z[0]);
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4]; v[4] = v[5]; v[5] = v[6]; v[6] = v[7]; v[7] = x;
    z[0] = z[1]; z[1] = z[2]; z[2] = z[3]; z[3] = z[4]; z[4] = z[5]; z[5] = z[6]; z[6] = z[7];
  }
}

// epilogue_store8 with the activations applied through act8_*: compact code for the activation GEMMs
template <bool OUT_F32>
__device__ __forceinline__ void epilogue_store8r(const GemmArgs& p, long long idx, float (&v)[8]) {
  if (OUT_F32) {
    float* C = reinterpret_cast<float*>(p.C) + idx;
    if (p.beta != 0.f) {
      const float4 o0 = reinterpret_cast<const float4*>(C)[0], o1 = reinterpret_cast<const float4*>(C)[1];
      v[0] += p.beta * o0.x; v[1] += p.beta * o0.y; v[2] += p.beta * o0.z; v[3] += p.beta * o0.w;
      v[4] += p.beta * o1.x; v[5] += p.beta * o1.y; v[6] += p.beta * o1.z; v[7] += p.beta * o1.w;
    }
    if (p.R) {
      const float4* R = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.R) + idx);
      const float4 r0 = R[0], r1 = R[1];
      v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w; v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
    }
    if (p.act) act8_fwd(p.act, v);
    reinterpret_cast<float4*>(C)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(C)[1] = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    if (p.R) {
      const uint4 r = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(p.R) + idx);
      const uint32_t rw[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) { v[2 * t] += bf2f(rw[t] & 0xffff); v[2 * t + 1] += bf2f(rw[t] >> 16); }
    }
    if (p.mode == 1) {
      const uint4 zz = *reinterpret_cast<const uint4*>(p.Zin + idx);
      const uint32_t zw[4] = {zz.x, zz.y, zz.z, zz.w};
      float z[8];
#pragma unroll
      for (int t = 0; t < 4; ++t) { z[2 * t] = bf2f(zw[t] & 0xffff); z[2 * t + 1] = bf2f(zw[t] >> 16); }
      act8_grad_mul(p.act, v, z);
    } else {
      if (p.Zout)
        *reinterpret_cast<uint4*>(p.Zout + idx) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                                             pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
      if (p.act) act8_fwd(p.act, v);
    }
    *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(p.C) + idx) =
        make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
  }
}

}  // namespace

// the one-wave-per-SIMD 256x256 kernel (gemm4w.hip) for a GemmArgs filled by obst_gemm (ksplit / ws set)
hipError_t gemm4w_launch(const gemmk::GemmArgs* a, int a_t, int b_t, int out_f32, int batch, hipStream_t stream);
