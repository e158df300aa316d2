// Shared helpers for the gfx950 (CDNA4, MI355X) kernel library.
// Wave = 64 lanes; bf16 is carried as raw 16-bit patterns and converted in registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define OBST_API extern "C" __attribute__((visibility("default")))

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;     // MFMA 16x16x32 A/B fragment
typedef __attribute__((ext_vector_type(4))) float f32x4_t;       // MFMA 16x16 accumulator
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(8))) short s16x8_t;

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// LDS-DMA of 16 bytes per lane (1 KiB per wave-instruction) issued from inline asm: the compiler then does not know
// an LDS write is in flight, so it inserts no conservative `s_waitcnt vmcnt(0)` in front of every later LDS read
// (it cannot prove the DMA's destination buffer differs from the one being read, and that wait collapses any
// multi-stage pipeline). The price: every consumer must wait explicitly -- `vm_wait<N>()` before the barrier that
// publishes a staged tile (a fence/__syncthreads alone is not enough, the compiler believes nothing is pending).
// M0 is written here and used by no compiler-generated instruction in kernels that stage only through this helper.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds16_asm(const void* g, const void* lds_wave_base) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory", "m0");
}
// 4 bytes per lane (256 B per wave-instruction, lane-linear in LDS), same contract as glds16_asm
__device__ __forceinline__ void glds4_asm(const void* g, const void* lds_wave_base) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g), "s"(m0) : "memory", "m0");
}
#pragma clang diagnostic pop

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// round-to-nearest-even; NaN stays NaN (MI355X_MICROARCH correctness table: plain cast keeps NaN)
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}

typedef __bf16 obst_bf16x2_t __attribute__((ext_vector_type(2)));
typedef float obst_f32x2_t __attribute__((ext_vector_type(2)));
// one v_cvt_pk_bf16_f32 (two scalar conversions + shift + or were four instructions)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((obst_f32x2_t{lo, hi}), obst_bf16x2_t));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x = NW*64; `red` must hold NW floats of LDS.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += red[i];
  return t;
}

// ---- activation functions shared by the GEMM epilogue and the elementwise kernels -------------------------------
// Semantics follow the reference activations (src/model/activation.py): gelu is the tanh approximation,
// lecun_tanh = tanh(x) + 0.1x, mish = x*tanh(softplus(x)), softsign = x/(1+|x|).
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_SILU = 3, ACT_SIGMOID = 4, ACT_TANH = 5,
                 ACT_LECUN_TANH = 6, ACT_MISH = 7, ACT_SOFTSIGN = 8, ACT_EXP = 9 };

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float softplusf_(float x) { return x > 20.f ? x : log1pf(__expf(x)); }

// tanh-form gelu through the identity 0.5 (1 + tanh(u)) = sigmoid(2u): one v_exp_f32 + one reciprocal instead of
// the libm tanhf (~30 VALU with range branches) -- the elementwise gelu passes were VALU-bound
__device__ __forceinline__ float gelu_s(float x) {   // sigmoid(2u), u = k0 (x + k1 x^3)
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  // v_exp_f32 (2^x) and v_rcp_f32 directly: __frcp_rn is a correctly rounded reciprocal (a Newton sequence), and
  // the gelu epilogues of the one-wave-per-SIMD GEMM are issue-bound on these instructions
  const float t = -2.f * k0 * 1.4426950408889634f * (x + k1 * x * x * x);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(t));
}

__device__ __forceinline__ float act_fwd(int act, float x) {
  switch (act) {
    case ACT_RELU: return fmaxf(x, 0.f);
    case ACT_GELU: return x * gelu_s(x);
    case ACT_SILU: return x * sigmoidf_(x);
    case ACT_SIGMOID: return sigmoidf_(x);
    case ACT_TANH: return tanhf(x);
    case ACT_LECUN_TANH: return tanhf(x) + 0.1f * x;
    case ACT_MISH: return x * tanhf(softplusf_(x));
    case ACT_SOFTSIGN: return x / (1.f + fabsf(x));
    case ACT_EXP: return __expf(x);
    default: return x;
  }
}

// d act(x) / dx
__device__ __forceinline__ float act_grad(int act, float x) {
  switch (act) {
    case ACT_RELU: return x > 0.f ? 1.f : 0.f;
    case ACT_GELU: {   // d/dx x s(2u) = s + 2 x s (1 - s) u'(x), s = sigmoid(2u) = 0.5 (1 + tanh u)
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      const float s = gelu_s(x);
      return s + 2.f * x * s * (1.f - s) * k0 * (1.f + 3.f * k1 * x * x);
    }
    case ACT_SILU: { float s = sigmoidf_(x); return s * (1.f + x * (1.f - s)); }
    case ACT_SIGMOID: { float s = sigmoidf_(x); return s * (1.f - s); }
    case ACT_TANH: { float t = tanhf(x); return 1.f - t * t; }
    case ACT_LECUN_TANH: { float t = tanhf(x); return 1.1f - t * t; }
    case ACT_MISH: {
      float sp = softplusf_(x), tsp = tanhf(sp), s = sigmoidf_(x);
      return tsp + x * (1.f - tsp * tsp) * s;
    }
    case ACT_SOFTSIGN: { float d = 1.f + fabsf(x); return 1.f / (d * d); }
    case ACT_EXP: return __expf(x);
    default: return 1.f;
  }
}

static inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }
