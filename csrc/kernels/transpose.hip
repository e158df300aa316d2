// Batched bf16 2-D transpose Y[b][c][r] = X[b][r][c] through a 64x64 LDS tile.
// Used to put GEMM operands into the K-contiguous form the MFMA kernels read fastest (ds_read_b128 fragments instead
// of ds_read_b64_tr_b16 pairs, bench: 1325 vs 875-1035 TFLOP/s at 8192^3): the transposed bf16 weight copy for the
// forward GEMM and the token-major activations / output gradients of the weight-gradient GEMM.
// Loads and stores are 16 B per lane (8 elements); the LDS tile is padded by 8 elements per row (bank spread).
#include "common.h"

namespace {

constexpr int TT = 64, PADW = TT + 8, NTH = 256;

__global__ __launch_bounds__(NTH) void transpose_kernel(const bf16_t* __restrict__ X, bf16_t* __restrict__ Y,
                                                        long long rows, long long cols, long long ldx, long long ldy,
                                                        long long sx, long long sy) {
  __shared__ bf16_t tile[TT][PADW];
  const long long r0 = (long long)blockIdx.y * TT, c0 = (long long)blockIdx.x * TT;
  const bf16_t* Xb = X + blockIdx.z * sx;
  bf16_t* Yb = Y + blockIdx.z * sy;
  const int tid = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int q = tid + it * NTH;         // 512 chunks of 8 elements: row q>>3, chunk q&7
    const int r = q >> 3, cc = (q & 7) * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + r < rows && c0 + cc < cols) v = *reinterpret_cast<const uint4*>(Xb + (r0 + r) * ldx + c0 + cc);
    *reinterpret_cast<uint4*>(&tile[r][cc]) = v;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int q = tid + it * NTH;         // output row (= input column) q>>3, 8 input rows from (q&7)*8
    const int c = q >> 3, rr = (q & 7) * 8;
    if (c0 + c < cols && r0 + rr < rows) {
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = (uint32_t)tile[rr + 2 * j][c] | ((uint32_t)tile[rr + 2 * j + 1][c] << 16);
      *reinterpret_cast<uint4*>(Yb + (c0 + c) * ldy + r0 + rr) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

// Y[b][r][c] = X[b][r][c] between two strided 2-D layouts, 16 B per lane: the row interleave of the stacked
// q / k / v weights ([3][K][N] -> [K][3N], the data-gradient GEMM's concatenated operand)
__global__ __launch_bounds__(NTH) void copy2d_kernel(const bf16_t* __restrict__ X, bf16_t* __restrict__ Y,
                                                     long long rows, long long cv, long long ldx, long long ldy,
                                                     long long sx, long long sy) {
  const long long per = rows * cv;
  for (long long i = (long long)blockIdx.x * NTH + threadIdx.x; i < per; i += (long long)gridDim.x * NTH) {
    const long long r = i / cv, c = (i - r * cv) * 8;
    *reinterpret_cast<uint4*>(Y + blockIdx.y * sy + r * ldy + c) =
        *reinterpret_cast<const uint4*>(X + blockIdx.y * sx + r * ldx + c);
  }
}

// Y[b][r][c] = c <= r ? X[b][r][c] : 0 over square S x S slices (the causal token mixer's masked weight), 8
// elements per lane
__global__ __launch_bounds__(NTH) void tril_kernel(const bf16_t* __restrict__ X, bf16_t* __restrict__ Y, long long S,
                                                   long long nvec) {
  for (long long v = (long long)blockIdx.x * NTH + threadIdx.x; v < nvec; v += (long long)gridDim.x * NTH) {
    const long long e = v * 8, r = (e / S) % S, c = e % S;
    uint4 u = *reinterpret_cast<const uint4*>(X + e);
    if (c + 7 > r) {
      uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (c + 2 * j > r) w[j] &= 0xffff0000u;
        if (c + 2 * j + 1 > r) w[j] &= 0x0000ffffu;
      }
      u = make_uint4(w[0], w[1], w[2], w[3]);
    }
    *reinterpret_cast<uint4*>(Y + e) = u;
  }
}

}  // namespace

// rows/cols of X; ldx/ldy row strides (elements); sx/sy batch strides. rows, cols, ldx, ldy multiples of 8.
OBST_API int obst_transpose(const void* X, void* Y, long long rows, long long cols, long long ldx, long long ldy,
                            int batch, long long sx, long long sy, hipStream_t st) {
  if (rows <= 0 || cols <= 0 || batch <= 0) return -1;
  if (rows % 8 || cols % 8 || ldx % 8 || ldy % 8 || sx % 8 || sy % 8) return -2;
  if ((((uintptr_t)X) | ((uintptr_t)Y)) & 15) return -3;
  dim3 grid((unsigned)((cols + TT - 1) / TT), (unsigned)((rows + TT - 1) / TT), (unsigned)batch);
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(NTH), 0, st, (const bf16_t*)X, (bf16_t*)Y, rows, cols, ldx, ldy,
                     sx, sy);
  return (int)hipGetLastError();
}

// Y[b][r][c] = X[b][r][c]; cols, strides multiples of 8
OBST_API int obst_copy2d(const void* X, void* Y, long long rows, long long cols, long long ldx, long long ldy,
                         int batch, long long sx, long long sy, hipStream_t st) {
  if (rows <= 0 || cols <= 0 || batch <= 0) return -1;
  if (cols % 8 || ldx % 8 || ldy % 8 || sx % 8 || sy % 8) return -2;
  if ((((uintptr_t)X) | ((uintptr_t)Y)) & 15) return -3;
  const long long per = rows * (cols / 8);
  const unsigned gx = (unsigned)(per / NTH + 1 < 2048 ? per / NTH + 1 : 2048);
  hipLaunchKernelGGL(copy2d_kernel, dim3(gx, (unsigned)batch), dim3(NTH), 0, st, (const bf16_t*)X, (bf16_t*)Y, rows,
                     cols / 8, ldx, ldy, sx, sy);
  return (int)hipGetLastError();
}

// Y = tril(X) for `batch` contiguous S x S bf16 slices (S % 8 == 0)
OBST_API int obst_tril(const void* X, void* Y, long long S, long long batch, hipStream_t st) {
  if (S <= 0 || batch <= 0 || S % 8) return -1;
  if ((((uintptr_t)X) | ((uintptr_t)Y)) & 15) return -3;
  const long long nvec = batch * S * S / 8;
  const unsigned g = (unsigned)(nvec / NTH + 1 < 4096 ? nvec / NTH + 1 : 4096);
  hipLaunchKernelGGL(tril_kernel, dim3(g), dim3(NTH), 0, st, (const bf16_t*)X, (bf16_t*)Y, S, nvec);
  return (int)hipGetLastError();
}

// bytes of zeros (the flat gradient buffer at the start of a step): the runtime's fill, not a framework kernel
OBST_API int obst_zero(void* p, long long bytes, hipStream_t st) {
  return (int)hipMemsetAsync(p, 0, (size_t)bytes, st);
}
