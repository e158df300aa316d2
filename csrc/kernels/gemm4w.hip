// Dispatch of the one-wave-per-SIMD 256x256 GEMM (gemm4w.h) over the operand layouts; the instantiations live in
// gemm4w_<a_t><b_t>.hip.
#include "gemm_kern.h"

hipError_t gemm4w_launch_00(const gemmk::GemmArgs* a, int out_f32, int batch, hipStream_t stream);
hipError_t gemm4w_launch_01(const gemmk::GemmArgs* a, int out_f32, int batch, hipStream_t stream);
hipError_t gemm4w_launch_10(const gemmk::GemmArgs* a, int out_f32, int batch, hipStream_t stream);
hipError_t gemm4w_launch_11(const gemmk::GemmArgs* a, int out_f32, int batch, hipStream_t stream);

hipError_t gemm4w_launch(const gemmk::GemmArgs* a, int a_t, int b_t, int out_f32, int batch, hipStream_t stream) {
  if (a_t == 0 && b_t == 0) return gemm4w_launch_00(a, out_f32, batch, stream);
  if (a_t == 0 && b_t == 1) return gemm4w_launch_01(a, out_f32, batch, stream);
  if (a_t == 1 && b_t == 0) return gemm4w_launch_10(a, out_f32, batch, stream);
  return gemm4w_launch_11(a, out_f32, batch, stream);
}

