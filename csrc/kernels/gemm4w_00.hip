// gemm4w kernels for A_T = 0, B_T = 0 (kernel: gemm4w.h)
#include "gemm4w.h"

OBST_GEMM4W_TU(0, 0)
