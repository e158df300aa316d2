// gemm4w kernels for A_T = 1, B_T = 1 (kernel: gemm4w.h)
#include "gemm4w.h"

OBST_GEMM4W_TU(1, 1)
