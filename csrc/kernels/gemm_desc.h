// Host-side GEMM descriptor of the MFMA kernels (gemm.hip, gemm4w.h); the ctypes mirror is GemmDesc in
// homebrewnlp_mtf_amd/ops/_lib.py. (tools/lab/blaslt.cpp, the vendor-library A/B harness, takes the same descriptor.)
#pragma once
struct ObstGemmDesc {
  const void* A; const void* B; void* C; const void* R; void* Zout; const void* Zin;
  long long lda, ldb, ldc;
  long long a_s1, a_s2, b_s1, b_s2, c_s1, c_s2;
  int M, N, K, batch1, batch2;
  int a_t, b_t, out_f32, act, mode;
  float alpha, beta;
  int tri;
  // split contraction index (gemm4w, K-contiguous operands only): k -> (k / kin) * sk + k % kin, i.e.
  // K = (outer, inner) with inner blocks of kin contiguous elements and an outer stride a_sk / b_sk (0: plain K)
  int kin;
  long long a_sk, b_sk;
};

// (tools/lab only) the same products through the vendor GEMM library: 0 done, 1 not eligible, < 0 library error
int obst_blaslt_gemm(const ObstGemmDesc* d, hipStream_t stream);
