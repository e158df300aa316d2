#!/usr/bin/env python3
"""Runs one GEMM shape a few times (for rocprofv3 --pmc counter collection): gemm_one.py M N K a_t b_t [f32]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

M, N, K, at, bt = (int(x) for x in sys.argv[1:6])
f32 = len(sys.argv) > 6 and sys.argv[6] == "f32"
dev = torch.device("cuda")
A = (torch.rand(M * K, device=dev) * 2 - 1).to(torch.bfloat16)
B = (torch.rand(N * K, device=dev) * 2 - 1).to(torch.bfloat16)
C = torch.zeros(M * N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
ops = (raw.Operand(A, at, K if at == 0 else M), raw.Operand(B, bt, K if bt == 0 else N), raw.Operand(C, 0, N))
for _ in range(int(os.environ.get("REPS", 3))):
    raw.gemm(*ops, M, N, K, beta=1.0 if f32 else 0.0)
torch.cuda.synchronize()
