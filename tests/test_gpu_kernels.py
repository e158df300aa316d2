"""HIP kernel numerics vs the PyTorch fp32 oracle of the same op (ops/raw.py CPU path).

Every test builds inputs on the CPU, runs the CPU oracle, copies the inputs to the GPU, runs the gfx950 kernel
through the same ``raw`` entry point, and compares.
"""
import math

import pytest
import torch

from homebrewnlp_mtf_amd.ops import _lib as L
from homebrewnlp_mtf_amd.ops import raw
from homebrewnlp_mtf_amd.ops import functional as F

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _close(gpu, ref, atol, rtol, what=""):
    g = gpu.float().cpu()
    r = ref.float()
    err = (g - r).abs()
    tol = atol + rtol * r.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{what}: {bad}/{r.numel()} out of tolerance, max err {err.max().item():.4g}"




def g4w_calls() -> int:
    """dispatches the hand-written one-wave-per-SIMD gemm4w kernel has taken so far"""
    import ctypes
    f = L.lib().obst_gemm4w_calls
    f.restype = ctypes.c_longlong
    return int(f())


# ----------------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("a_t,b_t", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (200, 136, 72), (512, 384, 256), (64, 8, 8)])
def test_gemm_layouts(cuda, a_t, b_t, M, N, K):
    torch.manual_seed(M + N + K + 10 * a_t + b_t)
    A = (torch.randn(M * K) * 0.5).to(BF)
    B = (torch.randn(N * K) * 0.5).to(BF)
    lda = K if a_t == 0 else M
    ldb = K if b_t == 0 else N
    C = torch.zeros(M * N, dtype=BF)
    raw.gemm(raw.Operand(A, a_t, lda), raw.Operand(B, b_t, ldb), raw.Operand(C, 0, N), M, N, K)
    Cg = torch.zeros(M * N, dtype=BF, device=cuda)
    raw.gemm(raw.Operand(A.to(cuda), a_t, lda), raw.Operand(B.to(cuda), b_t, ldb), raw.Operand(Cg, 0, N), M, N, K)
    torch.cuda.synchronize()
    _close(Cg, C, 2e-2 * math.sqrt(K / 64), 2e-2, f"gemm {a_t}{b_t} {M}x{N}x{K}")


def test_gemm_identity_asymmetric(cuda):
    """A = I with an asymmetric B catches a transposed C write (cdna guide §3)."""
    n = 128
    A = torch.eye(n).to(BF)
    B = torch.arange(n * n, dtype=torch.float32).view(n, n).remainder(97).to(BF)  # stored [K][N]
    Cg = torch.zeros(n * n, dtype=BF, device=cuda)
    raw.gemm(raw.Operand(A.reshape(-1).to(cuda), 0, n), raw.Operand(B.reshape(-1).to(cuda), 1, n),
             raw.Operand(Cg, 0, n), n, n, n)
    torch.cuda.synchronize()
    assert torch.equal(Cg.view(n, n).cpu(), B)


def test_gemm_batched_epilogues(cuda):
    torch.manual_seed(3)
    H, M, K, N = 3, 96, 64, 40
    A = (torch.randn(M, H, K) * 0.5).to(BF)            # [M][H][K] -> batch stride K, ld H*K
    B = (torch.randn(H, K, N) * 0.5).to(BF)            # [H][K][N]
    R = (torch.randn(M, H, N) * 0.5).to(BF)
    outs = {}
    for dev in ("cpu", cuda):
        C = torch.zeros(M, H, N, dtype=BF, device=dev)
        Z = torch.zeros(M, H, N, dtype=BF, device=dev)
        raw.gemm(raw.Operand(A.to(dev), 0, H * K, K), raw.Operand(B.to(dev), 1, N, K * N),
                 raw.Operand(C, 0, H * N, N), M, N, K, batch=(H, 1), act="gelu", R=R.to(dev), Zout=Z)
        D = torch.zeros(M, H, N, dtype=BF, device=dev)   # activation-backward epilogue: (acc + R) * gelu'(Z)
        raw.gemm(raw.Operand(A.to(dev), 0, H * K, K), raw.Operand(B.to(dev), 1, N, K * N),
                 raw.Operand(D, 0, H * N, N), M, N, K, batch=(H, 1), act="gelu", act_bwd=True, Zin=Z, R=R.to(dev))
        G = torch.ones(H, K, N, dtype=torch.float32, device=dev)   # fp32 accumulate (beta = 1)
        raw.gemm(raw.Operand(A.to(dev), 1, H * K, K), raw.Operand(R.to(dev), 1, H * N, N),
                 raw.Operand(G, 0, N, K * N), K, N, M, batch=(H, 1), beta=1.0)
        C2 = torch.zeros(M, H, N, dtype=BF, device=dev)   # activation + pre-activation output, no residual
        Z2 = torch.zeros(M, H, N, dtype=BF, device=dev)
        raw.gemm(raw.Operand(A.to(dev), 0, H * K, K), raw.Operand(B.to(dev), 1, N, K * N),
                 raw.Operand(C2, 0, H * N, N), M, N, K, batch=(H, 1), act="gelu", Zout=Z2)
        D2 = torch.zeros(M, H, N, dtype=BF, device=dev)   # activation backward without residual
        raw.gemm(raw.Operand(A.to(dev), 0, H * K, K), raw.Operand(B.to(dev), 1, N, K * N),
                 raw.Operand(D2, 0, H * N, N), M, N, K, batch=(H, 1), act="gelu", act_bwd=True, Zin=Z)
        outs[str(dev)] = (C, Z, D, G, C2, Z2, D2)
    torch.cuda.synchronize()
    for name, g, c in zip(["C", "Z", "D", "G", "C2", "Z2", "D2"], outs[str(cuda)], outs["cpu"]):
        _close(g, c, 5e-2, 3e-2, f"batched epilogue {name}")


@pytest.mark.parametrize("case", ["residual", "f32_accumulate", "shared_A_batch", "shared_A_batch_bt0",
                                  "two_level_batch"])
def test_gemm_plain_paths(cuda, case):
    """the plain-GEMM shapes the model issues (residual input, fp32 accumulate, q/k/v batch over one input)"""
    torch.manual_seed(5)
    M, K, N, H = 256, 192, 136, 3
    outs = {}
    A = (torch.randn(M * H * K) * 0.5).to(BF)
    B = (torch.randn(H * K * N) * 0.5).to(BF)
    R = (torch.randn(M * H * N) * 0.5).to(BF)
    for dev in ("cpu", cuda):
        a, b, r = A.to(dev), B.to(dev), R.to(dev)
        if case == "residual":
            C = torch.zeros(M * N, dtype=BF, device=dev)
            raw.gemm(raw.Operand(a, 0, K), raw.Operand(b, 1, N), raw.Operand(C, 0, N), M, N, K, R=r)
        elif case == "f32_accumulate":   # weight gradient: C[K][N] += A[M][K]^T B[M][N]
            C = torch.ones(K * N, dtype=torch.float32, device=dev)
            raw.gemm(raw.Operand(a, 1, K), raw.Operand(r, 1, N), raw.Operand(C, 0, N), K, N, M, beta=1.0)
        elif case == "shared_A_batch":   # out[j] = A · B_j  (A batch stride 0)
            C = torch.zeros(H * M * N, dtype=BF, device=dev)
            raw.gemm(raw.Operand(a, 0, K, 0), raw.Operand(b, 1, N, K * N), raw.Operand(C, 0, N, M * N), M, N, K,
                     batch=(H, 1))
        elif case == "shared_A_batch_bt0":
            # broadcast A, K-contiguous B, interleaved C columns as in the k|q|v projection
            C = torch.zeros(M * H * N, dtype=BF, device=dev)
            raw.gemm(raw.Operand(a, 0, K, 0), raw.Operand(b, 0, K, K * N), raw.Operand(C, 0, H * N, N), M, N, K,
                     batch=(H, 1))
        else:                            # batch = (2, H) with compatible strides
            C = torch.zeros(2 * H * 64 * N, dtype=BF, device=dev)
            raw.gemm(raw.Operand(a, 0, K, H * 64 * K, 64 * K), raw.Operand(b, 1, N, 0, K * N),
                     raw.Operand(C, 0, N, H * 64 * N, 64 * N), 64, N, K, batch=(2, H))
        outs[str(dev)] = C
    torch.cuda.synchronize()
    _close(outs[str(cuda)], outs["cpu"], 5e-2, 3e-2, f"plain gemm {case}")


@pytest.mark.parametrize("act_bwd", [False, True])
@pytest.mark.parametrize("with_r", [False, True])
@pytest.mark.parametrize("act", ["gelu", "relu"])
def test_gemm_activation_split(cuda, act_bwd, with_r, act):
    """activation GEMMs as the model issues them (contiguous, unbatched): gemm4w + elementwise or fused MFMA
    (gelu and relu take gemm4w's direct epilogue without a residual; ragged N = 520 masks columns per lane)"""
    torch.manual_seed(9)
    M, K, N = 384, 256, 520
    A = (torch.randn(M * K) * 0.5).to(BF)
    B = (torch.randn(N * K) * 0.5).to(BF)
    R = (torch.randn(M * N) * 0.5).to(BF)
    Zi = (torch.randn(M * N) * 1.5).to(BF)
    outs = {}
    for dev in ("cpu", cuda):
        C = torch.zeros(M * N, dtype=BF, device=dev)
        Z = torch.zeros(M * N, dtype=BF, device=dev)
        raw.gemm(raw.Operand(A.to(dev), 0, K), raw.Operand(B.to(dev), 0, K), raw.Operand(C, 0, N), M, N, K,
                 act=act, act_bwd=act_bwd, R=R.to(dev) if with_r else None,
                 Zout=None if act_bwd else Z, Zin=Zi.to(dev) if act_bwd else None)
        outs[str(dev)] = (C, Z)
    torch.cuda.synchronize()
    for name, g, c in zip("CZ", outs[str(cuda)], outs["cpu"]):
        _close(g, c, 5e-2, 3e-2, f"activation gemm {act} {name} bwd={act_bwd} R={with_r}")


def test_gemm_oob_rejected(cuda):
    A = torch.zeros(64 * 64, dtype=BF, device=cuda)
    B = torch.zeros(64 * 64, dtype=BF, device=cuda)
    C = torch.zeros(64 * 64, dtype=BF, device=cuda)
    with pytest.raises(Exception):
        raw.gemm(raw.Operand(A, 0, 64), raw.Operand(B, 0, 64), raw.Operand(C, 0, 64), 128, 64, 64)


# ----------------------------------------------------------------------------------------------------------------
def _attention_case(cuda, B, S, H, D, causal, layout):
    """layout "separate": q, k, v, o each [T][H*D]; "kqv": q, k, v (and dq, dk, dv) column slices of ONE
    [T][3*H*D] buffer with o / do at their own stride H*D -- the layout training uses (ld != ld_o)"""
    N = H * D
    ld = 3 * N if layout == "kqv" else N
    scale = D ** -0.5
    T = B * S
    g = torch.Generator().manual_seed(D + S + H)
    if layout == "kqv":
        buf = (torch.randn(T, 3 * N, generator=g) * 0.8).to(BF)
        k, q, v = buf[:, :N], buf[:, N:2 * N], buf[:, 2 * N:]
    else:
        q, k, v = [(torch.randn(T, N, generator=g) * 0.8).to(BF) for _ in range(3)]
    do = (torch.randn(T, N, generator=g) * 0.8).to(BF)
    res = {}
    for dev in ("cpu", cuda):
        if layout == "kqv":
            b = buf.to(dev)
            t = [b[:, N:2 * N], b[:, :N], b[:, 2 * N:]]
            dbuf = torch.zeros(T, 3 * N, dtype=BF, device=dev)
            dq, dk, dv = dbuf[:, N:2 * N], dbuf[:, :N], dbuf[:, 2 * N:]
        else:
            t = [x.to(dev).reshape(-1) for x in (q, k, v)]
            dq, dk, dv = [torch.zeros(T * N, dtype=BF, device=dev) for _ in range(3)]
        o = torch.zeros(T * N, dtype=BF, device=dev)
        lse = torch.zeros(B * H * S, dtype=torch.float32, device=dev)
        raw.attn_fwd(t[0], t[1], t[2], o, lse, B, S, H, D, ld, scale, causal, ld_o=N)
        delta = torch.zeros(B * H * S, dtype=torch.float32, device=dev)
        raw.attn_bwd(t[0], t[1], t[2], o, do.reshape(-1).to(dev), lse, delta, dq, dk, dv, B, S, H, D, ld, scale,
                     causal, ld_o=N)
        res[str(dev)] = (o, lse, dq, dk, dv)
    torch.cuda.synchronize()
    for name, gg, c in zip(["o", "lse", "dq", "dk", "dv"], res[str(cuda)], res["cpu"]):
        _close(gg, c, 3e-2, 3e-2, f"attention B={B} S={S} H={H} D={D} causal={causal} {layout} {name}")


@pytest.mark.parametrize("layout", ["separate", "kqv"])
@pytest.mark.parametrize("D", [32, 64, 96, 128])
@pytest.mark.parametrize("S,causal", [(128, True), (200, True), (256, False), (64, True), (576, True), (1000, False)])
def test_attention_fwd_bwd(cuda, D, S, causal, layout):
    _attention_case(cuda, 2, S, 3, D, causal, layout)


@pytest.mark.parametrize("D", [64, 128])
def test_attention_training_shape(cuda, D):
    """the step's shape class: S = 2048, H = 16, B = 4, causal, interleaved k|q|v (multi-block causal paths of the
    forward, dQ and dK/dV kernels against the fp32 oracle)"""
    _attention_case(cuda, 4, 2048, 16, D, True, "kqv")


@pytest.mark.parametrize("D", [64, 96, 128])
def test_attention_fused_residual(cuda, D):
    """out = bf16(o) + residual written by the forward epilogue == the unfused o, then the elementwise add"""
    torch.manual_seed(3)
    B, S, H = 2, 320, 3
    ld = H * D
    q, k, v, r = [(torch.randn(B * S * ld) * 0.8).to(BF).to(cuda) for _ in range(4)]
    o1, o2, out = [torch.zeros(B * S * ld, dtype=BF, device=cuda) for _ in range(3)]
    l1, l2 = [torch.zeros(B * H * S, device=cuda) for _ in range(2)]
    raw.attn_fwd(q, k, v, o1, l1, B, S, H, D, ld, D ** -0.5, True)
    raw.attn_fwd(q, k, v, o2, l2, B, S, H, D, ld, D ** -0.5, True, residual=r, out=out)
    ref = torch.empty_like(o1)
    raw.elementwise("add", o1, ref, z=r)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2) and torch.equal(l1, l2)
    assert torch.equal(out, ref)


# ----------------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("F_,groups,nrows", [(2048, 1, 96), (128, 16, 96), (64, 1, 96), (1000, 1, 96),
                                           (128, 1, 5000), (256, 8, 4000), (32, 4, 3001)])
def test_norm(cuda, F_, groups, nrows):
    torch.manual_seed(F_)
    rows = nrows * groups
    x = (torch.randn(rows * F_) * 2 + 0.3).to(BF)
    dy = torch.randn(rows * F_).to(BF)
    sc = torch.randn(groups * F_) * 0.1 + 1
    sh = torch.randn(groups * F_) * 0.1
    res = {}
    for dev in ("cpu", cuda):
        y = torch.zeros(rows * F_, dtype=BF, device=dev)
        st = torch.zeros(2 * rows, device=dev)
        raw.norm_fwd(x.to(dev), sc.to(dev), sh.to(dev), y, st, rows, F_, groups)
        dx = torch.zeros(rows * F_, dtype=BF, device=dev)
        dsc = torch.zeros(groups * F_, device=dev)
        dsh = torch.zeros(groups * F_, device=dev)
        raw.norm_bwd(x.to(dev), dy.to(dev), sc.to(dev), st, dx, dsc, dsh, rows, F_, groups)
        res[str(dev)] = (y, st, dx, dsc, dsh)
    torch.cuda.synchronize()
    for name, g, c in zip(["y", "stats", "dx", "dscale", "dshift"], res[str(cuda)], res["cpu"]):
        _close(g, c, 3e-2, 2e-2, f"norm F={F_} {name}")


@pytest.mark.parametrize("F_,groups,nrows", [(256, 8, 500), (192, 1, 700), (512, 8, 100), (96, 3, 1000),
                                           (2048, 1, 64)])
def test_norm_bwd_residual_one_chunk(cuda, F_, groups, nrows):
    """the backward with the bf16 residual / stream gradient added (F.GradSink, bf16 streams) and parameter
    gradients: rows of one 16-byte chunk per lane take norm_bwd1_kernel (lanes past F idle at F 192 / 96; per-lane-
    group parameter slabs for every group count), 2048-wide rows the general body -- against the fp32 oracle"""
    torch.manual_seed(F_ + groups)
    rows = nrows * groups
    x = (torch.randn(rows * F_) * 2 + 0.3).to(BF)
    dy = torch.randn(rows * F_).to(BF)
    r = torch.randn(rows * F_).to(BF)
    sc = torch.randn(groups * F_) * 0.1 + 1
    res = {}
    for dev in ("cpu", cuda):
        y = torch.zeros(rows * F_, dtype=BF, device=dev)
        st = torch.zeros(2 * rows, device=dev)
        raw.norm_fwd(x.to(dev), sc.to(dev), None, y, st, rows, F_, groups)
        dx = torch.full((rows * F_,), float("nan"), dtype=BF, device=dev)
        dsc = torch.zeros(groups * F_, device=dev)
        dsh = torch.zeros(groups * F_, device=dev)
        raw.norm_bwd(x.to(dev), dy.to(dev), sc.to(dev), st, dx, dsc, dsh, rows, F_, groups, R=r.to(dev))
        res[str(dev)] = (y, dx, dsc, dsh)
    torch.cuda.synchronize()
    for name, g, c in zip(["y", "dx", "dscale", "dshift"], res[str(cuda)], res["cpu"]):
        _close(g, c, 3e-2, 2e-2, f"norm+R F={F_} groups={groups} {name}")


@pytest.mark.parametrize("act", ["gelu", "relu", "silu"])
@pytest.mark.parametrize("F_,groups,nrows", [(256, 8, 300), (2048, 1, 96), (128, 1, 2000)])
def test_norm_with_fused_activation(cuda, F_, groups, nrows, act):
    """norm + the following activation layer in one kernel (forward y = act(z)); the backward takes dy through
    act'(z) with z recomputed from the row statistics (its own kernel instantiation) -- against the fp32 oracle"""
    torch.manual_seed(F_ + len(act))
    rows = nrows * groups
    x = (torch.randn(rows * F_) * 2 + 0.3).to(BF)
    dy = torch.randn(rows * F_).to(BF)
    sc = torch.randn(groups * F_) * 0.1 + 1
    sh = torch.randn(groups * F_) * 0.3
    res = {}
    for dev in ("cpu", cuda):
        y = torch.zeros(rows * F_, dtype=BF, device=dev)
        st = torch.zeros(2 * rows, device=dev)
        raw.norm_fwd(x.to(dev), sc.to(dev), sh.to(dev), y, st, rows, F_, groups, act=act)
        dx = torch.zeros(rows * F_, dtype=BF, device=dev)
        dsc = torch.zeros(groups * F_, device=dev)
        dsh = torch.zeros(groups * F_, device=dev)
        raw.norm_bwd(x.to(dev), dy.to(dev), sc.to(dev), st, dx, dsc, dsh, rows, F_, groups, shift=sh.to(dev), act=act)
        res[str(dev)] = (y, dx, dsc, dsh)
    torch.cuda.synchronize()
    for name, g, c in zip(["y", "dx", "dscale", "dshift"], res[str(cuda)], res["cpu"]):
        _close(g, c, 3e-2, 2e-2, f"norm+{act} F={F_} {name}")


@pytest.mark.parametrize("F_,groups,nrows", [(512, 8, 200), (2048, 1, 96)])
def test_norm_bwd_input_relu_mask(cuda, F_, groups, nrows):
    """the norm of a relu product: its backward multiplies dx by [x > 0] (F.ReluGrad) in the kernel"""
    torch.manual_seed(F_ + 1)
    rows = nrows * groups
    x = torch.relu(torch.randn(rows * F_) * 2).to(BF)
    dy = torch.randn(rows * F_).to(BF)
    sc = torch.randn(groups * F_) * 0.1 + 1
    res = {}
    for dev in ("cpu", cuda):
        y = torch.zeros(rows * F_, dtype=BF, device=dev)
        st = torch.zeros(2 * rows, device=dev)
        raw.norm_fwd(x.to(dev), sc.to(dev), None, y, st, rows, F_, groups)
        dx = torch.full((rows * F_,), float("nan"), dtype=BF, device=dev)
        dsc = torch.zeros(groups * F_, device=dev)
        raw.norm_bwd(x.to(dev), dy.to(dev), sc.to(dev), st, dx, dsc, None, rows, F_, groups, in_relu=True)
        res[str(dev)] = (dx, dsc)
    torch.cuda.synchronize()
    for name, g, c in zip(["dx", "dscale"], res[str(cuda)], res["cpu"]):
        _close(g, c, 3e-2, 2e-2, f"norm in_relu F={F_} {name}")
    assert torch.all(res[str(cuda)][0].cpu()[x == 0] == 0)


@pytest.mark.parametrize("F_,groups,nrows", [(256, 8, 300), (2048, 1, 96), (64, 4, 1000)])
def test_norm_bwd_fp32_stream_gradient(cuda, F_, groups, nrows):
    """the RevNet stream-gradient form of the norm backward (F.GradSink): dx32 = dx + g32 in fp32 (its own kernel
    instantiation), dx = its bf16 copy"""
    torch.manual_seed(F_ + groups)
    rows = nrows * groups
    x = (torch.randn(rows * F_) * 2 + 0.3).to(BF)
    dy = torch.randn(rows * F_).to(BF)
    g32 = torch.randn(rows * F_) * 3
    sc = torch.randn(groups * F_) * 0.1 + 1
    res = {}
    for dev in ("cpu", cuda):
        y = torch.zeros(rows * F_, dtype=BF, device=dev)
        st = torch.zeros(2 * rows, device=dev)
        raw.norm_fwd(x.to(dev), sc.to(dev), None, y, st, rows, F_, groups)
        dx = torch.zeros(rows * F_, dtype=BF, device=dev)
        dx32 = torch.full((rows * F_,), float("nan"), device=dev)
        dsc = torch.zeros(groups * F_, device=dev)
        raw.norm_bwd(x.to(dev), dy.to(dev), sc.to(dev), st, dx, dsc, None, rows, F_, groups, R32=g32.to(dev),
                     dx32=dx32)
        res[str(dev)] = (dx32, dsc, dx)
    torch.cuda.synchronize()
    for name, g, c in zip(["dx32", "dscale"], res[str(cuda)][:2], res["cpu"][:2]):
        _close(g, c, 3e-2, 2e-2, f"norm stream gradient F={F_} {name}")
    dx32, _, dx = res[str(cuda)]
    assert torch.equal(dx.cpu(), dx32.cpu().to(BF)), "dx is not the bf16 copy of dx32"


@pytest.mark.parametrize("op,act", [("act", "gelu"), ("act", "relu"), ("act_bwd", "gelu"), ("act_bwd", "mish"),
                                    ("act", "silu"), ("act", "lecun_tanh"), ("add", None), ("axpby", None),
                                    ("mul", None), ("dropout", None), ("act_bwd", "softsign")])
def test_elementwise(cuda, op, act):
    torch.manual_seed(7)
    n = 4096 + 8
    x = torch.randn(n).to(BF)
    z = torch.randn(n).to(BF)
    out = {}
    for dev in ("cpu", cuda):
        y = torch.zeros(n, dtype=BF, device=dev)
        raw.elementwise(op, x.to(dev), y, z=z.to(dev), act=act, alpha=0.7, beta=-1.3, seed=1234, keep=0.8)
        out[str(dev)] = y
    torch.cuda.synchronize()
    _close(out[str(cuda)], out["cpu"], 2e-2, 2e-2, f"{op}/{act}")


@pytest.mark.parametrize("n", [4096 + 8, 4099])
def test_add_to_bf16(cuda, n):
    """bf16(a + b) of two fp32 tensors in one pass (the reversible body's output and input gradient, HIP add2
    kernel), ragged tail included, against the fp32 sum rounded once on the CPU"""
    torch.manual_seed(5)
    a, b = torch.randn(n) * 3, torch.randn(n)
    got = raw.add_to_bf16(a.to(cuda), b.to(cuda))
    torch.cuda.synchronize()
    assert got.dtype == BF and torch.equal(got.cpu(), (a + b).to(BF))


def test_to_f32_and_copy2d(cuda):
    """bf16 -> fp32 cast (the RevNet body's fp32 streams) is exact; the strided copy interleaves the stacked
    [3][K][N] q / k / v weights into [K][3N] exactly as the permute + contiguous it replaces"""
    torch.manual_seed(6)
    x = torch.randn(4096 * 8).to(BF)
    y = raw.to_f32(x.to(cuda))
    K, N = 96, 40
    w = torch.randn(3, K, N).to(BF)
    cat = torch.empty(K, 3 * N, dtype=BF, device=cuda)
    raw.copy2d(w.to(cuda), cat, K, N, N, 3 * N, batch=3, sx=K * N, sy=N)
    torch.cuda.synchronize()
    assert y.dtype == torch.float32 and torch.equal(y.cpu(), x.float())
    assert torch.equal(cat.cpu(), w.permute(1, 0, 2).reshape(K, 3 * N))
    m = torch.randn(3, 72, 72).to(BF)
    z = torch.randn(1000 * 8 + 8)
    zg = z.to(cuda)
    raw.zero_(zg[8:])
    got = raw.tril(m.to(cuda))
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), torch.tril(m))
    assert torch.equal(zg[:8].cpu(), z[:8]) and not zg[8:].any()


def test_xent(cuda):
    torch.manual_seed(11)
    rows, V, Vp = 64, 1000, 1024
    logits = (torch.randn(rows * Vp) * 3).to(BF)
    tgt = torch.randint(0, V, (rows,), dtype=torch.int32)
    res = {}
    for dev in ("cpu", cuda):
        lse, loss, hit = [torch.zeros(rows, device=dev) for _ in range(3)]
        raw.xent_fwd(logits.to(dev), tgt.to(dev), lse, loss, hit, rows, V, Vp, 1e-4)
        g = torch.zeros(rows * Vp, dtype=BF, device=dev)
        raw.xent_bwd(logits.to(dev), tgt.to(dev), lse, g, None, 1.0 / rows, rows, V, Vp, 1e-4)
        res[str(dev)] = (lse, loss, hit, g)
    torch.cuda.synchronize()
    for name, g, c in zip(["lse", "loss", "hit", "grad"], res[str(cuda)], res["cpu"]):
        _close(g, c, 2e-2, 1e-2, f"xent {name}")


def test_gather_scatter(cuda):
    torch.manual_seed(5)
    V, Fd, T = 300, 64, 1000
    table = torch.randn(V * Fd).to(BF)
    idx = torch.randint(0, V, (T,), dtype=torch.int32)
    dy = torch.randn(T * Fd).to(BF)
    res = {}
    for dev in ("cpu", cuda):
        out = torch.zeros(T * Fd, dtype=BF, device=dev)
        raw.gather(idx.to(dev), table.to(dev), out, T, Fd, V)
        dt = torch.zeros(V * Fd, device=dev)
        raw.scatter_add(idx.to(dev), dy.to(dev), dt, T, Fd, V)
        res[str(dev)] = (out, dt)
    torch.cuda.synchronize()
    _close(res[str(cuda)][0], res["cpu"][0], 0, 0, "gather")
    _close(res[str(cuda)][1], res["cpu"][1], 1e-3, 1e-3, "scatter_add")


@pytest.mark.parametrize("dist", ["uniform", "zipf", "padding30", "one_id"])
def test_scatter_add_skewed_ids_deterministic(cuda, dist):
    """the chunked sorted scatter (64-row chunks, fixed-order fold of runs crossing chunks) on skewed id
    distributions: matches the fp32 oracle and repeats bitwise"""
    g = torch.Generator().manual_seed(11)
    V, Fd, T = 512, 72, 5000
    if dist == "uniform":
        idx = torch.randint(0, V, (T,), generator=g)
    elif dist == "zipf":
        p = 1.0 / torch.arange(1, V + 1, dtype=torch.float64) ** 1.2
        idx = torch.multinomial(p / p.sum(), T, replacement=True, generator=g)
    elif dist == "padding30":
        idx = torch.randint(0, V, (T,), generator=g)
        idx[torch.rand(T, generator=g) < 0.3] = 7
    else:
        idx = torch.full((T,), 3)
    idx = idx.to(torch.int32)
    dy = torch.randn(T * Fd, generator=g).to(BF)
    ref = torch.zeros(V * Fd)
    raw.scatter_add(idx, dy, ref, T, Fd, V)
    outs = []
    for _ in range(2):
        dt = torch.ones(V * Fd, device=cuda)
        raw.scatter_add(idx.to(cuda), dy.to(cuda), dt, T, Fd, V)
        outs.append(dt)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    _close(outs[0] - 1, ref, 2e-3, 1e-3, f"scatter_add {dist}")


def test_pkm_gather_bwd_deterministic(cuda):
    torch.manual_seed(4)
    R, H, Fk, P = 3000, 4, 32, 64
    idx = torch.randint(0, P, (R,), dtype=torch.int32)
    idx[:1000] = 5                                   # a hot value row
    val = torch.randn(R)
    table = torch.randn(P * H * Fk).to(BF)
    dy = torch.randn(R * Fk).to(BF)
    dt_ref, dv_ref = torch.zeros(P * H * Fk), torch.zeros(R)
    raw.pkm_gather_bwd(idx, val, table, dy, dt_ref, dv_ref, R, H, Fk, P)
    outs = []
    for _ in range(2):
        dt, dv = torch.zeros(P * H * Fk, device=cuda), torch.zeros(R, device=cuda)
        raw.pkm_gather_bwd(idx.to(cuda), val.to(cuda), table.to(cuda), dy.to(cuda), dt, dv, R, H, Fk, P)
        outs.append((dt, dv))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    _close(outs[0][0], dt_ref, 2e-3, 1e-3, "pkm dtable")
    _close(outs[0][1], dv_ref, 2e-3, 1e-3, "pkm dval")


def test_cumsum(cuda):
    torch.manual_seed(9)
    x = torch.randn(2, 50, 3, 8).to(BF)
    for rev, mean, grad in [(False, False, False), (True, True, True), (False, True, False)]:
        out = {}
        for dev in ("cpu", cuda):
            y = torch.zeros_like(x, device=dev)
            raw.cumsum(x.to(dev), y, 2, 50, 24, rev, mean, grad)
            out[str(dev)] = y
        torch.cuda.synchronize()
        _close(out[str(cuda)], out["cpu"], 5e-2, 2e-2, f"cumsum {rev}{mean}{grad}")


@pytest.mark.parametrize("K", [64, 128, 576])
@pytest.mark.parametrize("a_t,b_t", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_big_tile(cuda, a_t, b_t, K):
    """shapes that take the 256x256 LDS-DMA kernels (>= 512 tiles), incl. ragged M/N edges; K = 576 runs the
    K loop's steady state (counted vmcnt) for 9 K-tiles. Repeats must be bitwise identical (race screen). On the
    "mfma" leg every product must run on gemm4w (persistent, direct and beta epilogues)."""
    torch.manual_seed(21 + a_t + 2 * b_t + K)
    c0 = g4w_calls()
    M, N = 4160, 8128
    A = (torch.randn(M * K) * 0.5).to(BF)
    B = (torch.randn(N * K) * 0.5).to(BF)
    lda = K if a_t == 0 else M
    ldb = K if b_t == 0 else N
    av = A.view(M, K) if a_t == 0 else A.view(K, M).t()
    bv = B.view(N, K).t() if b_t == 0 else B.view(K, N)
    ref = av.float() @ bv.float()
    Ad, Bd = A.to(cuda), B.to(cuda)
    outs = []
    for _ in range(4):
        Cg = torch.zeros(M * N, dtype=BF, device=cuda)
        raw.gemm(raw.Operand(Ad, a_t, lda), raw.Operand(Bd, b_t, ldb), raw.Operand(Cg, 0, N), M, N, K)
        outs.append(Cg)
    torch.cuda.synchronize()
    _close(outs[0].view(M, N), ref, 4e-2, 2e-2, f"gemm256 {a_t}{b_t} K{K}")
    for o in outs[1:]:
        assert torch.equal(o, outs[0]), "run-to-run difference: LDS race"
    # fp32 output with accumulation (the wgrad epilogue)
    Cf = torch.ones(M * N, dtype=torch.float32, device=cuda)
    raw.gemm(raw.Operand(Ad, a_t, lda), raw.Operand(Bd, b_t, ldb), raw.Operand(Cf, 0, N), M, N, K, beta=1.0)
    torch.cuda.synchronize()
    _close(Cf.view(M, N), ref + 1, 2e-2, 2e-2, f"gemm256 f32 {a_t}{b_t} K{K}")
    assert g4w_calls() - c0 == 5, "gemm4w did not run"


@pytest.mark.parametrize("a_t,b_t", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("out_f32", [False, True])
def test_gemm4w_ragged(cuda, a_t, b_t, out_f32):
    """gemm4w directly on ragged M / N -- 1, 17, 255, 257 rows (decode-sized products up to one row
    past a tile), padded ldc -- bf16 and fp32 outputs, batched, against the fp32 oracle"""
    for M, N, K, nb in ((1, 264, 128, 3), (17, 8, 64, 2), (255, 520, 192, 1), (257, 256, 320, 2)):
        if a_t == 1 and M % 8:
            continue   # a [K][M] operand needs 16-byte rows
        torch.manual_seed(M + N + K)
        ldc = N + 8
        A = (torch.randn(nb * M * K) * 0.5).to(BF)
        B = (torch.randn(nb * N * K) * 0.5).to(BF)
        lda = K if a_t == 0 else M
        ldb = K if b_t == 0 else N
        av = A.view(nb, M, K) if a_t == 0 else A.view(nb, K, M).transpose(1, 2)
        bv = B.view(nb, N, K).transpose(1, 2) if b_t == 0 else B.view(nb, K, N)
        ref = av.float() @ bv.float()
        dt = torch.float32 if out_f32 else BF
        C = torch.full((nb * M * ldc,), 7.0, dtype=dt, device=cuda)
        c0 = g4w_calls()
        raw.gemm(raw.Operand(A.to(cuda), a_t, lda, M * K), raw.Operand(B.to(cuda), b_t, ldb, N * K),
                 raw.Operand(C, 0, ldc, M * ldc), M, N, K, batch=(nb, 1))
        torch.cuda.synchronize()
        assert g4w_calls() - c0 == 1, f"{M}x{N}x{K} did not run gemm4w"
        Cv = C.view(nb, M, ldc)
        _close(Cv[:, :, :N], ref, 3e-2 * math.sqrt(K / 64), 2e-2, f"gemm4w {a_t}{b_t} {M}x{N}x{K} f32={out_f32}")
        assert torch.all(Cv[:, :, N:].float().cpu() == 7.0), "wrote past N into the ldc padding"


def g4w_queue_calls() -> int:
    import ctypes
    f = L.lib().obst_gemm4w_queue_calls
    f.restype = ctypes.c_longlong
    return int(f())


@pytest.mark.parametrize("a_t,b_t", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("out_f32", [False, True])
def test_gemm4w_tile_queue(cuda, a_t, b_t, out_f32):
    """products with more tiles than blocks and >= 3 K-tiles take the dynamic per-XCD tile queue (OBST_G4W_QUEUE,
    default on): every tile exactly once (ragged M, padded ldc) against the fp32 oracle, twice in a row (the
    counters of the ring slot are zeroed per launch)"""
    M, N, K, ldc = 8000, 2304, 448, 2304 + 8
    torch.manual_seed(5)
    A = (torch.randn(M * K) * 0.5).to(BF)
    B = (torch.randn(N * K) * 0.5).to(BF)
    av = A.view(M, K) if a_t == 0 else A.view(K, M).t()
    bv = B.view(N, K).t() if b_t == 0 else B.view(K, N)
    ref = av.float() @ bv.float()
    dt = torch.float32 if out_f32 else BF
    Ad, Bd = A.to(cuda), B.to(cuda)
    for rep in range(2):
        C = torch.full((M * ldc,), 7.0, dtype=dt, device=cuda)
        c0, q0 = g4w_calls(), g4w_queue_calls()
        raw.gemm(raw.Operand(Ad, a_t, K if a_t == 0 else M, M * K), raw.Operand(Bd, b_t, K if b_t == 0 else N, N * K),
                 raw.Operand(C, 0, ldc, M * ldc), M, N, K)
        torch.cuda.synchronize()
        assert g4w_calls() - c0 == 1 and g4w_queue_calls() - q0 == 1, "the product did not take the tile queue"
        Cv = C.view(M, ldc)
        _close(Cv[:, :N], ref, 3e-2 * math.sqrt(K / 64), 2e-2, f"queued gemm4w {a_t}{b_t} f32={out_f32} rep {rep}")
        assert torch.all(Cv[:, N:].float().cpu() == 7.0), "wrote past N into the ldc padding"


@pytest.mark.parametrize("a_t,b_t,M,N,K", [(0, 0, 1024, 1536, 16384), (1, 1, 1024, 1536, 16384),
                                           (1, 0, 512, 768, 131072), (0, 1, 512, 768, 131072)])
def test_gemm_splitk_wgrad(cuda, a_t, b_t, M, N, K):
    """few output tiles + long K + fp32 accumulate into C (beta = 1): K is split over the persistent grid into fp32
    slabs and folded deterministically (gemm4w split-K + splitk_reduce_kernel on the "mfma" leg; K = 131072 is the
    weight gradient of a 64 x 2048-token step, ks = 8)"""
    torch.manual_seed(5)
    c0 = g4w_calls()
    A = (torch.randn(M * K) * 0.5).to(BF)
    B = (torch.randn(N * K) * 0.5).to(BF)
    lda = K if a_t == 0 else M
    ldb = K if b_t == 0 else N
    av = A.view(M, K) if a_t == 0 else A.view(K, M).t()
    bv = B.view(N, K).t() if b_t == 0 else B.view(K, N)
    ref = av.float() @ bv.float() + 2.0
    Cf = torch.full((M * N,), 2.0, dtype=torch.float32, device=cuda)
    raw.gemm(raw.Operand(A.to(cuda), a_t, lda), raw.Operand(B.to(cuda), b_t, ldb), raw.Operand(Cf, 0, N), M, N, K,
             beta=1.0)
    torch.cuda.synchronize()
    _close(Cf.view(M, N), ref, 5e-2 * math.sqrt(K / 16384), 1e-2, f"splitk {a_t}{b_t} K{K}")
    assert g4w_calls() - c0 == 1, "gemm4w did not run"


@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_gemm4w_batched_splitk(cuda, beta):
    """batched fp32 weight gradients with few tiles per batch (the per-head group linear: gw[h] = x[:, h]^T dy[:, h]):
    gemm4w splits K into per-(batch, split) fp32 slabs and folds them per batch into the strided C"""
    torch.manual_seed(8)
    H, K, N, M = 4, 256, 512, 16384    # gw[h][K][N] over M tokens: 4 x 2 tiles per launch without the split
    x = (torch.randn(M, H, K) * 0.5).to(BF)
    dy = (torch.randn(M, H, N) * 0.5).to(BF)
    ref = torch.einsum("mhk,mhn->hkn", x.float(), dy.float()) + (2.0 if beta else 0.0)
    c0 = g4w_calls()
    G = torch.full((H, K, N), 2.0, dtype=torch.float32, device=cuda)
    raw.gemm(raw.Operand(x.to(cuda), 1, H * K, K), raw.Operand(dy.to(cuda), 1, H * N, N),
             raw.Operand(G, 0, N, K * N), K, N, M, batch=(H, 1), beta=beta)
    torch.cuda.synchronize()
    assert g4w_calls() - c0 == 1
    _close(G.cpu(), ref, 5e-2 * math.sqrt(M / 16384), 1e-2, f"batched split-K beta {beta}")


@pytest.mark.parametrize("out_f32", [False, True])
@pytest.mark.parametrize("a_t,b_t", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_persistent(cuda, a_t, b_t, out_f32):
    """many whole 256x256 tiles: 6 tiles per batch x 90 batches = 540 tiles (uneven per XCD, a partial last round
    per CU), 5 K-tiles; then tri = 3 (only the lower triangle of C receives the product) on square tiles (the
    128x128 kernel; gemm4w takes tri 3 with a split contraction index only). Repeats are bitwise identical."""
    torch.manual_seed(7 + a_t + 2 * b_t + 4 * out_f32)
    for M, N, K, nb, tri in ((768, 512, 320, 90, 0), (512, 512, 320, 140, 3)):
        A = (torch.randn(nb * M * K) * 0.5).to(BF)
        B = (torch.randn(nb * N * K) * 0.5).to(BF)
        lda = K if a_t == 0 else M
        ldb = K if b_t == 0 else N
        av = A.view(nb, M, K) if a_t == 0 else A.view(nb, K, M).transpose(1, 2)
        bv = B.view(nb, N, K).transpose(1, 2) if b_t == 0 else B.view(nb, K, N)
        ref = av.float() @ bv.float()
        if tri == 3:
            ref = ref * torch.ones(M, N).tril()
        Ad, Bd = A.to(cuda), B.to(cuda)
        outs = []
        for _ in range(2):
            C = torch.zeros(nb * M * N, dtype=torch.float32 if out_f32 else BF, device=cuda)
            raw.gemm(raw.Operand(Ad, a_t, lda, M * K), raw.Operand(Bd, b_t, ldb, N * K), raw.Operand(C, 0, N, M * N),
                     M, N, K, batch=(nb, 1), tri=tri)
            outs.append(C)
        torch.cuda.synchronize()
        _close(outs[0].view(nb, M, N), ref, 4e-2, 2e-2, f"persistent gemm {a_t}{b_t} f32={out_f32} tri={tri}")
        assert torch.equal(outs[0], outs[1]), "run-to-run difference"


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("S,Bb", [(512, 8), (1024, 4)])
def test_gemm4w_split_index_tri3_splitk(cuda, causal, S, Bb):
    """the mixer weight-gradient form on gemm4w with few tiles: kin = F contraction read in place, tri 3 (causal)
    lower-triangle tiles, fp32 accumulate into C (beta 1) through the split-K slabs and their masked fold; the upper
    triangle keeps its old values"""
    torch.manual_seed(S + Bb)
    H, Fd = 2, 128
    hf = H * Fd
    a = (torch.randn(Bb, S, H, Fd) * 0.5).to(BF)
    b = (torch.randn(Bb, S, H, Fd) * 0.5).to(BF)
    c0v = torch.randn(H, S, S)
    c = c0v.to(cuda).flatten().contiguous()
    n0 = g4w_calls()
    raw.gemm(raw.Operand(a.to(cuda).flatten(), 0, hf, 0, Fd), raw.Operand(b.to(cuda).flatten(), 0, hf, 0, Fd),
             raw.Operand(c, 0, S, 0, S * S), S, S, Bb * Fd, batch=(1, H), beta=1.0, tri=3 if causal else 0,
             kin=Fd, a_sk=S * hf, b_sk=S * hf)
    torch.cuda.synchronize()
    assert g4w_calls() - n0 == 1
    prod = torch.einsum("bshf,bthf->hst", a.float(), b.float())
    if causal:
        prod = prod * torch.ones(S, S).tril()
    _close(c.view(H, S, S).cpu(), prod + c0v, 3e-2, 2e-2, f"kin tri3 splitk S={S} causal={causal}")


@pytest.mark.parametrize("B,S", [(16, 1024), (1, 512), (3, 512)])
@pytest.mark.parametrize("causal", [True, False])
def test_token_mixer_big_tiles(cuda, causal, B, S):
    """K03 on gemm4w: y = tril(W) x and dx = tril(W)^T dy with per-tile K ranges (tri 1 / 2), and the weight
    gradient dW = dy . x^T over the split contraction index (kin = F, read in place from [B, S, H, F]) into the
    lower-triangle tiles only (tri 3) for the causal mixer. One sequence: the weight gradient is a plain row-strided
    product (no split index); an odd batch of the causal mixer cannot start its split-K slabs on whole (b, f) blocks
    and takes the copied [H][S][B*F] operands -- both causal forms then run tri 3 on the 128x128 kernel"""
    from homebrewnlp_mtf_amd.ops import functional as F
    torch.manual_seed(3)
    H, Fd = 8, 256
    x = (torch.randn(B, S, H, Fd) * 0.5).to(BF)
    w = (torch.randn(H, S, S) * 0.05).to(BF)
    dy = (torch.randn(B, S, H, Fd) * 0.5).to(BF)
    xg, wg = x.to(cuda).requires_grad_(True), w.to(cuda).requires_grad_(True)
    c0, q0 = g4w_calls(), g4w_queue_calls()
    y = F.token_mixer(xg, wg, causal)
    y.backward(dy.to(cuda))
    torch.cuda.synchronize()
    # y, dx and dW: all three products on gemm4w (no phase kernel left)
    assert g4w_calls() - c0 == (2 if causal and B % 2 else 3)
    # y and dx (triangular A when causal) take the tile queue once they have more tiles than blocks; dW never does
    assert g4w_queue_calls() - q0 == (2 if B * H * (S // 256) > 256 else 0)
    xf, wf = x.float().requires_grad_(True), w.float().requires_grad_(True)
    wm = torch.tril(wf) if causal else wf
    ref = torch.einsum("hst,bthf->bshf", wm, xf)
    ref.backward(dy.float())
    _close(y, ref, 5e-2, 3e-2, "mixer y")
    _close(xg.grad, xf.grad, 5e-2, 3e-2, "mixer dx")
    _close(wg.grad, wf.grad, 1e-1, 3e-2, "mixer dw")


@pytest.mark.parametrize("group", [0, 8, 3])
def test_token_mixer_work_orders(cuda, group):
    """the triangular products' work orders (obst_gemm4w_tri_group; production: auto, 8 past 512 MiB of B operands):
    tile rows slowest (0), batch groups of 8 with the XCD interleave on one residue class, and groups of 3 whose last
    group is short (B x H = 80 = 26 x 3 + 2) -- every tile exactly once, on the tile queue (320 tiles), against the
    fp32 oracle"""
    import ctypes
    from homebrewnlp_mtf_amd.ops import functional as F
    setg = L.lib().obst_gemm4w_tri_group
    setg.argtypes = [ctypes.c_int]
    torch.manual_seed(7)
    B, S, H, Fd = 10, 1024, 8, 256
    x = (torch.randn(B, S, H, Fd) * 0.5).to(BF)
    w = (torch.randn(H, S, S) * 0.05).to(BF)
    dy = (torch.randn(B, S, H, Fd) * 0.5).to(BF)
    xg, wg = x.to(cuda).requires_grad_(True), w.to(cuda).requires_grad_(True)
    setg(group)
    try:
        q0 = g4w_queue_calls()
        y = F.token_mixer(xg, wg, True)
        y.backward(dy.to(cuda))
        torch.cuda.synchronize()
    finally:
        setg(-1)
    assert g4w_queue_calls() - q0 == 2, "y and dx did not take the tile queue"
    xf, wf = x.float().requires_grad_(True), w.float().requires_grad_(True)
    ref = torch.einsum("hst,bthf->bshf", torch.tril(wf), xf)
    ref.backward(dy.float())
    _close(y, ref, 5e-2, 3e-2, f"mixer y, order {group}")
    _close(xg.grad, xf.grad, 5e-2, 3e-2, f"mixer dx, order {group}")


@pytest.mark.parametrize("M,K,N", [(1, 2048, 2048), (7, 96, 64), (16, 2048, 8192), (32, 8192, 2048),
                                   (32, 2048, 6144), (20, 1024, 1040), (32, 2048, 50304), (17, 4096, 2048)])
def test_skinny_gemm_matches_fp32(cuda, M, K, N, monkeypatch):
    """decode-step GEMM (M <= 32 tokens) on the MFMA kernel of csrc/kernels/skinny.hip (weight as the K-contiguous
    [N][K] copy, split-K slabs for the narrow shapes) vs a PyTorch fp32 reference; a second call gives the same bits"""
    monkeypatch.setattr(raw, "_SKINNY", True)
    assert raw.skinny_ok(M, N, K)
    g = torch.Generator().manual_seed(M * 7 + K)
    a = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(K, N, generator=g) / math.sqrt(K)).bfloat16()
    wt = w.t().contiguous()
    c = torch.full((M * N,), float("nan"), dtype=torch.bfloat16, device=cuda)
    op = lambda: raw.gemm(raw.Operand(a.to(cuda).flatten(), 0, K), raw.Operand(wt.to(cuda).flatten(), 0, K),  # noqa
                          raw.Operand(c, 0, N), M, N, K)
    op()
    first = c.clone()
    op()
    assert torch.equal(first, c)
    ref = a.float() @ w.float()
    _close(c.view(M, N).float().cpu(), ref, 2e-2, 2e-2, f"skinny {M}x{K}x{N}")


@pytest.mark.parametrize("M,K,N,ks_expected", [(32, 4096, 2048, True), (5, 2048, 4096, False),
                                                (32, 2048, 8192, False)])
def test_skinny_gemm_fused_epilogue(cuda, M, K, N, ks_expected, monkeypatch):
    """the decode-step GEMM with its epilogue fused (split-K: in the combine kernel): C = gelu(alpha A.W + R) with the
    pre-activation in Zout, against the fp32 reference; the guard words around C / Zout stay untouched"""
    monkeypatch.setattr(raw, "_SKINNY", True)
    assert (L.lib().obst_skinny_ws(M, N, K) > 0) == ks_expected
    g = torch.Generator().manual_seed(M + N)
    a = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(K, N, generator=g) / math.sqrt(K)).bfloat16()
    r = torch.randn(M, N, generator=g).bfloat16()
    pad = 64
    c = torch.full((M * N + 2 * pad,), float("nan"), dtype=torch.bfloat16, device=cuda)
    z = torch.full((M * N + 2 * pad,), float("nan"), dtype=torch.bfloat16, device=cuda)
    raw.gemm(raw.Operand(a.to(cuda).flatten(), 0, K), raw.Operand(w.t().contiguous().to(cuda).flatten(), 0, K),
             raw.Operand(c[pad:pad + M * N], 0, N), M, N, K, alpha=0.5, act="gelu", R=r.to(cuda).flatten(),
             Zout=z[pad:pad + M * N])
    torch.cuda.synchronize()
    pre = 0.5 * (a.float() @ w.float()) + r.float()
    ref = torch.nn.functional.gelu(pre, approximate="tanh")
    _close(z[pad:pad + M * N].view(M, N).float().cpu(), pre, 2e-2, 2e-2, "skinny Zout")
    _close(c[pad:pad + M * N].view(M, N).float().cpu(), ref, 2e-2, 2e-2, "skinny gelu(C)")
    for t in (c, z):
        assert torch.isnan(t[:pad].float()).all() and torch.isnan(t[pad + M * N:].float()).all()


@pytest.mark.parametrize("out_f32", [False, True])
def test_gemm_split_contraction_index(cuda, out_f32):
    """C[h] = A_h · B_hᵀ with the contraction over (b, f) pairs of [B, S, H, F] tensors read in place (kin = F)"""
    torch.manual_seed(11)
    Bb, S, H, Fd = 4, 512, 2, 128
    a = (torch.randn(Bb, S, H, Fd) * 0.5).to(BF)
    b = (torch.randn(Bb, S, H, Fd) * 0.5).to(BF)
    hf = H * Fd
    c = torch.zeros(H * S * S, device=cuda, dtype=torch.float32 if out_f32 else BF)
    raw.gemm(raw.Operand(a.to(cuda).flatten(), 0, hf, 0, Fd), raw.Operand(b.to(cuda).flatten(), 0, hf, 0, Fd),
             raw.Operand(c, 0, S, 0, S * S), S, S, Bb * Fd, batch=(1, H), kin=Fd, a_sk=S * hf, b_sk=S * hf)
    ref = torch.einsum("bshf,bthf->hst", a.float(), b.float())
    _close(c.view(H, S, S).float().cpu(), ref, 3e-2, 2e-2, "split-index gemm")


@pytest.mark.parametrize("b_t,tri,batch", [(0, 0, (3, 1)), (1, 1, (2, 3)), (1, 0, (1, 1)), (0, 0, (150, 1)),
                                           (1, 0, (75, 2))])
@pytest.mark.parametrize("alpha", [1.0, -1.0])
def test_gemm_fp32_stream_update_with_bf16_copy(cuda, b_t, tri, batch, alpha):
    """the fused RevNet stream update (F.StreamSink): C = R + alpha * A.B in fp32 with Zout = bf16(C), written by
    gemm4w's own instantiation (row layout for K-contiguous B, fragment layout for the mixer's N-contiguous B)"""
    torch.manual_seed(11)
    M, N, K = 512, 256, 512
    b1, b2 = batch
    nb = b1 * b2
    a = (torch.randn(nb, M, K) * 0.3).to(BF)
    if tri:
        a = torch.tril(a)
    bm = (torch.randn(nb, K, N) * 0.3).to(BF)
    r = torch.randn(nb, M, N)
    bs = bm.transpose(1, 2).contiguous() if b_t == 0 else bm     # stored [N][K] (K-contiguous) or [K][N]
    c = torch.full((nb, M, N), float("nan"), device=cuda)
    z = torch.full((nb, M, N), float("nan"), device=cuda).to(BF)
    c0, q0 = g4w_calls(), g4w_queue_calls()
    raw.gemm(raw.Operand(a.to(cuda), 0, K, b2 * M * K, M * K),
             raw.Operand(bs.to(cuda), b_t, K if b_t == 0 else N, b2 * K * N, K * N),
             raw.Operand(c, 0, N, b2 * M * N, M * N), M, N, K, batch=batch, alpha=alpha, R=r.to(cuda), Zout=z, tri=tri)
    torch.cuda.synchronize()
    assert g4w_calls() - c0 == 1
    assert g4w_queue_calls() - q0 == (1 if tri == 0 and nb * 2 > 256 else 0), "tile queue use"
    ref = r + alpha * torch.matmul(a.float(), bm.float())
    _close(c, ref, 2e-2, 1e-2, f"stream update b_t={b_t} tri={tri}")
    assert torch.equal(z.cpu(), c.cpu().to(BF)), "Zout is not the bf16 copy of C"
