"""Raw (non-autograd) compute primitives. Each has two implementations with identical semantics:

* CUDA tensors → the hand-written gfx950 HIP kernels in ``csrc/kernels`` (never a silent PyTorch fallback);
* CPU / meta tensors → a plain PyTorch fp32 oracle (the CPU plumbing path, and the numerics reference the
  GPU tests compare against).

The autograd ops (``ops/functional.py``) and the model are written once against these primitives, so the CPU
test-suite exercises exactly the orchestration (strides, batching, fusion flags) the GPU path runs.
Before every launch the host checks that the largest element each operand descriptor can touch lies inside the
tensor's storage (a kernel fault can reset every GPU of the node).
"""
from __future__ import annotations

import math
import ctypes
import typing

import torch

from . import _lib as L

ACTS = {None: 0, "none": 0, "identity": 0, "relu": 1, "gelu": 2, "silu": 3, "sigmoid": 4, "tanh": 5,
        "lecun_tanh": 6, "mish": 7, "softsign": 8, "exp": 9}


def _f(t: torch.Tensor) -> torch.Tensor:
    return t if t.dtype == torch.float64 else t.float()


def on_gpu(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


def gemm_backend() -> str:
    """which kernels run the GEMMs: "gemm4w" (every product on the hand-written gfx950 MFMA kernels -- gemm4w, the
    128x128 fallback and the decode-step skinny kernel; no library GEMM is linked)"""
    if not L.available():
        return "torch-cpu"
    return "gemm4w"


def gemm4w_calls() -> int:
    """products dispatched to gemm4w so far (tests assert which kernel ran)"""
    return int(L.lib().obst_gemm4w_calls())


def _room(t: torch.Tensor) -> int:
    """elements addressable from t.data_ptr() to the end of its storage"""
    return t.untyped_storage().nbytes() // t.element_size() - t.storage_offset()


def _need(t: typing.Optional[torch.Tensor], max_index: int, name: str):
    if t is None:
        return
    if max_index >= _room(t):
        raise L.KernelError(f"operand {name}: descriptor reaches element {max_index} but storage holds {_room(t)}")


# ----------------------------------------------------------------------------------------------------------------
# activations (torch oracle; the kernels implement the same formulas in csrc/kernels/common.h)
def act_fwd_t(act: typing.Optional[str], x: torch.Tensor) -> torch.Tensor:
    if act in (None, "none", "identity"):
        return x
    if act == "relu":
        return torch.relu(x)
    if act == "gelu":
        return 0.5 * x * (1 + torch.tanh(math.sqrt(2 / math.pi) * (x + 0.044715 * x ** 3)))
    if act == "silu":
        return x * torch.sigmoid(x)
    if act == "sigmoid":
        return torch.sigmoid(x)
    if act == "tanh":
        return torch.tanh(x)
    if act == "lecun_tanh":
        return torch.tanh(x) + 0.1 * x
    if act == "mish":
        return x * torch.tanh(torch.nn.functional.softplus(x))
    if act == "softsign":
        return x / (1 + x.abs())
    if act == "exp":
        return torch.exp(x)
    raise ValueError(act)


def act_grad_t(act: typing.Optional[str], x: torch.Tensor) -> torch.Tensor:
    if act in (None, "none", "identity"):
        return torch.ones_like(x)
    if act == "relu":
        return (x > 0).to(x.dtype)
    if act == "gelu":
        k0, k1 = math.sqrt(2 / math.pi), 0.044715
        t = torch.tanh(k0 * (x + k1 * x ** 3))
        return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k0 * (1 + 3 * k1 * x * x)
    if act == "silu":
        s = torch.sigmoid(x)
        return s * (1 + x * (1 - s))
    if act == "sigmoid":
        s = torch.sigmoid(x)
        return s * (1 - s)
    if act == "tanh":
        return 1 - torch.tanh(x) ** 2
    if act == "lecun_tanh":
        return 1.1 - torch.tanh(x) ** 2
    if act == "mish":
        sp = torch.nn.functional.softplus(x)
        tsp = torch.tanh(sp)
        return tsp + x * (1 - tsp * tsp) * torch.sigmoid(x)
    if act == "softsign":
        return 1 / (1 + x.abs()) ** 2
    if act == "exp":
        return torch.exp(x)
    raise ValueError(act)


# ----------------------------------------------------------------------------------------------------------------
# GEMM
class Operand(typing.NamedTuple):
    t: torch.Tensor
    trans: int            # A: 0 = [M][K], 1 = [K][M];  B: 0 = [N][K], 1 = [K][N]
    ld: int
    s1: int = 0
    s2: int = 0


# Decode-step projections (M <= 32 tokens) run on the MFMA weight-streaming kernel (csrc/kernels/skinny.hip) against
# the cached K-contiguous weight copy, epilogue fused: a 32-row product on gemm4w would fill one 256-row tile row per
# N tile on a few CUs. OBST_SKINNY_GEMM=0 sends them to gemm4w (A/B only).
_SKINNY_ENV = __import__("os").environ.get("OBST_SKINNY_GEMM", "auto")
_SKINNY = None if _SKINNY_ENV == "auto" else _SKINNY_ENV == "1"
_SKINNY_WS: typing.Dict[typing.Any, torch.Tensor] = {}


def skinny_ok(M: int, N: int, K: int) -> bool:
    if not (0 < M <= 32 and N % 16 == 0 and K % 32 == 0):
        return False
    return _SKINNY if _SKINNY is not None else True


def _skinny_ws(device, n: int) -> typing.Optional[torch.Tensor]:
    """per-device fp32 workspace of the split-K skinny GEMM, grown on demand and reused"""
    if n <= 0:
        return None
    ws = _SKINNY_WS.get(device)
    if ws is None or ws.numel() < n:
        ws = torch.empty(max(n, 1 << 20), dtype=torch.float32, device=device)
        _SKINNY_WS[device] = ws
    return ws


def gemm(a: Operand, b: Operand, c: Operand, M: int, N: int, K: int, batch: typing.Tuple[int, int] = (1, 1),
         alpha: float = 1.0, beta: float = 0.0, act: typing.Optional[str] = None, act_bwd: bool = False,
         R: typing.Optional[torch.Tensor] = None, Zout: typing.Optional[torch.Tensor] = None,
         Zin: typing.Optional[torch.Tensor] = None, tri: int = 0, kin: int = 0, a_sk: int = 0, b_sk: int = 0):
    """C = epilogue(alpha * A·B). R, Zout, Zin share C's leading dims / batch strides.
    tri: 1/2 = A is lower/upper triangular (zero tiles are skipped, A must hold the zeros), 3 = only the lower
    triangle (n <= m) of C receives the product (M == N).
    kin > 0 (K-contiguous A and B only): the contraction index is split, k -> (k // kin) * sk + k % kin with the
    outer strides a_sk / b_sk -- a product over (batch, feature) pairs of a [B, S, H, F] tensor reads it in place.

    epilogue (act_bwd False): v = alpha*acc (+ beta*C if C is fp32) (+ R); Zout <- v; C <- act(v)
      (fp32 C without activation: Zout <- bf16(v), the output's bf16 copy -- the fused RevNet stream update)
    epilogue (act_bwd True) : C <- (alpha*acc + R) * act'(Zin)"""
    if c.t.device.type == "meta":
        return c.t
    b1, b2 = batch
    if kin and (a.trans or b.trans or K % kin):
        raise L.KernelError("split contraction index needs K-contiguous operands and K % kin == 0")
    if (not kin and on_gpu(c.t) and skinny_ok(M, N, K) and not act_bwd and Zin is None
            and tri == 0 and b1 * b2 == 1 and a.trans == 0 and b.trans == 0
            and c.t.dtype == torch.bfloat16 and a.t.dtype == torch.bfloat16 and b.t.dtype == torch.bfloat16
            and (R is None or R.dtype == torch.bfloat16) and (Zout is None or Zout.dtype == torch.bfloat16)
            and a.ld % 8 == 0 and b.ld % 8 == 0 and c.ld % 4 == 0 and a.ld >= K and b.ld >= K and c.ld >= N
            and a.t.data_ptr() % 16 == 0 and b.t.data_ptr() % 16 == 0 and c.t.data_ptr() % 8 == 0
            and (R is None or R.data_ptr() % 8 == 0) and (Zout is None or Zout.data_ptr() % 8 == 0)):
        # decode-step projection (M = batch tokens) against the K-contiguous weight: the MFMA weight-streaming kernel
        # with the epilogue fused (alpha, residual R, pre-activation Zout, activation; R / Zout in C's layout)
        _need(a.t, (M - 1) * a.ld + K - 1, "A")
        _need(b.t, (N - 1) * b.ld + K - 1, "B")
        for nm, t in (("C", c.t), ("R", R), ("Zout", Zout)):
            _need(t, (M - 1) * c.ld + N - 1, nm)
        ws = _skinny_ws(c.t.device, int(L.lib().obst_skinny_ws(M, N, K)))
        L.check(L.lib().obst_skinny_gemm(a.t.data_ptr(), a.ld, b.t.data_ptr(), b.ld, c.t.data_ptr(), c.ld, M, N, K,
                                         L.ptr(ws), L.ptr(R), L.ptr(Zout), float(alpha), ACTS[act],
                                         L.stream_ptr()), "skinny_gemm")
        return c.t
    if (not kin and on_gpu(c.t) and act is not None and tri == 0
            # decode-step activation backward: the skinny kernel + the elementwise pass
            and (act_bwd and skinny_ok(M, N, K) and R is None and alpha == 1.0 and a.trans == 0 and b.trans == 0)
            and c.t.dtype == torch.bfloat16
            and b1 * b2 == 1 and c.ld == N and (M * N) % 8 == 0 and c.t.is_contiguous() and c.t.numel() == M * N):
        # activation backward of a decode-step product: plain product, then the elementwise kernel
        if not act_bwd:
            z = Zout if Zout is not None else torch.empty(M * N, dtype=torch.bfloat16, device=c.t.device)
            gemm(a, b, Operand(z, 0, N), M, N, K, alpha=alpha, R=R)
            elementwise("act", z, c.t, act=act)
        else:
            gemm(a, b, c, M, N, K, alpha=alpha, R=R)
            elementwise("act_bwd", Zin, c.t, z=c.t, act=act)    # in place: C = C * act'(Zin)
        return c.t
    if on_gpu(c.t):
        out_f32 = c.t.dtype == torch.float32
        for nm, t in (("A", a.t), ("B", b.t)):
            if t.dtype != torch.bfloat16:
                raise L.KernelError(f"gemm operand {nm} must be bfloat16 on the GPU, got {t.dtype}")
        if not out_f32 and c.t.dtype != torch.bfloat16:
            raise L.KernelError(f"gemm output must be bf16 or fp32, got {c.t.dtype}")
        if out_f32 and (act_bwd or (Zout is not None and act is not None)):
            # (fp32 output with Zout and no activation: Zout is the output's bf16 copy)
            raise L.KernelError("pre-activation output / activation-backward epilogue need a bf16 output")
        bo = (b1 - 1) * a.s1 + (b2 - 1) * a.s2
        kext_a = (K // kin - 1) * a_sk + kin - 1 if kin else K - 1
        kext_b = (K // kin - 1) * b_sk + kin - 1 if kin else K - 1
        _need(a.t, bo + ((M - 1) * a.ld + kext_a if a.trans == 0 else (K - 1) * a.ld + M - 1), "A")
        bo = (b1 - 1) * b.s1 + (b2 - 1) * b.s2
        _need(b.t, bo + ((N - 1) * b.ld + kext_b if b.trans == 0 else (K - 1) * b.ld + N - 1), "B")
        cmax = (b1 - 1) * c.s1 + (b2 - 1) * c.s2 + (M - 1) * c.ld + N - 1
        for nm, t in (("C", c.t), ("R", R), ("Zout", Zout), ("Zin", Zin)):
            _need(t, cmax, nm)
        d = L.GemmDesc(a.t.data_ptr(), b.t.data_ptr(), c.t.data_ptr(), L.ptr(R), L.ptr(Zout), L.ptr(Zin),
                       a.ld, b.ld, c.ld, a.s1, a.s2, b.s1, b.s2, c.s1, c.s2, M, N, K, b1, b2,
                       a.trans, b.trans, int(out_f32), ACTS[act], int(act_bwd), float(alpha), float(beta), int(tri),
                       int(kin), int(a_sk), int(b_sk))
        L.check(L.lib().obst_gemm(d, L.stream_ptr()), "gemm")
        return c.t
    # ---- torch oracle
    if kin:
        ko = K // kin
        av = torch.as_strided(a.t, (b1, b2, M, ko, kin), (a.s1, a.s2, a.ld, a_sk, 1),
                              a.t.storage_offset()).reshape(b1, b2, M, K)
        bv = torch.as_strided(b.t, (b1, b2, N, ko, kin), (b.s1, b.s2, b.ld, b_sk, 1),
                              b.t.storage_offset()).reshape(b1, b2, N, K).transpose(2, 3)
    else:
        av = torch.as_strided(a.t, (b1, b2, M, K), (a.s1, a.s2, a.ld, 1) if a.trans == 0 else (a.s1, a.s2, 1, a.ld),
                              a.t.storage_offset())
        bv = torch.as_strided(b.t, (b1, b2, K, N), (b.s1, b.s2, 1, b.ld) if b.trans == 0 else (b.s1, b.s2, b.ld, 1),
                              b.t.storage_offset())
    shape, strides = (b1, b2, M, N), (c.s1, c.s2, c.ld, 1)

    def view(t):
        return None if t is None else torch.as_strided(t, shape, strides, t.storage_offset())

    cv = view(c.t)
    acc = torch.matmul(_f(av), _f(bv)) * alpha
    if tri == 3:
        acc = acc * torch.ones(M, N, dtype=acc.dtype, device=acc.device).tril()
    if act_bwd:
        if R is not None:
            acc = acc + _f(view(R))
        acc = acc * act_grad_t(act, _f(view(Zin)))
    else:
        if beta != 0.0:
            acc = acc + beta * _f(cv)
        if R is not None:
            acc = acc + _f(view(R))
        if Zout is not None:
            view(Zout).copy_(acc)
        acc = act_fwd_t(act, acc)
    cv.copy_(acc)
    return c.t


# ----------------------------------------------------------------------------------------------------------------
# flash attention on token-major [B, S, H, D] tensors with row stride ld (elements)
def _bshd(t: torch.Tensor, B, S, H, D, ld):
    return torch.as_strided(t, (B, S, H, D), (S * ld, ld, D, 1), t.storage_offset())


def attn_fwd(q, k, v, o, lse, B, S, H, D, ld, scale: float, causal: bool, ld_o: int = 0, residual=None, out=None):
    """ld: token stride of q / k / v (H*D, or 3*H*D for an interleaved k|q|v buffer); ld_o: that of o (0: ld).
    residual / out (optional, o's layout): the epilogue also writes out = bf16(o) + residual (the block's residual
    add, fused: o is still written -- the backward reads it)"""
    if q.device.type == "meta":
        return None
    ld_o = ld_o or ld
    if (residual is None) != (out is None):
        raise L.KernelError("attention residual and out come together")
    if on_gpu(q):
        if D not in (32, 64, 96, 128):
            raise L.KernelError(f"attention head dim {D} not supported by the HIP kernel (32/64/96/128)")
        ts = (("q", q, ld), ("k", k, ld), ("v", v, ld), ("o", o, ld_o))
        if out is not None:
            ts += (("residual", residual, ld_o), ("out", out, ld_o))
        for nm, t, l in ts:
            if t.dtype != torch.bfloat16:
                raise L.KernelError(f"attention {nm} must be bf16")
            _need(t, (B * S - 1) * l + (H - 1) * D + D - 1, nm)
        _need(lse, B * H * S - 1, "lse")
        d = L.AttnDesc(q.data_ptr(), k.data_ptr(), v.data_ptr(), 0, 0, o.data_ptr(), 0, 0, 0, lse.data_ptr(), 0,
                       B, S, H, D, ld, float(scale), int(causal), ld_o, L.ptr(residual), L.ptr(out))
        L.check(L.lib().obst_attn_fwd(d, L.stream_ptr()), "attn_fwd")
        return
    qv, kv, vv = (_f(_bshd(t, B, S, H, D, ld)) for t in (q, k, v))
    s = torch.einsum("bqhd,bkhd->bhqk", qv, kv) * scale
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    m = s.logsumexp(-1)
    p = torch.exp(s - m.unsqueeze(-1))
    _bshd(o, B, S, H, D, ld_o).copy_(torch.einsum("bhqk,bkhd->bqhd", p, vv))
    lse.view(B, H, S).copy_(m)
    if out is not None:
        _bshd(out, B, S, H, D, ld_o).copy_(_f(_bshd(o, B, S, H, D, ld_o)) + _f(_bshd(residual, B, S, H, D, ld_o)))


def attn_bwd(q, k, v, o, do, lse, delta, dq, dk, dv, B, S, H, D, ld, scale: float, causal: bool, ld_o: int = 0):
    """ld: token stride of q / k / v and dq / dk / dv; ld_o: that of o and do (0: ld)"""
    if q.device.type == "meta":
        return None
    ld_o = ld_o or ld
    if on_gpu(q):
        if D not in (32, 64, 96, 128):
            raise L.KernelError(f"attention head dim {D} not supported by the HIP kernel (32/64/96/128)")
        for nm, t, l in (("q", q, ld), ("k", k, ld), ("v", v, ld), ("o", o, ld_o), ("do", do, ld_o), ("dq", dq, ld),
                         ("dk", dk, ld), ("dv", dv, ld)):
            if t.dtype != torch.bfloat16:
                raise L.KernelError(f"attention {nm} must be bf16")
            _need(t, (B * S - 1) * l + (H - 1) * D + D - 1, nm)
        _need(lse, B * H * S - 1, "lse")
        _need(delta, B * H * S - 1, "delta")
        d = L.AttnDesc(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(), 0, dq.data_ptr(),
                       dk.data_ptr(), dv.data_ptr(), lse.data_ptr(), delta.data_ptr(), B, S, H, D, ld, float(scale),
                       int(causal), ld_o)
        L.check(L.lib().obst_attn_bwd(d, L.stream_ptr()), "attn_bwd")
        return
    qv, kv, vv = (_f(_bshd(t, B, S, H, D, ld)) for t in (q, k, v))
    ov, dov = (_f(_bshd(t, B, S, H, D, ld_o)) for t in (o, do))
    s = torch.einsum("bqhd,bkhd->bhqk", qv, kv) * scale
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    p = torch.exp(s - lse.view(B, H, S).unsqueeze(-1))
    dlt = (dov * ov).sum(-1).permute(0, 2, 1)  # [B,H,S]
    delta.view(B, H, S).copy_(dlt)
    _bshd(dv, B, S, H, D, ld).copy_(torch.einsum("bhqk,bqhd->bkhd", p, dov))
    dp = torch.einsum("bqhd,bkhd->bhqk", dov, vv)
    ds = p * (dp - dlt.unsqueeze(-1))
    _bshd(dq, B, S, H, D, ld).copy_(torch.einsum("bhqk,bkhd->bqhd", ds, kv) * scale)
    _bshd(dk, B, S, H, D, ld).copy_(torch.einsum("bhqk,bqhd->bkhd", ds, qv) * scale)


# ----------------------------------------------------------------------------------------------------------------
# attention with learned per-head maps (csrc/kernels/attn_map.hip): contiguous [B, S, H, D] q / k / v / o, fp32
# [H, S, S] maps -- bias added to the scaled logits before the softmax, cmap multiplied into the probabilities after it
def attn_map_bsplit(B: int, S: int, H: int) -> int:
    """batch slices of the dk/dv kernel (= partial map gradients the host allocates)"""
    return int(L.lib().obst_attn_map_bsplit(B, S, H))


def _map_logits(q, k, bias, B, S, H, D, scale, causal):
    s = torch.einsum("bqhd,bkhd->bhqk", _f(q.view(B, S, H, D)), _f(k.view(B, S, H, D))) * scale
    if bias is not None:
        s = s + _f(bias).unsqueeze(0)
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    return s


# OBST_MAP_FLASH (default 1): the bias-only D = 128 map forward (S % 128 == 0) on the flash kernel; 0: attn_map.hip
_MAP_FLASH = __import__("os").environ.get("OBST_MAP_FLASH", "1") != "0"
map_flash_bwd_calls = 0
map_flash_calls = 0   # (tests: forwards that took the flash path)


def attn_map_fwd(q, k, v, o, lse, bias, cmap, B, S, H, D, scale: float, causal: bool):
    if q.device.type == "meta":
        return None
    if on_gpu(q):
        if D not in (32, 64, 96, 128):
            raise L.KernelError(f"attention head dim {D} not supported by the HIP kernel (32/64/96/128)")
        for nm, t in (("q", q), ("k", k), ("v", v), ("o", o)):
            if t.dtype != torch.bfloat16 or not t.is_contiguous():
                raise L.KernelError(f"attention map {nm} must be contiguous bf16")
            _need(t, B * S * H * D - 1, nm)
        for nm, t in (("bias", bias), ("cmap", cmap)):
            if t is not None:
                if t.dtype != torch.float32 or not t.is_contiguous():
                    raise L.KernelError(f"attention map {nm} must be contiguous fp32")
                _need(t, H * S * S - 1, nm)
        _need(lse, B * H * S - 1, "lse")
        if _MAP_FLASH and bias is not None and cmap is None and D == 128 and S % 128 == 0:
            # biased_softmax on the flash forward (attention.hip attn_fwd32_kernel with the map hook); the map
            # kernels' backward consumes its o / lse unchanged
            global map_flash_calls
            map_flash_calls += 1
            d = L.AttnDesc(q.data_ptr(), k.data_ptr(), v.data_ptr(), 0, 0, o.data_ptr(), 0, 0, 0, lse.data_ptr(), 0,
                           B, S, H, D, H * D, float(scale), int(causal), H * D, 0, 0)
            L.check(L.lib().obst_attn_fwd_bias(d, bias.data_ptr(), L.stream_ptr()), "attn_fwd_bias")
            return
        d = L.MapDesc(q.data_ptr(), k.data_ptr(), v.data_ptr(), 0, 0, o.data_ptr(), 0, 0, 0, L.ptr(bias), L.ptr(cmap),
                      0, 0, 0, 0, lse.data_ptr(), 0, B, S, H, D, 1, float(scale), int(causal))
        L.check(L.lib().obst_attn_map_fwd(d, L.stream_ptr()), "attn_map_fwd")
        return
    s = _map_logits(q, k, bias, B, S, H, D, scale, causal)
    m = s.logsumexp(-1)
    p = torch.exp(s - m.unsqueeze(-1))
    if cmap is not None:
        p = p * _f(cmap).unsqueeze(0)
    o.view(B, S, H, D).copy_(torch.einsum("bhqk,bkhd->bqhd", p, _f(v.view(B, S, H, D))))
    lse.view(B, H, S).copy_(m)


def attn_map_flash_bwd(B: int, S: int, H: int, D: int, has_bias: bool, has_cmap: bool) -> bool:
    """biased_softmax backward on the flash kernels (attention.hip, map hook): bias only, D = 128, S % 128 == 0, and
    the per-batch partial map gradients ([B, H, S, S] fp32) within 16 GiB"""
    return (_MAP_FLASH and has_bias and not has_cmap and D == 128 and S % 128 == 0
            and B * H * S * S * 4 <= 16 << 30)


def attn_map_bwd(q, k, v, o, do, lse, delta, dq, dk, dv, bias, cmap, dbias, dcmap, B, S, H, D, scale: float,
                 causal: bool, dbias_part=None, dcmap_part=None):
    """dbias / dcmap: [H, S, S] fp32 outputs (None: not needed); *_part: zeroed [bsplit, H, S, S] partial maps the
    dk/dv kernel accumulates into (GPU; None when bsplit == 1 -- the kernel then accumulates into a zeroed dbias)"""
    if q.device.type == "meta":
        return None
    if on_gpu(q):
        if D not in (32, 64, 96, 128):
            raise L.KernelError(f"attention head dim {D} not supported by the HIP kernel (32/64/96/128)")
        for nm, t in (("q", q), ("k", k), ("v", v), ("o", o), ("do", do), ("dq", dq), ("dk", dk), ("dv", dv)):
            if t.dtype != torch.bfloat16 or not t.is_contiguous():
                raise L.KernelError(f"attention map {nm} must be contiguous bf16")
            _need(t, B * S * H * D - 1, nm)
        bsplit = attn_map_bsplit(B, S, H)
        for nm, t in (("bias", bias), ("cmap", cmap), ("dbias", dbias), ("dcmap", dcmap)):
            if t is not None:
                if t.dtype != torch.float32 or not t.is_contiguous():
                    raise L.KernelError(f"attention map {nm} must be contiguous fp32")
                _need(t, H * S * S - 1, nm)
        if attn_map_flash_bwd(B, S, H, D, bias is not None, cmap is not None):
            # dQ and dK/dV kernels of the main flash backward with the map hook; dS per batch into dbias_part
            # ([B, H, S, S], written whole over the causal triangle: no zeroing), folded over the batch in order
            global map_flash_bwd_calls
            map_flash_bwd_calls += 1
            if dbias is None:
                dbias = torch.empty(H, S, S, device=q.device)
            if dbias_part is None or dbias_part.numel() < B * H * S * S:
                dbias_part = torch.empty(B, H, S, S, device=q.device)
            if dbias_part.dtype != torch.float32 or not dbias_part.is_contiguous():
                raise L.KernelError("attention map dbias_part must be contiguous fp32")
            _need(dbias_part, B * H * S * S - 1, "dbias_part")
            _need(lse, B * H * S - 1, "lse")
            _need(delta, B * H * S - 1, "delta")
            d = L.AttnDesc(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(), 0, dq.data_ptr(),
                           dk.data_ptr(), dv.data_ptr(), lse.data_ptr(), delta.data_ptr(), B, S, H, D, H * D,
                           float(scale), int(causal), H * D, 0, 0)
            L.check(L.lib().obst_attn_bwd_bias(d, bias.data_ptr(), dbias_part.data_ptr(), dbias.data_ptr(),
                                               L.stream_ptr()), "attn_bwd_bias")
            return
        # the kernels accumulate the gradient of every present map (one instantiation per map set): a map whose
        # gradient is not wanted gets a scratch output
        if bias is not None and dbias is None:
            dbias = torch.empty(H, S, S, device=q.device)
            dbias_part = torch.zeros(bsplit, H, S, S, device=q.device) if bsplit > 1 else None
        if cmap is not None and dcmap is None:
            dcmap = torch.empty(H, S, S, device=q.device)
            dcmap_part = torch.zeros(bsplit, H, S, S, device=q.device) if bsplit > 1 else None
        parts = []
        for nm, out, part in (("dbias", dbias, dbias_part), ("dcmap", dcmap, dcmap_part)):
            if out is None:
                parts.append(None)
                continue
            if bsplit == 1:
                out.zero_()
                parts.append(out)
                continue
            if part is None or part.dtype != torch.float32 or not part.is_contiguous():
                raise L.KernelError(f"attention map {nm}: a zeroed fp32 [{bsplit}, H, S, S] partial buffer is needed")
            _need(part, bsplit * H * S * S - 1, nm + "_part")
            parts.append(part)
        _need(lse, B * H * S - 1, "lse")
        _need(delta, B * H * S - 1, "delta")
        d = L.MapDesc(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(), 0, dq.data_ptr(),
                      dk.data_ptr(), dv.data_ptr(), L.ptr(bias), L.ptr(cmap), L.ptr(parts[0]), L.ptr(parts[1]),
                      L.ptr(dbias), L.ptr(dcmap), lse.data_ptr(), delta.data_ptr(), B, S, H, D, bsplit, float(scale),
                      int(causal))
        L.check(L.lib().obst_attn_map_bwd(d, L.stream_ptr()), "attn_map_bwd")
        return
    s = _map_logits(q, k, bias, B, S, H, D, scale, causal)
    p = torch.exp(s - lse.view(B, H, S).unsqueeze(-1))
    c = _f(cmap).unsqueeze(0) if cmap is not None else None
    qv, kv, vv = (_f(t.view(B, S, H, D)) for t in (q, k, v))
    dov = _f(do.view(B, S, H, D))
    dlt = (dov * _f(o.view(B, S, H, D))).sum(-1).permute(0, 2, 1)
    delta.view(B, H, S).copy_(dlt)
    pc = p * c if c is not None else p
    dv.view(B, S, H, D).copy_(torch.einsum("bhqk,bqhd->bkhd", pc, dov))
    dp = torch.einsum("bqhd,bkhd->bhqk", dov, vv)
    ds = p * ((dp * c if c is not None else dp) - dlt.unsqueeze(-1))
    dq.view(B, S, H, D).copy_(torch.einsum("bhqk,bkhd->bqhd", ds, kv) * scale)
    dk.view(B, S, H, D).copy_(torch.einsum("bhqk,bqhd->bkhd", ds, qv) * scale)
    if dbias is not None:
        dbias.copy_(ds.sum(0))
    if dcmap is not None:
        dcmap.copy_((p * dp).sum(0))


# ----------------------------------------------------------------------------------------------------------------
# norm (reference normalization.py:22-34); x viewed as [rows, F], params indexed by row % groups
EPS = 1e-5


def norm_fwd(x, scale, shift, y, stats, rows: int, F: int, groups: int, ext_stats=None, act=None):
    """y = norm(x) * scale + shift per row (groups: row % groups selects the parameter row); act: a following
    activation fused, y = act(...)"""
    if x.device.type == "meta":
        return None
    if on_gpu(x):
        if x.dtype != torch.bfloat16:
            raise L.KernelError("norm input must be bf16 on the GPU")
        for nm, t in (("x", x), ("y", y)):
            _need(t, rows * F - 1, nm)
        _need(stats, 2 * rows - 1, "stats")
        for nm, t in (("scale", scale), ("shift", shift)):
            if t is not None:
                if t.dtype != torch.float32:
                    raise L.KernelError("norm scale/shift must be fp32 master views")
                _need(t, groups * F - 1, nm)
        d = L.NormDesc(x.data_ptr(), L.ptr(scale), L.ptr(shift), y.data_ptr(), L.ptr(stats), 0, 0, 0, 0, 0,
                       L.ptr(ext_stats), rows, F, groups, F, EPS)
        d.act = ACTS[act]
        L.check(L.lib().obst_norm_fwd(d, L.stream_ptr()), "norm_fwd")
        return
    xv = _f(x.reshape(rows, F))
    if ext_stats is not None:
        mean, rstd = ext_stats.view(rows, 2)[:, 0:1], ext_stats.view(rows, 2)[:, 1:2]
    else:
        mean = xv.mean(-1, keepdim=True)
        rstd = torch.rsqrt(((xv - mean) ** 2).mean(-1, keepdim=True) + EPS)
    out = (xv - mean) * rstd
    g = torch.arange(rows, device=x.device) % groups
    if scale is not None:
        out = out * scale.reshape(groups, F)[g]
    if shift is not None:
        out = out + shift.reshape(groups, F)[g]
    y.reshape(rows, F).copy_(act_fwd_t(act, out))
    if stats is not None:
        stats.view(rows, 2).copy_(torch.cat([mean, rstd], -1))


def norm_partial(x, out, rows: int, F: int):
    """per-row (sum x, sum x^2) of this rank's slice (TP statistics, collective X05)"""
    if x.device.type == "meta":
        return None
    if on_gpu(x):
        _need(x, rows * F - 1, "x")
        _need(out, 2 * rows - 1, "out")
        d = L.NormDesc(x.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0, out.data_ptr(), 0, rows, F, 1, F, EPS)
        L.check(L.lib().obst_norm_partial(d, L.stream_ptr()), "norm_partial")
        return
    xv = _f(x.reshape(rows, F))
    out.view(rows, 2).copy_(torch.stack([xv.sum(-1), (xv * xv).sum(-1)], -1))


def norm_bwd(x, dy, scale, stats, dx, dscale, dshift, rows: int, F: int, groups: int, Ffull: int = 0,
             partial=None, ext_dsum=None, R=None, R32=None, dx32=None, shift=None, act=None, in_relu=False):
    """dx (and parameter grads accumulated into fp32 dscale/dshift). With `partial` set, only the per-row partial
    sums (sum dxh, sum dxh*xh) are written (TP phase 1); phase 2 passes them back as `ext_dsum`. R (same layout as
    dx) is added to dx. R32 / dx32 (fp32, together, instead of R): dx32 = dx + R32 in fp32 and dx its bf16 copy (the
    RevNet stream gradient, F.GradSink). act (with the forward's shift): the norm's output went through that
    activation, dy is taken through act'(z) first (z recomputed from x, stats, scale, shift). in_relu: x was the
    relu output of the producing product, dx *= [x > 0] (that product's activation backward)."""
    if x.device.type == "meta":
        return None
    Ffull = Ffull or F
    if on_gpu(x):
        _need(x, rows * F - 1, "x")
        _need(dy, rows * F - 1, "dy")
        if dx is not None:
            _need(dx, rows * F - 1, "dx")
        _need(stats, 2 * rows - 1, "stats")
        for nm, t in (("scale", scale), ("dscale", dscale), ("dshift", dshift)):
            if t is not None:
                _need(t, groups * F - 1, nm)
        if R is not None:
            if R.dtype != torch.bfloat16 or not R.is_contiguous():
                raise L.KernelError("norm_bwd residual gradient must be contiguous bf16")
            _need(R, rows * F - 1, "R")
        if (R32 is None) != (dx32 is None) or (R32 is not None and (R is not None or act is not None or in_relu)):
            raise L.KernelError("norm_bwd: R32 and dx32 come together, without R or an activation")
        if act is not None and (partial is not None or ext_dsum is not None):
            raise L.KernelError("norm_bwd: no fused activation on the TP statistics path")
        if shift is not None:
            _need(shift, groups * F - 1, "shift")
        for nm, t in (("R32", R32), ("dx32", dx32)):
            if t is not None:
                if t.dtype != torch.float32 or not t.is_contiguous():
                    raise L.KernelError(f"norm_bwd {nm} must be contiguous fp32")
                _need(t, rows * F - 1, nm)
        d = L.NormDesc(x.data_ptr(), L.ptr(scale), 0, 0, stats.data_ptr(), dy.data_ptr(), L.ptr(dx), L.ptr(dscale),
                       L.ptr(dshift), L.ptr(partial), L.ptr(ext_dsum), rows, F, groups, Ffull, EPS, L.ptr(R))
        d.R32, d.DX32 = L.ptr(R32), L.ptr(dx32)
        d.shift, d.act, d.in_relu = L.ptr(shift), ACTS[act], int(bool(in_relu))
        nws = int(L.lib().obst_norm_bwd_ws(d))
        ws = torch.empty(max(nws, 1), dtype=torch.float32, device=x.device) if nws else None
        d.ws = L.ptr(ws)     # parameter-gradient partial slab, folded in a fixed order (no float atomics)
        L.check(L.lib().obst_norm_bwd(d, L.stream_ptr()), "norm_bwd")
        return
    xv = _f(x.reshape(rows, F))
    dyv = _f(dy.reshape(rows, F))
    st = stats.view(rows, 2)
    xh = (xv - st[:, 0:1]) * st[:, 1:2]
    g = torch.arange(rows, device=x.device) % groups
    gs = _f(scale.reshape(groups, F)[g]) if scale is not None else 1.0
    if act is not None:
        z = xh * gs + (_f(shift.reshape(groups, F)[g]) if shift is not None else 0.0)
        dyv = dyv * act_grad_t(act, z)
    dxh = dyv * gs
    if partial is not None:
        partial.view(rows, 2).copy_(torch.stack([dxh.sum(-1), (dxh * xh).sum(-1)], -1))
        return
    if dscale is not None:
        dscale.reshape(groups, F).index_add_(0, g, (dyv * xh).to(dscale.dtype))
    if dshift is not None:
        dshift.reshape(groups, F).index_add_(0, g, dyv.to(dshift.dtype))
    if ext_dsum is not None:
        s1, s2 = ext_dsum.view(rows, 2)[:, 0:1], ext_dsum.view(rows, 2)[:, 1:2]
    else:
        s1, s2 = dxh.sum(-1, keepdim=True), (dxh * xh).sum(-1, keepdim=True)
    out = st[:, 1:2] * (dxh - s1 / Ffull - xh * s2 / Ffull)
    if R is not None:
        out = out + _f(R.reshape(rows, F))
    if in_relu:
        out = out * (xv > 0).to(out.dtype)
    if R32 is not None:
        out = out + R32.reshape(rows, F).to(out.dtype)
        dx32.reshape(rows, F).copy_(out)
    dx.reshape(rows, F).copy_(out)


# ----------------------------------------------------------------------------------------------------------------
# elementwise
_EW = {"act": 0, "act_bwd": 1, "add": 2, "mul_scalar": 3, "dropout": 4, "axpby": 5, "mul": 6}


def elementwise(op: str, x, y, z=None, act=None, sptr=None, alpha=1.0, beta=1.0, seed=0, keep=1.0):
    """act: y=act(x); act_bwd: y = z * act'(x); add: y = x + z; mul_scalar: y = x * sptr[0];
    dropout: y = x * keep_mask / keep; axpby: y = alpha x + beta z; mul: y = x * z"""
    if x.device.type == "meta":
        return y
    n = x.numel()
    if on_gpu(x):
        for t in (x, y, z):
            if t is not None and (t.dtype != torch.bfloat16 or not t.is_contiguous()):
                raise L.KernelError("elementwise operands must be contiguous bf16 on the GPU")
            if t is not None:
                _need(t, n - 1, "ew")
        if n % 8:
            raise L.KernelError(f"elementwise size {n} must be a multiple of 8")
        d = L.EwDesc(x.data_ptr(), L.ptr(z), y.data_ptr(), L.ptr(sptr), n, _EW[op], ACTS[act], float(alpha),
                     float(beta), int(seed) & (2 ** 64 - 1), float(keep))
        L.check(L.lib().obst_elementwise(d, L.stream_ptr()), "elementwise")
        return y
    xf = _f(x)
    if op == "act":
        r = act_fwd_t(act, xf)
    elif op == "act_bwd":
        r = _f(z) * act_grad_t(act, xf)
    elif op == "add":
        r = xf + _f(z)
    elif op == "mul_scalar":
        r = xf * _f(sptr.reshape(-1)[0])
    elif op == "dropout":
        r = xf * (dropout_mask(n, seed, keep, x.device).view_as(xf)) / keep
    elif op == "axpby":
        r = alpha * xf + beta * _f(z)
    elif op == "mul":
        r = xf * _f(z)
    else:
        raise ValueError(op)
    y.copy_(r.view_as(y))
    return y


def dropout_mask(n: int, seed: int, keep: float, device) -> torch.Tensor:
    """The same counter-based hash as the kernel (splitmix64 finaliser), so CPU and GPU masks agree."""
    u = hash_u24(torch.arange(n, dtype=torch.int64, device=device), seed).double() / 16777216.0
    return (u < keep).to(torch.float32)


def hash_u24(i: torch.Tensor, seed: int) -> torch.Tensor:
    """top 24 bits of the splitmix64 finaliser of (i * golden ^ seed): the kernels' counter RNG (int64 tensor)"""
    device = i.device
    m64 = (1 << 64) - 1

    def _u(v):
        return torch.tensor(v - (1 << 64) if v >= (1 << 63) else v, dtype=torch.int64, device=device)

    h = (i * _u(0x9E3779B97F4A7C15)) ^ _u(seed & m64)

    def srl(v, k):  # logical shift right on int64
        return (v >> k) & ((1 << (64 - k)) - 1)
    h = h ^ srl(h, 33)
    h = h * _u(0xff51afd7ed558ccd)
    h = h ^ srl(h, 33)
    h = h * _u(0xc4ceb9fe1a85ec53)
    h = h ^ srl(h, 33)
    return srl(h, 40)


def dot(x, dy, out):
    """out[0] += sum(x * dy)"""
    if x.device.type == "meta":
        return None
    if on_gpu(x):
        n = x.numel()
        if n % 8:
            raise L.KernelError("dot size must be a multiple of 8")
        part = torch.empty(int(L.lib().obst_dot_parts(n)), dtype=torch.float32, device=x.device)
        L.check(L.lib().obst_dot(x.data_ptr(), dy.data_ptr(), out.data_ptr(), part.data_ptr(), n, L.stream_ptr()),
                "dot")
        return
    out.view(-1)[0] += (_f(x) * _f(dy)).sum()


def mix_f32(x, z, alpha: float, beta: float, y=None, yb=None):
    """y(fp32) = alpha * x(fp32) + beta * z(low precision); optionally also writes the bf16 copy `yb`"""
    if y is None:
        y = torch.empty_like(x)
    if x.device.type == "meta":
        return y
    if on_gpu(x) and z.dtype == torch.bfloat16 and x.dtype == torch.float32 and x.numel() % 8 == 0:
        x, z = x.contiguous(), z.contiguous()       # raw pointers below: block outputs may be permuted views
        if z.shape != x.shape:
            z = z.reshape(x.shape)
        L.check(L.lib().obst_mix_f32(x.data_ptr(), z.data_ptr(), y.data_ptr(), L.ptr(yb), x.numel(), float(alpha),
                                     float(beta), L.stream_ptr()), "mix_f32")
        return y
    torch.add(x * alpha, z.to(x.dtype), alpha=beta, out=y)
    if yb is not None:
        yb.copy_(y)
    return y


def add_to_bf16(a, b, out=None):
    """bf16(a + b) of two fp32 tensors in one pass on the GPU (HIP add2 kernel); a + b then a cast elsewhere"""
    if out is None:
        out = torch.empty(a.shape, dtype=torch.bfloat16, device=a.device)
    if a.device.type == "meta":
        return out
    if on_gpu(a) and a.dtype == torch.float32 and b.dtype == torch.float32 and a.shape == b.shape:
        a, b = a.contiguous(), b.contiguous()
        L.check(L.lib().obst_add2_f32_bf16(a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), L.stream_ptr()),
                "add2_f32_bf16")
        return out
    out.copy_(a + b)
    return out


def to_f32(x, out=None):
    """bf16 -> fp32 copy through the HIP cast kernel on the GPU"""
    if out is None:
        out = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    if on_gpu(x) and x.dtype == torch.bfloat16 and x.numel() % 8 == 0:
        x = x.contiguous()
        L.check(L.lib().obst_cast_bf16_f32(x.data_ptr(), out.data_ptr(), x.numel(), L.stream_ptr()), "cast")
        return out
    out.copy_(x)
    return out


def tril(x):
    """lower triangle (diagonal included) of the trailing S x S of x: one HIP pass for bf16 on the GPU"""
    S = x.shape[-1]
    if on_gpu(x) and x.dtype == torch.bfloat16 and x.shape[-2] == S and S % 8 == 0:
        x = x.contiguous()
        y = torch.empty_like(x)
        L.check(L.lib().obst_tril(x.data_ptr(), y.data_ptr(), S, x.numel() // (S * S), L.stream_ptr()), "tril")
        return y
    return torch.tril(x)


_ZERO_MEMSET = __import__("os").environ.get("OBST_ZERO_MEMSET", "1") != "0"


def zero_(t):
    """t[:] = 0 (contiguous): the runtime's memset on the GPU (OBST_ZERO_MEMSET=0: torch's fill)"""
    if _ZERO_MEMSET and on_gpu(t) and t.is_contiguous():
        L.check(L.lib().obst_zero(t.data_ptr(), t.numel() * t.element_size(), L.stream_ptr()), "zero")
        return t
    return t.zero_()


def to_bf16(x, out=None):
    """fp32 -> bf16 copy through the HIP cast kernel on the GPU"""
    if out is None:
        out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    if on_gpu(x) and x.dtype == torch.float32:
        x = x.contiguous()
        L.check(L.lib().obst_cast_f32_bf16(x.data_ptr(), out.data_ptr(), x.numel(), L.stream_ptr()), "cast")
        return out
    out.copy_(x)
    return out


def transpose(x, y, rows: int, cols: int, ldx: int, ldy: int, batch: int = 1, sx: int = 0, sy: int = 0):
    """y[b][c][r] = x[b][r][c] (bf16 on the GPU; any dtype on the CPU)"""
    if x.device.type == "meta":
        return None
    if on_gpu(x):
        if x.dtype != torch.bfloat16 or y.dtype != torch.bfloat16:
            raise L.KernelError("transpose is bf16")
        _need(x, (batch - 1) * sx + (rows - 1) * ldx + cols - 1, "x")
        _need(y, (batch - 1) * sy + (cols - 1) * ldy + rows - 1, "y")
        L.check(L.lib().obst_transpose(x.data_ptr(), y.data_ptr(), rows, cols, ldx, ldy, batch, sx, sy,
                                       L.stream_ptr()), "transpose")
        return
    xv = torch.as_strided(x, (batch, rows, cols), (sx, ldx, 1), x.storage_offset())
    yv = torch.as_strided(y, (batch, cols, rows), (sy, ldy, 1), y.storage_offset())
    yv.copy_(xv.transpose(1, 2))


def copy2d(x, y, rows: int, cols: int, ldx: int, ldy: int, batch: int = 1, sx: int = 0, sy: int = 0):
    """y[b][r][c] = x[b][r][c] between strided layouts (bf16 HIP kernel on the GPU; any dtype on the CPU)"""
    if x.device.type == "meta":
        return None
    if on_gpu(x):
        if x.dtype != torch.bfloat16 or y.dtype != torch.bfloat16:
            raise L.KernelError("copy2d is bf16")
        _need(x, (batch - 1) * sx + (rows - 1) * ldx + cols - 1, "x")
        _need(y, (batch - 1) * sy + (rows - 1) * ldy + cols - 1, "y")
        L.check(L.lib().obst_copy2d(x.data_ptr(), y.data_ptr(), rows, cols, ldx, ldy, batch, sx, sy,
                                    L.stream_ptr()), "copy2d")
        return
    xv = torch.as_strided(x, (batch, rows, cols), (sx, ldx, 1), x.storage_offset())
    yv = torch.as_strided(y, (batch, rows, cols), (sy, ldy, 1), y.storage_offset())
    yv.copy_(xv)


def gather(idx, table, out, T: int, F: int, V: int):
    if table.device.type == "meta":
        return None
    if on_gpu(table):
        if idx.dtype != torch.int32:
            raise L.KernelError("gather indices must be int32")
        _need(idx, T - 1, "idx")
        _need(table, V * F - 1, "table")
        _need(out, T * F - 1, "out")
        L.check(L.lib().obst_gather(idx.data_ptr(), table.data_ptr(), out.data_ptr(), T, F, V, L.stream_ptr()),
                "gather")
        return
    out.reshape(T, F).copy_(table.reshape(V, F)[idx.reshape(T).long().clamp(0, V - 1)])


def scatter_add(idx, dy, dtable, T: int, F: int, V: int):
    if dy.device.type == "meta":
        return None
    if on_gpu(dy):
        _need(idx, T - 1, "idx")
        _need(dy, T * F - 1, "dy")
        _need(dtable, V * F - 1, "dtable")
        if F % 8 == 0 and dy.data_ptr() % 16 == 0 and dtable.data_ptr() % 16 == 0:
            # deterministic: stable sort of the (clamped) ids, then fixed 64-row chunks of the sorted order with a
            # fixed-order fold of the runs that cross chunks (bounded work per block under skewed ids)
            sidx, perm = torch.sort(idx.reshape(-1)[:T].clamp(0, V - 1).to(torch.int32), stable=True)
            sorted_scatter(sidx, perm, dy, None, dtable, T, F)
            return
        L.check(L.lib().obst_scatter_add(idx.data_ptr(), dy.data_ptr(), dtable.data_ptr(), T, F, V, L.stream_ptr()),
                "scatter_add")
        return
    dtable.reshape(V, F).index_add_(0, idx.reshape(T).long().clamp(0, V - 1), _f(dy.reshape(T, F)).to(dtable.dtype))


_SCATTER_WS = {}


def sorted_scatter(sidx, perm, dy, scale, dtable, T: int, F: int):
    """dtable[sidx[i]] += dy[perm[i]] (* scale[perm[i]]) for stable-sorted int32 ids sidx and int64 perm: the
    deterministic chunked scatter (csrc/kernels/elementwise.hip scatter_chunk / scatter_fold)"""
    n = int(L.lib().obst_scatter_ws(T, F))
    ws = _SCATTER_WS.get(dy.device)
    if ws is None or ws.numel() < n:
        ws = torch.empty(max(n, 1 << 16), dtype=torch.float32, device=dy.device)
        _SCATTER_WS[dy.device] = ws
    L.check(L.lib().obst_scatter_add_chunked(sidx.data_ptr(), perm.data_ptr(), dy.data_ptr(), L.ptr(scale),
                                             dtable.data_ptr(), T, F, ws.data_ptr(), L.stream_ptr()),
            "scatter_add_chunked")


def cumsum(x, y, outer: int, S: int, inner: int, reverse: bool, mean: bool, grad: bool):
    if x.device.type == "meta":
        return None
    if on_gpu(x):
        _need(x, outer * S * inner - 1, "x")
        _need(y, outer * S * inner - 1, "y")
        L.check(L.lib().obst_cumsum(x.data_ptr(), y.data_ptr(), outer, S, inner, int(reverse), int(mean), int(grad),
                                    L.stream_ptr()), "cumsum")
        return
    xv = _f(x.reshape(outer, S, inner))
    pos = torch.arange(1, S + 1, device=x.device, dtype=torch.float32).view(1, S, 1)
    if mean and grad:
        xv = xv / pos
    if reverse:
        r = xv.flip(1).cumsum(1).flip(1)
    else:
        r = xv.cumsum(1)
    if mean and not grad:
        r = r / pos
    y.reshape(outer, S, inner).copy_(r)


def xent_fwd(logits, tgt, lse, loss, hit, rows: int, V: int, Vp: int, z_loss: float):
    if logits.device.type == "meta":
        return None
    if on_gpu(logits):
        if tgt.dtype != torch.int32:
            raise L.KernelError("targets must be int32")
        _need(logits, rows * Vp - 1, "logits")
        for nm, t in (("tgt", tgt), ("lse", lse), ("loss", loss), ("hit", hit)):
            _need(t, rows - 1, nm)
        L.check(L.lib().obst_xent_fwd(logits.data_ptr(), tgt.data_ptr(), lse.data_ptr(), loss.data_ptr(),
                                      hit.data_ptr(), rows, V, Vp, float(z_loss), L.stream_ptr()), "xent_fwd")
        return
    lv = _f(logits.reshape(rows, Vp)[:, :V])
    t = tgt.reshape(rows).long()
    m = lv.logsumexp(-1)
    ly = lv.gather(1, t.clamp(0, V - 1).unsqueeze(1)).squeeze(1)
    lse.copy_(m)
    loss.copy_(-(ly - m) + z_loss * m * m)
    hit.copy_((lv.argmax(-1) == t).to(hit.dtype))


def xent_bwd(logits, tgt, lse, grad, gscale_ptr, gscale: float, rows: int, V: int, Vp: int, z_loss: float):
    if logits.device.type == "meta":
        return None
    if on_gpu(logits):
        _need(logits, rows * Vp - 1, "logits")
        _need(grad, rows * Vp - 1, "grad")
        L.check(L.lib().obst_xent_bwd(logits.data_ptr(), tgt.data_ptr(), lse.data_ptr(), grad.data_ptr(),
                                      L.ptr(gscale_ptr), float(gscale), rows, V, Vp, float(z_loss), L.stream_ptr()),
                "xent_bwd")
        return
    lv = _f(logits.reshape(rows, Vp))
    p = torch.exp(lv - lse.view(rows, 1))
    p[:, V:] = 0
    g = gscale * (_f(gscale_ptr.reshape(-1)[0]) if gscale_ptr is not None else 1.0)
    d = p * (1 + 2 * z_loss * lse.view(rows, 1))
    d[torch.arange(rows, device=lv.device), tgt.reshape(rows).long()] -= 1
    grad.reshape(rows, Vp).copy_(d * g)


# ----------------------------------------------------------------------------------------------------------------
# block-grammar ops off the GPT-Neo hot path (csrc/kernels/aux_ops.hip); bf16 on the GPU, torch oracles elsewhere
def _bf16_contig(name: str, *ts):
    for t in ts:
        if t is not None and (t.dtype != torch.bfloat16 or not t.is_contiguous()):
            raise L.KernelError(f"{name} operands must be contiguous bf16 on the GPU")


def glu(a, g, y, dy=None, dg=None):
    """dy None: y = a * sigmoid(g); else y = da = dy * s(g), dg = dy * a * s (1 - s)"""
    if a.device.type == "meta":
        return None
    n = a.numel()
    if on_gpu(a):
        _bf16_contig("glu", a, g, y, dy, dg)
        for nm, t in (("a", a), ("g", g), ("y", y), ("dy", dy), ("dg", dg)):
            _need(t, n - 1, nm)
        if n % 8:
            raise L.KernelError(f"glu size {n} must be a multiple of 8")
        L.check(L.lib().obst_glu(a.data_ptr(), g.data_ptr(), L.ptr(dy), y.data_ptr(), L.ptr(dg), n,
                                 L.stream_ptr()), "glu")
        return None
    s = torch.sigmoid(_f(g))
    if dy is None:
        y.copy_(_f(a) * s)
        return None
    d = _f(dy)
    y.copy_(d * s)
    dg.copy_(d * _f(a) * s * (1 - s))
    return None


def pkm_top1(x, idx, val, stats, aidx, R: int, A: int, F: int):
    """x [R][A][F]: idx[r] = sum_a argmax_a * F^a, val[r] = prod_a softmax_a(argmax_a); stats [R][A][2] = (max, sum
    exp), aidx [R][A] kept for pkm_top1_bwd"""
    if x.device.type == "meta":
        return None
    if on_gpu(x):
        _bf16_contig("pkm_top1", x)
        _need(x, R * A * F - 1, "x")
        _need(stats, R * A * 2 - 1, "stats")
        _need(aidx, R * A - 1, "aidx")
        for nm, t in (("idx", idx), ("val", val)):
            _need(t, R - 1, nm)
        if idx.dtype != torch.int32 or aidx.dtype != torch.int32 or val.dtype != torch.float32:
            raise L.KernelError("pkm_top1: int32 indices and fp32 values")
        L.check(L.lib().obst_pkm_top1(x.data_ptr(), idx.data_ptr(), val.data_ptr(), stats.data_ptr(),
                                      aidx.data_ptr(), R, A, F, L.stream_ptr()), "pkm_top1")
        return None
    xv = _f(x.reshape(R, A, F))
    m, mi = xv.max(-1)
    s = torch.exp(xv - m.unsqueeze(-1)).sum(-1)
    mult = F ** torch.arange(A, device=x.device, dtype=torch.int64)
    idx.reshape(R).copy_((mi * mult).sum(-1))
    val.reshape(R).copy_((1.0 / s).prod(-1))
    stats.reshape(R, A, 2).copy_(torch.stack([m, s], -1))
    aidx.reshape(R, A).copy_(mi)
    return None


def pkm_top1_bwd(x, val, dval, stats, aidx, dx, R: int, A: int, F: int):
    if x.device.type == "meta":
        return None
    if on_gpu(x):
        _bf16_contig("pkm_top1_bwd", x, dx)
        _need(dx, R * A * F - 1, "dx")
        L.check(L.lib().obst_pkm_top1_bwd(x.data_ptr(), val.data_ptr(), dval.data_ptr(), stats.data_ptr(),
                                          aidx.data_ptr(), dx.data_ptr(), R, A, F, L.stream_ptr()), "pkm_top1_bwd")
        return None
    xv = _f(x.reshape(R, A, F))
    st = stats.reshape(R, A, 2).to(xv.dtype)
    p = torch.exp(xv - st[..., :1]) / st[..., 1:]
    hot = torch.nn.functional.one_hot(aidx.reshape(R, A).long(), F).to(xv.dtype)
    g = (dval.reshape(R) * val.reshape(R)).to(xv.dtype).view(R, 1, 1)
    dx.reshape(R, A, F).copy_(g * (hot - p))
    return None


def pkm_gather(idx, val, table, out, R: int, H: int, Fk: int, P: int):
    """out[r] = table[idx[r], r % H] * val[r]   (table [P][H][Fk])"""
    if table.device.type == "meta":
        return None
    if on_gpu(table):
        _bf16_contig("pkm_gather", table, out)
        _need(table, P * H * Fk - 1, "table")
        _need(out, R * Fk - 1, "out")
        _need(idx, R - 1, "idx")
        _need(val, R - 1, "val")
        L.check(L.lib().obst_pkm_gather(idx.data_ptr(), val.data_ptr(), table.data_ptr(), out.data_ptr(), R, H, Fk,
                                        P, L.stream_ptr()), "pkm_gather")
        return None
    rows = idx.reshape(R).long().clamp(0, P - 1) * H + torch.arange(R, device=idx.device) % H
    out.reshape(R, Fk).copy_(_f(table.reshape(P * H, Fk))[rows] * val.reshape(R, 1).to(_f(table).dtype))
    return None


def pkm_gather_bwd(idx, val, table, dy, dtable, dval, R: int, H: int, Fk: int, P: int):
    """dtable[idx[r], r % H] += dy[r] * val[r] (fp32); dval[r] = <dy[r], table[idx[r], r % H]>"""
    if table.device.type == "meta":
        return None
    if on_gpu(table):
        _bf16_contig("pkm_gather_bwd", table, dy)
        _need(dtable, P * H * Fk - 1, "dtable")
        _need(dy, R * Fk - 1, "dy")
        _need(dval, R - 1, "dval")
        det = Fk % 8 == 0 and dy.data_ptr() % 16 == 0 and dtable.data_ptr() % 16 == 0 and val.dtype == torch.float32
        L.check(L.lib().obst_pkm_gather_bwd(idx.data_ptr(), val.data_ptr(), table.data_ptr(), dy.data_ptr(),
                                            0 if det else dtable.data_ptr(), dval.data_ptr(), R, H, Fk, P,
                                            L.stream_ptr()), "pkm_gather_bwd")
        if det:   # dtable rows (value, head) through the deterministic sorted scatter, scaled by val
            rows = (idx.reshape(-1)[:R].long().clamp(0, P - 1) * H +
                    torch.arange(R, device=idx.device) % H).to(torch.int32)
            sidx, perm = torch.sort(rows, stable=True)
            sorted_scatter(sidx, perm, dy, val.reshape(-1), dtable, R, Fk)
        return None
    rows = idx.reshape(R).long().clamp(0, P - 1) * H + torch.arange(R, device=idx.device) % H
    d = _f(dy.reshape(R, Fk))
    dval.reshape(R).copy_((d * _f(table.reshape(P * H, Fk))[rows]).sum(-1))
    dtable.reshape(P * H, Fk).index_add_(0, rows, (d * val.reshape(R, 1).to(d.dtype)).to(dtable.dtype))
    return None


def moe_ok(E: int) -> bool:
    lanes = E // 8
    return E % 8 == 0 and 1 <= lanes <= 64 and lanes & (lanes - 1) == 0


def moe_fwd(u, lg, p, y, T: int, N: int, E: int):
    """p[t] = softmax(lg[t]) (fp32), y[t][n] = sum_e u[t][n][e] p[t][e]"""
    if u.device.type == "meta":
        return None
    if on_gpu(u):
        _bf16_contig("moe_fwd", u, lg, y)
        if not moe_ok(E):
            raise L.KernelError(f"moe kernel: experts {E} must be 8 * 2^k <= 512")
        _need(u, T * N * E - 1, "u")
        _need(lg, T * E - 1, "lg")
        _need(p, T * E - 1, "p")
        _need(y, T * N - 1, "y")
        L.check(L.lib().obst_moe_fwd(u.data_ptr(), lg.data_ptr(), p.data_ptr(), y.data_ptr(), T, N, E,
                                     L.stream_ptr()), "moe_fwd")
        return None
    lv = _f(lg.reshape(T, E))
    pv = torch.softmax(lv - lv.amax(-1, keepdim=True), -1)
    p.reshape(T, E).copy_(pv)
    y.reshape(T, N).copy_(torch.einsum("tne,te->tn", _f(u.reshape(T, N, E)), pv.to(_f(u).dtype)))
    return None


def moe_bwd(dy, u, p, du, dlg, T: int, N: int, E: int):
    """du = dy ⊗ p; dlg = p (dp - <p, dp>), dp[t][e] = sum_n dy[t][n] u[t][n][e]"""
    if u.device.type == "meta":
        return None
    if on_gpu(u):
        _bf16_contig("moe_bwd", dy, u, du, dlg)
        _need(du, T * N * E - 1, "du")
        _need(dlg, T * E - 1, "dlg")
        L.check(L.lib().obst_moe_bwd(dy.data_ptr(), u.data_ptr(), p.data_ptr(), du.data_ptr(), dlg.data_ptr(), T, N,
                                     E, L.stream_ptr()), "moe_bwd")
        return None
    d = _f(dy.reshape(T, N))
    pv = p.reshape(T, E).to(d.dtype)
    du.reshape(T, N, E).copy_(d.unsqueeze(-1) * pv.unsqueeze(1))
    dp = torch.einsum("tn,tne->te", d, _f(u.reshape(T, N, E)))
    dlg.reshape(T, E).copy_(pv * (dp - (pv * dp).sum(-1, keepdim=True)))
    return None


def sum_axis(x, y, outer: int, H: int, inner: int):
    """y[o][i] = sum_h x[o][h][i]"""
    if x.device.type == "meta":
        return None
    if on_gpu(x):
        _bf16_contig("sum_axis", x, y)
        if inner % 8:
            raise L.KernelError("sum_axis inner size must be a multiple of 8")
        _need(x, outer * H * inner - 1, "x")
        _need(y, outer * inner - 1, "y")
        L.check(L.lib().obst_sum_axis(x.data_ptr(), y.data_ptr(), outer, H, inner, L.stream_ptr()), "sum_axis")
        return None
    y.reshape(outer, inner).copy_(_f(x.reshape(outer, H, inner)).sum(1))
    return None


# ----------------------------------------------------------------------------------------------------------------
# K12 axial positional embedding: out[i_0, .., i_{k-1}, f] = prod_m t_m[i_m, f]  (k <= 4 factor tables [n_m, F])
def axial_fwd(tables, out, F: int):
    if out.device.type == "meta":
        return None
    if on_gpu(out):
        if not 1 <= len(tables) <= 4:
            raise L.KernelError("axial embedding: 1-4 factor tables")
        for t in tables:
            _bf16_contig("axial table", t)
        _bf16_contig("axial out", out)
        n = [t.numel() // F for t in tables]
        _need(out, math.prod(n) * F - 1, "out")
        ptrs = (ctypes.c_void_p * 4)(*([t.data_ptr() for t in tables] + [0] * (4 - len(tables))))
        ns = (ctypes.c_int * 4)(*(n + [1] * (4 - len(n))))
        L.check(L.lib().obst_axial_fwd(ptrs, ns, len(tables), F, out.data_ptr(), L.stream_ptr()), "axial_fwd")
        return None
    acc = None
    k = len(tables)
    for m, t in enumerate(tables):
        shape = [1] * k + [F]
        shape[m] = t.numel() // F
        v = _f(t).reshape(shape)
        acc = v if acc is None else acc * v
    out.view(acc.shape).copy_(acc)
    return None


def axial_bwd(tables, gout, grads, F: int):
    """grads[m] [n_m, F] fp32 <- sum over the other axes of gout * prod of the other tables"""
    if gout.device.type == "meta":
        return None
    if on_gpu(gout):
        for t in tables:
            _bf16_contig("axial table", t)
        _bf16_contig("axial grad", gout)
        n = [t.numel() // F for t in tables]
        for g, nm in zip(grads, n):
            if g.dtype != torch.float32 or not g.is_contiguous():
                raise L.KernelError("axial factor gradients must be contiguous fp32")
            _need(g, nm * F - 1, "grad")
        ptrs = (ctypes.c_void_p * 4)(*([t.data_ptr() for t in tables] + [0] * (4 - len(tables))))
        gp = (ctypes.c_void_p * 4)(*([g.data_ptr() for g in grads] + [0] * (4 - len(grads))))
        ns = (ctypes.c_int * 4)(*(n + [1] * (4 - len(n))))
        L.check(L.lib().obst_axial_bwd(ptrs, ns, len(tables), F, gout.data_ptr(), gp, L.stream_ptr()), "axial_bwd")
        return None
    k = len(tables)
    n = [t.numel() // F for t in tables]
    go = _f(gout).reshape(n + [F])
    vs = []
    for m, t in enumerate(tables):
        shape = [1] * k + [F]
        shape[m] = n[m]
        vs.append(_f(t).reshape(shape))
    for m in range(k):
        prod = go
        for j in range(k):
            if j != m:
                prod = prod * vs[j]
        axes = [j for j in range(k) if j != m]
        grads[m].copy_((prod.sum(axes) if axes else prod).reshape(grads[m].shape))
    return None


def gumbel_scores(logits, temp, seed: int):
    """torch oracle of the sampling kernel's noisy scores: logit - T log(-log u), u = (hash24(r V + v) + 0.5) / 2^24"""
    rows, V = logits.shape
    i = torch.arange(rows * V, dtype=torch.int64, device=logits.device)
    u = (hash_u24(i, seed).to(torch.float32) + 0.5) / 16777216.0
    noise = torch.log(-torch.log(u)).view(rows, V)
    return logits.float() - temp.view(rows, 1).float() * noise


_SAMPLE_WS: typing.Dict[str, torch.Tensor] = {}


def _sample_ws(device, n: int) -> torch.Tensor:
    """per-device (value, index) partials of the split sampler, grown as needed and reused across steps"""
    key = str(device)
    t = _SAMPLE_WS.get(key)
    if t is None or t.numel() < n:
        t = torch.empty(n, dtype=torch.float32, device=device)
        _SAMPLE_WS[key] = t
    return t


def sample(logits, temp, pred, seed: int, x=None, pos=None, end=None, patch: int = 1):
    """pred[r] = argmax_v(logits[r][v] - temp[r // patch] log(-log u)); with x [B][S][patch] (int32) the winner is
    also written to x[b][min(pos_b, S-1)][r % patch] for rows whose pos_b < end_b"""
    rows, V = logits.shape
    B = rows // patch
    if on_gpu(logits):
        if logits.dtype != torch.float32 or not logits.is_contiguous():
            raise L.KernelError("sample: contiguous fp32 logits")
        if temp.dtype != torch.float32 or temp.numel() < B or pred.dtype != torch.int32 or pred.numel() < rows:
            raise L.KernelError("sample: fp32 temperatures [B], int32 predictions [rows]")
        S = 0
        if x is not None:
            if (x.dtype != torch.int32 or not x.is_contiguous() or x.numel() % (B * patch) or pos.dtype != torch.int64
                    or end.dtype != torch.int64 or pos.numel() < B or end.numel() < B):
                raise L.KernelError("sample: int32 token buffer, int64 pos / end")
            S = x.numel() // (B * patch)
        nb = int(L.lib().obst_sample_parts(rows, V))
        ws = _sample_ws(logits.device, rows * nb * 2) if nb > 1 else None
        L.check(L.lib().obst_sample(logits.data_ptr(), rows, V, patch, temp.data_ptr(), L.ptr(pos), L.ptr(end),
                                    L.ptr(x), S, pred.data_ptr(), int(seed) & (2 ** 64 - 1), L.ptr(ws),
                                    L.stream_ptr()), "sample")
        return pred
    t = temp.reshape(-1)[:B].repeat_interleave(patch)
    scores = gumbel_scores(logits, t, seed)
    scores = torch.where(t.view(rows, 1) == 0, logits.float(), scores)
    pred.copy_(scores.argmax(-1).to(pred.dtype))
    if x is not None:
        S = x.numel() // (B * patch)
        xv = x.view(B, S, patch)
        rb = torch.arange(B, device=x.device)
        wpos = pos.clamp(max=S - 1)
        cur = xv[rb, wpos]
        xv[rb, wpos] = torch.where((pos < end).view(B, 1), pred.view(B, patch).to(x.dtype), cur)
    return pred


def frames(v, y, rows: int, C: int, folds: int = 1, base: int = 256):
    """y[r][i * C + c] = ((v[r][c] // base^i) % base) / 255  (folds == 1: v / 255); v uint8 or int32"""
    if v.device.type == "meta":
        return None
    if on_gpu(v):
        if y.dtype != torch.bfloat16 or not y.is_contiguous() or not v.is_contiguous():
            raise L.KernelError("frames: contiguous input, bf16 output")
        nb = {torch.uint8: 1, torch.int32: 4}.get(v.dtype)
        if nb is None:
            raise L.KernelError(f"frames: uint8 or int32 input, got {v.dtype}")
        _need(v, rows * C - 1, "v")
        _need(y, rows * C * folds - 1, "y")
        L.check(L.lib().obst_frames(v.data_ptr(), nb, y.data_ptr(), rows, C, folds, base, L.stream_ptr()), "frames")
        return None
    vv = v.reshape(rows, C).long()
    if folds == 1:
        parts = [vv]
    else:
        parts = [(vv // base ** i) % base for i in range(folds)]
    y.reshape(rows, C * folds).copy_(torch.cat(parts, -1).to(y.dtype) / 255.0)
    return None


def l1(fo, g, mask, inner: int, loss=None, dfo=None, gptr=None, gscale: float = 1.0):
    """d = (fo - g) * mask[e // inner]; loss[0] += sum |d|  or (dfo given) dfo = sign(d) mask gscale (* gptr[0])"""
    if fo.device.type == "meta":
        return None
    n = fo.numel()
    if on_gpu(fo):
        _bf16_contig("l1", fo, g, dfo)
        _need(g, n - 1, "g")
        if mask is not None:
            if mask.dtype != torch.float32 or not mask.is_contiguous():
                raise L.KernelError("l1 mask must be contiguous fp32")
            _need(mask, (n - 1) // inner, "mask")
        L.check(L.lib().obst_l1(fo.data_ptr(), g.data_ptr(), L.ptr(mask), inner, n, L.ptr(loss), L.ptr(dfo),
                                L.ptr(gptr), float(gscale), L.stream_ptr()), "l1")
        return None
    m = 1.0 if mask is None else _f(mask).reshape(-1, 1)
    d = (_f(fo).reshape(-1, inner) - _f(g).reshape(-1, inner)) * m
    if dfo is None:
        loss.view(-1)[0] += d.abs().sum().to(loss.dtype)
        return None
    gs = gscale * (_f(gptr.reshape(-1)[0]) if gptr is not None else 1.0)
    dfo.reshape(-1, inner).copy_(torch.sign(d) * m * gs)
    return None


# OBST_DECODE_BLOCKS: target block count of the split-K decode attention (key chunks x B x H); A/B knob
_DEC_BLOCKS = int(__import__("os").environ.get("OBST_DECODE_BLOCKS", "2048"))


def decode_attn(q, kn, vn, k, v, o, pos, B: int, S: int, H: int, D: int, scale: float):
    """KV-cache decode step: k[b][pos_b] = kn[b], v[b][pos_b] = vn[b], then
    o[b][h] = softmax_j(scale q[b][h].k[b][j][h], j <= pos_b) . v[b][j][h]; q, kn, vn, o [B][H][D]; caches [B][S][H][D]"""
    if q.device.type == "meta":
        return None
    if on_gpu(q):
        _bf16_contig("decode_attn", q, kn, vn, k, v, o)
        if pos.dtype != torch.int64 or pos.numel() < B:
            raise L.KernelError("decode_attn: int64 positions [B]")
        for nm, t, n in (("q", q, B * H * D), ("kn", kn, B * H * D), ("vn", vn, B * H * D), ("k", k, B * S * H * D),
                         ("v", v, B * S * H * D), ("o", o, B * H * D)):
            _need(t, n - 1, nm)
        # key splits so that the grid has >= ~2048 blocks (8 per CU), each split >= 64 keys
        nsplit = max(1, min(-(-_DEC_BLOCKS // (B * H)), -(-S // 64))) if D % 8 == 0 else 1
        ws = torch.empty(B * H * nsplit * (D + 2) if nsplit > 1 else 1, dtype=torch.float32, device=q.device)
        L.check(L.lib().obst_decode_attn(q.data_ptr(), kn.data_ptr(), vn.data_ptr(), k.data_ptr(), v.data_ptr(),
                                         o.data_ptr(), pos.data_ptr(), B, S, H, D, float(scale), nsplit,
                                         ws.data_ptr(), L.stream_ptr()),
                "decode_attn")
        return None
    kc, vc = k.view(B, S, H, D), v.view(B, S, H, D)
    rows = torch.arange(B, device=q.device)
    ok = (pos >= 0) & (pos < S)
    kc[rows[ok], pos[ok]] = kn.reshape(B, H, D)[ok].to(kc.dtype)
    vc[rows[ok], pos[ok]] = vn.reshape(B, H, D)[ok].to(vc.dtype)
    qv = _f(q.reshape(B, H, D)) * scale
    s = torch.einsum("bhd,bjhd->bhj", qv, _f(kc))
    valid = torch.arange(S, device=q.device).view(1, 1, S) <= pos.reshape(B, 1, 1)
    s = s.masked_fill(~valid, float("-inf"))
    p = torch.softmax(s, -1).nan_to_num(0.0)
    o.reshape(B, H, D).copy_(torch.einsum("bhj,bjhd->bhd", p, _f(vc)))
    return None
