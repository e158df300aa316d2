"""Parameter store: every trainable tensor lives in ONE flat fp32 master buffer, ONE flat compute-dtype (bf16)
shadow buffer and ONE flat fp32 gradient buffer.

Why flat: the optimizer step is then a handful of multi-tensor HIP launches over contiguous memory (K20), the DP
gradient all-reduce is a few large RCCL calls over contiguous buckets (X08), and checkpoints are streamed views.

Naming and cross-depth sharing follow the reference: deterministic per-prefix scope counters
(``src/utils_core.py:16-19,57-67``), ``get_variable`` names (``src/utils_mtf.py:271-280``) and ALBERT-style
``shared`` reuse keyed on (block config, layer function, occurrence) (``src/model/backend.py:43-94``).
Initialisers: ``OrthogonalInit`` incl. quirks A2/A3 (``src/model/backend.py:18-40``), normal and constant.
"""
from __future__ import annotations

import contextlib
import hashlib
import math
import typing

import torch

from ..config import Dim
from . import dims as D

_ALIGN = 64  # elements; every tensor starts 256-B aligned in the fp32 buffers


class VarSpec:
    def __init__(self, name: str, dims: typing.List[Dim], init: typing.Callable[[torch.Generator, torch.device],
                                                                                  torch.Tensor],
                 tp_dim: typing.Optional[int], tp_size: int, trainable: bool = True):
        self.name = name
        self.dims = list(dims)                      # global (unsharded) named shape
        self.full_shape = [d.size for d in dims]
        self.tp_dim = tp_dim                        # axis split over the TP group (the ``heads`` axis) or None
        self.local_shape = list(self.full_shape)
        if tp_dim is not None:
            self.local_shape[tp_dim] //= tp_size
        self.numel = 1
        for s in self.local_shape:
            self.numel *= s
        self.init = init
        self.trainable = trainable
        self.offset = -1
        # optimizer classification (ref src/optimizer/__init__.py:46-61)
        self.is_rezero = "rezero" in name

    def weight_decay_eligible(self, params) -> bool:
        var_dims = self.dims
        features_used = D.feature_dims_used(params, var_dims)
        large = features_used and len(var_dims) > len(params.feature_dims)
        large |= (not features_used) and len(var_dims) >= 2
        large &= D.size(var_dims) > 1
        n = self.name
        large &= "norm" not in n
        large &= "rezero" not in n
        large &= "embed" not in n
        large &= "input" not in n or "lang_in" in n or "vid_in" in n
        large &= "output" not in n or "lang_out" in n or "vid_out" in n
        return bool(large)


def _seed_for(name: str, base_seed: int) -> int:
    return int.from_bytes(hashlib.sha256(f"{base_seed}/{name}".encode()).digest()[:7], "little")


# GPU init through CholeskyQR2 (OBST_CHOLQR_INIT=0: rocSOLVER Householder). Round 1 kept it opt-in after a flaky
# graph-vs-eager test; the cause was not the init: fp32 atomics in the norm-parameter / embedding / optimizer-statistics
# reductions made every run (eager ones too) differ in the last bits, and SM3's 1/sqrt(accumulator) amplifies that
# noise on rarely-updated embedding rows (tools/diag_graph.py: eager-vs-eager 2.6e-4 apart after 5 steps). Those
# reductions are fixed-order now and test_hip_graph_step_matches_eager asserts bitwise equality.
_CHOLQR = __import__("os").environ.get("OBST_CHOLQR_INIT", "1") == "1"


def orthonormal_columns(g: torch.Tensor) -> torch.Tensor:
    """Q of the QR factorisation of a tall ``g`` [m, n] (m >= n) with R's diagonal made positive -- the unique
    orthonormal basis the reference's sign-corrected Householder QR returns.

    On the GPU this is CholeskyQR2 in fp64 (two rounds of Gram GEMM + Cholesky + triangular solve): rocSOLVER's
    Householder QR of a 8192x2048 block issues tens of thousands of tiny launches (1.58 M launches, 7.6 s of GPU time
    for GPT-Neo-1.3B init, profiles/r1h_decode_kv.md), whereas this is a handful of GEMM-shaped calls. Cholesky's R
    has a positive diagonal, so Q is the same matrix as the sign-corrected Householder Q up to rounding. Falls back to
    Householder if the Gram matrix is numerically not positive definite. The CPU path keeps Householder QR.
    ``OBST_CHOLQR_INIT=0`` selects Householder on the GPU too."""
    if g.device.type == "cuda" and _CHOLQR:
        q = cholesky_qr2(g)
        if q is not None:
            return q
    q, r = torch.linalg.qr(g)
    return q * torch.sign(torch.diagonal(r)).unsqueeze(0)


def cholesky_qr2(g: torch.Tensor) -> typing.Optional[torch.Tensor]:
    """CholeskyQR2 in fp64 on any device; None if a Gram matrix is not numerically positive definite."""
    x = g.double()
    for _ in range(2):
        chol, info = torch.linalg.cholesky_ex(x.t() @ x)
        if int(info) != 0:
            return None
        x = torch.linalg.solve_triangular(chol, x.t(), upper=False).t()
    return x.to(g.dtype)


def orthogonal_init(full_shape: typing.List[int], fan_in: int, scale_by_depth: bool, depth: int):
    """ref ``OrthogonalInit`` (``src/model/backend.py:18-40``). ``fan_in`` is 1 when the caller passes no fan-in dims
    (quirk A2): the "orthogonal" tensor is then one unit-norm Gaussian vector."""
    total = 1
    for s in full_shape:
        total *= s
    fan_out = total // fan_in

    def _init(gen: torch.Generator, device: torch.device) -> torch.Tensor:
        transpose = fan_out > fan_in
        shape = (fan_out, fan_in) if transpose else (fan_in, fan_out)
        g = torch.randn(shape, generator=gen, device=device, dtype=torch.float32)
        if min(shape) == 1:
            q = g / g.norm()
        else:
            q = orthonormal_columns(g)
        if transpose:
            q = q.t()
        out = q.reshape(full_shape)
        if scale_by_depth:
            out = out / depth ** 0.5
        return out
    return _init


def normal_init(full_shape, stddev: float, mean: float):
    def _init(gen, device):
        return torch.randn(full_shape, generator=gen, device=device, dtype=torch.float32) * stddev + mean
    return _init


def constant_init(full_shape, value: float):
    def _init(gen, device):
        return torch.full(full_shape, float(value), device=device, dtype=torch.float32)
    return _init


class ParamStore:
    """Registration phase (shapes only) → ``finalize`` allocates flat buffers and runs the initialisers."""

    def __init__(self, params, tp_rank: int = 0, tp_size: int = 1):
        self.params = params
        self.tp_rank = tp_rank
        self.tp_size = tp_size
        self.specs: typing.Dict[str, VarSpec] = {}
        self.order: typing.List[str] = []
        self.finalized = False
        self.master: typing.Optional[torch.Tensor] = None
        self.compute: typing.Optional[torch.Tensor] = None
        self.grad: typing.Optional[torch.Tensor] = None
        self.total = 0
        self._leaves: typing.Dict[str, torch.Tensor] = {}

    # -- registration ---------------------------------------------------------------------------------------------
    def register(self, name: str, dims: typing.List[Dim], init, trainable: bool = True,
                 shard: typing.Optional[Dim] = None) -> VarSpec:
        """dims: global; the TP-split axis is ``heads`` unless ``shard`` names another one (tp_layout intermediate)"""
        if name in self.specs:
            return self.specs[name]
        if self.finalized:
            raise KeyError(f"variable {name} requested after the parameter store was finalized")
        tp_dim = None
        if self.tp_size > 1 and shard is not None:
            tp_dim = list(dims).index(shard)
        elif self.tp_size > 1 and self.params.head_dim in dims:
            tp_dim = list(dims).index(self.params.head_dim)
        spec = VarSpec(name, dims, init, tp_dim, self.tp_size, trainable)
        self.specs[name] = spec
        self.order.append(name)
        return spec

    # -- allocation -----------------------------------------------------------------------------------------------
    def finalize(self, device: torch.device, compute_dtype: torch.dtype, init_device: typing.Optional[torch.device]
                 = None):
        off = 0
        for name in self.order:
            spec = self.specs[name]
            spec.offset = off
            off += (spec.numel + _ALIGN - 1) // _ALIGN * _ALIGN
        self.total = max(off, _ALIGN)
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        self.master = torch.zeros(self.total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=device)
        init_device = torch.device(init_device or device)
        for name in self.order:
            spec = self.specs[name]
            gen = torch.Generator(device=init_device)
            gen.manual_seed(_seed_for(name, self.params.seed))
            full = spec.init(gen, init_device)
            if spec.tp_dim is not None:
                n = spec.local_shape[spec.tp_dim]
                full = full.narrow(spec.tp_dim, self.tp_rank * n, n)
            self.master_view(name).copy_(full.reshape(spec.local_shape))
        if compute_dtype == torch.float32:
            self.compute = self.master
        else:
            self.compute = self.master.to(compute_dtype)
        self.finalized = True
        self._leaves = {}

    def master_view(self, name: str) -> torch.Tensor:
        s = self.specs[name]
        return self.master[s.offset:s.offset + s.numel].view(s.local_shape)

    def grad_view(self, name: str) -> torch.Tensor:
        s = self.specs[name]
        return self.grad[s.offset:s.offset + s.numel].view(s.local_shape)

    def compute_view(self, name: str) -> torch.Tensor:
        s = self.specs[name]
        return self.compute[s.offset:s.offset + s.numel].view(s.local_shape)

    def leaf(self, name: str) -> torch.Tensor:
        """Autograd leaf aliasing the compute buffer. Ops accumulate its gradient straight into ``.main_grad``
        (a view of the flat fp32 grad buffer) and return ``None`` to autograd."""
        t = self._leaves.get(name)
        if t is None:
            t = self.compute_view(name).detach().requires_grad_(self.specs[name].trainable)
            t.main_grad = self.grad_view(name)
            t.master = self.master_view(name)
            t.var_name = name
            t.store = self
            self._leaves[name] = t
        return t

    def grad_view_of(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        """view of variable `name` inside any flat buffer laid out like ``grad``"""
        s = self.specs[name]
        return flat[s.offset:s.offset + s.numel].view(s.local_shape)

    def sync_compute(self):
        """master (fp32) → compute (bf16) copy; the fused optimizer kernel does this itself on the GPU."""
        if self.compute is not self.master:
            self.compute.copy_(self.master)
        self.bump()

    def bump(self):
        """the compute copy changed (optimizer step, restore): cached transposed weights are stale"""
        self.version = getattr(self, "version", 0) + 1

    def transposed(self, name: str, H: int, K: int, N: int) -> torch.Tensor:
        """bf16 copy of a linear weight with every [K][N] block stored as [N][K] (same flat offsets as ``compute``,
        so weights adjacent in ``compute`` stay adjacent here). Re-transposed lazily after each ``bump``."""
        from ..ops import raw
        s = self.specs[name]
        if getattr(self, "compute_t", None) is None:
            self.compute_t = torch.empty_like(self.compute)
            self._t_version: typing.Dict[str, int] = {}
        out = self.compute_t[s.offset:s.offset + s.numel]
        ver = getattr(self, "version", 0)
        if self._t_version.get(name) != ver:
            src = self.compute[s.offset:s.offset + s.numel]
            raw.transpose(src, out, K, N, N, K, H, K * N, K * N)
            self._t_version[name] = ver
        return out

    def derived(self, name: str, tag: str, fn: typing.Callable[[], torch.Tensor]) -> torch.Tensor:
        """a tensor computed from variable `name`'s compute copy (e.g. the masked token-mixer weight), cached until
        the next ``bump``: a depth-shared weight is derived once per step instead of once per use"""
        cache = self.__dict__.setdefault("_derived", {})
        ver = getattr(self, "version", 0)
        hit = cache.get((name, tag))
        if hit is None or hit[0] != ver:
            hit = (ver, fn())
            cache[(name, tag)] = hit
        return hit[1]

    def zero_grad(self):
        from ..ops import raw
        raw.zero_(self.grad)
        # variables whose gradient has received no contribution yet this step: their first weight-gradient GEMM
        # may overwrite (beta = 0) instead of accumulating (ops/functional.py::_acc_grad_beta)
        self.fresh = set(self.order)

    def fold_leaf_grads(self):
        """Paths that use plain torch autograd (exotic layer variants) leave gradients on the leaves' ``.grad``;
        fold them into the flat fp32 buffer so the optimizer/all-reduce see one gradient."""
        for t in self._leaves.values():
            if t.grad is not None:
                self.leaf_grads_seen = True     # a plain-autograd path is active: no whole-step hipGraph
                t.main_grad.add_(t.grad.float())
                t.grad = None

    def numel(self) -> int:
        return sum(s.numel for s in self.specs.values())

    def global_numel(self) -> int:
        return sum(D.size(s.dims) for s in self.specs.values())


class Scope:
    """Deterministic scope naming: ``scope(name)`` enters ``name{counter}`` (ref ``src/utils_core.py:16-19``).

    Unlike the reference's process-global per-prefix counters, counters here are local to the parent scope, so
    the names inside a block depend only on that block -- a block recomputed in backward (RevNet, checkpoint)
    re-enters exactly the same names."""

    def __init__(self):
        self.stack: typing.List[str] = []
        self.counters: typing.Dict[tuple, int] = {}

    def reset(self):
        self.stack = []
        self.counters = {}

    @contextlib.contextmanager
    def __call__(self, name: str):
        key = (self.path, name)
        idx = self.counters.get(key, -1) + 1
        self.counters[key] = idx
        self.stack.append(f"{name}{idx}")
        try:
            yield self.stack[-1]
        finally:
            self.stack.pop()

    @contextlib.contextmanager
    def exact(self, name: str):
        """enter a scope with a fixed name (no counter)"""
        self.stack.append(name)
        try:
            yield name
        finally:
            self.stack.pop()

    def snapshot(self) -> typing.List[str]:
        return list(self.stack)

    @contextlib.contextmanager
    def restore(self, stack: typing.List[str]):
        """Re-enter a previously snapshotted scope with fresh child counters (for recomputation)."""
        saved_stack, saved_counters = self.stack, self.counters
        self.stack = list(stack)
        prefix = "/".join(stack)
        self.counters = {k: v for k, v in saved_counters.items() if not (k[0] == prefix or
                                                                          k[0].startswith(prefix + "/"))}
        try:
            yield
        finally:
            self.stack, self.counters = saved_stack, saved_counters

    @property
    def path(self) -> str:
        return "/".join(self.stack)


class SharedCache:
    """Cross-depth parameter sharing (``shared`` extra): the first depth creates, later depths reuse in order.

    Key = (block config index, layer function, occurrence of that function within the block config)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.table: typing.Dict[tuple, typing.List[str]] = {}
        self.cursor: typing.Dict[tuple, int] = {}

    def begin_layer(self, key: tuple):
        self.cursor[key] = 0

    def lookup(self, key: tuple, depth: int, create: typing.Callable[[], str]) -> str:
        names = self.table.setdefault(key, [])
        idx = self.cursor.get(key, 0)
        self.cursor[key] = idx + 1
        if depth == 0 or idx >= len(names):
            name = create()
            if idx >= len(names):
                names.append(name)
            return name
        return names[idx]


def fan_in_size(dims: typing.Optional[typing.List[Dim]]) -> int:
    return int(math.prod(d.size for d in dims)) if dims else 1
