"""Model-build context: the eager replacement of the reference's (params, mtf.Graph, variable scope) triple.

``Builder`` carries the config, the flat ``ParamStore``, deterministic scope naming, cross-depth sharing state, the
TP layout and a "register" mode: the first forward runs on meta tensors (no compute) and only records variables,
after which the store allocates its flat buffers and every later forward reads views by name.

``Act`` is a tensor plus its static named dims (reference ``mtf.Tensor.shape``); ``BlockArgs`` mirrors
``src/dataclass.py:387-419`` (with bug A14 fixed).
"""
from __future__ import annotations

import copy
import typing

import torch

from ..config import Dim, ModelParameter
from . import dims as D
from .variables import ParamStore, Scope, SharedCache


class Act:
    __slots__ = ("t", "dims")

    def __init__(self, t: torch.Tensor, dims: typing.Sequence[Dim]):
        self.t = t
        self.dims = list(dims)
        if tuple(t.shape) != tuple(d.size for d in self.dims):
            raise ValueError(f"tensor shape {tuple(t.shape)} != named dims {self.dims}")

    def __repr__(self):
        return f"Act({[f'{d.name}:{d.size}' for d in self.dims]})"


class KVCache:
    """Per-attention-layer key / value caches for incremental decoding (serving). ``mode`` "prefill": the attention
    layers run over the whole context and keep k / v [B, S, H, D]; "decode": the input is one token per row at
    position ``pos[b]``, whose k / v are appended to the caches and whose query attends over keys [0, pos[b]]."""

    def __init__(self, persist: typing.Optional[dict] = None):
        self.layers: typing.Dict[int, typing.Tuple[torch.Tensor, torch.Tensor, float]] = {}
        self.mode = "prefill"
        self.pos: typing.Optional[torch.Tensor] = None
        self.idx = 0
        # sequence-mixing layers other than dot-product attention: the learned token mixer keeps its input
        # [B, S, H, F] and masked weight, cumsum / cummean their running fp32 sums; keyed by the attention index
        # (mixers) or ("c", n) (cumsum layers). `unsupported`: a mixing layer ran uncached during the prefill
        self.states: typing.Dict[typing.Any, dict] = {}
        self.cidx = 0
        self.unsupported = False
        # state that outlives one request: cache buffers per layer (reused while the shape stays) and the decode
        # step's hipGraph (Model._decode_graphed), which bakes their addresses in
        self.persist = persist if persist is not None else {"bufs": {}, "graph": None}

    def keep(self, i: int, k: torch.Tensor, v: torch.Tensor, scale: float):
        bufs = self.persist["bufs"]
        old = bufs.get(i)
        if old is not None and old[0].shape == k.shape and old[0].dtype == k.dtype and old[0].device == k.device:
            old[0].copy_(k)
            old[1].copy_(v)
        else:
            old = bufs[i] = (k, v)
            self.persist["graph"] = None
        self.layers[i] = (old[0], old[1], scale)

    def keep_state(self, key, **tensors):
        """per-layer decode state (persistent buffers reused while shapes stay, like the k / v caches)"""
        bufs = self.persist["bufs"]
        old = bufs.get(("state", key))
        if old is not None and all(k in old and old[k].shape == t.shape and old[k].dtype == t.dtype and
                                   old[k].device == t.device for k, t in tensors.items()):
            for k, t in tensors.items():
                if old[k].data_ptr() != t.data_ptr():
                    old[k].copy_(t)
        else:
            old = bufs[("state", key)] = {k: t.clone() for k, t in tensors.items()}
            self.persist["graph"] = None
        self.states[key] = old


class Builder:
    def __init__(self, params: ModelParameter, tp_rank: int = 0, tp_size: int = 1):
        # local (TP-sharded) view of the config: `heads` has size heads / tp
        local = copy.copy(params)
        local.__dict__ = dict(params.__dict__)
        if params.heads % tp_size:
            raise ValueError("heads must be divisible by tp")
        local.head_dim = Dim("heads", params.heads // tp_size)
        local.feature_dims = [local.head_dim, params.key_dim]
        self.params = local
        self.global_params = params
        self.tp_rank, self.tp_size = tp_rank, tp_size
        self.store = ParamStore(params, tp_rank, tp_size)
        self.scope = Scope()
        self.shared = SharedCache()
        self.register = True
        self.train = True
        self.device = torch.device("cpu")
        self.dtype = torch.float32
        self.depth_idx = 0
        self.config_idx = 0
        self.fn_occurrence: typing.Dict[tuple, int] = {}
        self.dropout_counter = 0
        self.step_seed = 0
        self.use_counts: typing.Dict[str, int] = {}
        self.kv: typing.Optional[KVCache] = None

    # ---- per forward ------------------------------------------------------------------------------------------------
    def begin_forward(self):
        self.scope.reset()
        self.shared.reset()
        self.params.attention_idx = 0
        self.dropout_counter = 0
        if self.kv is not None:
            self.kv.idx = 0
            self.kv.cidx = 0
        if self.register:
            self.use_counts = {}

    def next_dropout_seed(self) -> int:
        self.dropout_counter += 1
        return (self.step_seed * 1_000_003 + self.dropout_counter * 7919) & (2 ** 63 - 1)

    # ---- variables ----------------------------------------------------------------------------------------------------
    def _global_dims(self, dims: typing.List[Dim]) -> typing.List[Dim]:
        return [self.global_params.head_dim if d == self.params.head_dim else d for d in dims]

    def variable(self, args: "BlockArgs", kind: str, dims: typing.List[Dim], init_factory,
                 shard: typing.Optional[typing.Tuple[Dim, Dim]] = None) -> torch.Tensor:
        """``init_factory(global_dims) -> init(gen, device)``. Returns the variable as a compute-dtype tensor.
        ``shard = (local_dim, global_dim)``: the TP-split axis instead of ``heads`` (dims then hold the global heads)"""
        dims = D.deduplicate(dims)

        def gdims():
            g = self._global_dims(dims)
            return [shard[1] if shard is not None and d == shard[0] else d for d in g]

        def create() -> str:
            with self.scope(kind):
                name = self.scope.path
            if self.register:
                self.store.register(name, gdims(), init_factory(gdims()),
                                    shard=shard[1] if shard is not None else None)
            return name

        if "shared" in args:
            key = (self.config_idx, args.fn_name, args.fn_occurrence)
            name = self.shared.lookup(key, self.depth_idx, create)
        else:
            name = create()
        if self.register:
            self.use_counts[name] = self.use_counts.get(name, 0) + 1
            return torch.zeros([d.size for d in dims], device="meta", dtype=self.dtype)
        return self.store.leaf(name)


class BlockArgs:
    def __init__(self, builder: Builder, tensor: typing.Optional[Act], name_extras: typing.List[str],
                 is_last: bool = False):
        self.builder = builder
        self.params = builder.params
        self.tensor = tensor
        self.name_extras = list(name_extras)
        self.is_last = is_last
        self.fn_name = ""
        self.fn_occurrence = 0
        self.residual: typing.Optional[Act] = None  # set by the frontend for fusable last layers of skip blocks
        self.stream_sink = None  # RevNet: the block's last layer may fuse the fp32 stream update (F.StreamSink)
        self.grad_sink = None    # RevNet: the block's opening norm may fuse the fp32 stream gradient (F.GradSink)
        self.fused_act = None    # norm followed by an activation layer: applied in the norm kernel
        self.fused_act_done = False

    def __call__(self, *args) -> "BlockArgs":
        new = BlockArgs(self.builder, self.tensor, self.name_extras[:], self.is_last)
        new.fn_name, new.fn_occurrence = self.fn_name, self.fn_occurrence
        for a in args:
            if isinstance(a, Act):
                new.tensor = a
            elif isinstance(a, (list, tuple)):
                new.name_extras = list(a)
            elif isinstance(a, str):
                new.name_extras.append(a)  # reference appends the `str` type (bug A14)
            else:
                raise ValueError(f"unsupported BlockArgs argument {a!r}")
        return new

    def __iter__(self):
        return iter(self.name_extras)

    def __contains__(self, item):
        return item in self.name_extras

    def __len__(self):
        return len(self.name_extras)

    def __getitem__(self, idx):
        return self.name_extras[idx]
