"""Run/model configuration: the JSON schema of the reference's ``ModelParameter``.

Behavioural parity with ``src/dataclass.py:34-337`` of the reference: the same key names, the same defaults,
the same derived dimensions (``features``, ``features_per_head``, ``intermediate``, ``vocab`` ...). What changes is
the *layout* rule: the reference derives a TPU mesh ``b = tpu_size / heads, h = heads`` and silently overwrites
any JSON mesh (``src/dataclass.py:247-252``, quirk A18). Here the mesh is an explicit ``{dp, tp}`` pair that defaults
to ``dp = world_size, tp = 1`` and may be overridden (``mesh`` key), with the constraint ``heads % tp == 0``.

Fixed reference bugs: A13 (``__getitem__`` used the attribute ``key``), A11 (gradient
accumulation rejected) and A14 (``BlockArgs`` appended the ``str`` type).
"""
from __future__ import annotations

import copy
import json
import os
import typing

import torch

from .utils.log import log

Dim = typing.NamedTuple("Dim", (("name", str), ("size", int)))

_DTYPES = {"float32": torch.float32, "float64": torch.float64, "bfloat16": torch.bfloat16, "float16": torch.float16}


def anonymize_dim(dim: Dim, new_size: typing.Optional[int] = None) -> Dim:
    """``_name`` marks a replicated (non-split) copy of a dimension (ref ``src/utils_mtf.py:82-95``)."""
    name = dim.name if dim.name.startswith('_') else '_' + dim.name
    return Dim(name, dim.size if new_size is None else new_size)


def unanonymize_dim(dim: Dim) -> Dim:
    return Dim(dim.name[1:] if dim.name.startswith('_') else dim.name, dim.size)


class BlockConfig:
    """One entry of ``block_config`` (ref ``src/dataclass.py:12-19``): ``{"layer": [...], "skip": bool}``."""

    def __init__(self, config: typing.Union[dict, "BlockConfig"], memory_reduction_strategy: str):
        if isinstance(config, BlockConfig):
            config = dict(config.__dict__)
        self.layer: typing.List[str] = []
        self.skip = False
        self.memory_reduction_strategy = memory_reduction_strategy
        self.__dict__.update(config)

    def to_dict(self):
        return {"layer": list(self.layer), "skip": self.skip}


class LearningRateConfig:
    def __init__(self, start_step: int = 0, final_step: int = 0, factor: float = 1.):
        self.start_step = start_step
        self.final_step = final_step
        self.factor = factor


_DEFAULTS: typing.Dict[str, typing.Any] = dict(
    position_embedding="absolute", token_embedding="absolute", empty_frame_embedding="absolute",
    output_embedding="absolute-orthogonal", use_video=True, save_graph=False, use_language=True,
    contrastive_across_samples=False, contrastive_across_token_embeddings=False, input_dropout=0.,
    output_offset=1, weight_standardisation=True, use_checkpointing=False, max_checkpoints_keep=1,
    steps_per_checkpoint=100_000, time_patch=1, patch_size=16, frame_width=320, frame_height=176,
    opt_beta1=0.9, opt_beta2=0.999, vocab_size=256, color_channels=3, three_axes=True, dataset_configs=[],
    data_seed=456772, parallel_batch=None, parallel_interleave=None, use_random_dataloader=False, train=True,
    debug_sample=False, padding_token=0, concat_token=4, sequence_length=32, heads=8, features=None,
    features_per_head=None, depth=16, buffer_size=4, combine_assignments=False, shuffle_buffer=256,
    interleaved_datasets=256, token_patch_size=1, learning_rate=5e-5, storage_dtype="float32",
    slice_dtype="float32", calculation_dtype="float32", optimizer_slice_dtype="float32",
    optimizer_calculation_dtype="float32", learning_rate_config={}, train_batch_size=1, grad_accumulation=1,
    macro_batching=1, macro_batch_loss_smoothing=False, reduce_lr_on_plateau_timespan=0,
    reduce_lr_on_plateau_reduction=2, momentumnet_alpha=0.99, current_step=0, tpu_size=32,
    default_sleep_duration=0.1, lookahead_steps=0, lookahead_alpha=0, momentum=0.95,
    prefix="datasets/full_hd_video", model_path="runs/default", tensorflow_optimization_settings={},
    language_token_per_frame=0, weight_decay=0.001, vocab_weight_factorization=0.125, train_steps=2 ** 30,
    warmup_steps=3000, rezero_lr_multiplier=0.1, learning_rate_decay_multi=1, convolution_size=16,
    learning_rate_decay_start_step=100_000, learning_rate_decay_min=5e-10, iterations=2500,
    initial_autoregressive_position=128, use_autoregressive_sampling=False, sampling_temperature=0,
    weight_centralisation=True, shuffle_input_filenames=True, calc_accuracy=False, num_of_sample=10,
    web_workers=1, equal_debugging_items_per_check=16, group_linear_factor=2, embedding_stddev=0.04,
    color_quantization_value=256, experts=64, pkm_axes=2, use_bit_fold_input_pipeline=False, bit_fold_value=4,
    debug_train_step=False, model_mode='jannet', optimizer='learning_rate', multi_loss_strategy="linear",
    memory_reduction_strategy="revnet", debug_gradients=False, use_initial_position_embedding=False,
    intermediate_feed_forward_multiplier=None, intermediate_feed_forward_multiplier_multiplier=None,
    own_color="\x1b[32;1m", other_color="\x1b[0m", scale_by_depth=True, z_loss=1e-4,
    block_config=[{'layer': ["norm-group-shift-scale", "feed_forward-in_relu-group-in_glu_add-in_norm"]},
                  {'layer': ["norm-group-std-shift-scale", "attention-in_relu-embedded-relative"]}],
    input_block_config=[], output_block_config=[], masked_attention_dimensions=[0], split_grad_accumulation=True,
    log_dict_keys=[],
    # ---- keys new in this framework (MI355X-native runtime) ----
    mesh=None,                   # {"dp": int, "tp": int}; default dp=world, tp=1
    tp_layout="heads",           # "heads": the reference layout (intermediate replicated over TP); "intermediate":
                                 # feed-forward weights split over the intermediate axis (layers.feed_forward)
    attention_scale="sequence",  # "sequence" (reference quirk A1, spatial.py:60) or "head" (1/sqrt(fph))
    shared_key_value_mixing=True,  # shared_key_value attention mixes the keys (P K); False: the reference's
                                   # rowsum(P) * key (quirk A19, spatial.py:63-64,81 -- no mixing, docs/PARITY.md)
    seed=0,                      # parameter-init seed
    grad_bucket_mb=0,            # DP gradient bucket size in MiB of fp32; 0: the buffer in 12 buckets (>= 16 MiB)
    allreduce_dtype="bfloat16",  # DP wire dtype: bf16 with fp32 accumulation (all-to-all + sum + all-gather), or
                                 # "float32" (one fp32 all-reduce per bucket)
    force_grad_sync=False,       # run the DP collectives at world 1 too (tests of the capture path on one GPU)
    # RevNet residual streams: "float32" (exact-to-fp32 reconstruction x1 = y2 - F(x2)) or "calculation" (the streams in
    # calculation_dtype, as the reference's RevGradOp keeps them: ref src/model/revnet.py:23,69 -- a third of the
    # stream bytes, bf16 reconstruction error over the depth; profiles/r6_revnet_stream.md)
    revnet_stream_dtype="float32",
    # the RevNet GRADIENT streams under fp32 activation streams: "calculation" (bf16, the usual mixed-precision
    # convention for activation gradients; the reconstruction stays exact; ctx32_mixer -7 % step time with the same
    # gradient error against the fp32 oracle -- profiles/r6_revnet_stream.md) or "float32"
    revnet_grad_stream_dtype="calculation",
    use_hip_graphs=False,        # capture the whole training step in hipGraphs (Trainer._graph_step; 1 GPU, no dropout)
    # also capture with world > 1 (the RCCL all-reduces inside the graph; opt-in: RCCL graph capture is exercised only
    # where several GPUs are visible, which the 1-GPU test boxes are not)
    hip_graphs_distributed=False,
    kv_cache=True,               # incremental decoding over per-layer KV caches for causal-attention bodies (Sampler)
    decode_hip_graphs=True,      # replay the single-token decode step from a hipGraph (Model._decode_graphed)
    log_every=10, metrics_path=None, pad_vocab_to=128,
    tokenizer_path=None,         # tokenizers JSON for vocab_size > 256 (the reference downloads GPT-2's)
    web_host="0.0.0.0", web_port=62220, serve_max_batch=8,
    heartbeat_path=None,         # file touched every logged step (watchdog liveness)
    tensorboard=False,           # also write TensorBoard scalars (if the tensorboard package is importable)
    dist_timeout_s=1800,         # torch.distributed collective timeout
)

# keys the reference reads nowhere outside dataclass.py -- accepted silently
_DEAD_KEYS = {"adaptive_gradient_clipping", "gradient_clip"}


class ModelParameter:
    """Config object. ``ModelParameter(json_dict)``; attribute access; ``dict()`` gives the JSON-able form."""

    def __init__(self, config: typing.Union[dict, "ModelParameter", None] = None, warn_unknown: bool = True):
        if isinstance(config, ModelParameter):
            config = config.raw
        config = dict(config or {})
        self.__dict__.update(copy.deepcopy(_DEFAULTS))
        for k, v in config.items():
            if k not in _DEFAULTS and k not in _DEAD_KEYS and warn_unknown:
                log(f"WARNING: Unknown ModelParameter {k}={v!r}")
            self.__dict__[k] = copy.deepcopy(v)
        self.raw = {k: copy.deepcopy(v) for k, v in config.items()}
        self._derive()

    # -- derivations (ref src/dataclass.py:189-337) --------------------------------------------------------------
    def _derive(self):
        if self.macro_batching < 1:
            raise ValueError("MacroBatching has to be >=1, where 1 means it's disabled")
        if self.grad_accumulation < 1:
            raise ValueError("grad_accumulation has to be >= 1")
        for key in ("position_embedding", "token_embedding", "output_embedding", "empty_frame_embedding"):
            val = getattr(self, key)
            if isinstance(val, str):
                setattr(self, key, val.split('-'))
        self.multi_loss_strategy = self.multi_loss_strategy.lower()
        if self.multi_loss_strategy not in ("linear", "pcgrad", "mgda"):
            log(f"{self.multi_loss_strategy} is not a supported multi-loss strategy; defaulting to 'linear'")
            self.multi_loss_strategy = "linear"
        if not self.use_language and not self.use_video:
            raise ValueError("Language and video mode are disabled. No model can be built.")
        if self.weight_standardisation and not self.weight_centralisation:
            self.weight_centralisation = True
        if self.features is None and self.features_per_head is None:
            raise ValueError("Either features or features_per_head has to be specified")
        if self.features is None:
            self.features = self.features_per_head * self.heads
        if self.features_per_head is None:
            self.features_per_head = self.features // self.heads
        if self.use_video and (self.frame_width * self.frame_height // self.patch_size) % self.experts:
            raise ValueError("Frame size has to be divisible by number of experts. Set \"experts\" to 1")
        if self.intermediate_feed_forward_multiplier_multiplier is not None:
            self.intermediate_feed_forward_multiplier = (self.group_linear_factor *
                                                         self.intermediate_feed_forward_multiplier_multiplier /
                                                         self.heads)
        if self.intermediate_feed_forward_multiplier is None:
            self.intermediate_feed_forward_multiplier = self.group_linear_factor / self.heads
        if not self.use_video and self.language_token_per_frame != self.sequence_length:
            self.language_token_per_frame = self.sequence_length
        if self.macro_batching > 1 and self.grad_accumulation > 1 and self.macro_batching % self.grad_accumulation:
            raise ValueError('"macro_batching" needs do be divisible by "grad_accumulation"')

        self.torch_storage_dtype = _DTYPES[self.storage_dtype]
        self.torch_calculation_dtype = _DTYPES[self.calculation_dtype]
        self.torch_slice_dtype = _DTYPES[self.slice_dtype]
        self.torch_optimizer_dtype = _DTYPES[self.optimizer_calculation_dtype]
        self.learning_rate_modules = {key: LearningRateConfig(**conf) for key, conf in
                                      dict(self.learning_rate_config).items()}

        self.block_configs = [BlockConfig(c, self.memory_reduction_strategy) for c in self.block_config]
        self.input_block_configs = [BlockConfig(c, "checkpoint") for c in self.input_block_config]
        self.output_block_configs = [BlockConfig(c, "checkpoint") for c in self.output_block_config]

        self.time_patch_size = self.sequence_length // self.time_patch
        self.frame_height_patch = self.frame_height // self.patch_size
        self.frame_width_patch = self.frame_width // self.patch_size
        self.channel_color_size = self.color_channels * self.time_patch * self.patch_size ** 2
        self.fold_count = 32 // self.bit_fold_value
        self.language_token_patch = self.language_token_per_frame // self.token_patch_size
        if self.use_bit_fold_input_pipeline:
            self.channel_color_size = self.channel_color_size // self.fold_count

        # named dimensions (ref src/dataclass.py:273-309)
        self.product_key_value_vectors = self.features_per_head ** 2
        self.product_key_value_dim = Dim("product_key_value_dim", self.product_key_value_vectors)
        self.head_dim = Dim("heads", self.heads)
        self.key_dim = Dim("features_per_head", self.features // self.heads)
        self.pkm_dim = Dim("pkm_axes", self.pkm_axes)
        self.feature_dims = [self.head_dim, self.key_dim]
        self.intermediate = [Dim("intermediate", int(self.heads * self.key_dim.size *
                                                     self.intermediate_feed_forward_multiplier))]
        self.expert_dim = Dim("experts", self.experts)
        self.vocab_dim = Dim("vocab", self.vocab_size)
        self.batch_dim = Dim("batch", self.train_batch_size)
        self.sequence_dim = Dim("sequence", self.time_patch_size)
        self.token_patch_dim = Dim("language_token_patch", self.token_patch_size)
        self.color_channel_dim = Dim("color_channels", self.channel_color_size)
        self.discrete_color_dim = Dim("color_quantization", self.color_quantization_value)
        self.attention_idx = 0

    # -- mesh ------------------------------------------------------------------------------------------------------
    def resolve_mesh(self, world_size: int) -> typing.Tuple[int, int]:
        """(dp, tp) for ``world_size`` ranks. TP splits ``heads`` (ref layout ``heads:h``); DP splits ``batch``."""
        mesh = self.mesh or {}
        tp = int(mesh.get("tp", 1))
        dp = int(mesh.get("dp", world_size // tp))
        if dp * tp != world_size:
            raise ValueError(f"mesh dp={dp} x tp={tp} != world_size={world_size}")
        if self.heads % tp:
            raise ValueError(f"heads={self.heads} not divisible by tp={tp}")
        if self.train_batch_size % dp:
            raise ValueError(f"train_batch_size={self.train_batch_size} not divisible by dp={dp}")
        return dp, tp

    # -- dict-like interface (A13 fixed) ----------------------------------------------------------------------------
    def __getitem__(self, key: str):
        return getattr(self, key)

    def __setitem__(self, key: str, value):
        setattr(self, key, value)

    def get(self, key: str, default=None):
        return self.__dict__.get(key, default)

    def dict(self) -> typing.Dict[str, typing.Any]:
        out = copy.deepcopy(_DEFAULTS)
        out.update(self.raw)
        return out

    def __repr__(self):
        return f"ModelParameter({self.raw})"


def load_config(path_or_name: str, overrides: typing.Optional[dict] = None) -> ModelParameter:
    """``--model`` accepts a JSON path or a name under ``configs/`` (ref ``src/main.py:55``)."""
    path = path_or_name
    if not path.endswith(".json"):
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", path + ".json")
    with open(path) as f:
        cfg = json.load(f)
    if overrides:
        cfg.update(overrides)
    return ModelParameter(cfg)
