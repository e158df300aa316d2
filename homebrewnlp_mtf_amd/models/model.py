"""Model assembly: input -> body -> output -> loss (ref src/model/__init__.py:32-259).

``Model(params, device, tp_rank, tp_size)`` runs one registration forward on meta tensors (shapes only) to create
every variable in the flat ``ParamStore``, allocates + initialises the buffers, then serves real forwards.

Language ("gpt") mode: gather embedding [vocab, intermediate*vocab_weight_factorization] -> linear to features ->
body (revnet | momentum | checkpoint | none) -> output embedding einsum over the features -> softmax cross-entropy
with z-loss (+ accuracy). The vocabulary is padded to a multiple of ``pad_vocab_to`` for the GEMMs; padded columns
are masked out of the loss and receive zero gradient.
Video ("jannet") mode: frames are patch tokens [batch, time+1, height, width, channels] scaled to [0, 1]; the model
predicts the next frame with a sigmoid output and a masked L1-style loss (ref src/model/__init__.py:34-67,147-199).
"""
from __future__ import annotations

import math
import typing

import torch

from ..config import Dim, ModelParameter
from ..ops import functional as F
from . import dims as D
from .context import Act, BlockArgs, Builder
from .frontend import block_part_fn
from .layers import embed, gather_embed, linear, linear_to_features, named_einsum, dropout
from .reversible import run_body


def padded_vocab(params: ModelParameter) -> int:
    m = int(params.pad_vocab_to or 1)
    return (params.vocab_size + m - 1) // m * m


class Model:
    def __init__(self, params: ModelParameter, device: typing.Union[str, torch.device] = "cpu",
                 tp_rank: int = 0, tp_size: int = 1, dtype: typing.Optional[torch.dtype] = None,
                 init_device: typing.Optional[torch.device] = None, local_batch: typing.Optional[int] = None):
        self.params = params
        self.device = torch.device(device)
        self.dtype = dtype or params.torch_calculation_dtype
        if self.device.type == "cuda" and self.dtype != torch.bfloat16:
            raise ValueError(f"the gfx950 kernels compute in bfloat16 (fp32 accumulate); calculation_dtype "
                             f"{self.dtype} is only supported by the CPU oracle")
        self.builder = Builder(params, tp_rank, tp_size)
        p = self.builder.params
        p.vocab_dim = Dim("vocab", padded_vocab(params))
        self.builder.dtype = self.dtype
        self.builder.device = self.device
        self.local_batch = local_batch or params.train_batch_size
        # registration pass on meta tensors
        self.builder.register = True
        with torch.no_grad():
            self._forward(self._dummy_inputs("meta"))
        self.builder.register = False
        self.builder.store.finalize(self.device, self.dtype, init_device=init_device)
        self.store = self.builder.store

    # ---------------------------------------------------------------------------------------------------------------
    def _dummy_inputs(self, device):
        p = self.params
        B = self.local_batch
        x = torch.zeros([B, p.sequence_length // p.token_patch_size, p.token_patch_size], dtype=torch.int64,
                        device=device) if p.use_language else None
        vid = None
        if p.use_video:
            shape = [B, p.time_patch_size + 1, p.frame_height_patch, p.frame_width_patch, p.channel_color_size]
            if not p.three_axes:
                shape = [B, p.time_patch_size + 1, p.frame_height_patch * p.frame_width_patch, p.channel_color_size]
            vid = torch.zeros(shape, dtype=self.dtype, device=device)
        return {"token_x": x, "token_y": x, "frame": vid}

    def forward(self, token_x=None, token_y=None, frame=None, vid_msk_src=None, vid_msk_tgt=None, train=True,
                step_seed: int = 0) -> typing.Dict[str, torch.Tensor]:
        self.builder.train = train
        self.builder.step_seed = step_seed
        return self._forward({"token_x": token_x, "token_y": token_y, "frame": frame,
                              "vid_msk_src": vid_msk_src, "vid_msk_tgt": vid_msk_tgt})

    __call__ = forward

    @torch.no_grad()
    def logits(self, token_x: torch.Tensor, positions: typing.Optional[torch.Tensor] = None,
               frame: typing.Optional[torch.Tensor] = None) -> torch.Tensor:
        """Inference forward (ref src/run/inference.py:77-85 ``build`` inside the sampling loop).

        Returns fp32 logits [batch, sequence, patch, vocab_size]; with ``positions`` ([batch] int) only the
        hidden state of those positions goes through the output projection -> [batch, 1, patch, vocab_size]
        (exact for causal bodies; the reference computes every position and then uses one)."""
        self.builder.train = False
        self._positions = positions
        try:
            out = self._forward({"token_x": token_x, "token_y": None, "frame": frame}, logits_only=True)
        finally:
            self._positions = None
        return out[..., :self.params.vocab_size].float()

    def _forward(self, batch: dict, logits_only: bool = False):
        b = self.builder
        p = b.params
        b.begin_forward()
        with b.scope(p.model_mode):
            with b.scope("input"):
                src, vid_tgt = self._input(batch)
            with b.scope("body"):
                out = run_body(b, src, p.memory_reduction_strategy, p.block_configs, p.depth)
            pos = getattr(self, "_positions", None)
            if logits_only and pos is not None and not p.output_block_configs:
                if out.dims[0].name != "batch" or out.dims[1].name != "sequence":
                    raise NotImplementedError(f"position slicing needs [batch, sequence, ...], got {out.dims}")
                t = out.t[torch.arange(out.t.shape[0], device=out.t.device), pos.to(out.t.device).long()]
                out = Act(t.unsqueeze(1).contiguous(), [out.dims[0], Dim("sequence", 1)] + list(out.dims[2:]))
            with b.scope("output"):
                frame_out, token_out = self._output(out)
            if logits_only:
                if pos is not None and p.output_block_configs:
                    idx = pos.to(token_out.t.device).long()
                    return token_out.t[torch.arange(token_out.t.shape[0], device=idx.device), idx].unsqueeze(1)
                return token_out.t
            with b.scope("loss"):
                return self._loss(frame_out, token_out, batch, vid_tgt)

    # ---------------------------------------------------------------------------------------------------------------
    def _input(self, batch):
        b = self.builder
        p = b.params
        tgt = None
        src = None
        if p.use_video:
            vid = batch["frame"]
            vdims = [Dim("batch", vid.shape[0]), Dim("_sequence", vid.shape[1])]
            vdims += [Dim("height", vid.shape[2])] + ([Dim("width", vid.shape[3])] if p.three_axes else [])
            vdims += [p.color_channel_dim]
            v = vid.to(b.dtype) / 255.0
            seq = Dim("sequence", vid.shape[1] - 1)
            src_t, tgt_t = v[:, :-1], v[:, 1:]
            sdims = [vdims[0], seq] + vdims[2:]
            src = Act(src_t.contiguous(), sdims)
            tgt = Act(tgt_t.contiguous(), sdims)
            args = BlockArgs(b, src, [''])
            if p.empty_frame_embedding is not None:
                e = embed(args(list(p.empty_frame_embedding)), sdims[2:])
                msk = batch.get("vid_msk_src")
                if msk is not None:
                    m = msk.to(b.dtype).view(list(msk.shape) + [1] * (len(sdims) - 2))
                    src = Act(src.t * m + e.t * (1 - m), sdims)
            src = linear_to_features(args(src), [p.color_channel_dim])
            for ci, cfg in enumerate(p.input_block_configs):
                src = block_part_fn(b, cfg, src, 0, ci, prefix="vid_inp")
        if p.use_language:
            tok = batch["token_x"]
            tdims = [Dim("batch", tok.shape[0]), Dim("sequence", tok.shape[1]), p.token_patch_dim]
            args = BlockArgs(b, Act(tok, tdims), [''])
            inter = Dim(p.intermediate[0].name, int(p.intermediate[0].size * p.vocab_weight_factorization))
            txt = gather_embed(args(list(p.token_embedding)), [p.vocab_dim, inter], tok, tdims)
            txt = dropout(args(txt, [f"dropout_rate{p.input_dropout}"]))
            txt = linear_to_features(args(txt), [p.token_patch_dim, inter])
            for ci, cfg in enumerate(p.input_block_configs):
                txt = block_part_fn(b, cfg, txt, 0, ci, prefix="lang_inp")
            if src is not None:
                # language tokens concatenated with video on the spatial axis (ref __init__.py:87-88)
                raise NotImplementedError("joint language+video input concatenation")
            src = txt
        if p.use_initial_position_embedding:
            args = BlockArgs(b, src, [''])
            for dim in D.subtract(src.dims, p.feature_dims)[1:]:
                pe = embed(args(list(p.position_embedding)), [dim] + list(p.feature_dims))
                src = Act(src.t + _bcast(pe, src), src.dims)
        return src, tgt

    def _output(self, out: Act):
        b = self.builder
        p = b.params
        token_out = frame_out = None
        args = BlockArgs(b, out, [''])
        if p.use_language:
            x = out
            for ci, cfg in enumerate(p.output_block_configs):
                x = block_part_fn(b, cfg, x, 0, ci, prefix="lang_out")
            new = [p.token_patch_dim, p.vocab_dim]
            w = embed(args(x, list(p.output_embedding)), list(p.feature_dims) + new)
            odims = D.subtract(x.dims, p.feature_dims) + new
            try:
                y = F.linear(x.t, w.t, x.dims, w.dims, odims)
            except NotImplementedError:
                y = F.tp_reduce(named_einsum([x, w], odims).t)
            token_out = Act(y, odims)
        if p.use_video:
            x = out
            for ci, cfg in enumerate(p.output_block_configs):
                x = block_part_fn(b, cfg, x, 0, ci, prefix="vid_out")
            y = linear(args(x), p.feature_dims, [p.color_channel_dim])
            frame_out = Act(torch.sigmoid(y.t.float()).to(y.t.dtype), y.dims)
        return frame_out, token_out

    def _loss(self, frame_out, token_out, batch, vid_tgt) -> typing.Dict[str, torch.Tensor]:
        p = self.builder.params
        res: typing.Dict[str, torch.Tensor] = {}
        losses = []
        if p.use_language:
            tgt = batch["token_y"]
            n = tgt.numel()
            if self.builder.register:
                loss = torch.zeros([], device="meta")
                acc = torch.zeros([], device="meta")
            else:
                loss, acc = F.softmax_xent(token_out.t, tgt, p.vocab_size, p.z_loss, n)
            res["token_loss"] = loss
            res["accuracy"] = acc
            losses.append(loss)
        if p.use_video:
            out = frame_out.t.float() - vid_tgt.t.float()
            msk = batch.get("vid_msk_tgt")
            if msk is not None:
                m = msk.float().view(list(msk.shape) + [1] * (out.dim() - msk.dim()))
                out = out * m
            vloss = (out * torch.sign(out.detach())).sum() / out.numel()   # ref __init__.py:189-192
            res["video_loss"] = vloss
            losses.append(vloss)
        total = losses[0]
        for extra in losses[1:]:
            total = total + extra
        res["loss"] = total
        return res


def _bcast(pe: Act, like: Act) -> torch.Tensor:
    order = [d for d in like.dims if d in pe.dims]
    t = pe.t.permute([pe.dims.index(d) for d in order])
    return t.reshape([d.size if d in pe.dims else 1 for d in like.dims])


def count_flops_per_token(params: ModelParameter, store) -> float:
    """training FLOPs per token: 6 x (matmul parameters touched per token) + attention score/value products."""
    p = params
    n_mm = sum(s.numel for s in store.specs.values() if len(s.local_shape) >= 2)
    emb = sum(s.numel for n, s in store.specs.items() if "gather" in n)
    attn = 0
    for cfg in p.block_configs:
        for layer in cfg.layer:
            if layer.startswith("attention") and "dot_product" in layer:
                attn += 1
    S = p.sequence_length
    d = p.features
    # causal: half the S x S products; fwd 2 products x 2 FLOP, bwd 2x fwd
    attn_flops = attn * p.depth * 3 * 2 * 2 * S * d / 2
    return 6.0 * (n_mm - emb) + attn_flops
