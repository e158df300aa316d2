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
from ..ops import aux as X
from ..ops import functional as F
from ..ops import raw as R
from . import dims as D
from .context import Act, BlockArgs, Builder, KVCache
from .frontend import block_part_fn
from .layers import embed, gather_embed, linear, linear_to_features, named_einsum, dropout
from .reversible import run_body


def padded_vocab(params: ModelParameter) -> int:
    m = int(params.pad_vocab_to or 1)
    return (params.vocab_size + m - 1) // m * m


class Model:
    def __init__(self, params: ModelParameter, device: typing.Union[str, torch.device] = "cpu",
                 tp_rank: int = 0, tp_size: int = 1, dtype: typing.Optional[torch.dtype] = None,
                 init_device: typing.Optional[torch.device] = None, local_batch: typing.Optional[int] = None,
                 finalize: bool = True):
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
        self.store = self.builder.store
        if finalize:   # finalize=False: shapes only (memory sizing, utils/memory.py) -- no buffers are allocated
            self.store.finalize(self.device, self.dtype, init_device=init_device)

    # ---------------------------------------------------------------------------------------------------------------
    def _dummy_inputs(self, device):
        p = self.params
        B = self.local_batch
        x = None
        if p.use_language:
            shape = [B, p.sequence_length // p.token_patch_size, p.token_patch_size]
            if p.use_video:   # jannet: [batch, time, language_token_patch, token_patch]
                shape = [B, p.time_patch_size, p.language_token_patch, p.token_patch_size]
            x = torch.zeros(shape, dtype=torch.int64, device=device)
        vid = None
        if p.use_video:
            shape = [B, p.time_patch_size + 1, p.frame_height_patch, p.frame_width_patch, p.channel_color_size]
            if not p.three_axes:
                shape = [B, p.time_patch_size + 1, p.frame_height_patch * p.frame_width_patch, p.channel_color_size]
            vid = torch.zeros(shape, dtype=torch.uint8, device=device)
        return {"token_x": x, "token_y": x, "frame": vid}

    def forward(self, token_x=None, token_y=None, frame=None, vid_msk_src=None, vid_msk_tgt=None, cat_mask_x=None,
                cat_mask_y=None, txt_msk=None, train=True, step_seed: int = 0) -> typing.Dict[str, torch.Tensor]:
        self.builder.train = train
        self.builder.step_seed = step_seed
        return self._forward({"token_x": token_x, "token_y": token_y, "frame": frame,
                              "vid_msk_src": vid_msk_src, "vid_msk_tgt": vid_msk_tgt,
                              "cat_mask_x": cat_mask_x, "cat_mask_y": cat_mask_y})

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

    # ---- incremental decoding (serving) ----------------------------------------------------------------------------
    def supports_kv_cache(self) -> bool:
        """bodies whose only sequence mixing is causal dot-product attention on the fused path (GPT-style) decode
        incrementally; everything else recomputes the context per token (as the reference does)"""
        p = self.params
        cfg = " ".join(str(c.layer) for c in list(p.block_configs) + list(p.input_block_configs) +
                       list(p.output_block_configs))
        # cumsum / cummean and the learned token mixer (biased_attention_map on input_as_value) decode from their
        # own caches (layers._cumsum_any / _mixer_kv); a layer that runs uncached during the prefill makes it fail
        mixing = ("convolution", "transpose_sequence_features", "biased_softmax", "scale_attention_map",
                  "embedded", "positional", "shared_key_value")
        return (p.use_language and not p.use_video and not p.use_initial_position_embedding
                and not p.input_block_configs and not p.output_block_configs and self.builder.tp_size == 1
                and ("attention" in cfg or "cumsum" in cfg or "cummean" in cfg) and not any(m in cfg for m in mixing)
                and not (p.contrastive_across_samples or p.contrastive_across_token_embeddings))

    @torch.no_grad()
    def prefill(self, token_x: torch.Tensor, positions: torch.Tensor) -> torch.Tensor:
        """Start incremental decoding: one forward over the whole context that fills the per-layer KV caches;
        returns the logits at ``positions`` ([B, 1, patch, vocab])"""
        if not hasattr(self, "_kv_persist"):
            self._kv_persist = {"bufs": {}, "graph": None}
        kv = KVCache(self._kv_persist)
        self.builder.kv = kv
        try:
            out = self.logits(token_x, positions=positions)
        except BaseException:
            self.builder.kv = None
            raise
        if kv.idx != self.builder.params.attention_idx or (kv.idx == 0 and kv.cidx == 0) or kv.unsupported:
            self.builder.kv = None          # a mixing layer bypassed the cache: not decodable incrementally
            raise NotImplementedError("body is not KV-cache decodable")
        kv.mode = "decode"
        return out

    @torch.no_grad()
    def decode(self, tokens: torch.Tensor, positions: torch.Tensor) -> torch.Tensor:
        """One incremental step: ``tokens`` [B, 1, patch] sit at ``positions`` [B]; their k / v join the caches and
        the logits of that position come back ([B, 1, patch, vocab])"""
        kv = self.builder.kv
        if kv is None or kv.mode != "decode":
            raise RuntimeError("decode() needs prefill() first")
        if self.device.type == "cuda" and getattr(self.params, "decode_hip_graphs", True):
            return self._decode_graphed(kv, tokens, positions)
        kv.pos = positions.to(self.device, torch.int64).contiguous()
        return self.logits(tokens)

    def _decode_graphed(self, kv: KVCache, tokens: torch.Tensor, positions: torch.Tensor) -> torch.Tensor:
        """A decode step is ~25 small launches per layer at sequence length 1: launch-bound. It is captured once per
        batch shape and cache layout in a hipGraph and replayed, across requests too (KVCache.persist); tokens /
        positions go through static device buffers, the KV caches keep fixed addresses and the decode kernel reads
        the positions from device memory. A re-run of a step is idempotent (the cache append rewrites the same
        k / v), so the eager warm-up runs feed the very step they warm up. The returned logits are the graph's
        static output: valid until the next step."""
        g = kv.persist["graph"]
        if g is None or g["shape"] != tuple(tokens.shape):
            tok = tokens.to(self.device).clone()
            kv.pos = positions.to(self.device, torch.int64).clone()
            side = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):
                for _ in range(2):     # first-use GEMM plans, workspaces, allocator growth
                    self.logits(tok)
            torch.cuda.current_stream(self.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                out = self.logits(tok)
            g = kv.persist["graph"] = {"shape": tuple(tokens.shape), "graph": graph, "tok": tok, "pos": kv.pos,
                                       "out": out}
        else:
            g["tok"].copy_(tokens, non_blocking=True)
            g["pos"].copy_(positions, non_blocking=True)
        g["graph"].replay()
        return g["out"]

    def end_decode(self):
        self.builder.kv = None

    @torch.no_grad()
    def predict(self, batch: dict) -> typing.Tuple[typing.Optional[torch.Tensor], typing.Optional[torch.Tensor]]:
        """Inference forward returning (frame_out [B, T, ..., C] in [0, 1], token logits) for the video sampling loop
        (ref src/run/inference.py:27-36)."""
        self.builder.train = False
        return self._forward(dict(batch, token_y=None), logits_only="outputs")

    def _forward(self, batch: dict, logits_only: typing.Union[bool, str] = False):
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
            if logits_only == "outputs":
                return (None if frame_out is None else frame_out.t), (None if token_out is None else token_out.t)
            if logits_only:
                if pos is not None and p.output_block_configs:
                    idx = pos.to(token_out.t.device).long()
                    return token_out.t[torch.arange(token_out.t.shape[0], device=idx.device), idx].unsqueeze(1)
                return token_out.t
            with b.scope("loss"):
                return self._loss(frame_out, token_out, batch, vid_tgt)

    # ---------------------------------------------------------------------------------------------------------------
    def _contrastive_samples(self, token_out: Act) -> torch.Tensor:
        return _contrastive_samples_impl(token_out.t, token_out.dims, self.builder.params)

    def _contrastive_embeddings(self, token_out: Act, tgt: torch.Tensor) -> torch.Tensor:
        """ref __init__.py:172-179 taken literally: the features and the embedding table share no named dim, so both
        einsums reduce to products of sums: (sum(out) * sum(E) - 2 * sum(out) * sum(E[tgt])) / (|out| * vocab)"""
        p = self.builder.params
        table = self._text_table
        gathered = table[tgt.reshape(-1).long().clamp(0, table.shape[0] - 1)].float()
        so = token_out.t.sum()
        loss = so * table.float().sum() - 2 * so * gathered.sum()
        return loss / (token_out.t.numel() * p.vocab_size)

    def _frames(self, vid: torch.Tensor) -> torch.Tensor:
        """uint8 (or bit-folded int) frames -> activation dtype in [0, 1] (ref __init__.py:37-55)"""
        p = self.builder.params
        folds = p.fold_count if p.use_bit_fold_input_pipeline else 1
        if (R.on_gpu(vid) and self.builder.dtype == torch.bfloat16 and vid.dtype in (torch.uint8, torch.int32)
                and not self.builder.register):
            # one pass: bit unfold + scale to [0, 1] in the frame kernel (K24)
            C = vid.shape[-1]
            y = torch.empty(list(vid.shape[:-1]) + [C * folds], dtype=torch.bfloat16, device=vid.device)
            R.frames(vid.contiguous(), y, vid.numel() // C, C, folds,
                     2 ** p.bit_fold_value if p.use_bit_fold_input_pipeline else 256)
            return y
        if p.use_bit_fold_input_pipeline:
            v = vid.long()
            base = 2 ** p.bit_fold_value
            parts = [((v // base ** i) % base).to(torch.uint8) for i in range(p.fold_count)]
            vid = torch.cat(parts, -1)
        return vid.to(self.builder.dtype) / 255.0

    def _input(self, batch):
        """ref src/model/__init__.py:32-91: video patches and/or language tokens -> features; jannet concatenates
        language tokens and frame patches along the spatial ("height") axis."""
        b = self.builder
        p = b.params
        tgt = None
        src = None
        if p.use_video:
            vid = batch["frame"]
            vdims = [Dim("batch", vid.shape[0]), Dim("_sequence", vid.shape[1])]
            vdims += [Dim("height", vid.shape[2])] + ([Dim("width", vid.shape[3])] if p.three_axes else [])
            v = self._frames(vid)
            vdims += [Dim(p.color_channel_dim.name, v.shape[-1])]
            v = dropout(BlockArgs(b, Act(v, vdims), [f"dropout_rate{p.input_dropout}"])).t
            seq = Dim("sequence", vid.shape[1] - 1)
            sdims = [vdims[0], seq] + vdims[2:]
            src = Act(v[:, :-1].contiguous(), sdims)
            tgt = Act(v[:, 1:].contiguous(), sdims)
            args = BlockArgs(b, src, [''])
            if p.empty_frame_embedding is not None:
                e = embed(args(list(p.empty_frame_embedding)), sdims[2:])
                for key in ("vid_msk_src", "cat_mask_x"):       # weighted_add(src, embed, mask) twice (ref :60-62)
                    msk = batch.get(key)
                    if msk is not None:
                        m = msk.to(b.dtype).view(list(msk.shape) + [1] * (len(sdims) - 2))
                        src = Act(src.t * m + e.t.unsqueeze(0).unsqueeze(0) * (1 - m), sdims)
            src = linear_to_features(args(src), [sdims[-1]])
            for ci, cfg in enumerate(p.input_block_configs):
                src = block_part_fn(b, cfg, src, 0, ci, prefix="vid_inp")
        if p.use_language:
            tok = batch["token_x"]
            tdims = [Dim("batch", tok.shape[0]), Dim("sequence", tok.shape[1])]
            if tok.dim() == 4:                                    # jannet: [batch, time, lang_patch, token_patch]
                tdims.append(Dim("height", tok.shape[2]))
            tdims.append(p.token_patch_dim)
            args = BlockArgs(b, Act(tok, tdims), [''])
            inter = Dim(p.intermediate[0].name, int(p.intermediate[0].size * p.vocab_weight_factorization))
            txt = gather_embed(args(list(p.token_embedding)), [p.vocab_dim, inter], tok, tdims)
            self._text_table = b.last_gather_table
            txt = dropout(args(txt, [f"dropout_rate{p.input_dropout}"]))
            txt = linear_to_features(args(txt), [p.token_patch_dim, inter])
            for ci, cfg in enumerate(p.input_block_configs):
                txt = block_part_fn(b, cfg, txt, 0, ci, prefix="lang_inp")
            if src is not None:
                src = _concat_height(txt, src)
            else:
                src = txt
        if p.use_initial_position_embedding:
            args = BlockArgs(b, src, [''])
            for dim in D.subtract(src.dims, p.feature_dims)[1:]:
                pe = embed(args(list(p.position_embedding)), [dim] + list(p.feature_dims))
                src = Act(src.t + _bcast(pe, src), src.dims)
        return src, tgt

    def _output(self, out: Act):
        """ref src/model/__init__.py:133-156: the first language_token_patch spatial slots are tokens, the rest frames"""
        b = self.builder
        p = b.params
        token_out = frame_out = None
        joint = p.use_video and p.use_language
        lp = p.language_token_patch
        contrastive = p.contrastive_across_samples or p.contrastive_across_token_embeddings
        if p.use_language and contrastive:
            # ref __init__.py:138-139,165: the contrastive losses work on the body's features (no output embedding)
            x = _slice_height(out, 0, lp) if joint else out
            fi = [x.dims.index(d) for d in p.feature_dims]
            t = x.t.float()
            t = t / t.pow(2).sum(fi, keepdim=True).sqrt()
            token_out = Act(t, x.dims)
        elif p.use_language:
            x = _slice_height(out, 0, lp) if joint else out
            for ci, cfg in enumerate(p.output_block_configs):
                x = block_part_fn(b, cfg, x, 0, ci, prefix="lang_out")
            args = BlockArgs(b, x, [''])
            new = [p.token_patch_dim, p.vocab_dim]
            w = embed(args(x, list(p.output_embedding)), list(p.feature_dims) + new)
            odims = D.subtract(x.dims, p.feature_dims) + new
            try:
                y = F.linear(x.t, w.t, x.dims, w.dims, odims)
            except NotImplementedError:
                y = F.tp_reduce(named_einsum([x, w], odims).t)
            token_out = Act(y, odims)
        if p.use_video:
            x = _slice_height(out, lp, None) if joint else out
            for ci, cfg in enumerate(p.output_block_configs):
                x = block_part_fn(b, cfg, x, 0, ci, prefix="vid_out")
            y = linear(BlockArgs(b, x, ['']), p.feature_dims, [p.color_channel_dim])
            if R.on_gpu(y.t) and (y.t.dtype != torch.bfloat16 or y.t.numel() % 8):
                frame_out = Act(torch.sigmoid(y.t.float()).to(y.t.dtype), y.dims)
            else:
                frame_out = Act(F.activation(y.t, "sigmoid"), y.dims)
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
            elif p.contrastive_across_samples:
                loss, acc = self._contrastive_samples(token_out), None
            elif p.contrastive_across_token_embeddings:
                loss, acc = self._contrastive_embeddings(token_out, tgt), None
            else:
                loss, acc = F.softmax_xent(token_out.t, tgt, p.vocab_size, p.z_loss, n)
            res["token_loss"] = loss
            if acc is not None:
                res["accuracy"] = acc
            losses.append(loss)
        if p.use_video:
            if self.builder.register:
                vloss = torch.zeros([], device="meta")
                res["video_loss"] = vloss
                losses.append(vloss)
            else:
                fo, tg = frame_out.t, vid_tgt.t
                scale = 1.0
                masks = []
                for key in ("vid_msk_tgt", "cat_mask_y"):
                    msk = batch.get(key)
                    if msk is not None:
                        masks.append(msk.float())
                        scale *= msk.numel() / masks[-1].sum().clamp(min=1.0)
                mask = None
                if masks:        # masks cover leading dims of the frames (ref: mask broadcast over the trailing dims)
                    r = max(m.dim() for m in masks)
                    for m in masks:
                        m = m.view(list(m.shape) + [1] * (r - m.dim()))
                        mask = m if mask is None else mask * m
                    mask = mask.expand(list(fo.shape[:r]))
                # masked L1 (sum |d| with gradient sign(d) * mask) in one pass (K24), ref __init__.py:187-199
                vloss = X.masked_l1(fo, tg, mask) / fo.numel()
                losses.append(vloss)
                res["video_loss_raw"] = vloss
                res["video_loss"] = vloss.detach() * scale                  # reported loss rescaled by the masks
        if not losses:
            raise ValueError("neither use_language nor use_video")
        total = losses[0]
        for extra in losses[1:]:
            total = total + extra
        res["loss"] = total
        return res


def _contrastive_samples_impl(t: torch.Tensor, dims, p) -> torch.Tensor:
    """ref __init__.py:167-171: (|sum over batch|^2 / B - |sum over sequence|^2 / S) / (B S)"""
    names = [d.name for d in dims]
    bi, si = names.index("batch"), names.index("sequence")
    over_samples = t.sum(si)
    over_batch = t.sum(bi)
    B, S = t.shape[bi], t.shape[si]
    loss = over_batch.pow(2).sum() / B - over_samples.pow(2).sum() / S
    return loss / (B * S)


def _concat_height(a: Act, b: Act) -> Act:
    """concatenate two activations along their "height" axis (all other dims equal)"""
    ia = [d.name for d in a.dims].index("height")
    ib = [d.name for d in b.dims].index("height")
    rest_a = [d for d in a.dims if d.name != "height"]
    rest_b = [d for d in b.dims if d.name != "height"]
    if rest_a != rest_b or ia != ib:
        raise ValueError(f"cannot concatenate {a.dims} and {b.dims} along height (jannet needs three_axes=false)")
    t = torch.cat([a.t, b.t], ia)
    dims = list(a.dims)
    dims[ia] = Dim("height", a.dims[ia].size + b.dims[ib].size)
    return Act(t, dims)


def _slice_height(x: Act, start: int, stop: typing.Optional[int]) -> Act:
    i = [d.name for d in x.dims].index("height")
    stop = x.dims[i].size if stop is None else stop
    t = x.t.narrow(i, start, stop - start).contiguous()
    dims = list(x.dims)
    dims[i] = Dim("height", stop - start)
    return Act(t, dims)


def _bcast(pe: Act, like: Act) -> torch.Tensor:
    order = [d for d in like.dims if d in pe.dims]
    t = pe.t.permute([pe.dims.index(d) for d in order])
    return t.reshape([d.size if d in pe.dims else 1 for d in like.dims])


def count_flops_per_token(params: ModelParameter, store) -> float:
    """training FLOPs per token: 6 x (matmul parameters touched per token) + attention score/value products + the
    learned token mixers, counted per application (layers._note_mixer: 3 x 2 x features x mixed positions, the
    causal half) and not as 6 x their weight -- a depth-shared [heads, S, S] mixer weight is one variable that
    every block applies."""
    p = params
    mixer_vars = getattr(store, "mixer_vars", set())
    n_mm = sum(s.numel for n, s in store.specs.items() if len(s.local_shape) >= 2 and n not in mixer_vars)
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
    return 6.0 * (n_mm - emb) + attn_flops + float(getattr(store, "mixer_flops", 0.0))
