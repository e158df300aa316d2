"""Fused multi-tensor optimizer step on the GPU (K20, csrc/kernels/optim.hip).

The chain is compiled into *segments*: a segment is one ``opt_apply`` launch over every tensor (chunk table ->
tensor table), and starts at each stage that needs a per-tensor reduction of its input (adaptive/l2/global clip,
gradient centralisation, NovoGrad, Adafactor). Reductions of the raw gradient / weights come from one ``opt_stats``
pass; later ones are accumulated by the previous segment's launch (``emit_stats``). A one-block ``opt_scalar``
launch turns statistics into per-tensor factors. The last segment applies rezero / weight decay, ``w -= u`` and
writes the bf16 compute copy. For the shipped chain ``adaptive_clip-sm3-momentum-learning_rate`` this is three
launches for all parameters together.

Under TP, statistics of sharded tensors are summed over the TP group and SM3 accumulators of non-head dims are
max-reduced (collectives X10-X12), each as ONE packed RCCL call per step.
"""
from __future__ import annotations

import math
import os
import struct
import typing

import torch
import torch.distributed as dist

from ..ops import _lib as L
from ..parallel import state as pstate
from ..utils import debug
from .chain import parse_chain

OP = dict(none=0, adaptive_clip=1, l2norm_clip=2, global_l2norm_clip=3, value_clip=4, gradient_centralisation=5,
          weight_centralisation=6, sm3=7, momentum=8, adam=9, novograd=10, learning_rate=11, adafactor=12,
          adafactor_clip=13, scale=14)
REDUCTIONS = {"adaptive_clip", "l2norm_clip", "global_l2norm_clip", "gradient_centralisation", "novograd",
              "adafactor", "adafactor_clip"}
CHUNK = int(os.environ.get("OBST_OPT_CHUNK", 65536))   # elements per stats / generic-apply block
RW_COLS = 8192                                           # row-tiled apply: column range per chunk (optim.hip)
RW_ELEMS = int(os.environ.get("OBST_OPT_RW_ELEMS", 262144))   # row-tiled apply: elements per chunk (whole rows)


def _f2i(x: float) -> int:
    return struct.unpack("<i", struct.pack("<f", float(x)))[0]


class Segment:
    def __init__(self):
        self.opener: typing.Optional[typing.Tuple[str, tuple]] = None
        self.stages: typing.List[typing.Tuple[str, tuple]] = []
        self.emit_stats = False
        self.emit_factored = False
        self.stats_only = False    # no output: graft's probe of its inner stage (only sum(h^2) is kept)
        self.reuse_input = False   # reads the previous segment's INPUT (graft applies its factor to g, not h)
        self.save_sq = False       # keep sum(g^2) of the input before this segment's statistics replace it


def _graft_inner_ok(args) -> bool:
    """graft:<inner> is fused for every inner stage but Adafactor (its factored statistics need their own pre-pass)
    and the pseudo-stages. A reducing inner stage (novograd, the clips, centralisation) opens the probe segment with
    its own per-tensor factors from the statistics of the graft input -- the same statistics graft keeps."""
    return (bool(args) and args[0] in OP and args[0] not in ("adafactor", "adafactor_clip", "graft", "scale", "none"))


def supported(chain: str) -> bool:
    return all(n != "graft" or _graft_inner_ok(a) for n, a in parse_chain(chain))


def unsupported_reason(chain: str) -> str:
    bad = [a[0] if a else "" for n, a in parse_chain(chain) if n == "graft" and not _graft_inner_ok(a)]
    return f"graft over {bad[0]!r} is not fused" if bad else "supported"


def compile_chain(chain: str) -> typing.Tuple[typing.List[Segment], bool, bool]:
    """-> (segments, needs a pre-pass that materialises factored stats of the raw grad, weight_centralisation)"""
    stages = []
    for n, a in parse_chain(chain):
        stages.append((n, a))
        if n == "adafactor":
            stages.append(("adafactor_clip", ()))
    segs = [Segment()]
    pre_factored = False
    wc = any(n == "weight_centralisation" for n, _ in stages)
    first = True
    for n, a in stages:
        if n == "graft":
            # graft:<inner> (ref src/optimizer/optimizers.py:145-151): u = g * |inner(g)| / |g| per tensor. The
            # probe segment runs the inner stage (its state advances once) for sum(h^2) only; the next segment
            # re-reads g and scales it (opener "graft"), then the chain continues
            if not _graft_inner_ok(a):
                raise ValueError(f"graft over {a!r} is not fused")
            if not first:
                segs[-1].emit_stats = True        # sum(g^2) of the graft input
            probe = Segment()
            probe.stages = [(a[0], tuple(a[1:]))]
            if a[0] in REDUCTIONS:   # the inner stage's per-tensor factors from the graft input's statistics
                probe.opener = (a[0], tuple(a[1:]))
            probe.stats_only = probe.emit_stats = probe.save_sq = True
            apply = Segment()
            apply.opener = ("graft", ())
            apply.reuse_input = True
            apply.stages = [("scale", ())]
            if first:
                segs = [probe, apply]
            else:
                segs += [probe, apply]
            first = False
            continue
        if n in REDUCTIONS:
            if first and n != "adafactor":
                segs[0].opener = (n, a)          # statistics of the raw gradient come from the stats pass
            else:
                if first and n == "adafactor":
                    pre_factored = True           # identity pre-pass emits row/col sums of g^2
                elif n == "adafactor":
                    segs[-1].emit_factored = True
                else:
                    segs[-1].emit_stats = True
                s = Segment()
                s.opener = (n, a)
                segs.append(s)
        segs[-1].stages.append((n, a))
        first = False
    if pre_factored:
        segs[0].emit_factored = True
    return segs, pre_factored, wc


class FusedOptimizer:
    def __init__(self, store, params):
        L.lib()
        self.store, self.params = store, params
        self.chain = params.optimizer
        self.segments, self.pre_factored, self.wc = compile_chain(self.chain)
        names = [n for n in store.order if store.specs[n].trainable]
        self.names = names
        dev = store.device
        self.tp = pstate.tp_size()
        # stage names incl. graft's inner stage (graft:adam needs adam's state)
        chain_names = {n for n, _ in parse_chain(self.chain)} | {a[0] for n, a in parse_chain(self.chain)
                                                                 if n == "graft" and a}
        need_sm3 = "sm3" in chain_names
        need_mom = "momentum" in chain_names or "novograd" in chain_names
        need_adam = "adam" in chain_names
        need_af = "adafactor" in chain_names
        # --- tensor table ----------------------------------------------------------------------------------------
        recs, chunks = [], []
        sm3_local, sm3_red = [], []     # (tensor idx, dim) lists for the two SM3 regions
        fac_total = 0
        self.sharded = []
        for ti, n in enumerate(names):
            s = store.specs[n]
            shape = list(s.local_shape)
            if len(shape) > 4:  # merge leading dims (SM3 then keeps one accumulator for the merged prefix)
                shape = [int(math.prod(shape[:len(shape) - 3]))] + shape[-3:]
            self.sharded.append(s.tp_dim is not None)
            for d in range(len(shape)):
                local = self.tp == 1 or (s.tp_dim is not None and d == s.tp_dim)
                (sm3_local if local else sm3_red).append((ti, d, shape[d]))
            recs.append([s.offset, s.numel, len(shape), shape])
            for st in range(0, s.numel, CHUNK):
                chunks.append(struct.pack("<iiqq", ti, 0, st, min(CHUNK, s.numel - st)))
        # SM3 offsets: local region first, then the region that is max-reduced over TP
        sm3_off = {}
        off = 0
        for ti, d, sz in sm3_local:
            sm3_off[(ti, d)] = off
            off += sz
        self.sm3_red_start = off
        for ti, d, sz in sm3_red:
            sm3_off[(ti, d)] = off
            off += sz
        self.sm3_total = max(off, 1)
        packed = []
        self.fac = {}
        self.tinfo = []
        for ti, (offset, numel, ndim, shape) in enumerate(recs):
            flags = 0
            n = names[ti]
            if store.specs[n].weight_decay_eligible(params):
                flags |= 1
            if store.specs[n].is_rezero:
                flags |= 2
            if self.sharded[ti]:
                flags |= 4
                if need_af and ndim >= 2:   # Adafactor: which factored axis is head-sharded (optim.hip OP_ADAFACTOR)
                    flags |= 16 if store.specs[n].tp_dim == len(store.specs[n].local_shape) - 1 else 8
            dims = (shape + [1, 1, 1, 1])[:4]
            so = [sm3_off.get((ti, d), 0) for d in range(4)]
            frows = fcols = 0
            foff = 0
            if need_af and ndim >= 2:
                fcols = shape[-1]
                frows = numel // fcols
                foff = fac_total
                fac_total += frows + fcols
            packed.append(struct.pack("<qqii4i4qqii", offset, numel, ndim, flags, *dims, *so, foff, frows, fcols))
            self.tinfo.append((offset, numel, shape, [sm3_off.get((ti, d)) for d in range(ndim)], foff, frows, fcols))
        self.ntensors = len(packed)
        self.nchunks = len(chunks)
        # Adafactor: work items of the deterministic factored-statistics kernel (optim.hip opt_factored_kernel,
        # tiles of <= 64 rows x <= 1024 columns) and of its fold, partial-sum slabs, and the TP masks
        fch, folds = [], []
        cp_tot = rp_tot = 0
        af_mask = torch.zeros(max(fac_total, 1), dtype=torch.float32)
        rows_sharded = []
        for ti, (offset, numel, shape, _, foff, frows, fcols) in enumerate(self.tinfo):
            if not frows:
                continue
            nrt, ncc = -(-frows // 64), -(-fcols // 1024)
            cp_off, rp_off = cp_tot, rp_tot
            cp_tot += nrt * fcols
            rp_tot += ncc * frows
            for rt in range(nrt):
                for cc in range(ncc):
                    fch.append(struct.pack("<8iqq", ti, rt * 64, min(64, frows - rt * 64), cc * 1024,
                                           min(1024, fcols - cc * 1024), rt, cc, 0, cp_off, rp_off))
            for r0 in range(0, frows, 256):
                folds.append(struct.pack("<4iqii", ti, 0, r0, min(256, frows - r0), rp_off, ncc, 0))
            for c0 in range(0, fcols, 256):
                folds.append(struct.pack("<4iqii", ti, 1, c0, min(256, fcols - c0), cp_off, nrt, 0))
            fl = struct.unpack_from("<qqii", packed[ti])[3]
            if fl & 16:
                af_mask[foff:foff + frows] = 1.0          # row sums partial: the columns are sharded
            if fl & 8:
                af_mask[foff + frows:foff + frows + fcols] = 1.0   # column sums partial: the rows are sharded
                rows_sharded.append(ti)
        self.nfchunks, self.nfolds = len(fch), len(folds)
        # row-tiled apply (optim.hip opt_rows_kernel) for every >= 1-D tensor when the chain has no Adafactor;
        # the generic apply then only runs the 0-dim tensors
        self.use_rows = not need_af and os.environ.get("OBST_OPT_ROWS", "1") != "0"
        rchunks, schunks = [], []
        for ti, (offset, numel, ndim, shape) in enumerate(recs):
            if not self.use_rows or ndim == 0:
                schunks.extend(c for c in chunks if struct.unpack_from("<i", c)[0] == ti)
                continue
            C = shape[-1]
            R = numel // C
            vec = int(offset % 4 == 0 and C % 4 == 0)
            lpr = C // (4 if vec else 1)
            if lpr <= 64 and lpr & (lpr - 1) == 0:      # narrow rows: several whole rows per block iteration
                vec |= 2
                per = max(1, RW_ELEMS // C)
                for row0 in range(0, R, per):
                    rchunks.append(struct.pack("<6i", ti, row0, min(per, R - row0), 0, C, vec))
                continue
            for col0 in range(0, C, RW_COLS):
                ncols = min(RW_COLS, C - col0)
                per = max(1, RW_ELEMS // ncols)
                for row0 in range(0, R, per):
                    rchunks.append(struct.pack("<6i", ti, row0, min(per, R - row0), col0, ncols, vec))
        self.nrchunks, self.nschunks = len(rchunks), len(schunks)
        # per-tensor (first, count) partial rows for the deterministic statistics fold (optim.hip opt_fold_kernel):
        # over the chunk table, and over [row-tiled chunks..., generic chunks...] for the row-tiled apply
        tid = lambda c: struct.unpack_from("<i", c)[0]  # noqa: E731
        def ranges(tables):
            rng = [[0, 0] for _ in names]
            base = 0
            for table in tables:
                for i, c in enumerate(table):
                    t = tid(c)
                    if rng[t][1] == 0:
                        rng[t][0] = base + i
                    rng[t][1] += 1
                base += len(table)
            return torch.tensor(rng or [[0, 0]], dtype=torch.int32, device=dev).view(-1)
        self.rng_chunks = ranges([chunks])
        self.rng_rows = ranges([rchunks, schunks]) if self.use_rows else self.rng_chunks
        self.part = torch.zeros(max(self.nchunks, self.nrchunks + self.nschunks, 1) * 4, dtype=torch.float32,
                                device=dev)
        self.t_tensors = torch.tensor(bytearray(b"".join(packed)), dtype=torch.uint8, device=dev)
        self.t_chunks = torch.tensor(bytearray(b"".join(chunks)), dtype=torch.uint8, device=dev)
        self.t_rchunks = torch.tensor(bytearray(b"".join(rchunks) or b"\0" * 24), dtype=torch.uint8, device=dev)
        self.t_schunks = torch.tensor(bytearray(b"".join(schunks) or b"\0" * 24), dtype=torch.uint8, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        self.stats = torch.zeros(self.ntensors * 8, **f32)
        self.facs = torch.zeros(self.ntensors * 8, **f32)
        self.sstate = torch.zeros(self.ntensors * 4, **f32)
        self.shard_mask = torch.tensor([1.0 if s else 0.0 for s in self.sharded], **f32).view(-1, 1)
        total = store.total
        self.mom = torch.zeros(total, **f32) if need_mom else None
        self.adam_m = torch.zeros(total, **f32) if need_adam else None
        self.adam_v = torch.zeros(total, **f32) if (need_adam or need_af) else None
        self.sm3 = [torch.zeros(self.sm3_total, **f32), torch.zeros(self.sm3_total, **f32)] if need_sm3 else None
        self.af_state = torch.zeros(max(fac_total, 1), **f32) if need_af else None
        self.af_sums = torch.zeros(max(fac_total, 1), **f32) if need_af else None
        if need_af:
            self.t_fchunks = torch.tensor(bytearray(b"".join(fch) or b"\0" * 48), dtype=torch.uint8, device=dev)
            self.t_folds = torch.tensor(bytearray(b"".join(folds) or b"\0" * 32), dtype=torch.uint8, device=dev)
            self.colpart = torch.empty(max(cp_tot, 1), **f32)
            self.rowpart = torch.empty(max(rp_tot, 1), **f32)
            self.af_mask = af_mask.to(dev)
            rs = torch.zeros(self.ntensors, **f32)
            rs[rows_sharded] = 1.0
            self.af_rows_sharded = rs.view(-1, 1)
            self.af_factored = torch.tensor([1.0 if t[5] else 0.0 for t in self.tinfo], **f32)
        n_out = sum(1 for sg in self.segments[:-1] if not sg.stats_only) + int(self.pre_factored)
        self.u = torch.empty(total, **f32) if n_out >= 1 else None
        self.u2 = torch.empty(total, **f32) if n_out >= 2 else None
        self.graft_g2 = torch.zeros(self.ntensors, **f32) if any(sg.save_sq for sg in self.segments) else None
        self.flip = 0
        # [lr, step_count] on the device: the kernels read them from here, so a captured step (hipGraph replay,
        # Trainer with use_hip_graphs) sees each step's values; ``external_dyn``: the caller fills them
        self.dyn = torch.zeros(2, **f32)
        self.external_dyn = False

    # ------------------------------------------------------------------------------------------------------------
    def _desc(self, lr, step_count, grad_scale):
        s = self.store
        d = L.OptDesc()
        d.tensors, d.chunks = self.t_tensors.data_ptr(), self.t_chunks.data_ptr()
        d.ntensors, d.nchunks = self.ntensors, self.nchunks
        d.grad, d.master = s.grad.data_ptr(), s.master.data_ptr()
        d.compute = s.compute.data_ptr() if s.compute is not s.master else 0
        d.stats, d.fac, d.sstate = self.stats.data_ptr(), self.facs.data_ptr(), self.sstate.data_ptr()
        d.mom = L.ptr(self.mom)
        d.adam_m, d.adam_v = L.ptr(self.adam_m), L.ptr(self.adam_v)
        if self.sm3 is not None:
            d.sm3_old, d.sm3_new = self.sm3[self.flip].data_ptr(), self.sm3[1 - self.flip].data_ptr()
        d.af_state = L.ptr(self.af_state)
        d.af_rows_sum = d.af_cols_sum = L.ptr(self.af_sums)
        p = self.params
        d.lr, d.wd, d.rezero_mult, d.grad_scale = lr, p.weight_decay, p.rezero_lr_multiplier, grad_scale
        d.beta1, d.beta2, d.step_count = p.opt_beta1, p.opt_beta2, float(step_count)
        d.tp_size = self.tp
        d.dyn = self.dyn.data_ptr()
        d.part, d.part_base = self.part.data_ptr(), 0
        return d

    def set_dyn(self, lr: float, step_count: int):
        """stream-ordered fills of the device-side learning rate / step (outside any captured region)"""
        self.dyn[0].fill_(float(lr))
        self.dyn[1].fill_(float(step_count))

    def _set_stages(self, d, stages):
        if len(stages) > 8:
            raise ValueError("at most 8 stages per fused segment")
        arr = [0] * 32
        for i, (n, a) in enumerate(stages):
            vals = [float(x) for x in a[:3]] + [0.0] * (3 - len(a[:3]))
            if n == "adafactor":
                vals = [float(a[0]) if a else 0.0, 0.0, 0.0]
            arr[4 * i:4 * i + 4] = [OP[n], _f2i(vals[0]), _f2i(vals[1]), _f2i(vals[2])]
        d.stages = (L.c_i * 32)(*arr)
        d.nst = len(stages)

    def _reduce_stats(self):
        if self.tp > 1:
            st = self.stats.view(-1, 8)
            part = st * self.shard_mask
            pstate.tp_all_reduce(part)
            st.copy_(part + st * (1 - self.shard_mask))

    def _scalar(self, d, stage):
        if stage[0] == "graft":    # F[0] = sqrt(sum h^2 / sum g^2) (0 where g is all zero: no NaN update)
            st, fac = self.stats.view(-1, 8), self.facs.view(-1, 8)
            g2 = self.graft_g2
            fac[:, 0] = torch.where(g2 > 0, torch.sqrt(st[:, 0]) * torch.rsqrt(g2.clamp(min=1e-38)),
                                    torch.zeros_like(g2))
            return
        self._set_stages(d, [stage])
        L.check(L.lib().obst_opt_scalar(d, L.stream_ptr()), "opt_scalar")
        if stage[0] == "adafactor" and self.tp > 1:
            # the mean of the row factors over the FULL rows: sum(R) partial where the rows are head-sharded
            fac = self.facs.view(-1, 8)
            part = fac[:, 6:7] * self.af_rows_sharded
            pstate.tp_all_reduce(part)
            msum = part + fac[:, 6:7] * (1 - self.af_rows_sharded)
            fac[:, 5:6] = torch.where(self.af_factored.view(-1, 1) > 0, fac[:, 7:8] / msum.clamp(min=1e-30),
                                      fac[:, 5:6])

    def _factored(self, d, u):
        """Adafactor row / column sums of the segment output u into af_sums (deterministic), TP-reduced"""
        L.check(L.lib().obst_opt_factored(d, u.data_ptr(), self.t_fchunks.data_ptr(), self.nfchunks,
                                          self.t_folds.data_ptr(), self.nfolds, self.colpart.data_ptr(),
                                          self.rowpart.data_ptr(), L.stream_ptr()), "opt_factored")
        if self.tp > 1:
            part = self.af_sums * self.af_mask
            pstate.tp_all_reduce(part)
            self.af_sums.copy_(part + self.af_sums * (1 - self.af_mask))

    @torch.no_grad()
    def step(self, lr: float, step_count: int, grad_scale: float = 1.0):
        lib = L.lib()
        sp = L.stream_ptr()
        if not self.external_dyn:
            self.set_dyn(lr, step_count)
        d = self._desc(lr, step_count, grad_scale)
        L.check(lib.obst_opt_stats(d, sp), "opt_stats")
        L.check(lib.obst_opt_fold(d, self.rng_chunks.data_ptr(), 4, sp), "opt_fold")
        self._reduce_stats()
        if self.wc:
            self._scalar(d, ("weight_centralisation", ()))
        if self.sm3 is not None:
            self.sm3[1 - self.flip].zero_()
        src = prev_src = None    # None = raw gradient
        bufs = [self.u, self.u2]
        bi = 0
        if self.pre_factored:
            d.uin, d.uout = 0, bufs[bi].data_ptr()
            self._set_stages(d, [])
            d.final_seg, d.emit_stats, d.emit_factored = 0, 0, 0
            L.check(lib.obst_opt_apply(d, sp), "opt_apply(pre)")
            self._factored(d, bufs[bi])
            src, bi = bufs[bi], 1 - bi
        segs = self.segments[1:] if (self.pre_factored and not self.segments[0].stages) else self.segments
        for k, seg in enumerate(segs):
            if seg.opener is not None:
                self._scalar(d, seg.opener)
            last = k == len(segs) - 1
            if seg.reuse_input:
                src = prev_src
            prev_src = src
            if seg.save_sq:
                self.graft_g2.copy_(self.stats.view(-1, 8)[:, 0])
            d.uin = 0 if src is None else src.data_ptr()
            d.uout = 0 if (last or seg.stats_only) else bufs[bi].data_ptr()
            self._set_stages(d, seg.stages)
            d.final_seg, d.emit_stats, d.emit_factored = int(last), int(seg.emit_stats), 0
            if self.use_rows:
                d.part_base = 0
                L.check(lib.obst_opt_apply_rows(d, self.t_rchunks.data_ptr(), self.nrchunks, sp), "opt_apply_rows")
                d.chunks, d.nchunks, d.part_base = self.t_schunks.data_ptr(), self.nschunks, self.nrchunks
                L.check(lib.obst_opt_apply(d, sp), "opt_apply")
                d.chunks, d.nchunks, d.part_base = self.t_chunks.data_ptr(), self.nchunks, 0
            else:
                L.check(lib.obst_opt_apply(d, sp), "opt_apply")
            if seg.emit_stats:
                L.check(lib.obst_opt_fold(d, self.rng_rows.data_ptr(), 2, sp), "opt_fold")
                self._reduce_stats()
            if seg.emit_factored:
                self._factored(d, bufs[bi])
            if not last and not seg.stats_only:
                src, bi = bufs[bi], 1 - bi
        self.store.bump()
        if self.sm3 is not None:
            if self.tp > 1 and self.sm3_red_start < self.sm3_total:
                red = self.sm3[1 - self.flip][self.sm3_red_start:]
                debug.record("tp_all_reduce_max", red)
                dist.all_reduce(red, op=dist.ReduceOp.MAX, group=pstate.mesh().tp_group)
            self.flip = 1 - self.flip

    # ------------------------------------------------------------------------------------------------------------
    def named_slots(self) -> typing.Dict[str, torch.Tensor]:
        """views of the optimizer state per variable, keyed like the reference's slot variables
        (``<var>/<optimizer string with : -> _>/<slot>``, src/optimizer/backend.py:23-25) and like
        ``ReferenceOptimizer.state_dict`` -- so checkpoints move between the fused and the reference optimizer."""
        chain = {n for n, _ in parse_chain(self.chain)} | {a[0] for n, a in parse_chain(self.chain) if n == "graft" and a}
        opt_str = self.chain.replace(':', '_')
        out: typing.Dict[str, torch.Tensor] = {}
        for ti, name in enumerate(self.names):
            offset, numel, shape, sm3o, foff, frows, fcols = self.tinfo[ti]
            full = list(self.store.specs[name].local_shape)
            key = f"{name}/{opt_str}/"
            flat = lambda buf: buf[offset:offset + numel].view(full)  # noqa: E731
            if not full:       # 0-dim: sm3/novograd/adam all fall back to scalar adam state
                if chain & {"sm3", "novograd", "adam"}:
                    out[key + "exp_avg_p1"] = self.sstate[ti * 4:ti * 4 + 1].view(())
                    out[key + "exp_avg_p2"] = self.sstate[ti * 4 + 1:ti * 4 + 2].view(())
                if "momentum" in chain:
                    out[key + "momentum"] = flat(self.mom)
                continue
            if "sm3" in chain:
                for d, o in enumerate(sm3o):
                    out[key + f"dim{d}"] = self.sm3[self.flip][o:o + shape[d]]
            if "adam" in chain:
                out[key + "exp_avg_p1"] = flat(self.adam_m)
                out[key + "exp_avg_p2"] = flat(self.adam_v)
            if "novograd" in chain:
                out[key + "exp_avg_p1"] = flat(self.mom)
                out[key + "exp_avg_p2"] = self.sstate[ti * 4 + 2:ti * 4 + 3].view(())
            elif "momentum" in chain:
                out[key + "momentum"] = flat(self.mom)
            if "adafactor" in chain:
                if frows:
                    out[key + "af_rows"] = self.af_state[foff:foff + frows]
                    out[key + "af_cols"] = self.af_state[foff + frows:foff + frows + fcols]
                else:
                    out[key + "af_v"] = flat(self.adam_v)
        return out

    def state_dict(self) -> typing.Dict[str, torch.Tensor]:
        out = {"flip": torch.tensor(self.flip)}
        for k in ("mom", "adam_m", "adam_v", "af_state", "sstate"):
            v = getattr(self, k)
            if v is not None:
                out[k] = v
        if self.sm3 is not None:
            out["sm3"] = self.sm3[self.flip]
        return out

    def load_state_dict(self, sd):
        for k in ("mom", "adam_m", "adam_v", "af_state", "sstate"):
            if k in sd and getattr(self, k) is not None:
                getattr(self, k).copy_(sd[k])
        if self.sm3 is not None and "sm3" in sd:
            self.flip = 0
            self.sm3[0].copy_(sd["sm3"])
