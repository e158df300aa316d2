"""Data-parallel gradient all-reduce over RCCL, bucketed and overlapped with backward (collective X08/X09).

The flat fp32 gradient buffer is cut into contiguous buckets in *reverse* registration order (the order backward
produces them: output projection first, input embedding last). Every op that writes a weight gradient calls
``grad_ready(weight)``; when the last use of every variable in a bucket has reported, the bucket's reduction is
queued on RCCL's stream (``async_op=True`` orders it after the current compute stream's work without blocking it).
``finish()`` flushes the remaining buckets (incl. variables whose gradients arrive via plain autograd) and makes the
compute stream wait for all of them before the optimizer step.

Bucket sizing for xGMI: a ring collective is per-link bound (~153 GB/s per link), so few large buckets
beat many small ones, but the last bucket is exposed after backward. ``grad_bucket_mb = 0`` (default) sizes them
from the model: the gradient buffer in ``target_buckets`` (12) pieces, at least 16 MiB each -- GPT-Neo-1.3B issues 12
reductions of ~450 MiB fp32 per step instead of ~80 of 64 MiB.

Wire dtype (``allreduce_dtype``):
  * "bfloat16" (default): each bucket travels as bf16 with fp32 accumulation -- an all-to-all hands every rank one
    1/world slice of every rank's bf16 bucket, the rank sums its slice in fp32 (one bf16 rounding of the result
    instead of one per ring step of a bf16 all-reduce), and an all-gather returns the summed slices. The bytes on
    the wire are a bf16 ring all-reduce's: half of the fp32 wire's 2 (w-1)/w x 4 B per parameter. The casts and the
    fp32 slice sum run on a side stream between the two collectives.
  * "float32": one RCCL all-reduce of the fp32 bucket.
The embedding gradient (reference bug A5: no DP reduction) is part of the buffer, so it is reduced like every other
gradient.
"""
from __future__ import annotations

import typing

import torch
import torch.distributed as dist

from ..utils import debug

from ..ops import functional as F


def bucket_cap(total_numel: int, bucket_mb: float, target_buckets: int = 12, min_mb: float = 16.0) -> int:
    """fp32 elements per bucket: ``bucket_mb`` if set (> 0), else the buffer in ``target_buckets`` pieces of at least
    ``min_mb``"""
    if bucket_mb and bucket_mb > 0:
        return max(int(bucket_mb * 2 ** 20 // 4), 1)
    return max(-(-int(total_numel) // target_buckets), int(min_mb * 2 ** 20 // 4), 1)


class GradSync:
    def __init__(self, store, group, world: int, bucket_mb: float = 0.0, dtype: torch.dtype = torch.bfloat16,
                 use_counts: typing.Optional[typing.Dict[str, int]] = None, force: bool = False):
        self.store = store
        self.group = group
        self.world = world
        self.dtype = dtype
        # force: run the collectives at world 1 too (tests of the capture path on a one-GPU RCCL group)
        self.enabled = world > 1 or force
        self.use_counts = dict(use_counts or {})
        total = sum(store.specs[n].numel for n in store.order)
        cap = bucket_cap(total, bucket_mb)
        self.buckets: typing.List[typing.Tuple[int, int, typing.List[str]]] = []
        names = list(reversed(store.order))
        cur: typing.List[str] = []
        for n in names:
            cur.append(n)
            lo = min(store.specs[m].offset for m in cur)
            hi = max(store.specs[m].offset + store.specs[m].numel for m in cur)
            if hi - lo >= cap:
                self.buckets.append((lo, hi, cur))
                cur = []
        if cur:
            lo = min(store.specs[m].offset for m in cur)
            hi = max(store.specs[m].offset + store.specs[m].numel for m in cur)
            self.buckets.append((lo, hi, cur))
        # make buckets tile the buffer without gaps (alignment padding belongs to a neighbour)
        self.var_bucket = {}
        for bi, (_, _, vs) in enumerate(self.buckets):
            for v in vs:
                self.var_bucket[v] = bi
        self._wire = None       # bf16 wire buffers (send / gather and receive), one slice per bucket, lazily
        self._side = None
        self.reset()

    def reset(self):
        self.remaining = {n: self.use_counts.get(n, 1) for n in self.store.order}
        self.pending = [len(vs) for _, _, vs in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.works = []

    # -- bf16 wire, fp32 accumulation -----------------------------------------------------------------------------
    def _padded(self, lo: int, hi: int) -> int:
        return -(-(hi - lo) // self.world) * self.world

    def _wire_buffers(self, device):
        if self._wire is None:
            offs, o = [], 0
            for lo, hi, _ in self.buckets:
                offs.append(o)
                o += self._padded(lo, hi)
            send = torch.zeros(o, dtype=self.dtype, device=device)
            recv = torch.empty(o, dtype=self.dtype, device=device)
            self._wire = (offs, send, recv)
            if device.type == "cuda":
                self._side = torch.cuda.Stream(device=device)
        return self._wire

    def _launch_lowp(self, bi: int, t: torch.Tensor):
        lo, hi, _ = self.buckets[bi]
        offs, send_all, recv_all = self._wire_buffers(t.device)
        n, npad = hi - lo, self._padded(lo, hi)
        send = send_all[offs[bi]:offs[bi] + npad]
        recv = recv_all[offs[bi]:offs[bi] + npad]
        chunk = npad // self.world
        send[:n].copy_(t)   # bf16 cast on the compute stream, in order after the bucket's last gradient
        side = self._side
        ctx = torch.cuda.stream(side) if side is not None else _nullctx()
        if side is not None:
            side.wait_stream(torch.cuda.current_stream(t.device))
        with ctx:
            debug.record("dp_all_to_all", send)
            w1 = dist.all_to_all_single(recv, send, group=self.group, async_op=True)
            w1.wait()
            # this rank's slice of every rank's bucket, summed in fp32, rounded once, into its slot of the send
            # buffer (free again: the all-to-all has consumed it)
            mine = send[self.rank_in_group() * chunk:(self.rank_in_group() + 1) * chunk]
            mine.copy_(recv.view(self.world, chunk).float().sum(0))
            debug.record("dp_all_gather", mine)
            w2 = dist.all_gather_into_tensor(recv, mine, group=self.group, async_op=True)
        self.works.append((w2, t, recv[:n]))

    def wire_bytes_per_step(self) -> int:
        """bytes each rank sends per step for the DP reduction: a ring all-reduce of b payload bytes sends
        2 (w - 1) / w b; the bf16 all-to-all and all-gather send (w - 1) / w of their 2-byte payload each"""
        w = self.world
        if not self.enabled or w <= 1:
            return 0
        tot = 0
        for lo, hi, _ in self.buckets:
            if self.dtype == torch.float32:
                tot += 2 * (w - 1) * (hi - lo) * 4 // w
            else:
                tot += 2 * (w - 1) * self._padded(lo, hi) * 2 // w
        return tot

    def rank_in_group(self) -> int:
        if not hasattr(self, "_rank"):
            self._rank = dist.get_rank(self.group) if self.group is not None else dist.get_rank()
        return self._rank

    def _launch(self, bi: int):
        if self.launched[bi]:
            return
        self.launched[bi] = True
        lo, hi, _ = self.buckets[bi]
        t = self.store.grad[lo:hi]
        if self.dtype != torch.float32:
            self._launch_lowp(bi, t)
        else:
            debug.record("dp_all_reduce", t)
            work = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self.works.append((work, None, None))

    def grad_ready(self, w: torch.Tensor):
        name = getattr(w, "var_name", None)
        if name is None or not self.enabled:
            return
        r = self.remaining.get(name, 0) - 1
        self.remaining[name] = r
        if r == 0:
            bi = self.var_bucket[name]
            self.pending[bi] -= 1
            if self.pending[bi] == 0:
                self._launch(bi)

    def attach(self):
        F.GRAD_HOOK = self.grad_ready if self.enabled else None

    def detach(self):
        F.GRAD_HOOK = None

    def finish(self, average: bool = True):
        """flush every bucket not yet launched, wait for all, scale to the mean over the DP group"""
        if not self.enabled:
            return
        for bi in range(len(self.buckets)):
            self._launch(bi)
        for work, full, low in self.works:
            work.wait()
            if full is not None:
                full.copy_(low)
        if self._side is not None and self.works:
            torch.cuda.current_stream(self._side.device).wait_stream(self._side)   # join the side stream (capture)
        if average:
            self.store.grad.mul_(1.0 / self.world)
        self.reset()


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
