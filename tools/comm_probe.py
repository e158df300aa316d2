"""Collective bus-bandwidth probe over the job's process group (RCCL over xGMI on GPUs; gloo on the CPU).

Measures all_reduce / reduce_scatter / all_gather / all_to_all at a sweep of message sizes and reports, per size,
the mean time, the algorithm bandwidth (bytes / time) and the bus bandwidth with the usual ring corrections
(all_reduce 2(n-1)/n, reduce_scatter / all_gather / all_to_all (n-1)/n) -- the per-link figure to hold against
xGMI's ~153 GB/s per link direction when choosing the DP bucket size (grad_bucket_mb) and the TP degree
(SURVEY §2.4, §5.8).

  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/comm_probe.py --sizes-mb 1,16,64,256
  OBST_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/comm_probe.py

Rank 0 prints one JSON line per (collective, size).
"""
from __future__ import annotations

import argparse
import json
import os
import time

import torch
import torch.distributed as dist

FACTORS = {"all_reduce": lambda n: 2.0 * (n - 1) / n, "reduce_scatter": lambda n: (n - 1) / n,
           "all_gather": lambda n: (n - 1) / n, "all_to_all": lambda n: (n - 1) / n}


def _run(op: str, buf: torch.Tensor, out: torch.Tensor, world: int):
    if op == "all_reduce":
        dist.all_reduce(buf)
    elif op == "reduce_scatter":
        dist.reduce_scatter_tensor(out, buf)
    elif op == "all_gather":
        dist.all_gather_into_tensor(buf, out)
    else:
        dist.all_to_all_single(out, buf)


def probe(sizes_mb, ops, iters: int, warmup: int, dtype: torch.dtype, device: torch.device):
    world = dist.get_world_size()
    rows = []
    for op in ops:
        for mb in sizes_mb:
            n = max(int(mb * 2 ** 20) // torch.tensor([], dtype=dtype).element_size() // world * world, world)
            buf = torch.ones(n, dtype=dtype, device=device)
            out = torch.empty(n // world if op in ("reduce_scatter", "all_gather") else n, dtype=dtype,
                              device=device)
            for _ in range(warmup):
                _run(op, buf, out, world)
            if device.type == "cuda":
                torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                _run(op, buf, out, world)
            if device.type == "cuda":
                torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / iters
            t = torch.tensor([dt], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t)
            nbytes = n * buf.element_size()
            algbw = nbytes / dt / 1e9
            rows.append({"op": op, "bytes": nbytes, "world": world, "us": round(dt * 1e6, 1),
                         "algbw_GBps": round(algbw, 2), "busbw_GBps": round(algbw * FACTORS[op](world), 2),
                         "dtype": str(dtype).replace("torch.", ""), "backend": dist.get_backend()})
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,16,64,256")
    ap.add_argument("--ops", default="all_reduce,reduce_scatter,all_gather,all_to_all")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", default="bfloat16")
    args = ap.parse_args(argv)
    backend = os.environ.get("OBST_DIST_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", 0))
    if backend == "nccl":
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        dist.init_process_group("nccl", device_id=device)
    else:
        device = torch.device("cpu")
        dist.init_process_group(backend)
    rows = probe([float(s) for s in args.sizes_mb.split(",")], args.ops.split(","), args.iters, args.warmup,
                 getattr(torch, args.dtype), device)
    if dist.get_rank() == 0:
        for r in rows:
            print(json.dumps(r), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
