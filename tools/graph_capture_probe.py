"""RCCL collectives inside a captured hipGraph, on a one-rank ``nccl`` group (the 1-GPU box; the 8-GPU bench runs the
same code with ``--hip-graphs-dist 1``):

  1. an async ``all_reduce`` + ``wait`` captured in ``torch.cuda.graph`` and replayed matches the eager result;
  2. the bf16-wire DP reduction (all-to-all, fp32 slice sum on a side stream, all-gather; parallel/grad_sync.py) and
     the whole training step captured by ``Trainer`` (``use_hip_graphs`` + ``hip_graphs_distributed``, GradSync forced
     on at world 1) give the eager Trainer's losses and weights.

  python tools/graph_capture_probe.py [--part P]          (one rank, no launcher: the child's own stderr is kept)
  python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 tools/graph_capture_probe.py [--part P]

Without a launcher the probe sets RANK / WORLD_SIZE / MASTER_* itself, so a crash inside RCCL leaves its own text (not
the elastic agent's ChildFailedError) on stderr; faulthandler prints the Python stack of a SIGSEGV / SIGABRT. Run it
with NCCL_DEBUG=INFO TORCH_SHOW_CPP_STACKTRACES=1 for RCCL's and PyTorch's own account.

--part: all_reduce | all_to_all | all_gather | side_stream | trainer | trainer_fp32 (the fp32 all-reduce wire) | all
(default). Prints one JSON line per part as
it completes (a crash inside a capture still leaves the earlier lines); exit status 1 when one fails.
"""
from __future__ import annotations

import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import faulthandler
    faulthandler.enable(all_threads=True)
    if "WORLD_SIZE" not in os.environ:
        import socket
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from homebrewnlp_mtf_amd.config import ModelParameter
    from homebrewnlp_mtf_amd.parallel import state as pstate
    from homebrewnlp_mtf_amd.run.trainer import Trainer

    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--part", default="all")
    ap.add_argument("--capture-mode", default=os.environ.get("OBST_CAPTURE_MODE", "global"),
                    choices=("global", "thread_local", "relaxed"),
                    help="torch.cuda.graph capture_error_mode (the Trainer reads OBST_CAPTURE_MODE)")
    args = ap.parse_args()
    part = args.part
    global CAPTURE_MODE
    CAPTURE_MODE = args.capture_mode
    os.environ["OBST_CAPTURE_MODE"] = CAPTURE_MODE
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    ok_all = True
    for name, fn in (("all_reduce", _capture_all_reduce), ("all_to_all", _capture_all_to_all),
                     ("all_gather", _capture_all_gather), ("side_stream", _capture_side_stream),
                     ("trainer", lambda d, o: _capture_trainer(d, o, ModelParameter, pstate, Trainer)),
                     ("trainer_fp32", lambda d, o: _capture_trainer(d, o, ModelParameter, pstate, Trainer,
                                                                    "float32"))):
        if part not in ("all", name):
            continue
        out = {"part": name, "capture_mode": CAPTURE_MODE}
        try:
            fn(dev, out)
        except Exception:
            import traceback
            out["error"] = traceback.format_exc()[-2500:]
        if name.startswith("trainer"):
            out["ok"] = bool("error" not in out and out.get("graphs_captured") == 2
                             and out.get("max_loss_diff", 1) < 1e-3 and out.get("max_weight_diff", 1) < 1e-4
                             and ("dp_all_to_all" in out.get("graph_comm", {}) or name == "trainer_fp32"))
        else:
            out["ok"] = bool("error" not in out and out.get("equal"))
        ok_all &= out["ok"]
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok_all else 1)


CAPTURE_MODE = "global"


def _quiesce():
    """let ProcessGroupNCCL's watchdog reap the completed eager collectives before a capture starts: it polls its
    work queue's events from its own thread (~every 100 ms), and a hipEventQuery that lands inside the capture raises
    in WorkNCCL::isCompleted and aborts the process (HIPEvent.h:109 from Watchdog::runLoop, both capture modes on this
    image; profiles/r6_rccl_capture.md)"""
    import time
    torch.cuda.synchronize()
    time.sleep(0.5)


def _capture(dev, fn):
    """warm fn up eagerly on a side stream, capture it, replay once"""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    _quiesce()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
        fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    return g


def _capture_all_to_all(dev, out):
    x = torch.arange(1 << 20, dtype=torch.float32, device=dev).to(torch.bfloat16)
    y = torch.empty_like(x)
    g = _capture(dev, lambda: dist.all_to_all_single(y, x, async_op=True).wait())
    y.zero_()
    g.replay()
    torch.cuda.synchronize()
    out["equal"] = bool(torch.equal(y, x))


def _capture_all_gather(dev, out):
    x = torch.arange(1 << 20, dtype=torch.float32, device=dev).to(torch.bfloat16)
    y = torch.empty_like(x)
    g = _capture(dev, lambda: dist.all_gather_into_tensor(y, x, async_op=True).wait())
    y.zero_()
    g.replay()
    torch.cuda.synchronize()
    out["equal"] = bool(torch.equal(y, x))


def _capture_side_stream(dev, out):
    """the bf16 wire's shape: cast on the capture stream, the collectives + fp32 sum on a side stream, join"""
    x = torch.randn(1 << 20, device=dev)
    send = torch.empty(1 << 20, dtype=torch.bfloat16, device=dev)
    recv = torch.empty_like(send)
    side = torch.cuda.Stream()

    def step():
        send.copy_(x)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            dist.all_to_all_single(recv, send, async_op=True).wait()
            send.copy_(recv.float() * 2)
            w = dist.all_gather_into_tensor(recv, send, async_op=True)
        w.wait()
        torch.cuda.current_stream().wait_stream(side)
    g = _capture(dev, step)
    recv.zero_()
    g.replay()
    torch.cuda.synchronize()
    out["equal"] = bool(torch.equal(recv, (x.to(torch.bfloat16).float() * 2).to(torch.bfloat16)))


def _capture_all_reduce(dev, out):
    # 1. async all_reduce + wait inside a captured graph
    x = torch.arange(1 << 20, dtype=torch.float32, device=dev)
    y = torch.empty_like(x)
    eager = x * 3.0
    dist.all_reduce(eager)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):   # warm-up outside capture (communicator init, RCCL plans)
        y.copy_(x * 3.0)
        dist.all_reduce(y, async_op=True).wait()
    torch.cuda.current_stream().wait_stream(s)
    _quiesce()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
        y.copy_(x * 3.0)
        w = dist.all_reduce(y, async_op=True)
        w.wait()
        z = y + 1.0
    y.zero_()
    g.replay()
    torch.cuda.synchronize()
    out["equal"] = bool(torch.equal(z, eager + 1.0))


def _capture_trainer(dev, out, ModelParameter, pstate, Trainer, wire="bfloat16"):
    # 2. Trainer step captured with the DP collectives inside (world 1, GradSync forced on)
    cfg = dict(model_mode="gpt", use_video=False, use_language=True, heads=4, features_per_head=64, depth=2,
               sequence_length=128, train_batch_size=4, vocab_size=512, intermediate_feed_forward_multiplier=2,
               memory_reduction_strategy="none", calculation_dtype="bfloat16", learning_rate=1e-4,
               optimizer="adaptive_clip:0.003-sm3-momentum:0.9:1:1-learning_rate", grad_bucket_mb=0.25,
               force_grad_sync=True, allreduce_dtype=wire,
               block_config=[{"layer": ["norm-shift-scale", "attention-dot_product-context"], "skip": True},
                             {"layer": ["norm-shift-scale", "feed_forward-in:gelu"], "skip": True}])
    gen = torch.Generator().manual_seed(5)
    batches = []
    for _ in range(6):
        t = torch.randint(0, 512, (4, 129, 1), generator=gen)
        batches.append({"token_x": t[:, :-1].contiguous().to(dev), "token_y": t[:, 1:].contiguous().to(dev)})
    runs = []
    for graphs in (False, True):
        mesh = pstate.Mesh(dp=1, tp=1, rank=0).build_groups()
        torch.manual_seed(0)
        tr = Trainer(ModelParameter(dict(cfg, use_hip_graphs=graphs, hip_graphs_distributed=graphs)), dev, mesh)
        losses = [float(tr.step(b)["loss"]) for b in batches]
        torch.cuda.synchronize()
        runs.append((tr, losses, getattr(tr, "_graph", None)))
    (e, le, _), (c, lc, gstate) = runs
    out["buckets"] = len(c.grad_sync.buckets)
    out["graphs_captured"] = 0 if not gstate else len(gstate["graphs"])
    out["graph_comm"] = {k: list(v) for k, v in getattr(c, "graph_comm", {}).items()}
    out["loss_eager"], out["loss_graph"] = le, lc
    out["max_loss_diff"] = max(abs(a - b) for a, b in zip(le, lc))
    out["max_weight_diff"] = float((e.store.master - c.store.master).abs().max())


if __name__ == "__main__":
    main()
