#!/usr/bin/env python3
"""Diagnose graph-vs-eager divergence of the whole-step hipGraph.

Builds three trainers from one seed (eager, eager, graph) exactly like
tests/test_gpu_runtime.py::test_hip_graph_step_matches_eager and, after EVERY step, prints
  * max |master_a - master_b| (eager noise floor) and max |master_a - master_g|,
  * the variables where a and g differ most, and the same for the optimizer slots.
Set OBST_CHOLQR_INIT=1 in the environment to reproduce the round-1 failure mode.

    python tools/diag_graph.py [--strategy none] [--steps 7]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from homebrewnlp_mtf_amd.config import ModelParameter  # noqa: E402
from homebrewnlp_mtf_amd.parallel import state as pstate  # noqa: E402
from homebrewnlp_mtf_amd.run.trainer import Trainer  # noqa: E402

CFG = dict(model_mode="gpt", use_video=False, use_language=True, heads=4, features_per_head=64, depth=2,
           sequence_length=128, train_batch_size=2, vocab_size=500, intermediate_feed_forward_multiplier=2,
           memory_reduction_strategy="revnet", learning_rate=1e-3, calculation_dtype="bfloat16",
           optimizer="adaptive_clip:0.003-sm3-momentum:0.9:1:1-learning_rate",
           learning_rate_config={"linear_warmup": {"final_step": 10}},
           block_config=[{"layer": ["norm-shift-scale", "attention-dot_product-context"]},
                         {"layer": ["norm-shift-scale", "feed_forward-in:gelu"]}])


def batch(seed, device):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(0, 500, (2, 129, 1), generator=g)
    return {"token_x": t[:, :-1].contiguous().to(device), "token_y": t[:, 1:].contiguous().to(device)}


def per_var(store_a, store_b, flat_a, flat_b, top=4):
    out = []
    for n in store_a.order:
        d = (store_a.grad_view_of(flat_a, n) - store_b.grad_view_of(flat_b, n)).abs().max().item()
        out.append((d, n))
    out.sort(reverse=True)
    return out[:top]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--strategy", default="none")
    ap.add_argument("--steps", type=int, default=7)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    pstate.set_mesh(pstate.Mesh())
    cfg = dict(CFG, memory_reduction_strategy=args.strategy)
    runs = []
    for graphs in (False, False, True):
        torch.manual_seed(0)
        runs.append(Trainer(ModelParameter(dict(cfg, use_hip_graphs=graphs)), dev))
    a, b, g = runs
    print("init: |a-b| %.3g |a-g| %.3g" % ((a.store.master - b.store.master).abs().max().item(),
                                            (a.store.master - g.store.master).abs().max().item()), flush=True)
    print("init compute: |a-g| %.3g" % (a.store.compute.float() - g.store.compute.float()).abs().max().item())
    for i in range(args.steps):
        bt = batch(i, dev)
        la = float(a.step(bt)["loss"])
        lb = float(b.step(bt)["loss"])
        lg = float(g.step(bt)["loss"])
        torch.cuda.synchronize()
        ab = (a.store.master - b.store.master).abs().max().item()
        ag = (a.store.master - g.store.master).abs().max().item()
        mode = "graph" if getattr(g, "_graph", None) and g._graph["graphs"] else "eager-warm"
        print(f"step {i} ({mode}): loss a {la:.6f} b {lb:.6f} g {lg:.6f} | master |a-b| {ab:.3g} |a-g| {ag:.3g}",
              flush=True)
        print("   compute |a-g| %.3g, grad |a-g| %.3g" % (
            (a.store.compute.float() - g.store.compute.float()).abs().max().item(),
            (a.store.grad - g.store.grad).abs().max().item()))
        for d, n in per_var(a.store, g.store, a.store.master, g.store.master):
            print(f"   master {d:.3g} {n}")
        for d, n in per_var(a.store, g.store, a.store.grad, g.store.grad, top=3):
            print(f"   grad   {d:.3g} {n}")
        sa, sg = a.opt.named_slots(), g.opt.named_slots()
        worst = sorted(((sa[k].float() - sg[k].float()).abs().max().item(), k) for k in sa)[-3:]
        for d, k in reversed(worst):
            print(f"   slot   {d:.3g} {k}")


if __name__ == "__main__":
    main()
