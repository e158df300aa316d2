"""Which PyTorch (at::native) kernels does a training step still launch, and from where? One eager step of a config
under torch.profiler with Python stacks; prints the aten ops with device time, grouped by their top frames.

  python tools/lab/aten_census.py --config configs/ctx32_mixer.json --batch 32 [--depth 4]
"""
import argparse
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from homebrewnlp_mtf_amd.config import load_config  # noqa: E402
from homebrewnlp_mtf_amd.run.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="configs/ctx32_mixer.json")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--depth", type=int, default=0)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    ov = {"train_batch_size": a.batch, "use_hip_graphs": False}
    if a.depth:
        ov["depth"] = a.depth
    p = load_config(a.config, ov)
    dev = torch.device(a.device)
    tr = Trainer(p, dev)
    S = p.sequence_length
    toks = torch.randint(0, p.vocab_size, (a.batch, S + 1, 1), device=dev)
    batch = {"token_x": toks[:, :-1].contiguous(), "token_y": toks[:, 1:].contiguous()}
    for _ in range(3):
        tr.step(batch)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    # every aten op of one eager step that launches device work, with the repository frames that issued it
    import collections
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    skip = ("aten::view", "aten::_unsafe_view", "aten::reshape", "aten::permute", "aten::t", "aten::transpose",
            "aten::as_strided", "aten::expand", "aten::detach", "aten::alias", "aten::empty", "aten::empty_like",
            "aten::empty_strided", "aten::slice", "aten::select", "aten::unsqueeze", "aten::squeeze", "aten::split",
            "aten::_local_scalar_dense", "aten::is_nonzero", "aten::new_empty", "aten::new_empty_strided",
            "aten::unbind", "aten::narrow", "aten::lift_fresh", "aten::set_", "aten::result_type")
    seen = collections.Counter()

    class Census(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = "aten::" + func.__name__.split(".")[0]
            if name not in skip:
                fr = [f for f in traceback.extract_stack() if "homebrewnlp_mtf_amd" in f.filename][-3:]
                where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in reversed(fr))
                big = max((a.numel() for a in list(args) + list((kwargs or {}).values())
                           if isinstance(a, torch.Tensor)), default=0)
                seen[(name, where, big)] += 1
            return func(*args, **(kwargs or {}))

    with Census():
        tr.step(batch)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    for (name, where, big), n in sorted(seen.items(), key=lambda kv: -kv[0][2] * kv[1]):
        if big >= 1 << 20:
            print(f"x{n:<4d} {name:28s} numel {big:>12d}  {where}")
    print("---- profiler (device time) ----")
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        tr.step(batch)
        if dev.type == "cuda":
            torch.cuda.synchronize()
    ev = prof.key_averages(group_by_stack_n=6)
    rows = [e for e in ev if e.key.startswith("aten::") and getattr(e, "self_device_time_total", 0) > 0]
    rows.sort(key=lambda e: -e.self_device_time_total)
    for e in rows[:40]:
        print(f"{e.self_device_time_total / 1e3:9.3f} ms  x{e.count:<4d} {e.key}")
        for fr in (e.stack or [])[:6]:
            print(f"              {fr}")


if __name__ == "__main__":
    main()
