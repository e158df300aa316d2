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
    a = ap.parse_args()
    ov = {"train_batch_size": a.batch, "use_hip_graphs": False}
    if a.depth:
        ov["depth"] = a.depth
    p = load_config(a.config, ov)
    dev = torch.device("cuda", 0)
    tr = Trainer(p, dev)
    S = p.sequence_length
    toks = torch.randint(0, p.vocab_size, (a.batch, S + 1, 1), device=dev)
    batch = {"token_x": toks[:, :-1].contiguous(), "token_y": toks[:, 1:].contiguous()}
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        tr.step(batch)
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
