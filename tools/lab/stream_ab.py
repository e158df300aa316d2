"""RevNet stream dtype A/B on the reference's ctx32_mixer config: the same init and the same learnable synthetic
batches (per-sequence arithmetic byte sequences with random start / stride, so the loss falls), trained with fp32
streams and with streams in the compute dtype (revnet_stream_dtype "calculation", the reference's numerics); prints
the two loss curves, then times both at the config batch.

  python tools/lab/stream_ab.py [--steps 60] [--batch 32] [--time-batch 256]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from homebrewnlp_mtf_amd.config import load_config  # noqa: E402
from homebrewnlp_mtf_amd.run.trainer import Trainer  # noqa: E402


def batches(n, B, S, dev):
    g = torch.Generator().manual_seed(11)
    out = []
    for _ in range(n):
        start = torch.randint(0, 256, (B, 1), generator=g)
        stride = torch.randint(1, 8, (B, 1), generator=g)
        toks = (start + stride * torch.arange(S + 1)) % 256
        toks = toks.view(B, S + 1, 1).to(dev)
        out.append({"token_x": toks[:, :-1].contiguous(), "token_y": toks[:, 1:].contiguous()})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="configs/ctx32_mixer.json")
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--time-batch", type=int, default=256)
    ap.add_argument("--time-steps", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    curves = {}
    combos = (("float32", "float32"), ("calculation", "float32"), ("float32", "calculation"))
    for stream, gstream in combos:
        p = load_config(a.config, {"train_batch_size": a.batch, "revnet_stream_dtype": stream,
                                   "revnet_grad_stream_dtype": gstream, "use_hip_graphs": True})
        torch.manual_seed(1234)
        tr = Trainer(p, dev)
        data = batches(8, a.batch, p.sequence_length, dev)
        losses = []
        for i in range(a.steps):
            m = tr.step(data[i % len(data)])
            if i % 10 == 9 or i == 0:
                losses.append(round(float(m["loss"]), 4))
        curves[(stream, gstream)] = losses
        print(json.dumps({"stream": stream, "grad_stream": gstream, "batch": a.batch, "loss_every_10": losses}),
              flush=True)
        del tr
        torch.cuda.empty_cache()
    for stream, gstream in combos + combos:
        p = load_config(a.config, {"train_batch_size": a.time_batch, "revnet_stream_dtype": stream,
                                   "revnet_grad_stream_dtype": gstream, "use_hip_graphs": True})
        torch.manual_seed(1234)
        tr = Trainer(p, dev)
        data = batches(2, a.time_batch, p.sequence_length, dev)
        for i in range(3):
            tr.step(data[i % 2])
        tr.prepare_graphs()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.time_steps):
            tr.step(data[i % 2])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.time_steps
        print(json.dumps({"stream": stream, "grad_stream": gstream, "batch": a.time_batch,
                          "ms_per_step": round(dt * 1e3, 1),
                          "tokens_per_s": round(a.time_batch * p.sequence_length / dt, 1)}), flush=True)
        del tr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
