#!/usr/bin/env python3
"""Command line entry (ref main.py:12-30 + src/main.py:36-166).

    python main.py --model configs/gpt_neo_1.3b.json [--run_mode train|sample|query|debug|debug_old|web_api]
                   [--workers N] [--debug_grad 1] [--gpus N] [--synthetic] [--steps K] [--set key=value ...]

``--model`` takes a JSON path or a name under ``configs/`` (the reference's ``session_configs/``). ``--tpu`` is
accepted and ignored. ``--gpus N`` (N > 1) starts ``torch.distributed.run`` with one process per GPU as a CHILD
process before anything touches the GPU, and exits with its status.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

RUN_MODES = ("train", "sample", "query", "debug", "debug_old", "web_api")


def _parse_overrides(items):
    out = {}
    for it in items or []:
        k, _, v = it.partition("=")
        try:
            out[k] = json.loads(v)
        except json.JSONDecodeError:
            out[k] = v
    return out


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tpu", type=str, help="ignored (TPU name in the reference)")
    ap.add_argument("--model", type=str, required=True, help="JSON config path or name under configs/")
    ap.add_argument("--workers", type=int, default=1, help="web_api worker count")
    ap.add_argument("--run_mode", type=str, default="train", help=",".join(RUN_MODES))
    ap.add_argument("--debug_grad", default=None, help="log per-variable gradient norms")
    ap.add_argument("--gpus", type=int, default=0, help="launch N local ranks (one per GPU)")
    ap.add_argument("--synthetic", action="store_true", help="uniform random tokens instead of dataset_configs")
    ap.add_argument("--steps", type=int, default=None, help="stop after this many optimizer steps")
    ap.add_argument("--device", default="auto", choices=("auto", "cuda", "cpu"))
    ap.add_argument("--set", nargs="*", default=[], help="config overrides key=json_value")
    args = ap.parse_args(argv)
    if args.run_mode not in RUN_MODES:
        raise ValueError(f"'{args.run_mode}' is not a supported --run_mode, use one of {','.join(RUN_MODES)}")

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)]
        cmd += [a for a in (argv if argv is not None else sys.argv[1:])]
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        return subprocess.call(cmd, env=env)

    from homebrewnlp_mtf_amd.config import load_config
    model = args.model
    if not model.endswith(".json"):
        model = os.path.join(ROOT, "configs", model + ".json")
    params = load_config(model, _parse_overrides(args.set))
    params.web_workers = args.workers
    params.train = args.run_mode == "train"
    params.debug_sample = args.run_mode == "debug_old"

    if params.train:
        from homebrewnlp_mtf_amd.run.train import train
        out = train(params, debug_grad=args.debug_grad is not None, synthetic=args.synthetic, device=args.device,
                    max_steps=args.steps)
        print(json.dumps({k: v for k, v in out.items() if isinstance(v, (int, float, str))}))
        from homebrewnlp_mtf_amd.parallel import launch
        launch.shutdown()
        return 0
    return _inference(params, args)


def _inference(params, args) -> int:
    import torch
    from homebrewnlp_mtf_amd.config import ModelParameter
    from homebrewnlp_mtf_amd.parallel import launch
    from homebrewnlp_mtf_amd.run import infer
    from homebrewnlp_mtf_amd.run.trainer import Trainer
    from homebrewnlp_mtf_amd.utils import checkpoint as ckpt
    # inference batch: 2 for debug_old, else 1 (ref src/main.py:74-82); the mesh follows the real batch (A17)
    params.train_batch_size = 2 if params.debug_sample else 1
    if params.debug_sample:
        params.use_autoregressive_sampling = True
        params.sampling_temperature = 0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:   # A17: the inference batch is 1-2 sequences, so extra ranks split heads (TP), not the batch
        params.mesh = {"dp": 1, "tp": world}
    params = ModelParameter(params)
    mesh, dev = launch.init(params, args.device)
    tr = Trainer(params, dev, mesh, use_fused=False)
    path = ckpt.latest(params.model_path)
    if path:
        ckpt.restore(tr, path, strict=False)
    else:
        print(f"warning: no checkpoint under {params.model_path}; sampling from random weights", flush=True)
    tok = infer.Tokenizer(params)
    sampler = infer.Sampler(tr.model, params, dev)
    if args.run_mode == "sample" and params.use_video:
        from homebrewnlp_mtf_amd.data import video
        src = video.SyntheticVideo(params, 1, dev) if (args.synthetic or not params.dataset_configs) else \
            video.jannet_input(params, 1, 0, 1, dev)
        vs = infer.VideoSampler(tr.model, params, dev)
        infer.run_video_sample(vs, tok, params, iter(src.next, None),
                               save_prefix=os.path.join(params.model_path, "sample"))
        return 0
    if args.run_mode in ("sample", "debug_old"):
        from homebrewnlp_mtf_amd.data import pipeline as data
        src = data.SyntheticText(params, 1, dev) if (args.synthetic or not params.dataset_configs) else \
            data.text_input(params, 1, 0, 1, dev)
        infer.run_sample(sampler, tok, params, iter(src.next, None))
        return 0
    engine = infer.CompletionEngine(sampler, params, max_batch=int(params.serve_max_batch))
    if args.run_mode == "query":
        infer.run_query(engine, tok, params)
    elif args.run_mode == "debug":
        infer.run_debug(engine, params)
    else:
        from homebrewnlp_mtf_amd.run import serve
        api = serve.RestAPI(engine, tok, params)
        t = serve.serve(api, params.web_host, int(params.web_port), args.workers)
        try:
            t.join()
        except KeyboardInterrupt:
            pass
    engine.close()
    torch.cuda.synchronize() if dev.type == "cuda" else None
    return 0


if __name__ == "__main__":
    sys.exit(main())
