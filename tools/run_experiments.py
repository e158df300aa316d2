#!/usr/bin/env python3
"""Hyper-parameter sweep launcher (ref scripts/run_experiments.py:64-125).

``--run-config`` is a JSON dict whose values are lists; every combination (grid) × ``--repetitions`` becomes one run
with its own config file under ``--config-dir`` and ``model_path = <prefix><run name>``. Runs are started one after
another (``--parallel 1``) or as up to ``--parallel`` concurrent jobs, each optionally under tools/run_manager.py.
Instead of creating TPUs, each job gets ``--gpus-per-run`` GPUs through ``HIP_VISIBLE_DEVICES``.

    python tools/run_experiments.py --base-config configs/gpt_neo_125m_cpu.json \
        --run-config sweep.json --prefix runs/sweep/ --gpus-per-run 1 --parallel 8
"""
from __future__ import annotations

import argparse
import hashlib
import itertools
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_name(cfg: dict, keys, rep: int) -> str:
    name = "-".join(f"{k}={cfg[k]}" for k in keys) + f"-run={rep}"
    for a, b in ((" ", "_"), ("'", ""), (":", "="), (",", "-"), ("[", "|"), ("]", "|"), ("/", "_")):
        name = name.replace(a, b)
    return name if len(name) <= 120 else hashlib.sha256(name.encode()).hexdigest()


def expand(base: dict, grid: dict, repetitions: int, start: int = 0):
    keys = list(grid)
    for combo in itertools.product(*[grid[k] for k in keys]):
        cfg = dict(base)
        cfg.update(zip(keys, combo))
        for rep in range(start, repetitions):
            yield run_name(cfg, keys, rep), dict(cfg)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--base-config", required=True)
    ap.add_argument("--run-config", default="", help="JSON dict of lists")
    ap.add_argument("--prefix", default="runs/sweep/")
    ap.add_argument("--config-dir", default="runs/sweep_configs/")
    ap.add_argument("--repetitions", type=int, default=1)
    ap.add_argument("--repetition-start", type=int, default=0)
    ap.add_argument("--gpus-per-run", type=int, default=1)
    ap.add_argument("--total-gpus", type=int, default=8)
    ap.add_argument("--parallel", type=int, default=1)
    ap.add_argument("--use-manager", action="store_true")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--extra", nargs="*", default=[], help="extra main.py arguments")
    a = ap.parse_args(argv)
    base = json.load(open(a.base_config))
    grid = json.load(open(a.run_config)) if a.run_config else {}
    os.makedirs(a.config_dir, exist_ok=True)
    jobs = []
    for name, cfg in expand(base, grid, a.repetitions, a.repetition_start):
        cfg["model_path"] = a.prefix + name
        path = os.path.join(a.config_dir, name + ".json")
        with open(path, "w") as f:
            json.dump(cfg, f, indent=1)
        cmd = [sys.executable, os.path.join(ROOT, "main.py"), "--model", path, *a.extra]
        if a.gpus_per_run > 1:
            cmd += ["--gpus", str(a.gpus_per_run)]
        if a.use_manager:
            cmd = [sys.executable, os.path.join(ROOT, "tools", "run_manager.py"), "--log",
                   os.path.join(cfg["model_path"], "run.log"), "--heartbeat-glob",
                   os.path.join(cfg["model_path"], "heartbeat-*"), "--", *cmd]
        jobs.append((name, cmd))
    if a.dry_run:
        for name, cmd in jobs:
            print(name, " ".join(cmd))
        return 0
    slots = list(range(0, a.total_gpus, a.gpus_per_run))[:max(1, a.parallel)]
    running = {}
    pending = list(jobs)
    failures = 0
    while pending or running:
        for slot in slots:
            if slot not in running and pending:
                name, cmd = pending.pop(0)
                env = dict(os.environ, HIP_VISIBLE_DEVICES=",".join(str(slot + i) for i in range(a.gpus_per_run)))
                os.makedirs(a.prefix, exist_ok=True)
                running[slot] = (name, subprocess.Popen(cmd, env=env))
                print(f"started {name} on GPUs {env['HIP_VISIBLE_DEVICES']}", flush=True)
        for slot, (name, proc) in list(running.items()):
            rc = proc.poll()
            if rc is not None:
                print(f"finished {name}: status {rc}", flush=True)
                failures += rc != 0
                del running[slot]
        time.sleep(1)
    return 1 if failures else 0


if __name__ == "__main__":
    sys.exit(main())
