#!/usr/bin/env python3
"""Watchdog / auto-restart for a training job (ref scripts/run_manager.py:89-158).

The reference recreates a TPU and relaunches when the TPU health check fails. Here the job is a local process
group (``main.py --gpus N`` or ``torch.distributed.run``); it is declared unhealthy when

* it exits with a non-zero status (crash, fault injection, RCCL timeout), or
* no heartbeat file under ``--heartbeat-glob`` was touched for ``--stall-seconds`` (hung collective / GPU), or
* ``--gpu-check`` is given and ``rocm-smi`` stops answering.

The whole process group is then killed (SIGTERM, then SIGKILL) and the command relaunched; the trainer resumes
from its newest complete checkpoint on its own. Output is tee'd to ``--log``.

    python tools/run_manager.py --log runs/x/run.log --heartbeat-glob 'runs/x/heartbeat-*' \
        -- python main.py --model configs/gpt_neo_1.3b.json --gpus 8
"""
from __future__ import annotations

import argparse
import glob
import os
import signal
import subprocess
import sys
import threading
import time


def _tee(proc: subprocess.Popen, log):
    for line in iter(proc.stdout.readline, b""):
        sys.stdout.buffer.write(line)
        sys.stdout.flush()
        if log:
            log.write(line)
            log.flush()


def _newest_heartbeat(pattern: str) -> float:
    files = glob.glob(pattern)
    return max((os.path.getmtime(f) for f in files), default=0.0)


def _gpu_ok(timeout: float = 60.0) -> bool:
    try:
        r = subprocess.run(["rocm-smi", "--showuse"], capture_output=True, timeout=timeout)
        return r.returncode == 0
    except (OSError, subprocess.TimeoutExpired):
        return False


def _kill_group(proc: subprocess.Popen, grace: float):
    try:
        pgid = os.getpgid(proc.pid)
    except ProcessLookupError:
        return
    for sig, wait in ((signal.SIGTERM, grace), (signal.SIGKILL, 10.0)):
        try:
            os.killpg(pgid, sig)
        except ProcessLookupError:
            return
        try:
            proc.wait(timeout=wait)
            return
        except subprocess.TimeoutExpired:
            continue


def run(cmd, log_path=None, heartbeat_glob=None, stall_seconds=900.0, poll=10.0, max_restarts=100,
        gpu_check=False, grace=30.0, startup_grace=600.0) -> int:
    log = open(log_path, "ab") if log_path else None
    restarts = 0
    while True:
        start = time.time()
        proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True)
        t = threading.Thread(target=_tee, args=(proc, log), daemon=True)
        t.start()
        reason = None
        while True:
            rc = proc.poll()
            if rc is not None:
                if rc == 0:
                    t.join(timeout=5)
                    return 0
                reason = f"exit status {rc}"
                break
            now = time.time()
            if heartbeat_glob and now - start > startup_grace:
                hb = _newest_heartbeat(heartbeat_glob)
                if now - max(hb, start) > stall_seconds:
                    reason = f"no heartbeat for {now - max(hb, start):.0f}s"
                    break
            if gpu_check and not _gpu_ok():
                reason = "rocm-smi not responding"
                break
            time.sleep(poll)
        _kill_group(proc, grace)
        t.join(timeout=5)
        restarts += 1
        msg = f"[run_manager] job unhealthy ({reason}); restart {restarts}/{max_restarts}\n"
        sys.stderr.write(msg)
        if log:
            log.write(msg.encode())
            log.flush()
        if restarts > max_restarts:
            return 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--log", default=None)
    ap.add_argument("--heartbeat-glob", default=None)
    ap.add_argument("--stall-seconds", type=float, default=900.0)
    ap.add_argument("--startup-grace", type=float, default=600.0)
    ap.add_argument("--poll", type=float, default=10.0)
    ap.add_argument("--max-restarts", type=int, default=100)
    ap.add_argument("--gpu-check", action="store_true")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("missing command")
    return run(cmd, a.log, a.heartbeat_glob, a.stall_seconds, a.poll, a.max_restarts, a.gpu_check,
               startup_grace=a.startup_grace)


if __name__ == "__main__":
    sys.exit(main())
