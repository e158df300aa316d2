"""Rank-aware, timestamped logging (ref ``src/utils_core.py:43-48`` color_print)."""
import datetime
import os
import sys

_COLOR = "\x1b[32;1m"
_RESET = "\x1b[0m"


def _rank() -> int:
    return int(os.environ.get("RANK", "0"))


def log(*args, all_ranks: bool = False, color: bool = False):
    if not all_ranks and _rank() != 0:
        return
    msg = " ".join(str(a) for a in args)
    ts = datetime.datetime.now().strftime("%H:%M:%S")
    prefix = f"[{ts} r{_rank()}] "
    if color and sys.stderr.isatty():
        msg = _COLOR + msg + _RESET
    print(prefix + msg, file=sys.stderr, flush=True)
