"""The perf-regression gate of tools/kbench.py (--check profiles/kbench_floor.json): CPU-side logic only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import kbench  # noqa: E402


def test_floor_file_covers_the_hot_kernels():
    with open(os.path.join(ROOT, "profiles", "kbench_floor.json")) as f:
        floors = json.load(f)["floors"]
    assert any(k.startswith("gemm ") for k in floors) and "attention" in floors and "norm_bwd" in floors


def test_round3_norm_bwd_regression_fails_the_gate():
    with open(os.path.join(ROOT, "profiles", "kbench_floor.json")) as f:
        floors = json.load(f)["floors"]
    ok = {"kernel": "norm_bwd", "rows": 131072, "F": 2048, "us": 349.2, "gbps": 4612.5}
    # round 3's spill regression: 431 -> 833 us per call
    regressed = dict(ok, us=833.0, gbps=round(3 * 131072 * 2048 * 2 / 833.0 / 1e3, 1))
    assert kbench.check([ok], floors) == []
    bad = kbench.check([regressed], floors)
    assert bad and bad[0][0] == "norm_bwd" and bad[0][1] == "gbps"
    # within tolerance passes; an unfloored line is ignored
    assert kbench.check([dict(ok, gbps=ok["gbps"] * 0.96)], floors) == []
    assert kbench.check([{"kernel": "new_kernel", "gbps": 1.0}], floors) == []
