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
    gb = floors["norm_bwd"]["gbps"]   # a run at the floor itself
    ok = {"kernel": "norm_bwd", "rows": 131072, "F": 2048, "us": round(3 * 131072 * 2048 * 2 / gb / 1e3, 1), "gbps": gb}
    # round 3's spill regression: 431 -> 833 us per call
    regressed = dict(ok, us=833.0, gbps=round(3 * 131072 * 2048 * 2 / 833.0 / 1e3, 1))
    assert kbench.check([ok], floors) == []
    bad = kbench.check([regressed], floors)
    assert bad and bad[0][0] == "norm_bwd" and bad[0][1] == "gbps"
    # within tolerance passes; an unfloored line is ignored
    assert kbench.check([dict(ok, gbps=ok["gbps"] * 0.98)], floors) == []
    assert kbench.check([{"kernel": "new_kernel", "gbps": 1.0}], floors) == []


def test_ratio_floors_are_box_independent():
    """a key with ratio floors is judged on metric / same-process calibration: the same kernel on a slower box (lower
    absolute number, proportionally lower calibration) passes; a real regression at the same calibration fails"""
    floors = {"gemm fwd": {"tflops_gemm4w": 1400.0}}
    ratios = {"gemm fwd": {"tflops_gemm4w": 0.70}}
    row = {"kernel": "gemm", "shape": "fwd", "tflops_gemm4w": 1400.0, "ratio_tflops_gemm4w": 0.70}
    slow_box = dict(row, tflops_gemm4w=1260.0, ratio_tflops_gemm4w=0.70)      # 10 % lower clock, same code
    regressed = dict(row, tflops_gemm4w=1330.0, ratio_tflops_gemm4w=0.665)    # 5 % slower at the same clock
    assert kbench.check([slow_box], floors, 0.03, ratios) == []
    assert kbench.check([slow_box], floors, 0.03) != []                      # absolute floors would flag the box
    assert kbench.check([regressed], floors, 0.03, ratios)


def test_missing_floored_key_is_reported():
    floors = {"gemm fwd": {"tflops_gemm4w": 1.0}, "attention": {"pflops_fwd": 1.0}, "norm_fwd": {"gbps": 1.0}}
    assert kbench.missing(floors, {"attention"}, ["gemm", "attn"]) == ["gemm fwd"]
    assert kbench.missing(floors, {"attention", "gemm fwd"}, ["gemm", "attn"]) == []


def test_rows_get_calibration_ratios():
    kbench.PENDING.clear()
    kbench.EMITTED.clear()
    kbench.emit(kernel="attention", pflops_fwd=0.8, gbps=3000.0)
    kbench.flush_rows({"mfma_tflops": 2000.0, "copy_gbps": 5000.0})
    r = kbench.EMITTED[-1]
    assert r["ratio_pflops_fwd"] == 0.4 and r["ratio_gbps"] == 0.6
    kbench.EMITTED.clear()


def test_check_either_needs_both_floors_missed():
    """a row regresses only when it misses its ratio floor AND its absolute floor (box calibration drift alone does
    not fail it; a slower kernel fails both)"""
    floors = {"k": {"gbps": 100.0}}
    ratios = {"k": {"gbps": 1.0}}
    fast_calib = {"kernel": "k", "gbps": 101.0, "ratio_gbps": 0.9}    # calibration read high: ratio misses only
    assert kbench.check_either([fast_calib], floors, 0.03, ratios) == []
    slow = {"kernel": "k", "gbps": 90.0, "ratio_gbps": 0.9}
    assert kbench.check_either([slow], floors, 0.03, ratios) != []
