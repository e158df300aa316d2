"""The perf gate inside ``pytest -m gpu`` (SURVEY §4 perf baselines): one row per hot-kernel family -- the 1.3B step's
forward GEMM and its worst product (the logits weight gradient), the token mixer's triangular forward, flash
attention forward + backward, the norm backward and the gelu backward -- timed by ``tools/kbench.py gate`` (median
of individually timed calls, each row between its own two same-process calibrations) and checked against the
calibration-ratio floors of ``profiles/kbench_gate_floor.json`` (the gate's own runs: a row timed alone reads
slower than inside its full kbench section, e.g. norm_bwd 370-378 vs 343 us). A kernel that gets slower than its
floor by more than TOL fails the GPU suite; ``OBST_EW_CAP=2048`` (the round-1 grid-stride elementwise launch, ~20 %
slower gelu backward) is the deliberately slowed build the gate was checked against (profiles/r6_perf_gate.md)."""
import json
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import kbench  # noqa: E402

TOL = 0.08   # a healthy box read gelu_bwd 5.8 % under its absolute floor and 3.6 % under its ratio floor (round-6
# final kbench, profiles/r6/kbench_final_check.log); the deliberately slowed launch is ~20 % slower


def test_hot_kernels_meet_their_floors(cuda):
    kbench.EMITTED.clear()
    kbench.PENDING.clear()
    kbench.bench_gate(131072, 64, reps=9)
    with open(os.path.join(ROOT, "profiles", "kbench_gate_floor.json")) as f:
        spec = json.load(f)
    rows = list(kbench.EMITTED)
    seen = {kbench.line_key(r) for r in rows}
    assert kbench.gate_keys() <= seen, f"gate rows not emitted: {sorted(kbench.gate_keys() - seen)}"
    assert all(k in spec["floors"] for k in kbench.gate_keys()), "a gate row has no floor"
    for r in rows:
        print(json.dumps(r))
    # a row fails only when it misses both its calibration ratio and its absolute floor: the same-process
    # calibrations move between boxes (MFMA loop 1904-2091 TF/s, copy 4.6-5.3 TB/s) at equal kernel numbers
    bad = kbench.check_either(rows, spec["floors"], TOL, spec.get("ratios", {}))
    assert not bad, "perf regression: " + "; ".join(f"{k} {m} {v} < floor {fl} - {TOL:.0%}" for k, m, v, fl in bad)
