"""bench.py's predicted-scaling model (C3/C5 --phases) on hand-made task records: the LPT
makespan per level, the concurrency factor, and the driver's deferred-leaf batch as one more
level whose LPT runs over every leaf of the job (driver.py defer_leaves)."""
import importlib
import types

import pytest

import bench


@pytest.fixture(scope="module")
def par():
    return importlib.import_module(bench.PKG + ".parallel")


def _drv(levels, fixed=0.0):
    return types.SimpleNamespace(level_tasks=levels, timings={"bookkeeping": fixed})


def test_n1_is_the_measured_wall(par):
    lv = [{"phase_s": {"local_models": 2.0, "nearest_sample": 1.0, "bubbles": 0.5},
           "local_models": [(4.0, 1.0), (1.0, 1.0)]},
          {"phase_s": {"leaves": 3.0}, "deferred_leaves": True, "leaves": [(9.0, 2.0), (1.0, 1.0)]}]
    out = bench.predicted_scaling(_drv(lv, fixed=0.25), par, ns=(1,))
    assert out["seconds"]["1"] == pytest.approx(2.0 + 1.0 + 0.5 + 3.0 + 0.25)


def test_deferred_leaves_balance_over_the_whole_job(par):
    # four equal leaves of four different levels: per level each is alone (no speedup), but as
    # one deferred batch they spread over the ranks
    per_level = [{"phase_s": {"leaves": 1.0}, "leaves": [(1.0, 1.0)]} for _ in range(4)]
    deferred = [{"phase_s": {"leaves": 4.0}, "deferred_leaves": True, "leaves": [(1.0, 1.0)] * 4}]
    a = bench.predicted_scaling(_drv(per_level), par, ns=(1, 4))
    b = bench.predicted_scaling(_drv(deferred), par, ns=(1, 4))
    assert a["seconds"]["4"] == pytest.approx(4.0)
    assert b["seconds"]["4"] == pytest.approx(1.0)
    assert b["speedup"]["4"] == pytest.approx(4.0)


def test_concurrency_factor_scales_task_sums(par):
    # two tasks of 1 s each measured while overlapping (wall 1 s): at N = 2 each rank runs one
    lv = [{"phase_s": {"local_models": 1.0}, "local_models": [(1.0, 1.0), (1.0, 1.0)]}]
    out = bench.predicted_scaling(_drv(lv), par, ns=(1, 2))
    assert out["seconds"]["1"] == pytest.approx(1.0)
    assert out["seconds"]["2"] == pytest.approx(0.5)
