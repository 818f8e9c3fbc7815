"""scheduler_perf-style workload matrix (tools/sched_perf.py) at a tiny size:
every workload binds all of its measured pods (PreemptionBasic through
preemption), so the matrix measured on the box is a valid run."""
import pytest

from flex_gpu_scheduler_amd.tools import sched_perf


@pytest.mark.parametrize("name", list(sched_perf.WORKLOADS))
def test_workload_binds_everything(name):
    w = sched_perf.WORKLOADS[name](24, 48)
    r = sched_perf.run_spec(w)
    assert "error" not in r, r
    want = w["expect_bound"] if w["expect_bound"] is not None else len(w["pods"])
    assert r["bound"] == want, r
    assert r["pods_per_s"] > 0
