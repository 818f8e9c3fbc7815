"""scheduler_perf-style workload matrix (tools/sched_perf.py) at a tiny size:
every workload binds all of its measured pods (PreemptionBasic through
preemption), so the matrix measured on the box is a valid run."""
import pytest

from flex_gpu_scheduler_amd.tools import sched_perf


@pytest.mark.parametrize("name", list(sched_perf.WORKLOADS))
def test_workload_binds_everything(name):
    r = sched_perf.run_spec(sched_perf.WORKLOADS[name](24, 48))
    assert "error" not in r, r
    assert r["bound"] == r["pods"] or (name in ("SchedulingPodAntiAffinity", "PreemptionBasic") and r["bound"] == 24), r
    assert r["pods_per_s"] > 0
