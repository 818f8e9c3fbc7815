"""Score micro-benchmark harness (targetloadpacking_test.go:267-360 analogue):
the pass runs, scores every node, and TLP with a fresh per-cycle metrics view
still yields the reference's scores."""
from flex_gpu_scheduler_amd.tools import score_bench


def test_tlp_score_pass_runs():
    r = score_bench.run(100, 3)
    assert r["nodes"] == 100 and r["us_per_pass"] > 0


def test_mi355x_score_pass_runs():
    r = score_bench.run(16, 3, mi355x=True)
    assert r["nodes"] == 16 and r["scorers"].startswith("FlexGPU")


def test_timeline_reports_scheduling_thread_busy_span():
    from flex_gpu_scheduler_amd.tools.timeline import timeline

    t = timeline(nodes=8, warmup=1)
    assert t["pods"] > 0
    assert 0 < t["busy_fraction"] <= 1.0
    assert t["sched_thread_busy_ms"] <= t["sched_thread_span_ms"] + 1e-6
    assert t["first_cycle_ms"] <= t["last_cycle_end_ms"]


def test_parallel_filter_and_score_above_inline_threshold():
    """>= 128 nodes runs Filter/Score on the parallelizer's workers
    (parallelInlineBelow); a wave must bind completely there too."""
    from flex_gpu_scheduler_amd.utils.benchrun import Shard
    from flex_gpu_scheduler_amd.utils.workload import ClusterSpec

    sh = Shard(ClusterSpec(nodes=160), seed=1)
    try:
        r = sh.run(sh.wave(0), timeout_s=60)
        assert r.pods > 1500
        assert sh.sched.stats()["bound"] == r.pods
    finally:
        sh.close()
