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
