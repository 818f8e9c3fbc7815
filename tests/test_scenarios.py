"""The five BASELINE.json configurations (utils/scenarios.py) run and their
placement properties hold."""
from flex_gpu_scheduler_amd.utils import scenarios as sc


def test_coscheduling_cpu():
    r = sc.coscheduling_cpu(waves=1, groups=20, nodes=4)
    assert r["pods"] == 40 and r["pods_per_s"] > 0


def test_flexgpu_cpx_quarter_shares_one_gpu():
    r = sc.flexgpu_cpx_quarter(iterations=3)
    assert r["four_pods_share_one_gpu"] == "5/5"


def test_gang8_lands_on_one_xgmi_node():
    r = sc.gang8_xgmi(iterations=3)
    assert r["gangs_on_one_xgmi_node"] == "5/5"


def test_capacity_reclaims_exactly_borrowed_within_one_backoff():
    r = sc.capacity_preemption(iterations=1)
    assert r["exactly_borrowed_preempted"] == "1/1"
    assert r["reclaim_ms"][0] < 1900  # one 1 s backoff, not a cascade of rounds


def test_trimaran_tlp_prefers_target_utilisation():
    r = sc.trimaran_tlp(pods=16, sampler=type("S", (), {"gpu_samples": lambda self: []})())
    assert r["metrics_source"] == "synthetic"
    scores = r["tlp_scores"]
    # 26% busy + 1/8 GPU = 38.5% is closest below the 40% target.
    assert max(scores, key=scores.get) == r["first_gpu_pod_node"] == "mi355x-2"
