"""Trimaran load-aware scoring fed by load-watcher WatcherMetrics objects
(pkg/trimaran; golden values from targetloadpacking_test.go:137-190 and the
LVRB computeScore table in analysis_test.go)."""
import pytest

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.models import GPU, make_node, make_pod


def only_score(plugin, args=None):
    return {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
            "profiles": [{"schedulerName": "default-scheduler", "plugins": {
                "score": {"enabled": [{"name": plugin}], "disabled": [{"name": "*"}]}},
                "pluginConfig": [{"name": plugin, "args": args or {}}]}]}


def metrics(nodes: dict, end=0):
    return {"metadata": {"name": "cluster"}, "timestamp": end, "window": {"duration": "15m", "start": end - 900,
                                                                        "end": end},
            "source": "test", "data": {"NodeMetricsMap": {n: {"metrics": m} for n, m in nodes.items()}}}


def cpu(v, op="AVG"):
    return {"name": "cpu", "type": "CPU", "operator": op, "value": v}


def mem(v, op="AVG"):
    return {"name": "mem", "type": "Memory", "operator": op, "value": v}


def explain_scores(store, sched, pod):
    sched.sync_informers(20)
    return sched.explain(pod)["scores"]


def test_tlp_golden_values(store):
    for n in ("a", "b"):
        store.create("nodes", make_node(n, {"cpu": "64", "memory": "256Gi", "pods": "110"}))
    s = new_scheduler(store, load_config(only_score("TargetLoadPacking", {"defaultRequests": {"cpu": "0"}})))
    store.create("loadwatchermetrics", metrics({"a": [cpu(0)], "b": [cpu(50)]}))
    sc = explain_scores(store, s, make_pod("p"))
    assert sc["a"]["TargetLoadPacking*1"] == 40   # util 0, zero request
    assert sc["b"]["TargetLoadPacking*1"] == 33   # util = target + 10
    s.stop()


def test_tlp_missing_metrics_scores_min(store):
    store.create("nodes", make_node("a", {"cpu": "64", "memory": "256Gi", "pods": "110"}))
    store.create("nodes", make_node("b", {"cpu": "64", "memory": "256Gi", "pods": "110"}))
    s = new_scheduler(store, load_config(only_score("TargetLoadPacking")))
    store.create("loadwatchermetrics", metrics({"a": [cpu(10)]}))
    sc = explain_scores(store, s, make_pod("p", requests={"cpu": "1"}))
    assert sc["b"]["TargetLoadPacking*1"] == 0
    # 10% of 64 cores + 1.5 cores predicted (request x 1.5) -> 12.34% -> packs toward 40%
    assert sc["a"]["TargetLoadPacking*1"] == round((100 - 40) * (100 * (6400 + 1500) / 64000) / 40 + 40)
    s.stop()


def test_tlp_gpu_mode_packs_on_mi355x_busy(store):
    for n in ("a", "b"):
        store.create("nodes", make_node(n, {"cpu": "64", "memory": "256Gi", "pods": "110", GPU: "8"}))
    s = new_scheduler(store, load_config(only_score("TargetLoadPacking", {"resourceType": "GPU"})))
    store.create("loadwatchermetrics", metrics({"a": [{"type": "GPU", "operator": "AVG", "value": 25}],
                                                "b": [{"type": "GPU", "operator": "AVG", "value": 90}]}))
    sc = explain_scores(store, s, make_pod("p", limits={GPU: "1"}))
    # a: 25% + 1/8 GPU = 37.5% -> round(60*37.5/40+40) = 96; b: 102.5% -> 0
    assert sc["a"]["TargetLoadPacking*1"] == 96 and sc["b"]["TargetLoadPacking*1"] == 0
    s.stop()


@pytest.mark.parametrize("avg,std,margin,sens,expected", [
    (0, 0, 1, 1, 100), (50, 0, 1, 1, 75), (50, 10, 1, 1, 70), (50, 10, 2, 1, 65), (100, 0, 1, 1, 50),
])
def test_lvrb_compute_score(store, avg, std, margin, sens, expected):
    for n in ("a", "b"):
        store.create("nodes", make_node(n, {"cpu": "100", "memory": "100Gi", "pods": "110"}))
    s = new_scheduler(store, load_config(only_score("LoadVariationRiskBalancing",
                                                    {"safeVarianceMargin": margin, "safeVarianceSensitivity": sens})))
    store.create("loadwatchermetrics", metrics({"a": [cpu(avg), cpu(std, "STD")], "b": [cpu(0)]}))
    sc = explain_scores(store, s, make_pod("p"))
    assert sc["a"]["LoadVariationRiskBalancing*1"] == expected
    s.stop()


def test_lvrb_min_of_cpu_and_memory(store):
    for n in ("a", "b"):
        store.create("nodes", make_node(n, {"cpu": "100", "memory": "100Gi", "pods": "110"}))
    s = new_scheduler(store, load_config(only_score("LoadVariationRiskBalancing")))
    store.create("loadwatchermetrics", metrics({"a": [cpu(20), mem(60)], "b": [cpu(0), mem(0)]}))
    sc = explain_scores(store, s, make_pod("p"))
    assert sc["a"]["LoadVariationRiskBalancing*1"] == 70  # min(90, 70)
    s.stop()


def test_tlp_live_tool_logic_with_injected_load():
    """tools/tlp_live.py end to end with a stand-in sampler (the GPU tier
    runs it on the real MI355X through amd-smi)."""
    import time as _t

    from flex_gpu_scheduler_amd.gpu.telemetry import Sample
    from flex_gpu_scheduler_amd.tools import tlp_live

    state = {"busy": False}

    class FakeSampler:
        def sample(self):
            return Sample(_t.time(), 10.0, 20.0, 92.0 if state["busy"] else 3.0, 5.0)

    def start_load():
        state["busy"] = True
        return lambda: state.update(busy=False)

    r = tlp_live.run(0.2, 0.01, sampler=FakeSampler(), start_load=start_load)
    assert r["gpu_busy_avg"][tlp_live.BUSY] == 92.0 and r["gpu_busy_avg"][tlp_live.IDLE] == 3.0
    sc = r["tlp_scores"]
    # idle: 3% + 1/8 GPU = 15.5% -> round(60*15.5/40+40) = 63; busy: 104.5% -> 0
    assert sc[tlp_live.IDLE] == 63 and sc[tlp_live.BUSY] == 0
    assert r["predicted"] == r["landed"] == tlp_live.IDLE
