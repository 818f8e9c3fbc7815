"""The reference's Trimaran unit-test tables, case for case, against the
native plugins through Scheduler.plugin_call:

* LVRB computeScore        pkg/trimaran/loadvariationriskbalancing/analysis_test.go:74   TestComputeScore
* LVRB createResourceStats pkg/trimaran/loadvariationriskbalancing/analysis_test.go:212  Test_createResourceStats
* LVRB getResourceRequested pkg/trimaran/loadvariationriskbalancing/analysis_test.go:297 TestGetResourceRequested
* pod-assign cache cleanup pkg/trimaran/handler_test.go:12                               TestHandlerCacheCleanup
"""
import pytest

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_node, make_pod
from flex_gpu_scheduler_amd.models.objects import make_container


def harness(store, plugin="LoadVariationRiskBalancing"):
    cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": "default-scheduler", "plugins": {
               "score": {"enabled": [{"name": plugin}], "disabled": [{"name": "*"}]}}}]}
    store.create("nodes", make_node("node0", {"cpu": "1000m", "memory": "1Gi", "pods": "110"}))
    s = new_scheduler(store, load_config(cfg))
    s.sync_informers(50)
    return s


# name, margin, sensitivity, (capacity, req, usedAvg, usedStdev), expected
COMPUTE_SCORE = [
    ("valid data", 1, 1, (100, 10, 40, 36), 57),
    ("zero capacity", 1, 2, (0, 10, 40, 36), 0),
    ("negative usedAvg", 1, 2, (100, 10, -40, 36), 65),
    ("large usedAvg", 1, 2, (100, 10, 200, 36), 20),
    ("negative usedStdev", 1, 2, (100, 10, 40, -36), 75),
    ("large usedStdev", 1, 2, (100, 10, 40, 120), 25),
    ("large usedAvg (repeated row)", 1, 2, (100, 10, 200, 36), 20),
    ("negative margin", -1, 1, (100, 10, 40, 36), 75),
    ("negative sensitivity", 1, -1, (100, 10, 40, 36), 57),
    ("zero sensitivity", 1, 0, (100, 10, 40, 36), 75),
]


def go_round(x: float) -> int:
    """Go's math.Round: half away from zero."""
    import math

    return int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))


@pytest.mark.parametrize("name,margin,sens,rs,expected", COMPUTE_SCORE, ids=[c[0] for c in COMPUTE_SCORE])
def test_lvrb_compute_score(store, name, margin, sens, rs, expected):
    s = harness(store)
    cap, req, avg, std = rs
    out = s.plugin_call("LoadVariationRiskBalancing", "computeScore",
                        {"pod": make_pod("p"), "margin": margin, "sensitivity": sens, "capacity": cap, "req": req,
                         "usedAvg": avg, "usedStdev": std})
    assert go_round(out["score"]) == expected


METRICS = [
    {"name": "no_name", "type": "CPU", "operator": "", "value": 40},
    {"name": "cpu_running_avg", "type": "CPU", "operator": "AVG", "value": 40},
    {"name": "cpu_running_std", "type": "CPU", "operator": "STD", "value": 36},
    {"name": "mem_running_avg", "type": "Memory", "operator": "AVG", "value": 20},
    {"name": "mem_running_std", "type": "Memory", "operator": "STD", "value": 10},
]
POD_REQUEST = make_pod("pr", containers=[make_container("c", requests={"cpu": "100m", "memory": str(1024 * 1024)})])


@pytest.mark.parametrize("name,metrics,resource,want", [
    ("test-cpu", METRICS, "cpu", {"capacity": 1000, "req": 100, "usedAvg": 400, "usedStdev": 360}),
    ("test-missing", METRICS[3:5], "cpu", None),
    ("test-memory", METRICS, "memory", {"capacity": 1024, "req": 1, "usedAvg": 204.8, "usedStdev": 102.4}),
])
def test_lvrb_create_resource_stats(store, name, metrics, resource, want):
    s = harness(store)
    out = s.plugin_call("LoadVariationRiskBalancing", "createResourceStats",
                        {"pod": POD_REQUEST, "node": "node0", "metrics": metrics, "resource": resource})
    assert out["valid"] is (want is not None)
    if want:
        for k, v in want.items():
            assert out[k] == pytest.approx(v, rel=1e-12), k


def pod_with_overhead(overhead, init_cpu, init_mem, cont_cpu, cont_mem):
    """getPodWithContainersAndOverhead (loadvariationriskbalancing_test.go:398)."""
    conts = [make_container(f"test-container-{i}", requests={"cpu": f"{c}m", "memory": str(m)},
                            limits={"cpu": f"{c}m", "memory": str(m)}) for i, (c, m) in enumerate(zip(cont_cpu, cont_mem))]
    init = [make_container("test-init", requests={"cpu": f"{init_cpu}m", "memory": str(init_mem)})]
    return make_pod("p", containers=conts, init_containers=init, overhead={"cpu": f"{overhead}m"})


@pytest.mark.parametrize("init,want", [((100, 512), (1510, 3072)), ((2000, 4096), (2010, 4096))])
def test_lvrb_get_resource_requested(store, init, want):
    s = harness(store)
    out = s.plugin_call("LoadVariationRiskBalancing", "getResourceRequested",
                        {"pod": pod_with_overhead(10, init[0], init[1], [1000, 500], [2048, 1024])})
    assert (out["milliCPU"], out["memory"]) == want


# name, entries [(pod, age seconds | None = zero time)], pod to update, expected cache
HANDLER_CASES = [
    ("OnUpdate doesn't add unassigned pods", [("Pod-1", None), ("Pod-2", None), ("Pod-3", None)], "Pod-4",
     ["Pod-4"]),
    ("cleanupCache doesn't delete newly added pods", [("Pod-1", None), ("Pod-2", None), ("Pod-3", None),
                                                      ("Pod-4", 0)], "Pod-5", ["Pod-4", "Pod-5"]),
    ("cleanupCache deletes old pods", [("Pod-1", 300), ("Pod-2", 10), ("Pod-3", 5)], None, ["Pod-2", "Pod-3"]),
]


@pytest.mark.parametrize("plugin", ["TargetLoadPacking", "LoadVariationRiskBalancing"])
@pytest.mark.parametrize("name,entries,update,expected", HANDLER_CASES, ids=[c[0] for c in HANDLER_CASES])
def test_handler_cache_cleanup(store, plugin, name, entries, update, expected):
    s = harness(store, plugin)
    out = s.plugin_call(plugin, "podAssignCache", {
        "pod": make_pod("p"), "node": "node-1", "update": update,
        "entries": [{"name": n, "ageSeconds": age} for n, age in entries]})
    assert out["pods"] == expected
