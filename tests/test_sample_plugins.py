"""NodeResourcesAllocatable (pkg/noderesources/allocatable.go:94-129 +
resource_allocation.go), PodState (pkg/podstate/pod_state.go:59-97) and QOSSort
(pkg/qos/queue_sort.go:53-77)."""
from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_node, make_pod

from helpers import placements, wait_bound


def cfg(plugins: dict, args: dict | None = None):
    prof = {"schedulerName": "default-scheduler", "plugins": plugins}
    if args:
        prof["pluginConfig"] = [{"name": k, "args": v} for k, v in args.items()]
    return {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
            "profiles": [prof]}


def score_only(name, args=None):
    return cfg({"score": {"enabled": [{"name": name}], "disabled": [{"name": "*"}]}},
               {name: args} if args is not None else None)


def test_allocatable_least_prefers_smallest_node(store):
    store.create("nodes", make_node("small", {"cpu": "8", "memory": "32Gi", "pods": "110"}))
    store.create("nodes", make_node("mid", {"cpu": "32", "memory": "128Gi", "pods": "110"}))
    store.create("nodes", make_node("big", {"cpu": "256", "memory": "1Ti", "pods": "110"}))
    s = new_scheduler(store, load_config(score_only("NodeResourcesAllocatable", {})))
    s.sync_informers(20)
    out = s.explain(make_pod("p", requests={"cpu": "1"}))
    sc = {n: v["NodeResourcesAllocatable*1"] for n, v in out["scores"].items()}
    assert sc["small"] == 100 and sc["big"] == 0 and 0 < sc["mid"] < 100
    assert out["selected"] == "small"
    s.stop()


def test_allocatable_most_prefers_biggest_node(store):
    store.create("nodes", make_node("small", {"cpu": "8", "memory": "32Gi", "pods": "110"}))
    store.create("nodes", make_node("big", {"cpu": "256", "memory": "1Ti", "pods": "110"}))
    s = new_scheduler(store, load_config(score_only(
        "NodeResourcesAllocatable", {"mode": "Most", "resources": [{"name": "cpu", "weight": 1}]})))
    s.sync_informers(20)
    out = s.explain(make_pod("p"))
    assert out["scores"]["big"]["NodeResourcesAllocatable*1"] == 100
    assert out["scores"]["small"]["NodeResourcesAllocatable*1"] == 0
    s.stop()


def test_allocatable_equal_nodes_score_min(store):
    for n in ("a", "b"):
        store.create("nodes", make_node(n, {"cpu": "8", "memory": "32Gi", "pods": "110"}))
    s = new_scheduler(store, load_config(score_only("NodeResourcesAllocatable", {})))
    s.sync_informers(20)
    out = s.explain(make_pod("p"))
    assert {v["NodeResourcesAllocatable*1"] for v in out["scores"].values()} == {0}
    s.stop()


def test_podstate_prefers_nodes_with_terminating_pods(store):
    for n in ("a", "b", "c"):
        store.create("nodes", make_node(n, {"cpu": "64", "memory": "64Gi", "pods": "110"}))
    for i in range(2):
        p = make_pod(f"t{i}", node_name="b")
        p["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:00Z"
        store.create("pods", p)
    store.create("pods", make_pod("running", node_name="c"))
    s = new_scheduler(store, load_config(score_only("PodState")))
    s.sync_informers(20)
    out = s.explain(make_pod("p"))
    sc = {n: v["PodState*1"] for n, v in out["scores"].items()}
    assert sc["b"] == 100 and sc["a"] == 0 and sc["c"] == 0
    assert out["selected"] == "b"
    s.stop()


def test_qossort_orders_by_priority_then_qos(store):
    # A one-slot node: the first pod the queue pops is the one that binds.
    store.create("nodes", make_node("n", {"cpu": "64", "memory": "64Gi", "pods": "1"}))
    plugins = {"queueSort": {"enabled": [{"name": "QOSSort"}], "disabled": [{"name": "*"}]}}
    s = new_scheduler(store, load_config(cfg(plugins)), start=False)
    store.create("pods", make_pod("besteffort"))
    store.create("pods", make_pod("burstable", requests={"cpu": "1"}))
    store.create("pods", make_pod("guaranteed", requests={"cpu": "1", "memory": "1Gi"},
                                  limits={"cpu": "1", "memory": "1Gi"}))
    s.sync_informers(20)
    assert s.schedule_one(1000)
    wait_bound(s, 1)
    assert placements(store)["guaranteed"] == "n"
    s.stop()


def test_qossort_priority_dominates_qos(store):
    store.create("nodes", make_node("n", {"cpu": "64", "memory": "64Gi", "pods": "1"}))
    plugins = {"queueSort": {"enabled": [{"name": "QOSSort"}], "disabled": [{"name": "*"}]}}
    s = new_scheduler(store, load_config(cfg(plugins)), start=False)
    store.create("pods", make_pod("guaranteed", requests={"cpu": "1", "memory": "1Gi"},
                                  limits={"cpu": "1", "memory": "1Gi"}))
    store.create("pods", make_pod("urgent-besteffort", priority=1000))
    s.sync_informers(20)
    assert s.schedule_one(1000)
    wait_bound(s, 1)
    assert placements(store)["urgent-besteffort"] == "n"
    s.stop()
