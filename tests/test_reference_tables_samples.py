"""The reference's unit tables for the sample plugins, case for case, through
Scheduler.plugin_call:

* pkg/noderesources/allocatable_test.go:40  TestNodeResourcesAllocatable (14 cases)
* pkg/qos/queue_sort_test.go:28             TestSortLess (8 cases)
* pkg/podstate/pod_state_test.go:39         TestPodState (5 cases)
"""
import pytest

from flex_gpu_scheduler_amd import Store, load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_container, make_node, make_pod

MIN, MAX = 0, 100


def score_only(plugin, args=None):
    return {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
            "profiles": [{"schedulerName": "default-scheduler", "plugins": {
                "filter": {"disabled": [{"name": "*"}]}, "preFilter": {"disabled": [{"name": "*"}]},
                "score": {"enabled": [{"name": plugin}], "disabled": [{"name": "*"}]}},
                "pluginConfig": [{"name": plugin, "args": args or {}}] if args is not None else []}]}


# ---------------------------------------------------------------- Allocatable
def machine(name, milli_cpu, memory):
    """makeNodeInfo(node, milliCPU, memory) (allocatable_test.go:303)."""
    return make_node(name, {"cpu": f"{milli_cpu}m", "memory": str(memory), "pods": "110"})


DEFAULT_SET = [{"name": "cpu", "weight": 1 << 20}, {"name": "memory", "weight": 1}]  # 1 millicore ~ 1 MiB
CPU_SET = [{"name": "cpu", "weight": 1 << 30}, {"name": "memory", "weight": 1}]      # 1 millicore ~ 1 GiB
NO_RES = None
CPU_AND_MEM = {"cpu": "1000m", "memory": "1Gi"}
BIG_CPU = {"cpu": "8000m", "memory": "1Gi"}
SCHEDULED = ("machine1", [{"cpu": "1000m", "memory": "0"}, {"cpu": "2000m", "memory": "0"}])
M1_PODS = [("machine1", None), ("machine1", None), ("machine2", None), ("machine2", None)]

ALLOC_CASES = [
    ("nothing scheduled, nothing requested", NO_RES, [("machine1", 4000, 10000), ("machine2", 4000, 10000)],
     DEFAULT_SET, "Least", [], [MIN, MIN]),
    ("nothing scheduled, resources requested, differently sized machines, least mode", CPU_AND_MEM,
     [("machine1", 4000, 10000), ("machine2", 6000, 10000)], DEFAULT_SET, "Least", [], [MAX, MIN]),
    ("nothing scheduled, resources requested, differently sized machines, most mode", CPU_AND_MEM,
     [("machine1", 4000, 10000), ("machine2", 6000, 10000)], DEFAULT_SET, "Most", [], [MIN, MAX]),
    ("no resources requested, pods scheduled", NO_RES, [("machine1", 4000, 10000), ("machine2", 4000, 10000)],
     DEFAULT_SET, "Least", M1_PODS, [MIN, MIN]),
    ("no resources requested, pods scheduled with resources", NO_RES,
     [("machine1", 10000, 20000), ("machine2", 10000, 20000)], DEFAULT_SET, "Least", [SCHEDULED], [MIN, MIN]),
    ("resources requested, pods scheduled with resources", CPU_AND_MEM,
     [("machine1", 10000, 20000), ("machine2", 10000, 20000)], DEFAULT_SET, "Least", [SCHEDULED], [MIN, MIN]),
    ("resources requested with more than the node, differently sized machines, least mode", BIG_CPU,
     [("machine1", 4000, 1000), ("machine2", 5000, 1000)], DEFAULT_SET, "Least", [], [MAX, MIN]),
    ("resources requested with more than the node, differently sized machines, most mode", BIG_CPU,
     [("machine1", 4000, 1000), ("machine2", 5000, 1000)], DEFAULT_SET, "Most", [], [MIN, MAX]),
    ("nothing scheduled, resources requested, differently sized machines, cpu weighted, least mode", CPU_AND_MEM,
     [("machine1", 1000, 2000), ("machine2", 1005, 1000)], CPU_SET, "Least", [], [MAX, MIN]),
    ("nothing scheduled, resources requested, differently sized machines, cpu weighted, most mode", CPU_AND_MEM,
     [("machine1", 1000, 2000), ("machine2", 1005, 1000)], CPU_SET, "Most", [], [MIN, MAX]),
    ("nothing scheduled, resources requested, 3 differently sized machines, least mode", CPU_AND_MEM,
     [("machine1", 1000, 1000 << 20), ("machine2", 2000, 2000 << 20), ("machine3", 3000, 3000 << 20)],
     DEFAULT_SET, "Least", [], [MAX, (MIN + MAX) // 2, MIN]),
    ("nothing scheduled, resources requested, 3 differently sized machines, most mode", CPU_AND_MEM,
     [("machine1", 1000, 1000 << 20), ("machine2", 2000, 2000 << 20), ("machine3", 3000, 3000 << 20)],
     DEFAULT_SET, "Most", [], [MIN, (MIN + MAX) // 2, MAX]),
]


@pytest.mark.parametrize("name,req,machines,resources,mode,pods,expected", ALLOC_CASES,
                         ids=[c[0] for c in ALLOC_CASES])
def test_node_resources_allocatable(name, req, machines, resources, mode, pods, expected):
    store = Store()
    for m in machines:
        store.create("nodes", machine(*m))
    for i, (node, conts) in enumerate(pods):
        cs = [make_container(f"c{j}", requests=r) for j, r in enumerate(conts or [])]
        store.create("pods", make_pod(f"scheduled{i}", containers=cs, node_name=node))
    s = new_scheduler(store, load_config(score_only("NodeResourcesAllocatable",
                                                    {"resources": resources, "mode": mode})))
    try:
        s.sync_informers(50)
        pod = make_pod("p", containers=[make_container("p", requests=req)] if req else [])
        out = s.plugin_call("NodeResourcesAllocatable", "score", {"pod": pod, "nodes": [m[0] for m in machines]})
        assert [out["scores"][m[0]] for m in machines] == expected
    finally:
        s.stop()


@pytest.mark.parametrize("resources,err", [
    ([{"name": "memory", "weight": -1}, {"name": "cpu", "weight": 1}],
     "resource Weight of memory should be a positive value, got -1"),
    ([{"name": "memory", "weight": 1}, {"name": "cpu", "weight": 0}],
     "resource Weight of cpu should be a positive value, got 0"),
])
def test_node_resources_allocatable_rejects_non_positive_weights(resources, err):
    store = Store()
    store.create("nodes", machine("machine", 4000, 10000))
    with pytest.raises(Exception, match=err):
        new_scheduler(store, load_config(score_only("NodeResourcesAllocatable", {"resources": resources})))


# ----------------------------------------------------------------- QOSSort
def qos_pod(name, prio, requests=None, limits=None):
    """makePod(name, priority, requests, limits) (queue_sort_test.go:131)."""
    c = make_container(name)
    if requests:
        c["resources"]["requests"] = dict(requests)
    if limits:
        c["resources"]["limits"] = dict(limits)
    return make_pod(name, containers=[c], priority=prio)


def res(cpu, mem):
    return {"cpu": cpu, "memory": mem}


G = (res("100m", "100Mi"), res("100m", "100Mi"))       # Guaranteed: requests == limits
B = (res("100m", "100Mi"), res("200m", "200Mi"))       # Burstable
QOS_CASES = [
    ("p1's priority greater than p2", (100, None, None), (50, None, None), True),
    ("p1's priority less than p2", (50, None, None), (80, None, None), False),
    ("p1 and p2 are both BestEfforts", (0, None, None), (0, None, None), True),
    ("p1 is BestEfforts, p2 is Guaranteed", (0, None, None), (0, *G), False),
    ("p1 is Burstable, p2 is Guaranteed", (0, *B), (0, *G), False),
    ("both p1 and p2 are Burstable", (0, *B), (0, *B), True),
    ("p1 is Guaranteed, p2 is Burstable", (0, *G), (0, *B), True),
    ("both p1 and p2 are Guaranteed", (0, *G), (0, *G), True),
]


@pytest.fixture(scope="module")
def qos_sched():
    cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": "default-scheduler", "plugins": {
               "queueSort": {"enabled": [{"name": "QOSSort"}], "disabled": [{"name": "*"}]}}}]}
    s = new_scheduler(Store(), load_config(cfg))
    yield s
    s.stop()


@pytest.mark.parametrize("name,p1,p2,want", QOS_CASES, ids=[c[0] for c in QOS_CASES])
def test_qos_sort_less(qos_sched, name, p1, p2, want):
    a, b = qos_pod("p1", *p1), qos_pod("p2", *p2)
    assert qos_sched.plugin_call("QOSSort", "less", {"a": a, "b": b})["less"] is want


# ---------------------------------------------------------------- PodState
def pod_state_node(store, node, terminating, nominated, regular):
    """makeNodeInfo(node, terminating, nominated, regular) (pod_state_test.go:122):
    terminating pods carry a deletionTimestamp; nominated pods are pending
    pods whose status nominates the node (the nominator holds them)."""
    store.create("nodes", make_node(node, {"cpu": "64", "memory": "64Gi", "pods": "110"}))
    for i in range(terminating):
        p = make_pod(f"tpod-{node}-{i + 1}", node_name=node)
        p["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:00Z"
        store.create("pods", p)
    for i in range(nominated):
        p = make_pod(f"npod-{node}-{i + 1}")
        p["status"] = {"phase": "Pending", "nominatedNodeName": node}
        store.create("pods", p)
    for i in range(regular):
        store.create("pods", make_pod(f"rpod-{node}-{i + 1}", node_name=node))


POD_STATE_CASES = [
    ("more terminating pods score higher; regular pods only score lowest",
     [("node1", 6, 0, 10), ("node2", 3, 0, 10), ("node3", 0, 0, 10)], [MAX, 50, MIN]),
    ("more nominated pods score lower; regular pods only score highest",
     [("node1", 0, 2, 10), ("node2", 0, 1, 10), ("node3", 0, 0, 10)], [MIN, 50, MAX]),
    ("more (terminating - nominated) scores higher",
     [("node1", 5, 2, 10), ("node2", 3, 1, 10)], [MAX, MIN]),
    ("less (terminating - nominated) scores lower",
     [("node1", 5, 4, 10), ("node2", 3, 1, 10)], [MIN, MAX]),
    ("more (terminating - nominated) scores higher, 4 nodes",
     [("node1", 5, 0, 10), ("node2", 3, 1, 10), ("node3", 2, 1, 10), ("node4", 0, 1, 10)], [MAX, 50, 33, MIN]),
]


@pytest.mark.parametrize("name,nodes,expected", POD_STATE_CASES, ids=[c[0] for c in POD_STATE_CASES])
def test_pod_state(name, nodes, expected):
    store = Store()
    for n in nodes:
        pod_state_node(store, *n)
    s = new_scheduler(store, load_config(score_only("PodState")))
    try:
        s.sync_informers(50)
        out = s.plugin_call("PodState", "score", {"pod": make_pod("p"), "nodes": [n[0] for n in nodes]})
        assert [out["scores"][n[0]] for n in nodes] == expected
    finally:
        s.stop()
