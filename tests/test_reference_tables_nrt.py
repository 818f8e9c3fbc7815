"""The reference's NodeResourceTopologyMatch unit tables, case for case,
against the native plugin through Scheduler.plugin_call("filter"/"score"):

* pkg/noderesourcetopology/filter_test.go:51   TestNodeResourceTopology (QoS classes, pod/container scope)
* pkg/noderesourcetopology/filter_test.go:413  TestNodeResourceTopologyMultiContainerPodScope
* pkg/noderesourcetopology/filter_test.go:638  TestNodeResourceTopologyMultiContainerContainerScope
* pkg/noderesourcetopology/score_test.go:38    TestNodeResourcesScoreWithStrategy (see below)

Fixtures follow the reference's helpers: a Node's capacity/allocatable is the
sum of its NRT zones' *available* values (makeResourceListFromZones,
pluginhelpers.go:106-118) plus the case's extra node resources; a pod built by
makePodByResourceList has one container (named "container1" by the test) with
requests = limits."""
import re

import pytest

from flex_gpu_scheduler_amd import Store, load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_container, make_node, make_nrt, make_pod

CPU, MEM, EXT, HUGE, NIC = "cpu", "memory", "namespace/extended", "hugepages-2Mi", "vendor/nic1"
NIC_NONE, NIC_NO_NUMA = "vendor/notexistingnic", "vendor.com/old-nic-model"
POD_LEVEL, CNT_LEVEL = "SingleNUMANodePodLevel", "SingleNUMANodeContainerLevel"

_UNITS = {"": 1, "k": 10 ** 3, "M": 10 ** 6, "G": 10 ** 9, "Ki": 1 << 10, "Mi": 1 << 20, "Gi": 1 << 30}


def qty(s: str) -> int:
    m = re.fullmatch(r"(\d+)([KMG]i?|k)?", s)
    return int(m.group(1)) * _UNITS[m.group(2) or ""]


def zone(i, *res):
    """MakeTopologyResInfo(name, capacity, available) triples as zone node-<i>."""
    return {"name": f"node-{i}", "type": "Node",
            "resources": [{"name": n, "capacity": c, "allocatable": c, "available": a} for n, c, a in res]}


def node_for(name, zones, extra=None):
    alloc: dict[str, int] = {}
    for z in zones:
        for r in z["resources"]:
            alloc[r["name"]] = alloc.get(r["name"], 0) + qty(r["available"])
    alloc = {k: str(v) for k, v in alloc.items()}
    alloc.update(extra or {})
    alloc.setdefault("pods", "110")
    return make_node(name, alloc)


def harness(descs):
    """descs: [(node name, policy, zones, extra node resources)]."""
    store = Store()
    for name, policy, zones, extra in descs:
        store.create("nodes", node_for(name, zones, extra))
        store.create("noderesourcetopologies", make_nrt(name, zones, (policy,)))
    cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": "default-scheduler", "plugins": {
               "filter": {"enabled": [{"name": "NodeResourceTopologyMatch"}], "disabled": [{"name": "*"}]},
               "score": {"enabled": [{"name": "NodeResourceTopologyMatch"}], "disabled": [{"name": "*"}]}}}]}
    s = new_scheduler(store, load_config(cfg))
    s.sync_informers(50)
    return s


def filter_on(s, pod, node):
    out = s.plugin_call("NodeResourceTopologyMatch", "filter", {"pod": pod, "nodes": [node]})
    st = out["nodes"][node]
    return None if st["code"] == "Success" else (st["code"], st["message"])


def pod_by_resources(res: dict, n: int = 1, name: str = ""):
    """makePodByResourceList / ...WithManyContainers; the first container is
    named container1 by the test (filter_test.go:389-391)."""
    cs = [make_container("container1" if i == 0 else f"c{i}", requests=res, limits=res) for i in range(n)]
    return make_pod(name, containers=cs)


# ---------------------------------------------------------- TestNodeResourceTopology (:51)
DESCS = [
    ("node1", CNT_LEVEL, [zone(0, (CPU, "20", "4"), (MEM, "8Gi", "8Gi"), (NIC, "30", "10")),
                          zone(1, (CPU, "30", "8"), (MEM, "8Gi", "8Gi"), (NIC, "30", "10"))], None),
    ("node2", CNT_LEVEL, [zone(0, (CPU, "20", "2"), (MEM, "8Gi", "4Gi"), (HUGE, "128Mi", "128Mi"), (NIC, "30", "5")),
                          zone(1, (CPU, "30", "4"), (MEM, "8Gi", "4Gi"), (HUGE, "128Mi", "128Mi"), (NIC, "30", "2"))],
     {NIC_NO_NUMA: "4"}),
    ("node3", POD_LEVEL, [zone(0, (CPU, "20", "2"), (MEM, "8Gi", "4Gi"), (NIC, "30", "5")),
                          zone(1, (CPU, "30", "4"), (MEM, "8Gi", "4Gi"), (NIC, "30", "2"))], None),
    ("badly-formed-node", POD_LEVEL, [zone(0, (CPU, "20", "2"), (MEM, "8Gi", "4Gi"), (NIC, "30", "5")),
                                      zone(75, (CPU, "30", "4"), (MEM, "8Gi", "4Gi"), (NIC, "30", "2"))], None),
    ("extended", CNT_LEVEL, [zone(0, (CPU, "20", "4"), (MEM, "8Gi", "8Gi"), (NIC, "30", "10")),
                             zone(1, (CPU, "30", "8"), (MEM, "8Gi", "8Gi"), (NIC, "30", "10"))], {EXT: "1"}),
]
N = [d[0] for d in DESCS]
CANNOT_CNT = ("Unschedulable", "cannot align container: container1")
CANNOT_POD = ("Unschedulable", "cannot align pod: ")

BASIC = [
    ("Guaranteed QoS, pod with extended resource fit", {CPU: "2", MEM: "2Gi", EXT: "1", NIC: "3"}, 1, N[4], None),
    ("Best effort QoS, pod fit", None, 0, N[0], None),
    ("Guaranteed QoS, minimal, pod fit", {CPU: "2", MEM: "2Gi"}, 1, N[0], None),
    ("Guaranteed QoS, minimal, saturating zone, pod fit", {CPU: "8", MEM: "8Gi"}, 1, N[0], None),
    ("Guaranteed QoS, zero quantity of unavailable resource, pod fit",
     {CPU: "2", MEM: "2Gi", HUGE: "0", NIC: "3"}, 1, N[0], None),
    ("Guaranteed QoS, pod fit", {CPU: "2", MEM: "2Gi", NIC: "3"}, 1, N[1], None),
    ("Guaranteed QoS, hugepages, pod fit", {CPU: "2", MEM: "2Gi", HUGE: "64Mi", NIC: "3"}, 1, N[1], None),
    ("Burstable QoS, pod fit", {CPU: "4", NIC: "3"}, 1, N[1], None),
    ("Burstable QoS, pod doesn't fit", {CPU: "4", NIC: "11"}, 1, N[1], CANNOT_CNT),
    ("Guaranteed QoS, hugepages, pod doesn't fit", {CPU: "2", MEM: "2Gi", HUGE: "256Mi", NIC: "3"}, 1, N[1],
     CANNOT_CNT),
    ("Guaranteed QoS, pod doesn't fit", {CPU: "9", MEM: "1Gi", NIC: "3"}, 1, N[0], CANNOT_CNT),
    ("Guaranteed QoS, pod fit (zero of a resource no zone has)", {CPU: "2", MEM: "1Gi", NIC_NONE: "0"}, 1, N[0], None),
    ("Guaranteed QoS Topology Scope, pod doesn't fit", {CPU: "3", MEM: "1Gi", NIC_NONE: "0"}, 3, N[2], CANNOT_POD),
    ("Guaranteed QoS Topology Scope, minimal, pod fit", {CPU: "1", MEM: "1Gi"}, 1, N[2], None),
    ("Guaranteed QoS TopologyScope, minimal, saturating zone, pod fit", {CPU: "2", MEM: "4Gi"}, 1, N[3], None),
    ("Guaranteed QoS Topology Scope, pod fit", {CPU: "1", MEM: "1Gi", NIC_NONE: "0"}, 3, N[2], None),
    ("Guaranteed QoS Topology Scope, invalid node", {CPU: "1", MEM: "1Gi", NIC_NONE: "0"}, 3, N[3], CANNOT_POD),
    ("Guaranteed QoS, hugepages, non-NUMA affine NIC, pod fit", {CPU: "2", MEM: "2Gi", HUGE: "64Mi", NIC_NO_NUMA: "3"},
     1, N[1], None),
]


@pytest.fixture(scope="module")
def basic_sched():
    s = harness(DESCS)
    yield s
    s.stop()


@pytest.mark.parametrize("name,res,n,node,want", BASIC, ids=[c[0] for c in BASIC])
def test_node_resource_topology(basic_sched, name, res, n, node, want):
    pod = make_pod("", containers=[]) if res is None else pod_by_resources(res, n)
    assert filter_on(basic_sched, pod, node) == want


# ------------------------------------------- MultiContainer pod scope (:413) / container scope (:638)
HOST0_ZONES = [zone(0, (CPU, "32", "30"), (MEM, "64Gi", "60Gi"), (HUGE, "384Mi", "384Mi"), (NIC, "16", "16")),
               zone(1, (CPU, "32", "32"), (MEM, "64Gi", "64Gi"), (HUGE, "512Mi", "512Mi"), (NIC, "32", "32"))]


def multi(name, cnts, inits=()):
    """makePod(name, withMultiInitContainers, withMultiContainers): containers
    cnt-1..n with requests = limits."""
    def mk(lst):
        return [make_container(f"cnt-{i + 1}", requests=r, limits=r) for i, r in enumerate(lst)]
    return make_pod(name, containers=mk(cnts), init_containers=mk(inits))


POD_SCOPE = [
    ("gu pod fits only on a numa node", [{CPU: "2", MEM: "2Gi"}, {CPU: "4", MEM: "8Gi"},
                                         {CPU: "26", MEM: "32Gi", HUGE: "512Mi", NIC: "26"}], None),
    ("gu pod does not fit - not enough CPUs available on any NUMA node",
     [{CPU: "2", MEM: "2Gi"}, {CPU: "8", MEM: "8Gi"}, {CPU: "26", MEM: "26Gi", HUGE: "52Mi", NIC: "26"}], "testpod"),
    ("gu pod does not fit - not enough memory available on any NUMA node",
     [{CPU: "2", MEM: "4Gi"}, {CPU: "4", MEM: "16Gi"}, {CPU: "26", MEM: "52Gi", HUGE: "52Mi", NIC: "26"}], "testpod"),
    ("gu pod does not fit - not enough Hugepages available on any NUMA node",
     [{CPU: "2", MEM: "2Gi"}, {CPU: "4", MEM: "8Gi"}, {CPU: "26", MEM: "32Gi", HUGE: "3328Mi", NIC: "26"}], "testpod"),
    ("gu pod does not fit - not enough devices available on any NUMA node",
     [{CPU: "2", MEM: "2Gi"}, {CPU: "4", MEM: "8Gi"}, {CPU: "26", MEM: "26Gi", HUGE: "52Mi", NIC: "52"}], "testpod"),
]


@pytest.mark.parametrize("name,cnts,err_pod", POD_SCOPE, ids=[c[0] for c in POD_SCOPE])
def test_multi_container_pod_scope(name, cnts, err_pod):
    s = harness([("host0", POD_LEVEL, HOST0_ZONES, None)])
    try:
        pod = multi("testpod", cnts)
        pod["spec"]["containers"][0]["name"] = "container1"  # the test renames the first container
        want = None if err_pod is None else ("Unschedulable", f"cannot align pod: {err_pod}")
        assert filter_on(s, pod, "host0") == want
    finally:
        s.stop()


def r(cpu, mem, **more):
    d = {CPU: cpu, MEM: mem}
    d.update({HUGE if k == "huge" else NIC: v for k, v in more.items()})
    return d


CONTAINER_SCOPE = [
    ("[1][tier3] single container with good allocation - fit", [], [r("2", "4G")], ""),
    ("[2][tier3] single container with cpu over allocation", [], [r("40", "4G")], "cannot align container: cnt-1"),
    ("[2][tier3] single container with memory over allocation", [], [r("2", "100G")], "cannot align container: cnt-1"),
    ("[2][tier3] single container with cpu and memory over allocation", [], [r("40", "100G")],
     "cannot align container: cnt-1"),
    ("[4][tier2] multi-containers with good allocation, spread across NUMAs - fit", [],
     [r("20", "40G"), r("20", "40G")], ""),
    ("[4][tier1] multi containers with good devices and hugepages allocation, spread across NUMAs - fit", [],
     [r("2", "6G", huge="500Mi", nic="16"), r("2", "6G", huge="50Mi", nic="8")], ""),
    ("[7][tier1] init container with cpu over allocation, multi-containers with good allocation - not fit",
     [r("40", "40G")], [r("1", "4G"), r("1", "4G")], "cannot align init container: cnt-1"),
    ("[7][tier1] init container with memory over allocation, multi-containers with good allocation - not fit",
     [r("4", "70G")], [r("1", "4G"), r("1", "4G")], "cannot align init container: cnt-1"),
    ("[11][tier1] init container with good allocation, multi-containers spread across NUMAs - fit",
     [r("4", "10G")], [r("20", "40G"), r("20", "40G")], ""),
    ("[17][tier1] multi init containers with good allocation, multi-containers spread across NUMAs - fit",
     [r("4", "10G")] * 3, [r("20", "40G"), r("20", "40G"), r("6", "10G")], ""),
    ("[24][tier1] multi init containers with good allocation, multi-containers with over cpu allocation - not fit",
     [r("30", "10G")] * 2, [r("20", "40G"), r("20", "40G"), r("20", "6G")], "cannot align container: cnt-3"),
    ("[27][tier1] multi init containers with good allocation, container with cpu over allocation - not fit",
     [r("30", "10G")] * 2, [r("35", "40G")], "cannot align container: cnt-1"),
    ("[28][tier1] multi init containers with good allocation, multi-containers with good allocation - fit",
     [r("30", "10G")] * 2, [r("20", "40G"), r("20", "40G")], ""),
    ("[29][tier1] multi init containers cpu sum over allocatable, multi-containers with good allocation - fit",
     [r("30", "10G")] * 3, [r("20", "40G"), r("20", "40G"), r("2", "6G")], ""),
    ("[29][tier1] multi init containers memory sum over allocatable, multi-containers with good allocation - fit",
     [r("3", "50G")] * 3, [r("20", "40G"), r("20", "40G"), r("2", "6G")], ""),
    ("[32][tier1] multi init containers with over cpu allocation - not fit",
     [r("40", "50G"), r("3", "50G"), r("3", "50G")], [r("20", "40G"), r("2", "6G")],
     "cannot align init container: cnt-1"),
    ("[32][tier1] multi init containers with over memory allocation - not fit",
     [r("20", "50G"), r("40", "50G"), r("3", "50G")], [r("20", "40G"), r("2", "6G")],
     "cannot align init container: cnt-2"),
]


@pytest.fixture(scope="module")
def cnt_sched():
    s = harness([("host0", CNT_LEVEL, HOST0_ZONES, None)])
    yield s
    s.stop()


@pytest.mark.parametrize("name,inits,cnts,err", CONTAINER_SCOPE, ids=[c[0] for c in CONTAINER_SCOPE])
def test_multi_container_container_scope(cnt_sched, name, inits, cnts, err):
    pod = multi(f"testpod{CONTAINER_SCOPE.index((name, inits, cnts, err))}", cnts, inits)
    assert filter_on(cnt_sched, pod, "host0") == (("Unschedulable", err) if err else None)


# ------------------------------------------------------- TestNodeResourceScorePlugin (score_test.go:38)
SCORE_DESCS = [
    ("node1", CNT_LEVEL, [zone(0, (CPU, "4", "4"), (MEM, "500Mi", "500Mi")),
                          zone(1, (CPU, "4", "4"), (MEM, "500Mi", "500Mi"))], None),
    ("node2", CNT_LEVEL, [zone(0, (CPU, "2", "2"), (MEM, "50Mi", "50Mi")),
                          zone(1, (CPU, "2", "2"), (MEM, "50Mi", "50Mi"))], None),
    ("node3", CNT_LEVEL, [zone(0, (CPU, "6", "6"), (MEM, "60Mi", "60Mi")),
                          zone(1, (CPU, "6", "6"), (MEM, "60Mi", "60Mi"))], None),
]


@pytest.mark.parametrize("strategy,want_node,want_score", [
    ("MostAllocated", "node2", 70),       # cpu 2/2 = 100%, memory 20M/50M = 40% -> (100 + 40) / 2
    ("BalancedAllocation", "node3", 100),  # cpu 2/6 = memory 20M/60M -> no variance
    ("LeastAllocated", "node1", 73),      # ((100 - 50) + (100 - 4)) / 2
])
def test_node_resource_score_strategy(strategy, want_node, want_score):
    store = Store()
    for name, policy, zones, extra in SCORE_DESCS:
        store.create("nodes", node_for(name, zones, extra))
        store.create("noderesourcetopologies", make_nrt(name, zones, (policy,)))
    cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": "default-scheduler", "plugins": {
               "score": {"enabled": [{"name": "NodeResourceTopologyMatch"}], "disabled": [{"name": "*"}]}},
               "pluginConfig": [{"name": "NodeResourceTopologyMatch",
                                 "args": {"scoringStrategy": {"type": strategy}}}]}]}
    s = new_scheduler(store, load_config(cfg))
    try:
        s.sync_informers(50)
        pod = pod_by_resources({CPU: "2", MEM: str(20 * 1024 * 1024)}, name="pod1")
        raw = s.plugin_call("NodeResourceTopologyMatch", "score", {"pod": pod})["raw"]
        # findMaxScoreNode: the highest score (ties to the later node in map order)
        best = max(raw.values())
        assert raw[want_node] == best == want_score, raw
    finally:
        s.stop()
