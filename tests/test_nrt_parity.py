"""NodeResourceTopologyMatch: the reference's integration cases
(test/integration/noderesourcetopology_test.go:176-860), verbatim shapes.

Two nodes (64 cpu, 128Gi, 32 pods, 896Mi hugepages-2Mi, 48 vendor/nic1) and
per-case NRT objects; a default profile (upstream defaults + NRT filter/score
with MostAllocated) and three single-purpose profiles (QueueSort + NRT
filter/score + DefaultBinder) named after their scoring strategy
(:60-64, :112-137, :997-1040). The SingleNUMANodeContainerLevel matrix
(pkg/noderesourcetopology/TESTS.md:19-40, :620-858) runs against fake-node-1
with fake-node-2's availability zeroed; "not fit" rows must fail with the
reference's FailedScheduling message ("cannot align [init ]container: <name>").
"""
import time

import pytest

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_container, make_node, make_nrt, make_pod

HUGE, NIC = "hugepages-2Mi", "vendor/nic1"
POD = "topology-aware-scheduler-pod"
MOST, BALANCED, LEAST = "MostAllocated-scheduler", "BalancedAllocation-scheduler", "LeastAllocated-scheduler"


def _profile(name, strategy):
    none = [{"name": "*"}]
    pts = ("preFilter", "filter", "postFilter", "preScore", "score", "reserve", "permit", "preBind", "postBind")
    plugins = {p: {"disabled": none} for p in pts}
    plugins["queueSort"] = {"enabled": [{"name": "PrioritySort"}], "disabled": none}
    plugins["filter"] = {"enabled": [{"name": "NodeResourceTopologyMatch"}], "disabled": none}
    plugins["score"] = {"enabled": [{"name": "NodeResourceTopologyMatch"}], "disabled": none}
    plugins["bind"] = {"enabled": [{"name": "DefaultBinder"}], "disabled": none}
    return {"schedulerName": name, "plugins": plugins,
            "pluginConfig": [{"name": "NodeResourceTopologyMatch", "args": {"scoringStrategy": {"type": strategy}}}]}


CONFIG = {
    "apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
    "profiles": [
        {"schedulerName": "default-scheduler",
         "plugins": {"filter": {"enabled": [{"name": "NodeResourceTopologyMatch"}]},
                     "score": {"enabled": [{"name": "NodeResourceTopologyMatch"}]}},
         "pluginConfig": [{"name": "NodeResourceTopologyMatch",
                           "args": {"scoringStrategy": {"type": "MostAllocated"}}}]},
        _profile(MOST, "MostAllocated"), _profile(BALANCED, "BalancedAllocation"), _profile(LEAST, "LeastAllocated"),
    ],
}


def zone(i, *res):
    """MakeTopologyResInfo(name, capacity, available) triples."""
    return {"name": f"node-{i}", "type": "Node", "resources": [
        {"name": n, "capacity": c, "allocatable": c, "available": a} for n, c, a in res]}


def nrt(node, policy, *zones):
    return make_nrt(node, [zone(i, *z) for i, z in enumerate(zones)], (policy,))


CNT = "SingleNUMANodeContainerLevel"
PODL = "SingleNUMANodePodLevel"


def pod(containers=(), inits=(), scheduler=None, requests=None):
    """withLimits(): limits only (requests default to limits -> Guaranteed)."""
    if requests is not None:
        return make_pod(POD, requests=requests, scheduler_name=scheduler)
    cs = [make_container(f"cnt-{i + 1}", limits=r, requests=r) for i, r in enumerate(containers)]
    ics = [make_container(f"initcnt-{i + 1}", limits=r, requests=r) for i, r in enumerate(inits)]
    if not cs:
        cs = [make_container("pause")]
    return make_pod(POD, containers=cs, init_containers=ics or None, scheduler_name=scheduler)


def cm(c, m):
    return {"cpu": c, "memory": m}


NAMED = [
    ("Filtering out nodes that cannot fit resources on a single numa node in case of Guaranteed pod",
     pod([cm("4", "5Gi")]),
     [nrt("fake-node-1", CNT, [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")], [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")]),
      nrt("fake-node-2", CNT, [("cpu", "4", "4"), ("memory", "8Gi", "8Gi")], [("cpu", "0", "0"), ("memory", "8Gi", "8Gi")])],
     ["fake-node-2"]),
    ("Scheduling of a burstable pod requesting only cpus",
     pod(requests={"cpu": "4"}),
     [nrt("fake-node-1", CNT, [("cpu", "4", "4")], [("cpu", "0", "0")]),
      nrt("fake-node-2", CNT, [("cpu", "2", "2")], [("cpu", "2", "2")])],
     ["fake-node-1", "fake-node-2"]),
    ("Scheduling of a burstable pod requesting only memory",
     pod(requests={"memory": "5Gi"}),
     [nrt("fake-node-1", CNT, [("foo", "2", "2")], [("foo", "2", "2")]),
      nrt("fake-node-2", "foo", [("foo", "2", "2")], [("foo", "2", "2")])],
     ["fake-node-1", "fake-node-2"]),
    ("Scheduling Guaranteed pod with most-allocated strategy scheduler",
     pod([cm("1", "4Gi")], scheduler=MOST),
     [nrt("fake-node-1", CNT, [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")], [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")]),
      nrt("fake-node-2", CNT, [("cpu", "1", "1"), ("memory", "4Gi", "4Gi")], [("cpu", "1", "1"), ("memory", "4Gi", "4Gi")])],
     ["fake-node-2"]),
    ("Scheduling Guaranteed pod with balanced-allocation strategy scheduler",
     pod([cm("2", "2Gi")], scheduler=BALANCED),
     [nrt("fake-node-1", CNT, [("cpu", "4", "4"), ("memory", "50Gi", "50Gi")],
          [("cpu", "4", "4"), ("memory", "50Gi", "50Gi")]),
      nrt("fake-node-2", CNT, [("cpu", "6", "6"), ("memory", "6Gi", "6Gi")], [("cpu", "6", "6"), ("memory", "6Gi", "6Gi")])],
     ["fake-node-2"]),
    ("Scheduling Guaranteed pod with least-allocated strategy scheduler",
     pod([cm("1", "4Gi")], scheduler=LEAST),
     [nrt("fake-node-1", CNT, [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")], [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")]),
      nrt("fake-node-2", CNT, [("cpu", "1", "1"), ("memory", "4Gi", "4Gi")], [("cpu", "1", "1"), ("memory", "4Gi", "4Gi")])],
     ["fake-node-1"]),
    ("Scheduling Best-Effort pod with most-allocated strategy scheduler", pod(scheduler=MOST), [],
     ["fake-node-1", "fake-node-2"]),
    ("Scheduling Best-Effort pod with balanced-allocation strategy scheduler", pod(scheduler=BALANCED), [],
     ["fake-node-1", "fake-node-2"]),
    ("Scheduling Best-Effort pod with least-allocated strategy scheduler", pod(scheduler=LEAST), [],
     ["fake-node-1", "fake-node-2"]),
    ("SingleNUMANodePodLevel: Filtering out nodes that cannot fit resources in case of Guaranteed pod with multi containers",
     pod([cm("2", "4Gi"), cm("2", "4Gi")]),
     [nrt("fake-node-1", PODL, [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")], [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")]),
      nrt("fake-node-2", PODL, [("cpu", "4", "4"), ("memory", "8Gi", "8Gi")], [("cpu", "4", "4"), ("memory", "8Gi", "8Gi")])],
     ["fake-node-2"]),
    ("SingleNUMANodeContainerLevel: Filtering out nodes that cannot fit resources in case of Guaranteed pod "
     "with multi containers",
     pod([cm("3", "5Gi"), cm("3", "5Gi")]),
     [nrt("fake-node-1", CNT, [("cpu", "8", "6"), ("memory", "8Gi", "8Gi")], [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")]),
      nrt("fake-node-2", CNT, [("cpu", "4", "4"), ("memory", "8Gi", "8Gi")], [("cpu", "4", "4"), ("memory", "8Gi", "8Gi")])],
     ["fake-node-2"]),
    ("SingleNUMANodeContainerLevel: Filtering out nodes that cannot fit resources in case of Guaranteed pod with init container",
     pod([cm("2", "4Gi")], [cm("4", "4Gi")]),
     [nrt("fake-node-1", CNT, [("cpu", "4", "3"), ("memory", "8Gi", "8Gi")], [("cpu", "4", "3"), ("memory", "8Gi", "8Gi")]),
      nrt("fake-node-2", CNT, [("cpu", "4", "4"), ("memory", "8Gi", "8Gi")], [("cpu", "4", "4"), ("memory", "8Gi", "8Gi")])],
     ["fake-node-2"]),
    ("SingleNUMANodeContainerLevel: Cannot fit resources in case of Guaranteed pod with multi containers",
     pod([cm("4", "4Gi"), cm("2", "4Gi")]),
     [nrt("fake-node-1", CNT, [("cpu", "4", "4"), ("memory", "8Gi", "8Gi")], [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")]),
      nrt("fake-node-2", CNT, [("cpu", "6", "3"), ("memory", "8Gi", "8Gi")], [("cpu", "4", "3"), ("memory", "8Gi", "8Gi")])],
     ["fake-node-1"]),
    ("Negative: SingleNUMANodeContainerLevel: Cannot fit resources in case of Guaranteed pod with init container",
     pod([cm("2", "4Gi")], [cm("4", "10Gi")]),
     [nrt("fake-node-1", CNT, [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")], [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")]),
      nrt("fake-node-2", CNT, [("cpu", "4", "4"), ("memory", "8Gi", "8Gi")], [("cpu", "4", "4"), ("memory", "8Gi", "8Gi")])],
     []),
    ("Negative: SingleNUMANodeContainerLevel: Cannot fit resources in case of Guaranteed pod with multi containers",
     pod([cm("4", "4Gi"), cm("4", "6Gi")]),
     [nrt("fake-node-1", CNT, [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")], [("cpu", "2", "2"), ("memory", "8Gi", "8Gi")]),
      nrt("fake-node-2", CNT, [("cpu", "4", "4"), ("memory", "8Gi", "8Gi")], [("cpu", "4", "4"), ("memory", "8Gi", "3Gi")])],
     []),
]


def _c(cpu, mem, huge=None, nic=None):
    d = {"cpu": cpu, "memory": mem}
    if huge:
        d[HUGE] = huge
    if nic:
        d[NIC] = nic
    return d


# (TESTS.md row + description, init containers, containers, expected FailedScheduling substring or "")
MATRIX = [
    ("[4] multi containers with good devices and hugepages allocation, spread across NUMAs - fit",
     [], [_c("2", "6Gi", "500Mi", "16"), _c("2", "6Gi", "50Mi", "8")], ""),
    ("[5] multi containers with hugepages over allocation, spread across NUMAs - not fit",
     [], [_c("2", "6Gi", "400Mi"), _c("2", "6Gi", "400Mi")], "cannot align container: cnt-2"),
    ("[5] multi containers with device over allocation, spread across NUMAs - not fit",
     [], [_c("2", "6Gi", "50Mi", "20"), _c("2", "6Gi", "500Mi", "20")], "cannot align container: cnt-2"),
    ("[7] init container with cpu over allocation, multi-containers with good allocation - not fit",
     [_c("40", "40Gi")], [_c("1", "4Gi"), _c("1", "4Gi")], "cannot align init container: initcnt-1"),
    ("[7] init container with memory over allocation, multi-containers with good allocation - not fit",
     [_c("4", "70Gi")], [_c("1", "4Gi"), _c("1", "4Gi")], "cannot align init container: initcnt-1"),
    ("[11] init container with good allocation, multi-containers spread across NUMAs - fit",
     [_c("4", "10Gi")], [_c("20", "40Gi"), _c("20", "40Gi")], ""),
    ("[12] init container with good allocation, multi-containers with cpu over allocation - not fit",
     [_c("4", "10Gi")], [_c("20", "40Gi"), _c("20", "40Gi"), _c("20", "10Gi")], "cannot align container: cnt-3"),
    ("[12] init container with good allocation, multi-containers with memory over allocation - not fit",
     [_c("4", "10Gi")], [_c("20", "40Gi"), _c("20", "40Gi"), _c("2", "40Gi")], "cannot align container: cnt-3"),
    ("[17] multi init containers with good allocation, multi-containers spread across NUMAs - fit",
     [_c("4", "10Gi")] * 3, [_c("20", "40Gi"), _c("20", "40Gi"), _c("6", "10Gi")], ""),
    ("[18] multi init containers with good allocation, multi-containers with cpu over allocation - not fit",
     [_c("4", "10Gi")] * 3, [_c("20", "40Gi"), _c("20", "40Gi"), _c("20", "10Gi")], "cannot align container: cnt-3"),
    ("[18] multi init containers with good allocation, multi-containers with memory over allocation - not fit",
     [_c("4", "10Gi")] * 3, [_c("20", "35Gi"), _c("20", "35Gi"), _c("2", "50Gi")], "cannot align container: cnt-3"),
    ("[24] multi init containers with good allocation, multi-containers with cpu over allocation - not fit",
     [_c("30", "10Gi")] * 2, [_c("20", "40Gi"), _c("20", "40Gi"), _c("20", "6Gi")], "cannot align container: cnt-3"),
    ("[24] multi init containers with good allocation, multi-containers with memory over allocation - not fit",
     [_c("30", "10Gi")] * 2, [_c("20", "35Gi"), _c("20", "35Gi"), _c("2", "50Gi")], "cannot align container: cnt-3"),
    ("[27] multi init containers with good allocation, container with cpu over allocation - not fit",
     [_c("30", "10Gi")] * 2, [_c("35", "40Gi")], "cannot align container: cnt-1"),
    ("[28] multi init containers with good allocation, multi-containers with good allocation - fit",
     [_c("30", "10Gi")] * 2, [_c("20", "40Gi"), _c("20", "40Gi")], ""),
    ("[29] multi init containers whose cpus together exceed allocatable, multi-containers with good allocation - fit",
     [_c("30", "10Gi")] * 3, [_c("20", "40Gi"), _c("20", "40Gi"), _c("2", "6Gi")], ""),
    ("[29] multi init containers whose memory together exceeds allocatable, multi-containers with good allocation - fit",
     [_c("3", "50Gi")] * 3, [_c("20", "40Gi"), _c("20", "40Gi"), _c("2", "6Gi")], ""),
    ("[32] multi init containers with cpu over allocation - not fit",
     [_c("40", "50Gi"), _c("3", "50Gi"), _c("3", "50Gi")], [_c("20", "40Gi"), _c("2", "6Gi")],
     "cannot align init container: initcnt-1"),
    ("[32] multi init containers with over memory allocation - not fit",
     [_c("20", "50Gi"), _c("20", "65Gi"), _c("3", "50Gi")], [_c("20", "40Gi"), _c("2", "6Gi")],
     "cannot align init container: initcnt-2"),
]

MATRIX_NRTS = [
    nrt("fake-node-1", CNT,
        [("cpu", "32", "30"), ("memory", "64Gi", "60Gi"), (HUGE, "384Mi", "384Mi"), (NIC, "16", "16")],
        [("cpu", "32", "32"), ("memory", "64Gi", "64Gi"), (HUGE, "512Mi", "512Mi"), (NIC, "32", "32")]),
    # fake-node-2 has nothing available, so every case runs against fake-node-1.
    nrt("fake-node-2", CNT,
        [("cpu", "32", "0"), ("memory", "64Gi", "0"), (HUGE, "384Mi", "0"), (NIC, "16", "0")],
        [("cpu", "32", "0"), ("memory", "64Gi", "0"), (HUGE, "512Mi", "0"), (NIC, "32", "0")]),
]


@pytest.fixture
def cluster(store):
    res = {"cpu": "64", "memory": "128Gi", "pods": "32", HUGE: "896Mi", NIC: "48"}
    for n in ("fake-node-1", "fake-node-2"):
        store.create("nodes", make_node(n, res, labels={"node": n}))
    s = new_scheduler(store, load_config(CONFIG), start=True)
    yield s
    s.stop()


def _run(store, sched, p, nrts, expected, err=""):
    for o in nrts:
        store.create("noderesourcetopologies", o)
    sched.sync_informers(50)
    store.create("pods", p)
    if expected:
        deadline = time.time() + 20
        while time.time() < deadline and not (store.get("pods", "default", POD)["spec"].get("nodeName")):
            time.sleep(0.01)
        node = store.get("pods", "default", POD)["spec"].get("nodeName")
        assert node in expected, (node, expected)
    else:
        deadline = time.time() + 20
        msgs: list[str] = []
        while time.time() < deadline:
            evs, _ = store.list("events", "default")
            msgs = [e.get("message", "") for e in evs if e.get("reason") == "FailedScheduling"
                    and (e.get("involvedObject") or {}).get("name") == POD]
            if msgs and (not err or any(err in m for m in msgs)):
                break
            time.sleep(0.02)
        assert msgs, "no FailedScheduling event"
        assert not err or any(err in m for m in msgs), msgs
        assert not store.get("pods", "default", POD)["spec"].get("nodeName")


@pytest.mark.parametrize("name,p,nrts,expected", NAMED, ids=[c[0] for c in NAMED])
def test_nrt_integration_cases(store, cluster, name, p, nrts, expected):
    _run(store, cluster, p, nrts, expected)


@pytest.mark.parametrize("name,inits,cnts,err", MATRIX, ids=[c[0] for c in MATRIX])
def test_nrt_container_scope_matrix(store, cluster, name, inits, cnts, err):
    _run(store, cluster, pod(cnts, inits), MATRIX_NRTS, [] if err else ["fake-node-1"], err)
