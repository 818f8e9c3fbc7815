"""The reference's per-plugin unit-test tables, case for case, against the
native plugins through Scheduler.plugin_call (one extension point of one
plugin on the calling thread, FakeClock, no scheduling loop):

* Coscheduling QueueSort      pkg/coscheduling/coscheduling_test.go:42  TestLess
* Coscheduling Permit         pkg/coscheduling/coscheduling_test.go:269 TestPermit
* Coscheduling PostFilter     pkg/coscheduling/coscheduling_test.go:335 TestPostFilter (+ the <=10% gap branch,
                              coscheduling.go:140-176)
* PodGroupManager PreFilter   pkg/coscheduling/core/core_test.go:42     TestPreFilter
* PodGroupManager Permit      pkg/coscheduling/core/core_test.go:178    TestPermit
* PodGroupManager PostBind    pkg/coscheduling/core/core_test.go:242    TestPostBind
* CheckClusterResource        pkg/coscheduling/core/core_test.go:303    TestCheckClusterResource
* CapacityScheduling PreFilter pkg/capacityscheduling/capacity_scheduling_test.go:52  TestPreFilter
* CapacityScheduling dry run   pkg/capacityscheduling/capacity_scheduling_test.go:166 TestDryRunPreemption

The reference builds its fixtures from test/util/utils.go MakeNodesAndPods
(30 nodes of cpu 1 / pods 20, 60 pods labelled test=a spread over them) and
MakePG (scheduleTimeoutSeconds 10); the same fixtures are created in a store
here. Where the reference injects internal state (a pre-filled denied cache,
ElasticQuota `Used` values) the same state is produced the plugin's own way:
the group is denied through the plugin, `Used` comes from assigned pods.
"""
import time

import pytest

from flex_gpu_scheduler_amd import FakeClock, Store, load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_elastic_quota, make_node, make_pod, make_pod_group
from flex_gpu_scheduler_amd.models.objects import make_container
from helpers import coscheduling_config

LOW, HIGH, MID = 10, 100, 50
NOW = 1_790_000_000  # whole seconds: creationTimestamp has second resolution


def rfc3339(sec: int) -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(sec))


def make_pg(name, ns, min_member, created=None, min_resources=None):
    pg = make_pod_group(name, ns, min_member, min_resources=min_resources, schedule_timeout_seconds=10)
    if created is not None:
        pg["metadata"]["creationTimestamp"] = rfc3339(created)
    return pg


def nodes_and_pods(store, labels: dict, n_pods: int, n_nodes: int, ns: str = "default"):
    """test/util MakeNodesAndPods: pod i on node i % n_nodes, with the first
    (i % len(labels)) + 1 labels."""
    for i in range(n_nodes):
        store.create("nodes", make_node(f"node{i}", {"cpu": "1", "pods": "20"}))
    items = list(labels.items())
    for i in range(n_pods):
        lab = dict(items[:i % len(items) + 1])
        store.create("pods", make_pod(f"pod{i}", ns, node_name=f"node{i % n_nodes}", labels=lab))


def harness(store, cfg):
    s = new_scheduler(store, load_config(cfg), clock=FakeClock(NOW * 1_000_000))
    s.sync_informers(50)
    return s


def pod(name, ns, prio=None, pg=None, **kw):
    return make_pod(name, ns, priority=prio, pod_group=pg, uid=name, **kw)


# ------------------------------------------------------------- TestLess ----
TIMES = [NOW + d for d in (0, 1, 2, 3, -2, -1)]
NS1, NS2 = "namespace1", "namespace2"
LESS_CASES = [
    ("p1.priority less than p2.priority", (LOW, None, None), (HIGH, None, None), False),
    ("p1.priority greater than p2.priority", (HIGH, None, None), (LOW, None, None), True),
    ("equal priority. p1 is added to schedulingQ earlier than p2", (HIGH, None, 0), (HIGH, None, 1), True),
    ("equal priority. p2 is added to schedulingQ earlier than p1", (HIGH, None, 1), (HIGH, None, 0), False),
    ("p1.priority less than p2.priority, p1 belongs to podGroup1", (LOW, "pg1", None), (HIGH, None, None), False),
    ("p1.priority greater than p2.priority, p1 belongs to podGroup1", (HIGH, "pg1", None), (LOW, None, None), True),
    ("equal priority. p1 is added to schedulingQ earlier than p2, p1 belongs to podGroup3",
     (HIGH, "pg3", 0), (HIGH, None, 1), True),
    ("equal priority. p2 is added to schedulingQ earlier than p1, p1 belongs to podGroup3",
     (HIGH, "pg3", 1), (HIGH, None, 0), False),
    ("p1.priority less than p2.priority, p1 belongs to podGroup1 and p2 belongs to podGroup2",
     (LOW, "pg1", None), (HIGH, "pg2", None), False),
    ("p1.priority greater than p2.priority, p1 belongs to podGroup1 and p2 belongs to podGroup2",
     (HIGH, "pg1", None), (LOW, "pg2", None), True),
    ("equal priority. p1 is added to schedulingQ earlier than p2, p1 belongs to podGroup1 and p2 belongs to podGroup2",
     (HIGH, "pg1", 0), (HIGH, "pg2", 1), True),
    ("equal priority. p2 is added to schedulingQ earlier than p1, p1 belongs to podGroup4 and p2 belongs to podGroup3",
     (HIGH, "pg4", 1), (HIGH, "pg3", 0), False),
    ("equal priority and creation time, p1 belongs to podGroup1 and p2 belongs to podGroup2",
     (HIGH, "pg1", 0), (HIGH, "pg2", 0), True),
    ("equal priority and creation time, p2 belong to podGroup2", (HIGH, None, 0), (HIGH, "pg2", 0), True),
]


@pytest.fixture(scope="module")
def less_harness():
    store = Store()
    for name, ns, t in (("pg1", NS1, 2), ("pg2", NS2, 3), ("pg3", NS2, 4), ("pg4", NS2, 5)):
        store.create("podgroups", make_pg(name, ns, 5, created=TIMES[t]))
    nodes_and_pods(store, {"test": "a"}, 60, 30)
    s = harness(store, coscheduling_config(permit_wait=10, denied=3))
    yield s
    s.stop()


@pytest.mark.parametrize("name,p1,p2,expected", LESS_CASES, ids=[c[0] for c in LESS_CASES])
def test_coscheduling_less(less_harness, name, p1, p2, expected):
    def mk(nm, ns, spec):
        prio, pg, t = spec
        return pod(nm, ns, prio, pg), (TIMES[t] * 1_000_000 if t is not None else 0)

    a, ta = mk("pod1", NS1, p1)
    b, tb = mk("pod2", NS2, p2)
    # The reference's p2 is in namespace2, where pg1 does not exist: a pod of
    # namespace1's pg1 is only ever p1 (as in the table).
    got = less_harness.plugin_call("Coscheduling", "less",
                                   {"a": a, "b": b, "a_initial_attempt_us": ta, "b_initial_attempt_us": tb})
    assert got["less"] is expected


# ------------------------------------------- TestPermit (coscheduling) ----
@pytest.mark.parametrize("name,p,expected", [
    ("pods do not belong to any podGroup", pod("pod1", "default"), "Success"),
    ("pods belong to a podGroup, Wait", pod("pod1", "ns1", pg="pg1"), "Wait"),
    ("pods belong to a podGroup, Allow", pod("pod1", "ns1", pg="pg2"), "Success"),
])
def test_coscheduling_permit(store, name, p, expected):
    store.create("podgroups", make_pg("pg1", "ns1", 2))
    store.create("podgroups", make_pg("pg2", "ns1", 1))
    nodes_and_pods(store, {"test": "a"}, 60, 30)
    s = harness(store, coscheduling_config())
    try:
        got = s.plugin_call("Coscheduling", "permit", {"pod": p, "node": "node0"})
        assert got["code"] == expected, got
        if expected == "Wait":
            assert got["timeout_us"] == 10_000_000  # MakePG's scheduleTimeoutSeconds
    finally:
        s.stop()


# ----------------------------------------------------------- TestPostFilter --
@pytest.mark.parametrize("name,p,group_pods,expected_empty_msg", [
    ("pod does not belong to any pod group", pod("pod1", "ns1"), False, False),
    ("enough pods assigned, do not reject all", pod("pod1", "ns1", pg="pg"), True, True),
    ("pod failed at filter phase, reject all pods", pod("pod1", "ns1", pg="pg"), False, False),
])
def test_coscheduling_post_filter(store, name, p, group_pods, expected_empty_msg):
    store.create("podgroups", make_pg("pg", "ns1", 2))
    if group_pods:  # MakeNodesAndPods({PodGroupLabel: pg}, 10, 30) in ns1
        nodes_and_pods(store, {"pod-group.scheduling.sigs.k8s.io": "pg"}, 10, 30, ns="ns1")
    else:
        nodes_and_pods(store, {"test": "a"}, 60, 30)
    s = harness(store, coscheduling_config())
    try:
        got = s.plugin_call("Coscheduling", "postFilter", {"pod": p, "statuses": {"node1": "Success"}})
        assert (got["message"] == "") is expected_empty_msg, got
        assert got["code"] in ("Unschedulable", "UnschedulableAndUnresolvable")
    finally:
        s.stop()


@pytest.mark.parametrize("assigned,min_member,rejects", [(9, 10, False), (8, 10, True), (0, 2, True)])
def test_coscheduling_post_filter_gap_branch(store, assigned, min_member, rejects):
    """coscheduling.go:159-166: with at most 10% of minMember unassigned the
    group is not rejected (plain Unschedulable, no message, not denied)."""
    store.create("podgroups", make_pg("big", "ns1", min_member))
    for i in range(max(min_member, 2)):
        store.create("nodes", make_node(f"n{i}", {"cpu": "4", "pods": "20"}))
    for i in range(assigned):
        store.create("pods", pod(f"m{i}", "ns1", pg="big", node_name=f"n{i}"))
    s = harness(store, coscheduling_config())
    try:
        me = pod("last", "ns1", pg="big")
        got = s.plugin_call("Coscheduling", "postFilter", {"pod": me, "statuses": {"n0": "Unschedulable"}})
        assert (got["message"] != "") is rejects, got
        # A rejected group is denied: its next PreFilter fails (core.go:155-157).
        pf = s.plugin_call("Coscheduling", "preFilter", {"pod": me})
        assert ("last failed" in pf["message"]) is rejects, pf
    finally:
        s.stop()


# ---------------------------------------------------- core TestPreFilter ----
def _pre_filter_world(store):
    store.create("podgroups", make_pg("pg", "ns1", 2))
    store.create("podgroups", make_pg("pg1", "ns1", 2))
    store.create("podgroups", make_pg("pg2", "ns1", 2, min_resources={"cpu": "4"}))
    store.create("podgroups", make_pg("pg3", "ns1", 2, min_resources={"cpu": "40"}))
    nodes_and_pods(store, {"test": "a"}, 60, 30)


PRE_FILTER_CASES = [
    ("pod does not belong to any pg", pod("p", "ns1"),
     [("pg1-1", "pg1"), ("pg2-1", "pg2")], False, True),
    ("pg was previously denied", pod("p1", "ns1", pg="pg1"), [], True, False),
    ("pod belongs to a non-existing pg", pod("p2", "ns1", pg="pg-notexisting"), [], False, True),
    ("pod count less than minMember", pod("p2", "ns1", pg="pg1"), [("pg2-1", "pg2")], False, False),
    ("pod count equal minMember", pod("p2", "ns1", pg="pg1"), [("pg1-1", "pg1"), ("pg2-1", "pg1")], False, True),
    ("pod count more minMember", pod("p2", "ns1", pg="pg1"),
     [("pg1-1", "pg1"), ("pg2-1", "pg1"), ("pg3-1", "pg1")], False, True),
    ("cluster resource enough, min Resource", pod("p2-1", "ns1", pg="pg2", requests={"cpu": "1"}),
     [("pg1-1", "pg2"), ("pg2-1", "pg2")], False, True),
    ("cluster resource not enough, min Resource", pod("p2-1", "ns1", pg="pg3", requests={"cpu": "20"}),
     [("pg1-1", "pg3"), ("pg2-1", "pg3")], False, False),
    ("cluster resource enough not required", pod("p2-1", "ns1", pg="pg1"),
     [("pg1-1", "pg1"), ("pg2-1", "pg1")], False, True),
]


@pytest.mark.parametrize("name,p,siblings,denied,expected_success", PRE_FILTER_CASES,
                         ids=[c[0] for c in PRE_FILTER_CASES])
def test_core_pre_filter(store, name, p, siblings, denied, expected_success):
    _pre_filter_world(store)
    for nm, pg in siblings:  # unscheduled pods in the pod lister
        store.create("pods", pod(nm, "ns1", pg=pg, scheduler_name="other-scheduler"))
    s = harness(store, coscheduling_config())
    try:
        if denied:  # the reference pre-fills lastDeniedPG with ns1/pg1
            s.plugin_call("Coscheduling", "deny", {"pod": p})
        got = s.plugin_call("Coscheduling", "preFilter", {"pod": p})
        assert (got["code"] == "Success") is expected_success, got
        if not expected_success:
            assert got["code"] == "UnschedulableAndUnresolvable"  # coscheduling.go:129-137
    finally:
        s.stop()


def test_denied_group_expires_with_the_ttl(store):
    _pre_filter_world(store)
    for nm in ("a", "b"):
        store.create("pods", pod(nm, "ns1", pg="pg1", scheduler_name="other-scheduler"))
    clock = FakeClock(NOW * 1_000_000)
    s = new_scheduler(store, load_config(coscheduling_config(denied=3)), clock=clock)
    s.sync_informers(50)
    try:
        me = pod("c", "ns1", pg="pg1")
        s.plugin_call("Coscheduling", "deny", {"pod": me})
        assert s.plugin_call("Coscheduling", "preFilter", {"pod": me})["code"] == "UnschedulableAndUnresolvable"
        clock.advance(3.1)
        assert s.plugin_call("Coscheduling", "preFilter", {"pod": me})["code"] == "Success"
    finally:
        s.stop()


# ------------------------------------------------------- core TestPermit ----
@pytest.mark.parametrize("name,p,member_bound,expected", [
    ("pod does not belong to any pg, allow", pod("p", "ns1"), True, "Success"),      # PodGroupNotSpecified
    ("pod belongs to a non-existing pg", pod("p", "ns1", pg="pg-noexist"), True, "Unschedulable"),  # NotFound
    ("pod belongs to a pg that doesn't have enough pods", pod("p", "ns1", pg="pg1"), False, "Wait"),
    ("pod belongs to a pg that has enough pods", pod("p", "ns1", pg="pg1"), True, "Success"),
])
def test_core_permit(store, name, p, member_bound, expected):
    store.create("podgroups", make_pg("pg", "ns1", 2))
    store.create("podgroups", make_pg("pg1", "ns1", 2))
    store.create("nodes", make_node("node0", {"cpu": "1", "pods": "20"}))
    if member_bound:  # MakeNodesAndPods({PodGroupLabel: pg1}, 1, 1), assigned, in ns1
        store.create("pods", pod("pod0", "ns1", pg="pg1", node_name="node0"))
    s = harness(store, coscheduling_config())
    try:
        got = s.plugin_call("Coscheduling", "permit", {"pod": p, "node": "node0"})
        assert got["code"] == expected, got
    finally:
        s.stop()


# ----------------------------------------------------- core TestPostBind ----
@pytest.mark.parametrize("name,pg,want_phase,want_scheduled", [
    ("pg status convert to scheduled", "pg", "Scheduled", 1),
    ("pg status convert to scheduling", "pg1", "Scheduling", 1),
    ("pg status does not convert, although scheduled pods change", "pg2", "Scheduling", 1),
])
def test_core_post_bind(store, name, pg, want_phase, want_scheduled):
    store.create("podgroups", make_pg("pg", "ns1", 1))
    store.create("podgroups", make_pg("pg1", "ns1", 2))
    pg2 = make_pg("pg2", "ns1", 3)
    pg2["status"] = {"phase": "Scheduling", "scheduled": 1}
    store.create("podgroups", pg2)
    store.create("nodes", make_node("node0", {"cpu": "1", "pods": "20"}))
    s = harness(store, coscheduling_config())
    try:
        s.plugin_call("Coscheduling", "postBind", {"pod": pod("p", "ns1", pg=pg), "node": "node0"})
        st = store.get("podgroups", "ns1", pg)["status"]
        assert st["phase"] == want_phase and st["scheduled"] == want_scheduled, st
    finally:
        s.stop()


# ------------------------------------------ core TestCheckClusterResource ----
@pytest.mark.parametrize("name,need,group_pod,member_group,enough", [
    ("Cluster resource enough", "10", None, "pg1-1", True),
    ("Cluster resource not enough", "1000", None, "pg1-1", False),
    ("Cluster resource enough, some resources of the pods belonging to the group have been included",
     "250", "pg1-1", "pg1-1", True),
    # Not in the reference's table (its assumed pod has no node, so the third
    # case passes either way): the same pod in ANOTHER group is not free.
    ("another group's pod is not counted as free", "250", "pg-other", "pg1-1", False),
])
def test_core_check_cluster_resource(store, name, need, group_pod, member_group, enough):
    store.create("nodes", make_node("fake-node", {"memory": "300", "pods": "110"}))
    if group_pod:
        store.create("pods", make_pod("t1-p1-3", "default", node_name="fake-node", pod_group=group_pod,
                                      containers=[make_container("c", requests={"memory": "100"})]))
    s = harness(store, coscheduling_config())
    try:
        got = s.plugin_call("Coscheduling", "checkClusterResource",
                            {"pod": pod("member", "default", pg=member_group), "need": {"memory": need}})
        assert got["enough"] is enough
    finally:
        s.stop()


# ------------------------------------------------ capacity TestPreFilter ----
def capacity_config():
    return {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
            "profiles": [{"schedulerName": "default-scheduler", "plugins": {
                "preFilter": {"enabled": [{"name": "CapacityScheduling"}]},
                "postFilter": {"enabled": [{"name": "CapacityScheduling"}], "disabled": [{"name": "*"}]},
                "reserve": {"enabled": [{"name": "CapacityScheduling"}]}}}]}


def quota_world(store, quotas: dict, used: dict, nodes=("big",), node_memory="100000"):
    """ElasticQuotas {ns: (min, max)} on memory; `used` {ns: [memory...]} as
    assigned pods (the reference sets ElasticQuotaInfo.Used directly)."""
    for n in nodes:
        store.create("nodes", make_node(n, {"memory": node_memory, "cpu": "100", "pods": "110"}))
    for ns, (mn, mx) in quotas.items():
        store.create("elasticquotas", make_elastic_quota(f"eq-{ns}", ns, min={"memory": str(mn)},
                                                         max={"memory": str(mx)}))
    for ns, mems in used.items():
        for i, m in enumerate(mems):
            store.create("pods", make_pod(f"used-{ns}-{i}", ns, node_name=nodes[0], uid=f"used-{ns}-{i}",
                                          containers=[make_container("c", requests={"memory": str(m)})]))


@pytest.mark.parametrize("name,quotas,used,pods,expected", [
    ("pod subjects to ElasticQuota", {"ns1": (1000, 2000)}, {"ns1": [300]},
     [("ns1-p1", "ns1", 500), ("ns1-p2", "ns1", 1800)], ["Success", "Unschedulable"]),
    ("the sum of used is bigger than the sum of min", {"ns1": (1000, 2000), "ns2": (1000, 2000)},
     {"ns1": [1800], "ns2": [200]}, [("ns2-p1", "ns2", 500)], ["Unschedulable"]),
])
def test_capacity_pre_filter(store, name, quotas, used, pods, expected):
    quota_world(store, quotas, used)
    s = harness(store, capacity_config())
    try:
        for (nm, ns, mem), want in zip(pods, expected):
            p = make_pod(nm, ns, uid=nm, containers=[make_container("c", requests={"memory": str(mem)})])
            got = s.plugin_call("CapacityScheduling", "preFilter", {"pod": p})
            assert got["code"] == want, (nm, got)
    finally:
        s.stop()


# ------------------------------------------ capacity TestDryRunPreemption ----
def _mem_pod(name, ns, mem, prio, node=None):
    return make_pod(name, ns, uid=name, priority=prio, node_name=node,
                    containers=[make_container("c", requests={"memory": str(mem)})])


@pytest.mark.parametrize("name,quotas,victims_prio,want", [
    ("in-namespace preemption", {"ns1": (50, 200), "ns2": (200, 200)},
     {"t1-p1": MID, "t1-p2": MID, "t1-p3": MID}, [("node-a", ["t1-p1"])]),
    ("cross-namespace preemption", {"ns1": (150, 200), "ns2": (50, 200)},
     {"t1-p1": MID, "t1-p2": HIGH, "t1-p3": MID}, [("node-a", ["t1-p3"])]),
])
def test_capacity_dry_run_preemption(store, name, quotas, victims_prio, want):
    store.create("nodes", make_node("node-a", {"memory": "150", "cpu": "100", "pods": "110"}))
    for ns, (mn, mx) in quotas.items():
        store.create("elasticquotas", make_elastic_quota(f"eq-{ns}", ns, min={"memory": str(mn)},
                                                         max={"memory": str(mx)}))
    for nm, ns in (("t1-p1", "ns1"), ("t1-p2", "ns2"), ("t1-p3", "ns2")):
        store.create("pods", _mem_pod(nm, ns, 50, victims_prio[nm], node="node-a"))
    cfg = capacity_config()
    cfg["profiles"][0]["plugins"]["filter"] = {"enabled": [{"name": "NodeResourcesFit"}]}
    s = harness(store, cfg)
    try:
        got = s.plugin_call("CapacityScheduling", "dryRunPreemption",
                            {"pod": _mem_pod("t1-p", "ns1", 50, HIGH), "runPreFilter": True})
        cands = sorted((c["node"], sorted(c["victims"])) for c in got["candidates"])
        assert cands == want, got
        assert all(c["numPDBViolations"] == 0 for c in got["candidates"])
    finally:
        s.stop()


def test_capacity_dry_run_memo_follows_quota_changes(store):
    """The dry-run memo (Evaluator, guarded by the quota predicates the
    victim selection read) must not serve a result across a quota change
    that flips those predicates: the same node, preemptor template and node
    version give the in-namespace victim under one quota set and the
    cross-namespace one under the other, then the first again."""
    store.create("nodes", make_node("node-a", {"memory": "150", "cpu": "100", "pods": "110"}))
    configs = {"in-namespace": ({"ns1": (50, 200), "ns2": (200, 200)}, ["t1-p1"]),
               "cross-namespace": ({"ns1": (150, 200), "ns2": (50, 200)}, ["t1-p3"])}
    for ns, (mn, mx) in configs["in-namespace"][0].items():
        store.create("elasticquotas", make_elastic_quota(f"eq-{ns}", ns, min={"memory": str(mn)},
                                                         max={"memory": str(mx)}))
    prios = {"t1-p1": MID, "t1-p2": HIGH, "t1-p3": MID}
    for nm, ns in (("t1-p1", "ns1"), ("t1-p2", "ns2"), ("t1-p3", "ns2")):
        store.create("pods", _mem_pod(nm, ns, 50, prios[nm], node="node-a"))
    cfg = capacity_config()
    cfg["profiles"][0]["plugins"]["filter"] = {"enabled": [{"name": "NodeResourcesFit"}]}
    s = harness(store, cfg)
    preemptor = _mem_pod("t1-p", "ns1", 50, HIGH)
    try:
        for step in ("in-namespace", "in-namespace", "cross-namespace", "cross-namespace", "in-namespace"):
            quotas, want = configs[step]
            for ns, (mn, mx) in quotas.items():
                eq = store.get("elasticquotas", ns, f"eq-{ns}")
                if eq["spec"]["min"]["memory"] != str(mn):
                    eq["spec"]["min"]["memory"] = str(mn)
                    store.update("elasticquotas", eq)
            s.sync_informers(50)
            got = s.plugin_call("CapacityScheduling", "dryRunPreemption", {"pod": preemptor, "runPreFilter": True})
            assert [(c["node"], sorted(c["victims"])) for c in got["candidates"]] == [("node-a", want)], (step, got)
    finally:
        s.stop()
