"""The reference's envtest integration cases, case for case, over HTTP.

test/integration/coscheduling_test.go:127-348 (9 gang cases) and
test/integration/capacity_scheduling_test.go:116-560 (7 ElasticQuota cases)
run against a real kube-apiserver + etcd with nodes as plain API objects and
no kubelet. Here the analog is the HTTP `ApiServer` over the native store plus
the remote-mode scheduler (its own store mirror, informers and REST writes).
The node shapes, pod requests, priorities (utils.go:44: 0 / 100 / 1000),
PodGroup / ElasticQuota specs and expected pod lists are the reference's. The
reference only polls that the expected pods get scheduled; these tests also
check the complement (no other pod is bound), after a settle delay, except
where the reference's own expectation admits survivors of member-wise
preemption.
"""
import time

import pytest

from flex_gpu_scheduler_amd import load_config
from flex_gpu_scheduler_amd.control import ApiServer, RestClient
from flex_gpu_scheduler_amd.control.remote import RemoteScheduler
from flex_gpu_scheduler_amd.models import make_elastic_quota, make_node, make_pod, make_pod_group
from helpers import coscheduling_config

LOW, MID, HIGH = 0, 100, 1000


def _wait(fn, timeout=20.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if fn():
            return True
        time.sleep(0.02)
    return bool(fn())


def _bound(client) -> dict[str, str]:
    pods, _ = client.list("pods")
    return {p["metadata"]["name"]: p["spec"].get("nodeName", "") for p in pods}


@pytest.fixture
def http_cluster(store):
    srv = ApiServer(store).start()
    yield RestClient(srv.url)
    srv.stop()


# ------------------------------------------------------------ coscheduling --
def cpod(name, mem, pg=None, prio=MID):
    return make_pod(name, "default", requests={"memory": str(mem)}, pod_group=pg, priority=prio)


def _seq(prefix, pg, mem, n, prio=MID):
    return [cpod(f"{prefix}-{i}", mem, pg, prio) for i in range(1, n + 1)]


def _interleave(*lists):
    out = []
    for i in range(max(len(x) for x in lists)):
        for x in lists:
            if i < len(x):
                out.append(x[i])
    return out


COSCHED_CASES = [
    ("equal priority, sequentially pg1 meet min and pg2 not meet min",
     _seq("t1-p1", "pg1-1", 50, 3) + _seq("t1-p2", "pg1-2", 100, 4),
     [("pg1-1", 3, None), ("pg1-2", 4, None)], ["t1-p1-1", "t1-p1-2", "t1-p1-3"]),
    ("equal priority, not sequentially pg1 meet min and pg2 not meet min",
     _interleave(_seq("t2-p1", "pg2-1", 50, 3), _seq("t2-p2", "pg2-2", 100, 4)),
     [("pg2-1", 3, None), ("pg2-2", 4, None)], ["t2-p1-1", "t2-p1-2", "t2-p1-3"]),
    ("equal priority, not sequentially pg1 not meet min and 3 regular pods",
     [cpod("t3-p1-1", 50, "pg3-1"), cpod("t3-p2", 100), cpod("t3-p1-2", 50, "pg3-1"), cpod("t3-p3", 100),
      cpod("t3-p1-3", 50, "pg3-1")],
     [("pg3-1", 4, None)], ["t3-p2", "t3-p3"]),
    ("different priority, sequentially pg1 meet min and pg2 meet min",
     _seq("t4-p1", "pg4-1", 100, 3) + _seq("t4-p2", "pg4-2", 50, 3, HIGH),
     [("pg4-1", 3, None), ("pg4-2", 3, None)], ["t4-p2-1", "t4-p2-2", "t4-p2-3"]),
    ("different priority, not sequentially pg1 meet min and pg2 meet min",
     _interleave(_seq("t5-p1", "pg5-1", 100, 3), _seq("t5-p2", "pg5-2", 50, 3, HIGH)),
     [("pg5-1", 3, None), ("pg5-2", 3, None)], ["t5-p2-1", "t5-p2-2", "t5-p2-3"]),
    ("different priority, not sequentially pg1 meet min and 3 regular pods",
     [cpod("t6-p1-1", 50, "pg6-1"), cpod("t6-p2", 100, prio=HIGH), cpod("t6-p1-2", 50, "pg6-1"),
      cpod("t6-p3", 100, prio=HIGH), cpod("t6-p1-3", 50, "pg6-1"), cpod("t6-p4", 100, prio=HIGH)],
     [("pg6-1", 3, None)], ["t6-p2", "t6-p3", "t6-p4"]),
    ("equal priority, not sequentially pg1 meet min and p2 p3 not meet min",
     _interleave(_seq("t7-p1", "pg7-1", 50, 3), _seq("t7-p2", "pg7-2", 100, 4), _seq("t7-p3", "pg7-3", 100, 4)),
     [("pg7-1", 3, None), ("pg7-2", 4, None), ("pg7-3", 4, None)], ["t7-p1-1", "t7-p1-2", "t7-p1-3"]),
    ("equal priority, not sequentially pg1 meet min and p2 p3 not meet min, pgs have min resources",
     _interleave(_seq("t8-p1", "pg8-1", 50, 3), _seq("t8-p2", "pg8-2", 100, 4), _seq("t8-p3", "pg8-3", 100, 4)),
     [("pg8-1", 3, "150"), ("pg8-2", 4, "400"), ("pg8-3", 4, "400")], ["t8-p1-1", "t8-p1-2", "t8-p1-3"]),
    ("equal priority, not sequentially pg1 meet min and pg2 not meet min, pgs have min resources",
     _interleave(_seq("t9-p1", "pg9-1", 50, 3), _seq("t9-p2", "pg9-2", 100, 4)),
     [("pg9-1", 3, "150"), ("pg9-2", 4, "400")], ["t9-p1-1", "t9-p1-2", "t9-p1-3"]),
]


@pytest.mark.parametrize("name,pods,groups,expected", COSCHED_CASES, ids=[c[0] for c in COSCHED_CASES])
def test_coscheduling_integration(http_cluster, name, pods, groups, expected):
    client = http_cluster
    client.create("nodes", make_node("fake-node", {"pods": "32", "memory": "300"}, labels={"node": "fake-node"}))
    rs = RemoteScheduler(client, load_config(coscheduling_config(permit_wait=10, denied=3))).start()
    try:
        for g, m, min_mem in groups:
            client.create("podgroups", make_pod_group(g, "default", m,
                                                      min_resources={"memory": min_mem} if min_mem else None))
        for p in pods:  # in the reference's creation order
            client.create("pods", p)
        assert _wait(lambda: all(_bound(client).get(n) for n in expected)), (name, _bound(client))
        if name.startswith("different priority, ") and "regular pods" not in name:
            # When the mid-priority gang is bound before the high-priority one
            # arrives, DefaultPreemption evicts only as many members as the
            # high gang needs; the survivor stays bound (member-wise
            # preemption, as upstream). The reference asserts only the
            # expected pods for these cases, so do the same.
            return
        time.sleep(0.5)
        got = sorted(n for n, node in _bound(client).items() if node)
        assert got == sorted(expected), (name, got)
    finally:
        rs.stop()


# ------------------------------------------------------ capacityscheduling --
CAP_CONFIG = {
    "apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
    "profiles": [{"schedulerName": "default-scheduler", "plugins": {
        "preFilter": {"enabled": [{"name": "CapacityScheduling"}]},
        "postFilter": {"enabled": [{"name": "CapacityScheduling"}], "disabled": [{"name": "*"}]},
        "reserve": {"enabled": [{"name": "CapacityScheduling"}]}}}],
}


def qpod(name, ns, mem, cpu_milli, prio, node=""):
    """test/util/utils.go:92-103 MakePod(name, ns, memReq, cpuReq(milli), priority, uid, nodeName)."""
    return make_pod(name, ns, requests={"memory": str(mem), "cpu": f"{cpu_milli}m"}, priority=prio, uid=name,
                    node_name=node or None)


def eq(name, ns, min_mem, min_cpu_m, max_mem, max_cpu_m):
    return make_elastic_quota(name, ns, min={"memory": str(min_mem), "cpu": f"{min_cpu_m}m"},
                              max={"memory": str(max_mem), "cpu": f"{max_cpu_m}m"})


STD_EQS = [eq("eq1", "ns1", 100, 100, 200, 200), eq("eq2", "ns2", 100, 100, 200, 200)]

CAP_CASES = [
    ("cross-namespace preemption",
     [qpod("t1-p1", "ns1", 50, 10, MID, "fake-node-1"), qpod("t1-p2", "ns1", 50, 10, MID, "fake-node-1"),
      qpod("t1-p3", "ns1", 50, 10, LOW, "fake-node-2")],
     [qpod("t1-p4", "ns2", 50, 10, MID), qpod("t1-p5", "ns2", 50, 10, MID), qpod("t1-p6", "ns2", 50, 10, LOW)],
     STD_EQS, ["t1-p1", "t1-p2", "t1-p4", "t1-p5"]),
    ("in-namespace preemption",
     [qpod("t2-p1", "ns1", 50, 10, MID, "fake-node-1"), qpod("t2-p2", "ns1", 50, 10, LOW, "fake-node-1"),
      qpod("t2-p3", "ns2", 50, 10, MID, "fake-node-2"), qpod("t2-p4", "ns2", 50, 10, LOW, "fake-node-2")],
     [qpod("t2-p5", "ns1", 50, 10, MID), qpod("t2-p6", "ns2", 50, 10, MID)],
     STD_EQS, ["t2-p1", "t2-p3", "t2-p5", "t2-p6"]),
    ("regular preemption without Elastic Quota",
     [qpod("t3-p1", "ns1", 50, 10, HIGH, "fake-node-1"), qpod("t3-p2", "ns1", 50, 10, LOW, "fake-node-1"),
      qpod("t3-p3", "ns2", 50, 10, HIGH, "fake-node-2"), qpod("t3-p4", "ns2", 50, 10, LOW, "fake-node-2")],
     [qpod("t3-p5", "ns1", 50, 10, MID), qpod("t3-p6", "ns2", 50, 10, MID)],
     [], ["t3-p1", "t3-p3", "t3-p5", "t3-p6"]),
    ("in-namespace preemption failed because it can't find node which is suitable for preemption",
     [qpod("t4-p1", "ns1", 50, 10, MID, "fake-node-1"), qpod("t4-p2", "ns1", 50, 10, MID, "fake-node-1"),
      qpod("t4-p3", "ns1", 50, 10, LOW, "fake-node-2"), qpod("t4-p4", "ns2", 50, 10, MID, "fake-node-2")],
     [qpod("t4-p5", "ns1", 150, 10, HIGH), qpod("t4-p6", "ns2", 150, 10, HIGH)],
     STD_EQS, ["t4-p1", "t4-p2", "t4-p3", "t4-p4"]),
    ("pod subjects to overused quota can't preempt pods subjects to other quotas",
     [qpod("t5-p1", "ns1", 50, 10, MID, "fake-node-1"), qpod("t5-p2", "ns2", 50, 10, HIGH, "fake-node-1"),
      qpod("t5-p3", "ns2", 50, 10, HIGH, "fake-node-2"), qpod("t5-p4", "ns2", 50, 10, HIGH, "fake-node-2")],
     [qpod("t5-p5", "ns2", 50, 10, HIGH)],
     STD_EQS, ["t5-p1", "t5-p2", "t5-p3", "t5-p4"]),
    ("cross-node preemption isn't supported",
     [qpod("t6-p1", "ns1", 50, 10, LOW, "fake-node-1"), qpod("t6-p2", "ns1", 50, 10, LOW, "fake-node-2"),
      qpod("t6-p3", "ns2", 50, 10, MID, "fake-node-1"), qpod("t6-p4", "ns2", 50, 10, MID, "fake-node-2")],
     [qpod("t6-p5", "ns1", 100, 20, HIGH), qpod("t6-p6", "ns2", 100, 20, HIGH)],
     STD_EQS, ["t6-p1", "t6-p2", "t6-p3", "t6-p4"]),
    ("cross-namespace preemption with three elasticquota",
     [qpod("t7-p1", "ns1", 0, 1, HIGH, "fake-node-1"), qpod("t7-p2", "ns1", 0, 1, MID, "fake-node-2"),
      qpod("t7-p3", "ns1", 0, 1, MID, "fake-node-2"), qpod("t7-p5", "ns2", 0, 1, MID, "fake-node-2"),
      qpod("t7-p6", "ns2", 0, 1, MID, "fake-node-1"), qpod("t7-p7", "ns2", 0, 1, MID, "fake-node-2")],
     [qpod(f"t7-p{i}", "ns3", 0, 1, MID) for i in (9, 10, 11, 12)],
     [eq("eq1", "ns1", 100, 1, 200, 3), eq("eq2", "ns2", 100, 3, 200, 3), eq("eq3", "ns3", 100, 3, 200, 4)],
     ["t7-p1", "t7-p5", "t7-p6", "t7-p7", "t7-p9", "t7-p10", "t7-p11"]),
]


@pytest.mark.parametrize("name,exist,add,eqs,expected", CAP_CASES, ids=[c[0] for c in CAP_CASES])
def test_capacity_scheduling_integration(http_cluster, name, exist, add, eqs, expected):
    client = http_cluster
    for n in ("fake-node-1", "fake-node-2"):
        client.create("nodes", make_node(n, {"pods": "32", "memory": "100", "cpu": "100"}, labels={"node": n}))
    rs = RemoteScheduler(client, load_config(CAP_CONFIG)).start()
    try:
        for q in eqs:
            client.create("elasticquotas", q)
        # Quotas and pods come on separate watches; let the quota informer
        # sync first, as the reference's test waits for its informers.
        assert _wait(lambda: rs.scheduler.lister_counts()["elasticquotas"] >= len(eqs), 10)
        for p in exist:
            client.create("pods", p)
        assert _wait(lambda: all(_bound(client).get(p["metadata"]["name"]) for p in exist), 10)
        # The existing pods are created already bound; make sure the
        # scheduler's informers (quota usage, node accounting) have them
        # before the contenders arrive.
        assert _wait(lambda: rs.scheduler.cache_counts()["pods"] >= len(exist), 10)
        for p in add:
            client.create("pods", p)
        # Preemption re-schedules after the preemptor's backoff (1 s initial).
        assert _wait(lambda: all(_bound(client).get(n) for n in expected), 20), (name, _bound(client))
        time.sleep(1.5)
        got = sorted(n for n, node in _bound(client).items() if node)
        assert got == sorted(expected), (name, got)
    finally:
        rs.stop()
