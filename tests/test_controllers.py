"""PodGroup / ElasticQuota controllers and leader election.

Cases mirror pkg/controller/podgroup_test.go:24-170 (phase machine table,
occupiedBy) and pkg/controller/elasticquota_test.go:45-215 (status.used from
Running pods), run against both the in-process client and the HTTP server.
"""
import threading
import time

import pytest

from flex_gpu_scheduler_amd.control import (ApiServer, ControllerManager, ElasticQuotaController, LeaderElector,
                                            LocalClient, PodGroupController, RestClient)
from flex_gpu_scheduler_amd.models import make_container, make_elastic_quota, make_pod, make_pod_group


@pytest.fixture(params=["local", "rest"])
def client(request, store):
    if request.param == "local":
        yield LocalClient(store)
        return
    srv = ApiServer(store).start()
    yield RestClient(srv.url)
    srv.stop()


def _pg(name, min_member, phase, created=None):
    pg = make_pod_group(name, min_member=min_member)
    pg["status"] = {"occupiedBy": "test", "scheduled": min_member, "scheduleStartTime": "2026-01-01T00:00:00Z",
                    "phase": phase}
    pg["metadata"]["creationTimestamp"] = created or "2026-01-01T00:00:00Z"
    return pg


def _pods(names, pg, phase, owners=None):
    out = []
    for n in names:
        p = make_pod(n, pod_group=pg)
        p["status"] = {"phase": phase}
        if owners:
            p["metadata"]["ownerReferences"] = [{"name": o, "kind": "Job", "apiVersion": "batch/v1", "uid": o}
                                                for o in owners]
        out.append(p)
    return out


def wait_for(fn, timeout=15.0):  # generous: the suite runs under xdist
    deadline = time.time() + timeout
    while time.time() < deadline:
        v = fn()
        if v:
            return v
        time.sleep(0.02)
    return fn()


PG_CASES = [
    # name, min, pods, pod phase, previous PG phase, desired, next pod phase, created
    ("running", 2, ["p1", "p2"], "Running", "Scheduled", "Running", None, None),
    ("failed", 2, ["p1", "p2"], "Failed", "Scheduled", "Failed", None, None),
    ("finished", 2, ["p1", "p2"], "Succeeded", "Scheduled", "Finished", None, None),
    ("scheduling->scheduled", 2, ["p1", "p2"], "Pending", "Scheduling", "Scheduled", None, None),
    ("scheduling->finished", 2, ["p1", "p2"], "Pending", "Scheduling", "Finished", "Succeeded", None),
    ("pending->...->finished", 2, ["p1", "p2"], "Pending", "Pending", "Finished", "Succeeded", None),
    ("not enqueued: scheduling started >48h after creation", 2, ["p1", "p2"], "Running", "Pending", "Pending", None,
     "2025-12-01T00:00:00Z"),
    ("min member above pod count", 3, ["p1", "p2"], "Pending", "Pending", "Pending", None, None),
    ("running->pending without pods", 2, [], "Pending", "Running", "Pending", None, None),
]


@pytest.mark.parametrize("case", PG_CASES, ids=[c[0] for c in PG_CASES])
def test_podgroup_phase_machine(store, client, case):
    _, min_member, names, pod_phase, prev, desired, next_phase, created = case
    store.create("podgroups", _pg("pg", min_member, prev, created))
    for p in _pods(names, "pg", pod_phase):
        store.create("pods", p)
    ctrl = PodGroupController(client).run()
    try:
        if next_phase:
            for n in names:
                store.patch("pods", "default", n, {"status": {"phase": next_phase}})
        got = wait_for(lambda: (store.get("podgroups", "default", "pg")["status"]["phase"] == desired) or None)
        assert store.get("podgroups", "default", "pg")["status"]["phase"] == desired, got
        if desired == "Running" and prev == "Scheduled":
            st = store.get("podgroups", "default", "pg")["status"]
            assert st["running"] == 2 and st["failed"] == 0 and st["succeeded"] == 0
    finally:
        ctrl.stop()
        ctrl.factory.stop()


@pytest.mark.parametrize("owners,want", [(["new-occupied"], "default/new-occupied"),
                                         (["new-occupied-2", "new-occupied-1"],
                                          "default/new-occupied-1,default/new-occupied-2")])
def test_podgroup_occupied_by(store, client, owners, want):
    store.create("podgroups", _pg("pg", 2, "Pending"))
    for p in _pods(["p1", "p2"], "pg", "Pending", owners):
        store.create("pods", p)
    ctrl = PodGroupController(client).run()
    try:
        assert wait_for(lambda: store.get("podgroups", "default", "pg")["status"].get("occupiedBy") == want)
        assert store.get("podgroups", "default", "pg")["status"]["phase"] == "PreScheduling"
    finally:
        ctrl.stop()
        ctrl.factory.stop()


def test_podgroup_occupied_filled_when_empty(store):
    """Appendix C6 fix: the reference never initialises an empty occupiedBy."""
    pg = _pg("pg", 2, "Pending")
    pg["status"].pop("occupiedBy")
    store.create("podgroups", pg)
    for p in _pods(["p1", "p2"], "pg", "Pending", ["job-a"]):
        store.create("pods", p)
    ctrl = PodGroupController(LocalClient(store)).run()
    try:
        assert wait_for(lambda: store.get("podgroups", "default", "pg")["status"].get("occupiedBy") == "default/job-a")
    finally:
        ctrl.stop()
        ctrl.factory.stop()


def test_podgroup_pods_are_namespaced(store):
    """Appendix C6 fix: a same-named group in another namespace does not count."""
    store.create("podgroups", _pg("pg", 2, "Pending"))
    for n in ("p1", "p2"):
        store.create("pods", make_pod(n, "other", pod_group="pg"))
    ctrl = PodGroupController(LocalClient(store)).run()
    try:
        time.sleep(0.3)
        assert ctrl.wait_idle()
        assert store.get("podgroups", "default", "pg")["status"]["phase"] == "Pending"
    finally:
        ctrl.stop()
        ctrl.factory.stop()


def _rl(cpu, mem, gpu=None):
    d = {"cpu": str(cpu), "memory": f"{mem}Gi"}
    if gpu is not None:
        d["amd.com/gpu"] = str(gpu)
    return d


def _pod(ns, name, phase, containers, inits=()):
    p = make_pod(name, ns, containers=[make_container(f"c{i}", requests=r) for i, r in enumerate(containers)],
                 init_containers=[make_container(f"i{i}", requests=r) for i, r in enumerate(inits)] or None)
    p["status"] = {"phase": phase}
    return p


def _used(store, ns, name):
    return (store.get("elasticquotas", ns, name).get("status") or {}).get("used")


def _eq_norm(d):
    from flex_gpu_scheduler_amd._native import native
    return {k: native().parse_quantity(v)[0] for k, v in (d or {}).items()}


EQ_CASES = [
    ("no init containers",
     [("t1", "eq1", _rl(3, 5), _rl(5, 15, 1))],
     [_pod("t1", "pod1", "Running", [_rl(1, 2, 1)])],
     {("t1", "eq1"): _rl(1, 2, 1)}),
    ("init containers",
     [("t2", "eq1", _rl(3, 5), _rl(5, 15))],
     [_pod("t2", "pod1", "Running", [_rl(1, 2), _rl(1, 2)]),
      _pod("t2", "pod2", "Running", [_rl(2, 1), _rl(1, 1)], [_rl(2, 1), _rl(2, 3)])],
     {("t2", "eq1"): _rl(5, 7)}),
    ("pending pods do not count; pods only count in their namespace",
     [("t3", "eq1", _rl(3, 5), _rl(5, 15)), ("t3b", "eq2", _rl(3, 5), _rl(5, 15))],
     [_pod("t3", "pod1", "Pending", [_rl(2, 1), _rl(1, 1)], [_rl(2, 1), _rl(2, 3)]),
      _pod("t3b", "pod2", "Running", [_rl(3, 1), _rl(1, 1)], [_rl(2, 1), _rl(2, 3)])],
     {("t3", "eq1"): _rl(0, 0), ("t3b", "eq2"): _rl(4, 3)}),
    ("min and max with different fields",
     [("t5", "eq1", _rl(3, 5, 2), _rl(5, 15))], [],
     {("t5", "eq1"): _rl(0, 0, 0)}),
]


@pytest.mark.parametrize("case", EQ_CASES, ids=[c[0] for c in EQ_CASES])
def test_elasticquota_used(store, client, case):
    _, eqs, pods, want = case
    for ns, name, mn, mx in eqs:
        store.create("elasticquotas", make_elastic_quota(name, ns, min=mn, max=mx))
    for p in pods:
        store.create("pods", p)
    ctrl = ElasticQuotaController(client).run()
    try:
        for (ns, name), w in want.items():
            assert wait_for(lambda: _eq_norm(_used(store, ns, name)) == _eq_norm(w)), (_used(store, ns, name), w)
        # The Synced event is recorded after the status patch lands.
        assert wait_for(lambda: any(e["reason"] == "Synced" for e in store.list("events", "")[0]))
    finally:
        ctrl.stop()
        ctrl.factory.stop()


def test_elasticquota_tracks_pod_transitions(store):
    store.create("elasticquotas", make_elastic_quota("eq", "ns", min=_rl(4, 8, 4), max=_rl(8, 16, 8)))
    store.create("pods", _pod("ns", "a", "Pending", [_rl(1, 1, 2)]))
    ctrl = ElasticQuotaController(LocalClient(store), record_events=False).run()
    try:
        assert wait_for(lambda: _eq_norm(_used(store, "ns", "eq")) == _eq_norm(_rl(0, 0, 0)))
        store.patch("pods", "ns", "a", {"status": {"phase": "Running"}})
        assert wait_for(lambda: _eq_norm(_used(store, "ns", "eq")) == _eq_norm(_rl(1, 1, 2)))
        store.delete("pods", "ns", "a")
        assert wait_for(lambda: _eq_norm(_used(store, "ns", "eq")) == _eq_norm(_rl(0, 0, 0)))
    finally:
        ctrl.stop()
        ctrl.factory.stop()


def test_controller_manager_end_to_end(store):
    mgr = ControllerManager(LocalClient(store)).run()
    try:
        store.create("podgroups", make_pod_group("g", min_member=2))
        assert wait_for(lambda: (store.get("podgroups", "default", "g").get("status") or {}).get("phase") == "Pending")
        for n in ("a", "b"):
            store.create("pods", make_pod(n, pod_group="g"))
        assert wait_for(lambda: store.get("podgroups", "default", "g")["status"]["phase"] == "PreScheduling")
        assert mgr.wait_idle()
    finally:
        mgr.stop()


def test_leader_election_single_holder_and_failover(store):
    c = LocalClient(store)
    started = []
    a = LeaderElector(c, "sched-plugins-controller", "kube-system", "a", lease_duration=0.6, renew_deadline=0.4,
                      retry_period=0.1, on_started_leading=lambda: started.append("a"))
    b = LeaderElector(c, "sched-plugins-controller", "kube-system", "b", lease_duration=0.6, renew_deadline=0.4,
                      retry_period=0.1, on_started_leading=lambda: started.append("b"))
    ta = threading.Thread(target=a.run, daemon=True)
    ta.start()
    assert a.is_leader.wait(2)
    tb = threading.Thread(target=b.run, daemon=True)
    tb.start()
    time.sleep(0.8)
    assert not b.is_leader.is_set() and b.leader == "a"
    a.stop()          # releases the lease on the way out
    ta.join(2)
    assert b.is_leader.wait(3)
    lease = store.get("leases", "kube-system", "sched-plugins-controller")
    assert lease["spec"]["holderIdentity"] == "b" and lease["spec"]["leaseTransitions"] >= 1
    b.stop()
    tb.join(2)
    assert started == ["a", "b"]
