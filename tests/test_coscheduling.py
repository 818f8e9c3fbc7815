"""Gang scheduling end-to-end through the native scheduler.

Scenarios mirror the reference's envtest suite
(test/integration/coscheduling_test.go:127-348): one node with 300 units of
memory and 32 pods; PodGroups that fit (all members bound) or cannot reach
minMember (no member bound — the gang never partially starts)."""
import time

import pytest

from flex_gpu_scheduler_amd.models import make_node, make_pod, make_pod_group
from helpers import coscheduling_config, create_all, placements, start, wait_bound

MID, HIGH = 100, 200


def node():
    return make_node("fake-node", {"pods": "32", "memory": "300"}, labels={"node": "fake-node"})


def pod(name, mem, pg=None, prio=MID):
    return make_pod(name, requests={"memory": str(mem)}, pod_group=pg, priority=prio)


SCENARIOS = [
    ("equal priority, sequentially pg1 meets min, pg2 does not",
     [pod(f"t1-p1-{i}", 50, "pg1-1") for i in (1, 2, 3)] + [pod(f"t1-p2-{i}", 100, "pg1-2") for i in (1, 2, 3, 4)],
     [("pg1-1", 3), ("pg1-2", 4)], ["t1-p1-1", "t1-p1-2", "t1-p1-3"]),
    ("equal priority, interleaved pg1 meets min, pg2 does not",
     [pod("t2-p1-1", 50, "pg2-1"), pod("t2-p2-1", 100, "pg2-2"), pod("t2-p1-2", 50, "pg2-1"),
      pod("t2-p2-2", 100, "pg2-2"), pod("t2-p1-3", 50, "pg2-1"), pod("t2-p2-3", 100, "pg2-2"),
      pod("t2-p2-4", 100, "pg2-2")],
     [("pg2-1", 3), ("pg2-2", 4)], ["t2-p1-1", "t2-p1-2", "t2-p1-3"]),
    ("pg below minMember plus regular pods",
     [pod("t3-p1-1", 50, "pg3-1"), pod("t3-p2", 100), pod("t3-p1-2", 50, "pg3-1"), pod("t3-p3", 100),
      pod("t3-p1-3", 50, "pg3-1")],
     [("pg3-1", 4)], ["t3-p2", "t3-p3"]),
    ("different priority, both groups fit",
     [pod(f"t4-p1-{i}", 100, "pg4-1") for i in (1, 2)] + [pod(f"t4-p2-{i}", 50, "pg4-2", HIGH) for i in (1, 2)],
     [("pg4-1", 2), ("pg4-2", 2)], ["t4-p1-1", "t4-p1-2", "t4-p2-1", "t4-p2-2"]),
    ("higher priority group wins the capacity",
     [pod(f"t5-p1-{i}", 100, "pg5-1") for i in (1, 2, 3)] + [pod(f"t5-p2-{i}", 100, "pg5-2", HIGH) for i in (1, 2, 3)],
     [("pg5-1", 3), ("pg5-2", 3)], ["t5-p2-1", "t5-p2-2", "t5-p2-3"]),
]


@pytest.mark.parametrize("name,pods,groups,expected", SCENARIOS, ids=[s[0] for s in SCENARIOS])
def test_gang_scenarios(store, name, pods, groups, expected):
    store.create("nodes", node())
    sched = start(store, coscheduling_config())
    try:
        create_all(store, "podgroups", [make_pod_group(g, "default", m) for g, m in groups])
        create_all(store, "pods", pods)
        wait_bound(sched, len(expected))
        # The bound counter can reach len(expected) on a group that is later
        # preempted (the higher-priority scenario), so poll the placements
        # themselves as the reference does (coscheduling_test.go:365).
        t0 = time.time()
        while True:
            time.sleep(0.3)
            got = sorted(n for n, node_ in placements(store).items() if node_)
            if got == sorted(expected) or time.time() - t0 > 20:
                break
        assert got == sorted(expected)
    finally:
        sched.stop()


def test_min_resources_prefilter_denies(store):
    store.create("nodes", node())
    sched = start(store, coscheduling_config())
    try:
        store.create("podgroups", make_pod_group("big", "default", 2, min_resources={"memory": "1000"}))
        create_all(store, "pods", [pod(f"b{i}", 10, "big") for i in range(2)])
        time.sleep(0.5)
        assert all(not n for n in placements(store).values())
        cond = store.get("pods", "default", "b0")["status"]["conditions"][0]
        assert cond["reason"] == "Unschedulable"
    finally:
        sched.stop()


def test_permit_timeout_rejects_whole_group(store):
    # Two members fit, the third cannot: the two waiting at Permit time out
    # and are rejected together (waiting_pods_map.go:100 + Unreserve).
    store.create("nodes", make_node("n", {"pods": "32", "memory": "100"}))
    sched = start(store, coscheduling_config(permit_wait=1, denied=1))
    try:
        store.create("podgroups", make_pod_group("g", "default", 3))
        create_all(store, "pods", [pod("g1", 40, "g"), pod("g2", 40, "g"), pod("g3", 40, "g")])
        time.sleep(2.5)
        assert all(not n for n in placements(store).values())
        assert sched.waiting_pods() == []
        assert sched.stats()["bound"] == 0
    finally:
        sched.stop()


def test_post_bind_patches_podgroup_phase(store):
    store.create("nodes", node())
    sched = start(store, coscheduling_config())
    try:
        store.create("podgroups", make_pod_group("pg", "default", 2))
        create_all(store, "pods", [pod("a", 10, "pg"), pod("b", 10, "pg")])
        wait_bound(sched, 2)
        t0 = time.time()
        while store.get("podgroups", "default", "pg")["status"].get("phase") not in ("Scheduling", "Scheduled"):
            assert time.time() - t0 < 5
            time.sleep(0.01)
    finally:
        sched.stop()


def test_gang_latency_records(store):
    store.create("nodes", node())
    sched = start(store, coscheduling_config())
    try:
        create_all(store, "podgroups", [make_pod_group("g4", "default", 4)])
        create_all(store, "pods", [pod(f"m{i}", 10, "g4") for i in range(4)])
        wait_bound(sched, 4)
        recs = sched.gang_records()
        assert len(recs) == 1 and recs[0]["size"] == 4
        r = recs[0]
        assert r["first_enqueue_us"] <= r["admit_us"] <= r["bound_us"]
        assert "xsched_gang_admit_seconds_bucket" in sched.metrics_text()
    finally:
        sched.stop()


def test_denied_group_retries_when_the_denial_expires(store):
    """A gang denied after all its members exist (here: a Permit timeout
    while a blocker holds the room) is requeued when the denial runs out —
    not by the 60 s unschedulable flush. Freeing the room while it is still
    denied moves it once (rejected: denied); nothing else is left to move it."""
    store.create("nodes", make_node("n", {"pods": "32", "memory": "100"}))
    store.create("pods", make_pod("blocker", requests={"memory": "40"}, node_name="n", priority=10 ** 6))
    sched = start(store, coscheduling_config(permit_wait=1, denied=2),
                  podInitialBackoffSeconds=0.05, podMaxBackoffSeconds=0.1)
    try:
        store.create("podgroups", make_pod_group("g", "default", 2))
        create_all(store, "pods", [pod("g1", 40, "g"), pod("g2", 40, "g")])
        time.sleep(1.5)  # g1 waited at Permit, timed out; the group is denied
        assert all(not n for name, n in placements(store).items() if name != "blocker")
        store.delete("pods", "default", "blocker")
        t0 = time.time()
        wait_bound(sched, 2, timeout=10.0)
        assert time.time() - t0 < 6.0
    finally:
        sched.stop()
