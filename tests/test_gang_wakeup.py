"""Lost gang wake-up: a PodGroup member that is mid-cycle when Coscheduling's
denied-group requeue timer fires must not park in unschedulableQ until the
60 s flush.

The scheduler runs on a FakeClock with no scheduling loop (``schedule_one``
drives each cycle), and an HTTP filter extender holds the member inside its
scheduling cycle, so the interleaving is exact, not timing-dependent:

1. the gang is denied (extender rejects every node -> Coscheduling PostFilter
   rejects and denies the group, coscheduling.go:140-176) and the denied-group
   timer is armed;
2. the clock passes the denial TTL (not yet the timer's deadline, TTL + 1 ms);
   member ``a`` starts a cycle and blocks in
   the extender's filter call;
3. the timer fires (``run_timers``) and activates the group: ``a`` is in
   flight, so the queue can only mark it;
4. the extender fails ``a``'s cycle with an error: the failure handler must
   send ``a`` to activeQ because of the mark (upstream pairs
   AddUnschedulableIfNotPresent with moveRequestCycle for this race,
   vendor/k8s.io/kubernetes/pkg/scheduler/internal/queue/scheduling_queue.go:376-400);
5. both members then schedule and bind with no clock advance at all.
"""
import threading
import time

from flex_gpu_scheduler_amd import FakeClock, load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_node, make_pod, make_pod_group
from helpers import coscheduling_config, placements, wait_bound
from test_extenders import FakeExtender


class GatedExtender(FakeExtender):
    """Filter verb modes: "reject" (all nodes fail), "gate" (block until
    released, then return an extender error), "pass"."""

    def __init__(self):
        super().__init__()
        self.mode = "pass"
        self.entered = threading.Event()
        self.release = threading.Event()

    def handle(self, verb, body):
        if verb == "filter" and self.mode == "reject":
            self.reject = {n: "no room" for n in self.names(body)}
        elif verb == "filter" and self.mode == "gate":
            self.entered.set()
            assert self.release.wait(30)
            return {"Error": "extender backend restarted"}
        else:
            self.reject = {}
        return super().handle(verb, body)


def test_member_in_flight_when_denied_group_timer_fires_is_requeued():
    from flex_gpu_scheduler_amd import Store
    store = Store()
    ext = GatedExtender()
    clock = FakeClock()
    store.create("nodes", make_node("n0", {"pods": "32", "memory": "300", "cpu": "8"}))
    store.create("podgroups", make_pod_group("pg", "default", 2))
    for n in ("a", "b"):
        store.create("pods", make_pod(n, requests={"memory": "10"}, pod_group="pg"))
    cfg = coscheduling_config(denied=3)
    cfg["apiVersion"] = "kubescheduler.config.k8s.io/v1beta3"
    cfg["extenders"] = [{"urlPrefix": ext.url, "filterVerb": "filter"}]
    s = new_scheduler(store, load_config(cfg), clock=clock)
    try:
        s.sync_informers(20)
        # 1. deny the group: a fails on the extender, b on the denial.
        ext.mode = "reject"
        assert s.schedule_one(2000) and s.schedule_one(2000)
        q = s.queue_counts()
        assert q["unschedulable"] == 2 and q["active"] == 0, q
        # 2. past the TTL (3 s) but short of the requeue timer's deadline
        # (TTL + 1 ms): the timer thread polls the FakeClock on its own, so it
        # must not be due before `a` is in flight.
        clock.advance(3.0005)
        s.move_all()
        assert s.queue_counts()["active"] == 2
        ext.mode = "gate"
        t = threading.Thread(target=s.schedule_one, args=(10000,))
        t.start()
        assert ext.entered.wait(10)
        # 3. the denied-group timer fires while `a` is in its scheduling cycle.
        clock.advance(0.001)
        s.run_timers()
        q = s.queue_counts()
        assert q["in_flight"] == 1 and q["activation_marks"] == 1, q
        # 4. a's cycle fails: the mark sends it back to activeQ.
        ext.mode = "pass"
        ext.release.set()
        t.join(10)
        assert not t.is_alive()
        q = s.queue_counts()
        assert q["unschedulable"] == 0 and q["active"] == 2 and q["activation_marks"] == 0, q
        # 5. both members bind; the FakeClock never reaches the 60 s flush.
        assert s.schedule_one(2000) and s.schedule_one(2000)
        wait_bound(s, 2, timeout=10)
        assert placements(store) == {"a": "n0", "b": "n0"}
        s.sync_informers(20)  # the assigned-pod events end the in-flight entries
        assert s.queue_counts()["in_flight"] == 0
    finally:
        s.stop()
        ext.close()


def test_activation_marks_do_not_outlive_bound_pods(store):
    """Siblings activated from Permit while they wait in their own binding
    cycle carry marks; binding clears them (no growth across gangs)."""
    from helpers import start
    store.create("nodes", make_node("n0", {"pods": "110", "memory": "3000", "cpu": "64"}))
    s = start(store, coscheduling_config())
    try:
        for g in range(20):
            store.create("podgroups", make_pod_group(f"g{g}", "default", 4))
            for i in range(4):
                store.create("pods", make_pod(f"g{g}-{i}", requests={"memory": "10"}, pod_group=f"g{g}"))
        wait_bound(s, 80)
        t0 = time.time()
        while s.queue_counts()["in_flight"] and time.time() - t0 < 5:
            time.sleep(0.01)
        q = s.queue_counts()
        assert q["in_flight"] == 0 and q["activation_marks"] == 0, q
    finally:
        s.stop()


def test_marked_member_retries_once_then_parks():
    """Retry cadence of the in-flight activation mark (a deliberate deviation,
    docs/STATUS.md): a member activated while in its cycle goes straight back
    to activeQ when that cycle fails -- once. Its next failure, with no new
    activation, parks it in unschedulableQ like any other; the mark does not
    turn into a retry loop while the group keeps failing."""
    from flex_gpu_scheduler_amd import Store
    store = Store()
    ext = GatedExtender()
    clock = FakeClock()
    store.create("nodes", make_node("n0", {"pods": "32", "memory": "300", "cpu": "8"}))
    store.create("podgroups", make_pod_group("pg", "default", 2))
    for n in ("a", "b"):
        store.create("pods", make_pod(n, requests={"memory": "10"}, pod_group="pg"))
    cfg = coscheduling_config(denied=3)
    cfg["apiVersion"] = "kubescheduler.config.k8s.io/v1beta3"
    cfg["extenders"] = [{"urlPrefix": ext.url, "filterVerb": "filter"}]
    s = new_scheduler(store, load_config(cfg), clock=clock)
    try:
        s.sync_informers(20)
        ext.mode = "reject"
        assert s.schedule_one(2000) and s.schedule_one(2000)
        clock.advance(3.0005)
        s.move_all()
        ext.mode = "gate"
        t = threading.Thread(target=s.schedule_one, args=(10000,))
        t.start()
        assert ext.entered.wait(10)
        clock.advance(0.001)
        s.run_timers()
        assert s.queue_counts()["activation_marks"] == 1
        # The marked cycle fails: one retry, straight to activeQ.
        ext.mode = "reject"
        ext.release.set()
        t.join(10)
        q = s.queue_counts()
        assert q["active"] == 2 and q["activation_marks"] == 0, q
        # Both fail again with no activation in between: they park.
        assert s.schedule_one(2000) and s.schedule_one(2000)
        q = s.queue_counts()
        assert q["active"] == 0 and q["backoff"] == 0 and q["unschedulable"] == 2, q
        assert q["activation_marks"] == 0 and q["in_flight"] == 0, q
        assert not s.schedule_one(200)  # nothing left to retry before the group's TTL
    finally:
        s.stop()
        ext.close()
