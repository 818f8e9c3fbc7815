"""Gang parking (Coscheduling transientShortage=Park, docs/ARCHITECTURE.md §4).

The reference denies a PodGroup for deniedPGExpirationTimeSeconds when one of
its members cannot be placed (pkg/coscheduling/coscheduling.go:140-176, 224-237).
When the shortfall is only GPUs that other gangs hold right now, this framework
parks the group instead and re-probes it on the next release of capacity, so the
gang is admitted as soon as its GPUs are free rather than after the TTL. Groups
that can never fit, and the "Deny" mode, keep the reference's behaviour."""
import time

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.models import GPU, make_pod, make_pod_group, mi355x_node
from flex_gpu_scheduler_amd.utils.workload import flagship_config


def gang(name, size, ns="default"):
    return (make_pod_group(name, ns, size),
            [make_pod(f"{name}-r{r}", ns, limits={GPU: "1"}, pod_group=name) for r in range(size)])


def submit(store, name, size):
    pg, pods = gang(name, size)
    store.create("podgroups", pg)
    for p in pods:
        store.create("pods", p)
    return [p["metadata"]["name"] for p in pods]


def bound(store, names):
    return [n for n in names if store.get("pods", "default", n)["spec"].get("nodeName")]


def wait_for(pred, timeout=10.0):
    t0 = time.time()
    while not pred():
        if time.time() - t0 > timeout:
            return False
        time.sleep(0.002)
    return True


def scheduler(store, mode="Park", denied_s=20):
    s = new_scheduler(store, load_config(flagship_config(permit_wait_s=10, denied_s=denied_s, transient_shortage=mode)),
                      podInitialBackoffSeconds=1, podMaxBackoffSeconds=10)
    s.start()
    return s


def delete_all(store, names):
    for n in names:
        store.delete("pods", "default", n)


def test_gang_parks_while_gpus_are_held_and_binds_on_release(store):
    store.create("nodes", mi355x_node("mi-0", mode="spx"))
    s = scheduler(store)
    try:
        a = submit(store, "a", 8)
        assert wait_for(lambda: len(bound(store, a)) == 8)
        b = submit(store, "b", 4)
        assert wait_for(lambda: s.gang_parks() >= 1)
        assert bound(store, b) == []
        assert s.gang_denials()[0] == 0  # parked, not denied
        t0 = time.time()
        delete_all(store, a)
        # Admitted on the release, far inside the 20 s denial TTL and the 1 s
        # pod backoff.
        assert wait_for(lambda: len(bound(store, b)) == 4, timeout=5.0)
        assert time.time() - t0 < 0.9
        assert s.gang_denials()[0] == 0
        park = s.plugin_call("Coscheduling", "parking", {"pod": store.get("pods", "default", b[0])})
        assert park["parked"] == [] and park["outstandingGpus"] == 0
    finally:
        s.stop()


def test_deny_mode_keeps_the_reference_ttl(store):
    store.create("nodes", mi355x_node("mi-0", mode="spx"))
    s = scheduler(store, mode="Deny", denied_s=20)
    try:
        a = submit(store, "a", 8)
        assert wait_for(lambda: len(bound(store, a)) == 8)
        b = submit(store, "b", 4)
        assert wait_for(lambda: s.gang_denials()[0] >= 1)
        delete_all(store, a)
        time.sleep(1.5)
        assert bound(store, b) == []  # still denied
        assert s.gang_parks() == 0
    finally:
        s.stop()


def test_group_bigger_than_the_cluster_is_denied_not_parked(store):
    store.create("nodes", mi355x_node("mi-0", mode="spx"))
    s = scheduler(store)
    try:
        big = submit(store, "big", 12)
        assert wait_for(lambda: s.gang_denials()[0] >= 1)
        assert s.gang_parks() == 0 and bound(store, big) == []
    finally:
        s.stop()


def test_oldest_parked_gang_goes_first(store):
    """The oldest parked group holds a reservation: younger small gangs do not
    take the GPUs it waits for (no starvation of 8-rank gangs)."""
    store.create("nodes", mi355x_node("mi-0", mode="spx"))
    s = scheduler(store)
    try:
        a = submit(store, "a", 8)
        assert wait_for(lambda: len(bound(store, a)) == 8)
        b = submit(store, "b", 8)
        assert wait_for(lambda: s.gang_parks() >= 1)
        time.sleep(1.1)  # a later creation second: younger in the queue order
        small = [submit(store, f"c{i}", 1)[0] for i in range(3)]
        assert wait_for(lambda: s.gang_parks() >= 4)
        delete_all(store, a)
        assert wait_for(lambda: len(bound(store, b)) == 8, timeout=5.0)
        assert bound(store, small) == []
        delete_all(store, b)
        assert wait_for(lambda: len(bound(store, small)) == 3, timeout=5.0)
        assert s.gang_denials()[0] == 0
    finally:
        s.stop()


def test_parking_mode_is_validated():
    import pytest

    from flex_gpu_scheduler_amd.config import ConfigError

    with pytest.raises(ConfigError):
        load_config(flagship_config(transient_shortage="Sometimes"))


def _parking(s, pod):
    return s.plugin_call("Coscheduling", "parking", {"pod": pod})


def test_group_deleted_at_permit_owes_no_gpus(store):
    """A gang deleted while a member waits at Permit (the PodGroup gone before
    the members' deletions reach Unreserve) leaves nothing owed: GPUs owed to
    a gang that no longer exists would hold every later gang's gate shut until
    the 15-min sweep."""
    store.create("nodes", mi355x_node("mi-0", mode="spx"))
    pg, pods = gang("g", 4)
    store.create("podgroups", pg)
    for p in pods:
        store.create("pods", p)
    s = new_scheduler(store, load_config(flagship_config(permit_wait_s=10, transient_shortage="Park")))
    try:
        s.sync_informers(50)
        assert s.schedule_one(2000)  # r0 waits at Permit: 3 more GPUs owed to the gang
        probe = store.get("pods", "default", "g-r1")
        assert _parking(s, probe)["outstandingGpus"] == 3
        store.delete("podgroups", "default", "g")
        s.sync_informers(50)
        for p in pods:
            store.delete("pods", "default", p["metadata"]["name"])
        s.sync_informers(50)
        assert wait_for(lambda: _parking(s, probe)["outstandingGpus"] == 0, timeout=5.0), _parking(s, probe)
    finally:
        s.stop()


def test_deleted_parked_group_leaves_the_line(store):
    """A parked group that is deleted leaves the parked list at once (it would
    otherwise reserve its need against every younger gang until a probe)."""
    store.create("nodes", mi355x_node("mi-0", mode="spx"))
    s = scheduler(store)
    try:
        a = submit(store, "a", 8)
        assert wait_for(lambda: len(bound(store, a)) == 8)
        b = submit(store, "b", 4)
        assert wait_for(lambda: s.gang_parks() >= 1)
        probe = store.get("pods", "default", b[0])
        assert [g["podGroup"] for g in _parking(s, probe)["parked"]] == ["default/b"]
        time.sleep(1.1)  # a later creation second: c queues behind b
        c = submit(store, "c", 2)
        assert wait_for(lambda: len(_parking(s, probe)["parked"]) == 2)
        # b (the head of the line) leaves: c is probed from the informer's
        # event (it finds the GPUs still held and parks again).
        store.delete("podgroups", "default", "b")
        delete_all(store, b)
        assert wait_for(lambda: [g["podGroup"] for g in _parking(s, probe)["parked"]] == ["default/c"],
                        timeout=5.0), _parking(s, probe)
        assert _parking(s, probe)["outstandingGpus"] == 0
        store.delete("podgroups", "default", "c")
        delete_all(store, c)
        assert wait_for(lambda: _parking(s, probe)["parked"] == [], timeout=5.0), _parking(s, probe)
    finally:
        s.stop()


def test_parked_head_that_lost_a_member_does_not_block_younger_gangs(store):
    """A parked head-of-line gang that loses a pod (the PodGroup kept) can no
    longer pass the gate; it must leave the line instead of reserving its need
    against every younger gang forever."""
    store.create("nodes", mi355x_node("mi-0", mode="spx"))
    s = scheduler(store)
    try:
        a = submit(store, "a", 8)
        assert wait_for(lambda: len(bound(store, a)) == 8)
        b = submit(store, "b", 8)
        assert wait_for(lambda: s.gang_parks() >= 1)
        time.sleep(1.1)  # younger than b in the queue order
        c = submit(store, "c", 2)
        assert wait_for(lambda: s.gang_parks() >= 2)
        store.delete("pods", "default", b[-1])  # b now has 7 pods for minMember 8
        time.sleep(0.1)
        delete_all(store, a)
        assert wait_for(lambda: len(bound(store, c)) == 2, timeout=5.0), _parking(s, store.get("pods", "default", c[0]))
        assert bound(store, b[:-1]) == []
        assert [g["podGroup"] for g in _parking(s, store.get("pods", "default", c[0]))["parked"]] == []
    finally:
        s.stop()


def test_xcd_gang_is_probed_apart_from_a_parked_whole_gpu_gang(store):
    """Parked whole-GPU and XCD gangs are probed per kind:
    an XCD gang parked behind an oversized whole-GPU gang is admitted as soon
    as CPX partitions are released, not at the 60 s unschedulable flush."""
    from flex_gpu_scheduler_amd.models.mi355x import GPU_XCD

    store.create("nodes", mi355x_node("mi-0", mode="spx"))
    store.create("nodes", mi355x_node("cpx-0", mode="cpx"))
    s = scheduler(store)
    try:
        a = submit(store, "a", 8)
        assert wait_for(lambda: len(bound(store, a)) == 8)
        b = submit(store, "b", 8)  # whole GPUs: parks at the head of the line
        assert wait_for(lambda: s.gang_parks() >= 1)
        time.sleep(1.1)

        def xgang(name):
            store.create("podgroups", make_pod_group(name, "default", 4))
            names = [f"{name}-r{r}" for r in range(4)]
            for n in names:
                store.create("pods", make_pod(n, limits={GPU_XCD: "2"}, pod_group=name))
            return names

        fill = [xgang(f"f{i}") for i in range(8)]  # 8 x 4 x 2 XCDs = the 64 XCDs of cpx-0
        assert wait_for(lambda: all(len(bound(store, f)) == 4 for f in fill))
        q = xgang("q")
        assert wait_for(lambda: s.gang_parks() >= 2)
        t0 = time.time()
        delete_all(store, fill[0])
        assert wait_for(lambda: len(bound(store, q)) == 4, timeout=5.0)
        assert time.time() - t0 < 2.0
        assert bound(store, b) == []
    finally:
        s.stop()


def test_parked_member_whose_spec_changes_is_retried(store):
    """A parked gang member whose spec is updated gets another attempt at once
    (upstream Update moves an updated unschedulable pod)
    instead of waiting for its gang's next probe or the 60 s flush. It still
    serves its backoff (upstream: backoffQ while backing off), which grows
    with the attempts the member happened to get before its gang parked; the
    short backoff here keeps that under the wait below."""
    store.create("nodes", mi355x_node("mi-0", mode="spx"))
    s = new_scheduler(store, load_config(flagship_config(permit_wait_s=10, denied_s=20, transient_shortage="Park")),
                      podInitialBackoffSeconds=0.05, podMaxBackoffSeconds=0.5)
    s.start()
    try:
        a = submit(store, "a", 8)
        assert wait_for(lambda: len(bound(store, a)) == 8)
        b = submit(store, "b", 4)
        assert wait_for(lambda: s.queue_counts()["parked"] == 4)
        before = s.stats()["attempts"]
        time.sleep(0.2)
        assert s.stats()["attempts"] == before  # parked: no cycles
        pod = store.get("pods", "default", b[0])
        pod["spec"]["containers"][0]["resources"]["requests"] = {"cpu": "2"}
        store.update("pods", pod)
        assert wait_for(lambda: s.stats()["attempts"] > before, timeout=3.0)
        assert wait_for(lambda: s.queue_counts()["parked"] == 4, timeout=3.0)  # parked again: GPUs still held
        assert bound(store, b) == []
    finally:
        s.stop()
