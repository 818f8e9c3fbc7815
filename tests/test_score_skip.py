"""All-zero Score skip (framework.cc run_score_plugins): TaintToleration is
skipped while no node carries a PreferNoSchedule taint (Snapshot index
recounted on node-epoch changes), ImageLocality while none of the pod's
images is on any node. These tests pin that the skip never hides a real
preference on the scheduling path (explain() always runs every plugin, so
it cannot cover this)."""
import time

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_node, make_pod

from helpers import placements


def node(name, images=None, taints=None):
    n = make_node(name, {"cpu": "32", "memory": "64Gi", "pods": "110"})
    if images:
        n["status"]["images"] = [{"names": [i], "sizeBytes": s} for i, s in images.items()]
    if taints:
        n["spec"]["taints"] = taints
    return n


def wait_placed(store, name, timeout=15.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        host = placements(store).get(name, "")
        if host:
            return host
        time.sleep(0.01)
    raise AssertionError(f"{name} not bound: {placements(store)}")


def test_prefer_no_schedule_taint_added_later_is_scored(store):
    store.create("nodes", node("a"))
    store.create("nodes", node("b"))
    s = new_scheduler(store, load_config(None))
    s.sync_informers(50)
    s.start()
    try:
        store.create("pods", make_pod("p0"))
        first = wait_placed(store, "p0")
        other = "b" if first == "a" else "a"
        # The empty node now gets a PreferNoSchedule taint; the next pod must
        # follow the taint (a stale skip would let LeastAllocated pick it).
        store.patch("nodes", "", other, {"spec": {"taints": [{"key": "soft", "effect": "PreferNoSchedule"}]}})
        time.sleep(0.3)
        for i in range(1, 4):
            store.create("pods", make_pod(f"p{i}"))
            assert wait_placed(store, f"p{i}") == first
    finally:
        s.stop()


def test_tolerated_prefer_no_schedule_taint(store):
    taint = [{"key": "soft", "effect": "PreferNoSchedule"}]
    store.create("nodes", node("t1", taints=taint))
    store.create("nodes", node("t2", taints=taint))
    store.create("nodes", node("clean"))
    s = new_scheduler(store, load_config(None))
    s.sync_informers(50)
    s.start()
    try:
        store.create("pods", make_pod("p"))
        assert wait_placed(store, "p") == "clean"
    finally:
        s.stop()


def test_image_locality_still_steers_when_image_present(store):
    big = 900 * 1024 * 1024
    store.create("nodes", node("warm", images={"rocm/pytorch:latest": big}))
    for i in range(3):
        store.create("nodes", node(f"cold{i}"))
    s = new_scheduler(store, load_config(None))
    s.sync_informers(50)
    s.start()
    try:
        store.create("pods", make_pod("img", containers=[{"name": "c", "image": "rocm/pytorch"}]))
        assert wait_placed(store, "img") == "warm"
        # An image nowhere in the cluster: ImageLocality is skipped and the
        # pod still schedules.
        store.create("pods", make_pod("none", containers=[{"name": "c", "image": "example/absent:v1"}]))
        assert wait_placed(store, "none") != ""
    finally:
        s.stop()
