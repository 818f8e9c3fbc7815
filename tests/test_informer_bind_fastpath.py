"""The informer builds the bound object of a pod it bound itself by copying
the assumed pod (Scheduler::bound_copy_of_assumed) instead of re-parsing the
Pod; the cache keeps the assumed object when the bound one accounts the same
(SchedulerCache::confirm_assumed_locked). Both must be indistinguishable from
a full parse of the stored object."""
import time

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd._native import native
from flex_gpu_scheduler_amd.models import GPU, GPU_XCD, make_pod, make_pod_group, mi355x_node
from flex_gpu_scheduler_amd.utils.workload import flagship_config

FIELDS = ("key", "request", "nonzero_request", "limits", "qos", "pod_group", "priority", "gpus", "partitions",
          "node_name", "uid", "resource_version", "labels", "annotations", "phase", "scheduled_at", "start_time",
          "template_hash", "spec_hash", "scheduler_name", "host_ports")


def wait(pred, timeout=10.0):
    end = time.time() + timeout
    while time.time() < end:
        if pred():
            return True
        time.sleep(0.01)
    return False


def test_bound_copy_matches_full_parse(store):
    store.create("nodes", mi355x_node("n0"))
    store.create("nodes", mi355x_node("n1", mode="cpx"))
    s = new_scheduler(store, load_config(flagship_config()), start=True)
    try:
        store.create("podgroups", make_pod_group("g", "default", 2))
        pods = [make_pod("w0", pod_group="g", requests={"cpu": "1"}, limits={GPU: "1"}, labels={"team": "a"}),
                make_pod("w1", pod_group="g", requests={"cpu": "1"}, limits={GPU: "1"}, labels={"team": "a"}),
                make_pod("x0", limits={GPU_XCD: "2"}), make_pod("plain", requests={"cpu": "500m"})]
        for p in pods:
            store.create("pods", p)
        names = [p["metadata"]["name"] for p in pods]
        assert wait(lambda: all(store.get("pods", "default", n)["spec"].get("nodeName") for n in names))
        for n in names:
            obj = store.get("pods", "default", n)
            assert wait(lambda: (s.lister_pod("default", n) or {}).get("resource_version") ==
                        int(obj["metadata"]["resourceVersion"]))
            got = s.lister_pod("default", n)
            want = native().pod_summary(obj)
            for f in FIELDS:
                assert got[f] == want[f], (n, f, got[f], want[f])
            assert got["scheduled_at"] > 0 and got["node_name"]
        # The cache still accounts every pod once on its node.
        placed = {}
        for n in names:
            placed.setdefault(store.get("pods", "default", n)["spec"]["nodeName"], 0)
            placed[store.get("pods", "default", n)["spec"]["nodeName"]] += 1
        for node, count in placed.items():
            assert s.node_info(node)["pods"] == count
    finally:
        s.stop()


def test_status_only_update_matches_full_parse(store):
    """A status-only patch (the PodScheduled=False condition a failed cycle
    writes) reaches the informer flagged WatchEvent::status_only; the lister's
    previous object is copied with the new status fields
    (Scheduler::status_copy_of_listed) and must equal a full parse."""
    store.create("nodes", mi355x_node("n0"))
    s = new_scheduler(store, load_config(flagship_config()), start=True)
    try:
        # Unschedulable (asks for more GPUs than any node has): its failed
        # cycle patches the condition; then patches of status alone follow.
        store.create("pods", make_pod("big", requests={"cpu": "1"}, limits={GPU: "16"}, labels={"team": "b"}))
        assert wait(lambda: any(c.get("type") == "PodScheduled" and c.get("status") == "False"
                                for c in store.get("pods", "default", "big").get("status", {}).get("conditions", [])))
        store.patch("pods", "default", "big", {"status": {"phase": "Pending", "nominatedNodeName": "n0",
                                                          "startTime": "2026-01-02T03:04:05Z"}})
        store.patch("pods", "default", "big", {"status": {"conditions": [
            {"type": "PodScheduled", "status": "True", "lastTransitionTime": "2026-01-02T03:04:06Z"}]}})
        obj = store.get("pods", "default", "big")
        assert wait(lambda: (s.lister_pod("default", "big") or {}).get("resource_version") ==
                    int(obj["metadata"]["resourceVersion"]))
        got = s.lister_pod("default", "big")
        want = native().pod_summary(obj)
        for f in FIELDS:
            assert got[f] == want[f], (f, got[f], want[f])
        assert got["start_time"] > 0 and got["scheduled_at"] > 0
        # A patch that is not status-only still parses (labels change the pod).
        store.patch("pods", "default", "big", {"metadata": {"labels": {"team": "c"}}})
        obj = store.get("pods", "default", "big")
        assert wait(lambda: (s.lister_pod("default", "big") or {}).get("resource_version") ==
                    int(obj["metadata"]["resourceVersion"]))
        assert s.lister_pod("default", "big")["labels"] == native().pod_summary(obj)["labels"]
    finally:
        s.stop()
