"""In-process API store: apiserver semantics the scheduler relies on
(envtest analog of test/integration/main_test.go)."""
import pytest

from flex_gpu_scheduler_amd._native import native
from flex_gpu_scheduler_amd.models import make_node, make_pod, make_pod_group

StoreError = native().StoreError


def test_create_get_conflict(store):
    p = store.create("pods", make_pod("a"))
    assert p["metadata"]["uid"] and p["metadata"]["resourceVersion"] == "1"
    assert p["status"]["phase"] == "Pending"
    with pytest.raises(StoreError) as e:
        store.create("pods", make_pod("a"))
    assert e.value.code == 409
    assert store.get("pods", "default", "a")["metadata"]["name"] == "a"
    assert store.get("pods", "default", "zz") is None


def test_update_resource_version_conflict(store):
    p = store.create("pods", make_pod("a"))
    p2 = dict(p)
    p2["metadata"] = dict(p["metadata"], labels={"x": "1"})
    store.update("pods", p2)
    with pytest.raises(StoreError) as e:
        store.update("pods", p2)  # stale resourceVersion
    assert e.value.code == 409


def test_binding_copies_annotations_and_rejects_double_bind(store):
    p = store.create("pods", make_pod("a", annotations={"keep": "1"}))
    b = store.bind("default", "a", p["metadata"]["uid"], "n1", {"amd.com/gpu-index": "2"})
    assert b["spec"]["nodeName"] == "n1"
    assert b["metadata"]["annotations"] == {"keep": "1", "amd.com/gpu-index": "2"}
    assert any(c["type"] == "PodScheduled" and c["status"] == "True" for c in b["status"]["conditions"])
    with pytest.raises(StoreError) as e:
        store.bind("default", "a", p["metadata"]["uid"], "n2", {})
    assert e.value.code == 409


def test_merge_patch_status_and_noop(store):
    store.create("podgroups", make_pod_group("pg", min_member=2))
    rv0 = store.resource_version
    out = store.patch("podgroups", "default", "pg", {"status": {"phase": "Scheduling", "scheduled": 1}})
    assert out["status"] == {"phase": "Scheduling", "scheduled": 1}
    rv1 = store.resource_version
    assert rv1 == rv0 + 1
    store.patch("podgroups", "default", "pg", {"status": {"phase": "Scheduling"}})
    assert store.resource_version == rv1  # no-op patch does not bump the version


def test_watch_order_and_replay(store):
    w = store.watch(["pods", "nodes"])
    store.create("nodes", make_node("n1"))
    store.create("pods", make_pod("a"))
    store.delete("pods", "default", "a")
    evs = w.next(100)
    assert [(t, k) for t, k, _, _ in evs] == [("ADDED", "nodes"), ("ADDED", "pods"), ("DELETED", "pods")]
    rvs = [rv for *_, rv in evs]
    assert rvs == sorted(rvs)
    replay = store.watch(["pods"], "", rvs[0])
    assert [t for t, *_ in replay.next(100)] == ["ADDED", "DELETED"]


def test_graceful_delete_sets_deletion_timestamp(store):
    store.create("pods", make_pod("a"))
    out = store.delete("pods", "default", "a", grace_seconds=30)
    assert "deletionTimestamp" in out["metadata"]
    assert store.get("pods", "default", "a") is not None
    store.delete("pods", "default", "a")
    assert store.get("pods", "default", "a") is None


def test_bulk_create_is_one_watch_batch(store):
    import json

    w = store.watch(["pods"])
    store.create_many("pods", json.dumps([make_pod(f"p{i}") for i in range(100)]))
    assert w.pending() == 100
    assert len(w.next(0)) == 100


def test_fault_injection(store):
    store.add_fault("create", "pods", fail_prob=1.0, remaining=1)
    with pytest.raises(StoreError) as e:
        store.create("pods", make_pod("a"))
    assert e.value.code == 500
    store.create("pods", make_pod("a"))  # rule exhausted
