"""CrossNodePreemption (pkg/crossnodepreemption/cross_node_preemption.go,
commented out upstream together with test/integration/cross_node_preemption_test.go:19-133).

The reference's two (commented-out) integration cases run at the end of this
file. The other scenarios pin the MI355X-relevant cross-node cases: a pod
blocked by an anti-affinity peer on a node it can never use is admitted by
evicting that peer; DefaultPreemption cannot do this because it only evicts
pods on the node being considered.
"""
import time

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.config import ConfigError, default_plugin_args
from flex_gpu_scheduler_amd.models import make_node, make_pod
from helpers import placements, wait_bound

import pytest


def cnp_config(**args):
    prof = {"schedulerName": "default-scheduler", "plugins": {
        "postFilter": {"enabled": [{"name": "CrossNodePreemption"}], "disabled": [{"name": "DefaultPreemption"}]}}}
    if args:
        prof["pluginConfig"] = [{"name": "CrossNodePreemption", "args": args}]
    return {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
            "profiles": [prof]}


DEFAULT = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration"}

ZONE = "topology.kubernetes.io/zone"


def anti_affinity(app):
    return {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"app": app}}, "topologyKey": ZONE}]}}


def wait_for(pred, timeout=10.0):
    t0 = time.time()
    while not pred():
        assert time.time() - t0 < timeout
        time.sleep(0.005)


def _zone_cluster(store):
    # Both nodes in zone a. Only `gpu` carries the label the preemptor needs;
    # the blocking peer sits on `cpu`, which the preemptor can never use.
    store.create("nodes", make_node("cpu", {"cpu": "8", "memory": "64Gi", "pods": "10"}, labels={ZONE: "a"}))
    store.create("nodes", make_node("gpu", {"cpu": "8", "memory": "64Gi", "pods": "10"},
                                    labels={ZONE: "a", "accel": "mi355x"}))
    store.create("pods", make_pod("peer", requests={"cpu": "1"}, priority=1, labels={"app": "db"}, node_name="cpu"))
    store.create("pods", make_pod("bystander", requests={"cpu": "1"}, priority=1, labels={"app": "web"},
                                  node_name="cpu"))


def _preemptor():
    return make_pod("trainer", requests={"cpu": "1"}, priority=100, node_selector={"accel": "mi355x"},
                    affinity=anti_affinity("db"))


def test_evicts_blocking_peer_on_another_node(store):
    _zone_cluster(store)
    s = new_scheduler(store, load_config(cnp_config()), start=True)
    try:
        s.sync_informers(50)
        store.create("pods", _preemptor())
        wait_for(lambda: store.get("pods", "default", "peer") is None)
        wait_bound(s, 1)
        assert placements(store)["trainer"] == "gpu"
        # Minimum-victim search: the unrelated low-priority pod survives.
        assert store.get("pods", "default", "bystander") is not None
    finally:
        s.stop()


def test_default_preemption_cannot_resolve_cross_node_block(store):
    _zone_cluster(store)
    s = new_scheduler(store, load_config(DEFAULT), start=True)
    try:
        s.sync_informers(50)
        store.create("pods", _preemptor())
        time.sleep(0.4)
        assert store.get("pods", "default", "peer") is not None
        assert placements(store)["trainer"] == ""
    finally:
        s.stop()


def test_higher_priority_peer_is_never_evicted(store):
    store.create("nodes", make_node("cpu", {"cpu": "8", "memory": "64Gi", "pods": "10"}, labels={ZONE: "a"}))
    store.create("nodes", make_node("gpu", {"cpu": "8", "memory": "64Gi", "pods": "10"},
                                    labels={ZONE: "a", "accel": "mi355x"}))
    store.create("pods", make_pod("peer", requests={"cpu": "1"}, priority=1000, labels={"app": "db"}, node_name="cpu"))
    s = new_scheduler(store, load_config(cnp_config()), start=True)
    try:
        s.sync_informers(50)
        store.create("pods", _preemptor())
        time.sleep(0.4)
        assert store.get("pods", "default", "peer") is not None
        assert placements(store)["trainer"] == ""
    finally:
        s.stop()


def test_two_victims_needed_across_nodes(store):
    # Peers on two different nodes of the zone both block; maxVictims=1 cannot
    # help, maxVictims=2 evicts exactly those two.
    for n in ("a1", "a2"):
        store.create("nodes", make_node(n, {"cpu": "8", "memory": "64Gi", "pods": "10"}, labels={ZONE: "a"}))
    store.create("nodes", make_node("gpu", {"cpu": "8", "memory": "64Gi", "pods": "10"},
                                    labels={ZONE: "a", "accel": "mi355x"}))
    for i, n in enumerate(("a1", "a2")):
        store.create("pods", make_pod(f"peer{i}", requests={"cpu": "1"}, priority=1, labels={"app": "db"}, node_name=n))
    store.create("pods", make_pod("other", requests={"cpu": "1"}, priority=1, labels={"app": "web"}, node_name="a1"))
    s = new_scheduler(store, load_config(cnp_config(maxVictims=1)), start=True)
    try:
        s.sync_informers(50)
        store.create("pods", _preemptor())
        time.sleep(0.4)
        assert store.get("pods", "default", "peer0") is not None
    finally:
        s.stop()
    store.delete("pods", "default", "trainer")
    s = new_scheduler(store, load_config(cnp_config(maxVictims=2)), start=True)
    try:
        s.sync_informers(50)
        store.create("pods", _preemptor())
        wait_for(lambda: store.get("pods", "default", "peer0") is None and store.get("pods", "default", "peer1") is None)
        wait_bound(s, 1)
        assert placements(store)["trainer"] == "gpu"
        assert store.get("pods", "default", "other") is not None
    finally:
        s.stop()


def test_resource_preemption_still_works_on_same_node(store):
    store.create("nodes", make_node("n", {"cpu": "4", "memory": "100", "pods": "10"}))
    s = new_scheduler(store, load_config(cnp_config()), start=True)
    try:
        store.create("pods", make_pod("big", requests={"memory": "80"}, priority=1))
        store.create("pods", make_pod("small", requests={"memory": "10"}, priority=1))
        wait_bound(s, 2)
        store.create("pods", make_pod("high", requests={"memory": "50"}, priority=100))
        wait_for(lambda: store.get("pods", "default", "big") is None)
        assert store.get("pods", "default", "small") is not None
    finally:
        s.stop()


def test_args_defaults_and_validation():
    a = default_plugin_args("CrossNodePreemption", {})
    assert a == {"maxVictims": 3, "maxPoolPods": 32, "maxCombinations": 20000}
    with pytest.raises(ConfigError):
        default_plugin_args("CrossNodePreemption", {"maxVictims": 0})
    with pytest.raises(ConfigError):
        default_plugin_args("CrossNodePreemption", {"bogus": 1})


# The reference's (commented-out) integration cases,
# test/integration/cross_node_preemption_test.go:40-73: a zone1 pair of
# low-priority "foo" pods must BOTH go for a high-priority pod whose hard
# spread constraint / required anti-affinity spans the zone; node-x (zone2)
# holds no pods. DefaultPreemption runs first and cannot help (one victim
# per node); CrossNodePreemption is appended after it, as upstream.
FOO_EXISTS = {"matchExpressions": [{"key": "foo", "operator": "Exists"}]}


def _reference_cluster(store):
    for n, zone, pods in (("node-a", "zone1", "10"), ("node-b", "zone1", "10"), ("node-x", "zone2", "0")):
        store.create("nodes", make_node(n, {"cpu": "8", "memory": "64Gi", "pods": pods}, labels={"zone": zone, "node": n}))
    for n in ("a", "b"):
        store.create("pods", make_pod(f"pod-{n}", labels={"foo": ""}, node_name=f"node-{n}", uid=f"pod-{n}"))


APPENDED = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
            "profiles": [{"schedulerName": "default-scheduler",
                          "plugins": {"postFilter": {"enabled": [{"name": "CrossNodePreemption"}]}}}]}


@pytest.mark.parametrize("kind", ["PodTopologySpread", "PodAntiAffinity"])
def test_reference_cases_preempt_two_pods_in_zone1(store, kind):
    _reference_cluster(store)
    if kind == "PodTopologySpread":
        p = make_pod("p", labels={"foo": ""}, priority=1000, uid="p")
        p["spec"]["topologySpreadConstraints"] = [{"maxSkew": 1, "topologyKey": "zone",
                                                   "whenUnsatisfiable": "DoNotSchedule", "labelSelector": FOO_EXISTS}]
    else:
        p = make_pod("p", labels={"foo": ""}, priority=1000, uid="p", affinity={"podAntiAffinity": {
            "requiredDuringSchedulingIgnoredDuringExecution": [{"labelSelector": FOO_EXISTS, "topologyKey": "zone"}]}})
    s = new_scheduler(store, load_config(APPENDED), start=True)
    try:
        s.sync_informers(50)
        store.create("pods", p)
        wait_for(lambda: store.get("pods", "default", "pod-a") is None and store.get("pods", "default", "pod-b") is None)
        wait_for(lambda: bool(store.get("pods", "default", "p")["spec"].get("nodeName")))
        assert store.get("pods", "default", "p")["spec"]["nodeName"] in ("node-a", "node-b")
    finally:
        s.stop()
