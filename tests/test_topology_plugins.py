"""PodTopologySpread, InterPodAffinity, ImageLocality (upstream default
plugins the reference gets from the vendored kube-scheduler; cases follow
vendor/.../plugins/{podtopologyspread,interpodaffinity,imagelocality}
*_test.go semantics for k8s 1.23)."""
import time

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_node, make_pod

from helpers import placements


def node(name, zone=None, images=None, **labels):
    lab = dict(labels)
    if zone:
        lab["topology.kubernetes.io/zone"] = zone
    n = make_node(name, {"cpu": "32", "memory": "64Gi", "pods": "110"}, labels=lab)
    if images:
        n["status"]["images"] = [{"names": [i], "sizeBytes": s} for i, s in images.items()]
    return n


def pod(name, labels=None, node_name=None, **spec):
    p = make_pod(name, labels=labels, node_name=node_name)
    p["spec"].update(spec)
    return p


def spread(key, skew=1, hard=True, app="x"):
    return {"maxSkew": skew, "topologyKey": key, "whenUnsatisfiable": "DoNotSchedule" if hard else "ScheduleAnyway",
            "labelSelector": {"matchLabels": {"app": app}}}


def term(key, **match):
    return {"labelSelector": {"matchLabels": match}, "topologyKey": key}


HOST = "kubernetes.io/hostname"
ZONE = "topology.kubernetes.io/zone"


def sched(store, **kw):
    s = new_scheduler(store, load_config(None), **kw)
    s.sync_informers(50)
    return s


def zones(store):
    for n, z in (("a1", "a"), ("a2", "a"), ("b1", "b"), ("b2", "b")):
        store.create("nodes", node(n, z))


def test_spread_hard_zone_skew(store):
    zones(store)
    for i, n in enumerate(("a1", "a2")):
        store.create("pods", pod(f"e{i}", {"app": "x"}, n))
    s = sched(store)
    out = s.explain(pod("p", {"app": "x"}, topologySpreadConstraints=[spread(ZONE)]))
    assert sorted(out["feasible"]) == ["b1", "b2"]
    assert out["filtered"]["a1"]["plugin"] == "PodTopologySpread"
    # maxSkew 3 tolerates the imbalance (2 + 1 - 0 <= 3)
    out = s.explain(pod("p", {"app": "x"}, topologySpreadConstraints=[spread(ZONE, skew=3)]))
    assert len(out["feasible"]) == 4
    # A pod that does not match its own selector adds no self count.
    out = s.explain(pod("p", {"app": "y"}, topologySpreadConstraints=[spread(ZONE, skew=2)]))
    assert len(out["feasible"]) == 4
    s.stop()


def test_spread_missing_label_is_unresolvable(store):
    zones(store)
    store.create("nodes", node("nozone"))
    s = sched(store)
    out = s.explain(pod("p", {"app": "x"}, topologySpreadConstraints=[spread(ZONE)]))
    assert "nozone" in out["filtered"] and len(out["feasible"]) == 4
    s.stop()


def test_spread_respects_node_affinity_domains(store):
    zones(store)
    store.create("nodes", node("c1", "c", pool="other"))
    for i in range(2):
        store.create("pods", pod(f"e{i}", {"app": "x"}, ["a1", "b1"][i]))
    s = sched(store)
    # c1 is excluded by the pod's nodeSelector, so zone c (0 pods) does not
    # lower the minimum: zones a and b (1 each) are both allowed.
    p = pod("p", {"app": "x"}, topologySpreadConstraints=[spread(ZONE)],
            affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
                {"matchExpressions": [{"key": ZONE, "operator": "In", "values": ["a", "b"]}]}]}}})
    out = s.explain(p)
    assert sorted(out["feasible"]) == ["a1", "a2", "b1", "b2"]
    s.stop()


def test_spread_soft_scores_fewer_matches_higher(store):
    for n in ("n1", "n2", "n3"):
        store.create("nodes", node(n))
    for i in range(3):
        store.create("pods", pod(f"e{i}", {"app": "x"}, "n1"))
    store.create("pods", pod("e3", {"app": "x"}, "n2"))
    s = sched(store)
    out = s.explain(pod("p", {"app": "x"}, topologySpreadConstraints=[spread(HOST, hard=False)]))
    sc = {n: v["PodTopologySpread*2"] for n, v in out["scores"].items()}
    assert sc["n3"] == 100 and sc["n3"] > sc["n2"] > sc["n1"]
    assert out["selected"] == "n3"
    s.stop()


def test_interpod_required_affinity(store):
    for n in ("n1", "n2", "n3"):
        store.create("nodes", node(n))
    store.create("pods", pod("db", {"app": "db"}, "n2"))
    s = sched(store)
    aff = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [term(HOST, app="db")]}}
    out = s.explain(pod("p", {"app": "web"}, affinity=aff))
    assert out["feasible"] == ["n2"]
    # Self-affinity: the first pod of a series may go anywhere.
    self_aff = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [term(HOST, app="cache")]}}
    out = s.explain(pod("c0", {"app": "cache"}, affinity=self_aff))
    assert len(out["feasible"]) == 3
    # ... but not when the selector matches nothing, including itself.
    out = s.explain(pod("c0", {"app": "other"}, affinity=self_aff))
    assert out["feasible"] == []
    s.stop()


def test_interpod_anti_affinity_both_directions(store):
    for n in ("n1", "n2"):
        store.create("nodes", node(n))
    store.create("pods", pod("web", {"app": "web"}, "n1"))
    guard = pod("guard", {"app": "guard"}, "n2",
                affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                    term(HOST, app="noisy")]}})
    store.create("pods", guard)
    s = sched(store)
    anti = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [term(HOST, app="web")]}}
    assert s.explain(pod("p", {"app": "web"}, affinity=anti))["feasible"] == ["n2"]
    # The existing guard pod repels app=noisy from n2.
    assert s.explain(pod("q", {"app": "noisy"}))["feasible"] == ["n1"]
    s.stop()


def test_interpod_namespace_scoping(store):
    for n in ("n1", "n2"):
        store.create("nodes", node(n))
    store.create("namespaces", {"metadata": {"name": "team", "labels": {"tier": "gold"}}})
    store.create("pods", make_pod("db", "team", labels={"app": "db"}, node_name="n1"))
    s = sched(store)
    # Default: the term looks only in the incoming pod's namespace.
    aff = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [term(HOST, app="db")]}}
    assert s.explain(pod("p", {"app": "web"}, affinity=aff))["feasible"] == []
    t = term(HOST, app="db")
    t["namespaces"] = ["team"]
    aff = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [t]}}
    assert s.explain(pod("p", {"app": "web"}, affinity=aff))["feasible"] == ["n1"]
    t = term(HOST, app="db")
    t["namespaceSelector"] = {"matchLabels": {"tier": "gold"}}
    aff = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [t]}}
    assert s.explain(pod("p", {"app": "web"}, affinity=aff))["feasible"] == ["n1"]
    s.stop()


def test_interpod_preferred_scores(store):
    for n in ("n1", "n2", "n3"):
        store.create("nodes", node(n))
    store.create("pods", pod("db", {"app": "db"}, "n1"))
    store.create("pods", pod("noisy", {"app": "noisy"}, "n3"))
    s = sched(store)
    aff = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        {"weight": 10, "podAffinityTerm": term(HOST, app="db")}]},
        "podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
            {"weight": 10, "podAffinityTerm": term(HOST, app="noisy")}]}}
    out = s.explain(pod("p", {"app": "web"}, affinity=aff))
    sc = {n: v["InterPodAffinity*1"] for n, v in out["scores"].items()}
    assert sc == {"n1": 100, "n2": 50, "n3": 0}
    s.stop()


def test_anti_affinity_preemption_uses_remove_pod(store):
    """DefaultPreemption dry-runs remove the victim through InterPodAffinity's
    RemovePod extension, so a high-priority pod evicts the pod it repels."""
    store.create("nodes", node("n1"))
    store.create("pods", make_pod("web", labels={"app": "web"}, node_name="n1", priority=0))
    s = sched(store, start=False)
    s.start()
    try:
        anti = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [term(HOST, app="web")]}}
        p = make_pod("vip", labels={"app": "vip"}, priority=1000)
        p["spec"]["affinity"] = anti
        store.create("pods", p)
        deadline = time.time() + 15
        while time.time() < deadline and placements(store).get("vip") != "n1":
            time.sleep(0.02)
        assert placements(store) == {"vip": "n1"}
    finally:
        s.stop()


def test_image_locality(store):
    big = 800 * 1024 * 1024
    store.create("nodes", node("warm", images={"rocm/pytorch:latest": big}))
    store.create("nodes", node("cold"))
    store.create("nodes", node("warm2", images={"docker.io/rocm/pytorch:latest": big}))
    s = sched(store)
    p = make_pod("p", containers=[{"name": "c", "image": "rocm/pytorch"}])
    out = s.explain(p)
    sc = {n: v["ImageLocality*1"] for n, v in out["scores"].items()}
    # 800 MiB present on 1 of 3 nodes: 800*1/3 = 266 MiB -> 100*(266-23)/(1000-23) = 24
    assert sc == {"warm": 24, "cold": 0, "warm2": 0}
    s.stop()


def test_hostname_anti_affinity_node_local_and_shared_hostnames(store):
    """Hostname-keyed anti-affinity is checked on the node's own pods while
    every hostname label equals its node's name; once two nodes share a
    hostname value the term is counted per domain again, as upstream does."""
    for n in ("n1", "n2", "n3"):
        store.create("nodes", node(n))
    store.create("pods", pod("web", {"app": "web"}, "n1"))
    store.create("pods", pod("guard", {"app": "guard"}, "n3", affinity={"podAntiAffinity": {
        "requiredDuringSchedulingIgnoredDuringExecution": [term(HOST, app="noisy")]}}))
    s = sched(store)
    anti = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [term(HOST, app="web")]}}
    assert sorted(s.explain(pod("p", {"app": "web"}, affinity=anti))["feasible"]) == ["n2", "n3"]
    assert sorted(s.explain(pod("q", {"app": "noisy"}))["feasible"]) == ["n1", "n2"]
    s.stop()
    # n2 now reports n1's hostname: both form one domain.
    shared = node("n2")
    shared["metadata"]["labels"][HOST] = "n1"
    store.update("nodes", shared)
    shared3 = node("n3")
    shared3["metadata"]["labels"][HOST] = "n1"
    store.update("nodes", shared3)
    s = sched(store)
    assert s.explain(pod("p", {"app": "web"}, affinity=anti))["feasible"] == []
    assert s.explain(pod("q", {"app": "noisy"}))["feasible"] == []
    s.stop()
