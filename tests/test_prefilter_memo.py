"""PodTopologySpread and InterPodAffinity keep their PreFilter / PreScore
states across cycles and replay the cache's pod events into them (csrc/plugins/topology.cc
StateMemo, Snapshot::replay_since). Parity: after random pod creations,
deletions, label changes, terminations and namespace label changes, a
long-lived scheduler (memoized, replayed states) must give exactly the
verdicts of a fresh scheduler that counts from scratch."""
import random

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_node, make_pod

HOST = "kubernetes.io/hostname"
ZONE = "topology.kubernetes.io/zone"


def template(name, app, ns="default"):
    p = make_pod(name, ns, labels={"app": app, "tier": "web"})
    p["spec"]["topologySpreadConstraints"] = [
        {"maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": "DoNotSchedule",
         "labelSelector": {"matchLabels": {"tier": "web"}}},
        {"maxSkew": 2, "topologyKey": HOST, "whenUnsatisfiable": "DoNotSchedule",
         "labelSelector": {"matchLabels": {"app": app}}}]
    ns_term = {"labelSelector": {"matchLabels": {"app": "db"}}, "topologyKey": ZONE,
               "namespaceSelector": {"matchLabels": {"team": "data"}}}
    p["spec"]["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"app": app}}, "topologyKey": HOST}, ns_term]}}
    return p


def preferred(name, app):
    p = make_pod(name, labels={"app": app, "tier": "web"})
    p["spec"]["affinity"] = {
        "podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
            {"weight": 7, "podAffinityTerm": {"labelSelector": {"matchLabels": {"app": "db"}}, "topologyKey": ZONE}}]},
        "podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
            {"weight": 3, "podAffinityTerm": {"labelSelector": {"matchLabels": {"app": app}},
                                              "topologyKey": HOST}}]}}
    return p


def soft_spread(name, app):
    p = make_pod(name, labels={"app": app, "tier": "web"})
    p["spec"]["topologySpreadConstraints"] = [
        {"maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": "ScheduleAnyway",
         "labelSelector": {"matchLabels": {"tier": "web"}}},
        {"maxSkew": 1, "topologyKey": HOST, "whenUnsatisfiable": "ScheduleAnyway",
         "labelSelector": {"matchLabels": {"app": app}}}]
    return p


def verdicts(s, pods):
    out = []
    for p in pods:
        e = s.explain(p)
        scores = sorted((n, v.get("InterPodAffinity*1"), v.get("PodTopologySpread*2"))
                        for n, v in e.get("scores", {}).items())
        out.append((sorted(e["feasible"]), sorted((n, v.get("plugin")) for n, v in e["filtered"].items()), scores))
    return out


def test_memoized_prefilter_matches_fresh_count(store):
    rng = random.Random(7)
    nodes = [f"n{i}" for i in range(12)]
    for i, n in enumerate(nodes):
        store.create("nodes", make_node(n, {"cpu": "64", "memory": "256Gi", "pods": "110"},
                                        labels={ZONE: f"z{i % 3}"}))
    store.create("namespaces", {"metadata": {"name": "team", "labels": {"team": "data"}}})
    guard = make_pod("guard", "default", labels={"app": "guard"}, node_name="n0")
    guard["spec"]["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"tier": "web"}}, "topologyKey": HOST}]}}
    store.create("pods", guard)
    probes = [template("probe-a", "a"), template("probe-b", "b"), preferred("probe-c", "a"), soft_spread("probe-d", "b")]
    live = new_scheduler(store, load_config(None))
    live.sync_informers(50)
    existing = []
    for step in range(60):
        op = rng.random()
        if op < 0.55 or not existing:
            name = f"e{step}"
            ns = "team" if rng.random() < 0.2 else "default"
            app = rng.choice(["a", "b", "db"])
            q = make_pod(name, ns, labels={"app": app, "tier": rng.choice(["web", "batch"])},
                         node_name=rng.choice(nodes))
            if rng.random() < 0.25:  # existing pods' own preferred / required affinity score the probes too
                q["spec"]["affinity"] = {"podAffinity": {
                    "preferredDuringSchedulingIgnoredDuringExecution": [
                        {"weight": 5, "podAffinityTerm": {"labelSelector": {"matchLabels": {"tier": "web"}},
                                                          "topologyKey": ZONE}}],
                    "requiredDuringSchedulingIgnoredDuringExecution": [
                        {"labelSelector": {"matchLabels": {"app": "a"}}, "topologyKey": HOST}]}}
            store.create("pods", q)
            existing.append((ns, name))
        elif op < 0.75:
            ns, name = existing.pop(rng.randrange(len(existing)))
            store.delete("pods", ns, name)
        elif op < 0.9:
            ns, name = rng.choice(existing)
            obj = store.get("pods", ns, name)
            obj["metadata"]["labels"]["app"] = rng.choice(["a", "b", "db"])
            if rng.random() < 0.3:
                obj["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:00Z"
            store.update("pods", obj)
        else:
            store.update("namespaces", {"metadata": {"name": "team",
                                                     "labels": {"team": rng.choice(["data", "ml"])}}})
        if step % 4 == 3:
            live.sync_informers(50)
            fresh = new_scheduler(store, load_config(None))
            fresh.sync_informers(50)
            try:
                assert verdicts(live, probes) == verdicts(fresh, probes), f"step {step}"
            finally:
                fresh.stop()
    live.stop()
