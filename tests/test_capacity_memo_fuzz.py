"""Differential check of CapacityScheduling's guarded dry-run memo
(`PreemptionPolicy::guarded_victims`, docs/ARCHITECTURE.md round 5).

A scheduler that lives through a random sequence of quota edits and pod
churn (its memo warm, entries guarded by the quota predicates they read) must
return exactly the dry-run candidates of a scheduler started fresh on the
same store (empty memo) for every preemptor asked along the way. Preemptors
come from a few templates so the warm memo is hit, and quota mins sit close
to the namespaces' usage so the guards flip.
"""
import random

import pytest

from flex_gpu_scheduler_amd import Store, load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_elastic_quota, make_node, make_pod
from flex_gpu_scheduler_amd.models.objects import make_container

NS = ("ns1", "ns2", "ns3")
CONFIG = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
          "profiles": [{"schedulerName": "default-scheduler", "plugins": {
              "preFilter": {"enabled": [{"name": "CapacityScheduling"}]},
              "filter": {"enabled": [{"name": "NodeResourcesFit"}]},
              "postFilter": {"enabled": [{"name": "CapacityScheduling"}], "disabled": [{"name": "*"}]},
              "reserve": {"enabled": [{"name": "CapacityScheduling"}]}}}]}


def mem_pod(name, ns, mem, prio, node=None):
    return make_pod(name, ns, uid=name, priority=prio, node_name=node,
                    containers=[make_container("c", requests={"memory": str(mem)})])


def dry_run(s, preemptor):
    got = s.plugin_call("CapacityScheduling", "dryRunPreemption", {"pod": preemptor, "runPreFilter": True})
    if "candidates" not in got:
        return ("status", got.get("code"), got.get("message"))
    return ("candidates", sorted((c["node"], tuple(sorted(c["victims"])), c["numPDBViolations"])
                                 for c in got["candidates"]))


@pytest.mark.parametrize("seed", range(6))
def test_guarded_memo_matches_a_cold_scheduler(seed):
    rng = random.Random(seed)
    store = Store()
    for i in range(6):
        store.create("nodes", make_node(f"n{i}", {"memory": "400", "cpu": "100", "pods": "110"}))
    for ns in NS:
        store.create("elasticquotas", make_elastic_quota(f"eq-{ns}", ns, min={"memory": "700"},
                                                         max={"memory": "2400"}))
    pods = {}
    k = 0
    for i in range(6):
        used = 0
        while used < 300:
            ns, mem = rng.choice(NS), rng.choice((50, 100))
            name = f"p{k}"
            k += 1
            store.create("pods", mem_pod(name, ns, mem, rng.choice((1, 5, 10)), node=f"n{i}"))
            pods[name] = ns
            used += mem
    templates = [mem_pod("pre", ns, mem, prio) for ns in NS for mem, prio in ((150, 10), (250, 20))]
    warm = new_scheduler(store, load_config(CONFIG))
    warm.sync_informers(50)
    try:
        hits = 0
        kinds = set()
        for step in range(25):
            action = rng.random()
            if action < 0.4:  # nudge one quota's min around the namespaces' usage
                ns = rng.choice(NS)
                eq = store.get("elasticquotas", ns, f"eq-{ns}")
                eq["spec"]["min"]["memory"] = str(rng.choice((400, 550, 650, 700, 750, 850, 1000)))
                store.update("elasticquotas", eq)
            elif action < 0.6 and pods:  # a pod leaves
                name = rng.choice(sorted(pods))
                store.delete("pods", pods.pop(name), name)
            elif action < 0.8:  # a pod arrives on a node
                ns, name = rng.choice(NS), f"p{k}"
                k += 1
                store.create("pods", mem_pod(name, ns, 50, rng.choice((1, 5, 10)), node=f"n{rng.randrange(6)}"))
                pods[name] = ns
            warm.sync_informers(50)
            cold = new_scheduler(store, load_config(CONFIG))
            cold.sync_informers(50)
            try:
                for pre in rng.sample(templates, 3):
                    a, b = dry_run(warm, pre), dry_run(cold, pre)
                    assert a == b, (seed, step, pre["metadata"]["namespace"], a, b)
                    hits += a[0] == "candidates" and bool(a[1])
                    kinds.add(a[0] if a[0] == "status" else ("candidates", bool(a[1])))
            finally:
                cold.stop()
        assert hits > 0, kinds  # the warm scheduler did answer with candidates along the way
    finally:
        warm.stop()
