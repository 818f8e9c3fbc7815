"""Cache debugger (upstream internal/cache/debugger: comparer + dumper, on
SIGUSR2 in kube-scheduler; here `check_cache()` / `dump_cache()`, the
scheduler daemon's /debug/cache/* routes and SIGUSR2). A churn soak — gangs,
whole-GPU / XCD / HBM-slice pods, plain pods, deletions, node label changes,
priority preemption — must leave the cache equal to the listers, every
NodeInfo's incremental accounting (resources, ports, GPU ledger, gang
counts) equal to one rebuilt from its pods, and the gang counters equal to a
recount."""
import random
import time

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.models import GPU, GPU_MEMORY, GPU_XCD, make_pod, make_pod_group, mi355x_node
from flex_gpu_scheduler_amd.utils.workload import flagship_config


def quiesce(s, timeout=20.0):
    """Until the queue is drained and no bind is in flight for a while."""
    end = time.time() + timeout
    last, stable = None, 0
    while time.time() < end:
        st, q = s.stats(), s.queue_counts()
        now = (st["bound"], st["attempts"], q["active"], q["backoff"], st["inflight_bindings"])
        idle = q["active"] == 0 and q["backoff"] == 0 and st["inflight_bindings"] == 0
        stable = stable + 1 if idle and now == last else 0
        if stable >= 5:
            return
        last = now
        time.sleep(0.05)


def test_churn_leaves_cache_consistent(store):
    rng = random.Random(11)
    for i in range(6):
        store.create("nodes", mi355x_node(f"mi-{i}", mode="cpx" if i % 3 == 2 else "spx", labels={"rack": "r0"}))
    s = new_scheduler(store, load_config(flagship_config(permit_wait_s=2, denied_s=1)),
                      podInitialBackoffSeconds=0.01, podMaxBackoffSeconds=0.05)
    s.start()
    try:
        live, gid, seq = [], 0, 0
        for round_ in range(4):
            for _ in range(30):
                op = rng.random()
                if op < 0.3:
                    size = rng.choice([1, 2, 4, 8])
                    g = f"g{gid}"
                    gid += 1
                    store.create("podgroups", make_pod_group(g, "default", size))
                    for r in range(size):
                        name = f"{g}-r{r}"
                        store.create("pods", make_pod(name, pod_group=g, requests={"cpu": "4"}, limits={GPU: "1"}))
                        live.append(name)
                elif op < 0.6:
                    kind = rng.choice([{GPU: "1"}, {GPU_XCD: "2"}, {GPU_MEMORY: "24"}, None])
                    seq += 1
                    name = f"p{seq}"
                    store.create("pods", make_pod(name, requests={"cpu": "2", "memory": "8Gi"}, limits=kind,
                                                  priority=rng.choice([0, 0, 100])))
                    live.append(name)
                elif op < 0.85 and live:
                    name = live.pop(rng.randrange(len(live)))
                    try:
                        store.delete("pods", "default", name)
                    except Exception:  # noqa: BLE001 - already gone (preempted)
                        pass
                else:
                    n = store.get("nodes", "", f"mi-{rng.randrange(6)}")
                    n["metadata"]["labels"]["rack"] = rng.choice(["r0", "r1"])
                    store.update("nodes", n)
            quiesce(s)
            report = s.check_cache()
            assert report["clean"], report
            dump = s.dump_cache()
            assert len(dump["nodes"]) == 6 and dump["pods"] >= 0
            assert set(dump["queue"]) >= {"active", "backoff", "unschedulable", "pods"}
        assert s.stats()["bound"] > 20
    finally:
        s.stop()


def test_compare_reports_a_node_only_the_store_has(store):
    store.create("nodes", mi355x_node("mi-0"))
    s = new_scheduler(store, load_config(flagship_config()))
    s.sync_informers(50)
    assert s.check_cache()["clean"]
    # A Node added to the store after the informer stopped syncing is
    # reported, as upstream's comparer reports lister/cache differences.
    store.create("nodes", mi355x_node("mi-1"))
    r = s.check_cache()
    assert r["missing_nodes"] == ["mi-1"] and not r["clean"]
    # A difference is read again before it is reported (the two reads are
    # not atomic); a clean cache takes one read.
    assert r["reads"] > 1
    s.sync_informers(50)
    r = s.check_cache()
    assert r["clean"] and r["reads"] == 1
    s.stop()


def test_bind_failures_recover_and_leave_cache_consistent(store):
    """Fault injection (ObjectStore.add_fault): a third of the bindings fail
    with a server error. Failed binds are unreserved and the pods retried;
    every pod ends up bound exactly once and the cache matches the listers
    (upstream handleBindingCycleError: ForgetPod + requeue)."""
    for i in range(4):
        store.create("nodes", mi355x_node(f"mi-{i}"))
    s = new_scheduler(store, load_config(flagship_config(permit_wait_s=2, denied_s=1)),
                      podInitialBackoffSeconds=0.01, podMaxBackoffSeconds=0.05)
    store.add_fault("bind", "pods", fail_prob=0.33)
    s.start()
    try:
        for g in range(4):
            store.create("podgroups", make_pod_group(f"g{g}", "default", 4))
            for r in range(4):
                store.create("pods", make_pod(f"g{g}-{r}", pod_group=f"g{g}", requests={"cpu": "2"},
                                              limits={GPU: "1"}))
        for i in range(16):
            store.create("pods", make_pod(f"x{i}", requests={"cpu": "1"}, limits={GPU_XCD: "2"}))
        deadline = time.time() + 30
        while time.time() < deadline:
            pods = store.list("pods", "default")[0]
            if all(p["spec"].get("nodeName") for p in pods):
                break
            time.sleep(0.05)
        store.clear_faults()
        assert all(p["spec"].get("nodeName") for p in store.list("pods", "default")[0])
        assert s.stats()["bind_failures"] > 0
        quiesce(s)
        report = s.check_cache()
        assert report["clean"], report
    finally:
        s.stop()


def test_dump_on_first_fit_error(store, tmp_path):
    """dumpOnFitError: the first Unschedulable cycle writes the cache dump,
    the failing pod and its diagnosis (and, with tracing on, the trace ring up
    to that cycle) — the post-mortem of an open-loop overload."""
    store.create("nodes", mi355x_node("mi-0", mode="spx"))
    path = tmp_path / "fit.json"
    s = new_scheduler(store, load_config(flagship_config()), dumpOnFitError=str(path), trace=True,
                      podInitialBackoffSeconds=0.01, podMaxBackoffSeconds=0.05)
    s.start()
    try:
        store.create("pods", make_pod("ok", "default", limits={GPU: "8"}))
        store.create("pods", make_pod("big", "default", limits={GPU: "8"}))
        end = time.time() + 10
        while not path.exists() and time.time() < end:
            time.sleep(0.02)
        import json

        d = json.loads(path.read_text())
        assert d["pod"] == "default/big" and "insufficient resource amd.com/gpu" in d["message"]
        (node,) = d["nodes"]
        assert node["name"] == "mi-0" and node["gpu"]["free_whole"] == 0 and len(node["pods"]) == 1
        trace = json.loads((tmp_path / "fit.json.trace.json").read_text())
        events = trace["traceEvents"] if isinstance(trace, dict) else trace
        assert any(e["name"] == "schedule" for e in events)
    finally:
        s.stop()


def test_repeated_failures_aggregate_into_one_event(store):
    """client-go's EventCorrelator: a pod failing for the same reason on every
    retry is one FailedScheduling Event whose count grows, not one object per
    attempt (the store would otherwise grow with every retry)."""
    store.create("nodes", mi355x_node("mi-0", mode="spx"))
    s = new_scheduler(store, load_config(flagship_config()), podInitialBackoffSeconds=0.01,
                      podMaxBackoffSeconds=0.02)
    s.start()
    try:
        store.create("pods", make_pod("big", "default", limits={GPU: "16"}))
        end = time.time() + 10
        evs = []
        while time.time() < end:
            evs = [e for e in store.list("events", "default")[0]
                   if e.get("reason") == "FailedScheduling" and e["involvedObject"]["name"] == "big"]
            if evs and evs[0].get("count", 1) >= 3:
                break
            # A node label change requeues the unschedulable pod (NodeUpdate).
            store.patch("nodes", "", "mi-0", {"metadata": {"labels": {"tick": str(time.time_ns())}}})
            time.sleep(0.05)
        assert len(evs) == 1 and evs[0]["count"] >= 2 and s.stats()["unschedulable"] >= evs[0]["count"]
        assert evs[0]["firstTimestamp"] <= evs[0]["lastTimestamp"]
    finally:
        s.stop()
