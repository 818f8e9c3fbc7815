"""Equivalence cache (Pod::template_hash + node-local Filter/Score reuse,
csrc/scheduler/scheduler.cc eq_entry / find_nodes_that_fit, Framework::run_score).

The cache must be exact: the same workload scheduled cycle by cycle with the
cache on and off must produce identical placements and GPU assignments. The
workload mixes gangs of identical ranks (cache hits), HBM-slice pods, pods
with spread constraints / anti-affinity (non-local: cache bypassed) and a
Node update mid-run (node epoch invalidation)."""
import json

from flex_gpu_scheduler_amd import Store, load_config, new_scheduler
from flex_gpu_scheduler_amd.models import (GPU, GPU_MEMORY, GPU_XCD, INDEX_ANNOTATION, default_gpus, make_container,
                                           make_pod, make_pod_group, mi355x_node, mi355x_nrt)
from flex_gpu_scheduler_amd.utils.workload import ClusterSpec, flagship_config, make_wave

ZONE = "topology.kubernetes.io/zone"


def _cluster(store, nodes=6):
    for i in range(nodes):
        n = mi355x_node(f"n{i}", gpus=default_gpus(8, "cpx" if i == 0 else "spx"))
        n["metadata"]["labels"][ZONE] = f"z{i % 2}"
        store.create("nodes", n)
        store.create("noderesourcetopologies", mi355x_nrt(f"n{i}"))


def _workload():
    pods, groups = [], []
    for g, size in enumerate((8, 4, 2, 8, 1, 4)):
        groups.append(make_pod_group(f"g{g}", "default", size))
        for r in range(size):
            c = make_container("t", requests={"cpu": "2", "memory": "8Gi"}, limits={GPU: "1"})
            pods.append(make_pod(f"g{g}-r{r}", containers=[c], pod_group=f"g{g}"))
    groups.append(make_pod_group("q", "default", 4))
    for r in range(4):
        pods.append(make_pod(f"q-r{r}", containers=[make_container("s", limits={GPU_XCD: "2"})], pod_group="q"))
    for m in range(6):
        pods.append(make_pod(f"m{m}", containers=[make_container("i", limits={GPU_MEMORY: "16"})]))
    for s in range(4):  # spread + anti-affinity: Filter/Score are not node-local for these
        p = make_pod(f"web{s}", requests={"cpu": "1"}, labels={"app": "web"})
        p["spec"]["topologySpreadConstraints"] = [{"maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": "DoNotSchedule",
                                                   "labelSelector": {"matchLabels": {"app": "web"}}}]
        pods.append(p)
    pods.append(make_pod("lonely", requests={"cpu": "1"}, affinity={"podAntiAffinity": {
        "requiredDuringSchedulingIgnoredDuringExecution": [
            {"labelSelector": {"matchLabels": {"app": "web"}}, "topologyKey": "kubernetes.io/hostname"}]}}))
    return groups, pods


def _run(eq: bool):
    store = Store()
    _cluster(store)
    cfg = load_config(flagship_config())
    s = new_scheduler(store, cfg, seed=7, equivalenceCache=eq, bindWorkers=1)
    groups, pods = _workload()
    store.create_many("podgroups", json.dumps(groups))
    half = len(pods) // 2
    store.create_many("pods", json.dumps(pods[:half]))
    s.sync_informers(100)
    while s.schedule_one(50):
        s.sync_informers(0)
    # A Node object update mid-run bumps the node epoch (cache invalidation).
    n1 = store.get("nodes", "", "n1")
    n1["metadata"]["labels"]["touched"] = "yes"
    store.update("nodes", n1)
    store.create_many("pods", json.dumps(pods[half:]))
    s.sync_informers(100)
    while s.schedule_one(50):
        s.sync_informers(0)
    s.wait_idle(5000)
    stats = s.stats()
    s.stop()
    placed, _ = store.list("pods", "default")
    out = {p["metadata"]["name"]: (p["spec"].get("nodeName", ""),
                                   (p["metadata"].get("annotations") or {}).get(INDEX_ANNOTATION, ""))
           for p in placed}
    return out, stats


def test_cache_on_and_off_place_identically():
    on, st_on = _run(True)
    off, st_off = _run(False)
    assert on == off
    assert sum(1 for v in on.values() if v[0]) >= 40
    assert st_on["eq_filter_hits"] > 0 and st_off["eq_filter_hits"] == 0


def test_bench_wave_identical_with_and_without_cache():
    spec = ClusterSpec(nodes=8)
    results = []
    for eq in (True, False):
        store = Store()
        store.create_many("nodes", json.dumps(spec.node_objects()))
        store.create_many("noderesourcetopologies", json.dumps(spec.nrt_objects()))
        s = new_scheduler(store, load_config(flagship_config()), seed=3, equivalenceCache=eq, bindWorkers=1)
        w = make_wave(spec, 0, namespace="bench", seed=11)
        store.create_many("podgroups", w.groups_json())
        store.create_many("pods", w.pods_json())
        s.sync_informers(100)
        while s.schedule_one(50):
            s.sync_informers(0)
        s.wait_idle(5000)
        s.stop()
        placed, _ = store.list("pods", "bench")
        results.append({p["metadata"]["name"]: p["spec"].get("nodeName", "") for p in placed})
    assert results[0] == results[1]
    assert all(results[0].values())


def _wave_stats(options: dict, colocation: str = "None") -> dict:
    """One burst wave on 300 MI355X nodes (the adaptive share of nodes to
    score is < 100% there, so the node window matters), scheduled by
    schedule_one on the calling thread; returns the scheduler's stats.
    Gang co-location is off by default here: with it, a gang's later ranks
    are evaluated on their siblings' node only (NodeRestriction), so the
    scan memo this exercises serves few cycles."""
    import json as _json

    from flex_gpu_scheduler_amd import Store, load_config, new_scheduler
    from flex_gpu_scheduler_amd.utils.workload import ClusterSpec, flagship_config, make_wave

    spec = ClusterSpec(nodes=300)
    store = Store()
    store.create_many("nodes", _json.dumps(spec.node_objects()))
    store.create_many("noderesourcetopologies", _json.dumps(spec.nrt_objects()))
    w = make_wave(spec, 1, namespace="w", fill=0.6)
    store.create_many("podgroups", _json.dumps(w.pod_groups))
    store.create_many("pods", _json.dumps(w.pods))
    s = new_scheduler(store, load_config(flagship_config(gang_colocation=colocation)), seed=7, **options)
    try:
        s.sync_informers(50)
        while s.schedule_one(200):
            pass
        assert s.wait_bound(len(w.pods), 20.0), s.stats()
        return s.stats()
    finally:
        s.stop()


def test_scan_memo_answers_as_the_full_scan():
    """EqEntry::scan re-evaluates only the changed nodes of a template's
    window and re-cuts the feasible list; with scanMemoVerify every answer is
    checked against the full Filter walk (same nodes, in order, same stop)."""
    st = _wave_stats({"scanMemo": True, "scanMemoVerify": True})
    assert st["scan_memo_served"] > 100, st
    assert st["scan_memo_mismatches"] == 0, st
    off = _wave_stats({"scanMemo": False})
    assert off["scan_memo_served"] == 0


def test_gang_scores_from_snapshot_arrays_match_per_node_scoring():
    """XGMIGangAffinity scores whole-GPU and XCD gang ranks from the
    snapshot's contiguous arrays (free GPUs, free XCDs, partition sizes) on
    the scheduling path; explain() runs every plugin per node. Mid-wave, with
    gangs partly placed and CPX partitions partly used, both must agree."""
    import json as _json

    from flex_gpu_scheduler_amd import Store, load_config, new_scheduler
    from flex_gpu_scheduler_amd.utils.workload import ClusterSpec, flagship_config, make_wave

    spec = ClusterSpec(nodes=48)
    store = Store()
    store.create_many("nodes", _json.dumps(spec.node_objects()))
    store.create_many("noderesourcetopologies", _json.dumps(spec.nrt_objects()))
    w = make_wave(spec, 1, namespace="w", fill=0.6)
    store.create_many("podgroups", _json.dumps(w.pod_groups))
    store.create_many("pods", _json.dumps(w.pods))
    s = new_scheduler(store, load_config(flagship_config()), seed=3)
    try:
        s.sync_informers(50)
        for _ in range(len(w.pods) // 2):
            if not s.schedule_one(200):
                break
        s.sync_informers(50)
        pods, _ = store.list("pods", "w")
        pending = [p for p in pods if not p["spec"].get("nodeName")]
        kinds = set()
        checked = 0
        for p in pending[:: max(1, len(pending) // 40)]:
            out = s.explain(p)
            if "scores" not in out:
                continue
            totals = {n: v["total"] for n, v in out["scores"].items()}
            assert out["hot_path_totals"] == totals, (p["metadata"]["name"], out)
            parts = p["metadata"]["name"].split("-")
            kinds.add(parts[2] if len(parts) > 3 else parts[-1])
            checked += 1
        assert checked >= 10 and {"q", "x8"} <= kinds, (checked, kinds)
    finally:
        s.stop()
