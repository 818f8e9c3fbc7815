"""All-zero Score skip (Framework::run_score in csrc/framework/framework.cc):
TaintToleration is skipped while no node carries a PreferNoSchedule taint
(a count the cache keeps per Node change), ImageLocality while none of the
pod's images is on any node (the Snapshot's image spread), NodeAffinity /
InterPodAffinity / PodTopologySpread while the pod has no preference terms.

A skipped plugin still adds its normalized constant (100 for the reversed
TaintToleration and PodTopologySpread normalizers) to every total, so the
scheduling path's totals equal explain()'s, which runs every plugin. These
tests pin that the skip never hides a real preference, including when the
inputs of the skip decision change after startup."""
import time

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_node, make_pod

from helpers import placements

SOFT = [{"key": "soft", "effect": "PreferNoSchedule"}]


def node(name, images=None, taints=None, labels=None):
    n = make_node(name, {"cpu": "32", "memory": "64Gi", "pods": "110"}, labels=labels)
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


def started(store):
    s = new_scheduler(store, load_config(None))
    s.sync_informers(50)
    s.start()
    return s


def assert_hot_totals_match(s, pod):
    out = s.explain(pod)
    totals = {n: v["total"] for n, v in out["scores"].items()}
    assert out["hot_path_totals"] == totals, out


def test_prefer_no_schedule_taint_added_later_is_scored(store):
    store.create("nodes", node("a"))
    store.create("nodes", node("b"))
    s = started(store)
    try:
        store.create("pods", make_pod("p0"))
        first = wait_placed(store, "p0")
        other = "b" if first == "a" else "a"
        # The empty node now gets a PreferNoSchedule taint; the next pod must
        # follow the taint (a stale skip would let LeastAllocated pick it).
        store.patch("nodes", "", other, {"spec": {"taints": SOFT}})
        time.sleep(0.3)
        for i in range(1, 4):
            store.create("pods", make_pod(f"p{i}"))
            assert wait_placed(store, f"p{i}") == first
    finally:
        s.stop()


def test_untolerated_prefer_no_schedule_taint_avoided(store):
    store.create("nodes", node("t1", taints=SOFT))
    store.create("nodes", node("t2", taints=SOFT))
    store.create("nodes", node("clean"))
    s = started(store)
    try:
        store.create("pods", make_pod("p"))
        assert wait_placed(store, "p") == "clean"
    finally:
        s.stop()


def test_removing_last_prefer_no_schedule_taint(store):
    """The count goes back to zero when the only tainted node loses its taint:
    TaintToleration is skipped again and LeastAllocated picks the emptier
    (previously tainted) node."""
    store.create("nodes", node("busy"))
    store.create("nodes", node("soft", taints=SOFT))
    s = started(store)
    try:
        store.create("pods", make_pod("p0", requests={"cpu": "8"}))
        assert wait_placed(store, "p0") == "busy"
        store.patch("nodes", "", "soft", {"spec": {"taints": None}})
        deadline = time.time() + 5
        while time.time() < deadline:  # wait until the informer has the untainted node
            out = s.explain(make_pod("probe", requests={"cpu": "1"}))
            if out["scores"]["soft"]["total"] > out["scores"]["busy"]["total"]:
                break
            time.sleep(0.02)
        assert_hot_totals_match(s, make_pod("probe", requests={"cpu": "1"}))
        store.create("pods", make_pod("p1", requests={"cpu": "1"}))
        assert wait_placed(store, "p1") == "soft"
    finally:
        s.stop()


def test_image_locality_still_steers_when_image_present(store):
    big = 900 * 1024 * 1024
    store.create("nodes", node("warm", images={"rocm/pytorch:latest": big}))
    for i in range(3):
        store.create("nodes", node(f"cold{i}"))
    s = started(store)
    try:
        store.create("pods", make_pod("img", containers=[{"name": "c", "image": "rocm/pytorch"}]))
        assert wait_placed(store, "img") == "warm"
        # An image nowhere in the cluster: ImageLocality is skipped and the
        # pod still schedules.
        store.create("pods", make_pod("none", containers=[{"name": "c", "image": "example/absent:v1"}]))
        assert wait_placed(store, "none") != ""
    finally:
        s.stop()


def test_image_pulled_later_steers_next_pod(store):
    """An image that shows up on a node through a Node status update after
    startup: the Snapshot's image spread picks it up and ImageLocality steers
    the next pod there."""
    big = 900 * 1024 * 1024
    for i in range(4):
        store.create("nodes", node(f"n{i}"))
    s = started(store)
    try:
        img = [{"name": "c", "image": "rocm/vllm:v1"}]
        assert_hot_totals_match(s, make_pod("probe", containers=img))
        store.patch("nodes", "", "n2", {"status": {"images": [{"names": ["rocm/vllm:v1"], "sizeBytes": big}]}})
        deadline = time.time() + 5
        while time.time() < deadline:
            if s.explain(make_pod("probe", containers=img))["scores"]["n2"]["ImageLocality*1"] > 0:
                break
            time.sleep(0.02)
        assert_hot_totals_match(s, make_pod("probe", containers=img))
        store.create("pods", make_pod("v", containers=img))
        assert wait_placed(store, "v") == "n2"
    finally:
        s.stop()


def test_skipped_reversed_normalizers_keep_totals_equal(store):
    """No PreferNoSchedule taint and no soft spread constraint: TaintToleration
    and PodTopologySpread are skipped on the scheduling path but still add
    100 x weight, so its totals equal explain()'s full run."""
    for i in range(3):
        store.create("nodes", node(f"n{i}"))
    s = started(store)
    try:
        store.create("pods", make_pod("seed", requests={"cpu": "4"}))
        wait_placed(store, "seed")
        assert_hot_totals_match(s, make_pod("probe", requests={"cpu": "1"}))
    finally:
        s.stop()


def test_soft_spread_with_nodes_missing_the_topology_key(store):
    """PodTopologySpread's NormalizeScore keys ignored nodes (missing the
    topology label) by name; the reused score rows must carry names for it,
    or an ignored node would normalize above 100 and fail the cycle."""
    store.create("nodes", node("z1a", labels={"topology.kubernetes.io/zone": "z1"}))
    store.create("nodes", node("z2a", labels={"topology.kubernetes.io/zone": "z2"}))
    store.create("nodes", node("nolabel"))
    s = started(store)
    try:
        spread = [{"maxSkew": 1, "topologyKey": "topology.kubernetes.io/zone",
                   "whenUnsatisfiable": "ScheduleAnyway", "labelSelector": {"matchLabels": {"app": "w"}}}]
        def spread_pod(name):
            p = make_pod(name, labels={"app": "w"})
            p["spec"]["topologySpreadConstraints"] = spread
            return p

        for i in range(4):
            store.create("pods", spread_pod(f"w{i}"))
            wait_placed(store, f"w{i}")
        assert_hot_totals_match(s, spread_pod("probe"))
        scores = s.explain(spread_pod("probe"))["scores"]
        pts = next(k for k in scores["nolabel"] if k.startswith("PodTopologySpread*"))
        assert scores["nolabel"][pts] == 0, scores  # ignored node: normalized to 0, not preferred
        st = s.stats()
        assert st["bound"] >= 4, st
    finally:
        s.stop()
