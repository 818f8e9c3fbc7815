"""DefaultPreemption + PreemptionToleration through the shared evaluator
(vendor/.../framework/preemption; pkg/preemptiontoleration)."""
import time

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_node, make_pdb, make_pod, make_priority_class
from helpers import placements, wait_bound

DEFAULT = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration"}


def pt_config():
    return {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
            "profiles": [{"schedulerName": "default-scheduler", "plugins": {
                "postFilter": {"enabled": [{"name": "PreemptionToleration"}],
                               "disabled": [{"name": "DefaultPreemption"}]}}}]}


def wait_for(pred, timeout=10.0):
    t0 = time.time()
    while not pred():
        assert time.time() - t0 < timeout
        time.sleep(0.005)


def test_default_preemption_evicts_lower_priority(store):
    store.create("nodes", make_node("n", {"cpu": "4", "memory": "100", "pods": "10"}))
    s = new_scheduler(store, load_config(DEFAULT), start=True)
    try:
        store.create("pods", make_pod("low", requests={"memory": "80"}, priority=1))
        wait_bound(s, 1)
        store.create("pods", make_pod("high", requests={"memory": "50"}, priority=100))
        wait_for(lambda: store.get("pods", "default", "low") is None)
        wait_bound(s, 2)
        assert placements(store) == {"high": "n"}
        assert "scheduler_preemption_victims" in s.metrics_text()
    finally:
        s.stop()


def test_no_preemption_of_equal_priority(store):
    store.create("nodes", make_node("n", {"cpu": "4", "memory": "100", "pods": "10"}))
    s = new_scheduler(store, load_config(DEFAULT), start=True)
    try:
        store.create("pods", make_pod("a", requests={"memory": "80"}, priority=5))
        wait_bound(s, 1)
        store.create("pods", make_pod("b", requests={"memory": "50"}, priority=5))
        time.sleep(0.3)
        assert placements(store) == {"a": "n", "b": ""}
    finally:
        s.stop()


def test_preempt_never_policy(store):
    store.create("nodes", make_node("n", {"cpu": "4", "memory": "100", "pods": "10"}))
    s = new_scheduler(store, load_config(DEFAULT), start=True)
    try:
        store.create("pods", make_pod("low", requests={"memory": "80"}, priority=1))
        wait_bound(s, 1)
        store.create("pods", make_pod("polite", requests={"memory": "50"}, priority=100, preemption_policy="Never"))
        time.sleep(0.3)
        assert store.get("pods", "default", "low") is not None
    finally:
        s.stop()


def test_pdb_violating_victims_are_avoided(store):
    # Two nodes, each with one low-priority pod; one pod is PDB-protected.
    for n in ("n1", "n2"):
        store.create("nodes", make_node(n, {"cpu": "4", "memory": "100", "pods": "10"}))
    s = new_scheduler(store, load_config(DEFAULT), start=True)
    try:
        store.create("poddisruptionbudgets", make_pdb("pdb", "default", {"app": "db"}, disruptions_allowed=0))
        store.create("pods", make_pod("protected", requests={"memory": "80"}, priority=1, labels={"app": "db"},
                                      node_name="n1"))
        store.create("pods", make_pod("plain", requests={"memory": "80"}, priority=1, node_name="n2"))
        s.sync_informers(50)
        store.create("pods", make_pod("high", requests={"memory": "50"}, priority=100))
        wait_for(lambda: store.get("pods", "default", "plain") is None)
        assert store.get("pods", "default", "protected") is not None
        wait_for(lambda: placements(store).get("high") == "n2")
    finally:
        s.stop()


def test_preemption_toleration_exempts_victims(store):
    store.create("nodes", make_node("n", {"cpu": "4", "memory": "100", "pods": "10"}))
    store.create("priorityclasses", make_priority_class("tolerant", 10, annotations={
        "preemption-toleration.scheduling.sigs.k8s.io/minimum-preemptable-priority": "1000",
        "preemption-toleration.scheduling.sigs.k8s.io/toleration-seconds": "-1"}))
    s = new_scheduler(store, load_config(pt_config()), start=True)
    try:
        store.create("pods", make_pod("victim", requests={"memory": "80"}, priority=10, priority_class="tolerant"))
        wait_bound(s, 1)
        store.create("pods", make_pod("mid", requests={"memory": "50"}, priority=500))
        time.sleep(0.4)
        assert store.get("pods", "default", "victim") is not None  # 500 < 1000: tolerated forever
        store.create("pods", make_pod("top", requests={"memory": "50"}, priority=2000))
        wait_for(lambda: store.get("pods", "default", "victim") is None)
    finally:
        s.stop()


def test_preemption_toleration_seconds_window(store):
    store.create("nodes", make_node("n", {"cpu": "4", "memory": "100", "pods": "10"}))
    store.create("priorityclasses", make_priority_class("short", 10, annotations={
        "preemption-toleration.scheduling.sigs.k8s.io/minimum-preemptable-priority": "1000",
        "preemption-toleration.scheduling.sigs.k8s.io/toleration-seconds": "1"}))
    s = new_scheduler(store, load_config(pt_config()), start=True)
    try:
        store.create("pods", make_pod("victim", requests={"memory": "80"}, priority=10, priority_class="short"))
        wait_bound(s, 1)
        store.create("pods", make_pod("mid", requests={"memory": "50"}, priority=500))
        time.sleep(0.3)
        assert store.get("pods", "default", "victim") is not None  # inside the 1 s toleration
        time.sleep(1.0)
        s.move_all()  # retry after the window (an event or the 60 s flush would do this)
        wait_for(lambda: store.get("pods", "default", "victim") is None)
    finally:
        s.stop()


def test_request_beyond_allocatable_verdict(store):
    """k8s 1.23 (the reference's version) reports a request larger than a
    node's allocatable as plain Unschedulable, so that node stays a
    preemption candidate. The opt-in NodeResourcesFit extension
    unresolvableBeyondAllocatable makes it UnschedulableAndUnresolvable
    (evicting pods cannot help; newer upstream does this); a node that is
    merely full stays Unschedulable either way."""
    from flex_gpu_scheduler_amd import load_config, new_scheduler
    from flex_gpu_scheduler_amd.models import make_node, make_pod

    store.create("nodes", make_node("small", {"cpu": "4", "memory": "8Gi", "pods": "10"}))
    store.create("nodes", make_node("big", {"cpu": "16", "memory": "8Gi", "pods": "10"}))
    store.create("pods", make_pod("filler", requests={"cpu": "12"}, node_name="big"))
    for opt_in, small_code in ((False, "Unschedulable"), (True, "UnschedulableAndUnresolvable")):
        cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration"}
        if opt_in:
            cfg["profiles"] = [{"pluginConfig": [{"name": "NodeResourcesFit",
                                                  "args": {"unresolvableBeyondAllocatable": True}}]}]
        s = new_scheduler(store, load_config(cfg))
        s.sync_informers(50)
        out = s.explain(make_pod("p", requests={"cpu": "8"}))
        assert out["filtered"]["small"]["code"] == small_code
        assert out["filtered"]["big"]["code"] == "Unschedulable"
        assert "Insufficient cpu" in out["filtered"]["small"]["reason"]
        s.stop()


def _nominated(name, node, **kw):
    """A pending pod nominated to `node` that cannot itself be placed (its
    node selector matches nothing), so the nomination stays outstanding."""
    p = make_pod(name, node_selector={"never": "matches"}, **kw)
    p["status"] = {"phase": "Pending", "nominatedNodeName": node}
    return p


ANTI_WEB = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
    {"labelSelector": {"matchLabels": {"app": "web"}}, "topologyKey": "topology.kubernetes.io/zone"}]}}


def test_nominated_pod_resources_count_for_equal_or_lower_priority(store):
    """addNominatedPods (vendor/.../runtime/framework.go): a nominated pod of
    priority >= the incoming pod's is counted on its node. It has no
    PreFilter-extension effect here, so the cycle's state is used as is."""
    store.create("nodes", make_node("n", {"cpu": "4", "memory": "100", "pods": "10"},
                                    labels={"kubernetes.io/hostname": "n"}))
    store.create("pods", _nominated("nom", "n", requests={"memory": "60"}, priority=100))
    s = new_scheduler(store, load_config(DEFAULT), start=True)
    try:
        store.create("pods", make_pod("same", requests={"memory": "50"}, priority=100))
        store.create("pods", make_pod("higher", requests={"memory": "50"}, priority=200))
        wait_bound(s, 1)
        time.sleep(0.3)
        assert placements(store) == {"nom": "", "same": "", "higher": "n"}
    finally:
        s.stop()


def test_nominated_pod_anti_affinity_applies_through_prefilter_extension(store):
    """A nominated pod with required anti-affinity changes InterPodAffinity's
    PreFilter state (AddPod), so that state is cloned and the incoming pod
    it repels stays off the node although its resources would fit. The
    zone key keeps Filter on the counted state (a hostname key is decided on
    the node's own pods)."""
    store.create("nodes", make_node("n", {"cpu": "4", "memory": "100", "pods": "10"},
                                    labels={"kubernetes.io/hostname": "n", "topology.kubernetes.io/zone": "z1"}))
    store.create("pods", _nominated("nom", "n", requests={"memory": "10"}, priority=100, affinity=ANTI_WEB))
    s = new_scheduler(store, load_config(DEFAULT), start=True)
    try:
        store.create("pods", make_pod("web", requests={"memory": "10"}, priority=100, labels={"app": "web"}))
        store.create("pods", make_pod("db", requests={"memory": "10"}, priority=100, labels={"app": "db"}))
        wait_bound(s, 1)
        time.sleep(0.3)
        assert placements(store) == {"nom": "", "web": "", "db": "n"}
    finally:
        s.stop()
