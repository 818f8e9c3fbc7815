"""CapacityScheduling / ElasticQuota on 8x MI355X (BASELINE config: "2
namespaces contend for 8 MI355X with preemption"). Scenarios follow the
reference's test/integration/capacity_scheduling_test.go:120-440."""
import time

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.models import GPU, make_elastic_quota, make_node, make_pod
from helpers import create_all, placements, wait_bound

CONFIG = {
    "apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
    "profiles": [{"schedulerName": "default-scheduler", "plugins": {
        "preFilter": {"enabled": [{"name": "CapacityScheduling"}]},
        "postFilter": {"enabled": [{"name": "CapacityScheduling"}], "disabled": [{"name": "*"}]},
        "reserve": {"enabled": [{"name": "CapacityScheduling"}]}}}],
}


def gpu_node(name="n", gpus=8):
    return make_node(name, {"cpu": "64", "memory": "512Gi", "pods": "64", GPU: str(gpus)})


def gpod(name, ns, prio=0, gpus=1):
    return make_pod(name, ns, requests={"cpu": "1"}, limits={GPU: str(gpus)}, priority=prio)


def count_bound(store, ns):
    return sum(1 for v in placements(store, ns).values() if v)


def wait_for(pred, timeout=10.0):
    t0 = time.time()
    while not pred():
        assert time.time() - t0 < timeout
        time.sleep(0.005)


def test_cross_namespace_preemption_reclaims_min(store):
    store.create("nodes", gpu_node())
    create_all(store, "elasticquotas",
               [make_elastic_quota("eq1", "ns1", min={GPU: "4", "cpu": "100"}, max={GPU: "8", "cpu": "100"}),
                make_elastic_quota("eq2", "ns2", min={GPU: "4", "cpu": "100"}, max={GPU: "8", "cpu": "100"})])
    s = new_scheduler(store, load_config(CONFIG), start=True)
    try:
        create_all(store, "pods", [gpod(f"a{i}", "ns1") for i in range(8)])  # ns1 borrows ns2's min
        wait_bound(s, 8)
        create_all(store, "pods", [gpod(f"b{i}", "ns2") for i in range(4)])
        wait_for(lambda: count_bound(store, "ns2") == 4, 15)
        assert count_bound(store, "ns1") == 4  # exactly the borrowed GPUs were reclaimed
    finally:
        s.stop()


def test_quota_without_cpu_rejects_cpu_requests(store):
    # cmp2 always compares cpu and memory: a quota whose max omits cpu admits
    # no pod that requests cpu (reference semantics, elasticquota.go:165-181).
    store.create("nodes", gpu_node())
    store.create("elasticquotas", make_elastic_quota("eq1", "ns1", min={GPU: "2"}, max={GPU: "3"}))
    s = new_scheduler(store, load_config(CONFIG), start=True)
    try:
        store.create("pods", gpod("a", "ns1"))
        time.sleep(0.3)
        assert count_bound(store, "ns1") == 0
    finally:
        s.stop()


def test_max_is_a_hard_cap(store):
    store.create("nodes", gpu_node())
    # ns2's unused min is what ns1 may borrow (Σused <= Σmin), up to its max.
    create_all(store, "elasticquotas", [
        make_elastic_quota("eq1", "ns1", min={GPU: "2", "cpu": "100"}, max={GPU: "3", "cpu": "100"}),
        make_elastic_quota("eq2", "ns2", min={GPU: "4", "cpu": "100"}, max={GPU: "4", "cpu": "100"})])
    s = new_scheduler(store, load_config(CONFIG), start=True)
    try:
        create_all(store, "pods", [gpod(f"a{i}", "ns1") for i in range(5)])
        wait_bound(s, 3)
        time.sleep(0.3)
        assert count_bound(store, "ns1") == 3
        msgs = [p["status"]["conditions"][0]["message"] for p in store.list("pods", "ns1")[0] if not p["spec"].get("nodeName")]
        assert all("more than Max" in m for m in msgs), msgs
    finally:
        s.stop()


def test_in_namespace_preemption_by_priority(store):
    store.create("nodes", gpu_node(gpus=2))
    store.create("elasticquotas", make_elastic_quota("eq1", "ns1", min={GPU: "2", "cpu": "100"}, max={GPU: "2", "cpu": "100"}))
    s = new_scheduler(store, load_config(CONFIG), start=True)
    try:
        create_all(store, "pods", [gpod("low1", "ns1", 1), gpod("low2", "ns1", 1)])
        wait_bound(s, 2)
        store.create("pods", gpod("high", "ns1", 100))
        wait_for(lambda: placements(store, "ns1").get("high") == "n", 15)
        assert count_bound(store, "ns1") == 2
    finally:
        s.stop()


def test_regular_preemption_without_quota(store):
    store.create("nodes", gpu_node(gpus=1))
    s = new_scheduler(store, load_config(CONFIG), start=True)
    try:
        store.create("pods", gpod("low", "free", 1))
        wait_bound(s, 1)
        store.create("pods", gpod("high", "free", 100))
        wait_for(lambda: placements(store, "free").get("high") == "n", 15)
    finally:
        s.stop()


def test_overused_quota_cannot_preempt_other_quota(store):
    store.create("nodes", gpu_node(gpus=4))
    create_all(store, "elasticquotas",
               [make_elastic_quota("eq1", "ns1", min={GPU: "1", "cpu": "50"}, max={GPU: "4", "cpu": "100"}),
                make_elastic_quota("eq2", "ns2", min={GPU: "3", "cpu": "50"}, max={GPU: "4", "cpu": "100"})])
    s = new_scheduler(store, load_config(CONFIG), start=True)
    try:
        create_all(store, "pods", [gpod(f"b{i}", "ns2", 1) for i in range(3)])
        wait_bound(s, 3)
        create_all(store, "pods", [gpod("a0", "ns1", 100), gpod("a1", "ns1", 100)])
        time.sleep(0.6)
        # a0 fits in the free GPU; a1 would push ns1 over min and may not evict ns2 (within its min).
        assert count_bound(store, "ns2") == 3
        assert count_bound(store, "ns1") == 1
    finally:
        s.stop()
