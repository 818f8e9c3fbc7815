"""The reference's remaining small unit tables, case for case:

* pkg/capacityscheduling/elasticquota_test.go:27  TestReserveResource
* pkg/capacityscheduling/elasticquota_test.go:79  TestUnReserveResource
  (ElasticQuotaInfo.used +/- computePodResourceRequest, through
  Scheduler.plugin_call("CapacityScheduling", ...); ResourceGPU is the
  MI355X whole-GPU resource here)
* pkg/util/resource_test.go:34  TestGetPodEffectiveRequest (6 cases; the
  native Pod decoder's request vector, api/types.cc)
* pkg/util/podgroup_test.go:31  TestCreateMergePatch (2 cases; the native
  Json::diff_merge_patch and the control plane's merge_patch_between over
  the marshaled objects, zero values included as Go marshals them)
"""
import json

import pytest

from flex_gpu_scheduler_amd import Store, load_config, new_scheduler
from flex_gpu_scheduler_amd._native import native
from flex_gpu_scheduler_amd.control.controllers import merge_patch_between
from flex_gpu_scheduler_amd.models import make_container, make_pod
from flex_gpu_scheduler_amd.models.mi355x import GPU

CS_CONFIG = {
    "apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
    "profiles": [{"schedulerName": "default-scheduler", "plugins": {
        "preFilter": {"enabled": [{"name": "CapacityScheduling"}]},
        "postFilter": {"enabled": [{"name": "CapacityScheduling"}], "disabled": [{"name": "*"}]},
        "reserve": {"enabled": [{"name": "CapacityScheduling"}]}}}],
}


def eq_pod(name, ns, mem, milli_cpu, gpus):
    """makePod(name, ns, memReq, cpuReq, gpuReq, ...) (capacity_scheduling_test.go)."""
    return make_pod(name, ns, containers=[make_container(name, requests={
        "memory": str(mem), "cpu": f"{milli_cpu}m", GPU: str(gpus)})])


EQ_PODS = [eq_pod("t1-p1", "ns1", 50, 1000, 1), eq_pod("t1-p2", "ns2", 100, 2000, 0), eq_pod("t1-p3", "ns2", 0, 0, 2)]


@pytest.fixture(scope="module")
def cs_sched():
    s = new_scheduler(Store(), load_config(CS_CONFIG))
    s.sync_informers(50)
    yield s
    s.stop()


@pytest.mark.parametrize("what,before,after", [
    ("reserveResource", {"cpu": "1000m", "memory": "200", GPU: "2"}, {"cpu": "4", "memory": "350", GPU: "5"}),
    ("unreserveResource", {"cpu": "4000m", "memory": "200", GPU: "5"}, {"cpu": "1", "memory": "50", GPU: "2"}),
])
def test_elastic_quota_reserve_unreserve(cs_sched, what, before, after):
    out = cs_sched.plugin_call("CapacityScheduling", what, {"pod": EQ_PODS[0], "used": before, "pods": EQ_PODS})
    assert out["used"] == after


def rl(milli_cpu, mem):
    """makeResourceList(cpu, mem) (resource_test.go:27)."""
    return {"cpu": f"{milli_cpu}m", "memory": str(mem)}


EFFECTIVE_CASES = [
    ("1 container", [rl(1, 1)], [], (1, 1)),
    ("2 containers", [rl(1, 1), rl(2, 3)], [], (3, 4)),
    ("2 containers and 1 init container", [rl(1, 1), rl(2, 3)], [rl(1, 1)], (3, 4)),
    ("2 containers and 1 init container with large cpu", [rl(1, 1), rl(2, 3)], [rl(10, 1)], (10, 4)),
    ("2 containers and 2 init containers with large cpu or mem", [rl(1, 1), rl(2, 3)], [rl(10, 1), rl(1, 10)],
     (10, 10)),
    ("2 containers and 2 init containers with only large cpu", [rl(1, 1), rl(2, 3)], [rl(10, 1), rl(1, 1)],
     (10, 4)),
]


@pytest.mark.parametrize("name,containers,inits,want", EFFECTIVE_CASES, ids=[c[0] for c in EFFECTIVE_CASES])
def test_get_pod_effective_request(name, containers, inits, want):
    pod = make_pod("p", containers=[make_container(f"c{i}", requests=r) for i, r in enumerate(containers)],
                   init_containers=[make_container(f"i{i}", requests=r) for i, r in enumerate(inits)])
    req = native().pod_summary(pod)["request"]
    assert req == {"cpu": f"{want[0]}m", "memory": str(want[1])}


def go_pod(hostname="", reason=""):
    """An internal core.Pod as encoding/json marshals it: no omitempty, so
    the zero values are present (the reference diffs those)."""
    return {"Spec": {"Hostname": hostname}, "Status": {"Reason": reason}}


@pytest.mark.parametrize("old,new,expected", [
    (go_pod(hostname="test"), go_pod(reason="test"), '{"Spec":{"Hostname":""},"Status":{"Reason":"test"}}'),
    (go_pod(hostname="test", reason="test1"), go_pod(reason="test"),
     '{"Spec":{"Hostname":""},"Status":{"Reason":"test"}}'),
])
def test_create_merge_patch(old, new, expected):
    for patch in (native().diff_merge_patch(old, new), merge_patch_between(old, new)):
        assert json.dumps(patch, separators=(",", ":"), sort_keys=True) == expected
        assert native().merge_patch(old, patch) == new
