"""PreemptionToleration: the reference's 8 integration cases
(test/integration/preemption_toleration_test.go:60-156), over the HTTP API
server and the remote-mode scheduler.

One node (3 cpu, 3Gi) that fits one 2-cpu/1Gi pod; a victim candidate at
priority 1000 in a PriorityClass carrying the toleration annotations; its
PodScheduled condition is back-dated by `scheduled_before` seconds; then a
preemptor arrives. Backoff is 0/0 as in the reference (:180-181). "Tolerates"
is checked for a shorter window than the reference's 15 s `consistently`.
"""
import datetime
import time

import pytest

from flex_gpu_scheduler_amd import load_config
from flex_gpu_scheduler_amd.control import ApiServer, RestClient
from flex_gpu_scheduler_amd.control.remote import RemoteScheduler
from flex_gpu_scheduler_amd.models import make_node, make_pod, make_priority_class

MIN_KEY = "preemption-toleration.scheduling.sigs.k8s.io/minimum-preemptable-priority"
SEC_KEY = "preemption-toleration.scheduling.sigs.k8s.io/toleration-seconds"
PRIO = 1000
REQ = {"cpu": "2", "memory": "1Gi"}
FOREVER = 10 ** 9

CONFIG = {
    "apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
    "profiles": [{"schedulerName": "default-scheduler", "plugins": {
        "postFilter": {"enabled": [{"name": "PreemptionToleration"}], "disabled": [{"name": "*"}]}},
        "pluginConfig": [{"name": "PreemptionToleration",
                          "args": {"minCandidateNodesPercentage": 10, "minCandidateNodesAbsolute": 100}}]}],
}

# name, PC annotations, preemptor priority, preemptor policy, victim scheduled before (s), can tolerate
CASES = [
    ("preemptor priority >= MinimumPreemptablePriority: can NOT tolerate",
     {MIN_KEY: str(PRIO + 10)}, PRIO + 10, None, 0, False),
    ("preemptor priority >= MinimumPreemptablePriority: TolerationSeconds has no effect",
     {MIN_KEY: str(PRIO + 10), SEC_KEY: "30"}, PRIO + 10, None, 0, False),
    ("preemptor priority < MinimumPreemptablePriority: no TolerationSeconds (default 0) tolerates nothing",
     {MIN_KEY: str(PRIO + 10)}, PRIO + 9, None, 0, False),
    ("preemptor priority < MinimumPreemptablePriority: tolerationSeconds = -1 tolerates forever",
     {MIN_KEY: str(PRIO + 10), SEC_KEY: "-1"}, PRIO + 9, None, FOREVER, True),
    ("preemptor priority < MinimumPreemptablePriority: tolerates within TolerationSeconds",
     {MIN_KEY: str(PRIO + 10), SEC_KEY: "30"}, PRIO + 5, None, 0, True),
    ("preemptor priority < MinimumPreemptablePriority: can NOT tolerate after TolerationSeconds elapsed",
     {MIN_KEY: str(PRIO + 10), SEC_KEY: "5"}, PRIO + 5, None, 10, False),
    ("unparsable policy: victim preempted when preemptor is PreemptLowerPriority",
     {MIN_KEY: "a"}, PRIO + 1, "PreemptLowerPriority", 0, False),
    ("unparsable policy: victim kept when preemptor is Never",
     {MIN_KEY: "a"}, PRIO + 1, "Never", FOREVER, True),
]


def _scheduled(client, name):
    p = client.get("pods", "default", name)
    return bool(p and p["spec"].get("nodeName"))


def _wait(fn, timeout):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if fn():
            return True
        time.sleep(0.02)
    return bool(fn())


@pytest.mark.parametrize("name,ann,prio,policy,before,tolerates", CASES, ids=[c[0] for c in CASES])
def test_preemption_toleration_integration(store, name, ann, prio, policy, before, tolerates):
    srv = ApiServer(store).start()
    client = RestClient(srv.url)
    rs = None
    try:
        client.create("nodes", make_node("node-a", {"cpu": "3", "memory": "3Gi", "pods": "110"}))
        client.create("priorityclasses", make_priority_class("pc-victims", PRIO, annotations=ann))
        rs = RemoteScheduler(client, load_config(CONFIG), podInitialBackoffSeconds=0, podMaxBackoffSeconds=0).start()
        client.create("pods", make_pod("victim-candidate", requests=REQ, priority=PRIO, priority_class="pc-victims"))
        assert _wait(lambda: _scheduled(client, "victim-candidate"), 20)
        when = datetime.datetime.now(datetime.timezone.utc) - datetime.timedelta(seconds=min(before, 10 ** 8))
        client.patch("pods", "default", "victim-candidate", {"status": {"conditions": [
            {"type": "PodScheduled", "status": "True",
             "lastTransitionTime": when.strftime("%Y-%m-%dT%H:%M:%SZ")}]}})
        time.sleep(0.2)  # let the scheduler's mirror observe the back-dated condition
        client.create("pods", make_pod("p", requests=REQ, priority=prio, preemption_policy=policy))
        if tolerates:
            deadline = time.time() + 2.0
            while time.time() < deadline:
                assert _scheduled(client, "victim-candidate") and not _scheduled(client, "p")
                time.sleep(0.1)
        else:
            assert _wait(lambda: _scheduled(client, "p") and client.get("pods", "default", "victim-candidate") is None,
                         20)
    finally:
        if rs:
            rs.stop()
        srv.stop()
