"""The reference's PreemptionToleration unit tables, case for case, through
Scheduler.plugin_call:

* pkg/preemptiontoleration/preemption_toleration_test.go:50-203
  ExemptedFromPreemption (11 cases over 5 tests)
* pkg/preemptiontoleration/preemption_toleration_policy_test.go:26
  parsePreemptionTolerationPolicy (5 cases)

The victim's PriorityClass lives in the store (the reference's fake client
and informer); `nowUs` pins the clock the reference passes as `now`.
"""
import datetime
import time

import pytest

from flex_gpu_scheduler_amd import Store, load_config, new_scheduler
from flex_gpu_scheduler_amd.models import make_pod, make_priority_class

MIN_KEY = "preemption-toleration.scheduling.sigs.k8s.io/minimum-preemptable-priority"
SEC_KEY = "preemption-toleration.scheduling.sigs.k8s.io/toleration-seconds"
PC = "priority-class"  # testPriorityClassName

CONFIG = {
    "apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
    "profiles": [{"schedulerName": "default-scheduler", "plugins": {
        "postFilter": {"enabled": [{"name": "PreemptionToleration"}], "disabled": [{"name": "*"}]}}}],
}

NOW = int(time.time()) * 1_000_000


def rfc3339(us):
    return datetime.datetime.fromtimestamp(us / 1e6, datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def victim(priority, scheduled_at=None):
    """makePod().PriorityClassName(..).ScheduledAt(at).Priority(p)."""
    p = make_pod("victim", priority=priority, priority_class=PC)
    if scheduled_at is not None:
        p["status"] = {"conditions": [{"type": "PodScheduled", "status": "True",
                                       "lastTransitionTime": rfc3339(scheduled_at)}]}
    return p


def preemptor(priority, policy=None):
    return make_pod("preemptor", priority=priority, preemption_policy=policy)


def sched_with(pc):
    store = Store()
    if pc is not None:
        store.create("priorityclasses", pc)
    s = new_scheduler(store, load_config(CONFIG))
    s.sync_informers(50)
    return s


# name, victim PC (value, annotations) or None, victim, preemptor, want (bool or error substring)
EXEMPT_CASES = [
    # TestExemptedFromPreemptionWithNonExitingPriorityClass
    ("priority class does not exist: error", None, victim(3), preemptor(2, "PreemptLowerPriority"),
     f'priorityclass.scheduling.k8s.io "{PC}" not found'),
    # TestExemptedFromPreemptionWithUnparsalbePolicy
    ("MinimumPreemptablePriority not parsable: false", (1, {MIN_KEY: "a"}), victim(3),
     preemptor(2, "PreemptLowerPriority"), False),
    ("TolerationSeconds not parsable: false", (1, {MIN_KEY: "10", SEC_KEY: "a"}), victim(3),
     preemptor(2, "PreemptLowerPriority"), False),
    # TestExemptedFromPreemptionWithoutPolicy
    ("preemptor PreemptNever: true", (1, None), victim(1), preemptor(2, "Never"), True),
    ("PreemptLowerPriority, victim PC below preemptor: false", (1, None), victim(1),
     preemptor(2, "PreemptLowerPriority"), False),
    ("PreemptLowerPriority, victim PC not below preemptor: true", (3, None), victim(3),
     preemptor(2, "PreemptLowerPriority"), True),
    # ...WhenPreemptorPriorityHigherOrEqualMinimumPreemptablePriority
    ("preemptor above MinimumPreemptablePriority: false", (100, {MIN_KEY: "200"}), victim(100, NOW),
     preemptor(201), False),
    ("preemptor equal to MinimumPreemptablePriority: false", (100, {MIN_KEY: "200"}), victim(100, NOW),
     preemptor(200), False),
    # ...WhenPreemptorPriorityLowerThanMinimumPreemptablePriority
    ("TolerationSeconds 0: false", (100, {MIN_KEY: "200", SEC_KEY: "0"}), victim(100, NOW), preemptor(199), False),
    ("TolerationSeconds negative: tolerates forever", (100, {MIN_KEY: "200", SEC_KEY: "-1"}),
     victim(100, 1_000_000), preemptor(199), True),
    ("TolerationSeconds elapsed: false", (100, {MIN_KEY: "200", SEC_KEY: "100"}),
     victim(100, NOW - 101_000_000), preemptor(199), False),
    ("within TolerationSeconds: true", (100, {MIN_KEY: "200", SEC_KEY: "100"}),
     victim(100, NOW - 10_000_000), preemptor(199), True),
]


@pytest.mark.parametrize("name,pc,vic,pre,want", EXEMPT_CASES, ids=[c[0] for c in EXEMPT_CASES])
def test_exempted_from_preemption(name, pc, vic, pre, want):
    s = sched_with(make_priority_class(PC, pc[0], annotations=pc[1]) if pc else None)
    try:
        out = s.plugin_call("PreemptionToleration", "exemptedFromPreemption",
                            {"pod": pre, "victim": vic, "preemptor": pre, "nowUs": NOW})
        if isinstance(want, str):
            assert want in out["error"]
        else:
            assert "error" not in out
            assert out["exempted"] is want
    finally:
        s.stop()


POLICY_CASES = [
    ("defaults", None, {"minimumPreemptablePriority": 2, "tolerationSeconds": 0}),
    ("both values", {MIN_KEY: "100", SEC_KEY: "10"}, {"minimumPreemptablePriority": 100, "tolerationSeconds": 10}),
    ("unparsable MinimumPreemptablePriority", {MIN_KEY: "a"}, 'strconv.ParseInt: parsing "a": invalid syntax'),
    ("unparsable TolerationSeconds", {SEC_KEY: "a"}, 'strconv.ParseInt: parsing "a": invalid syntax'),
    ("negative TolerationSeconds", {MIN_KEY: "100", SEC_KEY: "-1"},
     {"minimumPreemptablePriority": 100, "tolerationSeconds": -1}),
]


@pytest.fixture(scope="module")
def pt_sched():
    s = sched_with(None)
    yield s
    s.stop()


@pytest.mark.parametrize("name,ann,want", POLICY_CASES, ids=[c[0] for c in POLICY_CASES])
def test_parse_policy(pt_sched, name, ann, want):
    out = pt_sched.plugin_call("PreemptionToleration", "parsePolicy",
                               {"pod": preemptor(1), "priorityClass": make_priority_class(PC, 1, annotations=ann)})
    if isinstance(want, str):
        assert out == {"error": want}  # cmp.Diff on err.Error()
    else:
        assert out == want


def test_parse_policy_out_of_range(pt_sched):
    out = pt_sched.plugin_call("PreemptionToleration", "parsePolicy",
                               {"pod": preemptor(1),
                                "priorityClass": make_priority_class(PC, 1, annotations={MIN_KEY: "4294967296"})})
    assert out == {"error": 'strconv.ParseInt: parsing "4294967296": value out of range'}
