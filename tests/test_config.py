"""KubeSchedulerConfiguration decoding, defaulting and profile expansion.

Mirrors the reference's config tests:
  * apis/config/scheme/scheme_test.go:43-338 — decode v1beta2 YAML with every
    out-of-tree plugin's args, the all-defaults variant, and the strict-codec
    error for an unknown Coscheduling field (message shape kept);
  * apis/config/v1beta2/defaults_test.go:30-169 (identical for v1beta3) —
    SetDefaults_* per Args type;
  * cmd/scheduler/main_test.go:48-644 — the expanded plugin set per extension
    point for each per-plugin config file, v1beta2 and v1beta3 (multiPoint),
    against upstream's defaults.PluginsV1beta2 / ExpandedPluginsV1beta3
    (vendor/k8s.io/kubernetes/pkg/scheduler/apis/config/testing/defaults/
    defaults.go:183-274), volume plugins included.
"""
import pytest

from flex_gpu_scheduler_amd.config import ConfigError, default_plugin_args, load_config

V2 = "kubescheduler.config.k8s.io/v1beta2"
V3 = "kubescheduler.config.k8s.io/v1beta3"

# defaults.PluginsV1beta2: point -> [(name, weight)]
PLUGINS_V1BETA2 = {
    "queueSort": [("PrioritySort", 0)],
    "preFilter": [("NodeResourcesFit", 0), ("NodePorts", 0), ("VolumeRestrictions", 0), ("PodTopologySpread", 0),
                  ("InterPodAffinity", 0), ("VolumeBinding", 0), ("NodeAffinity", 0)],
    "filter": [("NodeUnschedulable", 0), ("NodeName", 0), ("TaintToleration", 0), ("NodeAffinity", 0),
               ("NodePorts", 0), ("NodeResourcesFit", 0), ("VolumeRestrictions", 0), ("EBSLimits", 0),
               ("GCEPDLimits", 0), ("NodeVolumeLimits", 0), ("AzureDiskLimits", 0), ("VolumeBinding", 0),
               ("VolumeZone", 0), ("PodTopologySpread", 0), ("InterPodAffinity", 0)],
    "postFilter": [("DefaultPreemption", 0)],
    "preScore": [("InterPodAffinity", 0), ("PodTopologySpread", 0), ("TaintToleration", 0), ("NodeAffinity", 0)],
    "score": [("NodeResourcesBalancedAllocation", 1), ("ImageLocality", 1), ("InterPodAffinity", 1),
              ("NodeResourcesFit", 1), ("NodeAffinity", 1), ("PodTopologySpread", 2), ("TaintToleration", 1)],
    "reserve": [("VolumeBinding", 0)], "permit": [], "preBind": [("VolumeBinding", 0)],
    "bind": [("DefaultBinder", 0)], "postBind": [],
}

# defaults.ExpandedPluginsV1beta3
EXPANDED_V1BETA3 = {
    "queueSort": [("PrioritySort", 0)],
    "preFilter": [("NodeAffinity", 0), ("NodePorts", 0), ("NodeResourcesFit", 0), ("VolumeRestrictions", 0),
                  ("VolumeBinding", 0), ("PodTopologySpread", 0), ("InterPodAffinity", 0)],
    "filter": [("NodeUnschedulable", 0), ("NodeName", 0), ("TaintToleration", 0), ("NodeAffinity", 0),
               ("NodePorts", 0), ("NodeResourcesFit", 0), ("VolumeRestrictions", 0), ("EBSLimits", 0),
               ("GCEPDLimits", 0), ("NodeVolumeLimits", 0), ("AzureDiskLimits", 0), ("VolumeBinding", 0),
               ("VolumeZone", 0), ("PodTopologySpread", 0), ("InterPodAffinity", 0)],
    "postFilter": [("DefaultPreemption", 0)],
    "preScore": [("TaintToleration", 0), ("NodeAffinity", 0), ("PodTopologySpread", 0), ("InterPodAffinity", 0)],
    "score": [("TaintToleration", 3), ("NodeAffinity", 2), ("NodeResourcesFit", 1), ("VolumeBinding", 1),
              ("PodTopologySpread", 2), ("InterPodAffinity", 2), ("NodeResourcesBalancedAllocation", 1),
              ("ImageLocality", 1)],
    "reserve": [("VolumeBinding", 0)], "permit": [], "preBind": [("VolumeBinding", 0)],
    "bind": [("DefaultBinder", 0)], "postBind": [],
}


def expanded(prof) -> dict:
    """Profile -> the ListPlugins() view: point -> [(name, weight)] (weights on score only)."""
    return {pt: [(n, prof.score_weights.get(n, 1) if pt == "score" else 0) for n in names]
            for pt, names in prof.plugins.items()}


def with_points(base: dict, **points) -> dict:
    d = {k: list(v) for k, v in base.items()}
    d.update(points)
    return d


def cfg(api, plugins=None, plugin_config=None, name=None):
    prof = {}
    if name:
        prof["schedulerName"] = name
    if plugins is not None:
        prof["plugins"] = plugins
    if plugin_config is not None:
        prof["pluginConfig"] = plugin_config
    return {"apiVersion": api, "kind": "KubeSchedulerConfiguration", "profiles": [prof]}


ALL = [{"name": "*"}]

# ------------------------------------------------------- main_test.go -------
MAIN_CASES = [
    ("default config", {"apiVersion": V3, "kind": "KubeSchedulerConfiguration"}, EXPANDED_V1BETA3),
    ("default config - v1beta2", {"apiVersion": V2, "kind": "KubeSchedulerConfiguration"}, PLUGINS_V1BETA2),
    ("single profile config - PodState - v1beta2",
     cfg(V2, {"preFilter": {"disabled": ALL}, "filter": {"disabled": ALL}, "preScore": {"disabled": ALL},
              "score": {"enabled": [{"name": "PodState"}], "disabled": ALL}}),
     with_points(PLUGINS_V1BETA2, preFilter=[], filter=[], preScore=[], score=[("PodState", 1)])),
    ("single profile config - QOSSort",
     cfg(V3, {"queueSort": {"enabled": [{"name": "QOSSort"}], "disabled": ALL}, "preFilter": {"disabled": ALL},
              "filter": {"disabled": ALL}, "preScore": {"disabled": ALL}, "score": {"disabled": ALL}}),
     with_points(EXPANDED_V1BETA3, queueSort=[("QOSSort", 0)], preFilter=[], filter=[], preScore=[], score=[])),
    ("single profile config - Coscheduling",
     cfg(V3, {"multiPoint": {"enabled": [{"name": "Coscheduling"}]},
              "queueSort": {"disabled": [{"name": "PrioritySort"}]},
              "filter": {"disabled": ALL}, "score": {"disabled": ALL}, "preScore": {"disabled": ALL}},
         [{"name": "Coscheduling", "args": {"permitWaitingTimeSeconds": 10}}]),
     with_points(EXPANDED_V1BETA3, queueSort=[("Coscheduling", 0)],
                 preFilter=EXPANDED_V1BETA3["preFilter"] + [("Coscheduling", 0)], filter=[],
                 postFilter=[("DefaultPreemption", 0), ("Coscheduling", 0)], preScore=[], score=[],
                 reserve=[("VolumeBinding", 0), ("Coscheduling", 0)], permit=[("Coscheduling", 0)],
                 postBind=[("Coscheduling", 0)])),
    ("single profile config - Node Resources Allocatable with args",
     cfg(V3, {"score": {"enabled": [{"name": "NodeResourcesAllocatable"}], "disabled": ALL}},
         [{"name": "NodeResourcesAllocatable", "args": {"mode": "Least", "resources": [
             {"name": "cpu", "weight": 1000000}, {"name": "memory", "weight": 1}]}}]),
     with_points(EXPANDED_V1BETA3, score=[("NodeResourcesAllocatable", 1)])),
    ("single profile config - Capacityscheduling - v1beta2",
     cfg(V2, {"preFilter": {"enabled": [{"name": "CapacityScheduling"}]},
              "postFilter": {"enabled": [{"name": "CapacityScheduling"}], "disabled": ALL},
              "reserve": {"enabled": [{"name": "CapacityScheduling"}]}}, name="default-scheduler"),
     with_points(PLUGINS_V1BETA2, preFilter=PLUGINS_V1BETA2["preFilter"] + [("CapacityScheduling", 0)],
                 postFilter=[("CapacityScheduling", 0)], reserve=[("VolumeBinding", 0), ("CapacityScheduling", 0)])),
    # Commented out upstream (k/k#108083); expandMultiPointPlugins puts the
    # point's explicit plugins first.
    ("single profile config - Capacityscheduling - v1beta3",
     cfg(V3, {"preFilter": {"enabled": [{"name": "CapacityScheduling"}]},
              "postFilter": {"enabled": [{"name": "CapacityScheduling"}], "disabled": ALL},
              "reserve": {"enabled": [{"name": "CapacityScheduling"}]}}, name="default-scheduler"),
     with_points(EXPANDED_V1BETA3, preFilter=[("CapacityScheduling", 0)] + EXPANDED_V1BETA3["preFilter"],
                 postFilter=[("CapacityScheduling", 0)], reserve=[("CapacityScheduling", 0), ("VolumeBinding", 0)])),
    ("single profile config - TargetLoadPacking with args",
     cfg(V3, {"score": {"enabled": [{"name": "TargetLoadPacking"}], "disabled": ALL}},
         [{"name": "TargetLoadPacking", "args": {"targetUtilization": 60, "defaultRequests": {"cpu": "1000m"},
                                                 "defaultRequestsMultiplier": "1.8",
                                                 "watcherAddress": "http://deadbeef:2020"}}]),
     with_points(EXPANDED_V1BETA3, score=[("TargetLoadPacking", 1)])),
    ("single profile config - TargetLoadPacking with prometheus metric provider args",
     cfg(V3, {"score": {"enabled": [{"name": "TargetLoadPacking"}], "disabled": ALL}},
         [{"name": "TargetLoadPacking", "args": {
             "metricProvider": {"type": "Prometheus", "address": "http://prometheus-k8s.monitoring.svc.cluster.local:9090",
                                "insecureSkipVerify": False},
             "targetUtilization": 60, "defaultRequests": {"cpu": "1000m"}, "defaultRequestsMultiplier": "1.8",
             "watcherAddress": "http://deadbeef:2020"}}]),
     with_points(EXPANDED_V1BETA3, score=[("TargetLoadPacking", 1)])),
    ("single profile config - LoadVariationRiskBalancing with args",
     cfg(V3, {"score": {"enabled": [{"name": "LoadVariationRiskBalancing"}], "disabled": ALL}},
         [{"name": "LoadVariationRiskBalancing", "args": {
             "metricProvider": {"type": "Prometheus", "address": "http://prometheus-k8s.monitoring.svc.cluster.local:9090"},
             "safeVarianceMargin": 1, "safeVarianceSensitivity": 2.5, "watcherAddress": "http://deadbeef:2020"}}]),
     with_points(EXPANDED_V1BETA3, score=[("LoadVariationRiskBalancing", 1)])),
    ("single profile config - NodeResourceTopologyMatch with args",
     cfg(V3, {"filter": {"enabled": [{"name": "NodeResourceTopologyMatch"}], "disabled": ALL},
              "score": {"enabled": [{"name": "NodeResourceTopologyMatch"}], "disabled": ALL}}),
     with_points(EXPANDED_V1BETA3, filter=[("NodeResourceTopologyMatch", 0)],
                 score=[("NodeResourceTopologyMatch", 1)])),
]


@pytest.mark.parametrize("name,doc,want", MAIN_CASES, ids=[c[0] for c in MAIN_CASES])
def test_expanded_plugins_per_profile(name, doc, want):
    assert expanded(load_config(doc).profiles[0]) == want


def test_multiple_profiles():
    c = load_config({"apiVersion": V3, "kind": "KubeSchedulerConfiguration", "profiles": [
        {"schedulerName": "profile-default-plugins"},
        {"schedulerName": "profile-disable-all-filter-and-score-plugins", "plugins": {
            p: {"disabled": ALL} for p in ("preFilter", "filter", "postFilter", "preScore", "score")}}]})
    assert expanded(c.profile("profile-default-plugins")) == EXPANDED_V1BETA3
    assert expanded(c.profile("profile-disable-all-filter-and-score-plugins")) == with_points(
        EXPANDED_V1BETA3, preFilter=[], filter=[], postFilter=[], preScore=[], score=[])


def test_reenabled_default_keeps_its_position_and_takes_the_weight():
    # mergePluginSet: "Update the default plugin in place to preserve order."
    c = load_config(cfg(V2, {"score": {"enabled": [{"name": "ImageLocality", "weight": 5},
                                                   {"name": "PodState", "weight": 2}]}}))
    want = [(n, 5 if n == "ImageLocality" else w) for n, w in PLUGINS_V1BETA2["score"]] + [("PodState", 2)]
    assert expanded(c.profiles[0])["score"] == want


def test_explicit_point_overrides_multipoint_weight_v1beta3():
    c = load_config(cfg(V3, {"score": {"enabled": [{"name": "TaintToleration", "weight": 7}]}}))
    got = expanded(c.profiles[0])["score"]
    assert got[0] == ("TaintToleration", 7)  # explicit point plugins first, multiPoint after
    assert [n for n, _ in got].count("TaintToleration") == 1


def test_multipoint_disable_all_and_v1beta2_rejects_multipoint():
    c = load_config(cfg(V3, {"multiPoint": {"disabled": ALL, "enabled": [{"name": "PrioritySort"},
                                                                          {"name": "DefaultBinder"}]}}))
    e = expanded(c.profiles[0])
    assert e["queueSort"] == [("PrioritySort", 0)] and e["bind"] == [("DefaultBinder", 0)] and e["filter"] == []
    with pytest.raises(ConfigError):
        load_config(cfg(V2, {"multiPoint": {"enabled": [{"name": "Coscheduling"}]}}))


def test_duplicate_registration_is_an_error():
    with pytest.raises(ConfigError, match="already registered"):
        load_config(cfg(V2, {"score": {"enabled": [{"name": "PodState"}, {"name": "PodState"}]}}))


# ----------------------------------------------------- scheme_test.go -------
def test_decode_all_plugin_args_v1beta2():
    c = load_config({"apiVersion": V2, "kind": "KubeSchedulerConfiguration", "profiles": [{
        "schedulerName": "scheduler-plugins", "pluginConfig": [
            {"name": "Coscheduling", "args": {"permitWaitingTimeSeconds": 10, "deniedPGExpirationTimeSeconds": 3}},
            {"name": "NodeResourcesAllocatable", "args": {"mode": "Least", "resources": [
                {"name": "cpu", "weight": 1000000}, {"name": "memory", "weight": 1}]}},
            {"name": "TargetLoadPacking", "args": {
                "targetUtilization": 60, "defaultRequests": {"cpu": "1000m"}, "defaultRequestsMultiplier": "1.8",
                "watcherAddress": "http://deadbeef:2020",
                "metricProvider": {"type": "Prometheus",
                                   "address": "http://prometheus-k8s.monitoring.svc.cluster.local:9090"}}},
            {"name": "LoadVariationRiskBalancing", "args": {
                "metricProvider": {"type": "Prometheus", "address": "http://prometheus-k8s.monitoring.svc.cluster.local:9090",
                                   "insecureSkipVerify": False},
                "safeVarianceMargin": 1.0, "safeVarianceSensitivity": 1.0, "watcherAddress": "http://deadbeef:2020"}},
            {"name": "PreemptionToleration", "args": {"minCandidateNodesPercentage": 20,
                                                      "minCandidateNodesAbsolute": 200}}]}]})
    p = c.profile("scheduler-plugins")
    assert expanded(p) == PLUGINS_V1BETA2
    pc = p.plugin_config
    assert pc["Coscheduling"] == {"permitWaitingTimeSeconds": 10, "deniedPGExpirationTimeSeconds": 3}
    assert pc["NodeResourcesAllocatable"] == {"mode": "Least", "resources": [{"name": "cpu", "weight": 1000000},
                                                                            {"name": "memory", "weight": 1}]}
    tlp = pc["TargetLoadPacking"]
    assert tlp["targetUtilization"] == 60 and tlp["defaultRequestsMultiplier"] == "1.8"
    assert tlp["metricProvider"] == {"type": "Prometheus",
                                     "address": "http://prometheus-k8s.monitoring.svc.cluster.local:9090",
                                     "insecureSkipVerify": True}
    lvrb = pc["LoadVariationRiskBalancing"]
    assert lvrb["metricProvider"]["insecureSkipVerify"] is False
    assert lvrb["safeVarianceMargin"] == 1.0 and lvrb["safeVarianceSensitivity"] == 1.0
    assert pc["PreemptionToleration"] == {"minCandidateNodesPercentage": 20, "minCandidateNodesAbsolute": 200}
    # in-tree defaults materialized for the default plugins
    assert pc["DefaultPreemption"] == {"minCandidateNodesPercentage": 10, "minCandidateNodesAbsolute": 100}
    assert pc["InterPodAffinity"] == {"hardPodAffinityWeight": 1}
    assert pc["NodeResourcesBalancedAllocation"]["resources"] == [{"name": "cpu", "weight": 1},
                                                                  {"name": "memory", "weight": 1}]
    assert pc["NodeResourcesFit"]["scoringStrategy"] == {"type": "LeastAllocated", "resources": [
        {"name": "cpu", "weight": 1}, {"name": "memory", "weight": 1}]}
    assert pc["PodTopologySpread"]["defaultingType"] == "System"


@pytest.mark.parametrize("api", [V2, V3])
def test_decode_unspecified_args_get_defaults(api):
    c = load_config({"apiVersion": api, "kind": "KubeSchedulerConfiguration", "profiles": [{
        "schedulerName": "scheduler-plugins", "pluginConfig": [
            {"name": n, "args": None} for n in ("Coscheduling", "NodeResourcesAllocatable", "TargetLoadPacking",
                                                 "LoadVariationRiskBalancing", "PreemptionToleration")]}]})
    pc = c.profile("scheduler-plugins").plugin_config
    assert pc["Coscheduling"] == {"permitWaitingTimeSeconds": 60, "deniedPGExpirationTimeSeconds": 20}
    assert pc["NodeResourcesAllocatable"] == {"mode": "Least", "resources": [{"name": "cpu", "weight": 1048576},
                                                                            {"name": "memory", "weight": 1}]}
    tlp = pc["TargetLoadPacking"]
    assert (tlp["targetUtilization"], tlp["defaultRequestsMultiplier"], tlp["defaultRequests"]) == (
        40, "1.5", {"cpu": "1000m"})
    assert tlp["metricProvider"] == {"type": "KubernetesMetricsServer"}
    lvrb = pc["LoadVariationRiskBalancing"]
    assert lvrb["metricProvider"] == {"type": "KubernetesMetricsServer"}
    assert (lvrb["safeVarianceMargin"], lvrb["safeVarianceSensitivity"]) == (1.0, 1.0)
    assert pc["PreemptionToleration"] == {"minCandidateNodesPercentage": 10, "minCandidateNodesAbsolute": 100}


@pytest.mark.parametrize("api", [V2, V3])
def test_strict_decoding_error_shape(api):
    with pytest.raises(ConfigError) as ei:
        load_config({"apiVersion": api, "kind": "KubeSchedulerConfiguration", "profiles": [{
            "schedulerName": "scheduler-plugins", "pluginConfig": [
                {"name": "Coscheduling", "args": {"kubeConfigPath": "/var/run/kubernetes/kube.config"}}]}]})
    assert str(ei.value) == ('decoding .profiles[0].pluginConfig[0]: decoding args for plugin Coscheduling: '
                             'strict decoding error: unknown field "kubeConfigPath"')


# ---------------------------------------------------- defaults_test.go ------
DEFAULTS_CASES = [
    ("empty config CoschedulingArgs", "Coscheduling", {},
     {"permitWaitingTimeSeconds": 60, "deniedPGExpirationTimeSeconds": 20}),
    ("set non default CoschedulingArgs", "Coscheduling",
     {"permitWaitingTimeSeconds": 60, "deniedPGExpirationTimeSeconds": 10},
     {"permitWaitingTimeSeconds": 60, "deniedPGExpirationTimeSeconds": 10}),
    ("empty config NodeResourcesAllocatableArgs", "NodeResourcesAllocatable", {},
     {"resources": [{"name": "cpu", "weight": 1 << 20}, {"name": "memory", "weight": 1}], "mode": "Least"}),
    ("set non default NodeResourcesAllocatableArgs", "NodeResourcesAllocatable",
     {"resources": [{"name": "cpu", "weight": 1 << 10}, {"name": "memory", "weight": 2}], "mode": "Most"},
     {"resources": [{"name": "cpu", "weight": 1 << 10}, {"name": "memory", "weight": 2}], "mode": "Most"}),
    ("empty config TargetLoadPackingArgs", "TargetLoadPacking", {},
     {"defaultRequests": {"cpu": "1000m"}, "defaultRequestsMultiplier": "1.5", "targetUtilization": 40,
      "metricProvider": {"type": "KubernetesMetricsServer"}, "resourceType": "CPU"}),
    ("set non default TargetLoadPackingArgs", "TargetLoadPacking",
     {"defaultRequests": {"cpu": "100m"}, "defaultRequestsMultiplier": "2.5", "targetUtilization": 50,
      "watcherAddress": "http://localhost:2020"},
     {"defaultRequests": {"cpu": "100m"}, "defaultRequestsMultiplier": "2.5", "targetUtilization": 50,
      "watcherAddress": "http://localhost:2020", "metricProvider": {}, "resourceType": "CPU"}),
    ("empty config LoadVariationRiskBalancingArgs", "LoadVariationRiskBalancing", {},
     {"metricProvider": {"type": "KubernetesMetricsServer"}, "safeVarianceMargin": 1.0,
      "safeVarianceSensitivity": 1.0}),
    ("set non default LoadVariationRiskBalancingArgs", "LoadVariationRiskBalancing",
     {"safeVarianceMargin": 2.0, "safeVarianceSensitivity": 2.0},
     {"metricProvider": {"type": "KubernetesMetricsServer"}, "safeVarianceMargin": 2.0,
      "safeVarianceSensitivity": 2.0}),
    ("empty config NodeResourceTopologyMatchArgs", "NodeResourceTopologyMatch", {},
     {"scoringStrategy": {"type": "LeastAllocated", "resources": [{"name": "cpu", "weight": 1},
                                                                  {"name": "memory", "weight": 1}]}}),
    ("empty config PreeemptionTolerationArgs", "PreemptionToleration", {},
     {"minCandidateNodesPercentage": 10, "minCandidateNodesAbsolute": 100}),
]


@pytest.mark.parametrize("name,plugin,args,want", DEFAULTS_CASES, ids=[c[0] for c in DEFAULTS_CASES])
def test_set_defaults(name, plugin, args, want):
    assert default_plugin_args(plugin, args) == want


@pytest.mark.parametrize("plugin,args", [
    ("NodeResourcesAllocatable", {"mode": "Sideways"}),
    ("TargetLoadPacking", {"resourceType": "TPU"}),
    ("NodeResourceTopologyMatch", {"scoringStrategy": {"type": "Random"}}),
    ("PreemptionToleration", {"minCandidateNodesPercentage": 0, "minCandidateNodesAbsolute": 0}),
    ("PreemptionToleration", {"minCandidateNodesPercentage": 101}),
    ("Coscheduling", {"permitWaitingTimeSeconds": -1}),
])
def test_validation_errors(plugin, args):
    with pytest.raises(ConfigError):
        default_plugin_args(plugin, args)


def test_flagship_config_uses_v1beta3_weights():
    from flex_gpu_scheduler_amd.utils.workload import flagship_config

    w = load_config(flagship_config()).profiles[0].score_weights
    assert w["TaintToleration"] == 3 and w["NodeAffinity"] == 2 and w["NodeResourceTopologyMatch"] == 2


def test_selector_spread_is_ignored_with_a_warning(caplog):
    import logging

    from flex_gpu_scheduler_amd import load_config

    with caplog.at_level(logging.WARNING, logger="flex_gpu_scheduler_amd.config"):
        c = load_config({"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
                         "profiles": [{"schedulerName": "s", "plugins": {
                             "preScore": {"enabled": [{"name": "SelectorSpread"}]},
                             "score": {"enabled": [{"name": "SelectorSpread", "weight": 1}]}}}]})
    assert "SelectorSpread" not in c.profiles[0].plugins["score"]
    assert any("SelectorSpread" in r.getMessage() and "ignored" in r.getMessage() for r in caplog.records)
