"""KubeSchedulerConfiguration loading, plugin-set resolution and plugin-args
defaulting.

Accepts the same YAML the reference ships (``kubescheduler.config.k8s.io``
v1beta2 and v1beta3, e.g. manifests/flexgpu/templates/configmap.yaml and
manifests/*/scheduler-config.yaml) and resolves it into the flat per-profile
plugin lists the native framework consumes.

Semantics reproduced:
  * mergePluginSet: a re-enabled default keeps its position and takes the
    user's weight, other ``enabled`` plugins are appended, ``disabled``
    removes defaults (``"*"`` removes all);
  * v1beta3: defaults live in ``multiPoint`` with v1beta3's weights, and each
    point expands as frameworkImpl.expandMultiPointPlugins does (explicit
    point plugins first, then the multiPoint plugins implementing it);
  * plugin args defaults of apis/config/v1beta2/defaults.go:28-157
    (identical in v1beta3) and upstream DefaultPreemptionArgs;
  * strict decoding: unknown fields are errors, at the top level, in
    leaderElection / clientConnection / profiles / plugin sets / extenders
    and in every plugin's args (apis/config/scheme/scheme.go:35 uses the
    strict codec);
  * extenders (kube-scheduler/config/v1beta{2,3} Extender): validated as
    validation.go validateExtenders does (positive weight with a prioritize
    verb, at most one binder, unique extended managedResources), ignorable
    extenders moved to the tail and ignoredByScheduler resources written into
    every profile's NodeResourcesFit ignoredResources (factory.go:90-130).
"""
from __future__ import annotations

import base64
import copy
import json
import logging
import re
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any

import yaml

_log = logging.getLogger(__name__)

API_VERSIONS = ("kubescheduler.config.k8s.io/v1beta2", "kubescheduler.config.k8s.io/v1beta3")
EXT_POINTS = ("queueSort", "preFilter", "filter", "postFilter", "preScore", "score", "reserve", "permit",
              "preBind", "bind", "postBind")

# Extension points each native plugin implements (csrc/plugins/*.cc).
PLUGIN_POINTS: dict[str, tuple[str, ...]] = {
    # in-tree defaults
    "PrioritySort": ("queueSort",),
    "NodeUnschedulable": ("filter",),
    "NodeName": ("filter",),
    "NodePorts": ("preFilter", "filter"),
    "NodeResourcesFit": ("preFilter", "filter", "score"),
    "NodeResourcesBalancedAllocation": ("score",),
    "TaintToleration": ("filter", "preScore", "score"),
    "NodeAffinity": ("preFilter", "filter", "preScore", "score"),
    "PodTopologySpread": ("preFilter", "filter", "preScore", "score"),
    "InterPodAffinity": ("preFilter", "filter", "preScore", "score"),
    "ImageLocality": ("score",),
    "DefaultPreemption": ("postFilter",),
    "DefaultBinder": ("bind",),
    "VolumeRestrictions": ("preFilter", "filter"),
    # Score: 0 everywhere without the alpha VolumeCapacityPriority gate, but
    # listed, as upstream's multiPoint expansion lists it.
    "VolumeBinding": ("preFilter", "filter", "score", "reserve", "preBind"),
    "VolumeZone": ("filter",),
    "NodeVolumeLimits": ("filter",),
    "EBSLimits": ("filter",),
    "GCEPDLimits": ("filter",),
    "AzureDiskLimits": ("filter",),
    "CinderLimits": ("filter",),
    # out-of-tree (the reference's pkg/*)
    "FlexGPU": ("filter", "score", "reserve", "bind"),
    "Coscheduling": ("queueSort", "preFilter", "postFilter", "reserve", "permit", "postBind"),
    "CapacityScheduling": ("preFilter", "postFilter", "reserve"),
    "NodeResourcesAllocatable": ("score",),
    "NodeResourceTopologyMatch": ("preFilter", "filter", "preScore", "score"),
    "TargetLoadPacking": ("score",),
    "LoadVariationRiskBalancing": ("score",),
    "PreemptionToleration": ("postFilter",),
    "CrossNodePreemption": ("postFilter",),
    "PodState": ("score",),
    "QOSSort": ("queueSort",),
}

# SelectorSpread (deprecated, not in 1.23's default set) is accepted in configs
# and ignored.
NOT_APPLICABLE = {"SelectorSpread"}

# kube-scheduler 1.23 v1beta2 default plugin set (default_plugins.go:34-106).
DEFAULT_PLUGINS: dict[str, list[tuple[str, int]]] = {
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
    "reserve": [("VolumeBinding", 0)],
    "permit": [],
    "preBind": [("VolumeBinding", 0)],
    "bind": [("DefaultBinder", 0)],
    "postBind": [],
}


# kube-scheduler 1.23 v1beta3 defaults: every default plugin in multiPoint,
# with v1beta3's own score weights (v1beta3/default_plugins.go:30-56).
V1BETA3_MULTIPOINT: list[tuple[str, int]] = [
    ("PrioritySort", 0), ("NodeUnschedulable", 0), ("NodeName", 0), ("TaintToleration", 3), ("NodeAffinity", 2),
    ("NodePorts", 0), ("NodeResourcesFit", 1), ("VolumeRestrictions", 0), ("EBSLimits", 0), ("GCEPDLimits", 0),
    ("NodeVolumeLimits", 0), ("AzureDiskLimits", 0), ("VolumeBinding", 0), ("VolumeZone", 0),
    ("PodTopologySpread", 2), ("InterPodAffinity", 2), ("DefaultPreemption", 0),
    ("NodeResourcesBalancedAllocation", 1), ("ImageLocality", 1), ("DefaultBinder", 0),
]


class ConfigError(ValueError):
    pass


# Top-level fields of KubeSchedulerConfiguration (kube-scheduler/config/
# v1beta{2,3}/types.go; DebuggingConfiguration is inlined). v1beta3 dropped
# the two bind addresses.
_TOP_FIELDS = {"apiVersion", "kind", "parallelism", "leaderElection", "clientConnection", "enableProfiling",
               "enableContentionProfiling", "percentageOfNodesToScore", "podInitialBackoffSeconds",
               "podMaxBackoffSeconds", "profiles", "extenders"}
_V1BETA2_ONLY = {"healthzBindAddress", "metricsBindAddress"}
_LEADER_FIELDS = {"leaderElect", "leaseDuration", "renewDeadline", "retryPeriod", "resourceLock", "resourceName",
                  "resourceNamespace"}
_CLIENT_FIELDS = {"kubeconfig", "acceptContentTypes", "contentType", "qps", "burst"}
# percentageOfNodesToScore per profile is an extension of this scheduler
# (upstream added it in v1); the rest is KubeSchedulerProfile.
_PROFILE_FIELDS = {"schedulerName", "plugins", "pluginConfig", "percentageOfNodesToScore"}
_EXTENDER_FIELDS = {"urlPrefix", "filterVerb", "preemptVerb", "prioritizeVerb", "weight", "bindVerb", "enableHTTPS",
                    "tlsConfig", "httpTimeout", "nodeCacheCapable", "managedResources", "ignorable"}
_EXTENDER_TLS_FIELDS = {"insecure", "serverName", "certFile", "keyFile", "caFile", "certData", "keyData", "caData"}


def _strict_fields(where: str, obj: Any, allowed: set[str]) -> None:
    if obj is None:
        return
    if not isinstance(obj, dict):
        raise ConfigError(f"{where}: expected an object, got {type(obj).__name__}")
    extra = set(obj) - allowed
    if extra:
        raise ConfigError("strict decoding error: " + ", ".join(
            f'unknown field "{where + "." if where else ""}{f}"' for f in sorted(extra)))


_DURATION = re.compile(r"(\d+(?:\.\d*)?|\.\d+)(ns|us|µs|ms|s|m|h)")


def parse_duration_ms(v: Any, where: str) -> int:
    """metav1.Duration (Go time.ParseDuration syntax, e.g. "30s", "1m30s",
    "250ms") -> milliseconds. A bare number is taken as seconds."""
    if v is None or v == "":
        return 0
    if isinstance(v, (int, float)):
        return int(float(v) * 1000)
    s = str(v).strip()
    if s in ("0", "0s"):
        return 0
    scale = {"ns": 1e-6, "us": 1e-3, "µs": 1e-3, "ms": 1.0, "s": 1e3, "m": 60e3, "h": 3600e3}
    pos, total = 0, 0.0
    for m in _DURATION.finditer(s):
        if m.start() != pos:
            break
        total += float(m.group(1)) * scale[m.group(2)]
        pos = m.end()
    if pos != len(s) or pos == 0:
        raise ConfigError(f"{where}: invalid duration {v!r}")
    return int(round(total))


_QUALIFIED = re.compile(r"^([a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*)/"
                        r"([A-Za-z0-9]([-A-Za-z0-9_.]*[A-Za-z0-9])?)$")


def _extended_resource_name(name: str) -> bool:
    """validateExtendedResourceName: a domain-prefixed name outside
    kubernetes.io that is not a requests.* quota name."""
    m = _QUALIFIED.match(name or "")
    if not m:
        return False
    domain = m.group(1)
    if domain == "kubernetes.io" or domain.endswith(".kubernetes.io"):
        return False
    return not name.startswith("requests.")


def _pem(v: Any, where: str) -> str:
    """[]byte fields arrive base64-encoded (JSON/YAML of a Go byte slice)."""
    if not v:
        return ""
    try:
        return base64.b64decode(str(v), validate=True).decode()
    except Exception as e:  # noqa: BLE001
        raise ConfigError(f"{where}: not base64 data: {e}") from None


def resolve_extenders(raw: Any) -> tuple[list[dict], list[str]]:
    """Validated, defaulted extenders (non-ignorable first) and the resources
    they ask the scheduler to ignore."""
    if raw is None:
        return [], []
    if not isinstance(raw, list):
        raise ConfigError("extenders must be a list")
    out, ignorable, ignored, seen = [], [], [], set()
    binders = 0
    for i, e in enumerate(raw):
        where = f"extenders[{i}]"
        _strict_fields(where, e, _EXTENDER_FIELDS)
        if not isinstance(e, dict) or not e.get("urlPrefix"):
            raise ConfigError(f"{where}.urlPrefix: required")
        url = str(e["urlPrefix"])
        if not (url.startswith("http://") or url.startswith("https://")):
            raise ConfigError(f"{where}.urlPrefix: must be an http:// or https:// URL, got {url!r}")
        weight = int(e.get("weight") or 0)
        if e.get("prioritizeVerb") and weight <= 0:
            raise ConfigError(f"{where}.weight: Invalid value: {weight}: must have a positive weight applied to it")
        if e.get("bindVerb"):
            binders += 1
        managed = []
        for j, r in enumerate(e.get("managedResources") or []):
            _strict_fields(f"{where}.managedResources[{j}]", r, {"name", "ignoredByScheduler"})
            name = str((r or {}).get("name", ""))
            if not _extended_resource_name(name):
                raise ConfigError(f"{where}.managedResources[{j}].name: Invalid value: {name!r}: "
                                  "must be a fully qualified extended resource name")
            if name in seen:
                raise ConfigError(f"{where}.managedResources[{j}].name: Invalid value: {name!r}: "
                                  "duplicate extender managed resource name")
            seen.add(name)
            managed.append({"name": name, "ignoredByScheduler": bool(r.get("ignoredByScheduler", False))})
            if r.get("ignoredByScheduler"):
                ignored.append(name)
        tls = e.get("tlsConfig") or {}
        _strict_fields(f"{where}.tlsConfig", tls, _EXTENDER_TLS_FIELDS)
        ext = {
            "urlPrefix": url,
            "filterVerb": str(e.get("filterVerb") or ""),
            "preemptVerb": str(e.get("preemptVerb") or ""),
            "prioritizeVerb": str(e.get("prioritizeVerb") or ""),
            "bindVerb": str(e.get("bindVerb") or ""),
            "weight": weight,
            "enableHTTPS": bool(e.get("enableHTTPS", False)),
            "nodeCacheCapable": bool(e.get("nodeCacheCapable", False)),
            "ignorable": bool(e.get("ignorable", False)),
            "managedResources": managed,
            "httpTimeoutMs": parse_duration_ms(e.get("httpTimeout"), f"{where}.httpTimeout"),
            "tlsConfig": {"insecure": bool(tls.get("insecure", False)), "serverName": str(tls.get("serverName") or ""),
                          "certFile": str(tls.get("certFile") or ""), "keyFile": str(tls.get("keyFile") or ""),
                          "caFile": str(tls.get("caFile") or ""),
                          "certData": _pem(tls.get("certData"), f"{where}.tlsConfig.certData"),
                          "keyData": _pem(tls.get("keyData"), f"{where}.tlsConfig.keyData"),
                          "caData": _pem(tls.get("caData"), f"{where}.tlsConfig.caData")},
        }
        (ignorable if ext["ignorable"] else out).append(ext)
    if binders > 1:
        raise ConfigError(f"extenders: Invalid value: \"found {binders} extenders implementing bind\": "
                          "only one extender can implement bind")
    return out + ignorable, ignored


# ----------------------------------------------------------------- args ----
def _strict(name: str, args: dict, allowed: set[str]) -> None:
    extra = set(args) - allowed - {"apiVersion", "kind"}
    if extra:
        raise ConfigError("strict decoding error: " + ", ".join(f'unknown field "{f}"' for f in sorted(extra)))


def _resource_specs(v: Any, where: str) -> list[dict]:
    if v is None:
        return []
    if not isinstance(v, list):
        raise ConfigError(f"{where}: resources must be a list")
    out = []
    for r in v:
        if not isinstance(r, dict) or "name" not in r:
            raise ConfigError(f"{where}: resource spec needs a name")
        out.append({"name": str(r["name"]), "weight": int(r.get("weight", 0))})
    return out


def _metric_provider(args: dict, where: str) -> dict:
    mp = dict(args.get("metricProvider") or {})
    _strict(where + ".metricProvider", mp, {"type", "address", "token", "insecureSkipVerify"})
    return mp


def default_plugin_args(name: str, args: dict | None) -> dict:
    """Apply SetDefaults_<Name>Args (apis/config/v1beta2/defaults.go)."""
    a = copy.deepcopy(args or {})
    if name == "Coscheduling":
        # transientShortage (Park | Deny) is this framework's extension (the
        # native plugin defaults it to Park; docs/ARCHITECTURE.md §4).
        _strict(name, a, {"permitWaitingTimeSeconds", "deniedPGExpirationTimeSeconds", "transientShortage"})
        if a.get("transientShortage", "Park") not in ("Park", "Deny"):
            raise ConfigError(f"{name}Args.transientShortage must be Park or Deny, got {a['transientShortage']!r}")
        a.setdefault("permitWaitingTimeSeconds", 60)
        a.setdefault("deniedPGExpirationTimeSeconds", 20)
        for k in ("permitWaitingTimeSeconds", "deniedPGExpirationTimeSeconds"):
            if int(a[k]) < 0:
                raise ConfigError(f"{name}Args.{k} must be >= 0")
    elif name == "NodeResourcesAllocatable":
        _strict(name, a, {"resources", "mode"})
        res = _resource_specs(a.get("resources"), name)
        a["resources"] = res or [{"name": "cpu", "weight": 1 << 20}, {"name": "memory", "weight": 1}]
        a["mode"] = a.get("mode") or "Least"
        if a["mode"] not in ("Least", "Most"):
            raise ConfigError(f"{name}Args.mode must be Least or Most, got {a['mode']!r}")
    elif name == "TargetLoadPacking":
        _strict(name, a, {"defaultRequests", "defaultRequestsMultiplier", "targetUtilization", "metricProvider",
                          "watcherAddress", "resourceType"})
        a.setdefault("defaultRequests", {"cpu": "1000m"})
        a["resourceType"] = a.get("resourceType") or "CPU"
        if a["resourceType"] not in ("CPU", "GPU", "GPUMemoryBandwidth"):
            raise ConfigError(f"{name}Args.resourceType must be CPU, GPU or GPUMemoryBandwidth, "
                              f"got {a['resourceType']!r}")
        if a.get("defaultRequestsMultiplier") is None:
            a["defaultRequestsMultiplier"] = "1.5"
        if a.get("targetUtilization") is None or int(a["targetUtilization"]) <= 0:
            a["targetUtilization"] = 40
        mp = _metric_provider(a, name)
        if a.get("watcherAddress") is None and not mp.get("type"):
            mp["type"] = "KubernetesMetricsServer"
        if mp.get("type") == "Prometheus" and mp.get("insecureSkipVerify") is None:
            mp["insecureSkipVerify"] = True
        a["metricProvider"] = mp
    elif name == "LoadVariationRiskBalancing":
        _strict(name, a, {"metricProvider", "watcherAddress", "safeVarianceMargin", "safeVarianceSensitivity"})
        mp = _metric_provider(a, name)
        if a.get("watcherAddress") is None and not mp.get("type"):
            mp["type"] = "KubernetesMetricsServer"
        if mp.get("type") == "Prometheus" and mp.get("insecureSkipVerify") is None:
            mp["insecureSkipVerify"] = True
        a["metricProvider"] = mp
        if a.get("safeVarianceMargin") is None or float(a["safeVarianceMargin"]) < 0:
            a["safeVarianceMargin"] = 1.0
        if a.get("safeVarianceSensitivity") is None or float(a["safeVarianceSensitivity"]) < 0:
            a["safeVarianceSensitivity"] = 1.0
    elif name == "NodeResourceTopologyMatch":
        # gangColocation (Preferred | Required | None) is this framework's
        # extension: xGMI gang co-location in PreFilter (native default:
        # Preferred with XGMIGangAffinity, None otherwise).
        _strict(name, a, {"scoringStrategy", "gangColocation"})
        if a.get("gangColocation", "Preferred") not in ("Preferred", "Required", "None"):
            raise ConfigError(f"{name}Args.gangColocation must be Preferred, Required or None, "
                              f"got {a['gangColocation']!r}")
        ss = dict(a.get("scoringStrategy") or {})
        _strict(name + ".scoringStrategy", ss, {"type", "resources"})
        ss.setdefault("type", "LeastAllocated")
        if ss["type"] not in ("LeastAllocated", "MostAllocated", "BalancedAllocation", "XGMIGangAffinity"):
            raise ConfigError(f"{name}Args.scoringStrategy.type {ss['type']!r} is not supported")
        res = _resource_specs(ss.get("resources"), name) or [{"name": "cpu", "weight": 1}, {"name": "memory", "weight": 1}]
        for r in res:
            if r["weight"] == 0:
                r["weight"] = 1
        ss["resources"] = res
        a["scoringStrategy"] = ss
    elif name in ("PreemptionToleration", "DefaultPreemption"):
        _strict(name, a, {"minCandidateNodesPercentage", "minCandidateNodesAbsolute"})
        a.setdefault("minCandidateNodesPercentage", 10)
        a.setdefault("minCandidateNodesAbsolute", 100)
        p, n = int(a["minCandidateNodesPercentage"]), int(a["minCandidateNodesAbsolute"])
        if not 0 <= p <= 100:
            raise ConfigError(f"{name}Args.minCandidateNodesPercentage must be in [0, 100]")
        if n < 0 or (p == 0 and n == 0):
            raise ConfigError(f"{name}Args: both minCandidateNodes values cannot be zero")
    elif name == "CrossNodePreemption":
        # No Args type upstream (the plugin is commented out); these bound the
        # minimum-victim subset search (csrc/plugins/crossnode.cc).
        _strict(name, a, {"maxVictims", "maxPoolPods", "maxCombinations"})
        a.setdefault("maxVictims", 3)
        a.setdefault("maxPoolPods", 32)
        a.setdefault("maxCombinations", 20000)
        for k in ("maxVictims", "maxPoolPods", "maxCombinations"):
            if int(a[k]) < 1:
                raise ConfigError(f"{name}Args.{k} must be >= 1")
    elif name == "FlexGPU":
        _strict(name, a, {"gpuResourceName", "memoryResourceName", "xcdResourceName", "indexAnnotationKey",
                          "partitionAnnotationKey"})
        a.setdefault("gpuResourceName", "amd.com/gpu")
        a.setdefault("memoryResourceName", "amd.com/gpu-memory")
        a.setdefault("xcdResourceName", "amd.com/gpu-xcd")
        a.setdefault("indexAnnotationKey", "amd.com/gpu-index")
        a.setdefault("partitionAnnotationKey", "amd.com/gpu-partitions")
    elif name == "NodeResourcesFit":
        # unresolvableBeyondAllocatable is an extension (default off = k8s
        # 1.23): a request above the node's allocatable fails the node as
        # UnschedulableAndUnresolvable, so preemption does not try it.
        _strict(name, a, {"ignoredResources", "ignoredResourceGroups", "scoringStrategy",
                          "unresolvableBeyondAllocatable"})
        ss = dict(a.get("scoringStrategy") or {})
        ss.setdefault("type", "LeastAllocated")
        ss["resources"] = _resource_specs(ss.get("resources"), name) or [
            {"name": "cpu", "weight": 1}, {"name": "memory", "weight": 1}]
        a["scoringStrategy"] = ss
    elif name == "NodeResourcesBalancedAllocation":
        _strict(name, a, {"resources"})
        a["resources"] = _resource_specs(a.get("resources"), name) or [
            {"name": "cpu", "weight": 1}, {"name": "memory", "weight": 1}]
    elif name == "PodTopologySpread":
        _strict(name, a, {"defaultConstraints", "defaultingType"})
        a.setdefault("defaultingType", "System")
    elif name == "InterPodAffinity":
        _strict(name, a, {"hardPodAffinityWeight"})
        a.setdefault("hardPodAffinityWeight", 1)
    elif name == "NodeAffinity":
        _strict(name, a, {"addedAffinity"})
    elif name == "VolumeBinding":
        # VolumeBindingArgs (v1beta2/types.go); `shape` needs the alpha
        # VolumeCapacityPriority gate, off in 1.23. pollIntervalMillis is an
        # extension (the reference polls every second).
        _strict(name, a, {"bindTimeoutSeconds", "shape", "pollIntervalMillis"})
        if a.get("shape"):
            raise ConfigError(f"{name}Args.shape: Invalid value: feature gate VolumeCapacityPriority is not enabled")
        a.setdefault("bindTimeoutSeconds", 600)
        if int(a["bindTimeoutSeconds"]) < 0:
            raise ConfigError(f"{name}Args.bindTimeoutSeconds: Invalid value: must be >= 0")
        a.setdefault("pollIntervalMillis", 100)
    elif name in ("VolumeRestrictions", "VolumeZone", "NodeVolumeLimits", "EBSLimits", "GCEPDLimits",
                  "AzureDiskLimits", "CinderLimits"):
        _strict(name, a, set())
    return a


# -------------------------------------------------------------- profiles ----
@dataclass
class Profile:
    scheduler_name: str = "default-scheduler"
    plugins: dict[str, list[str]] = field(default_factory=dict)
    score_weights: dict[str, int] = field(default_factory=dict)
    plugin_config: dict[str, dict] = field(default_factory=dict)
    percentage_of_nodes_to_score: int = 0

    def to_native(self) -> dict:
        plugins = {}
        for pt in EXT_POINTS:
            names = self.plugins.get(pt, [])
            if not names:
                continue
            if pt == "score":
                plugins[pt] = [{"name": n, "weight": self.score_weights.get(n, 1)} for n in names]
            else:
                plugins[pt] = list(names)
        used = {n for names in self.plugins.values() for n in names}
        return {
            "schedulerName": self.scheduler_name,
            "plugins": plugins,
            "pluginConfig": {n: a for n, a in self.plugin_config.items() if n in used},
            "percentageOfNodesToScore": self.percentage_of_nodes_to_score,
        }


@dataclass
class SchedulerConfiguration:
    profiles: list[Profile]
    parallelism: int = 16
    percentage_of_nodes_to_score: int = 0
    pod_initial_backoff_seconds: float = 1.0
    pod_max_backoff_seconds: float = 10.0
    leader_elect: bool = False
    client_qps: float = 0.0   # clientConnection.qps (0 = unthrottled)
    client_burst: int = 0     # clientConnection.burst
    bind_workers: int = 16
    status_updates: bool = True
    trace: bool = False
    api_version: str = API_VERSIONS[0]
    extenders: list[dict] = field(default_factory=list)
    raw: dict = field(default_factory=dict)

    def to_native(self, **overrides) -> dict:
        opts = {
            "parallelism": self.parallelism,
            "percentageOfNodesToScore": self.percentage_of_nodes_to_score,
            "podInitialBackoffSeconds": self.pod_initial_backoff_seconds,
            "podMaxBackoffSeconds": self.pod_max_backoff_seconds,
            "bindWorkers": self.bind_workers,
            "statusUpdates": self.status_updates,
            "trace": self.trace,
        }
        opts.update(overrides)
        return {"profiles": [p.to_native() for p in self.profiles], "options": opts, "extenders": self.extenders}

    def profile(self, name: str) -> Profile:
        for p in self.profiles:
            if p.scheduler_name == name:
                return p
        raise KeyError(name)


def _names(entries: Any) -> list[tuple[str, int]]:
    out = []
    for e in entries or []:
        if isinstance(e, str):
            out.append((e, 0))
        elif isinstance(e, dict) and "name" in e:
            out.append((str(e["name"]), int(e.get("weight", 0) or 0)))
        else:
            raise ConfigError(f"invalid plugin entry {e!r}")
    return out


def _merge_plugin_set(defaults: list[tuple[str, int]], custom: dict) -> tuple[list[tuple[str, int]], set[str]]:
    """mergePluginSet (v1beta2/v1beta3 default_plugins.go): a default plugin
    re-enabled by the user is replaced *in place* (order kept, the user's
    weight wins); disabled defaults are dropped ("*" drops all); the remaining
    custom plugins are appended in the user's order. Returns (enabled,
    disabled names)."""
    disabled = {n for n, _ in _names(custom.get("disabled"))}
    enabled = _names(custom.get("enabled"))
    custom_idx = {n: i for i, (n, _) in enumerate(enabled)}
    out: list[tuple[str, int]] = []
    replaced: set[int] = set()
    if "*" not in disabled:
        for n, w in defaults:
            if n in disabled:
                continue
            if n in custom_idx:
                i = custom_idx[n]
                replaced.add(i)
                out.append(enabled[i])
            else:
                out.append((n, w))
    out += [e for i, e in enumerate(enabled) if i not in replaced]
    return out, disabled


def _resolve_profile(p: dict, api_version: str, available: set[str] | None, index: int = 0) -> Profile:
    """Resolve one profile the way kube-scheduler 1.23 does.

    v1beta2: per extension point, mergePluginSet(DEFAULT_PLUGINS[pt], user).
    v1beta3: the defaults live in multiPoint (V1BETA3_MULTIPOINT, with the
    v1beta3 weights: TaintToleration 3, NodeAffinity / PodTopologySpread /
    InterPodAffinity 2); multiPoint = mergePluginSet(defaults, user
    multiPoint) and each point is expanded as in frameworkImpl.
    expandMultiPointPlugins (framework/runtime/framework.go:420-485): the
    point's explicit plugins first, then every multiPoint plugin implementing
    the point that the point neither disables nor configures explicitly; a
    point with "*" disabled gets no multiPoint plugins. Score weights: an
    explicit score entry wins, else the multiPoint weight, 0 meaning 1.
    """
    _strict_fields(f"profiles[{index}]", p, _PROFILE_FIELDS)
    prof = Profile(scheduler_name=p.get("schedulerName") or "default-scheduler")
    if "percentageOfNodesToScore" in p and p["percentageOfNodesToScore"] is not None:
        prof.percentage_of_nodes_to_score = int(p["percentageOfNodesToScore"])
    spec = p.get("plugins") or {}
    unknown = set(spec) - set(EXT_POINTS) - {"multiPoint"}
    if unknown:
        raise ConfigError(f"unknown extension point(s) {sorted(unknown)}")
    for pt, ps in spec.items():
        _strict_fields(f"profiles[{index}].plugins.{pt}", ps, {"enabled", "disabled"})
        for k in ("enabled", "disabled"):
            for j, e in enumerate((ps or {}).get(k) or []):
                if isinstance(e, dict):
                    _strict_fields(f"profiles[{index}].plugins.{pt}.{k}[{j}]", e, {"name", "weight"})
    v1beta3 = api_version.endswith("v1beta3")
    if "multiPoint" in spec and not v1beta3:
        raise ConfigError("multiPoint requires kubescheduler.config.k8s.io/v1beta3")
    mp: list[tuple[str, int]] = []
    if v1beta3:
        mp, _ = _merge_plugin_set(V1BETA3_MULTIPOINT, spec.get("multiPoint") or {})
    weights: dict[str, int] = {}
    resolved: dict[str, list[str]] = {}
    for pt in EXT_POINTS:
        if v1beta3:
            explicit, disabled = _merge_plugin_set([], spec.get(pt) or {})
            cur = list(explicit)
            if "*" not in disabled:
                seen = {n for n, _ in explicit}
                for n, w in mp:
                    if pt in PLUGIN_POINTS.get(n, ()) and n not in disabled and n not in seen:
                        cur.append((n, w))
                        seen.add(n)
        else:
            cur, _ = _merge_plugin_set(DEFAULT_PLUGINS[pt], spec.get(pt) or {})
        names = []
        for n, w in cur:
            if n in NOT_APPLICABLE:
                # Upstream registers it (spreading the pods of one Service /
                # ReplicaSet / StatefulSet, default_plugins.go:119-127 behind a
                # feature gate); this scheduler has no such controllers' objects.
                _log.warning('plugin "%s" (%s) is not implemented by this scheduler and is ignored', n, pt)
                continue
            if n not in PLUGIN_POINTS:
                raise ConfigError(f'plugin "{n}" does not exist')
            if pt not in PLUGIN_POINTS[n]:
                raise ConfigError(f'plugin "{n}" does not extend {pt} plugin')
            if n in names:
                raise ConfigError(f'plugin "{n}" already registered as "{pt}"')
            if available is not None and n not in available:
                continue  # registered in config tables but not compiled into this build
            names.append(n)
            if pt == "score":
                weights[n] = w if w > 0 else 1
        if pt == "queueSort" and len(names) > 1:
            raise ConfigError(f"profile {prof.scheduler_name}: only one queueSort plugin may be enabled, got {names}")
        resolved[pt] = names
    prof.plugins = resolved
    prof.score_weights = weights
    for j, pc in enumerate(p.get("pluginConfig") or []):
        _strict_fields(f"profiles[{index}].pluginConfig[{j}]", pc, {"name", "args"})
        name = pc.get("name")
        if not name:
            raise ConfigError("pluginConfig entry without name")
        try:
            prof.plugin_config[name] = default_plugin_args(name, pc.get("args"))
        except ConfigError as e:
            # the strict codec's error shape (apis/config/scheme/scheme_test.go:313)
            raise ConfigError(f"decoding .profiles[{index}].pluginConfig[{j}]: decoding args for plugin {name}: {e}") \
                from None
    used = {n for names in resolved.values() for n in names}
    for n in used:
        if n not in prof.plugin_config:
            prof.plugin_config[n] = default_plugin_args(n, None)
    return prof


def _available_plugins() -> set[str] | None:
    try:
        from ._native import native

        return set(native().plugin_names())
    except Exception:  # pragma: no cover - config parsing works without the core
        return None


def load_config(src: str | Path | dict | None = None, *, restrict_to_native: bool = True) -> SchedulerConfiguration:
    """Load a KubeSchedulerConfiguration from a YAML path/string or a dict."""
    if src is None:
        doc: dict = {"apiVersion": API_VERSIONS[0], "kind": "KubeSchedulerConfiguration"}
    elif isinstance(src, dict):
        doc = copy.deepcopy(src)
    else:
        text = Path(src).read_text() if (isinstance(src, Path) or (isinstance(src, str) and "\n" not in src
                                                                   and Path(src).exists())) else str(src)
        doc = yaml.safe_load(text) or {}
    api = doc.get("apiVersion", API_VERSIONS[0])
    if api not in API_VERSIONS:
        raise ConfigError(f"unsupported apiVersion {api!r}")
    if doc.get("kind", "KubeSchedulerConfiguration") != "KubeSchedulerConfiguration":
        raise ConfigError(f"unsupported kind {doc.get('kind')!r}")
    _strict_fields("", doc, _TOP_FIELDS | (_V1BETA2_ONLY if api.endswith("v1beta2") else set()))
    _strict_fields("leaderElection", doc.get("leaderElection"), _LEADER_FIELDS)
    _strict_fields("clientConnection", doc.get("clientConnection"), _CLIENT_FIELDS)
    extenders, ignored = resolve_extenders(doc.get("extenders"))
    available = _available_plugins() if restrict_to_native else None
    profiles_raw = doc.get("profiles") or [{"schedulerName": "default-scheduler"}]
    profiles = [_resolve_profile(p, api, available, i) for i, p in enumerate(profiles_raw)]
    names = [p.scheduler_name for p in profiles]
    if len(set(names)) != len(names):
        raise ConfigError(f"duplicate profile schedulerName in {names}")
    qs = {tuple(p.plugins.get("queueSort", [])) for p in profiles}
    if len(qs) > 1:
        raise ConfigError("all profiles must use the same queueSort plugin")
    if ignored:
        # factory.go:112-130: the extenders' ignoredByScheduler resources
        # replace every profile's NodeResourcesFit ignoredResources.
        for prof in profiles:
            if "NodeResourcesFit" in prof.plugin_config:
                prof.plugin_config["NodeResourcesFit"]["ignoredResources"] = list(ignored)
    cfg = SchedulerConfiguration(profiles=profiles, api_version=api, extenders=extenders, raw=doc)
    if doc.get("parallelism") is not None:
        cfg.parallelism = int(doc["parallelism"])
        if cfg.parallelism <= 0:
            raise ConfigError("parallelism must be > 0")
    if doc.get("percentageOfNodesToScore") is not None:
        cfg.percentage_of_nodes_to_score = int(doc["percentageOfNodesToScore"])
    if doc.get("podInitialBackoffSeconds") is not None:
        cfg.pod_initial_backoff_seconds = float(doc["podInitialBackoffSeconds"])
    if doc.get("podMaxBackoffSeconds") is not None:
        cfg.pod_max_backoff_seconds = float(doc["podMaxBackoffSeconds"])
    cfg.leader_elect = bool((doc.get("leaderElection") or {}).get("leaderElect", False))
    cc = doc.get("clientConnection") or {}
    # Upstream defaults qps 50 / burst 100 (a 1.23 kube-scheduler then binds at
    # most 50 pods/s); here the writer is unthrottled unless configured.
    cfg.client_qps = float(cc.get("qps") or 0)
    cfg.client_burst = int(cc.get("burst") or 0)
    if cfg.client_qps < 0 or cfg.client_burst < 0:
        raise ConfigError("clientConnection.qps and .burst must be >= 0")
    return cfg


def native_config_json(cfg: SchedulerConfiguration, **overrides) -> str:
    return json.dumps(cfg.to_native(**overrides))
