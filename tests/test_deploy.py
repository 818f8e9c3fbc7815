"""Deploy artifacts: Helm charts render to valid objects whose embedded
scheduler configuration loads (reference: manifests/flexgpu,
manifests/install/charts/as-a-second-scheduler), sample configs per plugin
load (manifests/*/scheduler-config.yaml), and the generated CRDs accept the
example objects (manifests/*/crd.yaml)."""
import glob
import os

import pytest
import yaml

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.cli import load_objects
from flex_gpu_scheduler_amd.deploy import crds
from flex_gpu_scheduler_amd.deploy.helm import Renderer, render_chart

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHARTS = os.path.join(ROOT, "deploy", "charts")


def _config_from(objs):
    (cm,) = [o for o in objs if o["kind"] == "ConfigMap"]
    return load_config(yaml.safe_load(cm["data"]["scheduler-config.yaml"]))


@pytest.mark.parametrize("values", [None, "values.dev.yaml", "values.prod.yaml"])
def test_flexgpu_chart_renders(values):
    vals = None
    if values:
        with open(os.path.join(CHARTS, "flexgpu", values)) as f:
            vals = yaml.safe_load(f)
    objs = render_chart(os.path.join(CHARTS, "flexgpu"), vals)
    kinds = sorted(o["kind"] for o in objs)
    assert kinds == ["ClusterRole", "ClusterRoleBinding", "ConfigMap", "DaemonSet", "Deployment", "ServiceAccount"]
    cfg = _config_from(objs)
    prof = cfg.profile("flex-gpu-scheduler")
    assert prof.plugins["bind"] == ["FlexGPU"]
    assert "FlexGPU" in prof.plugins["filter"] and "Coscheduling" in prof.plugins["permit"]
    assert prof.score_weights["NodeResourceTopologyMatch"] == 2
    dep = next(o for o in objs if o["kind"] == "Deployment")
    cmd = dep["spec"]["template"]["spec"]["containers"][0]["command"]
    assert cmd[:3] == ["python", "-m", "flex_gpu_scheduler_amd"] and "scheduler" in cmd
    if values == "values.prod.yaml":
        assert dep["spec"]["replicas"] == 2 and "--leader-elect" in cmd and cfg.leader_elect
    if values == "values.dev.yaml":
        assert "--v=6" in cmd and "--trace" in cmd


def test_flexgpu_chart_reference_profile():
    """gang + xGMI off = the reference chart's FlexGPU-only profile
    (manifests/flexgpu/templates/configmap.yaml:13-28)."""
    objs = render_chart(os.path.join(CHARTS, "flexgpu"), {"scheduler": {"gang": {"enabled": False},
                                                                      "xgmiPlacement": {"enabled": False}},
                                                        "nodeAgent": {"enabled": False}})
    prof = _config_from(objs).profile("flex-gpu-scheduler")
    # v1beta2 defaults keep VolumeBinding at Reserve ahead of FlexGPU, as upstream.
    assert prof.plugins["reserve"] == ["VolumeBinding", "FlexGPU"] and prof.plugins["score"][-1] == "FlexGPU"
    assert "Coscheduling" not in prof.plugins.get("permit", [])
    assert not any(o["kind"] == "DaemonSet" for o in objs)


def test_second_scheduler_chart_builds_profile_from_values():
    objs = render_chart(os.path.join(CHARTS, "as-a-second-scheduler"))
    cfg = _config_from(objs)
    prof = cfg.profile("scheduler-plugins-scheduler")
    assert prof.plugins["queueSort"] == ["Coscheduling"]
    assert prof.plugins["preFilter"][-2:] == ["Coscheduling", "CapacityScheduling"]
    assert "NodeResourceTopologyMatch" in prof.plugins["filter"]
    assert "NodeResourcesAllocatable" in prof.plugins["score"]
    deps = {o["metadata"]["name"] for o in objs if o["kind"] == "Deployment"}
    assert deps == {"scheduler-plugins-scheduler", "scheduler-plugins-controller"}
    # Every plugin the chart can enable exists in the native registry (the
    # reference binary registers only FlexGPU).
    from flex_gpu_scheduler_amd._native import native
    names = set(native().plugin_names())
    vals = Renderer(os.path.join(CHARTS, "as-a-second-scheduler")).values
    assert set(vals["plugins"]["enabled"]) <= names
    # The rendered profile builds a working native scheduler.
    from flex_gpu_scheduler_amd import Store
    s = new_scheduler(Store(), cfg)
    s.stop()
    lw = render_chart(os.path.join(CHARTS, "as-a-second-scheduler"), {"loadWatcher": {"enabled": True}})
    assert {o["kind"] for o in lw} >= {"Service"}


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(ROOT, "deploy", "examples", "*-config.yaml"))),
                         ids=os.path.basename)
def test_example_configs_load(path):
    cfg = load_config(path)
    from flex_gpu_scheduler_amd import Store
    s = new_scheduler(Store(), cfg)
    s.stop()


# ----------------------------------------------------------------- CRDs ---
def _validate(schema: dict, value, path="$"):
    if schema.get("x-kubernetes-int-or-string"):
        assert isinstance(value, (int, str)), path
        return
    t = schema.get("type")
    if t == "object":
        assert isinstance(value, dict), path
        for k, v in value.items():
            if k in schema.get("properties", {}):
                _validate(schema["properties"][k], v, f"{path}.{k}")
            elif "additionalProperties" in schema:
                _validate(schema["additionalProperties"], v, f"{path}.{k}")
        for r in schema.get("required", []):
            assert r in value, f"{path}.{r} required"
    elif t == "array":
        assert isinstance(value, list), path
        for i, v in enumerate(value):
            _validate(schema["items"], v, f"{path}[{i}]")
    elif t == "integer":
        assert isinstance(value, int), path
    elif t == "string":
        assert isinstance(value, str), path
        if "enum" in schema:
            assert value in schema["enum"], path
    elif t == "number":
        assert isinstance(value, (int, float)), path


def test_crds_written_match_generator(tmp_path):
    crds.write_all(str(tmp_path))
    for fn in crds.ALL:
        assert (tmp_path / fn).read_text() == open(os.path.join(ROOT, "deploy", "crds", fn)).read(), \
            f"deploy/crds/{fn} is stale: run python -m flex_gpu_scheduler_amd.deploy.crds deploy/crds"


def test_examples_validate_against_crds():
    from flex_gpu_scheduler_amd.models import mi355x_nrt
    schemas = {}
    for make in crds.ALL.values():
        c = make()
        schemas[c["spec"]["names"]["kind"]] = c["spec"]["versions"][0]["schema"]["openAPIV3Schema"]
        assert c["metadata"]["name"] == f"{c['spec']['names']['plural']}.{c['spec']['group']}"
    objs = load_objects(os.path.join(ROOT, "deploy", "examples", "elasticquota-example.yaml"))
    objs += [o for o in load_objects(os.path.join(ROOT, "deploy", "examples", "gang-8rank-example.yaml"))
             if o["kind"] == "PodGroup"]
    objs.append(dict(mi355x_nrt("n0"), apiVersion="topology.node.k8s.io/v1alpha1", kind="NodeResourceTopology"))
    from flex_gpu_scheduler_amd.gpu.telemetry import NodeTelemetry, Sample
    t = NodeTelemetry("n0")
    t.add(Sample(1.0, 10, 20, 30, 40))
    objs.append(dict(t.watcher_metrics(now=2), apiVersion="xsched.amd.com/v1alpha1", kind="WatcherMetrics"))
    assert {o["kind"] for o in objs} == set(schemas)
    for o in objs:
        _validate(schemas[o["kind"]], o)
    with pytest.raises(AssertionError):
        _validate(schemas["PodGroup"], {"spec": {"minMember": "two"}})
