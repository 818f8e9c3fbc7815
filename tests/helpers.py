"""Shared test helpers: build a scheduler over a store and wait for binds."""
import json
import time

from flex_gpu_scheduler_amd import load_config, new_scheduler


def coscheduling_config(extra_plugins: dict | None = None, permit_wait=10, denied=3, **profile) -> dict:
    plugins = {
        "queueSort": {"enabled": [{"name": "Coscheduling"}], "disabled": [{"name": "*"}]},
        "preFilter": {"enabled": [{"name": "Coscheduling"}]},
        "postFilter": {"enabled": [{"name": "Coscheduling"}]},
        "permit": {"enabled": [{"name": "Coscheduling"}]},
        "reserve": {"enabled": [{"name": "Coscheduling"}]},
        "postBind": {"enabled": [{"name": "Coscheduling"}]},
    }
    for pt, spec in (extra_plugins or {}).items():
        cur = plugins.setdefault(pt, {})
        for k, v in spec.items():
            cur.setdefault(k, []).extend(v)
    return {
        "apiVersion": "kubescheduler.config.k8s.io/v1beta2",
        "kind": "KubeSchedulerConfiguration",
        "profiles": [{"schedulerName": "default-scheduler", "plugins": plugins,
                      "pluginConfig": [{"name": "Coscheduling", "args": {
                          "permitWaitingTimeSeconds": permit_wait, "deniedPGExpirationTimeSeconds": denied}}],
                      **profile}],
    }


FLEXGPU_PLUGINS = {
    "filter": {"enabled": [{"name": "FlexGPU"}]},
    "score": {"enabled": [{"name": "FlexGPU"}]},
    "reserve": {"enabled": [{"name": "FlexGPU"}]},
    "bind": {"enabled": [{"name": "FlexGPU"}], "disabled": [{"name": "DefaultBinder"}]},
}


def start(store, cfg, **opts):
    return new_scheduler(store, load_config(cfg), start=True, **opts)


def wait_bound(sched, n, timeout=20.0):
    t0 = time.time()
    while sched.stats()["bound"] < n:
        if time.time() - t0 > timeout:
            raise AssertionError(f"timeout waiting for {n} binds: {sched.stats()} {sched.queue_counts()}")
        time.sleep(0.001)


def placements(store, ns="default"):
    pods, _ = store.list("pods", ns)
    return {p["metadata"]["name"]: p["spec"].get("nodeName", "") for p in pods}


def annotations(store, name, ns="default"):
    return store.get("pods", ns, name)["metadata"].get("annotations", {})


def create_all(store, kind, objs):
    store.create_many(kind, json.dumps(objs))
