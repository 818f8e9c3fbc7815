"""The five BASELINE.json configurations as small, checked scenarios.

`bench.py`'s headline number is the mixed gang workload (utils/workload.py).
This module runs each named configuration on its own store and scheduler
(untimed by the bench contract; reported under `config.scenarios`), both to
measure it and to assert the placement property the configuration is about:

  coscheduling_cpu     PodGroups minMember=2 of CPU-only pods (plumbing)
  flexgpu_cpx_quarter  4 pods x 0.25 GPU (amd.com/gpu-xcd: 2) on one CPX MI355X
  gang8_xgmi           gangs of 2-8 ranks on 8x MI355X nodes with a real choice of
                       node, NRT XGMIGangAffinity + gangColocation
  capacity_preemption  2 namespaces contend for 8 MI355X (ElasticQuota + preemption)
  trimaran_tlp         TargetLoadPacking(GPU) fed by live amdgpu utilisation
"""
from __future__ import annotations

import json
import time
from typing import Callable

from ..config import load_config
from ..models.mi355x import GPU, GPU_XCD, INDEX_ANNOTATION, PARTITION_ANNOTATION, mi355x_node, mi355x_nrt
from ..models.objects import make_elastic_quota, make_node, make_pod, make_pod_group
from ..scheduler import Store, new_scheduler
from .workload import flagship_config, percentile


def _wait(pred: Callable[[], bool], timeout: float = 30.0, poll: float = 0.0002) -> bool:
    deadline = time.perf_counter() + timeout
    while not pred():
        if time.perf_counter() > deadline:
            return False
        time.sleep(poll)
    return True


def _summary(lat_ms: list[float], pods: int, seconds: float) -> dict:
    return {"pods": pods, "pods_per_s": round(pods / seconds, 1) if seconds > 0 else 0.0,
            "p50_ms": round(percentile(lat_ms, 50), 3), "p99_ms": round(percentile(lat_ms, 99), 3)}


def _bound(store, ns: str) -> list[dict]:
    return [p for p in store.list("pods", ns)[0] if p["spec"].get("nodeName")]


def _cosched_cfg(extra: dict | None = None, args: list | None = None) -> dict:
    plugins = {"queueSort": {"enabled": [{"name": "Coscheduling"}], "disabled": [{"name": "*"}]},
               "preFilter": {"enabled": [{"name": "Coscheduling"}]},
               "postFilter": {"enabled": [{"name": "Coscheduling"}]},
               "permit": {"enabled": [{"name": "Coscheduling"}]},
               "reserve": {"enabled": [{"name": "Coscheduling"}]},
               "postBind": {"enabled": [{"name": "Coscheduling"}]}}
    for pt, spec in (extra or {}).items():
        for k, v in spec.items():
            plugins.setdefault(pt, {}).setdefault(k, []).extend(v)
    return {"apiVersion": "kubescheduler.config.k8s.io/v1beta3", "kind": "KubeSchedulerConfiguration",
            "profiles": [{"schedulerName": "default-scheduler", "plugins": plugins, "pluginConfig": [
                {"name": "Coscheduling", "args": {"permitWaitingTimeSeconds": 10, "deniedPGExpirationTimeSeconds": 3}},
                *(args or [])]}]}


def coscheduling_cpu(waves: int = 4, groups: int = 100, nodes: int = 16) -> dict:
    store = Store()
    store.create_many("nodes", json.dumps([make_node(f"kind-{i}", {"cpu": "64", "memory": "256Gi", "pods": "110"})
                                           for i in range(nodes)]))
    s = new_scheduler(store, load_config(_cosched_cfg()), start=True)
    lat: list[float] = []
    t_total, pods = 0.0, 0
    try:
        for w in range(waves + 1):
            ns = f"cpu-{w}"
            pgs = [make_pod_group(f"pg{i}", ns, 2) for i in range(groups)]
            pl = [make_pod(f"pg{i}-{r}", ns, pod_group=f"pg{i}", requests={"cpu": "500m", "memory": "512Mi"})
                  for i in range(groups) for r in range(2)]
            t0 = time.perf_counter()
            store.create_many("podgroups", json.dumps(pgs))
            store.create_many("pods", json.dumps(pl))
            ok = _wait(lambda: s.stats()["bound"] >= (w + 1) * len(pl))
            dt = time.perf_counter() - t0
            recs = s.gang_records(True)
            if w > 0:  # first wave is warm-up
                t_total += dt
                pods += len(pl)
                lat += [(g["bound_us"] - g["first_enqueue_us"]) / 1000.0 for g in recs]
            store.delete_all("pods", ns)
            store.delete_all("podgroups", ns)
            _wait(lambda: s.cache_counts()["pods"] == 0)
            if not ok:
                return {"error": "wave did not bind"}
    finally:
        s.stop()
    return _summary(lat, pods, t_total) | {"groups_per_wave": groups, "nodes": nodes}


def flexgpu_cpx_quarter(iterations: int = 40) -> dict:
    """4 pods x amd.com/gpu-xcd: 2 on one MI355X in CPX mode: all four share the
    GPU, each on its own pair of XCD partitions."""
    store = Store()
    store.create("nodes", mi355x_node("mi355x-cpx", n_gpus=1, mode="cpx"))
    cfg = _cosched_cfg({"filter": {"enabled": [{"name": "FlexGPU"}]}, "score": {"enabled": [{"name": "FlexGPU"}]},
                        "reserve": {"enabled": [{"name": "FlexGPU"}]},
                        "bind": {"enabled": [{"name": "FlexGPU"}], "disabled": [{"name": "DefaultBinder"}]}})
    s = new_scheduler(store, load_config(cfg), start=True)
    lat: list[float] = []
    t_total, pods, shared_ok = 0.0, 0, 0
    try:
        for it in range(iterations + 2):
            ns = f"cpx-{it}"
            pl = [make_pod(f"q{i}", ns, limits={GPU_XCD: "2"}, requests={GPU_XCD: "2"}) for i in range(4)]
            t0 = time.perf_counter()
            store.create_many("pods", json.dumps(pl))
            ok = _wait(lambda: len(_bound(store, ns)) == 4)
            dt = time.perf_counter() - t0
            if not ok:
                return {"error": "quarter-GPU pods did not bind"}
            bound = _bound(store, ns)
            parts = [p["metadata"]["annotations"].get(PARTITION_ANNOTATION, "") for p in bound]
            flat = [x for ps in parts for x in ps.split(",") if x]
            if len(flat) == 8 and len(set(flat)) == 8 and {x.split(":")[0] for x in flat} == {"0"}:
                shared_ok += 1
            if it >= 2:
                t_total += dt
                pods += 4
                lat.append(dt * 1000.0)
            store.delete_all("pods", ns)
            _wait(lambda: s.cache_counts()["pods"] == 0)
    finally:
        s.stop()
    return _summary(lat, pods, t_total) | {"four_pods_share_one_gpu": f"{shared_ok}/{iterations + 2}",
                                            "latency": "4-pod batch create -> all bound"}


def gang8_xgmi(iterations: int = 30, nodes: int = 5) -> dict:
    """Gangs of 2-8 ranks with XGMIGangAffinity + gangColocation: every gang
    must land on one node's xGMI mesh although the scheduler has a real
    choice. Background load leaves 3 / 2 / 8 / 4 / 6 GPUs free on the five
    nodes: for every gang size some node can host the whole gang and others
    cannot, and the tightest nodes (which node bin-packing prefers) are
    often the ones that can only take part of it. Gang sizes cycle 4, 8, 2,
    6, 3; the 8-rank gang has exactly one choice."""
    store = Store()
    store.create_many("nodes", json.dumps([mi355x_node(f"mi355x-{i}") for i in range(nodes)]))
    store.create_many("noderesourcetopologies", json.dumps([mi355x_nrt(f"mi355x-{i}") for i in range(nodes)]))
    s = new_scheduler(store, load_config(flagship_config()), start=True)
    lat: list[float] = []
    t_total, pods, colocated, hostable = 0.0, 0, 0, 0
    by_size: dict[str, str] = {}
    sizes = (4, 8, 2, 6, 3)
    busy = (5, 6, 0, 4, 2)
    try:
        bg = []
        for i in range(nodes):
            for k in range(busy[i % len(busy)]):
                p = make_pod(f"bg-{i}-{k}", "bg", limits={GPU: "1"}, requests={GPU: "1"})
                p["spec"]["nodeSelector"] = {"kubernetes.io/hostname": f"mi355x-{i}"}
                bg.append(p)
        store.create_many("pods", json.dumps(bg))
        if not _wait(lambda: len(_bound(store, "bg")) == len(bg)):
            return {"error": "background pods did not bind"}
        ok_by: dict[int, list[int]] = {}
        for it in range(iterations + 2):
            k = sizes[it % len(sizes)]
            ns = f"g8-{it}"
            store.create("podgroups", make_pod_group("ranks", ns, k))
            pl = [make_pod(f"rank-{r}", ns, pod_group="ranks", limits={GPU: "1"}, requests={GPU: "1"})
                  for r in range(k)]
            t0 = time.perf_counter()
            store.create_many("pods", json.dumps(pl))
            ok = _wait(lambda: len(_bound(store, ns)) == k)
            dt = time.perf_counter() - t0
            if not ok:
                return {"error": f"gang of {k} did not bind"}
            bound = _bound(store, ns)
            one = len({p["spec"]["nodeName"] for p in bound}) == 1 and \
                len({p["metadata"]["annotations"][INDEX_ANNOTATION] for p in bound}) == k
            colocated += one
            ok_by.setdefault(k, [0, 0])
            ok_by[k][0] += one
            ok_by[k][1] += 1
            recs = s.gang_records(True)
            hostable += sum(1 for g in recs if g.get("hostable") == 1)
            if it >= 2:
                t_total += dt
                pods += k
                lat += [(g["bound_us"] - g["first_enqueue_us"]) / 1000.0 for g in recs] or [dt * 1000.0]
            store.delete_all("pods", ns)
            store.delete_all("podgroups", ns)
            _wait(lambda: s.cache_counts()["pods"] == len(bg))
        by_size = {str(k): f"{v[0]}/{v[1]}" for k, v in sorted(ok_by.items())}
    finally:
        s.stop()
    return _summary(lat, pods, t_total) | {"gangs_on_one_xgmi_node": f"{colocated}/{iterations + 2}",
                                            "by_size": by_size, "hostable_at_first_rank": hostable,
                                            "free_gpus_per_node": [8 - busy[i % len(busy)] for i in range(nodes)],
                                            "nodes": nodes}


def capacity_preemption(iterations: int = 2) -> dict:
    """Team A borrows all 8 GPUs; team B then claims its guaranteed 4:
    exactly team A's borrowed GPUs are preempted."""
    cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": "default-scheduler", "plugins": {
               "preFilter": {"enabled": [{"name": "CapacityScheduling"}]},
               "postFilter": {"enabled": [{"name": "CapacityScheduling"}], "disabled": [{"name": "*"}]},
               "reserve": {"enabled": [{"name": "CapacityScheduling"}]}}}]}
    lat: list[float] = []
    correct = 0
    for it in range(iterations):
        store = Store()
        store.create("nodes", mi355x_node("mi355x-0"))
        for team in ("team-a", "team-b"):
            store.create("elasticquotas", make_elastic_quota(f"q-{team}", team, min={GPU: "4", "cpu": "64"},
                                                             max={GPU: "8", "cpu": "256"}))
        s = new_scheduler(store, load_config(cfg), start=True)
        try:
            store.create_many("pods", json.dumps([make_pod(f"a{i}", "team-a", requests={"cpu": "1"},
                                                           limits={GPU: "1"}) for i in range(8)]))
            if not _wait(lambda: len(_bound(store, "team-a")) == 8):
                return {"error": "team-a did not bind"}
            t0 = time.perf_counter()
            store.create_many("pods", json.dumps([make_pod(f"b{i}", "team-b", requests={"cpu": "1"},
                                                           limits={GPU: "1"}) for i in range(4)]))
            ok = _wait(lambda: len(_bound(store, "team-b")) == 4, timeout=60)
            dt = time.perf_counter() - t0
            if ok:
                lat.append(dt * 1000.0)
                correct += int(len(_bound(store, "team-a")) == 4)
        finally:
            s.stop()
    return {"reclaim_ms": [round(x, 1) for x in lat], "p99_ms": round(percentile(lat, 99), 1) if lat else None,
            "exactly_borrowed_preempted": f"{correct}/{iterations}",
            "note": "includes upstream pod backoff (1s initial) between preemption and re-scheduling"}


def _readings(hs) -> tuple[list, str]:
    """Per-GPU readings of the host (telemetry.GpuReading list) and their
    source; [] when the sampler sees no GPU."""
    from ..gpu.telemetry import GpuReading

    if hasattr(hs, "per_gpu"):
        rs = hs.per_gpu()
        src = ("amd-smi (libamd_smi) gfx_activity / umc_activity" if getattr(hs, "smi", None) is not None
               else "amdgpu sysfs gpu_busy_percent")
    else:  # a bare sampler (tests): sysfs-style (busy, vram%) pairs
        rs = [GpuReading(i, None if b is None else float(b), m) for i, (b, m) in enumerate(hs.gpu_samples())]
        src = "amdgpu sysfs gpu_busy_percent"
    rs = [r for r in rs if r.gfx is not None]
    return rs, (src if rs else "synthetic")


def _mean_readings(hs, seconds: float, period: float = 0.05) -> tuple[dict, str]:
    """Per-GPU mean readings over `seconds`: {gpu index: GpuReading}."""
    from ..gpu.telemetry import GpuReading

    acc: dict[int, list] = {}
    src = "synthetic"
    t_end = time.perf_counter() + seconds
    while True:
        rs, src = _readings(hs)
        for r in rs:
            acc.setdefault(r.index, []).append(r)
        if time.perf_counter() >= t_end:
            break
        time.sleep(period)
    avg = (lambda xs: round(sum(xs) / len(xs), 1) if xs else None)
    out = {i: GpuReading(i, avg([r.gfx for r in v if r.gfx is not None]),
                         avg([r.vram_used_pct for r in v if r.vram_used_pct is not None]),
                         avg([r.umc for r in v if r.umc is not None]),
                         avg([r.xgmi_pct for r in v if r.xgmi_pct is not None])) for i, v in acc.items()}
    return out, src


def _cuda_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


def trimaran_tlp(pods: int = 256, nodes: int = 8, sampler=None, start_load=None, seconds: float = 1.0) -> dict:
    """TargetLoadPacking in GPU mode on `nodes` synthetic 8x MI355X nodes
    whose WatcherMetrics carry live per-GPU activity of this host
    (pkg/trimaran/targetloadpacking/targetloadpacking.go:181-270, target 40%):

    * with G >= 2 visible GPUs, synthetic node i is backed by physical GPU
      i mod G (all 8 of its GPU slots), and the GPUs of the upper half
      (index >= G/2) each run their own device copy loop; every node's
      document is the node agent's aggregate of its 8 GPUs' readings
      (telemetry.aggregate), so the loaded GPUs' nodes must score below the
      idle ones;
    * with one GPU, the first half of the nodes publish its idle sample and
      the second half the sample taken under load (`replicated_from_gpu0`);
    * without a GPU the values are synthetic.
    `start_load(device)` starts a load on one device and returns its stop();
    on a GPU host it defaults to tools/tlp_live.copy_loop_load."""
    from ..gpu.telemetry import GpuReading, NodeTelemetry, aggregate, publish
    from ..control.client import LocalClient

    try:
        if sampler is not None:
            hs = sampler
        else:
            from ..gpu.telemetry import HostSampler

            hs = HostSampler()
    except Exception:  # noqa: BLE001 - no amd-smi and no amdgpu sysfs
        hs = None
    if start_load is None and sampler is None and _cuda_available():
        from ..tools.tlp_live import copy_loop_load as start_load
    idle: dict = {}
    busy_r: dict = {}
    source = "synthetic"
    if hs is not None:
        idle, source = _mean_readings(hs, min(0.5, seconds))
    gpus = sorted(idle)
    n_gpu = len(gpus)
    if n_gpu >= 2 and start_load is not None:
        try:
            import torch

            n_dev = torch.cuda.device_count() if _cuda_available() else n_gpu
        except Exception:  # noqa: BLE001
            n_dev = n_gpu
        loaded = [g for g in gpus if g >= n_gpu // 2 and g < n_dev]
    else:
        loaded = [gpus[0]] if n_gpu == 1 and start_load is not None else []
    if loaded:
        stops = [start_load(g) for g in loaded]
        try:
            time.sleep(0.3)  # the activity counters ramp over a few samples
            busy_r, _ = _mean_readings(hs, seconds)
        finally:
            for stop in stops:
                stop()
    half = nodes // 2
    node_src: dict[str, object] = {}
    node_readings: list[list] = []
    if n_gpu >= 2:
        view = busy_r or idle
        for i in range(nodes):
            g = gpus[i % n_gpu]
            node_src[f"mi355x-{i}"] = g
            node_readings.append([view.get(g, idle[g])] * 8)  # the node's 8 GPUs, as the agent sees them
    elif n_gpu == 1:
        g = gpus[0]
        for i in range(nodes):
            r = busy_r.get(g) if (i >= half and busy_r) else idle[g]
            node_src[f"mi355x-{i}"] = g
            node_readings.append([r] * 8)
    else:
        for i in range(nodes):
            node_src[f"mi355x-{i}"] = None
            node_readings.append([GpuReading(j, float((i * 13) % 100)) for j in range(8)])
    now = time.time()
    samples = [aggregate(rs, now) for rs in node_readings]
    busy = [round(s.gpu, 1) if s.gpu is not None else None for s in samples]
    hbm = [round(s.hbm_bandwidth, 1) if s.hbm_bandwidth is not None else None for s in samples]
    store = Store()
    store.create_many("nodes", json.dumps([mi355x_node(f"mi355x-{i}") for i in range(nodes)]))
    c = LocalClient(store)
    for i in range(nodes):
        t = NodeTelemetry(f"mi355x-{i}", source=source)
        t.add(samples[i])
        publish(c, t.watcher_metrics())
    cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": "default-scheduler", "plugins": {
               "score": {"enabled": [{"name": "TargetLoadPacking"}], "disabled": [{"name": "*"}]}},
               "pluginConfig": [{"name": "TargetLoadPacking", "args": {"resourceType": "GPU"}}]}]}
    s = new_scheduler(store, load_config(cfg), start=True)
    try:
        _wait(lambda: s.cache_counts()["nodes"] == nodes)
        first = s.explain(make_pod("probe", "tlp", limits={GPU: "1"}, requests={GPU: "1"}))
        t0 = time.perf_counter()
        store.create_many("pods", json.dumps([make_pod(f"p{i}", "tlp", requests={"cpu": "100m"})
                                              for i in range(pods)]))
        ok = _wait(lambda: s.stats()["bound"] >= pods)
        dt = time.perf_counter() - t0
    finally:
        s.stop()
    scores = {n: v["TargetLoadPacking*1"] for n, v in (first.get("scores") or {}).items()}
    out = {"pods_per_s": round(pods / dt, 1) if ok else None, "metrics_source": source,
           "gpus_sampled": n_gpu, "replicated_from_gpu0": n_gpu == 1,
           "node_source_gpu": node_src, "loaded_gpus": loaded,
           "node_gpu_busy_pct": busy, "node_hbm_bandwidth_pct": hbm,
           "first_gpu_pod_node": first.get("selected"), "tlp_scores": scores}
    if busy_r and loaded:
        loaded_nodes = [n for n, g in node_src.items() if (g in loaded if n_gpu >= 2 else int(n.split("-")[1]) >= half)]
        idle_nodes = [n for n in node_src if n not in loaded_nodes]
        out["live_load"] = {
            "idle_gpu_busy_pct": {g: idle[g].gfx for g in gpus},
            "loaded_gpu_busy_pct": {g: busy_r[g].gfx for g in loaded if g in busy_r},
            "loaded_nodes": loaded_nodes,
            "busy_scores_below_idle": bool(idle_nodes) and max(scores[n] for n in loaded_nodes) < min(
                scores[n] for n in idle_nodes)}
    return out


ALL = {"coscheduling_cpu": coscheduling_cpu, "flexgpu_cpx_quarter": flexgpu_cpx_quarter, "gang8_xgmi": gang8_xgmi,
       "capacity_preemption": capacity_preemption, "trimaran_tlp": trimaran_tlp}


def run_all(names=None) -> dict:
    out = {}
    for name, fn in ALL.items():
        if names and name not in names:
            continue
        t0 = time.perf_counter()
        try:
            out[name] = fn()
        except Exception as e:  # noqa: BLE001 - a scenario failure is reported, not fatal
            out[name] = {"error": f"{type(e).__name__}: {e}"}
        out[name]["wall_s"] = round(time.perf_counter() - t0, 2)
    return out


if __name__ == "__main__":
    print(json.dumps(run_all(), indent=1))
