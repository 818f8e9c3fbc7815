"""FlexGPU on MI355X nodes: whole-GPU, CPX partition and HBM-slice packing.

The reference FlexGPU has no tests at all; these pin the
behaviour of pkg/flexgpu/{flex_gpu,gpu_node}.go plus the MI355X partition
model and the deliberate Appendix C fixes."""
import time

import pytest

from flex_gpu_scheduler_amd.models import (GPU, GPU_MEMORY, GPU_XCD, GpuInfo, make_pod, make_pod_group,
                                           mi355x_node)
from helpers import FLEXGPU_PLUGINS, annotations, coscheduling_config, create_all, placements, start, wait_bound


def cfg():
    return coscheduling_config(FLEXGPU_PLUGINS)


def test_whole_gpu_indexes_are_distinct(store):
    store.create("nodes", mi355x_node("n0"))
    s = start(store, cfg())
    try:
        create_all(store, "pods", [make_pod(f"p{i}", limits={GPU: "1"}) for i in range(8)])
        wait_bound(s, 8)
        idx = sorted(int(annotations(store, f"p{i}")["amd.com/gpu-index"]) for i in range(8))
        assert idx == list(range(8))
        store.create("pods", make_pod("p8", limits={GPU: "1"}))
        time.sleep(0.3)
        assert placements(store)["p8"] == ""  # 9th whole GPU does not exist
    finally:
        s.stop()


def test_multi_gpu_pod_prefers_one_socket(store):
    store.create("nodes", mi355x_node("n0"))
    s = start(store, cfg())
    try:
        store.create("pods", make_pod("one", limits={GPU: "1"}))
        wait_bound(s, 1)
        store.create("pods", make_pod("four", limits={GPU: "4"}))
        wait_bound(s, 2)
        gpus = [int(x) for x in annotations(store, "four")["amd.com/gpu-index"].split(",")]
        assert len(gpus) == 4 and len({g // 4 for g in gpus}) == 1  # all on one NUMA socket
    finally:
        s.stop()


def test_cpx_quarter_gpu_slices(store):
    # BASELINE config: 4 pods x 0.25 amd.com/gpu on one MI355X (CPX partition)
    store.create("nodes", mi355x_node("cpx", n_gpus=1, mode="cpx"))
    s = start(store, cfg())
    try:
        create_all(store, "pods", [make_pod(f"q{i}", limits={GPU_XCD: "2"}) for i in range(4)])
        wait_bound(s, 4)
        parts = set()
        for i in range(4):
            a = annotations(store, f"q{i}")
            assert a["amd.com/gpu-index"] == "0"
            ps = a["amd.com/gpu-partitions"].split(",")
            assert len(ps) == 2
            parts.update(ps)
        assert len(parts) == 8  # the 8 CPX partitions are split disjointly
        store.create("pods", make_pod("q4", limits={GPU_XCD: "1"}))
        time.sleep(0.3)
        assert placements(store)["q4"] == ""
    finally:
        s.stop()


def test_xcd_slice_avoids_stranding_spx_gpu(store):
    store.create("nodes", mi355x_node("spx", n_gpus=8, mode="spx"))
    store.create("nodes", mi355x_node("cpx", n_gpus=1, mode="cpx"))
    s = start(store, cfg())
    try:
        store.create("pods", make_pod("q", limits={GPU_XCD: "2"}))
        wait_bound(s, 1)
        assert placements(store)["q"] == "cpx"
    finally:
        s.stop()


def test_memory_slices_best_fit_and_capacity(store):
    # Per-GPU memory = allocatable / GPUs (gpu_node.go:51-55); best fit packs
    # slices onto the fullest GPU (Appendix C1 fixed: value semantics).
    store.create("nodes", mi355x_node("n", gpus=[GpuInfo(0, hbm_gib=100), GpuInfo(1, hbm_gib=100)]))
    s = start(store, cfg())
    try:
        store.create("pods", make_pod("m0", limits={GPU_MEMORY: "60"}))
        wait_bound(s, 1)
        g0 = annotations(store, "m0")["amd.com/gpu-index"]
        store.create("pods", make_pod("m1", limits={GPU_MEMORY: "30"}))
        wait_bound(s, 2)
        assert annotations(store, "m1")["amd.com/gpu-index"] == g0  # fits beside m0 -> same GPU
        store.create("pods", make_pod("m2", limits={GPU_MEMORY: "50"}))
        wait_bound(s, 3)
        assert annotations(store, "m2")["amd.com/gpu-index"] != g0
        store.create("pods", make_pod("m3", limits={GPU_MEMORY: "60"}))
        time.sleep(0.3)
        assert placements(store)["m3"] == ""  # 40 + 50 free, no single GPU has 60
    finally:
        s.stop()


def test_conflicting_resources_unresolvable(store):
    store.create("nodes", mi355x_node("n"))
    s = start(store, cfg())
    try:
        store.create("pods", make_pod("bad", limits={GPU: "1", GPU_MEMORY: "10"}))
        time.sleep(0.3)
        cond = store.get("pods", "default", "bad")["status"]["conditions"][0]
        assert "pod conflict resources" in cond["message"]
    finally:
        s.stop()


def test_node_without_gpu_resources_is_unresolvable(store):
    from flex_gpu_scheduler_amd.models import make_node

    store.create("nodes", make_node("cpu-only"))
    s = start(store, cfg())
    try:
        store.create("pods", make_pod("g", limits={GPU: "1"}))
        time.sleep(0.3)
        assert "unknown resource type" in store.get("pods", "default", "g")["status"]["conditions"][0]["message"] \
            or "Insufficient" in store.get("pods", "default", "g")["status"]["conditions"][0]["message"]
    finally:
        s.stop()


def test_gpu_freed_on_delete_is_reused(store):
    store.create("nodes", mi355x_node("n", n_gpus=1))
    s = start(store, cfg())
    try:
        store.create("pods", make_pod("a", limits={GPU: "1"}))
        wait_bound(s, 1)
        store.create("pods", make_pod("b", limits={GPU: "1"}))
        time.sleep(0.2)
        assert placements(store)["b"] == ""
        store.delete("pods", "default", "a")  # AssignedPodDelete re-queues b
        wait_bound(s, 2)
        assert placements(store)["b"] == "n"
    finally:
        s.stop()


def test_gang_ranks_colocate_on_one_node(store):

    from flex_gpu_scheduler_amd import load_config, new_scheduler
    from flex_gpu_scheduler_amd.models import mi355x_nrt
    from flex_gpu_scheduler_amd.utils.workload import flagship_config

    for i in range(4):
        store.create("nodes", mi355x_node(f"n{i}"))
        store.create("noderesourcetopologies", mi355x_nrt(f"n{i}"))
    s = new_scheduler(store, load_config(flagship_config()), start=True)
    try:
        # Partially fill two nodes so a naive bin-packer would split the gang.
        create_all(store, "pods", [make_pod(f"f{i}", limits={GPU: "1"}) for i in range(6)])
        wait_bound(s, 6)
        store.create("podgroups", make_pod_group("ring", "default", 8))
        create_all(store, "pods", [make_pod(f"r{i}", pod_group="ring", limits={GPU: "1"}) for i in range(8)])
        wait_bound(s, 14)
        nodes = {placements(store)[f"r{i}"] for i in range(8)}
        assert len(nodes) == 1, nodes  # all 8 ranks share one node's xGMI mesh
    finally:
        s.stop()


def _named_cfg(names: dict, scheduler_name="default-scheduler"):
    c = coscheduling_config(FLEXGPU_PLUGINS)
    c["profiles"][0]["schedulerName"] = scheduler_name
    c["profiles"][0]["pluginConfig"].append({"name": "FlexGPU", "args": names})
    return c


def test_gpu_resource_names_are_per_scheduler():
    """Two schedulers in one process with different FlexGPU resource names:
    each parses pods/nodes and writes index annotations with its own names
    (no process-global state; the second does not rename the first's)."""
    from flex_gpu_scheduler_amd.models import make_node
    from flex_gpu_scheduler_amd.scheduler import Store

    sa, sb = Store(), Store()
    sa.create("nodes", mi355x_node("n0"))
    sb.create("nodes", make_node("m0", {"cpu": "32", "memory": "64Gi", "pods": "110", "example.com/accel": "4"}))
    a = start(sa, cfg())
    b = start(sb, _named_cfg({"gpuResourceName": "example.com/accel", "indexAnnotationKey": "example.com/accel-index"}))
    try:
        create_all(sb, "pods", [make_pod(f"q{i}", limits={"example.com/accel": "1"}) for i in range(4)])
        wait_bound(b, 4)
        assert sorted(int(annotations(sb, f"q{i}")["example.com/accel-index"]) for i in range(4)) == [0, 1, 2, 3]
        sb.create("pods", make_pod("q4", limits={"example.com/accel": "1"}))
        create_all(sa, "pods", [make_pod(f"p{i}", limits={GPU: "1"}) for i in range(3)])
        wait_bound(a, 3)
        for i in range(3):
            ann = annotations(sa, f"p{i}")
            assert "amd.com/gpu-index" in ann and "example.com/accel-index" not in ann
        time.sleep(0.3)
        assert placements(sb)["q4"] == ""  # the 5th accel does not exist: B's ledger counts its own resource
    finally:
        a.stop()
        b.stop()


def test_profiles_of_one_scheduler_must_agree_on_gpu_names(store):
    from flex_gpu_scheduler_amd.scheduler import new_scheduler

    c = _named_cfg({"gpuResourceName": "example.com/accel"})
    other = _named_cfg({"gpuResourceName": "amd.com/gpu"}, scheduler_name="second")["profiles"][0]
    c["profiles"].append(other)
    with pytest.raises(Exception, match="FlexGPU resource names differ"):
        new_scheduler(store, c)


def _reference_place_whole(free: list[int], numa: dict[int, int], k: int) -> list[int]:
    """The whole-GPU chooser as first written (a map of NUMA node -> free
    GPUs): the NUMA node with the fewest free GPUs that still fits, lowest id
    among equals, -1 never; else the lowest free GPUs."""
    by: dict[int, list[int]] = {}
    for g in free:
        by.setdefault(numa[g], []).append(g)
    if len(by) > 1 or (len(by) == 1 and min(by) >= 0):
        best = None
        for n in sorted(by):
            if n < 0 or len(by[n]) < k:
                continue
            if best is None or len(by[n]) < len(by[best]):
                best = n
        if best is not None:
            return by[best][:k]
    return free[:k]


@pytest.mark.parametrize("seed", range(12))
def test_whole_gpu_choice_matches_reference_model(store, seed):
    """Randomised: GPUs held on a node with an irregular NUMA layout (some
    GPUs of unknown NUMA), then a k-GPU pod: the GPUs chosen equal the
    reference model's (place_whole is allocation-free since round 6)."""
    import random

    rng = random.Random(seed)
    numa = {g: rng.choice([-1, 0, 0, 1, 1, 2]) for g in range(8)}
    store.create("nodes", mi355x_node("n0", gpus=[GpuInfo(g, numa=numa[g]) for g in range(8)]))
    held = sorted(rng.sample(range(8), rng.randint(0, 5)))
    s = start(store, cfg())
    try:
        for g in held:
            p = make_pod(f"h{g}", limits={GPU: "1"})
            p["spec"]["nodeName"] = "n0"
            p["metadata"].setdefault("annotations", {})["amd.com/gpu-index"] = str(g)
            store.create("pods", p)
        free = [g for g in range(8) if g not in held]
        k = rng.randint(1, len(free))
        time.sleep(0.1)  # the held pods reach the cache before the new one is scheduled
        store.create("pods", make_pod("want", limits={GPU: str(k)}))
        wait_bound(s, 1)
        got = [int(x) for x in annotations(store, "want")["amd.com/gpu-index"].split(",")]
        assert got == _reference_place_whole(free, numa, k), (numa, held, k, got)
    finally:
        s.stop()
