"""amd-smi telemetry provider (gpu/amdsmi.py over csrc/telemetry/
amdsmi_sampler.cc) and the Trimaran dimensions it feeds: HBM-controller
activity ("GPUMemoryBandwidth") and xGMI traffic ("XGMI"). The native sampler
is exercised on the MI355X box (tests/test_gpu.py); here a recorded-shape
reader stands in for libamd_smi."""
from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.gpu.amdsmi import XGMI_LINK_GBPS, AmdSmiSampler, native_status
from flex_gpu_scheduler_amd.gpu.telemetry import HostSampler, NodeTelemetry, Sample
from flex_gpu_scheduler_amd.models import GPU, make_node, make_pod, make_pod_group

from test_trimaran import explain_scores, metrics, only_score


def smi_doc(index=0, gfx=30, umc=60, used=100_000, total=294_896, read_kb=(0,) * 8, write_kb=(0,) * 8, up=7):
    return {"index": index, "bdf": f"0000:{index + 5:02x}:00.0", "gfx_activity": gfx, "umc_activity": umc,
            "mm_activity": 0, "xcc_busy": [gfx] * 8, "vram_total_mb": total, "vram_used_mb": used,
            "socket_power_w": 640, "temp_hotspot_c": 55, "temp_mem_c": 48,
            "xgmi_read_kb": list(read_kb), "xgmi_write_kb": list(write_kb),
            "xgmi_link_up": [1] * up + [0] * (8 - up), "xgmi_link_speed": 32, "xgmi_link_width": 16,
            "vram_max_bandwidth_gbs": 8000, "firmware_timestamp_10ns": 0, "num_partition": 1}


class FakeReader:
    def __init__(self, frames):
        self.frames = list(frames)

    def __call__(self):
        return self.frames.pop(0)


def test_native_status_reports_reason_without_gpu():
    ok, err = native_status()
    assert isinstance(ok, bool) and isinstance(err, str)
    if not ok:
        assert err  # e.g. "amdsmi_init failed" on a host without the amdgpu driver


def test_xgmi_rate_from_accumulators():
    t = iter([10.0, 12.0])
    gb = 10 ** 9 / 1024  # KB per GB
    r = FakeReader([[smi_doc()], [smi_doc(read_kb=(int(40 * gb),) + (0,) * 7, write_kb=(int(20 * gb),) + (0,) * 7)]])
    s = AmdSmiSampler(reader=r, clock=lambda: next(t))
    first = s.sample()[0]
    assert first.xgmi_gbps is None and first.gfx == 30 and first.umc == 60
    assert abs(first.vram_used_pct - 100 * 100_000 / 294_896) < 1e-9
    second = s.sample()[0]
    assert abs(second.xgmi_gbps - 30.0) < 0.01  # 60 GB over 2 s
    assert abs(second.xgmi_pct - 100 * 30.0 / (7 * 2 * XGMI_LINK_GBPS)) < 0.01
    assert second.links_up == 7 and second.xcc_busy == [30.0] * 8


def test_host_sampler_prefers_injected_amdsmi():
    smi = AmdSmiSampler(reader=FakeReader([[smi_doc(0, gfx=20, umc=40), smi_doc(1, gfx=60, umc=80)]]))
    hs = HostSampler(root="/nonexistent", cards=[], smi=smi)
    assert hs.gpu_source == "amdsmi"
    s = hs.sample()
    assert s.gpu == 40 and s.hbm_bandwidth == 60 and s.xgmi is None


def test_watcher_document_carries_new_gpu_types():
    nt = NodeTelemetry("n0")
    nt.add(Sample(100.0, 10.0, 20.0, 30.0, 40.0, 55.0, 12.5))
    types = {m["type"] for m in nt.metrics()}
    assert {"CPU", "Memory", "GPU", "GPUMemory", "GPUMemoryBandwidth", "XGMI"} <= types


def gpu_metric(t, v, op="AVG"):
    return {"type": t, "operator": op, "value": v}


def test_lvrb_avoids_hbm_bandwidth_saturated_node(store):
    for n in ("a", "b"):
        store.create("nodes", make_node(n, {"cpu": "64", "memory": "256Gi", "pods": "110", GPU: "8"}))
    s = new_scheduler(store, load_config(only_score("LoadVariationRiskBalancing")))
    # Same GPU busy; node a's HBM controllers are at 90%.
    store.create("loadwatchermetrics", metrics({
        "a": [gpu_metric("GPU", 30), gpu_metric("GPUMemoryBandwidth", 90)],
        "b": [gpu_metric("GPU", 30), gpu_metric("GPUMemoryBandwidth", 10)]}))
    sc = explain_scores(store, s, make_pod("p", limits={GPU: "1"}, requests={GPU: "1"}))
    a, b = sc["a"]["LoadVariationRiskBalancing*1"], sc["b"]["LoadVariationRiskBalancing*1"]
    # bandwidth dim: mu = min(1, 0.9 + 1/8) = 1 -> (1 - 1/2) * 100 = 50 (min with GPU busy 78.75)
    assert a == 50 and b == 79, sc
    # A CPU-only pod ignores the GPU dimensions entirely.
    sc = explain_scores(store, s, make_pod("c", requests={"cpu": "1"}))
    assert sc["a"]["LoadVariationRiskBalancing*1"] == sc["b"]["LoadVariationRiskBalancing*1"]
    s.stop()


def test_lvrb_xgmi_dimension_only_for_gang_members(store):
    for n in ("a", "b"):
        store.create("nodes", make_node(n, {"cpu": "64", "memory": "256Gi", "pods": "110", GPU: "8"}))
    store.create("podgroups", make_pod_group("ranks", "default", 2))
    s = new_scheduler(store, load_config(only_score("LoadVariationRiskBalancing")))
    store.create("loadwatchermetrics", metrics({
        "a": [gpu_metric("GPU", 10), gpu_metric("XGMI", 95)],
        "b": [gpu_metric("GPU", 10), gpu_metric("XGMI", 5)]}))
    gang = explain_scores(store, s, make_pod("r0", pod_group="ranks", limits={GPU: "1"}, requests={GPU: "1"}))
    assert gang["a"]["LoadVariationRiskBalancing*1"] < gang["b"]["LoadVariationRiskBalancing*1"]
    solo = explain_scores(store, s, make_pod("solo", limits={GPU: "1"}, requests={GPU: "1"}))
    assert solo["a"]["LoadVariationRiskBalancing*1"] == solo["b"]["LoadVariationRiskBalancing*1"]
    s.stop()


def test_tlp_packs_on_hbm_bandwidth(store):
    for n in ("a", "b"):
        store.create("nodes", make_node(n, {"cpu": "64", "memory": "256Gi", "pods": "110", GPU: "8"}))
    s = new_scheduler(store, load_config(only_score("TargetLoadPacking", {"resourceType": "GPUMemoryBandwidth"})))
    store.create("loadwatchermetrics", metrics({"a": [gpu_metric("GPUMemoryBandwidth", 25)],
                                                "b": [gpu_metric("GPUMemoryBandwidth", 90)],
                                                }))
    sc = explain_scores(store, s, make_pod("p", limits={GPU: "1"}))
    # same arithmetic as GPU mode: a 37.5% -> 96, b 102.5% -> 0
    assert sc["a"]["TargetLoadPacking*1"] == 96 and sc["b"]["TargetLoadPacking*1"] == 0
    s.stop()
