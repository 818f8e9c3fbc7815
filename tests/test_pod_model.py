"""Pod request math (computePodResourceRequest, non-zero defaults, QoS) and
GPU assignment decoding — the parse-time views every plugin consumes."""
from flex_gpu_scheduler_amd._native import native
from flex_gpu_scheduler_amd.models import make_container, make_pod

X = native()


def test_effective_request_init_and_overhead():
    p = make_pod("p", containers=[make_container("a", requests={"cpu": "1", "memory": "1Gi"}),
                                  make_container("b", requests={"cpu": "500m"})],
                 init_containers=[make_container("i", requests={"cpu": "2", "memory": "512Mi"})],
                 overhead={"cpu": "100m"})
    s = X.pod_summary(p)
    # max(sum containers, each init) + overhead
    assert s["request"]["cpu"] == "2100m"
    assert s["request"]["memory"] == "1Gi"


def test_nonzero_defaults():
    s = X.pod_summary(make_pod("p"))
    assert s["nonzero_request"] == {"cpu": "100m", "memory": "200Mi"}
    assert s["qos"] == "BestEffort"


def test_qos_classes():
    g = make_pod("g", requests={"cpu": "1", "memory": "1Gi"}, limits={"cpu": "1", "memory": "1Gi"})
    assert X.pod_summary(g)["qos"] == "Guaranteed"
    lim_only = make_pod("l", limits={"cpu": "1", "memory": "1Gi"})  # requests default to limits
    assert X.pod_summary(lim_only)["qos"] == "Guaranteed"
    b = make_pod("b", requests={"cpu": "1"})
    assert X.pod_summary(b)["qos"] == "Burstable"


def test_gpu_annotation_decoding_bounds():
    p = make_pod("p", limits={"amd.com/gpu-xcd": "2"},
                 annotations={"amd.com/gpu-index": "3", "amd.com/gpu-partitions": "3:4,3:5"})
    s = X.pod_summary(p)
    assert s["gpus"] == [3] and s["partitions"] == [(3, 4), (3, 5)]
    bad = make_pod("q", limits={"amd.com/gpu": "1"}, annotations={"amd.com/gpu-index": "x"})
    assert X.pod_summary(bad)["gpus"] == []  # unparsable index is ignored, never a crash (Appendix C2)
