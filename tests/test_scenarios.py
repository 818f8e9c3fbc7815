"""The five BASELINE.json configurations (utils/scenarios.py) run and their
placement properties hold."""
from flex_gpu_scheduler_amd.utils import scenarios as sc


def test_coscheduling_cpu():
    r = sc.coscheduling_cpu(waves=1, groups=20, nodes=4)
    assert r["pods"] == 40 and r["pods_per_s"] > 0


def test_flexgpu_cpx_quarter_shares_one_gpu():
    r = sc.flexgpu_cpx_quarter(iterations=3)
    assert r["four_pods_share_one_gpu"] == "5/5"


def test_gang8_lands_on_one_xgmi_node():
    r = sc.gang8_xgmi(iterations=3)
    assert r["gangs_on_one_xgmi_node"] == "5/5"


def test_capacity_reclaims_exactly_borrowed_within_one_backoff():
    """Four team-b preemptors arrive at once. Usually each preempts its own
    victim in its first cycle and binds after the 1 s initial backoff. On a
    loaded host the last preemptor's first cycle can run while the quota
    infos still count the victims its siblings just preempted (the same
    informer race upstream has): it finds no room, backs off 2 s and preempts
    in its second cycle. So: every run within two backoffs, most within one."""
    r = sc.capacity_preemption(iterations=3)
    assert r["exactly_borrowed_preempted"] == "3/3"
    assert all(ms < 3600 for ms in r["reclaim_ms"]), r  # never a cascade of rounds
    assert sum(ms < 1900 for ms in r["reclaim_ms"]) >= 2, r  # one 1 s backoff as a rule


def test_trimaran_tlp_prefers_target_utilisation():
    r = sc.trimaran_tlp(pods=16, sampler=type("S", (), {"gpu_samples": lambda self: []})())
    assert r["metrics_source"] == "synthetic"
    scores = r["tlp_scores"]
    # 26% busy + 1/8 GPU = 38.5% is closest below the 40% target.
    assert max(scores, key=scores.get) == r["first_gpu_pod_node"] == "mi355x-2"


class FakeEightGpuHost:
    """An 8-GPU host for the TLP scenario: GPU i reads 3% GFX busy, or 97%
    while a load runs on it (start_load(i))."""

    def __init__(self):
        self.busy: set[int] = set()

    def per_gpu(self):
        from flex_gpu_scheduler_amd.gpu.telemetry import GpuReading

        return [GpuReading(i, 97.0 if i in self.busy else 3.0, 10.0, 60.0 if i in self.busy else 1.0, 0.0)
                for i in range(8)]

    def start_load(self, device):
        self.busy.add(device)
        return lambda: self.busy.discard(device)


def test_trimaran_tlp_maps_nodes_to_live_gpus():
    """With >= 2 GPUs each synthetic node is backed by its own physical GPU
    (node i <- GPU i), the upper half of the GPUs is loaded one device each,
    the node documents are the node agent's aggregate of the node's 8 GPUs,
    and the loaded GPUs' nodes score below the idle ones."""
    host = FakeEightGpuHost()
    r = sc.trimaran_tlp(pods=16, sampler=host, start_load=host.start_load, seconds=0.1)
    assert r["gpus_sampled"] == 8 and r["replicated_from_gpu0"] is False
    assert r["node_source_gpu"] == {f"mi355x-{i}": i for i in range(8)}
    assert r["loaded_gpus"] == [4, 5, 6, 7]
    assert r["node_gpu_busy_pct"] == [3.0] * 4 + [97.0] * 4
    assert r["node_hbm_bandwidth_pct"] == [1.0] * 4 + [60.0] * 4
    ll = r["live_load"]
    assert ll["loaded_nodes"] == [f"mi355x-{i}" for i in range(4, 8)] and ll["busy_scores_below_idle"]
    assert r["first_gpu_pod_node"] in {f"mi355x-{i}" for i in range(4)}


def test_trimaran_tlp_one_gpu_is_marked_replicated():
    class OneGpu(FakeEightGpuHost):
        def per_gpu(self):
            return super().per_gpu()[:1]

    host = OneGpu()
    r = sc.trimaran_tlp(pods=16, sampler=host, start_load=host.start_load, seconds=0.1)
    assert r["gpus_sampled"] == 1 and r["replicated_from_gpu0"] is True
    assert set(r["node_source_gpu"].values()) == {0}
    assert r["node_gpu_busy_pct"] == [3.0] * 4 + [97.0] * 4 and r["live_load"]["busy_scores_below_idle"]
