"""Open-loop gang admission (utils/openloop.py, csrc/scheduler/openloop.cc)."""
import json

from flex_gpu_scheduler_amd.utils.benchrun import Shard, gang_latency_summary
from flex_gpu_scheduler_amd.utils.openloop import GANG_TYPES, plan, run_open_loop
from flex_gpu_scheduler_amd.utils.workload import ClusterSpec


def test_plan_interleaves_types_and_sizes_hold():
    spec = ClusterSpec(nodes=16)
    gangs, kinds, offsets, hold_us = plan(spec, 4000.0, 1.0, seed=3)
    assert len(gangs) == len(kinds) == len(offsets) > 500
    assert offsets == sorted(offsets) and offsets[-1] < 1.5e6
    assert set(kinds) == set(GANG_TYPES)
    # Interleaved: CPX gangs are not all at the tail.
    first_cpx = kinds.index("cpx4")
    assert first_cpx < len(kinds) // 10
    names = [g["podgroup"]["metadata"]["name"] for g in gangs]
    assert len(set(names)) == len(names)
    for g, k in zip(gangs, kinds):
        assert len(g["pods"]) == (4 if k == "cpx4" else int(k)) == g["podgroup"]["spec"]["minMember"]
    # Occupancy 0.5 of 96 SPX GPUs at the whole-GPU GPU-seconds arrival rate.
    gang_rate = 4000.0 / 3.8
    assert abs(hold_us - 0.5 * 96 / (gang_rate * 0.8 * 3.75) * 1e6) < 1000


def test_open_loop_admits_every_gang_with_ordered_timeline():
    sh = Shard(ClusterSpec(nodes=16), namespace="b")
    try:
        gangs, kinds, offsets, hold_us = plan(sh.spec, 1000.0, 0.3, seed=1)
        from flex_gpu_scheduler_amd._native import native

        # 20 s: on an overloaded host a gang can be denied for the 3 s TTL and back
        # off before it binds; a healthy run returns as soon as every gang is bound.
        res = native().run_open_loop(sh.store, sh.sched, json.dumps(gangs), offsets, hold_us, 20_000_000)
        assert len(res["gangs"]) == len(gangs)
        for g, k in zip(res["gangs"], kinds):
            assert g["bound_us"] > 0, g
            assert g["create_us"] <= g["first_enqueue_us"] <= g["admit_us"] <= g["bound_us"]
            assert g["size"] == (4 if k == "cpx4" else int(k))
        # Every gang was deleted again: the cluster is empty afterwards.
        sh.sched.wait_idle(10_000)
        assert sh.sched.wait_cache_empty(10.0)
        assert sh.store.count("pods") == 0 and sh.store.count("podgroups") == 0
        out = run_open_loop(sh, 800.0, duration_s=0.2, seed=2)
        assert out["gangs"] > 0 and all(v["unbound"] == 0 for v in out["by_gang"].values())
        for v in out["by_gang"].values():
            assert v["create_to_bound_ms"]["p99"] >= v["create_to_bound_ms"]["p50"] > 0
    finally:
        sh.close()


def test_burst_summary_splits_cpx_gangs():
    recs = [{"pod_group": "ns/s1-0003-x4", "size": 4, "first_enqueue_us": 0, "bound_us": 1000},
            {"pod_group": "ns/s1-0001-q", "size": 4, "first_enqueue_us": 0, "bound_us": 9000},
            {"pod_group": "ns/s1-0000-x1", "size": 1, "first_enqueue_us": 0, "bound_us": 500}]
    mixed = gang_latency_summary(recs)
    assert mixed["4"]["n"] == 2
    typed = gang_latency_summary(recs, by_type=True)
    assert list(typed) == ["1", "4", "cpx4"]
    assert typed["4"]["p99_ms"] == 1.0 and typed["cpx4"]["p99_ms"] == 9.0


def test_recreated_podgroup_starts_a_fresh_gang_record():
    """A gang deleted before admission leaves no open record behind: a later
    PodGroup of the same name is timed from its own first enqueue (the open
    loop reuses names across runs; a stale record would both inflate the
    latency and count the old binds toward the new gang)."""
    import time

    from flex_gpu_scheduler_amd.models import GPU, make_pod, make_pod_group

    sh = Shard(ClusterSpec(nodes=2), namespace="b")
    try:
        st, s = sh.store, sh.sched
        st.create("podgroups", make_pod_group("g", "b", 2))
        st.create("pods", make_pod("g-0", "b", limits={GPU: "1"}, pod_group="g"))
        end = time.time() + 5
        while s.stats()["attempts"] == 0 and time.time() < end:
            time.sleep(0.01)
        st.delete("pods", "b", "g-0")
        st.delete("podgroups", "b", "g")
        time.sleep(0.5)
        st.create("podgroups", make_pod_group("g", "b", 2))
        st.create_many("pods", json.dumps([make_pod(f"g-{i}", "b", limits={GPU: "1"}, pod_group="g")
                                           for i in range(2)]))
        assert s.wait_bound(2, 10.0)
        end = time.time() + 5
        recs = []
        while not recs and time.time() < end:
            recs = [r for r in s.gang_records(True) if r["pod_group"] == "b/g"]
            time.sleep(0.01)
        (r,) = recs
        assert r["size"] == 2 and (r["bound_us"] - r["first_enqueue_us"]) < 400_000
    finally:
        sh.close()


def test_wave_chunks_write_each_podgroup_before_its_pods():
    """Wave.chunks_json (bench.py's default creation order): every PodGroup
    and pod exactly once, chunks of >= 64 pods ending on a gang boundary, and
    each pod's PodGroup in its own chunk or an earlier one. The shard binds
    the whole wave created that way."""
    from flex_gpu_scheduler_amd.models.objects import POD_GROUP_LABEL
    from flex_gpu_scheduler_amd.utils.workload import make_wave

    spec = ClusterSpec(nodes=16)
    w = make_wave(spec, 2)
    chunks = [(json.loads(g), json.loads(p)) for g, p in w.chunks_json()]
    assert sorted(pg["metadata"]["name"] for g, _ in chunks for pg in g) == \
        sorted(pg["metadata"]["name"] for pg in w.pod_groups)
    assert [p["metadata"]["name"] for _, ps in chunks for p in ps] == [p["metadata"]["name"] for p in w.pods]
    created: set[str] = set()
    for i, (groups, pods) in enumerate(chunks):
        created |= {pg["metadata"]["name"] for pg in groups}
        for p in pods:
            g = p["metadata"].get("labels", {}).get(POD_GROUP_LABEL)
            assert not g or g in created
        if i + 1 < len(chunks):
            assert len(pods) >= 64
            last = pods[-1]["metadata"].get("labels", {}).get(POD_GROUP_LABEL)
            first_next = chunks[i + 1][1][0]["metadata"].get("labels", {}).get(POD_GROUP_LABEL)
            assert not last or last != first_next
    sh = Shard(spec, namespace="bench")
    try:
        r = sh.run(w, prepared=w.chunks_json())
        assert r.pods == len(w.pods)
    finally:
        sh.close()


def test_burst_wave_interleaves_cpx_gangs_in_queue_order():
    """CPX quarter gangs are spread through the wave and their names sort in
    creation order (the queue's tie-break after PodGroup creation time), so
    they no longer all queue behind the whole-GPU gangs."""
    from flex_gpu_scheduler_amd.utils.workload import make_wave

    w = make_wave(ClusterSpec(nodes=64), 3)
    names = [pg["metadata"]["name"] for pg in w.pod_groups]
    assert names == sorted(names)
    cpx = [i for i, n in enumerate(names) if n.endswith("-q")]
    assert len(cpx) > 10 and len(names) - len(cpx) > 10
    # Evenly spread: the first CPX gang comes early, the last one late.
    assert cpx[0] < len(names) // 5 and cpx[-1] > len(names) * 4 // 5
    sizes = {pg["spec"]["minMember"] for pg in w.pod_groups if not pg["metadata"]["name"].endswith("-q")}
    assert sizes == {1, 2, 4, 8}


def test_capacity_search_reaches_the_burst_rate(monkeypatch):
    """The search's ladder must not cap the capacity below the burst rate:
    its last rung is the burst rate itself. It climbs x1.3, then x1.07 from
    one x1.3 step under the burst rate, stops at the first failed rate (no
    trial follows a failure), and runs one trial per rate, two near the top."""
    from flex_gpu_scheduler_amd.utils import openloop

    tried = []

    def fake_run(shard, rate, duration_s=1.0, seed=0, occupancy=0.5, timeline=False):
        tried.append(round(rate))
        ok = rate <= limit
        return {"all_gangs": {"p99_create_to_bound_ms": 1.0 if ok else 90.0, "unbound": 0,
                              "p999_create_to_bound_ms": 1.0, "max_create_to_bound_ms": 1.0},
                "gangs": 10, "wall_s": 1.0, "denials": {"total": 0, "causes": {}}, "denied_gang_fraction": 0.0,
                "parked_gangs": 0}

    monkeypatch.setattr(openloop, "run_open_loop", fake_run)
    limit = 1e9  # every rate served: the capacity is the burst rate
    assert openloop.open_loop_capacity(None, 120_000.0) == 120_000.0
    # One trial per rate, two within two x1.3 steps of the burst rate.
    top = 120_000.0 / 1.3 ** 2
    for r in set(tried):
        assert tried.count(r) == (2 if r >= top else 1), (r, tried)
    rates = sorted(set(tried))
    steps = [b / a for a, b in zip(rates, rates[1:])]
    assert all(abs(x - 1.3) < 1e-2 or x <= 1.07 + 1e-2 for x in steps), steps
    assert rates[-1] == 120_000 and any(x <= 1.071 for x in steps)
    tried.clear()
    limit = 110_000.0  # the edge under the burst rate: found to within one x1.07 step
    cap = openloop.open_loop_capacity(None, 120_000.0)
    assert 110_000 / 1.071 < cap <= 110_000, cap
    assert max(tried) > 110_000 and tried[-1] == max(tried)  # the failed rate is the last trial
    tried.clear()
    limit = 50_000.0  # an ordinary failing coarse step: the search ends there
    out: dict = {}
    cap = openloop.open_loop_capacity(None, 120_000.0, outcome=out)
    assert 50_000 / 1.31 < cap <= 50_000 and max(tried) < 120_000 and tried[-1] == max(tried)
    assert round(out["failed_at"]) == max(tried)
    # The retry in a fresh process resumes the ladder at the failed rung: a
    # transient failure (the rung passes now) lets the climb go on from it.
    tried.clear()
    limit = 110_000.0
    rung = out["failed_at"]
    cap2 = openloop.open_loop_capacity(None, 120_000.0, resume_at=rung, outcome=out)
    assert tried[0] == round(rung) and 110_000 / 1.071 < cap2 <= 110_000 and out["failed_at"] > 110_000
    tried.clear()
    limit = 1.0  # the resumed rung fails again: nothing gained
    assert openloop.open_loop_capacity(None, 120_000.0, resume_at=66_000.0, outcome=out) == 0.0
    assert tried == [66_000] and out["failed_at"] == 66_000.0


def test_capacity_report_in_a_gpu_free_child():
    """bench.py runs the open-loop block in a child process on a fresh shard
    (utils/openloop.py capacity_in_child): the child must not load torch (the
    GPU runtime in the process is what it avoids) and must return the search
    and both loads."""
    import subprocess
    import sys

    from flex_gpu_scheduler_amd.utils.openloop import capacity_in_child

    probe = subprocess.run([sys.executable, "-c", "import sys, flex_gpu_scheduler_amd.utils.openloop, "
                            "flex_gpu_scheduler_amd.utils.benchrun; print('torch' in sys.modules)"],
                           capture_output=True, text=True, check=True)
    assert probe.stdout.strip() == "False"
    rep = capacity_in_child(16, 0, {}, 2600.0, warm_waves=2, timeout_s=300)
    assert rep["capacity"] > 0 and rep["search"], rep
    assert {"load_50", "load_90"} <= set(rep)
    assert rep["load_90"]["all_gangs"]["unbound"] == 0
