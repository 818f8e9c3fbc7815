"""The bench's multi-rank path (one scheduler shard per rank, barrier-bracketed
timing, max-over-ranks time, summed pods) under torch.distributed.run with the
gloo backend on CPU — the same code path the 8-GPU run takes with RCCL."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
@pytest.mark.parametrize("n", [2, 4])
def test_bench_multi_rank_gloo(n):
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", str(n),
           "--steps", "2", "--warmup", "1", "--nodes", "8", "--waves-per-step", "2", "--no-gpu-probe",
           "--no-scenarios", "--no-open-loop", "--no-service-mode"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    d = lines[0]
    assert d["n_gpus"] == n and d["steps"] == 2 and d["scaling"] == "weak"
    assert d["value"] > 0 and d["config"]["parallelism"].startswith(f"{n} rank(s)")
    # Every rank's gangs are in the latency summary (gathered over ranks).
    total = sum(v["n"] for v in d["config"]["gang_admit"].values())
    assert total > 0


@pytest.mark.slow
def test_bench_launches_its_own_ranks():
    """`python bench.py --gpus 2` (no torchrun) starts two ranks itself, reports
    the real world size, and runs the placement validation: gangs scheduled on
    the node, resolved by the device plugin's Allocate, all-reduced on exactly
    the allocated ranks (gloo here; RCCL on the GPU node)."""
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--nodes", "8",
           "--waves-per-step", "2", "--no-gpu-probe", "--no-scenarios", "--no-service-mode", "--cpus", "none"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["parallelism"].startswith("2 rank")
    pl = d["config"]["rccl_placement"]
    assert [g["gang"] for g in pl["gangs"]] == [1, 2]
    g2 = pl["gangs"][1]
    assert sorted(g2["gpus"]) == [0, 1] and sorted(g2["ordinals"]) == [0, 1]
    assert g2["placed"]["ranks"] == [0, 1] and all(x["correct"] for x in g2["placed"]["results"])
    assert pl["summary"]["2"]["all_correct"]
    # Untimed open-loop admission latency, by interleaved gang type.
    ol = d["config"]["gang_admit_open_loop"]
    assert ol["capacity_pods_per_s"] > 0
    # The frozen search logs one trial per rate, with its gang denials.
    assert ol["capacity_search"] and all({"offered_pods_per_s", "served", "denied_gangs", "denial_causes"}
                                         <= set(t) for t in ol["capacity_search"])
    assert len(d["config"]["per_rank"]["pods_per_s"]) == 2
    for load in ("load_50", "load_90"):
        assert set(ol[load]["by_gang"]) <= {"1", "2", "4", "8", "cpx4"} and ol[load]["gangs"] > 0
    assert "cpx4" in d["config"]["gang_admit_by_type"]


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, PYTHONPATH=ROOT, WORLD_SIZE="1", RANK="0", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--steps", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


@pytest.mark.slow
def test_bench_eight_ranks_self_launched_gloo():
    """The 8-GPU shape of the driver's scaling run, rehearsed on CPU: `python
    bench.py --gpus 8` starts 8 ranks itself (GPUs counted from sysfs, no HIP
    in the parent), every rank reports its own rate, and the placement check
    fills the 1/2/4/8 gang rows with correct all-reduces on the placed ranks."""
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "8", "--steps", "1", "--warmup", "1", "--nodes", "4",
           "--waves-per-step", "1", "--no-gpu-probe", "--no-scenarios", "--no-open-loop", "--no-service-mode",
           "--cpus", "none"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == 8 and d["config"]["parallelism"].startswith("8 rank")
    pr = d["config"]["per_rank"]
    assert len(pr["pods_per_s"]) == 8 and min(pr["pods_per_s"]) > 0 and pr["spread"] >= 0
    assert "independent" in d["config"]["value_kind"]
    pl = d["config"]["rccl_placement"]
    assert "error" not in pl, pl
    assert [g["gang"] for g in pl["gangs"]] == [1, 2, 4, 8]
    for g in pl["gangs"][1:]:
        assert len(g["ordinals"]) == g["gang"] and sorted(g["placed"]["ranks"]) == sorted(g["ordinals"])
        assert all(x["correct"] for x in g["placed"]["results"])
        assert pl["summary"][str(g["gang"])]["all_correct"]
        # The xGMI model exists for every multi-rank gang of the (fake, full
        # mesh) node; on gloo there is no xGMI data plane to judge: n/a.
        assert g["model"]["model_busbw_GBps"] > 0 and g["model"]["direct_links_min"] == g["gang"] - 1
        assert g["verdict"] == "n/a" and pl["summary"][str(g["gang"])]["verdict"] == "n/a"
    assert pl["gangs"][0]["verdict"] == "n/a"
    # The single-node multi-GPU scalars lead `config` (the driver keeps
    # scalars): per gang size the verdict and placed busBW, the cross-socket
    # ratio, and the one-line headline that carries them.
    c = d["config"]
    keys = list(c)
    for k in ("2", "4", "8"):
        assert c[f"placement_verdict_{k}"] == "n/a"  # gloo: no xGMI data plane to judge
        assert isinstance(c[f"placed_busbw_GBps_{k}"], float) and c[f"placed_busbw_GBps_{k}"] > 0
        assert keys.index(f"placement_verdict_{k}") < keys.index("per_rank")
    assert "cross_socket_over_placed" in c and "placement[2/4/8]=n/a/n/a/n/a" in c["headline"]
    first_dict = next(i for i, k in enumerate(keys) if isinstance(c[k], (dict, list)))
    assert all(not isinstance(c[k], (dict, list)) for k in keys[:first_dict])
    assert keys.index("headline") < 5


def test_visible_gpu_count_honours_visibility_lists(tmp_path):
    from flex_gpu_scheduler_amd.gpu.discovery import visible_gpu_count

    assert visible_gpu_count(str(tmp_path), env={}) == 0  # no sysfs: unknown, not a refusal
    root = os.path.join(ROOT, "tests", "fixtures", "mi355x_box", "root")
    n = visible_gpu_count(root, env={})
    assert n >= 1
    assert visible_gpu_count(root, env={"HIP_VISIBLE_DEVICES": "0"}) == 1
    assert visible_gpu_count(root, env={"ROCR_VISIBLE_DEVICES": "0,1,2", "HIP_VISIBLE_DEVICES": "0"}) == min(3, n)


def test_placement_verdict_model():
    """busbw_model + judge_row on a full-mesh host: pass needs >= 70% of the
    model and a win over the host-staged path; gloo rows are n/a."""
    from flex_gpu_scheduler_amd.gpu.discovery import fake_host
    from flex_gpu_scheduler_amd.parallel.placement import RING_EFFICIENCY, busbw_model, judge_row

    host = fake_host(8)
    m8 = busbw_model(host, list(range(8)))
    # KFD io_links max_bandwidth is one way: the captured box reads 76,000
    # MB/s per xGMI link (below), as fake_host does: 7 links x 76 GB/s.
    assert m8["direct_links_min"] == 7 and abs(m8["model_busbw_GBps"] - RING_EFFICIENCY * 7 * 76.0) < 0.2
    assert busbw_model(host, [0, 5])["direct_links_min"] == 1
    assert busbw_model(host, [3])["model_busbw_GBps"] is None

    def row(placed, staged, correct=True):
        res = lambda bw: {"results": [{"MiB": 16, "busbw_GBps": bw / 4, "correct": correct},  # noqa: E731
                                      {"MiB": 256, "busbw_GBps": bw, "correct": correct}]}
        return {"gang": 8, "placed": res(placed), "host_staged": res(staged), "cross_socket": res(placed * 0.98)}

    good = judge_row(row(0.8 * m8["model_busbw_GBps"], 10.0), m8, "nccl")
    assert good["verdict"] == "pass" and abs(good["cross_socket_over_placed"] - 0.98) < 1e-6
    assert judge_row(row(0.5 * m8["model_busbw_GBps"], 10.0), m8, "nccl")["verdict"] == "fail"
    assert judge_row(row(0.8 * m8["model_busbw_GBps"], 1e6), m8, "nccl")["verdict"] == "fail"
    assert judge_row(row(0.8 * m8["model_busbw_GBps"], 10.0, correct=False), m8, "nccl")["verdict"] == "fail"
    assert judge_row(row(1.0, 1.0), m8, "gloo")["verdict"] == "n/a"


def test_busbw_model_from_the_captured_box_io_links():
    """The MI355X box's KFD io_links (captured under tests/fixtures/mi355x_box)
    report 76,000 MB/s per xGMI link: the per-direction half of the part's
    153.6 GB/s bidirectional link. A full 8-rank gang with those links models
    0.75 x 7 x 76 = 399 GB/s of all-reduce bus bandwidth (RING_EFFICIENCY is an
    assumption; parity with a measured 8-GPU run is unpinned)."""
    import glob

    from flex_gpu_scheduler_amd.gpu.discovery import discover_host, fake_host
    from flex_gpu_scheduler_amd.parallel.placement import XGMI_LINK_GBPS_BIDIR, busbw_model

    root = os.path.join(ROOT, "tests", "fixtures", "mi355x_box", "root")
    bws = []
    for f in glob.glob(os.path.join(root, "sys/class/kfd/kfd/topology/nodes/*/io_links/*/properties")):
        props = dict(line.split() for line in open(f) if len(line.split()) == 2)
        if props.get("type") == "11":  # xGMI
            bws.append(int(props["max_bandwidth"]))
    assert len(bws) >= 7 and set(bws) == {76000}
    assert abs(bws[0] / 1000 - XGMI_LINK_GBPS_BIDIR / 2) < 1.0  # one way
    live = discover_host(root)
    g = [g for g in live.gpus if g.xgmi_links][0]
    assert {lk.bandwidth_mbps for lk in g.xgmi_links} == {76000}
    m8 = busbw_model(fake_host(8), list(range(8)))
    assert 395 <= m8["model_busbw_GBps"] <= 405 and m8["source"] == "kfd io_links"
    # Without a usable KFD figure the spec's one-way 76.8 GB/s stands in.
    host = fake_host(8)
    for gg in host.gpus:
        for lk in gg.xgmi_links:
            lk.bandwidth_mbps = 0
    assert abs(busbw_model(host, list(range(8)))["model_busbw_GBps"] - 0.75 * 7 * 76.8) < 0.2


def test_headline_scalars_on_one_gpu_read_na():
    """bench.headline_scalars: on one GPU the placement scalars read "n/a";
    the headline string carries every number the scalars hold."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    by_type = {k: {"p99_ms": 2.5} for k in ("1", "2", "4", "8", "cpx4")}
    split = {k: {"n": 10, "split": 0, "avoidable": 0, "split_fraction": 0.0} for k in ("2", "4", "8", "cpx4")}
    extras = {"open_loop_capacity_pods_per_s": 100000.0, "nodes1024_pods_per_s": 60000.0,
              "service_mode_pods_per_s": 70000.0, "service_mode_generator_limited": False,
              "denied_gang_fraction": 0.0, "parked_gang_fraction": 0.001,
              **{f"open_loop_p99_create_to_bound_ms_{k}": 0.9 for k in ("1", "2", "4", "8", "cpx4")},
              "scenarios": {"trimaran_tlp": {"gpus_sampled": 1, "replicated_from_gpu0": True}}}
    h = bench.headline_scalars(118000.0, by_type, split, extras, 1)
    assert list(h)[0] == "headline"
    for k in ("2", "4", "8"):
        assert h[f"placement_verdict_{k}"] == "n/a" and h[f"placed_busbw_GBps_{k}"] == "n/a"
    assert h["cross_socket_over_placed"] == "n/a" and h["tlp_replicated_from_gpu0"] is True
    for k in ("1", "2", "4", "8", "cpx4"):
        assert h[f"p99_gang_admit_ms_{k}"] == 2.5 and h[f"open_loop_p99_create_to_bound_ms_{k}"] == 0.9
    for k in ("2", "4", "8", "cpx4"):
        assert h[f"gang_split_fraction_{k}"] == 0.0
    assert "burst=118.0k" in h["headline"] and "n1024=60.0k" in h["headline"] and "open_loop=100.0k" in h["headline"]


def test_gang_fractions_count_served_runs_apart_from_the_failed_rung():
    """bench.gang_fractions: the headline parked/denied fractions are over the
    served open-loop runs; the failed (overloaded) rung only enters the
    *_all_trials figures."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    search = [{"served": True, "gangs": 1000, "parked_gangs": 2, "denied_gangs": 0},
              {"served": True, "gangs": 1000, "parked_gangs": 4, "denied_gangs": 1},
              {"served": False, "gangs": 1000, "parked_gangs": 900, "denied_gangs": 0}]
    loads = [{"gangs": 500, "parked_gangs": 0, "denials": {"total": 1}},
             {"gangs": 500, "parked_gangs": 2, "denials": {"total": 0}}]
    f = bench.gang_fractions(search, loads)
    assert f["parked_gang_fraction"] == round(8 / 3000, 6) and f["denied_gang_fraction"] == round(2 / 3000, 6)
    assert f["parked_gang_fraction_all_trials"] == round(908 / 4000, 6)
    assert f["denied_gang_fraction_all_trials"] == 2 / 4000
    assert bench.gang_fractions([], [])["parked_gang_fraction"] == 0.0
