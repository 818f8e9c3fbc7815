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
           "--steps", "2", "--warmup", "1", "--nodes", "8", "--no-gpu-probe", "--no-scenarios", "--no-open-loop"]
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
           "--no-gpu-probe", "--no-scenarios", "--cpus", "none"]
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
    for load in ("load_50", "load_90"):
        assert set(ol[load]["by_gang"]) <= {"1", "2", "4", "8", "cpx4"} and ol[load]["gangs"] > 0
    assert "cpx4" in d["config"]["gang_admit_by_type"]


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, PYTHONPATH=ROOT, WORLD_SIZE="1", RANK="0", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--steps", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
