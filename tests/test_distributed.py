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
           "--steps", "2", "--warmup", "1", "--nodes", "8", "--no-gpu-probe", "--no-scenarios"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    d = lines[0]
    assert d["n_gpus"] == n and d["steps"] == 2 and d["scaling"] == "weak"
    assert d["value"] > 0 and d["config"]["parallelism"].startswith(f"{n} scheduler shard")
    # Every rank's gangs are in the latency summary (gathered over ranks).
    total = sum(v["n"] for v in d["config"]["gang_admit"].values())
    assert total > 0
