"""Service-mode throughput: the scheduler against an API server in another
process, over HTTP (the deployment shape: informers LIST/WATCH the remote
API, bindings and PodGroup patches go back as REST calls).

Starts `flex_gpu_scheduler_amd.cli apiserver` as a child process, loads
MI355X nodes and the pods (plain, or 8-rank gangs within the GPU capacity),
then starts RemoteScheduler in this process and reports pods/s from its start
(LIST/WATCH sync included) to the last binding seen by the API.

    python -m flex_gpu_scheduler_amd.tools.remote_bench [--nodes 64] [--pods 2000] [--gangs]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor


def run(nodes: int, pods: int, gangs: bool, bind_workers: int, clients: int, native_io: bool = True) -> dict:
    from ..config import load_config
    from ..control import RestClient
    from ..control.remote import RemoteScheduler
    from ..models import GPU, make_pod, make_pod_group, mi355x_node
    from ..utils.workload import flagship_config

    srv = subprocess.Popen([sys.executable, "-m", "flex_gpu_scheduler_amd.cli", "apiserver", "--port", "0",
                            "--bind-address", "127.0.0.1"], stdout=subprocess.PIPE, text=True)
    try:
        url = json.loads(srv.stdout.readline())["apiserver"]
        admin = RestClient(url)
        for i in range(nodes):
            admin.create("nodes", mi355x_node(f"mi-{i}"))
        cfg = load_config(flagship_config())
        objs = []
        if gangs:
            for g in range(min(pods, nodes * 8) // 8):
                objs.append(("podgroups", make_pod_group(f"g{g}", "default", 8)))
                objs += [("pods", make_pod(f"g{g}-r{r}", pod_group=f"g{g}", requests={"cpu": "4"},
                                           limits={GPU: "1"})) for r in range(8)]
        else:
            objs = [("pods", make_pod(f"p{i}", requests={"cpu": "1", "memory": "1Gi"})) for i in range(pods)]
        n_pods = sum(1 for k, _ in objs if k == "pods")
        # The pods exist before the scheduler starts (the API server's own
        # create rate is not what is measured): the clock runs from the
        # scheduler's start (LIST + WATCH sync) to the last binding the API
        # reports.
        pool = [RestClient(url) for _ in range(clients)]
        t_c = time.perf_counter()
        with ThreadPoolExecutor(clients) as ex:
            chunks = [objs[i::clients] for i in range(clients)]
            list(ex.map(lambda a: [a[0].create(k, o) for k, o in a[1]], zip(pool, chunks)))
        create_s = time.perf_counter() - t_c
        t0 = time.perf_counter()
        rs = RemoteScheduler(RestClient(url), cfg, native_io=native_io, bindWorkers=bind_workers).start()
        try:
            t_synced = time.perf_counter()
            deadline = t0 + 300
            diag = None
            while rs.scheduler.stats()["bound"] < n_pods and time.perf_counter() < deadline:
                if diag is None and time.perf_counter() - t0 > 5:  # stalled: record why
                    diag = {"stats": rs.scheduler.stats(), "queue": rs.scheduler.queue_counts(),
                            "cache": rs.scheduler.cache_counts(), "local_pods": rs.store.count("pods"),
                            "local_podgroups": rs.store.count("podgroups"),
                            "waiting": len(rs.scheduler.waiting_pods()),
                            "relists": getattr(rs.mirror, "relists", None)}
                    stuck = rs.scheduler.dump_cache()["queue"]["pods"]
                    if stuck:
                        ns, name = stuck[0].split("/", 1)
                        e = rs.scheduler.explain(rs.store.get("pods", ns, name))
                        diag["stuck"] = stuck[:8]
                        diag["explain"] = {k: e.get(k) for k in ("code", "message", "feasible")}
                        diag["filtered"] = dict(list((e.get("filtered") or {}).items())[:3])
                time.sleep(0.005)
            bound = rs.scheduler.stats()["bound"]
            t_bound = time.perf_counter()
            while time.perf_counter() < deadline:
                items = admin.list("pods", "default")[0]
                if sum(1 for p in items if p["spec"].get("nodeName")) >= n_pods:
                    break
                time.sleep(0.01)
            t_api = time.perf_counter()
            return {"nodes": nodes, "pods": n_pods, "gangs": gangs, "bind_workers": bind_workers, "native_io": rs.native_io,
                    "bound": bound, "create_s": round(create_s, 3), "sync_s": round(t_synced - t0, 3),
                    "bound_s": round(t_bound - t0, 3), "api_visible_s": round(t_api - t0, 3),
                    "pods_per_s": round(n_pods / (t_api - t0), 1), **({"stall": diag} if diag else {})}
        finally:
            rs.stop()
    finally:
        srv.terminate()
        srv.wait(10)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--pods", type=int, default=2000)
    ap.add_argument("--gangs", action="store_true")
    ap.add_argument("--bind-workers", type=int, default=16)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--python-io", action="store_true", help="Python mirror and writer instead of the native ones")
    a = ap.parse_args()
    print(json.dumps(run(a.nodes, a.pods, a.gangs, a.bind_workers, a.clients, native_io=not a.python_io)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
