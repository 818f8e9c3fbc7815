"""Service-mode throughput: the scheduler against an API server in another
process, over HTTP (the deployment shape: informers LIST/WATCH the remote
API, bindings and PodGroup patches go back as REST calls).

Starts `flex_gpu_scheduler_amd.cli apiserver` as a child process, loads
MI355X nodes and the pods (plain, or 8-rank gangs within the GPU capacity),
then starts RemoteScheduler in this process and reports pods/s from its start
(LIST/WATCH sync included) to the last binding the API server acknowledged,
the rate after the initial sync, and a per-phase timeline (first/half/all of
the pods mirrored, attempted, bound). The API server's HTTP front end is the
native one (csrc/apiserver) unless --python-http.

    python -m flex_gpu_scheduler_amd.tools.remote_bench [--nodes 128] [--pods 8000] [--gangs] [--matrix]
    python -m flex_gpu_scheduler_amd.tools.remote_bench --steady [--duration 2] [--creators 8]

`--steady` (run_steady) is the steady-state form: the scheduler is synced
first, then separate creator processes POST pods over HTTP for `duration`
seconds while it schedules them; the rate is the bindings completed per
second over the window that excludes the first quarter second, with the
offered create rate and the backlog next to it.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor


def _phases(timeline: list[tuple], n_pods: int, bound: int, t_bound: float) -> dict:
    """Seconds from the scheduler's start until the first/half/all of the
    pods were mirrored, attempted and bound, and the REST requests sent."""
    def first(col: int, target: float):
        for row in timeline:
            if row[col] >= target:
                return round(row[0], 4)
        return None

    out = {}
    for name, col in (("mirrored", 1), ("attempted", 2), ("bound", 3)):
        out[name] = {"first": first(col, 1), "half": first(col, n_pods / 2), "all": first(col, n_pods)}
    out["bound"]["all"] = round(t_bound, 4) if bound >= n_pods else None
    out["rest_requests"] = timeline[-1][4] if timeline else 0
    return out


def run(nodes: int, pods: int, gangs: bool, bind_workers: int, clients: int, native_io: bool = True,
        native_http: bool = True) -> dict:
    from ..config import load_config
    from ..control import RestClient
    from ..control.remote import RemoteScheduler
    from ..models import GPU, make_pod, make_pod_group, mi355x_node
    from ..utils.cpuaffinity import child_env
    from ..utils.workload import flagship_config

    srv = subprocess.Popen([sys.executable, "-m", "flex_gpu_scheduler_amd.cli", "apiserver", "--port", "0",
                            "--bind-address", "127.0.0.1"] + ([] if native_http else ["--python-http"]),
                           stdout=subprocess.PIPE, text=True, env=child_env())
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
            # Per-phase timeline (sampled every ~1 ms): pods mirrored into the
            # scheduler's store, scheduling attempts, bindings confirmed by
            # the scheduler, REST requests sent.
            timeline = []
            while rs.scheduler.stats()["bound"] < n_pods and time.perf_counter() < deadline:
                st = rs.scheduler.stats()
                timeline.append((time.perf_counter() - t0, rs.mirror.applied, st["attempts"], st["bound"],
                                 rs.client.requests() if hasattr(rs.client, "requests") else 0))
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
                time.sleep(0.001)
            bound = rs.scheduler.stats()["bound"]
            t_bound = time.perf_counter()
            # A binding counts once the API server answered the POST (the
            # scheduler's bound counter); one LIST afterwards (untimed)
            # checks that every pod carries its nodeName on the server.
            api_bound = sum(1 for p in admin.list("pods", "default")[0] if p["spec"].get("nodeName"))
            phases = _phases(timeline, n_pods, bound, t_bound - t0)
            return {"nodes": nodes, "pods": n_pods, "gangs": gangs, "bind_workers": bind_workers, "native_io": rs.native_io,
                    "apiserver": "native" if native_http else "python", "phases": phases,
                    "bound": bound, "api_bound": api_bound, "create_s": round(create_s, 3),
                    "sync_s": round(t_synced - t0, 3), "bound_s": round(t_bound - t0, 3),
                    # from the scheduler's start (LIST+WATCH sync included)
                    "pods_per_s": round(n_pods / (t_bound - t0), 1),
                    # after the initial sync: the steady binding rate
                    "pods_per_s_after_sync": round(n_pods / max(1e-9, t_bound - t_synced), 1),
                    **({"stall": diag} if diag else {})}
        finally:
            rs.stop()
    finally:
        srv.terminate()
        srv.wait(10)


def _creator(url: str, prefix: str, duration_s: float, out_fd: int, depth: int = 1) -> None:
    """One creator process: POST plain pods over one keep-alive connection
    for `duration_s` seconds, `depth` requests in flight (HTTP/1.1
    pipelining: a batch of requests is written, then their responses are
    read; the native API server parses requests from a buffered stream, so a
    batch costs one round trip instead of `depth`). Writes {"created", "t0",
    "t1"} (monotonic)."""
    import socket
    from urllib.parse import urlsplit

    from ..models import make_pod
    from ..utils.cpuaffinity import adopt_child_cpus

    adopt_child_cpus()
    u = urlsplit(url)
    sock = socket.create_connection((u.hostname, u.port))
    sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    tmpl = json.dumps(make_pod("NAME", requests={"cpu": "100m", "memory": "128Mi"}), separators=(",", ":"))
    head = (f"POST /api/v1/namespaces/default/pods HTTP/1.1\r\nHost: {u.hostname}\r\n"
            "Content-Type: application/json\r\nAccept: application/json\r\nContent-Length: ")
    buf = bytearray()

    def read_response() -> int:
        nonlocal buf
        while True:
            e = buf.find(b"\r\n\r\n")
            if e >= 0:
                break
            chunk = sock.recv(1 << 16)
            if not chunk:
                raise SystemExit("connection closed")
            buf += chunk
        hdr = bytes(buf[:e]).decode("latin-1")
        status = int(hdr.split(" ", 2)[1])
        length = 0
        for line in hdr.split("\r\n")[1:]:
            k, _, v = line.partition(":")
            if k.strip().lower() == "content-length":
                length = int(v.strip())
        while len(buf) < e + 4 + length:
            chunk = sock.recv(1 << 16)
            if not chunk:
                raise SystemExit("connection closed")
            buf += chunk
        del buf[:e + 4 + length]
        return status

    i = 0
    t0 = time.monotonic()
    end = t0 + duration_s
    depth = max(1, depth)
    while time.monotonic() < end:
        out = []
        for k in range(depth):
            body = tmpl.replace('"NAME"', f'"{prefix}-{i + k}"', 1).encode()
            out.append(head.encode() + str(len(body)).encode() + b"\r\n\r\n" + body)
        sock.sendall(b"".join(out))
        for _ in range(depth):
            st = read_response()
            if st not in (200, 201):
                raise SystemExit(f"create failed: {st}")
        i += depth
    sock.close()
    os.write(out_fd, json.dumps({"created": i, "t0": t0, "t1": time.monotonic()}).encode())


def run_steady(nodes: int = 128, duration_s: float = 2.0, creators: int = 8, bind_workers: int = 16,
               warm_s: float = 0.25, depth: int = 1) -> dict:
    """Steady-state service mode: pods are created over HTTP by `creators`
    separate processes (`depth` pipelined requests each) while the (already
    synced) scheduler binds them. `generator_limited` is true when the
    scheduler kept up (bound within 10% of the offered creates and a small
    backlog at the last create): the bound rate is then the generator's, not
    the scheduler's ceiling."""
    from ..config import load_config
    from ..control import RestClient
    from ..control.remote import RemoteScheduler
    from ..models import mi355x_node
    from ..utils.cpuaffinity import child_env
    from ..utils.workload import flagship_config

    srv = subprocess.Popen([sys.executable, "-m", "flex_gpu_scheduler_amd.cli", "apiserver", "--port", "0",
                            "--bind-address", "127.0.0.1"], stdout=subprocess.PIPE, text=True, env=child_env())
    procs: list[tuple[subprocess.Popen, int]] = []
    try:
        url = json.loads(srv.stdout.readline())["apiserver"]
        admin = RestClient(url)
        for i in range(nodes):  # room for every pod of the window (2,000 per node)
            admin.create("nodes", mi355x_node(f"mi-{i}", pods=2000))
        rs = RemoteScheduler(RestClient(url), load_config(flagship_config()), bindWorkers=bind_workers).start()
        try:
            code = ("import sys; from flex_gpu_scheduler_amd.tools.remote_bench import _creator; "
                    "_creator(sys.argv[1], sys.argv[2], float(sys.argv[3]), 1, int(sys.argv[4]))")
            root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            env = child_env()
            env["PYTHONPATH"] = root + os.pathsep + os.environ.get("PYTHONPATH", "")
            base = rs.scheduler.stats()["bound"]
            t_start = time.monotonic()
            for c in range(creators):
                p = subprocess.Popen([sys.executable, "-c", code, url, f"c{c}", str(duration_s), str(depth)],
                                     stdout=subprocess.PIPE, env=env)
                procs.append((p, c))
            samples = []  # (t, bound) every ~5 ms
            while any(p.poll() is None for p, _ in procs):
                samples.append((time.monotonic(), rs.scheduler.stats()["bound"] - base))
                time.sleep(0.005)
            made = []
            for p, _ in procs:
                out, _ = p.communicate(timeout=30)
                if p.returncode != 0:
                    raise RuntimeError(f"creator exited {p.returncode}")
                made.append(json.loads(out))
            created = sum(m["created"] for m in made)
            t_first = min(m["t0"] for m in made)
            t_last = max(m["t1"] for m in made)
            deadline = time.monotonic() + 60
            while rs.scheduler.stats()["bound"] - base < created and time.monotonic() < deadline:
                time.sleep(0.002)
            t_drained = time.monotonic()
            bound = rs.scheduler.stats()["bound"] - base
            # Steady window: from warm_s after the first create to the last one.
            w0, w1 = t_first + warm_s, t_last
            inwin = [(t, b) for t, b in samples if w0 <= t <= w1]
            rate = (inwin[-1][1] - inwin[0][1]) / (inwin[-1][0] - inwin[0][0]) if len(inwin) >= 2 else 0.0
            at_end = next((b for t, b in reversed(samples) if t <= t_last), 0)
            offered = created / max(1e-9, t_last - t_first)
            backlog = created - at_end
            return {"nodes": nodes, "creators": creators, "pipeline_depth": depth, "duration_s": duration_s,
                    "created": created, "bound": bound, "all_bound": bound >= created,
                    "offered_creates_per_s": round(offered, 1),
                    "pods_per_s": round(rate, 1),
                    "generator_limited": bool(rate >= 0.9 * offered and backlog <= 0.05 * created),
                    "window_s": round(max(0.0, w1 - w0), 3),
                    "backlog_at_last_create": created - at_end,
                    "drain_after_last_create_s": round(t_drained - t_last, 4),
                    "start_delay_s": round(t_first - t_start, 3)}
        finally:
            rs.stop()
    finally:
        for p, _ in procs:
            if p.poll() is None:
                p.kill()
        srv.terminate()
        srv.wait(10)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--nodes", type=int, default=128)
    ap.add_argument("--pods", type=int, default=8000)
    ap.add_argument("--gangs", action="store_true")
    ap.add_argument("--bind-workers", type=int, default=16)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--python-io", action="store_true", help="Python mirror and writer instead of the native ones")
    ap.add_argument("--python-http", action="store_true", help="the API server's http.server front end")
    ap.add_argument("--steady", action="store_true", help="steady-state: creates over HTTP while scheduling")
    ap.add_argument("--duration", type=float, default=2.0)
    ap.add_argument("--creators", type=int, default=8)
    ap.add_argument("--matrix", action="store_true",
                    help="plain and 8-rank gang runs, native and Python API server front ends")
    a = ap.parse_args()
    if a.steady:
        print(json.dumps(run_steady(a.nodes, a.duration, a.creators, a.bind_workers)), flush=True)
        return 0
    if a.matrix:
        for native_http in (True, False):
            for g, n in ((False, a.pods), (True, min(a.pods, a.nodes * 8))):
                print(json.dumps(run(a.nodes, n, g, a.bind_workers, a.clients, native_http=native_http)), flush=True)
        return 0
    print(json.dumps(run(a.nodes, a.pods, a.gangs, a.bind_workers, a.clients, native_io=not a.python_io,
                         native_http=not a.python_http)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
