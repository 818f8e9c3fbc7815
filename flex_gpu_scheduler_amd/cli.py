"""Command-line entry points (`python -m flex_gpu_scheduler_amd <command>`).

  scheduler    the scheduler service (reference: cmd/scheduler/main.go:30-51 =
               kube-scheduler + out-of-tree registry; here every plugin of the
               suite is registered, fixing SURVEY.md Appendix C9)
  controller   PodGroup + ElasticQuota controllers (cmd/controller, flags of
               cmd/controller/app/options.go:39-47)
  apiserver    the HTTP API server over the native store (envtest analog),
               with JSON checkpoint/restore of all objects
  node-agent   MI355X discovery -> Node/NRT/telemetry publisher
  manager      controller-runtime style PodGroup/ElasticQuota reconcilers
               (the kustomize scaffold's /manager, deploy/config)
  load-watcher GET /watcher over the published WatcherMetrics (:2020), or a
               library-mode watcher over metrics-server/Prometheus/SignalFx
  explain      dry-run one pod against the live cluster and print filter
               verdicts, per-plugin scores and the chosen node
  apply        create/replace objects from YAML/JSON files (a tiny kubectl)
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import signal
import socket
import sys
import threading
from pathlib import Path

log = logging.getLogger("xsched")


# ------------------------------------------------------------------ helpers
class JsonLogFormatter(logging.Formatter):
    """One JSON object per line, every field escaped by json.dumps (the
    native core writes the same shape, csrc/common/log.cc)."""

    def format(self, record: logging.LogRecord) -> str:
        d = {"ts": self.formatTime(record), "level": record.levelname, "logger": record.name,
             "caller": f"{record.filename}:{record.lineno}", "msg": record.getMessage()}
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d)


def _setup_logging(v: int, fmt: str = "json") -> None:
    """--v for both halves: Python logging level, and the native core's klog
    verbosity (V(6) dumps FlexGPU/NRT ledgers and chosen GPU indexes)."""
    level = logging.WARNING if v <= 0 else logging.INFO if v < 5 else logging.DEBUG
    handler = logging.StreamHandler()
    handler.setFormatter(JsonLogFormatter() if fmt == "json" else
                         logging.Formatter("%(levelname).1s%(asctime)s %(filename)s:%(lineno)d] %(message)s"))
    root = logging.getLogger()
    root.handlers[:] = [handler]
    root.setLevel(level)
    try:
        from ._native import native

        native().set_log_verbosity(int(v))
        native().set_log_json(fmt == "json")
    except ImportError:  # native core not built (CPU-only tooling)
        pass


def master_from_kubeconfig(path: str) -> tuple[str, str | None]:
    """(server URL, bearer token) of the current context of a kubeconfig."""
    from .control.client import kubeconfig_connection

    server, token, _ = kubeconfig_connection(path)
    return server, token


def _client(args):
    from .control.client import IN_CLUSTER_SA, RestClient, TLSConfig, kubeconfig_connection

    master = getattr(args, "master", None) or getattr(args, "masterUrl", None)
    token = getattr(args, "token", None)
    tls = TLSConfig(insecure=bool(getattr(args, "insecure_skip_tls_verify", False)))
    kc = getattr(args, "kubeconfig", None) or getattr(args, "kubeConfig", None)
    if kc and not master:
        master, kt, tls = kubeconfig_connection(kc)
        token = token or kt
    if getattr(args, "incluster", False) and not master:
        # rest.InClusterConfig: service host/port, the service-account token and CA.
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        master = f"https://{host}:{port}"
        tok, ca = os.path.join(IN_CLUSTER_SA, "token"), os.path.join(IN_CLUSTER_SA, "ca.crt")
        if os.path.exists(tok):
            token = Path(tok).read_text().strip()
        if os.path.exists(ca):
            tls = TLSConfig(ca_file=ca)
    return RestClient(master or "http://127.0.0.1:6443", token=token, tls=tls)


def _wait_forever(stop: threading.Event) -> None:
    def handler(*_):
        stop.set()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            signal.signal(sig, handler)
        except ValueError:  # not the main thread
            pass
    while not stop.is_set():
        stop.wait(1.0)


def _hostport(s: str, default_port: int) -> tuple[str, int]:
    if ":" not in s:
        return s or "127.0.0.1", default_port
    host, _, port = s.rpartition(":")
    return host or "127.0.0.1", int(port)


def load_objects(path: str) -> list[dict]:
    import yaml

    text = Path(path).read_text() if path != "-" else sys.stdin.read()
    docs = [d for d in yaml.safe_load_all(text) if d]
    out = []
    for d in docs:
        if d.get("kind", "").endswith("List") and "items" in d:
            out.extend(d["items"])
        else:
            out.append(d)
    return out


# ---------------------------------------------------------------- commands
def cmd_apiserver(args) -> int:
    from . import Store
    from .control.apiserver import ApiServer
    from .control.snapshot import restore, snapshot_to_file

    store = Store()
    store.set_event_ttl_us(int(args.event_ttl * 1e6))
    if args.load and os.path.exists(args.load):
        n = restore(store, json.loads(Path(args.load).read_text()))
        log.info("restored %d objects from %s", n, args.load)
    host, port = _hostport(args.bind_address, args.port)
    srv = ApiServer(store, host, port, token=args.token, tls_cert=args.tls_cert_file,
                    tls_key=args.tls_private_key_file, client_ca=args.client_ca_file,
                    native_http=False if args.python_http else None).start()
    print(json.dumps({"apiserver": srv.url}), flush=True)
    stop = threading.Event()
    if args.save and args.save_period > 0:
        def saver():
            while not stop.wait(args.save_period):
                snapshot_to_file(store, args.save)
        threading.Thread(target=saver, daemon=True).start()
    _wait_forever(stop)
    if args.save:
        snapshot_to_file(store, args.save)
    srv.stop()
    return 0


def _watcher_addresses(cfg) -> set[str]:
    out = set()
    for p in cfg.profiles:
        for name in ("TargetLoadPacking", "LoadVariationRiskBalancing"):
            addr = (p.plugin_config.get(name) or {}).get("watcherAddress")
            if addr:
                out.add(addr)
    return out


def _library_watchers(cfg, remote, store_client) -> list:
    """load-watcher library mode for Trimaran plugins without `watcherAddress`
    (targetloadpacking.go:125-138 starts watcher.NewWatcher over the
    configured metricProvider). Prometheus/SignalFx are started as given;
    KubernetesMetricsServer only if the cluster serves metrics.k8s.io (an
    in-process cluster relies on the node agents' own documents instead)."""
    from .gpu.providers import K8S_CLIENT_NAME, KubernetesMetricsServerProvider, Watcher, new_provider

    seen, out = set(), []
    for p in cfg.profiles:
        for name in ("TargetLoadPacking", "LoadVariationRiskBalancing"):
            a = p.plugin_config.get(name)
            if a is None or name not in p.plugins.get("score", []) or a.get("watcherAddress"):
                continue
            mp = a.get("metricProvider") or {}
            key = (mp.get("type"), mp.get("address"))
            if key in seen:
                continue
            seen.add(key)
            if (mp.get("type") or K8S_CLIENT_NAME) == K8S_CLIENT_NAME:
                if not hasattr(remote, "request") or not KubernetesMetricsServerProvider(remote).health():
                    continue
            try:
                prov = new_provider(mp, remote)
            except ValueError as e:
                log.error("%s metricProvider: %s", name, e)
                continue
            out.append(Watcher(prov).publish_to(store_client, f"load-watcher-{prov.name.lower()}"))
    return out


def _on_sigusr2(sched) -> None:
    """kube-scheduler's cache debugger signal: SIGUSR2 logs the cache
    comparison and the cache dump (one JSON line each) to stderr."""
    def handler(signum, frame):  # noqa: ARG001
        print(json.dumps({"cache_compare": sched.check_cache()}), file=sys.stderr, flush=True)
        print(json.dumps({"cache_dump": sched.dump_cache()}), file=sys.stderr, flush=True)
    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGUSR2, handler)


def cmd_scheduler(args) -> int:
    from .config import load_config
    from .control.client import LocalClient
    from .control.httpserve import ServiceHTTP
    from .control.leaderelection import LeaderElector
    from .control.remote import RemoteScheduler
    from .gpu.telemetry import WatcherFetcher

    from .utils.cpuaffinity import apply as pin_cpus

    cfg = load_config(args.config)
    remote = _client(args)
    pin_cpus(getattr(args, "cpu_affinity", "none"))  # before the scheduler's threads start
    options = {}
    if args.trace:
        options["trace"] = True
    rs = RemoteScheduler(remote, cfg, **options)
    fetchers = [WatcherFetcher(a, LocalClient(rs.store), name=f"load-watcher-{i}")
                for i, a in enumerate(sorted(_watcher_addresses(cfg)))]
    fetchers += _library_watchers(cfg, remote, LocalClient(rs.store))
    host, port = _hostport(args.metrics_bind_address, 10259)
    http = ServiceHTTP(host, port)
    http.add_metrics(rs.scheduler.metrics_text)
    http.add_route("GET", "/debug/trace", lambda q, b: (200, "application/json", rs.scheduler.trace_json()))
    http.add_route("POST", "/debug/explain", lambda q, b: (200, "application/json", rs.scheduler.explain(b)))
    http.add_route("GET", "/debug/stats", lambda q, b: (200, "application/json", {
        "stats": rs.scheduler.stats(), "queue": rs.scheduler.queue_counts(), "mirror_applied": rs.mirror.applied}))
    http.add_route("GET", "/debug/cache/compare", lambda q, b: (200, "application/json", rs.scheduler.check_cache()))
    http.add_route("GET", "/debug/cache/dump", lambda q, b: (200, "application/json", rs.scheduler.dump_cache()))
    _on_sigusr2(rs.scheduler)
    started = threading.Event()
    stall_s = float(getattr(args, "healthz_stall_seconds", 30.0))

    def loop_check() -> tuple[bool, str]:
        # The scheduling loop ticks at least every 100 ms, idle or not: a
        # cycle stuck in a plugin (or a dead loop thread) stops the ticks.
        if not started.is_set():
            return True, "not started"
        age = rs.scheduler.loop_age_seconds()
        return (age < stall_s, f"scheduling loop made no progress for {age:.1f}s")

    http.add_health_check("scheduling-loop", loop_check)
    http.add_health_check("informer-sync", lambda: (started.is_set(), "informers not synced yet"), ready_only=True)
    http.start()
    print(json.dumps({"scheduler": [p.scheduler_name for p in cfg.profiles], "metrics": http.url}), flush=True)
    stop = threading.Event()

    def lead():
        for f in fetchers:
            f.start()
        rs.start()
        started.set()

    if args.leader_elect or cfg.leader_elect:
        identity = f"{socket.gethostname()}_{os.getpid()}"
        le = LeaderElector(remote, args.lock_name or cfg.profiles[0].scheduler_name, args.lock_namespace, identity,
                           on_started_leading=lead, on_stopped_leading=stop.set)
        http.add_health_check("leaderElection", le.healthz)
        threading.Thread(target=le.run, daemon=True).start()
        _wait_forever(stop)
        le.stop()
    else:
        lead()
        _wait_forever(stop)
    for f in fetchers:
        f.stop()
    rs.stop()
    http.stop()
    return 0


def cmd_controller(args) -> int:
    from .control.controllers import ControllerManager
    from .control.leaderelection import LeaderElector

    client = _client(args)
    stop = threading.Event()
    provisioners = set(args.provisioners.split(",")) if args.provisioners else None
    mgr = ControllerManager(client, workers=args.workers, pv_controller=args.pv_controller, provisioners=provisioners)
    if args.enableLeaderElection:
        identity = f"{socket.gethostname()}_{os.getpid()}"
        le = LeaderElector(client, "sched-plugins-controller", "kube-system", identity,
                           on_started_leading=mgr.run, on_stopped_leading=stop.set)
        threading.Thread(target=le.run, daemon=True).start()
        _wait_forever(stop)
        le.stop()
        # The reference exits when the lease is lost (server.go:107-117).
    else:
        mgr.run()
        _wait_forever(stop)
    mgr.stop()
    return 0


def cmd_manager(args) -> int:
    """controller-runtime style manager (the `/manager` binary of the
    reference's config/manager/manager.yaml): PodGroup + ElasticQuota
    reconcilers, /healthz and /readyz on --health-probe-bind-address,
    controller-runtime metrics on --metrics-bind-address."""
    from .control.httpserve import ServiceHTTP
    from .control.runtime import ElasticQuotaReconciler, Manager, PodGroupReconciler

    client = _client(args)
    probe = ServiceHTTP(*_hostport(args.health_probe_bind_address, 8081))
    metrics = ServiceHTTP(*_hostport(args.metrics_bind_address, 8080))
    mgr = Manager(client, leader_election=args.leader_elect, leader_election_id=args.leader_election_id,
                  leader_election_namespace=args.leader_election_namespace,
                  identity=f"{socket.gethostname()}_{os.getpid()}", probe_http=probe, metrics_http=metrics)
    mgr.add(PodGroupReconciler(client)).add(ElasticQuotaReconciler(client))
    probe.start()
    metrics.start()
    mgr.start()
    print(json.dumps({"manager": [c.name for c in mgr.controllers], "probes": probe.url, "metrics": metrics.url}),
          flush=True)
    stop = threading.Event()
    threading.Thread(target=lambda: (mgr.wait_stopped(), stop.set()), daemon=True).start()
    _wait_forever(stop)
    mgr.stop()
    probe.stop()
    metrics.stop()
    return 0


def cmd_node_agent(args) -> int:
    from .control.node_agent import NodeAgent, hip_bandwidth_fn, hip_health_fn
    from .gpu.discovery import discover_host, fake_host

    client = _client(args)
    if args.fake_gpus:
        host_fn = lambda: fake_host(args.fake_gpus, args.fake_partition)  # noqa: E731
    else:
        host_fn = lambda: discover_host(args.sysfs_root)  # noqa: E731
    agent = NodeAgent(client, args.node_name or socket.gethostname(), host_fn=host_fn, root=args.sysfs_root,
                      heartbeat=args.heartbeat, telemetry_period=args.telemetry_period,
                      publish_metrics=not args.no_telemetry, reserved_cpu=args.reserved_cpu,
                      reserved_memory_gib=args.reserved_memory_gib,
                      health_fn=hip_health_fn() if args.health_probe else None,
                      bandwidth_fn=hip_bandwidth_fn() if args.bandwidth_probe else None,
                      kubelet_managed=args.kubelet_managed).start()
    if args.device_plugin:
        from .control.device_plugin import start_plugins

        agent.device_plugins = start_plugins(agent.host, client, agent.name, socket_dir=args.device_plugin_dir)
        for dp in agent.device_plugins:
            dp.set_unhealthy(agent.unhealthy)
    print(json.dumps({"node": agent.name, "gpus": len(agent.host.gpus)}), flush=True)
    stop = threading.Event()
    _wait_forever(stop)
    agent.stop()
    return 0


def cmd_load_watcher(args) -> int:
    from .control.httpserve import ServiceHTTP
    from .gpu.telemetry import LoadWatcherService

    host, port = _hostport(args.bind_address, args.port)
    http = ServiceHTTP(host, port)
    watcher = None
    if args.provider:
        # Standalone load-watcher over an external metrics source
        # (load-watcher's own binary: watcher.NewWatcher(client).StartWatching()).
        from .gpu.providers import Watcher, new_provider

        mp = {"type": args.provider, "address": args.provider_address, "token": args.provider_token,
              "insecureSkipVerify": args.insecure_skip_verify}
        client = _client(args) if args.provider == "KubernetesMetricsServer" else None
        watcher = Watcher(new_provider(mp, client), period=args.period).serve(http).start()
    else:
        LoadWatcherService(_client(args), http)
    http.start()
    print(json.dumps({"load-watcher": http.url + "/watcher"}), flush=True)
    stop = threading.Event()
    _wait_forever(stop)
    if watcher:
        watcher.stop()
    http.stop()
    return 0


def cmd_explain(args) -> int:
    from .config import load_config
    from .control.remote import RemoteScheduler

    rs = RemoteScheduler(_client(args), load_config(args.config))
    rs.mirror.start()
    rs.mirror.wait_for_sync(30)
    rs.scheduler.sync_informers(2000)
    pods = load_objects(args.pod)
    for p in pods:
        print(json.dumps(rs.scheduler.explain(p), indent=1 if args.pretty else None))
    rs.mirror.stop()
    rs.scheduler.stop()
    return 0


def cmd_apply(args) -> int:
    from .control.client import is_already_exists
    from .control.resources import resource

    client = _client(args)
    for path in args.files:
        for obj in load_objects(path):
            kind = resource(obj.get("kind", "")).kind_plural
            md = obj.setdefault("metadata", {})
            if args.namespace and resource(kind).namespaced:
                md.setdefault("namespace", args.namespace)
            try:
                client.create(kind, obj)
                print(f"{kind}/{md.get('name')} created")
            except Exception as e:  # noqa: BLE001
                if not is_already_exists(e):
                    raise
                cur = client.get(kind, md.get("namespace", ""), md["name"])
                md["resourceVersion"] = cur["metadata"]["resourceVersion"]
                client.update(kind, obj)
                print(f"{kind}/{md.get('name')} configured")
    return 0


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="xsched", description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    ap.add_argument("-v", "--v", type=int, default=2, dest="verbosity", help="log verbosity (klog-style)")
    ap.add_argument("--logging-format", default="json", choices=["json", "text"],
                    help="log line format of both the Python and the native logger")
    sub = ap.add_subparsers(dest="cmd", required=True)

    def conn(p, reference_flags=False):
        p.add_argument("--master", help="API server URL")
        p.add_argument("--kubeconfig", help="kubeconfig path (server + token of the current context)")
        p.add_argument("--token", help="bearer token")
        p.add_argument("--incluster", action="store_true", help="use the in-cluster service account")
        p.add_argument("--insecure-skip-tls-verify", action="store_true",
                       help="do not verify the API server certificate (with --master)")
        if reference_flags:
            p.add_argument("--masterUrl", help="alias of --master (reference controller flag)")
            p.add_argument("--kubeConfig", help="alias of --kubeconfig (reference controller flag)")
            p.add_argument("--qps", type=float, default=5.0, help="accepted for compatibility")
            p.add_argument("--burst", type=int, default=10, help="accepted for compatibility")

    p = sub.add_parser("apiserver", help="HTTP API server over the native store")
    p.add_argument("--bind-address", default="127.0.0.1")
    p.add_argument("--port", type=int, default=6443)
    p.add_argument("--token")
    p.add_argument("--tls-cert-file", help="serve HTTPS with this certificate (PEM)")
    p.add_argument("--tls-private-key-file", help="key of --tls-cert-file (PEM)")
    p.add_argument("--client-ca-file", help="require client certificates signed by this CA (mutual TLS)")
    p.add_argument("--load", help="restore objects from a JSON snapshot at start")
    p.add_argument("--save", help="write a JSON snapshot on exit (and every --save-period s)")
    p.add_argument("--save-period", type=float, default=0.0)
    p.add_argument("--python-http", action="store_true",
                   help="serve with the Python http.server front end instead of the native one")
    p.add_argument("--event-ttl", type=float, default=3600.0,
                   help="seconds an Event is kept (kube-apiserver --event-ttl)")
    p.set_defaults(fn=cmd_apiserver)

    p = sub.add_parser("scheduler", help="the scheduler service")
    conn(p)
    p.add_argument("--config", help="KubeSchedulerConfiguration YAML (v1beta2/v1beta3)")
    p.add_argument("--metrics-bind-address", default="127.0.0.1:10259")
    p.add_argument("--leader-elect", action="store_true")
    p.add_argument("--lock-name")
    p.add_argument("--lock-namespace", default="kube-system")
    p.add_argument("--healthz-stall-seconds", type=float, default=30.0,
                   help="/healthz fails when the scheduling loop has not ticked for this long")
    p.add_argument("--trace", action="store_true", help="record per-cycle phase traces (/debug/trace)")
    p.add_argument("--cpu-affinity", default="none",
                   help="pin the scheduler's threads: none | l3 | l3xK | CPU list (utils/cpuaffinity.py)")
    p.set_defaults(fn=cmd_scheduler)

    p = sub.add_parser("controller", help="PodGroup + ElasticQuota controllers")
    conn(p, reference_flags=True)
    p.add_argument("--workers", type=int, default=1)
    p.add_argument("--enableLeaderElection", action="store_true")
    p.add_argument("--pv-controller", action="store_true",
                   help="also bind PVs/PVCs and provision claims (clusters without kube-controller-manager)")
    p.add_argument("--provisioners", default="",
                   help="comma-separated StorageClass provisioners to provision for (default: all but "
                        "kubernetes.io/no-provisioner)")
    p.set_defaults(fn=cmd_controller)

    p = sub.add_parser("node-agent", help="MI355X node agent")
    conn(p)
    p.add_argument("--node-name")
    p.add_argument("--sysfs-root", default="/")
    p.add_argument("--fake-gpus", type=int, default=0, help="advertise a synthetic node with N GPUs")
    p.add_argument("--fake-partition", default="SPX")
    p.add_argument("--heartbeat", type=float, default=10.0)
    p.add_argument("--telemetry-period", type=float, default=60.0)
    p.add_argument("--no-telemetry", action="store_true")
    p.add_argument("--health-probe", action="store_true", help="run the HIP health probe on each GPU")
    p.add_argument("--bandwidth-probe", action="store_true",
                   help="measure HBM bandwidth per compute-partition size on each GPU and publish it "
                        "(amd.com/gpu-hbm-bandwidth)")
    p.add_argument("--reserved-cpu", type=int, default=0)
    p.add_argument("--reserved-memory-gib", type=int, default=0)
    p.add_argument("--device-plugin", action="store_true",
                   help="serve the kubelet device-plugin API for amd.com/gpu, gpu-xcd and gpu-memory")
    p.add_argument("--device-plugin-dir", default="/var/lib/kubelet/device-plugins/")
    p.add_argument("--kubelet-managed", action="store_true",
                   help="leave amd.com/* capacity to kubelet (device plugins) instead of writing node status")
    p.set_defaults(fn=cmd_node_agent)

    p = sub.add_parser("manager", help="controller-runtime style PodGroup/ElasticQuota reconcilers (kustomize deploy)")
    conn(p)
    p.add_argument("--leader-elect", action="store_true")
    p.add_argument("--leader-election-id", default="sched-plugins-manager")
    p.add_argument("--leader-election-namespace", default="kube-system")
    p.add_argument("--health-probe-bind-address", default=":8081")
    p.add_argument("--metrics-bind-address", default="127.0.0.1:8080")
    p.set_defaults(fn=cmd_manager)

    p = sub.add_parser("load-watcher", help="serve GET /watcher")
    conn(p)
    p.add_argument("--bind-address", default="127.0.0.1")
    p.add_argument("--port", type=int, default=2020)
    p.add_argument("--provider", choices=["KubernetesMetricsServer", "Prometheus", "SignalFx"],
                   help="library-mode watcher over this metrics source (default: serve the node agents' documents)")
    p.add_argument("--provider-address", default="")
    p.add_argument("--provider-token", default="")
    p.add_argument("--insecure-skip-verify", action="store_true")
    p.add_argument("--period", type=float, default=60.0, help="fetch period in seconds (load-watcher: 1 minute)")
    p.set_defaults(fn=cmd_load_watcher)

    p = sub.add_parser("explain", help="dry-run pods against the cluster")
    conn(p)
    p.add_argument("--config")
    p.add_argument("--pod", required=True, help="pod YAML/JSON file ('-' = stdin)")
    p.add_argument("--pretty", action="store_true")
    p.set_defaults(fn=cmd_explain)

    p = sub.add_parser("apply", help="create or replace objects from files")
    conn(p)
    p.add_argument("-f", "--filename", dest="files", action="append", required=True)
    p.add_argument("-n", "--namespace")
    p.set_defaults(fn=cmd_apply)
    return ap


def main(argv: list[str] | None = None) -> int:
    from .utils.cpuaffinity import adopt_child_cpus

    adopt_child_cpus()  # started by a pinned benchmark shard: stay off its CPUs
    args = build_parser().parse_args(argv)
    _setup_logging(args.verbosity, args.logging_format)
    return int(args.fn(args) or 0)


if __name__ == "__main__":
    sys.exit(main())
