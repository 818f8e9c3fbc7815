"""controller-runtime style Manager + Reconcilers (the reference's
pkg/controllers/* and config/ kustomize scaffold).

The reference carries kubebuilder-generated `PodGroupReconciler` and
`ElasticQuotaReconciler` (pkg/controllers/coscheduling/podgroup_controller.go:
30-62, pkg/controllers/CapacityScheduling/elasticquota_controller.go:30-60)
whose `Reconcile` is an empty TODO, plus a `config/manager/manager.yaml` that
runs a `/manager --leader-elect` binary with /healthz and /readyz on :8081 —
a binary the repository never builds.

Here that scaffold is made real:
  * `Request`/`Result` and a `Reconciler` protocol (`reconcile(req)`,
    `setup_with_manager(mgr)`) with controller-runtime's semantics: an
    exception requeues with rate-limited backoff, `Result.requeue` requeues
    rate-limited, `Result.requeue_after` requeues after a delay, success
    forgets the key's backoff;
  * `Manager`: one shared informer cache, controllers added through a
    `Builder` (`for_kind(...)`, `watches(kind, mapper)`), optional Lease
    leader election, /healthz + /readyz (readyz flips once caches sync and,
    under election, leadership is held) and controller-runtime's reconcile
    metrics (`controller_runtime_reconcile_total{controller,result}`,
    `controller_runtime_reconcile_errors_total`, `workqueue_depth`) on one
    ServiceHTTP;
  * `PodGroupReconciler` / `ElasticQuotaReconciler` reconcile with the same
    status logic as the cmd/controller controllers (controllers.py), so the
    kustomize deployment (deploy/config) and the Helm controller Deployment
    converge a cluster to the same PodGroup / ElasticQuota status.
"""
from __future__ import annotations

import logging
import threading
from dataclasses import dataclass
from typing import Callable, Protocol

from ..models.objects import POD_GROUP_LABEL
from .client import Client, is_not_found
from .controllers import (_TWO_DAYS_US, ElasticQuotaController, PodGroupController, _ts_us, merge_patch_between,
                          pod_effective_request)
from .informer import Informer, InformerFactory, WorkQueue, meta_key, split_key

log = logging.getLogger(__name__)


@dataclass(frozen=True)
class Request:
    namespace: str
    name: str

    @property
    def key(self) -> str:
        return f"{self.namespace}/{self.name}" if self.namespace else self.name

    @staticmethod
    def from_key(key: str) -> "Request":
        ns, name = split_key(key)
        return Request(ns, name)


@dataclass(frozen=True)
class Result:
    requeue: bool = False
    requeue_after: float = 0.0


class Reconciler(Protocol):
    def reconcile(self, req: Request) -> Result: ...

    def setup_with_manager(self, mgr: "Manager") -> None: ...


Mapper = Callable[[dict], list[Request]]


class Controller:
    """One reconciler behind a rate-limited work queue."""

    def __init__(self, name: str, reconciler: Reconciler, workers: int = 1):
        self.name, self.reconciler, self.workers = name, reconciler, workers
        self.queue = WorkQueue(name)
        self.counts = {"success": 0, "error": 0, "requeue": 0, "requeue_after": 0}
        self._threads: list[threading.Thread] = []

    def enqueue(self, req: Request) -> None:
        self.queue.add(req.key)

    def _worker(self) -> None:
        while True:
            key = self.queue.get()
            if key is None:
                return
            try:
                res = self.reconciler.reconcile(Request.from_key(key)) or Result()
            except Exception as e:  # noqa: BLE001 - reconcile errors requeue with backoff
                log.warning("%s: reconcile %s failed: %s", self.name, key, e)
                self.counts["error"] += 1
                self.queue.add_rate_limited(key)
            else:
                if res.requeue_after > 0:
                    self.counts["requeue_after"] += 1
                    self.queue.forget(key)
                    self.queue.add_after(key, res.requeue_after)
                elif res.requeue:
                    self.counts["requeue"] += 1
                    self.queue.add_rate_limited(key)
                else:
                    self.counts["success"] += 1
                    self.queue.forget(key)
            finally:
                self.queue.done(key)

    def start(self) -> None:
        for i in range(self.workers):
            t = threading.Thread(target=self._worker, name=f"{self.name}-{i}", daemon=True)
            t.start()
            self._threads.append(t)

    def stop(self) -> None:
        self.queue.shutdown()
        for t in self._threads:
            t.join(timeout=5)

    def idle(self) -> bool:
        q = self.queue
        with q._cv:
            return not q._queue and not q._processing and not q._delayed


class Builder:
    """ctrl.NewControllerManagedBy(mgr).For(...).Watches(...).Complete(r)."""

    def __init__(self, mgr: "Manager"):
        self.mgr = mgr
        self._for: str | None = None
        self._watches: list[tuple[str, Mapper, str | None]] = []
        self._name: str | None = None
        self._workers = 1

    def for_kind(self, kind: str) -> "Builder":
        self._for = kind
        return self

    def watches(self, kind: str, mapper: Mapper, label_selector: str | None = None) -> "Builder":
        self._watches.append((kind, mapper, label_selector))
        return self

    def named(self, name: str) -> "Builder":
        self._name = name
        return self

    def with_workers(self, n: int) -> "Builder":
        self._workers = max(1, n)
        return self

    def complete(self, reconciler: Reconciler) -> Controller:
        if not self._for:
            raise ValueError("Builder.complete: for_kind() is required")
        ctl = Controller(self._name or self._for, reconciler, self._workers)
        primary = self.mgr.informer(self._for)

        def own(obj: dict) -> None:
            ctl.enqueue(Request.from_key(meta_key(obj)))

        primary.add_event_handler(own, lambda o, n: own(n), own)
        for kind, mapper, sel in self._watches:
            inf = self.mgr.informer(kind, label_selector=sel)

            def mapped(obj: dict, mapper=mapper) -> None:
                for r in mapper(obj):
                    ctl.enqueue(r)

            inf.add_event_handler(mapped, lambda o, n, mapped=mapped: mapped(n), mapped)
        self.mgr.controllers.append(ctl)
        return ctl


class Manager:
    def __init__(self, client: Client, *, leader_election: bool = False, leader_election_id: str = "sched-plugins-manager",
                 leader_election_namespace: str = "kube-system", identity: str = "manager",
                 probe_http=None, metrics_http=None):
        self.client = client
        self.cache = InformerFactory(client)
        self.controllers: list[Controller] = []
        self.leader_election = leader_election
        self.le_id, self.le_ns, self.identity = leader_election_id, leader_election_namespace, identity
        self._synced = threading.Event()
        self._leading = threading.Event()
        self._stopped = threading.Event()
        self._elector = None
        if probe_http is not None:
            probe_http.add_route("GET", "/healthz", lambda q, b: (200, "text/plain", "ok"))
            probe_http.add_route("GET", "/readyz", lambda q, b: (200, "text/plain", "ok") if self.ready()
                                 else (503, "text/plain", "not ready"))
        if metrics_http is not None:
            metrics_http.add_metrics(self.metrics_text)

    def informer(self, kind: str, label_selector: str | None = None) -> Informer:
        return self.cache.informer(kind, label_selector=label_selector)

    def add(self, reconciler: Reconciler) -> "Manager":
        reconciler.setup_with_manager(self)
        return self

    def ready(self) -> bool:
        return self._synced.is_set() and (not self.leader_election or self._leading.is_set())

    def _run_controllers(self) -> None:
        self._leading.set()
        for c in self.controllers:
            c.start()

    def start(self, sync_timeout: float = 30.0) -> "Manager":
        self.cache.start()
        if not self.cache.wait_for_sync(sync_timeout):
            raise RuntimeError("manager: informer caches did not sync")
        self._synced.set()
        if self.leader_election:
            from .leaderelection import LeaderElector

            self._elector = LeaderElector(self.client, self.le_id, self.le_ns, self.identity,
                                          on_started_leading=self._run_controllers,
                                          on_stopped_leading=self._stopped.set)
            threading.Thread(target=self._elector.run, name="manager-leader-election", daemon=True).start()
        else:
            self._run_controllers()
        return self

    def wait_stopped(self, timeout: float | None = None) -> bool:
        """Set when leadership is lost (the manager must exit)."""
        return self._stopped.wait(timeout)

    def stop(self) -> None:
        if self._elector is not None:
            self._elector.stop()
        for c in self.controllers:
            c.stop()
        self.cache.stop()

    def wait_idle(self, timeout: float = 10.0) -> bool:
        import time

        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if all(c.idle() for c in self.controllers):
                return True
            time.sleep(0.01)
        return False

    def metrics_text(self) -> str:
        out = ["# HELP controller_runtime_reconcile_total Total number of reconciliations per controller",
               "# TYPE controller_runtime_reconcile_total counter"]
        for c in self.controllers:
            for res, n in c.counts.items():
                out.append(f'controller_runtime_reconcile_total{{controller="{c.name}",result="{res}"}} {n}')
        out += ["# HELP controller_runtime_reconcile_errors_total Total number of reconciliation errors per controller",
                "# TYPE controller_runtime_reconcile_errors_total counter"]
        out += [f'controller_runtime_reconcile_errors_total{{controller="{c.name}"}} {c.counts["error"]}'
                for c in self.controllers]
        out += ["# HELP workqueue_depth Current depth of workqueue", "# TYPE workqueue_depth gauge"]
        out += [f'workqueue_depth{{name="{c.name}"}} {len(c.queue)}' for c in self.controllers]
        return "\n".join(out) + "\n"


# ------------------------------------------------------------ reconcilers ----
class PodGroupReconciler:
    """Reconciles PodGroup.status from the group's pods (phase machine of
    pkg/controller/podgroup.go:185-273, as in controllers.PodGroupController)."""

    def __init__(self, client: Client):
        self.client = client
        self.pgs: Informer | None = None
        self.pods: Informer | None = None

    def setup_with_manager(self, mgr: Manager) -> None:
        self.pgs = mgr.informer("podgroups")
        self.pods = mgr.informer("pods", label_selector=POD_GROUP_LABEL)

        def pod_to_group(pod: dict) -> list[Request]:
            md = pod.get("metadata") or {}
            pg = (md.get("labels") or {}).get(POD_GROUP_LABEL)
            return [Request(md.get("namespace") or "default", pg)] if pg else []

        Builder(mgr).named("podgroup").for_kind("podgroups").watches(
            "pods", pod_to_group, label_selector=POD_GROUP_LABEL).complete(self)

    def reconcile(self, req: Request) -> Result:
        pg = self.pgs.get(req.namespace, req.name)
        if pg is None:
            return Result()  # deleted: nothing to do
        st, spec = pg.get("status") or {}, pg.get("spec") or {}
        if st.get("phase") in ("Finished", "Failed"):
            return Result()
        # podgroup.go:119-126: a group whose scheduling started >48 h after
        # creation with everything scheduled and nothing running is left alone.
        created = _ts_us((pg.get("metadata") or {}).get("creationTimestamp"))
        started = _ts_us(st.get("scheduleStartTime"))
        if (int(st.get("scheduled") or 0) == int(spec.get("minMember") or 0) and int(st.get("running") or 0) == 0
                and started and created and started - created > _TWO_DAYS_US):
            return Result()
        pods = self.pods.list(req.namespace, lambda p: ((p.get("metadata") or {}).get("labels") or {}).get(
            POD_GROUP_LABEL) == req.name)
        status = PodGroupController.next_status(pg, pods)
        old = pg.get("status") or {}
        if status == old:
            return Result()
        patch = {"status": merge_patch_between(old, status)}
        rv = (pg.get("metadata") or {}).get("resourceVersion")
        if rv:
            patch["metadata"] = {"resourceVersion": rv}
        try:
            self.client.patch("podgroups", req.namespace, req.name, patch)
        except Exception as e:  # noqa: BLE001
            if is_not_found(e):
                return Result()
            raise
        # The patched object comes back through the informer and is reconciled
        # again from there (one phase step per pass, as in the reference).
        return Result()


class ElasticQuotaReconciler:
    """Reconciles ElasticQuota.status.used (pkg/controller/elasticquota.go:
    168-224, as in controllers.ElasticQuotaController)."""

    def __init__(self, client: Client, record_events: bool = True):
        self.client = client
        self.record_events = record_events
        self.eqs: Informer | None = None
        self.pods: Informer | None = None

    def setup_with_manager(self, mgr: Manager) -> None:
        self.eqs = mgr.informer("elasticquotas")
        self.pods = mgr.informer("pods")

        def pod_to_quota(pod: dict) -> list[Request]:
            ns = (pod.get("metadata") or {}).get("namespace") or "default"
            return [Request.from_key(meta_key(eq)) for eq in self.eqs.list(ns)[:1]]

        Builder(mgr).named("elasticquota").for_kind("elasticquotas").watches("pods", pod_to_quota).complete(self)

    def reconcile(self, req: Request) -> Result:
        from .._native import native

        eq = self.eqs.get(req.namespace, req.name)
        if eq is None:
            return Result()
        n = native()
        used = ElasticQuotaController.zero_used(eq)
        for p in self.pods.list(req.namespace):
            if (p.get("status") or {}).get("phase") == "Running":
                used = n.resource_list_op(used, pod_effective_request(p), "add")
        old = (eq.get("status") or {}).get("used") or {}
        if set(used) == set(old) and all(n.quantity_cmp(used[k], str(old[k])) == 0 for k in used):
            return Result()
        try:
            self.client.patch("elasticquotas", req.namespace, req.name,
                              {"status": {"used": used | {k: None for k in old if k not in used}}})
        except Exception as e:  # noqa: BLE001
            if is_not_found(e):
                return Result()
            raise
        if self.record_events:
            self.client.record_event("ElasticQuota", req.namespace, req.name, "Normal", "Synced",
                                     f"Elastic Quota {req.key} synced successfully")
        return Result()
