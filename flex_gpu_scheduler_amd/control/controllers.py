"""PodGroup and ElasticQuota controllers (the reference's cmd/controller).

PodGroupController — pkg/controller/podgroup.go:52-303. Reconciles
`PodGroup.status` from the group's pods:
  ""          -> Pending
  Pending     -> PreScheduling once #labelled pods >= minMember (+ occupiedBy)
  otherwise   recount running/succeeded/failed, then
              no pods                                   -> Pending
              Scheduling and scheduled >= min           -> Scheduled
              Scheduled and succeeded+running >= min    -> Running
              failed>0 and failed+running+succeeded>=min-> Failed
              succeeded >= min                          -> Finished
Groups in Finished/Failed, or Scheduled==min with nothing running whose
scheduling started >48 h after creation, are not re-enqueued (:112-127).
Deliberate fixes: pods are listed in the group's own
namespace (the reference lists cluster-wide, :209-210), and occupiedBy is
filled from the first pod's owner references even when empty (the reference
returns early on an empty occupiedBy, :296-298).

ElasticQuotaController — pkg/controller/elasticquota.go:55-345. `status.used`
= zero for every key of min ∪ max, plus Σ requests of Running pods in the
namespace (requests = Σ containers, max'ed with each init container, plus
overhead — the reference drops overhead by discarding `quota.Add`'s result,
:323-325, fixed here). Patches only on change and records a `Synced` event.

Both run `workers` threads off a rate-limited work queue fed by informers
(:93-109 / :111-130), and PATCH with JSON merge patches (:275-289).
"""
from __future__ import annotations

import logging
import threading
import time

from .._native import native
from ..models.objects import POD_GROUP_LABEL
from .client import Client, is_not_found
from .informer import InformerFactory, WorkQueue, meta_key, split_key

log = logging.getLogger(__name__)

PG_PENDING, PG_PRESCHEDULING, PG_SCHEDULING = "Pending", "PreScheduling", "Scheduling"
PG_SCHEDULED, PG_RUNNING, PG_FINISHED, PG_FAILED = "Scheduled", "Running", "Finished", "Failed"
PG_UNKNOWN = "Unknown"
PG_PHASES = (PG_PENDING, PG_PRESCHEDULING, PG_SCHEDULING, PG_SCHEDULED, PG_RUNNING, PG_FINISHED, PG_FAILED, PG_UNKNOWN)
_TWO_DAYS_US = 48 * 3600 * 1_000_000


def _ts_us(s: str | None) -> int:
    if not s:
        return 0
    try:
        return native().parse_rfc3339(s)
    except Exception:  # noqa: BLE001
        return 0


def merge_patch_between(old: dict, new: dict) -> dict:
    """Two-way JSON merge patch (util.CreateMergePatch, pkg/util/podgroup.go)."""
    patch: dict = {}
    for k, v in new.items():
        ov = old.get(k, _MISSING)
        if isinstance(v, dict) and isinstance(ov, dict):
            sub = merge_patch_between(ov, v)
            if sub:
                patch[k] = sub
        elif ov is _MISSING or ov != v:
            patch[k] = v
    for k in old:
        if k not in new:
            patch[k] = None
    return patch


_MISSING = object()


class _Controller:
    name = "controller"

    def __init__(self, client: Client, workers: int = 1, factory: InformerFactory | None = None):
        self.client = client
        self.workers = workers
        # A factory passed in is shared and stopped by its owner; one made
        # here stops with the controller.
        self._own_factory = factory is None
        self.factory = factory or InformerFactory(client)
        self.queue = WorkQueue(self.name)
        self._threads: list[threading.Thread] = []
        self.syncs = 0
        self.errors = 0

    def sync(self, key: str) -> None:
        raise NotImplementedError

    def _worker(self) -> None:
        while True:
            key = self.queue.get()
            if key is None:
                return
            try:
                self.sync(key)
                self.syncs += 1
                self.queue.forget(key)
            except Exception as e:  # noqa: BLE001 - requeue with backoff (AddRateLimited)
                self.errors += 1
                log.warning("%s: sync %s failed: %s", self.name, key, e)
                self.queue.add_rate_limited(key)
            finally:
                self.queue.done(key)

    def run(self, start_informers: bool = True, sync_timeout: float = 30.0) -> "_Controller":
        if start_informers:
            self.factory.start()
        if not self.factory.wait_for_sync(sync_timeout):
            raise RuntimeError(f"{self.name}: informer caches did not sync")
        for i in range(self.workers):
            t = threading.Thread(target=self._worker, name=f"{self.name}-{i}", daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def stop(self) -> None:
        self.queue.shutdown()
        for t in self._threads:
            t.join(timeout=5)
        if self._own_factory:
            self.factory.stop()

    def wait_idle(self, timeout: float = 10.0) -> bool:
        """Test helper: queue empty and nothing in flight."""
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            with self.queue._cv:
                idle = not self.queue._queue and not self.queue._processing and not self.queue._delayed
            if idle:
                return True
            time.sleep(0.01)
        return False


class PodGroupController(_Controller):
    name = "PodGroup"

    def __init__(self, client: Client, workers: int = 1, factory: InformerFactory | None = None):
        super().__init__(client, workers, factory)
        self.pg_informer = self.factory.informer("podgroups")
        self.pod_informer = self.factory.informer("pods", label_selector=POD_GROUP_LABEL)
        self.pg_informer.add_event_handler(self.pg_added, lambda o, n: self.pg_added(n))
        self.pod_informer.add_event_handler(self.pod_added, lambda o, n: self.pod_added(n))

    def pg_added(self, pg: dict) -> None:
        st, spec = pg.get("status") or {}, pg.get("spec") or {}
        if st.get("phase") in (PG_FINISHED, PG_FAILED):
            return
        created = _ts_us((pg.get("metadata") or {}).get("creationTimestamp"))
        started = _ts_us(st.get("scheduleStartTime"))
        if (int(st.get("scheduled") or 0) == int(spec.get("minMember") or 0) and int(st.get("running") or 0) == 0
                and started and created and started - created > _TWO_DAYS_US):
            return
        self.queue.add(meta_key(pg))

    def pod_added(self, pod: dict) -> None:
        md = pod.get("metadata") or {}
        pg_name = (md.get("labels") or {}).get(POD_GROUP_LABEL)
        if not pg_name:
            return
        pg = self.pg_informer.get(md.get("namespace") or "default", pg_name)
        if pg is not None:
            self.pg_added(pg)

    def group_pods(self, ns: str, name: str) -> list[dict]:
        return self.pod_informer.list(
            ns, lambda p: ((p.get("metadata") or {}).get("labels") or {}).get(POD_GROUP_LABEL) == name)

    @staticmethod
    def fill_occupied(status: dict, pod: dict) -> None:
        md = pod.get("metadata") or {}
        refs = sorted(f"{md.get('namespace', 'default')}/{r.get('name', '')}" for r in md.get("ownerReferences") or [])
        if refs:
            status["occupiedBy"] = ",".join(refs)

    @staticmethod
    def next_status(pg: dict, pods: list[dict]) -> dict:
        status = dict(pg.get("status") or {})
        min_member = int((pg.get("spec") or {}).get("minMember") or 0)
        phase = status.get("phase") or ""
        if phase == "":
            status["phase"] = PG_PENDING
        elif phase == PG_PENDING:
            if len(pods) >= min_member:
                status["phase"] = PG_PRESCHEDULING
                if pods:
                    PodGroupController.fill_occupied(status, pods[0])
        else:
            counts = {"Running": 0, "Succeeded": 0, "Failed": 0}
            for p in pods:
                ph = (p.get("status") or {}).get("phase")
                if ph in counts:
                    counts[ph] += 1
            status["running"], status["succeeded"], status["failed"] = (counts["Running"], counts["Succeeded"],
                                                                        counts["Failed"])
            scheduled = int(status.get("scheduled") or 0)
            if not pods:
                status["phase"] = PG_PENDING
            else:
                if scheduled >= min_member and status.get("phase") == PG_SCHEDULING:
                    status["phase"] = PG_SCHEDULED
                if counts["Succeeded"] + counts["Running"] >= min_member and status.get("phase") == PG_SCHEDULED:
                    status["phase"] = PG_RUNNING
                if counts["Failed"] and counts["Failed"] + counts["Running"] + counts["Succeeded"] >= min_member:
                    status["phase"] = PG_FAILED
                if counts["Succeeded"] >= min_member:
                    status["phase"] = PG_FINISHED
        return status

    def sync(self, key: str) -> None:
        ns, name = split_key(key)
        pg = self.pg_informer.get(ns, name)
        if pg is None:
            return
        status = self.next_status(pg, self.group_pods(ns, name))
        old = pg.get("status") or {}
        if status != old:
            try:
                # resourceVersion precondition: the scheduler's PostBind also
                # writes status.phase; a stale cache copy must not overwrite
                # a newer phase (the reference patches unconditionally,
                # podgroup.go:275-289). On 409 the key is requeued.
                rv = (pg.get("metadata") or {}).get("resourceVersion")
                patch = {"status": merge_patch_between(old, status)}
                if rv:
                    patch["metadata"] = {"resourceVersion": rv}
                self.client.patch("podgroups", ns, name, patch)
            except Exception as e:  # noqa: BLE001
                if is_not_found(e):
                    return
                raise


def pod_effective_request(pod: dict) -> dict:
    """Σ container requests, max'ed with each init container, plus overhead
    (computePodResourceRequest, pkg/controller/elasticquota.go:315-331)."""
    return native().pod_summary(pod)["request"]


class ElasticQuotaController(_Controller):
    name = "ElasticQuota"

    def __init__(self, client: Client, workers: int = 1, factory: InformerFactory | None = None,
                 record_events: bool = True):
        super().__init__(client, workers, factory)
        self.record_events = record_events
        self.eq_informer = self.factory.informer("elasticquotas")
        self.pod_informer = self.factory.informer("pods")
        self.eq_informer.add_event_handler(self.eq_added, lambda o, n: self.eq_added(n), self.eq_added)
        self.pod_informer.add_event_handler(self.pod_added, self.pod_updated, self.pod_added)

    def eq_added(self, eq: dict) -> None:
        self.queue.add_rate_limited(meta_key(eq))

    def pod_added(self, pod: dict) -> None:
        ns = (pod.get("metadata") or {}).get("namespace") or "default"
        eqs = self.eq_informer.list(ns)
        if eqs:
            self.eq_added(eqs[0])

    def pod_updated(self, old: dict, new: dict) -> None:
        if (old.get("metadata") or {}).get("resourceVersion") == (new.get("metadata") or {}).get("resourceVersion"):
            return
        self.pod_added(new)

    @staticmethod
    def zero_used(eq: dict) -> dict:
        spec = eq.get("spec") or {}
        return {k: "0" for k in list((spec.get("min") or {})) + list((spec.get("max") or {}))}

    def compute_used(self, ns: str, eq: dict) -> dict:
        n = native()
        used = self.zero_used(eq)
        for p in self.pod_informer.list(ns):
            if (p.get("status") or {}).get("phase") == "Running":
                used = n.resource_list_op(used, pod_effective_request(p), "add")
        return used

    def sync(self, key: str) -> None:
        ns, name = split_key(key)
        eq = self.eq_informer.get(ns, name)
        if eq is None:
            return
        used = self.compute_used(ns, eq)
        old_used = (eq.get("status") or {}).get("used") or {}
        n = native()
        if set(used) == set(old_used) and all(n.quantity_cmp(used[k], str(old_used[k])) == 0 for k in used):
            return
        try:
            self.client.patch("elasticquotas", ns, name, {"status": {"used": used | {
                k: None for k in old_used if k not in used}}})
        except Exception as e:  # noqa: BLE001
            if is_not_found(e):
                return
            raise
        if self.record_events:
            self.client.record_event("ElasticQuota", ns, name, "Normal", "Synced",
                                     f"Elastic Quota {key} synced successfully")


class ControllerManager:
    """Runs both controllers over one informer factory (cmd/controller/app/
    server.go:55-122), optionally only while holding the leader lease."""

    def __init__(self, client: Client, workers: int = 1, record_events: bool = True,
                 pv_controller: bool = False, provisioners: set[str] | None = None):
        self.client = client
        self.factory = InformerFactory(client)
        self.podgroup = PodGroupController(client, workers, self.factory)
        self.elasticquota = ElasticQuotaController(client, workers, self.factory, record_events)
        self.controllers: list[_Controller] = [self.podgroup, self.elasticquota]
        if pv_controller:
            # Only for clusters without kube-controller-manager (this
            # framework's own API server): it completes the volume binding
            # the scheduler's VolumeBinding plugin starts.
            from .pv_controller import PersistentVolumeController

            self.controllers.append(PersistentVolumeController(client, workers, self.factory, provisioners))

    def run(self) -> "ControllerManager":
        self.factory.start()
        for c in self.controllers:
            c.run(start_informers=False)
        return self

    def stop(self) -> None:
        for c in self.controllers:
            c.stop()
        self.factory.stop()

    def wait_idle(self, timeout: float = 10.0) -> bool:
        return all(c.wait_idle(timeout) for c in self.controllers)
