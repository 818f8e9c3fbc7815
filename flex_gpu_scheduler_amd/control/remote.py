"""Run the native scheduler against a remote API server.

The C++ scheduler consumes a *local* ObjectStore (its informers are native
watchers, so no per-pod Python on the hot path). In service mode a
`StoreMirror` reflects the remote API's objects into that local store, and a
`RemoteApiClient` sends the scheduler's writes — pod bindings (v1.Binding with
annotations, pkg/flexgpu/flex_gpu.go:230-242), status/PodGroup patches,
preemption deletes, events — to the remote API. The binding becomes visible
to the scheduler cache when the mirror reflects the bound pod back, which is
the same assume → informer-confirm flow as against kube-apiserver
(SURVEY.md §3.2).
"""
from __future__ import annotations

import logging
import threading

from .._native import native
from .client import Client, is_already_exists, is_not_found
from .informer import Informer

log = logging.getLogger(__name__)

# Kinds the scheduler and its plugins watch (scheduler informers + plugin
# watched_kinds()).
SCHEDULER_KINDS = ("nodes", "pods", "podgroups", "elasticquotas", "noderesourcetopologies", "priorityclasses",
                   "poddisruptionbudgets", "namespaces", "loadwatchermetrics", "persistentvolumes",
                   "persistentvolumeclaims", "storageclasses", "csinodes")


class StoreMirror:
    def __init__(self, remote: Client, local_store, kinds=SCHEDULER_KINDS):
        self.remote, self.local = remote, local_store
        self.informers = [Informer(remote, k) for k in kinds]
        for inf in self.informers:
            kind = inf.kind
            inf.add_event_handler(lambda o, k=kind: self._upsert(k, o), lambda _o, n, k=kind: self._upsert(k, n),
                                  lambda o, k=kind: self._delete(k, o))
        self.applied = 0

    def _upsert(self, kind: str, obj: dict) -> None:
        md = obj.get("metadata") or {}
        try:
            self.local.create(kind, obj)
        except Exception as e:  # noqa: BLE001
            if not is_already_exists(e) and getattr(e, "code", 0) != 409:
                raise
            self.local.update(kind, obj, False)
        self.applied += 1
        log.debug("mirror %s %s/%s", kind, md.get("namespace", ""), md.get("name"))

    def _delete(self, kind: str, obj: dict) -> None:
        md = obj.get("metadata") or {}
        try:
            self.local.delete(kind, md.get("namespace") or "", md.get("name") or "")
        except Exception as e:  # noqa: BLE001
            if not is_not_found(e):
                raise
        self.applied += 1

    def start(self) -> "StoreMirror":
        for inf in self.informers:
            inf.start()
        return self

    def wait_for_sync(self, timeout: float = 30.0) -> bool:
        return all(inf.wait_for_sync(timeout) for inf in self.informers)

    def stop(self) -> None:
        for inf in self.informers:
            inf.stop()


def remote_api_client(remote: Client):
    """A native ApiClient whose writes go to `remote` (called from the C++
    binding executor threads; pybind acquires the GIL per call)."""
    base = native().ApiClient

    class RemoteApiClient(base):
        def __init__(self):
            base.__init__(self)
            self.remote = remote
            self.lock = threading.Lock()
            self.binds = 0

        def bind(self, ns, name, uid, node, annotations):
            self.remote.bind(ns, name, uid, node, annotations or {})
            self.binds += 1

        def delete_pod(self, ns, name, uid):
            try:
                self.remote.delete("pods", ns, name, 0, uid)
            except Exception as e:  # noqa: BLE001
                if not is_not_found(e):
                    raise

        def patch(self, kind, ns, name, patch):
            self.remote.patch(kind, ns, name, patch)

        def record_event(self, kind, ns, name, type_, reason, message):
            self.remote.record_event(kind, ns, name, type_, reason, message)

    return RemoteApiClient()


def rest_endpoint(remote: Client, qps: float = 0.0, burst: int = 0):
    """The native REST endpoint (host, port, bearer token, TLS settings) of a
    RestClient, or None for clients that are not plain REST endpoints."""
    from .client import RestClient

    if not isinstance(remote, RestClient):
        return None
    t = remote.tls
    return native().RestEndpoint(
        remote.host, remote.port, remote.token or "", remote.https, ca_file=t.ca_file or "",
        ca_pem=t.ca_data.decode() if t.ca_data else "", cert_file=t.cert_file or "", key_file=t.key_file or "",
        cert_pem=t.cert_data.decode() if t.cert_data else "", key_pem=t.key_data.decode() if t.key_data else "",
        insecure=t.insecure, timeout_ms=int(remote.timeout * 1000), qps=float(qps), burst=int(burst))


class NativeMirror:
    """StoreMirror's interface over the native LIST/WATCH mirror (rest/kube.h):
    one native thread per kind, no Python per event."""

    def __init__(self, endpoint, local_store, kinds=SCHEDULER_KINDS):
        self._m = native().RemoteMirror(endpoint, local_store, list(kinds))

    @property
    def applied(self) -> int:
        return self._m.applied

    @property
    def relists(self) -> int:
        return self._m.relists

    def start(self) -> "NativeMirror":
        self._m.start()
        return self

    def wait_for_sync(self, timeout: float = 30.0) -> bool:
        ok = self._m.wait_synced(int(timeout * 1000))
        if not ok and self._m.last_error():
            log.warning("native mirror not synced: %s", self._m.last_error())
        return ok

    def stop(self) -> None:
        self._m.stop()


class RemoteScheduler:
    """Native scheduler + mirror + remote writer, as one service.

    Against a REST endpoint (RestClient: our API server or kube-apiserver)
    the mirror and the writes are native (`native_io`, the default): bindings,
    patches, deletes and events go out from the binder threads over pooled
    keep-alive connections, and every watched kind is mirrored by a native
    thread. Other clients (e.g. LocalClient) use the Python mirror/writer."""

    def __init__(self, remote: Client, config=None, *, native_io: bool = True, **options):
        from ..scheduler import new_scheduler

        from ..config import SchedulerConfiguration, load_config

        cfg = config if isinstance(config, SchedulerConfiguration) else load_config(config)
        self.store = native().Store()
        ep = rest_endpoint(remote) if native_io else None
        if ep is not None:
            self.mirror = NativeMirror(ep, self.store)
            # Writes are throttled per clientConnection; LIST/WATCH are not
            # (a watch is one request).
            self.client = native().RestApiClient(rest_endpoint(remote, cfg.client_qps, cfg.client_burst))
        else:
            self.mirror = StoreMirror(remote, self.store)
            self.client = remote_api_client(remote)
        self.native_io = ep is not None
        self.scheduler = new_scheduler(self.store, cfg, client=self.client, **options)

    def start(self, sync_timeout: float = 30.0) -> "RemoteScheduler":
        self.mirror.start()
        if not self.mirror.wait_for_sync(sync_timeout):
            raise RuntimeError("remote API mirror did not sync")
        self.scheduler.start()
        return self

    def stop(self) -> None:
        self.mirror.stop()
        self.scheduler.stop()
