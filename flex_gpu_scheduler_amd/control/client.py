"""API clients: one interface over the in-process store and the HTTP server.

Plays the role of the reference's generated clientset + kube client
(pkg/generated/clientset/versioned/clientset.go:31-117, typed podgroup.go:40-51:
Create/Update/UpdateStatus/Delete/Get/List/Watch/Patch). Controllers, the node
agent, the telemetry publisher and the scheduler's remote mode are written
against `Client`, so the same code runs in-process (tests, bench) or as
separate processes talking to `ApiServer` over HTTP.
"""
from __future__ import annotations

import base64
import http.client
import json
import os
import queue
import socket
import ssl
import tempfile
import threading
import time
from dataclasses import dataclass
from typing import Any, Iterable
from urllib.parse import urlencode, urlsplit

from .. import _lifecycle
from .resources import RESOURCES, resource, with_type_meta
from .selectors import combine, field_matcher, label_matcher


class ApiException(Exception):
    def __init__(self, code: int, reason: str, message: str):
        super().__init__(f"{code} {reason}: {message}")
        self.code, self.reason, self.message = code, reason, message


def is_not_found(e: BaseException) -> bool:
    return getattr(e, "code", 0) == 404


def is_conflict(e: BaseException) -> bool:
    return getattr(e, "code", 0) == 409


def is_already_exists(e: BaseException) -> bool:
    return getattr(e, "code", 0) == 409 and getattr(e, "reason", "") == "AlreadyExists"


Event = tuple[str, str, Any, int]  # (type, kind, object, resourceVersion)


class WatchStream:
    """Iterator-style watch handle: `next(timeout_ms)` returns a batch."""

    def next(self, timeout_ms: int = 0, max: int = 4096) -> list[Event]:  # noqa: A002
        raise NotImplementedError

    def stop(self) -> None:
        raise NotImplementedError


class Client:
    def get(self, kind: str, ns: str, name: str) -> dict | None: ...
    def list(self, kind: str, ns: str = "", label_selector: str | None = None,
             field_selector: str | None = None) -> tuple[list[dict], int]: ...
    def create(self, kind: str, obj: dict) -> dict: ...
    def update(self, kind: str, obj: dict) -> dict: ...
    def patch(self, kind: str, ns: str, name: str, patch: dict) -> dict: ...
    def delete(self, kind: str, ns: str, name: str, grace_seconds: int = 0, uid: str = "") -> dict: ...
    def bind(self, ns: str, name: str, uid: str, node: str, annotations: dict | None = None) -> None: ...
    def watch(self, kinds: Iterable[str], ns: str = "", since_rv: int = 0) -> WatchStream: ...

    def record_event(self, kind: str, ns: str, name: str, type_: str, reason: str, message: str) -> None:
        """core/v1 Event, like client-go's EventRecorder (best effort)."""
        now = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
        try:
            self.create("events", {"metadata": {"generateName": f"{name}.", "namespace": ns or "default"},
                                   "involvedObject": {"kind": kind, "namespace": ns, "name": name},
                                   "type": type_, "reason": reason, "message": message, "count": 1,
                                   "firstTimestamp": now, "lastTimestamp": now,
                                   "source": {"component": "xsched"}})
        except Exception:  # noqa: BLE001 - events never fail the caller
            pass


# ------------------------------------------------------------------ local ---
class _LocalWatch(WatchStream):
    def __init__(self, store, w):
        self._store, self._w = store, w
        _lifecycle.register(self, _lifecycle.WATCH, "stop")

    def next(self, timeout_ms: int = 0, max: int = 4096) -> list[Event]:  # noqa: A002
        return self._w.next(timeout_ms, max)

    def stop(self) -> None:
        self._store.unwatch(self._w)


class LocalClient(Client):
    """Direct calls into a native `Store` (no serialization)."""

    def __init__(self, store):
        self.store = store

    @staticmethod
    def _wrap(fn, *a):
        try:
            return fn(*a)
        except Exception as e:  # noqa: BLE001
            if type(e).__name__ == "StoreError":
                raise ApiException(e.code, e.reason, str(e)) from None
            raise

    def get(self, kind, ns, name):
        return self.store.get(kind, ns, name)

    def list(self, kind, ns="", label_selector=None, field_selector=None):
        items, rv = self.store.list(kind, ns)
        m = combine(label_matcher(label_selector), field_matcher(field_selector))
        return ([o for o in items if m(o)] if m else items), rv

    def create(self, kind, obj):
        return self._wrap(self.store.create, kind, with_type_meta(kind, obj))

    def update(self, kind, obj):
        return self._wrap(self.store.update, kind, obj, True)

    def patch(self, kind, ns, name, patch):
        return self._wrap(self.store.patch, kind, ns, name, patch)

    def delete(self, kind, ns, name, grace_seconds=0, uid=""):
        return self._wrap(self.store.delete, kind, ns, name, grace_seconds, uid)

    def bind(self, ns, name, uid, node, annotations=None):
        self._wrap(self.store.bind, ns, name, uid, node, annotations or {})

    def watch(self, kinds, ns="", since_rv=0):
        return _LocalWatch(self.store, self._wrap(self.store.watch, list(kinds), ns, since_rv))


# ------------------------------------------------------------------- REST ---
class _RestWatch(WatchStream):
    """One streaming GET per kind; reader threads feed a shared queue and
    resume from the last seen resourceVersion after a server-side timeout or a
    dropped connection. A server ERROR event (e.g. 410 Expired) is surfaced as
    ("ERROR", kind, Status, 0) and ends that kind's stream: the consumer
    (Informer) relists and re-watches.

    `since_rv == 0` follows kube-apiserver semantics: synthetic ADDED events
    for the current state, then live events."""

    def __init__(self, client: "RestClient", kinds: list[str], ns: str, since_rv: int):
        self._c = client
        self._q: queue.Queue = queue.Queue()
        self._stop = threading.Event()
        self._conns: list[http.client.HTTPConnection] = []
        self._lock = threading.Lock()
        self._threads = [threading.Thread(target=self._run, args=(k, ns, since_rv), daemon=True,
                                          name=f"watch-{k}") for k in kinds]
        for t in self._threads:
            t.start()

    def _run(self, kind: str, ns: str, rv: int) -> None:
        res = RESOURCES[kind]
        failures = 0
        while not self._stop.is_set():
            conn = None
            try:
                conn = self._c._new_conn()
                with self._lock:
                    self._conns.append(conn)
                params = {"watch": "true", "allowWatchBookmarks": "true", "timeoutSeconds": "300",
                          "resourceVersion": str(rv)}
                conn.request("GET", f"{res.collection_path(ns)}?{urlencode(params)}", headers=self._c._headers())
                resp = conn.getresponse()
                if resp.status != 200:
                    body = resp.read()
                    raise ApiException(resp.status, "WatchFailed", body.decode(errors="replace")[:200])
                failures = 0
                while not self._stop.is_set():
                    line = resp.readline()
                    if not line:
                        break
                    ev = json.loads(line)
                    etype, obj = ev.get("type"), ev.get("object") or {}
                    if etype == "ERROR":
                        self._q.put(("ERROR", kind, obj, 0))
                        return
                    ev_rv = int((obj.get("metadata") or {}).get("resourceVersion") or 0)
                    if ev_rv:
                        rv = max(rv, ev_rv)
                    if etype == "BOOKMARK":
                        continue
                    self._q.put((etype, kind, obj, ev_rv))
            except (OSError, http.client.HTTPException, ValueError, AttributeError, ApiException) as e:
                # AttributeError: http.client raises it when stop() closes the
                # socket under a blocked readline.
                if self._stop.is_set():
                    break
                failures += 1
                if failures >= 50 or getattr(e, "code", 0) in (401, 403, 404):
                    self._q.put(("ERROR", kind, {"code": getattr(e, "code", 500), "message": str(e)}, 0))
                    return
                time.sleep(min(0.05 * failures, 1.0))
            finally:
                if conn is not None:
                    try:
                        conn.close()
                    except OSError:
                        pass
                    with self._lock:
                        if conn in self._conns:
                            self._conns.remove(conn)

    def next(self, timeout_ms: int = 0, max: int = 4096) -> list[Event]:  # noqa: A002
        out: list[Event] = []
        try:
            out.append(self._q.get(timeout=timeout_ms / 1000) if timeout_ms > 0 else self._q.get_nowait())
        except queue.Empty:
            return out
        while len(out) < max:
            try:
                out.append(self._q.get_nowait())
            except queue.Empty:
                break
        return out

    def stop(self) -> None:
        self._stop.set()
        with self._lock:
            for c in self._conns:
                try:
                    if c.sock is not None:
                        c.sock.shutdown(2)
                except OSError:
                    pass
                c.close()
        for t in self._threads:
            t.join(timeout=2)


@dataclass
class TLSConfig:
    """TLS settings of a kube-apiserver connection (client-go rest.TLSClientConfig):
    the cluster CA (file or PEM data), an optional client certificate/key (file
    or PEM data) and insecure-skip-tls-verify."""
    ca_file: str | None = None
    ca_data: bytes | None = None
    cert_file: str | None = None
    key_file: str | None = None
    cert_data: bytes | None = None
    key_data: bytes | None = None
    insecure: bool = False

    def context(self) -> ssl.SSLContext:
        ctx = ssl.create_default_context(cafile=self.ca_file,
                                         cadata=self.ca_data.decode() if self.ca_data else None)
        if self.insecure:
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        if self.cert_file or self.cert_data:
            if self.cert_data:
                # load_cert_chain takes paths only: stage the PEMs in 0600 files.
                with tempfile.TemporaryDirectory() as d:
                    cf, kf = os.path.join(d, "tls.crt"), os.path.join(d, "tls.key")
                    for path, data in ((cf, self.cert_data), (kf, self.key_data or self.cert_data)):
                        fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o600)
                        with os.fdopen(fd, "wb") as f:
                            f.write(data)
                    ctx.load_cert_chain(cf, kf)
            else:
                ctx.load_cert_chain(self.cert_file, self.key_file)
        return ctx


def kubeconfig_connection(path: str) -> tuple[str, str | None, TLSConfig]:
    """(server URL, bearer token, TLS settings) of the current context of a
    kubeconfig, following clientcmd: relative file paths resolve against the
    kubeconfig's directory, `*-data` fields are base64 PEM, `tokenFile` is read."""
    import yaml

    with open(path) as f:
        kc = yaml.safe_load(f) or {}
    base = os.path.dirname(os.path.abspath(path))
    ctx_name = kc.get("current-context")
    ctxs = {c["name"]: c.get("context") or {} for c in kc.get("contexts") or []}
    ctx = ctxs.get(ctx_name) or (next(iter(ctxs.values())) if ctxs else {})
    clusters = {c["name"]: c.get("cluster") or {} for c in kc.get("clusters") or []}
    users = {u["name"]: u.get("user") or {} for u in kc.get("users") or []}
    cluster = clusters.get(ctx.get("cluster")) or (next(iter(clusters.values())) if clusters else {})
    user = users.get(ctx.get("user")) or (next(iter(users.values())) if users else {})

    def path_of(v):
        return v if not v or os.path.isabs(v) else os.path.join(base, v)

    def data_of(v):
        return base64.b64decode(v) if v else None

    tls = TLSConfig(ca_file=path_of(cluster.get("certificate-authority")),
                    ca_data=data_of(cluster.get("certificate-authority-data")),
                    cert_file=path_of(user.get("client-certificate")), key_file=path_of(user.get("client-key")),
                    cert_data=data_of(user.get("client-certificate-data")),
                    key_data=data_of(user.get("client-key-data")),
                    insecure=bool(cluster.get("insecure-skip-tls-verify", False)))
    token = user.get("token")
    if not token and user.get("tokenFile"):
        with open(path_of(user["tokenFile"])) as f:
            token = f.read().strip()
    return cluster.get("server", "http://127.0.0.1:6443"), token, tls


IN_CLUSTER_SA = "/var/run/secrets/kubernetes.io/serviceaccount"


class RestClient(Client):
    """Kubernetes-REST client over `http.client` (one keep-alive connection
    per thread). Talks to `ApiServer` or any kube-apiserver exposing the same
    paths: bearer-token and/or client-certificate auth, TLS verified against
    the cluster CA (`TLSConfig`)."""

    def __init__(self, base_url: str, token: str | None = None, timeout: float = 30.0, tls: TLSConfig | None = None):
        u = urlsplit(base_url)
        self.host, self.port = u.hostname or "127.0.0.1", u.port or (443 if u.scheme == "https" else 80)
        self.https = u.scheme == "https"
        self.token, self.timeout = token, timeout
        self.tls = tls or TLSConfig()
        self._ssl = self.tls.context() if self.https else None
        self._tls = threading.local()

    def _new_conn(self, timeout: float | None = None) -> http.client.HTTPConnection:
        if self.https:
            conn = http.client.HTTPSConnection(self.host, self.port, timeout=timeout, context=self._ssl)
        else:
            conn = http.client.HTTPConnection(self.host, self.port, timeout=timeout)
        conn.connect()
        # Requests are small writes on a keep-alive connection: without
        # TCP_NODELAY each can wait ~40 ms on the server's delayed ACK.
        conn.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        return conn

    def _headers(self, ctype: str | None = None) -> dict:
        h = {"Accept": "application/json"}
        if ctype:
            h["Content-Type"] = ctype
        if self.token:
            h["Authorization"] = f"Bearer {self.token}"
        return h

    def request(self, method: str, path: str, body: Any = None, ctype: str = "application/json",
                ok=(200, 201)) -> Any:
        data = None if body is None else json.dumps(body, separators=(",", ":")).encode()
        for attempt in (0, 1):
            conn = getattr(self._tls, "conn", None)
            try:
                if conn is None:
                    conn = self._tls.conn = self._new_conn(self.timeout)
                conn.request(method, path, body=data, headers=self._headers(ctype if data is not None else None))
                resp = conn.getresponse()
                raw = resp.read()
                break
            except (ConnectionError, http.client.HTTPException, OSError):
                if conn is not None:
                    conn.close()
                self._tls.conn = None
                if attempt:
                    raise
        try:
            out = json.loads(raw) if raw else None
        except json.JSONDecodeError:
            out = raw.decode(errors="replace")
        if resp.status not in ok:
            if isinstance(out, dict):
                raise ApiException(resp.status, out.get("reason", ""), out.get("message", ""))
            raise ApiException(resp.status, HTTP_REASON.get(resp.status, ""), str(out))
        return out

    def get(self, kind, ns, name):
        try:
            return self.request("GET", resource(kind).object_path(ns, name))
        except ApiException as e:
            if e.code == 404:
                return None
            raise

    def list(self, kind, ns="", label_selector=None, field_selector=None):
        r = resource(kind)
        q = {}
        if label_selector:
            q["labelSelector"] = label_selector
        if field_selector:
            q["fieldSelector"] = field_selector
        path = r.collection_path(ns) + (f"?{urlencode(q)}" if q else "")
        out = self.request("GET", path)
        return out.get("items") or [], int(out["metadata"].get("resourceVersion") or 0)

    def create(self, kind, obj):
        r = resource(kind)
        ns = (obj.get("metadata") or {}).get("namespace") or ("default" if r.namespaced else "")
        return self.request("POST", r.collection_path(ns), with_type_meta(r.kind_plural, obj))

    def update(self, kind, obj):
        r = resource(kind)
        md = obj.get("metadata") or {}
        return self.request("PUT", r.object_path(md.get("namespace") or "default", md["name"]), obj)

    def patch(self, kind, ns, name, patch):
        return self.request("PATCH", resource(kind).object_path(ns, name), patch, "application/merge-patch+json")

    def delete(self, kind, ns, name, grace_seconds=0, uid=""):
        opts: dict = {"kind": "DeleteOptions", "apiVersion": "v1", "gracePeriodSeconds": int(grace_seconds)}
        if uid:
            opts["preconditions"] = {"uid": uid}
        return self.request("DELETE", resource(kind).object_path(ns, name), opts)

    def bind(self, ns, name, uid, node, annotations=None):
        md: dict = {"name": name, "namespace": ns}
        if uid:
            md["uid"] = uid
        if annotations:
            md["annotations"] = dict(annotations)
        self.request("POST", RESOURCES["pods"].object_path(ns, name, "binding"),
                     {"apiVersion": "v1", "kind": "Binding", "metadata": md, "target": {"kind": "Node", "name": node}})

    def watch(self, kinds, ns="", since_rv=0):
        return _RestWatch(self, [resource(k).kind_plural for k in kinds], ns, since_rv)

    def healthy(self) -> bool:
        try:
            conn = self._new_conn(2)
            conn.request("GET", "/healthz")
            return conn.getresponse().status == 200
        except OSError:
            return False


HTTP_REASON = {400: "BadRequest", 401: "Unauthorized", 403: "Forbidden", 404: "NotFound", 405: "MethodNotAllowed",
               409: "Conflict", 410: "Expired", 415: "UnsupportedMediaType", 422: "Invalid", 500: "InternalError"}


def client_for(target) -> Client:
    """A Client from a native Store, an existing Client or an http(s) URL."""
    if isinstance(target, Client):
        return target
    if isinstance(target, str):
        return RestClient(target)
    return LocalClient(target)
