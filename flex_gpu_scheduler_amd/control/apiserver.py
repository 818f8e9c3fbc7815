"""HTTP API server over the native ObjectStore: the envtest analog.

The reference's integration tier runs a real kube-apiserver + etcd through
controller-runtime envtest (test/integration/main_test.go:31-49) and talks to
it through client-go. We serve the same REST surface over the in-process C++
store so the scheduler, controllers, node agent and `kubectl`-style clients
can run as separate processes:

  GET    <collection>[?labelSelector=&fieldSelector=&watch=true&resourceVersion=N
                      &timeoutSeconds=&allowWatchBookmarks=true]
  POST   <collection>                       create (namespace from the path)
  GET    <collection>/<name>
  PUT    <collection>/<name>[/status]       update (resourceVersion precondition)
  PATCH  <collection>/<name>[/status]       merge / strategic-merge / json-patch
  DELETE <collection>/<name>                DeleteOptions{gracePeriodSeconds,
                                            preconditions.uid}
  POST   /api/v1/namespaces/<ns>/pods/<name>/binding   v1.Binding; copies
                                            Binding.metadata.annotations onto the
                                            pod (the behaviour FlexGPU's Bind
                                            relies on, pkg/flexgpu/flex_gpu.go:230-242)
  GET    /healthz /readyz /livez /version /api /apis

Watch streams are chunked JSON lines `{"type":..., "object":...}` exactly like
kube-apiserver; an expired resourceVersion yields an ERROR event carrying a 410
Status. `resourceVersion` unset/"0" starts with synthetic ADDED events for the
current state (list-then-watch without a gap: the watch is opened first and
events already covered by the list are dropped by resourceVersion).

Strategic-merge patches are applied as JSON merge patches (lists replace);
every writer in this framework sends merge patches.
"""
from __future__ import annotations

import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any
from urllib.parse import parse_qs, urlsplit

from .. import _lifecycle
from .._native import native
from .resources import RESOURCES, Resource, parse_path, with_type_meta
from .selectors import combine, field_matcher, label_matcher

VERSION_INFO = {"major": "1", "minor": "23", "gitVersion": "v1.23.3-xsched", "platform": "linux/amd64"}


def status_obj(code: int, reason: str, message: str) -> dict:
    return {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure" if code >= 400 else "Success",
            "message": message, "reason": reason, "code": code}


class ApiError(Exception):
    def __init__(self, code: int, reason: str, message: str):
        super().__init__(message)
        self.code, self.reason, self.message = code, reason, message


def apply_json_patch(doc: Any, ops: list) -> Any:
    """RFC 6902 JSON patch (add/remove/replace/move/copy/test)."""
    import copy

    def split(ptr: str) -> list[str]:
        if ptr == "":
            return []
        if not ptr.startswith("/"):
            raise ApiError(422, "Invalid", f"bad JSON pointer {ptr!r}")
        return [p.replace("~1", "/").replace("~0", "~") for p in ptr[1:].split("/")]

    def parent(d, parts):
        for p in parts[:-1]:
            d = d[int(p)] if isinstance(d, list) else d[p]
        return d

    doc = copy.deepcopy(doc)
    for op in ops:
        kind, parts = op.get("op"), split(op.get("path", ""))
        try:
            if kind == "test":
                cur = doc
                for p in parts:
                    cur = cur[int(p)] if isinstance(cur, list) else cur[p]
                if cur != op.get("value"):
                    raise ApiError(422, "Invalid", f"test failed at {op.get('path')}")
                continue
            if kind in ("move", "copy"):
                src = split(op["from"])
                sp = parent(doc, src)
                val = sp[int(src[-1])] if isinstance(sp, list) else sp[src[-1]]
                if kind == "move":
                    if isinstance(sp, list):
                        sp.pop(int(src[-1]))
                    else:
                        del sp[src[-1]]
                kind, op = "add", {"value": copy.deepcopy(val)}
            if not parts:
                doc = op.get("value")
                continue
            par, last = parent(doc, parts), parts[-1]
            if kind == "add":
                if isinstance(par, list):
                    par.insert(len(par) if last == "-" else int(last), op["value"])
                else:
                    par[last] = op["value"]
            elif kind == "remove":
                if isinstance(par, list):
                    par.pop(int(last))
                else:
                    del par[last]
            elif kind == "replace":
                if isinstance(par, list):
                    par[int(last)] = op["value"]
                else:
                    if last not in par:
                        raise KeyError(last)
                    par[last] = op["value"]
            else:
                raise ApiError(422, "Invalid", f"unknown json-patch op {kind!r}")
        except (KeyError, IndexError, ValueError, TypeError) as e:
            raise ApiError(422, "Invalid", f"json patch {op}: {e}") from None
    return doc


class ApiServer:
    """Owns a native Store and serves it over HTTP on background threads.

    By default the HTTP(S) layer is native (csrc/apiserver/apiserver.cc: same
    REST surface, TLS and mutual TLS through OpenSSL, no interpreter on the
    request path); `native_http=False` selects this module's http.server
    handler."""

    def __init__(self, store=None, host: str = "127.0.0.1", port: int = 0, *, token: str | None = None,
                 bookmark_interval: float = 10.0, tls_cert: str | None = None, tls_key: str | None = None,
                 client_ca: str | None = None, native_http: bool | None = None):
        self.store = store if store is not None else native().Store()
        self.token = token
        self.bookmark_interval = bookmark_interval
        self._stopping = threading.Event()
        self._active: set = set()
        self._active_lock = threading.Lock()
        self._py_requests = 0
        self.tls = bool(tls_cert)
        if native_http is None:
            native_http = True
        self._native = None
        self.httpd = None
        self._thread: threading.Thread | None = None
        if native_http:
            self._native = native().NativeApiServer(self.store, host, port, token or "",
                                                    int(bookmark_interval * 1000), tls_cert or "",
                                                    tls_key or "", client_ca or "")
            self._host = host
        else:
            handler = type("Handler", (_Handler,), {"api": self})
            self.httpd = _Server((host, port), handler)
            self.httpd.daemon_threads = True
            if tls_cert:
                # kube-apiserver's --tls-cert-file/--tls-private-key-file, and
                # --client-ca-file for client-certificate (mutual TLS) auth.
                import ssl

                ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
                ctx.load_cert_chain(tls_cert, tls_key or tls_cert)
                if client_ca:
                    ctx.verify_mode = ssl.CERT_REQUIRED
                    ctx.load_verify_locations(client_ca)
                # Handshakes run in each connection's handler thread, not in the
                # accept loop (a slow client must not stall every other one).
                self.httpd.socket = ctx.wrap_socket(self.httpd.socket, server_side=True, do_handshake_on_connect=False)
        _lifecycle.register(self)

    @property
    def native_http(self) -> bool:
        return self._native is not None

    @property
    def requests(self) -> int:
        return self._native.requests() if self._native is not None else self._py_requests

    @property
    def address(self) -> tuple[str, int]:
        if self._native is not None:
            return self._host, self._native.port
        return self.httpd.server_address[:2]

    @property
    def url(self) -> str:
        h, p = self.address
        return f"{'https' if self.tls else 'http'}://{h}:{p}"

    def start(self) -> "ApiServer":
        if self._native is not None:
            self._native.start()
            return self
        self._thread = threading.Thread(target=self.httpd.serve_forever, kwargs={"poll_interval": 0.05},
                                        name="apiserver", daemon=True)
        self._thread.start()
        return self

    def _wake_watches(self) -> None:
        self._stopping.set()
        with self._active_lock:
            active = list(self._active)
        for w in active:
            self.store.unwatch(w)

    def shutdown_for_exit(self) -> None:
        if self._native is not None:
            self._native.stop()
            return
        self._wake_watches()

    def stop(self) -> None:
        if self._native is not None:
            self._native.stop()
            return
        self._wake_watches()
        self.httpd.shutdown()
        self.httpd.server_close()
        if self._thread:
            self._thread.join(timeout=5)
        deadline = time.monotonic() + 5
        while time.monotonic() < deadline:
            with self._active_lock:
                if not self._active:
                    break
            time.sleep(0.01)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


class _Server(ThreadingHTTPServer):
    # A scheduler opens one watch per kind at once (and binder pools several
    # keep-alive connections): socketserver's default backlog of 5 drops the
    # surplus SYNs, which clients only retry after a second.
    request_queue_size = 128


def _store_error(e: Exception) -> ApiError:
    return ApiError(getattr(e, "code", 500), getattr(e, "reason", "InternalError"), str(e))


class _Handler(BaseHTTPRequestHandler):
    api: ApiServer
    protocol_version = "HTTP/1.1"
    server_version = "xsched-apiserver/1"
    # TCP_NODELAY: keep-alive request/response pairs must not wait on the
    # peer's delayed ACK (Nagle holds a small second segment ~40 ms).
    disable_nagle_algorithm = True

    def log_message(self, fmt, *args):  # quiet
        pass

    # ---------------------------------------------------------------- plumbing
    def _send(self, code: int, body: Any, content_type: str = "application/json") -> None:
        data = body if isinstance(body, (bytes, bytearray)) else (
            body.encode() if isinstance(body, str) else json.dumps(body, separators=(",", ":")).encode())
        self.send_response(code)
        self.send_header("Content-Type", content_type)
        self.send_header("Content-Length", str(len(data)))
        # Headers and body in one write (one segment for small responses).
        self._headers_buffer.append(b"\r\n")
        self._headers_buffer.append(data)
        self.flush_headers()

    def _error(self, e: ApiError) -> None:
        self._send(e.code, status_obj(e.code, e.reason, e.message))

    def _body(self) -> Any:
        n = int(self.headers.get("Content-Length") or 0)
        raw = self.rfile.read(n) if n else b""
        if not raw:
            return None
        try:
            return json.loads(raw)
        except json.JSONDecodeError as e:
            raise ApiError(400, "BadRequest", f"invalid JSON body: {e}") from None

    def _auth(self) -> None:
        if self.api.token and self.headers.get("Authorization") != f"Bearer {self.api.token}":
            raise ApiError(401, "Unauthorized", "Unauthorized")

    def _dispatch(self, verb: str) -> None:
        self.api._py_requests += 1
        url = urlsplit(self.path)
        q = {k: v[-1] for k, v in parse_qs(url.query).items()}
        try:
            if url.path in ("/healthz", "/readyz", "/livez"):
                return self._send(200, b"ok", "text/plain")
            if url.path == "/version":
                return self._send(200, VERSION_INFO)
            self._auth()
            if url.path == "/api":
                return self._send(200, {"kind": "APIVersions", "versions": ["v1"]})
            if url.path == "/apis":
                groups = sorted({r.group for r in RESOURCES.values() if r.group})
                return self._send(200, {"kind": "APIGroupList", "apiVersion": "v1", "groups": [
                    {"name": g, "versions": [{"groupVersion": f"{g}/{v}", "version": v} for v in
                                             sorted({r.version for r in RESOURCES.values() if r.group == g})]}
                    for g in groups]})
            parsed = parse_path(url.path)
            if parsed is None:
                raise ApiError(404, "NotFound", f"the server could not find the requested resource ({url.path})")
            res, ns, name, sub = parsed
            getattr(self, f"_{verb}")(res, ns, name, sub, q)
        except ApiError as e:
            self._error(e)
        except (BrokenPipeError, ConnectionResetError):
            pass
        except Exception as e:  # noqa: BLE001 - StoreError and friends
            if type(e).__name__ == "StoreError":
                self._error(_store_error(e))
            else:
                self._error(ApiError(500, "InternalError", f"{type(e).__name__}: {e}"))

    def do_GET(self):
        self._dispatch("get")

    def do_POST(self):
        self._dispatch("post")

    def do_PUT(self):
        self._dispatch("put")

    def do_PATCH(self):
        self._dispatch("patch")

    def do_DELETE(self):
        self._dispatch("delete")

    # ------------------------------------------------------------------ verbs
    def _get(self, res: Resource, ns: str, name: str, sub: str, q: dict) -> None:
        store = self.api.store
        if name:
            obj = store.get_json(res.kind_plural, ns, name)
            if obj is None:
                raise ApiError(404, "NotFound", f'{res.kind_plural} "{name}" not found')
            return self._send(200, obj)
        match = combine(label_matcher(q.get("labelSelector")), field_matcher(q.get("fieldSelector")))
        if q.get("watch") in ("true", "1"):
            return self._watch(res, ns, q, match)
        items_json, rv = store.list_json(res.kind_plural, ns)
        head = f'{{"kind":"{res.kind}List","apiVersion":"{res.api_version}","metadata":{{"resourceVersion":"{rv}"}},"items":'
        if match is None:
            return self._send(200, head + items_json + "}")
        items = [o for o in json.loads(items_json) if match(o)]
        return self._send(200, head + json.dumps(items, separators=(",", ":")) + "}")

    def _post(self, res: Resource, ns: str, name: str, sub: str, q: dict) -> None:
        body = self._body()
        if not isinstance(body, dict):
            raise ApiError(400, "BadRequest", "request body must be a JSON object")
        store = self.api.store
        if res.kind_plural == "pods" and name and sub == "binding":
            target = (body.get("target") or {}).get("name")
            if not target:
                raise ApiError(422, "Invalid", "Binding.target.name: Required value")
            md = body.get("metadata") or {}
            store.bind(ns or "default", name, md.get("uid", ""), target, md.get("annotations") or {})
            return self._send(201, status_obj(201, "", "") | {"status": "Success"})
        if name:
            raise ApiError(405, "MethodNotAllowed", "POST to a named resource")
        if res.namespaced:
            body.setdefault("metadata", {})
            if ns:
                if body["metadata"].get("namespace", ns) != ns:
                    raise ApiError(400, "BadRequest", "the namespace of the object does not match the request")
                body["metadata"]["namespace"] = ns
        body = with_type_meta(res.kind_plural, body)
        return self._send(201, store.create(res.kind_plural, body))

    def _put(self, res: Resource, ns: str, name: str, sub: str, q: dict) -> None:
        body = self._body()
        if not isinstance(body, dict):
            raise ApiError(400, "BadRequest", "request body must be a JSON object")
        md = body.setdefault("metadata", {})
        if md.get("name", name) != name:
            raise ApiError(400, "BadRequest", "the name of the object does not match the request")
        md["name"] = name
        if res.namespaced:
            md["namespace"] = ns or md.get("namespace") or "default"
        body = with_type_meta(res.kind_plural, body)
        return self._send(200, self.api.store.update(res.kind_plural, body, True))

    def _patch(self, res: Resource, ns: str, name: str, sub: str, q: dict) -> None:
        ctype = (self.headers.get("Content-Type") or "application/merge-patch+json").split(";")[0].strip()
        body = self._body()
        store = self.api.store
        if ctype == "application/json-patch+json":
            cur = store.get(res.kind_plural, ns, name)
            if cur is None:
                raise ApiError(404, "NotFound", f'{res.kind_plural} "{name}" not found')
            new = apply_json_patch(cur, body or [])
            return self._send(200, store.update(res.kind_plural, new, True))
        if ctype not in ("application/merge-patch+json", "application/strategic-merge-patch+json",
                         "application/apply-patch+yaml", "application/json"):
            raise ApiError(415, "UnsupportedMediaType", f"unsupported patch type {ctype}")
        if not isinstance(body, dict):
            raise ApiError(400, "BadRequest", "merge patch body must be an object")
        return self._send(200, store.patch(res.kind_plural, ns, name, body))

    def _delete(self, res: Resource, ns: str, name: str, sub: str, q: dict) -> None:
        store = self.api.store
        if not name:
            n = store.delete_all(res.kind_plural, ns)
            return self._send(200, status_obj(200, "", f"deleted {n}") | {"status": "Success"})
        opts = self._body() or {}
        grace = opts.get("gracePeriodSeconds", q.get("gracePeriodSeconds", 0))
        uid = ((opts.get("preconditions") or {}).get("uid")) or ""
        old = store.delete(res.kind_plural, ns, name, int(grace or 0), uid)
        return self._send(200, old)

    # ------------------------------------------------------------------ watch
    def _write_chunk(self, data: bytes) -> None:
        self.wfile.write(b"%x\r\n%s\r\n" % (len(data), data))
        self.wfile.flush()

    def _watch(self, res: Resource, ns: str, q: dict, match) -> None:
        store = self.api.store
        rv_param = q.get("resourceVersion", "")
        timeout = float(q.get("timeoutSeconds") or 0) or None
        bookmarks = q.get("allowWatchBookmarks") in ("true", "1")
        since = int(rv_param) if rv_param not in ("", "0") else 0
        expired = None
        try:
            w = store.watch([res.kind_plural], ns, since)
        except Exception as e:  # noqa: BLE001
            if getattr(e, "code", 0) != 410:
                raise
            expired, w = e, None
        if w is not None:
            with self.api._active_lock:
                self.api._active.add(w)
            if self.api._stopping.is_set():
                store.unwatch(w)
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Transfer-Encoding", "chunked")
        self.end_headers()
        try:
            if expired is not None:
                self._write_chunk(json.dumps({"type": "ERROR", "object": status_obj(410, "Expired", str(expired))})
                                  .encode() + b"\n")
                self._write_chunk(b"")
                return
            floor = 0
            if since == 0:
                items_json, floor = store.list_json(res.kind_plural, ns)
                for o in json.loads(items_json):
                    if match is None or match(o):
                        self._write_chunk(json.dumps({"type": "ADDED", "object": o}, separators=(",", ":"))
                                          .encode() + b"\n")
            deadline = time.monotonic() + timeout if timeout else None
            last_rv, last_beat = floor, time.monotonic()
            while not self.api._stopping.is_set():
                if deadline and time.monotonic() >= deadline:
                    break
                evs = w.next_json(500, 1024)
                if not evs:
                    if bookmarks and time.monotonic() - last_beat >= self.api.bookmark_interval:
                        bm = {"type": "BOOKMARK", "object": {"kind": res.kind, "apiVersion": res.api_version,
                                                             "metadata": {"resourceVersion": str(last_rv)}}}
                        self._write_chunk(json.dumps(bm).encode() + b"\n")
                        last_beat = time.monotonic()
                    continue
                out = []
                for etype, _kind, obj_json, rv in evs:
                    if rv <= floor:
                        continue
                    last_rv = rv
                    if match is not None or etype == "DELETED":
                        obj = json.loads(obj_json)
                        if match is not None and not match(obj):
                            continue
                        if etype == "DELETED":
                            obj.setdefault("metadata", {})["resourceVersion"] = str(rv)
                        obj_json = json.dumps(obj, separators=(",", ":"))
                    out.append(f'{{"type":"{etype}","object":{obj_json}}}\n')
                if out:
                    self._write_chunk("".join(out).encode())
                last_beat = time.monotonic()
            self._write_chunk(b"")
        finally:
            if w is not None:
                store.unwatch(w)
                with self.api._active_lock:
                    self.api._active.discard(w)
