"""Small routed HTTP endpoint for the services: /metrics, /healthz and
service-specific routes (the scheduler's /debug/trace and /debug/explain, the
load watcher's /watcher).

kube-scheduler serves Prometheus metrics and health on its secure port
(vendor/k8s.io/kubernetes/cmd/kube-scheduler/app/server.go:244-255); the
load-watcher serves `GET /watcher` on :2020
(vendor/github.com/paypal/load-watcher/pkg/watcher/watcher.go).
"""
from __future__ import annotations

import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Callable
from urllib.parse import parse_qs, urlsplit

Route = Callable[[dict, Any], tuple[int, str, Any]]  # (query, body) -> (code, content-type, body)


class ServiceHTTP:
    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self.routes: dict[tuple[str, str], Route] = {}
        self.metrics_providers: list[Callable[[], str]] = []
        # name -> () -> (ok, detail); /healthz (and /livez) fail when any
        # check fails, /readyz also when a readiness check fails.
        self.health_checks: dict[str, Callable[[], tuple[bool, str]]] = {}
        self.ready_checks: dict[str, Callable[[], tuple[bool, str]]] = {}
        self.add_route("GET", "/healthz", lambda q, b: self._health(q, self.health_checks))
        self.add_route("GET", "/livez", lambda q, b: self._health(q, self.health_checks))
        self.add_route("GET", "/readyz", lambda q, b: self._health(q, {**self.health_checks, **self.ready_checks}))
        self.add_route("GET", "/metrics", self._metrics)
        handler = type("Handler", (_Handler,), {"svc": self})
        self.httpd = ThreadingHTTPServer((host, port), handler)
        self.httpd.daemon_threads = True
        self._thread: threading.Thread | None = None

    def add_health_check(self, name: str, fn: Callable[[], tuple[bool, str]], ready_only: bool = False) -> None:
        (self.ready_checks if ready_only else self.health_checks)[name] = fn

    @staticmethod
    def _health(q: dict, checks: dict) -> tuple[int, str, str]:
        """The apiserver healthz format: "ok", or one "[+]name ok" /
        "[-]name failed: reason" line per check and a 500 when one fails
        (with ?verbose the lines are shown on success too)."""
        lines, ok = [], True
        for name, fn in checks.items():
            try:
                good, detail = fn()
            except Exception as e:  # noqa: BLE001
                good, detail = False, f"check raised {type(e).__name__}: {e}"
            ok &= good
            lines.append(f"[+]{name} ok" if good else f"[-]{name} failed: {detail}")
        if ok and "verbose" not in q:
            return 200, "text/plain", "ok"
        lines.append("healthz check passed" if ok else "healthz check failed")
        return (200 if ok else 500), "text/plain", "\n".join(lines) + "\n"

    def add_route(self, method: str, path: str, fn: Route) -> None:
        self.routes[(method, path)] = fn

    def add_metrics(self, provider: Callable[[], str]) -> None:
        self.metrics_providers.append(provider)

    def _metrics(self, q, b):
        parts = []
        for p in self.metrics_providers:
            try:
                parts.append(p())
            except Exception as e:  # noqa: BLE001
                parts.append(f"# provider error: {e}\n")
        return 200, "text/plain; version=0.0.4", "".join(x if x.endswith("\n") else x + "\n" for x in parts if x)

    @property
    def url(self) -> str:
        h, p = self.httpd.server_address[:2]
        return f"http://{h}:{p}"

    def start(self) -> "ServiceHTTP":
        self._thread = threading.Thread(target=self.httpd.serve_forever, kwargs={"poll_interval": 0.05},
                                        name="service-http", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()


class _Handler(BaseHTTPRequestHandler):
    svc: ServiceHTTP
    protocol_version = "HTTP/1.1"
    disable_nagle_algorithm = True  # keep-alive scrapes: no delayed-ACK stalls

    def log_message(self, fmt, *args):
        pass

    def _do(self, method: str) -> None:
        url = urlsplit(self.path)
        fn = self.svc.routes.get((method, url.path))
        if fn is None:
            code, ctype, body = 404, "text/plain", "not found"
        else:
            n = int(self.headers.get("Content-Length") or 0)
            raw = self.rfile.read(n) if n else b""
            try:
                payload = json.loads(raw) if raw else None
                code, ctype, body = fn({k: v[-1] for k, v in parse_qs(url.query).items()}, payload)
            except Exception as e:  # noqa: BLE001
                code, ctype, body = 500, "text/plain", f"{type(e).__name__}: {e}"
        if not isinstance(body, (bytes, str)):
            body = json.dumps(body)
        data = body.encode() if isinstance(body, str) else body
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def do_GET(self):
        self._do("GET")

    def do_POST(self):
        self._do("POST")


def counter_text(name: str, help_: str, value: float, labels: dict | None = None, kind: str = "counter") -> str:
    lab = ""
    if labels:
        lab = "{" + ",".join(f'{k}="{v}"' for k, v in labels.items()) + "}"
    return f"# HELP {name} {help_}\n# TYPE {name} {kind}\n{name}{lab} {value}\n"
