"""Native service mode (csrc/rest/): the REST writer and the LIST/WATCH
mirror RemoteScheduler uses against a REST endpoint. Bindings carry the
FlexGPU annotations, a relist drops objects deleted while not watching, and
TLS (server-verified and mutual) works end to end."""
import json
import shutil
import time

import pytest

from flex_gpu_scheduler_amd import load_config
from flex_gpu_scheduler_amd._native import native
from flex_gpu_scheduler_amd.control import ApiServer, RestClient
from flex_gpu_scheduler_amd.control.client import TLSConfig
from flex_gpu_scheduler_amd.control.remote import RemoteScheduler, rest_endpoint
from flex_gpu_scheduler_amd.models import GPU, INDEX_ANNOTATION, make_pod, make_pod_group, mi355x_node

from helpers import FLEXGPU_PLUGINS, coscheduling_config


def wait_for(fn, timeout=10.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if fn():
            return True
        time.sleep(0.02)
    return bool(fn())


def test_native_io_binds_gang_with_annotations(store):
    srv = ApiServer(store).start()
    try:
        client = RestClient(srv.url)
        client.create("nodes", mi355x_node("n0"))
        rs = RemoteScheduler(RestClient(srv.url), load_config(coscheduling_config(FLEXGPU_PLUGINS))).start()
        try:
            assert rs.native_io
            client.create("podgroups", make_pod_group("g", min_member=4))
            for i in range(4):
                client.create("pods", make_pod(f"w{i}", pod_group="g", limits={GPU: "1"}, requests={GPU: "1"}))
            assert wait_for(lambda: all(p["spec"].get("nodeName") for p in client.list("pods", "default")[0]))
            pods = client.list("pods", "default")[0]
            assert len({p["metadata"]["annotations"][INDEX_ANNOTATION] for p in pods}) == 4
            # PostBind's PodGroup status patch went out natively too.
            assert wait_for(lambda: client.get("podgroups", "default", "g")["status"].get("phase") == "Scheduled")
            assert rs.client.requests() >= 5 and rs.mirror.applied > 0
        finally:
            rs.stop()
    finally:
        srv.stop()


def test_native_mirror_relist_drops_objects_deleted_meanwhile(store):
    srv = ApiServer(store).start()
    try:
        client = RestClient(srv.url)
        for name in ("a", "b"):
            client.create("pods", make_pod(name))
        local = native().Store()
        ep = rest_endpoint(client)
        m = native().RemoteMirror(ep, local, ["pods"])
        m.start()
        assert m.wait_synced(5000)
        assert wait_for(lambda: local.count("pods") == 2)
        m.stop()
        client.delete("pods", "default", "a")
        client.create("pods", make_pod("c"))
        m2 = native().RemoteMirror(ep, local, ["pods"])
        m2.start()
        assert m2.wait_synced(5000)
        names = {p["metadata"]["name"] for p in local.list("pods", "default")[0]}
        assert names == {"b", "c"}
        # and it keeps watching
        client.create("pods", make_pod("d"))
        assert wait_for(lambda: local.count("pods") == 3)
        m2.stop()
    finally:
        srv.stop()


@pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI not available")
@pytest.mark.parametrize("mutual", [False, True], ids=["server-tls", "mtls"])
def test_native_io_over_tls(store, pki, mutual):
    srv = ApiServer(store, tls_cert=str(pki / "server.crt"), tls_key=str(pki / "server.key"),
                    client_ca=str(pki / "ca.crt") if mutual else None).start()
    try:
        url = srv.url
        assert url.startswith("https://")
        tls = TLSConfig(ca_file=str(pki / "ca.crt"),
                        cert_file=str(pki / "client.crt") if mutual else None,
                        key_file=str(pki / "client.key") if mutual else None)
        client = RestClient(url, tls=tls)
        client.create("nodes", mi355x_node("n0"))
        rs = RemoteScheduler(RestClient(url, tls=tls), load_config(coscheduling_config(FLEXGPU_PLUGINS))).start()
        try:
            assert rs.native_io
            client.create("pods", make_pod("p", limits={GPU: "1"}, requests={GPU: "1"}))
            assert wait_for(lambda: client.get("pods", "default", "p")["spec"].get("nodeName") == "n0")
        finally:
            rs.stop()
    finally:
        srv.stop()


@pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI not available")
def test_native_io_refuses_unknown_ca(store, pki):
    srv = ApiServer(store, tls_cert=str(pki / "server.crt"), tls_key=str(pki / "server.key")).start()
    try:
        url = srv.url
        ep = rest_endpoint(RestClient(url, tls=TLSConfig(ca_file=str(pki / "other.crt"))))
        m = native().RemoteMirror(ep, native().Store(), ["pods"])
        m.start()
        assert not m.wait_synced(1500)
        assert "TLS handshake" in m.last_error()
        m.stop()
    finally:
        srv.stop()


def test_native_mirror_treats_unserved_kind_as_empty():
    """A kind the API does not serve (a CRD that is not installed, e.g. NRT
    on a plain kube-apiserver) syncs as empty instead of blocking startup."""
    import http.server
    import threading

    class NotFound(http.server.BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def do_GET(self):  # noqa: N802
            body = b'{"kind":"Status","apiVersion":"v1","status":"Failure","reason":"NotFound","code":404,' \
                   b'"message":"the server could not find the requested resource"}'
            self.send_response(404)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    httpd = http.server.ThreadingHTTPServer(("127.0.0.1", 0), NotFound)
    threading.Thread(target=httpd.serve_forever, daemon=True).start()
    try:
        ep = native().RestEndpoint("127.0.0.1", httpd.server_address[1])
        local = native().Store()
        m = native().RemoteMirror(ep, local, ["noderesourcetopologies"])
        m.start()
        assert m.wait_synced(3000)
        assert "could not find the requested resource" in m.last_error()
        assert local.count("noderesourcetopologies") == 0
        m.stop()
    finally:
        httpd.shutdown()
        httpd.server_close()


def test_native_writer_honours_client_connection_qps(store):
    """clientConnection.qps/burst (client-go's token bucket) throttle the
    native writer: 25 bindings at qps 20 with a burst of 5 take >= 1 s."""
    from flex_gpu_scheduler_amd.control import ApiServer as _Api

    srv = _Api(store).start()
    try:
        client = RestClient(srv.url)
        client.create("nodes", mi355x_node("n0"))
        cfg = load_config({"apiVersion": "kubescheduler.config.k8s.io/v1beta3", "kind": "KubeSchedulerConfiguration",
                           "clientConnection": {"qps": 20, "burst": 5}})
        assert cfg.client_qps == 20 and cfg.client_burst == 5
        rs = RemoteScheduler(RestClient(srv.url), cfg).start()
        try:
            t0 = time.time()
            for i in range(25):
                client.create("pods", make_pod(f"p{i}", requests={"cpu": "100m"}))
            assert wait_for(lambda: all(p["spec"].get("nodeName") for p in client.list("pods", "default")[0]), 20)
            assert time.time() - t0 >= 0.95
        finally:
            rs.stop()
    finally:
        srv.stop()


class _BindServer:
    """A scripted API server for POST .../binding: `script` lists, per
    binding request, "ok", "stall" (no answer past the client's timeout),
    "ok_close" (answer, then drop the keep-alive connection without saying
    so), "apply_drop" (apply the binding, drop the connection unanswered) or
    "conflict" (409, the pod is already bound)."""

    def __init__(self, script):
        import http.server
        import threading

        self.script = list(script)
        self.posts = 0
        self.bound: dict[str, str] = {}
        srv = self

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def _send(self, code, obj):
                data = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def do_POST(self):  # noqa: N802
                body = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
                srv.posts += 1
                step = srv.script.pop(0) if srv.script else "ok"
                name, node = body["metadata"]["name"], body["target"]["name"]
                if step == "stall":
                    time.sleep(1.5)
                    self.close_connection = True
                    return
                if step == "apply_drop":
                    srv.bound[name] = node
                    self.close_connection = True
                    return
                if step == "conflict" or name in srv.bound:
                    self._send(409, {"kind": "Status", "code": 409, "reason": "Conflict",
                                     "message": f"pod {name} is already assigned to node {srv.bound.get(name)}"})
                    return
                srv.bound[name] = node
                self._send(201, {"kind": "Status", "status": "Success"})
                if step == "ok_close":
                    self.close_connection = True

            def do_GET(self):  # noqa: N802
                name = self.path.rsplit("/", 1)[-1]
                self._send(200, {"metadata": {"name": name, "namespace": "default", "uid": f"uid-{name}"},
                                 "spec": {"nodeName": srv.bound.get(name, "")}})

            def log_message(self, *a):
                pass

        import http.server as hs

        self.httpd = hs.ThreadingHTTPServer(("127.0.0.1", 0), H)
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        self.port = self.httpd.server_address[1]

    def client(self, timeout_ms=30000):
        return native().RestApiClient(native().RestEndpoint("127.0.0.1", self.port, timeout_ms=timeout_ms))

    def close(self):
        self.httpd.shutdown()
        self.httpd.server_close()


def _pod(name):
    return {"metadata": {"name": name, "namespace": "default", "uid": f"uid-{name}"}, "spec": {}}


def test_binding_is_not_resent_after_a_receive_timeout():
    """A binding whose answer does not arrive in time may have been applied:
    it is reported as failed, never sent again on another connection
    (ConnPool retried any error of a pooled connection)."""
    srv = _BindServer(["ok", "stall"])
    try:
        c = srv.client(timeout_ms=300)
        c.bind_json(_pod("a"), "n0")  # leaves a pooled keep-alive connection
        with pytest.raises(Exception):
            c.bind_json(_pod("b"), "n0")
        time.sleep(1.6)
        assert srv.posts == 2  # no retry of "b"
    finally:
        srv.close()


def test_stale_keepalive_connection_is_retried_once():
    srv = _BindServer(["ok_close", "ok"])
    try:
        c = srv.client()
        c.bind_json(_pod("a"), "n0")
        time.sleep(0.1)  # the server has closed the pooled connection
        c.bind_json(_pod("b"), "n1")
        assert srv.bound == {"a": "n0", "b": "n1"} and srv.posts == 2
    finally:
        srv.close()


def test_retried_binding_conflict_on_same_node_is_success():
    """The first attempt was applied but its connection died unanswered: the
    retry gets 409 'already assigned', and the pod bound to the same node
    makes that binding a success."""
    srv = _BindServer(["ok", "apply_drop"])
    try:
        c = srv.client()
        c.bind_json(_pod("a"), "n0")
        c.bind_json(_pod("b"), "n1")  # apply_drop, then the retry conflicts
        assert srv.bound["b"] == "n1" and srv.posts == 3
        # A conflict with another node is still an error.
        srv.script = ["conflict"]
        with pytest.raises(Exception):
            c.bind_json(_pod("c"), "n2")
    finally:
        srv.close()


@pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI not available")
@pytest.mark.parametrize("native_http", [True, False], ids=["native-http", "python-http"])
def test_mtls_server_requires_a_client_certificate(store, pki, native_http):
    """--client-ca-file: a client with the right CA but no certificate is
    refused at the handshake; one with a CA-signed certificate gets in."""
    srv = ApiServer(store, tls_cert=str(pki / "server.crt"), tls_key=str(pki / "server.key"),
                    client_ca=str(pki / "ca.crt"), native_http=native_http).start()
    try:
        assert srv.native_http is native_http and srv.url.startswith("https://")
        anon = RestClient(srv.url, tls=TLSConfig(ca_file=str(pki / "ca.crt")))
        with pytest.raises(Exception):
            anon.list("nodes")
        ok = RestClient(srv.url, tls=TLSConfig(ca_file=str(pki / "ca.crt"), cert_file=str(pki / "client.crt"),
                                                key_file=str(pki / "client.key")))
        assert ok.list("nodes")[0] == []
    finally:
        srv.stop()
