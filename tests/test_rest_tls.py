"""TLS to a kube-apiserver (client-go rest.TLSClientConfig semantics): a
kubeconfig's certificate-authority-data verifies the server, client
certificate data authenticates us (mTLS), insecure-skip-tls-verify skips
verification, and an unknown CA is refused. Certificates come from the
openssl CLI; the server is a stdlib HTTPS server answering one pod GET."""
import base64
import http.server
import json
import shutil
import ssl
import threading

import pytest

from flex_gpu_scheduler_amd.cli import master_from_kubeconfig
from flex_gpu_scheduler_amd.control.client import RestClient, TLSConfig, kubeconfig_connection

pytestmark = pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI not available")


class _Handler(http.server.BaseHTTPRequestHandler):
    def do_GET(self):  # noqa: N802
        body = json.dumps({"apiVersion": "v1", "kind": "Pod",
                           "metadata": {"name": "p", "namespace": "default"},
                           "client": self.request.getpeercert() is not None}).encode()
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def log_message(self, *a):
        pass


@pytest.fixture(params=[False, True], ids=["server-tls", "mtls"])
def server(request, pki):
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.load_cert_chain(pki / "server.crt", pki / "server.key")
    if request.param:
        ctx.verify_mode = ssl.CERT_REQUIRED
        ctx.load_verify_locations(pki / "ca.crt")
    httpd = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _Handler)
    httpd.socket = ctx.wrap_socket(httpd.socket, server_side=True)
    t = threading.Thread(target=httpd.serve_forever, daemon=True)
    t.start()
    yield f"https://127.0.0.1:{httpd.server_address[1]}", request.param
    httpd.shutdown()
    httpd.server_close()


def _kubeconfig(tmp_path, pki, url, *, ca=True, client=True, insecure=False):
    b64 = lambda p: base64.b64encode((pki / p).read_bytes()).decode()  # noqa: E731
    cluster = {"server": url}
    if ca:
        cluster["certificate-authority-data"] = b64("ca.crt")
    if insecure:
        cluster["insecure-skip-tls-verify"] = True
    user = {"token": "t0k"}
    if client:
        user.update({"client-certificate-data": b64("client.crt"), "client-key-data": b64("client.key")})
    kc = {"apiVersion": "v1", "kind": "Config", "current-context": "c",
          "clusters": [{"name": "k", "cluster": cluster}], "users": [{"name": "u", "user": user}],
          "contexts": [{"name": "c", "context": {"cluster": "k", "user": "u"}}]}
    p = tmp_path / "kubeconfig"
    p.write_text(json.dumps(kc))  # JSON is valid YAML
    return str(p)


def test_kubeconfig_ca_and_client_cert(tmp_path, pki, server):
    url, _ = server
    srv, token, tls = kubeconfig_connection(_kubeconfig(tmp_path, pki, url))
    assert (srv, token) == (url, "t0k")
    assert master_from_kubeconfig(_kubeconfig(tmp_path, pki, url)) == (url, "t0k")
    pod = RestClient(srv, token=token, tls=tls).get("pods", "default", "p")
    assert pod["metadata"]["name"] == "p"


def test_unknown_ca_is_refused(tmp_path, pki, server):
    url, _ = server
    c = RestClient(url, tls=TLSConfig(ca_file=str(pki / "other.crt")))
    with pytest.raises(ssl.SSLError):
        c.get("pods", "default", "p")


def test_insecure_skip_verify(tmp_path, pki, server):
    url, mtls = server
    _, _, tls = kubeconfig_connection(_kubeconfig(tmp_path, pki, url, ca=False, client=mtls, insecure=True))
    assert RestClient(url, tls=tls).get("pods", "default", "p")["kind"] == "Pod"


def test_relative_paths_and_token_file(tmp_path, pki):
    (tmp_path / "tok").write_text("from-file\n")
    kc = {"current-context": "c", "clusters": [{"name": "k", "cluster": {"server": "https://h:6443",
                                                                        "certificate-authority": "ca.crt"}}],
          "users": [{"name": "u", "user": {"tokenFile": "tok"}}],
          "contexts": [{"name": "c", "context": {"cluster": "k", "user": "u"}}]}
    (tmp_path / "kc").write_text(json.dumps(kc))
    srv, token, tls = kubeconfig_connection(str(tmp_path / "kc"))
    assert (srv, token) == ("https://h:6443", "from-file")
    assert tls.ca_file == str(tmp_path / "ca.crt")
