"""HTTP API server + REST client (the envtest analog) and the
informer/work-queue machinery shared by the controllers."""
import http.client
import json
import threading
import time

import pytest

from flex_gpu_scheduler_amd.control import ApiServer, Informer, LocalClient, RestClient, WorkQueue
from flex_gpu_scheduler_amd.control.apiserver import apply_json_patch
from flex_gpu_scheduler_amd.control.client import ApiException
from flex_gpu_scheduler_amd.control.resources import parse_path, resource
from flex_gpu_scheduler_amd.control.selectors import label_matcher, parse_selector
from flex_gpu_scheduler_amd.models import make_node, make_pod, make_pod_group


@pytest.fixture(params=[True, False], ids=["native-http", "python-http"])
def server(request, store):
    """Both HTTP front ends over the same store: the native one
    (csrc/apiserver, the default) and http.server (the TLS path)."""
    srv = ApiServer(store, native_http=request.param).start()
    assert srv.native_http is request.param
    yield srv
    srv.stop()


@pytest.fixture(params=["local", "rest"])
def client(request, store, server):
    return LocalClient(store) if request.param == "local" else RestClient(server.url)


def test_paths_roundtrip():
    r = resource("pg")
    assert r.kind_plural == "podgroups"
    p = r.object_path("team-a", "g1", "status")
    assert p == "/apis/scheduling.sigs.k8s.io/v1alpha1/namespaces/team-a/podgroups/g1/status"
    assert parse_path(p)[1:] == ("team-a", "g1", "status")
    assert parse_path("/api/v1/nodes/n1")[0].kind_plural == "nodes"
    assert parse_path("/api/v1/namespaces/kube-system")[0].kind_plural == "namespaces"
    assert parse_path("/api/v1/namespaces/x/pods")[1:] == ("x", "", "")


def test_selectors():
    m = label_matcher("app=web,tier!=db,env in (prod, staging),!legacy,team")
    assert m({"metadata": {"labels": {"app": "web", "env": "prod", "team": "x"}}})
    assert not m({"metadata": {"labels": {"app": "web", "env": "dev", "team": "x"}}})
    assert not m({"metadata": {"labels": {"app": "web", "env": "prod", "team": "x", "legacy": "1"}}})
    assert [r.op for r in parse_selector("a notin (x,y)")] == ["notin"]


def test_crud_and_errors(client):
    client.create("nodes", make_node("n1", {"cpu": "4"}))
    assert client.get("nodes", "", "n1")["metadata"]["name"] == "n1"
    assert client.get("nodes", "", "nope") is None
    with pytest.raises(ApiException) as e:
        client.create("nodes", make_node("n1", {"cpu": "4"}))
    assert e.value.code == 409
    pod = client.create("pods", make_pod("p", "ns1", requests={"cpu": "1"}, labels={"app": "x"}))
    assert pod["metadata"]["namespace"] == "ns1" and pod["status"]["phase"] == "Pending"
    assert pod["kind"] == "Pod" and pod["apiVersion"] == "v1"
    items, rv = client.list("pods", "ns1", label_selector="app=x")
    assert [p["metadata"]["name"] for p in items] == ["p"] and rv > 0
    assert client.list("pods", "ns1", label_selector="app=y")[0] == []
    assert len(client.list("pods", "", field_selector="metadata.name=p")[0]) == 1
    stale = dict(pod)
    client.patch("pods", "ns1", "p", {"metadata": {"labels": {"b": "1"}}})
    with pytest.raises(ApiException) as e:
        client.update("pods", stale)
    assert e.value.code == 409
    cur = client.get("pods", "ns1", "p")
    assert cur["metadata"]["labels"] == {"app": "x", "b": "1"}
    cur["spec"]["priority"] = 5
    assert client.update("pods", cur)["spec"]["priority"] == 5
    with pytest.raises(ApiException) as e:
        client.delete("pods", "ns1", "p", uid="wrong")
    assert e.value.code == 409
    client.delete("pods", "ns1", "p")
    assert client.get("pods", "ns1", "p") is None
    with pytest.raises(ApiException) as e:
        client.patch("pods", "ns1", "p", {"spec": {}})
    assert e.value.code == 404


def test_binding_copies_annotations(client):
    client.create("pods", make_pod("p"))
    client.bind("default", "p", "", "node-3", {"amd.com/gpu-index": "5"})
    p = client.get("pods", "default", "p")
    assert p["spec"]["nodeName"] == "node-3"
    assert p["metadata"]["annotations"]["amd.com/gpu-index"] == "5"
    assert any(c["type"] == "PodScheduled" and c["status"] == "True" for c in p["status"]["conditions"])
    with pytest.raises(ApiException) as e:
        client.bind("default", "p", "", "node-4")
    assert e.value.code == 409


def test_graceful_delete_sets_deletion_timestamp(client):
    client.create("pods", make_pod("p"))
    p = client.delete("pods", "default", "p", grace_seconds=30)
    assert p["metadata"]["deletionTimestamp"]
    assert client.get("pods", "default", "p")["metadata"]["deletionGracePeriodSeconds"] == 30


def test_json_patch_and_strategic(server, store):
    store.create("pods", make_pod("p", labels={"a": "1"}))
    conn = http.client.HTTPConnection(*server.address)
    ops = [{"op": "add", "path": "/metadata/labels/b", "value": "2"}, {"op": "remove", "path": "/metadata/labels/a"},
           {"op": "test", "path": "/metadata/name", "value": "p"}]
    conn.request("PATCH", "/api/v1/namespaces/default/pods/p", json.dumps(ops),
                 {"Content-Type": "application/json-patch+json"})
    r = conn.getresponse()
    assert r.status == 200, r.read()
    assert json.loads(r.read())["metadata"]["labels"] == {"b": "2"}
    conn.request("PATCH", "/api/v1/namespaces/default/pods/p/status", json.dumps({"status": {"phase": "Running"}}),
                 {"Content-Type": "application/strategic-merge-patch+json"})
    r = conn.getresponse()
    assert r.status == 200 and json.loads(r.read())["status"]["phase"] == "Running"
    conn.request("GET", "/api/v1/namespaces/default/pods/missing")
    r = conn.getresponse()
    body = json.loads(r.read())
    assert r.status == 404 and body["kind"] == "Status" and body["reason"] == "NotFound"
    conn.request("GET", "/version")
    assert json.loads(conn.getresponse().read())["minor"] == "23"
    assert apply_json_patch({"a": [1, 2]}, [{"op": "add", "path": "/a/-", "value": 3},
                                            {"op": "move", "from": "/a/0", "path": "/b"}]) == {"a": [2, 3], "b": 1}


def test_rest_watch_stream_and_resume(server, store):
    c = RestClient(server.url)
    store.create("pods", make_pod("before"))
    w = c.watch(["pods"], "default", 0)
    try:
        evs = []
        deadline = time.time() + 5
        while time.time() < deadline and not any(e[2]["metadata"]["name"] == "before" for e in evs):
            evs += w.next(200)
        assert evs[0][0] == "ADDED"  # synthetic ADDED for the current state
        store.create("pods", make_pod("after"))
        store.delete("pods", "default", "before")
        got = []
        deadline = time.time() + 5
        while time.time() < deadline and len(got) < 2:
            got += w.next(200)
        assert [(t, o["metadata"]["name"]) for t, _, o, _ in got] == [("ADDED", "after"), ("DELETED", "before")]
        assert got[1][3] > got[0][3]  # DELETED carries its own resourceVersion
    finally:
        w.stop()
    # Resume from a resourceVersion: only later events are replayed.
    rv = store.resource_version
    store.create("pods", make_pod("later"))
    w = c.watch(["pods"], "default", rv)
    try:
        got = []
        deadline = time.time() + 5
        while time.time() < deadline and not got:
            got += w.next(200)
        assert [o["metadata"]["name"] for _, _, o, _ in got] == ["later"]
    finally:
        w.stop()


def test_watch_label_selector_http(server, store):
    conn = http.client.HTTPConnection(*server.address)
    conn.request("GET", "/api/v1/pods?watch=true&labelSelector=app%3Dweb&timeoutSeconds=1")
    r = conn.getresponse()
    store.create("pods", make_pod("a", labels={"app": "web"}))
    store.create("pods", make_pod("b", labels={"app": "db"}))
    lines = [json.loads(x) for x in r.read().splitlines() if x.strip()]
    assert [x["object"]["metadata"]["name"] for x in lines] == ["a"]


def test_informer_tracks_store(client, store):
    store.create("podgroups", make_pod_group("g0", min_member=1))
    inf = Informer(client, "podgroups").start()
    seen = {"add": [], "upd": [], "del": []}
    inf.add_event_handler(lambda o: seen["add"].append(o["metadata"]["name"]),
                          lambda o, n: seen["upd"].append(n["metadata"]["name"]),
                          lambda o: seen["del"].append(o["metadata"]["name"]))
    try:
        assert inf.wait_for_sync(5)
        store.create("podgroups", make_pod_group("g1", min_member=2))
        store.patch("podgroups", "default", "g1", {"status": {"phase": "Pending"}})
        store.delete("podgroups", "default", "g0")
        deadline = time.time() + 5
        while time.time() < deadline and not (seen["del"] and seen["upd"]):
            time.sleep(0.02)
        assert seen["add"] == ["g0", "g1"] and seen["upd"] == ["g1"] and seen["del"] == ["g0"]
        assert inf.get("default", "g1")["status"]["phase"] == "Pending"
        assert inf.get("default", "g0") is None
    finally:
        inf.stop()


def test_informer_relists_after_expired_watch(store):
    inf = Informer(LocalClient(store), "pods").start()
    try:
        assert inf.wait_for_sync(5)
        store.create("pods", make_pod("x"))
        deadline = time.time() + 5
        while time.time() < deadline and inf.get("default", "x") is None:
            time.sleep(0.01)
        assert inf.get("default", "x") is not None and inf.relists == 1
    finally:
        inf.stop()


def test_workqueue_dedup_and_rate_limit():
    q = WorkQueue()
    q.add("a")
    q.add("a")
    q.add("b")
    assert len(q) == 2
    k = q.get(0.1)
    assert k == "a"
    q.add("a")           # re-added while processing: held until done()
    assert q.get(0.05) == "b"
    assert q.get(0.05) is None
    q.done("a")
    assert q.get(0.1) == "a"
    q.done("a")
    q.done("b")
    t0 = time.monotonic()
    q.add_rate_limited("c")
    q.add_rate_limited("c")  # second failure: 10 ms
    assert q.num_requeues("c") == 2
    assert q.get(1.0) == "c" and time.monotonic() - t0 < 0.5
    q.forget("c")
    assert q.num_requeues("c") == 0
    q.done("c")
    assert q.get(1.0) == "c"  # the second delayed add fires too (no coalescing across done)
    q.done("c")
    th = threading.Thread(target=lambda: (time.sleep(0.05), q.shutdown()))
    th.start()
    assert q.get() is None
    th.join()


def _raw(url: str, payload: bytes) -> bytes:
    import socket
    from urllib.parse import urlparse

    u = urlparse(url)
    with socket.create_connection((u.hostname, u.port), timeout=5) as s:
        s.sendall(payload)
        out = b""
        while True:
            chunk = s.recv(65536)
            if not chunk:
                break
            out += chunk
        return out


def test_native_http_rejects_oversized_and_malformed_chunks(store):
    """A chunk size near 2**64 used to wrap the size check and make the
    server read forever; it is 413 now, and a non-hex size line is 400."""
    srv = ApiServer(store, native_http=True).start()
    try:
        head = b"POST /api/v1/namespaces/default/pods HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n"
        out = _raw(srv.url, head + b"ffffffffffffffff\r\n")
        assert out.startswith(b"HTTP/1.1 400"), out[:80]  # 16 hex digits: more than any body
        out = _raw(srv.url, head + b"fffffffffffffff\r\n")
        assert out.startswith(b"HTTP/1.1 413"), out[:80]
        out = _raw(srv.url, head + b"zz\r\n")
        assert out.startswith(b"HTTP/1.1 400"), out[:80]
        # A well-formed chunked create still works.
        body = json.dumps(make_pod("chunked")).encode()
        head_close = head.replace(b"Host: x\r\n", b"Host: x\r\nConnection: close\r\n")
        out = _raw(srv.url, head_close + b"%x\r\n" % len(body) + body + b"\r\n0\r\n\r\n")
        assert out.startswith(b"HTTP/1.1 201"), out[:120]
    finally:
        srv.stop()


def test_native_http_refuses_unauthenticated_body_before_reading_it(store):
    srv = ApiServer(store, native_http=True, token="s3cret").start()
    try:
        # Claims a 200 MiB body and sends none: answered 401 at once.
        out = _raw(srv.url, b"POST /api/v1/namespaces/default/pods HTTP/1.1\r\nHost: x\r\n"
                            b"Content-Length: 209715200\r\n\r\n")
        assert out.startswith(b"HTTP/1.1 401"), out[:80]
        out = _raw(srv.url, b"GET /healthz HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
        assert out.startswith(b"HTTP/1.1 200")
    finally:
        srv.stop()
