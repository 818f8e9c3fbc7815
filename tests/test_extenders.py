"""HTTP scheduler extenders (the `extenders:` block of a KubeSchedulerConfiguration)
in the native scheduling cycle, against a Python http.server extender.

Reference behaviour: vendor/k8s.io/kubernetes/pkg/scheduler/extender.go:148-409
(Filter / Prioritize / Bind / ProcessPreemption, IsInterested, ignorable,
nodeCacheCapable), generic_scheduler.go:340-391 (findNodesThatPassExtenders)
and :449-488 (score x weight x 10), scheduler.go bind() (extendersBinding) and
preemption.go callExtenders; config validation in validation.go
validateExtenders and the strict codec of apis/config/scheme/scheme.go:35."""
import http.server
import json
import threading
import time

import pytest

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.config import ConfigError
from flex_gpu_scheduler_amd.models import make_node, make_pod
from helpers import placements, wait_bound

V1B3 = {"apiVersion": "kubescheduler.config.k8s.io/v1beta3", "kind": "KubeSchedulerConfiguration"}


class FakeExtender:
    """Records every call; verbs behave per the attributes below."""

    def __init__(self, store=None):
        self.calls: list[tuple[str, dict]] = []
        self.reject: dict[str, str] = {}          # node -> FailedNodes message
        self.unresolvable: dict[str, str] = {}    # node -> FailedAndUnresolvableNodes message
        self.scores: dict[str, int] = {}
        self.preempt_keep: set[str] | None = None  # nodes kept by the preempt verb
        self.error: str = ""
        self.store = store
        ext = self

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def do_POST(self):  # noqa: N802
                body = json.loads(self.rfile.read(int(self.headers["Content-Length"])) or b"{}")
                verb = self.path.rsplit("/", 1)[-1]
                ext.calls.append((self.path, body))
                out = ext.handle(verb, body)
                data = json.dumps(out).encode()
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def log_message(self, *a):
                pass

        self.httpd = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}/scheduler"

    def names(self, body):
        if body.get("NodeNames") is not None:
            return list(body["NodeNames"])
        return [n["metadata"]["name"] for n in body["Nodes"]["items"]]

    def handle(self, verb, body):
        if verb == "filter":
            if self.error:
                return {"Error": self.error}
            names = self.names(body)
            keep = [n for n in names if n not in self.reject and n not in self.unresolvable]
            res = {"FailedNodes": {n: m for n, m in self.reject.items() if n in names},
                   "FailedAndUnresolvableNodes": {n: m for n, m in self.unresolvable.items() if n in names}}
            if body.get("NodeNames") is not None:
                res["NodeNames"] = keep
            else:
                res["Nodes"] = {"items": [n for n in body["Nodes"]["items"] if n["metadata"]["name"] in keep]}
            return res
        if verb == "prioritize":
            return [{"Host": n, "Score": self.scores.get(n, 0)} for n in self.names(body)]
        if verb == "bind":
            self.store.bind(body["PodNamespace"], body["PodName"], body["PodUID"], body["Node"], {})
            return {"Error": ""}
        if verb == "preempt":
            vic = body.get("NodeNameToMetaVictims") or {
                n: {"Pods": [{"UID": p["metadata"]["uid"]} for p in v["Pods"]]}
                for n, v in (body.get("NodeNameToVictims") or {}).items()}
            keep = self.preempt_keep if self.preempt_keep is not None else set(vic)
            return {"NodeNameToMetaVictims": {n: v for n, v in vic.items() if n in keep}}
        return {}

    def verbs(self):
        return [p.rsplit("/", 1)[-1] for p, _ in self.calls]

    def close(self):
        self.httpd.shutdown()
        self.httpd.server_close()


@pytest.fixture
def ext(store):
    e = FakeExtender(store)
    yield e
    e.close()


def cfg(*extenders, **top):
    return {**V1B3, "extenders": list(extenders), **top}


def nodes(store, n=4, cpu="8"):
    for i in range(n):
        store.create("nodes", make_node(f"n{i}", {"cpu": cpu, "memory": "32Gi", "pods": "110"}))


def condition(store, name):
    for c in (store.get("pods", "default", name).get("status") or {}).get("conditions") or []:
        if c.get("type") == "PodScheduled":
            return c
    return {}


def wait_for(pred, timeout=10.0):
    t0 = time.time()
    while not pred():
        assert time.time() - t0 < timeout
        time.sleep(0.005)


def test_filter_prioritize_and_bind(store, ext):
    nodes(store)
    ext.reject = {"n0": "extender says no"}
    ext.unresolvable = {"n1": "never here"}
    ext.scores = {"n2": 0, "n3": 10}
    s = new_scheduler(store, load_config(cfg({"urlPrefix": ext.url, "filterVerb": "filter",
                                              "prioritizeVerb": "prioritize", "weight": 5, "bindVerb": "bind"})),
                      start=True)
    try:
        store.create("pods", make_pod("p", requests={"cpu": "1"}))
        wait_bound(s, 1)
        # n3: extender score 10 x weight 5 x 10 beats any plugin difference.
        assert placements(store) == {"p": "n3"}
        assert ext.verbs() == ["filter", "prioritize", "bind"]
        fbody = ext.calls[0][1]
        assert fbody["Pod"]["metadata"]["name"] == "p" and len(fbody["Nodes"]["items"]) == 4
        # The prioritize call only sees the nodes that passed the filter.
        assert sorted(ext.names(ext.calls[1][1])) == ["n2", "n3"]
        assert ext.calls[2][1] == {"PodName": "p", "PodNamespace": "default",
                                   "PodUID": store.get("pods", "default", "p")["metadata"]["uid"], "Node": "n3"}
    finally:
        s.stop()


def test_extender_filtering_everything_is_a_fit_error(store, ext):
    nodes(store, 2)
    ext.reject = {"n0": "no GPUs left"}
    ext.unresolvable = {"n1": "wrong rack"}
    s = new_scheduler(store, load_config(cfg({"urlPrefix": ext.url, "filterVerb": "filter"})), start=True)
    try:
        store.create("pods", make_pod("p", requests={"cpu": "1"}))
        wait_for(lambda: condition(store, "p").get("reason") == "Unschedulable")
        msg = condition(store, "p")["message"]
        assert msg.startswith("0/2 nodes are available:") and "no GPUs left" in msg and "wrong rack" in msg, msg
        assert placements(store) == {"p": ""}
    finally:
        s.stop()


def test_extender_error_fails_unless_ignorable(store, ext):
    nodes(store, 2)
    ext.error = "backend down"
    s = new_scheduler(store, load_config(cfg({"urlPrefix": ext.url, "filterVerb": "filter"})), start=True)
    try:
        store.create("pods", make_pod("p", requests={"cpu": "1"}))
        wait_for(lambda: condition(store, "p").get("reason") == "SchedulerError")
        assert "backend down" in condition(store, "p")["message"]
    finally:
        s.stop()
    # Ignorable: an unreachable extender is skipped (nothing listens on port 9).
    store.delete("pods", "default", "p")
    s = new_scheduler(store, load_config(cfg({"urlPrefix": "http://127.0.0.1:9/x", "filterVerb": "filter",
                                              "ignorable": True, "httpTimeout": "500ms"})), start=True)
    try:
        store.create("pods", make_pod("q", requests={"cpu": "1"}))
        wait_bound(s, 1)
        assert placements(store)["q"] in ("n0", "n1")
    finally:
        s.stop()


def test_managed_resources_and_node_cache_capable(store, ext):
    nodes(store, 3)
    for i in range(3):
        n = store.get("nodes", "", f"n{i}")
        n["status"]["allocatable"]["example.com/fpga"] = "2"
        store.update("nodes", n)
    ext.reject = {"n0": "no", "n1": "no"}
    s = new_scheduler(store, load_config(cfg({"urlPrefix": ext.url, "filterVerb": "filter", "nodeCacheCapable": True,
                                              "managedResources": [{"name": "example.com/fpga"}]})), start=True)
    try:
        store.create("pods", make_pod("plain", requests={"cpu": "1"}))
        wait_bound(s, 1)
        assert ext.calls == []  # not interested: no managed resource requested
        store.create("pods", make_pod("fpga", requests={"cpu": "1", "example.com/fpga": "1"},
                                      limits={"example.com/fpga": "1"}))
        wait_bound(s, 2)
        assert placements(store)["fpga"] == "n2"
        (path, body), = ext.calls
        assert path == "/scheduler/filter" and sorted(body["NodeNames"]) == ["n0", "n1", "n2"]
        assert "Nodes" not in body
    finally:
        s.stop()


def test_ignored_by_scheduler_resource_is_not_fit_checked(store, ext):
    nodes(store, 1)
    c = load_config(cfg({"urlPrefix": ext.url, "filterVerb": "filter",
                         "managedResources": [{"name": "example.com/lic", "ignoredByScheduler": True}]}))
    assert c.profiles[0].plugin_config["NodeResourcesFit"]["ignoredResources"] == ["example.com/lic"]
    s = new_scheduler(store, c, start=True)
    try:
        # The node advertises no example.com/lic: only the extender accounts it.
        store.create("pods", make_pod("p", requests={"cpu": "1", "example.com/lic": "3"},
                                      limits={"example.com/lic": "3"}))
        wait_bound(s, 1)
        assert placements(store) == {"p": "n0"} and ext.verbs() == ["filter"]
    finally:
        s.stop()


def test_preempt_verb_chooses_the_candidate(store, ext):
    for i in range(2):
        store.create("nodes", make_node(f"n{i}", {"cpu": "4", "memory": "100", "pods": "10"}))
    s = new_scheduler(store, load_config(cfg({"urlPrefix": ext.url, "preemptVerb": "preempt"})), start=True)
    try:
        store.create("pods", make_pod("low0", requests={"memory": "80"}, priority=1, node_name="n0"))
        store.create("pods", make_pod("low1", requests={"memory": "80"}, priority=1, node_name="n1"))
        s.sync_informers(2000)
        ext.preempt_keep = {"n1"}
        store.create("pods", make_pod("high", requests={"memory": "50"}, priority=100))
        wait_for(lambda: store.get("pods", "default", "low1") is None)
        wait_bound(s, 1)
        assert placements(store) == {"low0": "n0", "high": "n1"}
        (path, body), = [c for c in ext.calls if c[0].endswith("/preempt")][:1]
        # Not nodeCacheCapable: whole victim pods, both candidates offered.
        assert sorted(body["NodeNameToVictims"]) == ["n0", "n1"]
        assert body["NodeNameToVictims"]["n1"]["Pods"][0]["metadata"]["name"] == "low1"
    finally:
        s.stop()


# ----------------------------------------------------------------- config
def test_strict_top_level_decode():
    for bad, what in [({"foo": 1}, 'unknown field "foo"'),
                      ({"leaderElection": {"leaderElect": False, "bogus": 1}}, "leaderElection.bogus"),
                      ({"clientConnection": {"qps": 5, "burstt": 1}}, "clientConnection.burstt"),
                      ({"profiles": [{"schedulerName": "x", "plugin": {}}]}, "profiles[0].plugin"),
                      ({"profiles": [{"pluginConfig": [{"name": "Coscheduling", "arg": {}}]}]}, "pluginConfig[0].arg"),
                      ({"extenders": [{"urlPrefix": "http://e", "filterverb": "f"}]}, "filterverb"),
                      ({"healthzBindAddress": "0.0.0.0:10251"}, "healthzBindAddress")]:
        with pytest.raises(ConfigError, match=None) as ei:
            load_config({**V1B3, **bad})
        assert what in str(ei.value), (bad, str(ei.value))
    # v1beta2 still has the bind addresses; debugging fields are inline.
    load_config({"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
                 "healthzBindAddress": "0.0.0.0:10251", "metricsBindAddress": "0.0.0.0:10251",
                 "enableProfiling": True, "leaderElection": {"leaderElect": False, "resourceName": "s"}})


def test_extender_validation():
    def bad(*exts):
        with pytest.raises(ConfigError) as ei:
            load_config(cfg(*exts))
        return str(ei.value)

    assert "positive weight" in bad({"urlPrefix": "http://e", "prioritizeVerb": "p"})
    assert "only one extender can implement bind" in bad({"urlPrefix": "http://a", "bindVerb": "b"},
                                                         {"urlPrefix": "http://b", "bindVerb": "b"})
    assert "duplicate extender managed resource name" in bad(
        {"urlPrefix": "http://a", "managedResources": [{"name": "example.com/x"}]},
        {"urlPrefix": "http://b", "managedResources": [{"name": "example.com/x"}]})
    assert "extended resource name" in bad({"urlPrefix": "http://a", "managedResources": [{"name": "cpu"}]})
    assert "invalid duration" in bad({"urlPrefix": "http://a", "httpTimeout": "5 parsecs"})
    c = load_config(cfg({"urlPrefix": "http://i", "ignorable": True}, {"urlPrefix": "http://m", "httpTimeout": "1m30s"}))
    # Ignorable extenders run last (factory.go:98-110).
    assert [e["urlPrefix"] for e in c.extenders] == ["http://m", "http://i"]
    assert c.extenders[0]["httpTimeoutMs"] == 90000
