"""Leveled native logging (csrc/common/log.h) and the CLI's JSON log format.

The reference logs FlexGPU's and NRT's placement state at klog V(6)
(pkg/flexgpu/flex_gpu.go:42-50,103-107); --v drives the same here."""
import json
import logging
import subprocess
import sys
import textwrap
from pathlib import Path

from flex_gpu_scheduler_amd._native import native
from flex_gpu_scheduler_amd.cli import JsonLogFormatter
from flex_gpu_scheduler_amd.models import GPU, make_pod, mi355x_node, mi355x_nrt
from helpers import FLEXGPU_PLUGINS, coscheduling_config, start, wait_bound

ROOT = str(Path(__file__).resolve().parents[1])


def test_python_json_log_lines_escape_messages():
    rec = logging.LogRecord("xsched", logging.WARNING, "cli.py", 7, 'pod "a\\b"\nsecond line %s', ("x",), None)
    d = json.loads(JsonLogFormatter().format(rec))
    assert d["msg"] == 'pod "a\\b"\nsecond line x' and d["level"] == "WARNING" and d["caller"] == "cli.py:7"


def _cfg():
    plugins = {k: {"enabled": list(v["enabled"])} for k, v in FLEXGPU_PLUGINS.items()}
    plugins["filter"]["enabled"].append({"name": "NodeResourceTopologyMatch"})
    return coscheduling_config(plugins)


def test_v6_logs_gpu_ledger_and_chosen_indexes(store):
    store.create("nodes", mi355x_node("n0"))
    store.create("noderesourcetopologies", mi355x_nrt("n0"))
    native().set_log_capture(10000)
    s = start(store, _cfg())
    try:
        native().set_log_verbosity(6)
        store.create("pods", make_pod("p0", requests={"cpu": "1", "memory": "1Gi"}, limits={GPU: "2"}))
        wait_bound(s, 1)
        native().set_log_verbosity(0)
        lines = [json.loads(x) for x in native().drain_log()]
        msgs = {d["msg"] for d in lines}
        assert {"pod info", "node gpu usages", "assigned gpu indexes", "numa zone", "topology filter"} <= msgs
        usages = [d for d in lines if d["msg"] == "node gpu usages"]
        assert sorted(d["gpu"] for d in usages[:8]) == list(range(8)) and all(d["node"] == "n0" for d in usages)
        chosen = [d for d in lines if d["msg"] == "assigned gpu indexes"]
        assert chosen[0]["pod"] == "default/p0" and len(chosen[0]["indexes"].split(",")) == 2
        assert all(d["v"] == 6 and d["caller"] for d in lines)
        # V(0): the same path logs nothing.
        store.create("pods", make_pod("p1", limits={GPU: "1"}))
        wait_bound(s, 2)
        assert [x for x in native().drain_log() if "gpu" in x] == []
    finally:
        native().set_log_verbosity(0)
        native().set_log_capture(0)
        s.stop()


def test_resource_registry_overflow_is_reported():
    """A pod naming more distinct resources than the registry holds is dropped
    with a log line and a Warning event on the pod (a fresh process: the
    registry is process-wide and never shrinks)."""
    code = textwrap.dedent("""
        import json, time
        from flex_gpu_scheduler_amd._native import native
        from flex_gpu_scheduler_amd.models import make_pod, mi355x_node
        from flex_gpu_scheduler_amd.scheduler import Store, new_scheduler
        native().set_log_capture(1000)
        st = Store()
        st.create("nodes", json.dumps(mi355x_node("n0")))
        s = new_scheduler(st, None)
        s.start()
        limits = {f"example.com/r{i}": "1" for i in range(70)}
        st.create("pods", json.dumps(make_pod("big", requests=limits, limits=limits)))
        deadline = time.time() + 10
        evs = []
        while time.time() < deadline and not evs:
            evs = [e for e in st.list("events", "default")[0] if e.get("reason") == "FailedToDecode"]
            time.sleep(0.05)
        s.stop()
        logs = [json.loads(x) for x in native().drain_log()]
        print(json.dumps({"events": evs, "logs": logs}))
    """)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120,
                       env={"PYTHONPATH": ROOT, "PATH": "/usr/bin:/bin"})
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["events"] and out["events"][0]["involvedObject"]["name"] == "big"
    assert out["events"][0]["type"] == "Warning" and "too many distinct resource names" in out["events"][0]["message"]
    drops = [d for d in out["logs"] if d["msg"] == "informer dropped object"]
    assert drops and drops[0]["name"] == "big" and drops[0]["level"] == "WARNING"
