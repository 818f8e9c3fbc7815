"""Multi-process end to end on CPU: apiserver, node agents, controller and
scheduler as separate OS processes talking HTTP (the deployment shape of the
Helm charts), plus checkpoint/restore of the API store."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

from flex_gpu_scheduler_amd.control import RestClient

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn(*args, log=None):
    env = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.Popen([sys.executable, "-m", "flex_gpu_scheduler_amd", *args], cwd=ROOT, env=env,
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


def wait_for(fn, timeout=60.0):  # generous: five processes start under a loaded CI box
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            if fn():
                return True
        except Exception:  # noqa: BLE001
            pass
        time.sleep(0.05)
    return False


SCHED_CFG = """
apiVersion: kubescheduler.config.k8s.io/v1beta2
kind: KubeSchedulerConfiguration
leaderElection:
  leaderElect: false
profiles:
- schedulerName: flex-gpu-scheduler
  plugins:
    queueSort:
      enabled: [{name: Coscheduling}]
      disabled: [{name: "*"}]
    preFilter:
      enabled: [{name: Coscheduling}]
    postFilter:
      enabled: [{name: Coscheduling}]
    permit:
      enabled: [{name: Coscheduling}]
    reserve:
      enabled: [{name: Coscheduling}, {name: FlexGPU}]
    postBind:
      enabled: [{name: Coscheduling}]
    filter:
      enabled: [{name: FlexGPU}]
    score:
      enabled: [{name: FlexGPU}]
    bind:
      enabled: [{name: FlexGPU}]
      disabled: [{name: DefaultBinder}]
  pluginConfig:
  - name: Coscheduling
    args: {permitWaitingTimeSeconds: 10, deniedPGExpirationTimeSeconds: 3}
"""

WORKLOAD = """
apiVersion: scheduling.sigs.k8s.io/v1alpha1
kind: PodGroup
metadata: {name: train, namespace: default}
spec: {minMember: 4}
---
apiVersion: v1
kind: List
items:
""" + "".join(f"""- apiVersion: v1
  kind: Pod
  metadata:
    name: rank-{i}
    namespace: default
    labels: {{pod-group.scheduling.sigs.k8s.io: train}}
  spec:
    schedulerName: flex-gpu-scheduler
    containers:
    - name: c
      image: rocm/pytorch
      resources:
        limits: {{amd.com/gpu: "2"}}
        requests: {{amd.com/gpu: "2"}}
""" for i in range(4))


@pytest.mark.slow
def test_processes_schedule_a_gang(tmp_path):
    port = free_port()
    url = f"http://127.0.0.1:{port}"
    snap = tmp_path / "store.json"
    cfg = tmp_path / "sched.yaml"
    cfg.write_text(SCHED_CFG)
    wl = tmp_path / "wl.yaml"
    wl.write_text(WORKLOAD)
    procs = []
    try:
        procs.append(spawn("apiserver", "--port", str(port), "--save", str(snap)))
        c = RestClient(url)
        assert wait_for(c.healthy)
        procs.append(spawn("node-agent", "--master", url, "--node-name", "mi355x-a", "--fake-gpus", "8",
                           "--no-telemetry", "--heartbeat", "1"))
        procs.append(spawn("node-agent", "--master", url, "--node-name", "mi355x-b", "--fake-gpus", "8",
                           "--no-telemetry", "--heartbeat", "1"))
        procs.append(spawn("controller", "--masterUrl", url, "--enableLeaderElection"))
        procs.append(spawn("scheduler", "--master", url, "--config", str(cfg), "--metrics-bind-address",
                           f"127.0.0.1:{free_port()}"))
        assert wait_for(lambda: len(c.list("nodes")[0]) == 2)
        out = subprocess.run([sys.executable, "-m", "flex_gpu_scheduler_amd", "apply", "--master", url, "-f", str(wl)],
                             cwd=ROOT, capture_output=True, text=True, env=dict(os.environ, PYTHONPATH=ROOT))
        assert out.returncode == 0, out.stderr
        assert wait_for(lambda: all(p["spec"].get("nodeName") for p in c.list("pods", "default")[0])
                        and len(c.list("pods", "default")[0]) == 4, 60), c.list("pods", "default")[0]
        pods = c.list("pods", "default")[0]
        assert all("amd.com/gpu-index" in p["metadata"]["annotations"] for p in pods)
        # Four 2-GPU ranks fit one 8-GPU node: the xGMI-unaware FlexGPU score
        # still bin-packs, so they share a node.
        assert len({p["spec"]["nodeName"] for p in pods}) == 1
        assert wait_for(lambda: c.get("podgroups", "default", "train")["status"].get("phase") == "Scheduled")
        # The controller holds the lease.
        assert wait_for(lambda: c.get("leases", "kube-system", "sched-plugins-controller") is not None)
    finally:
        for p in reversed(procs):
            p.terminate()
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
    # The API server wrote a snapshot on shutdown; restore it into a fresh store.
    from flex_gpu_scheduler_amd import Store
    from flex_gpu_scheduler_amd.control.snapshot import restore
    data = json.loads(snap.read_text())
    s2 = Store()
    assert restore(s2, data) >= 7
    assert all(p["spec"]["nodeName"] for p in s2.list("pods", "default")[0])


def test_healthz_checks_fail_and_report():
    from flex_gpu_scheduler_amd.control.httpserve import ServiceHTTP
    import urllib.error
    import urllib.request

    http = ServiceHTTP().start()
    state = {"ok": True}
    http.add_health_check("loop", lambda: (state["ok"], "no progress for 31.0s"))
    http.add_health_check("sync", lambda: (False, "not synced"), ready_only=True)
    try:
        assert urllib.request.urlopen(http.url + "/healthz").read() == b"ok"
        with pytest.raises(urllib.error.HTTPError) as ei:
            urllib.request.urlopen(http.url + "/readyz")
        assert ei.value.code == 500 and b"[-]sync failed: not synced" in ei.value.read()
        state["ok"] = False
        with pytest.raises(urllib.error.HTTPError) as ei:
            urllib.request.urlopen(http.url + "/healthz")
        body = ei.value.read()
        assert ei.value.code == 500 and b"[-]loop failed: no progress" in body
    finally:
        http.stop()


def test_leader_healthz_adaptor():
    from flex_gpu_scheduler_amd.control.leaderelection import LeaderElector

    le = LeaderElector(None, "l", "kube-system", "me", lease_duration=15.0, renew_deadline=10.0, retry_period=2.0)
    assert le.healthz()[0]  # not leading
    le.is_leader.set()
    import time as _t

    le.renewed_at = _t.monotonic()
    assert le.healthz()[0]
    le.renewed_at = _t.monotonic() - 40
    ok, why = le.healthz()
    assert not ok and "renew" in why


def test_scheduler_loop_age_and_new_gauges(store):
    import time as _t

    from flex_gpu_scheduler_amd import load_config, new_scheduler

    s = new_scheduler(store, load_config(None), start=True)
    try:
        _t.sleep(1.3)
        assert 0 <= s.loop_age_seconds() < 1.0
        text = s.metrics_text()
        for line in ('scheduler_scheduler_goroutines{work="binding"}', 'scheduler_scheduler_cache_size{type="nodes"}',
                     'scheduler_scheduler_cache_size{type="assumed_pods"}'):
            assert line in text, line
    finally:
        s.stop()
    assert s.loop_age_seconds() == 0.0
