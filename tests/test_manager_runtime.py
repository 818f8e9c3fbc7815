"""controller-runtime style Manager + PodGroup/ElasticQuota reconcilers
(reference pkg/controllers/* are no-op kubebuilder stubs) and
the kustomize scaffold (config/, C30) rebuilt under deploy/config.

The reconcilers must converge to the same status as the cmd/controller
controllers, so they are driven through the same case tables as
test_controllers.py (pkg/controller/podgroup_test.go, elasticquota_test.go)."""
import json
import os
import subprocess
import sys
import threading
import time
import urllib.error
import urllib.request

import pytest
import yaml

from flex_gpu_scheduler_amd.control import LocalClient
from flex_gpu_scheduler_amd.control.httpserve import ServiceHTTP
from flex_gpu_scheduler_amd.control.runtime import (Builder, ElasticQuotaReconciler, Manager, PodGroupReconciler,
                                                    Request, Result)
from flex_gpu_scheduler_amd.models import make_elastic_quota, make_pod, make_pod_group
from test_controllers import EQ_CASES, PG_CASES, _eq_norm, _pg, _pods, _used, wait_for

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _manager(store, **kw):
    c = LocalClient(store)
    return Manager(c, **kw).add(PodGroupReconciler(c)).add(ElasticQuotaReconciler(c))


@pytest.mark.parametrize("case", PG_CASES, ids=[c[0] for c in PG_CASES])
def test_podgroup_reconciler_phase_machine(store, case):
    _, min_member, names, pod_phase, prev, desired, next_phase, created = case
    store.create("podgroups", _pg("pg", min_member, prev, created))
    for p in _pods(names, "pg", pod_phase):
        store.create("pods", p)
    mgr = _manager(store).start()
    try:
        if next_phase:
            for n in names:
                store.patch("pods", "default", n, {"status": {"phase": next_phase}})
        wait_for(lambda: store.get("podgroups", "default", "pg")["status"]["phase"] == desired)
        assert mgr.wait_idle()
        assert store.get("podgroups", "default", "pg")["status"]["phase"] == desired
    finally:
        mgr.stop()


@pytest.mark.parametrize("case", EQ_CASES, ids=[c[0] for c in EQ_CASES])
def test_elasticquota_reconciler_used(store, case):
    _, eqs, pods, want = case
    for ns, name, mn, mx in eqs:
        store.create("elasticquotas", make_elastic_quota(name, ns, min=mn, max=mx))
    for p in pods:
        store.create("pods", p)
    mgr = _manager(store).start()
    try:
        for (ns, name), w in want.items():
            assert wait_for(lambda: _eq_norm(_used(store, ns, name)) == _eq_norm(w)), (_used(store, ns, name), w)
    finally:
        mgr.stop()


def test_result_semantics(store):
    """Exceptions back off and retry, requeue_after re-delivers, success forgets."""
    calls: list[tuple[str, float]] = []

    class R:
        def setup_with_manager(self, mgr):
            self.ctl = Builder(mgr).named("probe").for_kind("podgroups").complete(self)

        def reconcile(self, req: Request) -> Result:
            calls.append((req.name, time.monotonic()))
            n = sum(1 for c in calls if c[0] == req.name)
            if req.name == "flaky" and n < 3:
                raise RuntimeError("transient")
            if req.name == "later" and n == 1:
                return Result(requeue_after=0.2)
            return Result()

    r = R()
    mgr = Manager(LocalClient(store)).add(r).start()
    try:
        store.create("podgroups", make_pod_group("flaky", min_member=1))
        store.create("podgroups", make_pod_group("later", min_member=1))
        assert wait_for(lambda: sum(1 for c in calls if c[0] == "flaky") >= 3)
        assert wait_for(lambda: sum(1 for c in calls if c[0] == "later") >= 2)
        later = [t for n, t in calls if n == "later"]
        assert later[1] - later[0] >= 0.15
        assert wait_for(mgr.wait_idle)
        assert r.ctl.counts["error"] == 2 and r.ctl.counts["requeue_after"] == 1
        assert 'controller_runtime_reconcile_total{controller="probe",result="error"} 2' in mgr.metrics_text()
    finally:
        mgr.stop()


def test_probes_and_leader_election(store):
    probe = ServiceHTTP().start()
    metrics = ServiceHTTP().start()
    mgrs = []
    try:
        a = _manager(store, leader_election=True, identity="a", probe_http=probe, metrics_http=metrics).start()
        mgrs.append(a)
        assert wait_for(a.ready)
        assert urllib.request.urlopen(probe.url + "/readyz").status == 200
        assert urllib.request.urlopen(probe.url + "/healthz").status == 200
        body = urllib.request.urlopen(metrics.url + "/metrics").read().decode()
        assert "controller_runtime_reconcile_total" in body and 'workqueue_depth{name="podgroup"}' in body
        b = _manager(store, leader_election=True, identity="b").start()
        mgrs.append(b)
        time.sleep(0.3)
        assert not b.ready()  # synced but not leading: controllers idle
        store.create("podgroups", make_pod_group("g", min_member=1))
        assert wait_for(lambda: (store.get("podgroups", "default", "g").get("status") or {}).get("phase") == "Pending")
        lease = store.get("leases", "kube-system", "sched-plugins-manager")
        assert lease["spec"]["holderIdentity"] == "a"
    finally:
        for m in mgrs:
            m.stop()
        probe.stop()
        metrics.stop()


def test_manager_end_to_end_podgroup_progress(store):
    mgr = _manager(store).start()
    try:
        store.create("podgroups", make_pod_group("g", min_member=2))
        assert wait_for(lambda: (store.get("podgroups", "default", "g").get("status") or {}).get("phase") == "Pending")
        for n in ("a", "b"):
            store.create("pods", make_pod(n, pod_group="g"))
        assert wait_for(lambda: store.get("podgroups", "default", "g")["status"]["phase"] == "PreScheduling")
    finally:
        mgr.stop()


def _kustomize_files(d):
    k = yaml.safe_load(open(os.path.join(d, "kustomization.yaml")))
    out = []
    for r in k.get("resources", []):
        p = os.path.normpath(os.path.join(d, r))
        if os.path.isdir(p):
            out += _kustomize_files(p)
        else:
            out.append(p)
    return out


def test_kustomize_scaffold_resources_parse():
    files = _kustomize_files(os.path.join(ROOT, "deploy", "config", "default"))
    kinds = []
    for f in files:
        assert os.path.exists(f), f
        kinds += [d["kind"] for d in yaml.safe_load_all(open(f)) if d]
    assert {"CustomResourceDefinition", "ClusterRole", "Deployment", "ServiceAccount", "Role"} <= set(kinds)
    dep = [d for d in yaml.safe_load_all(open(os.path.join(ROOT, "deploy", "config", "manager", "manager.yaml")))
           if d and d["kind"] == "Deployment"][0]
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["command"][-1] == "manager" and "--leader-elect" in c["args"]
    # Every flag the Deployment passes is accepted by the CLI.
    from flex_gpu_scheduler_amd.cli import build_parser

    parser = build_parser()
    args = parser.parse_args(["manager"] + [a.replace("$(POD_NAMESPACE)", "ns") for a in c["args"]])
    assert args.leader_elect and args.leader_election_namespace == "ns"
    assert os.path.exists(os.path.join(ROOT, "deploy", "config", "prometheus", "monitor.yaml"))


def test_manager_cli_process(store):
    from flex_gpu_scheduler_amd.control import ApiServer

    srv = ApiServer(store).start()
    env = dict(os.environ, PYTHONPATH=ROOT)
    proc = subprocess.Popen([sys.executable, "-m", "flex_gpu_scheduler_amd", "manager", "--master", srv.url,
                             "--health-probe-bind-address", "127.0.0.1:0", "--metrics-bind-address", "127.0.0.1:0"],
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, text=True)
    try:
        line = {}
        t = threading.Thread(target=lambda: line.update(json.loads(proc.stdout.readline())), daemon=True)
        t.start()
        t.join(60)
        assert line.get("manager") == ["podgroup", "elasticquota"], line
        assert urllib.request.urlopen(line["probes"] + "/readyz").status == 200
        store.create("podgroups", make_pod_group("cli", min_member=1))
        assert wait_for(lambda: (store.get("podgroups", "default", "cli").get("status") or {}).get("phase")
                        == "Pending", timeout=15)
    finally:
        proc.terminate()
        try:
            proc.wait(10)
        except subprocess.TimeoutExpired:
            proc.kill()
        srv.stop()
