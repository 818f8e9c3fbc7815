import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer-running CPU test")
    # Build the native core in-tree once per session (incremental).
    from flex_gpu_scheduler_amd import build_ext

    build_ext.build_core(verbose=False)


@pytest.fixture(autouse=True)
def _stop_leaked_informers(request):
    """Python informers a test started and left running are stopped at its
    end (their API server is gone, so they would retry and log forever)."""
    from flex_gpu_scheduler_amd.control.informer import STARTED

    before = set(STARTED)
    yield
    leaked = [i for i in list(STARTED) if i not in before and i.running()]
    for inf in leaked:
        inf.stop()
    if leaked:
        request.node.user_properties.append(("leaked_informers", sorted(i.kind for i in leaked)))
        import warnings

        warnings.warn(f"{request.node.nodeid} left informers running: {sorted(i.kind for i in leaked)}")


@pytest.fixture
def store():
    from flex_gpu_scheduler_amd import Store

    return Store()


def _openssl(*args, cwd):
    subprocess.run(["openssl", *args], cwd=cwd, check=True, capture_output=True)


@pytest.fixture(scope="session")
def pki(tmp_path_factory):
    """CA, server (SAN 127.0.0.1) and client certificates from the openssl CLI,
    plus an unrelated CA (TLS tests)."""
    d = tmp_path_factory.mktemp("pki")
    _openssl("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", "ca.key", "-out", "ca.crt", "-days", "2",
             "-subj", "/CN=test-ca", cwd=d)
    (d / "san.cnf").write_text("subjectAltName=IP:127.0.0.1,DNS:localhost\n")
    for name, cn in (("server", "127.0.0.1"), ("client", "system:kube-scheduler")):
        _openssl("req", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{name}.key", "-out", f"{name}.csr",
                 "-subj", f"/CN={cn}", cwd=d)
        extra = ["-extfile", "san.cnf"] if name == "server" else []
        _openssl("x509", "-req", "-in", f"{name}.csr", "-CA", "ca.crt", "-CAkey", "ca.key", "-CAcreateserial",
                 "-out", f"{name}.crt", "-days", "2", *extra, cwd=d)
    _openssl("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", "other.key", "-out", "other.crt",
             "-days", "2", "-subj", "/CN=other-ca", cwd=d)
    return d
