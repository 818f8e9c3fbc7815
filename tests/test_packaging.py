"""Packaging: pyproject console scripts, Makefile targets, `make verify`
(lint, CRD regeneration diff, charts, example configs, Dockerfile); the
reference's Makefile:43-129, build/*/Dockerfile and hack/verify-crdgen.sh."""
import importlib
import re
import subprocess
import sys
from pathlib import Path

import tomli

ROOT = Path(__file__).resolve().parents[1]


def test_pyproject_console_scripts_resolve():
    meta = tomli.loads((ROOT / "pyproject.toml").read_text())
    scripts = meta["project"]["scripts"]
    assert scripts["xsched"] == "flex_gpu_scheduler_amd.cli:main"
    for target in scripts.values():
        mod, fn = target.split(":")
        assert callable(getattr(importlib.import_module(mod), fn)), target
    assert meta["project"]["version"] == re.search(r"^IMAGE_TAG \?= (\S+)", (ROOT / "Makefile").read_text(), re.M)[1]


def test_makefile_has_the_targets():
    mk = (ROOT / "Makefile").read_text()
    for t in ("build", "test", "test-gpu", "verify", "crds", "image", "bench"):
        assert re.search(rf"^{re.escape(t)}:", mk, re.M), t
    # Recipes are tab-indented (make requires it).
    assert "\n\t$(PYTHON) -m flex_gpu_scheduler_amd.tools.verify" in mk


def test_make_verify_is_clean():
    r = subprocess.run([sys.executable, "-m", "flex_gpu_scheduler_amd.tools.verify"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert r.stdout.count(": ok") == 7


def test_verify_catches_problems(tmp_path, monkeypatch):
    from flex_gpu_scheduler_amd.tools import verify

    bad = tmp_path / "bad.py"
    bad.write_text("import os\nx = 1 \n")
    import ast

    text = bad.read_text()
    errs = verify._text_checks(bad, text) + verify.unused_imports(bad, ast.parse(text), text)
    assert any("trailing whitespace" in e for e in errs) and any("unused import os" in e for e in errs)


def test_logging_lint_wants_constant_messages():
    from flex_gpu_scheduler_amd.tools.verify import log_call_errors

    good = 'XS_LOGV(6, "fit indexes").kv("pod", p.key());\nXS_WARN("dropped").kv("err", e.what());'
    bad = 'XS_WARN("dropped " + name);\nXS_LOGV(6, msg).kv("x", 1);'
    assert log_call_errors("a.cc", good) == []
    errs = log_call_errors("b.cc", bad)
    assert len(errs) == 2 and errs[0].startswith("b.cc:1:") and errs[1].startswith("b.cc:2:")
